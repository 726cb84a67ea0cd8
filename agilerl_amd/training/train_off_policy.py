"""Drop-in ``train_off_policy`` (agilerl/training/train_off_policy.py:41-616)
for DQN / RainbowDQN populations on the agx HBM replay buffers.

The loop mirrors the reference: agents in turn collect ``evo_steps`` from the
shared env with epsilon-greedy (DQN, epsilon decayed per step) or noisy-net
(Rainbow) actions into the SHARED memory (one replay for the population,
train_off_policy.py:249, 340-345), learn every ``learn_step`` env steps once
``len(memory) >= batch_size`` and ``memory.size > learning_delay`` (PER:
sample with the agent's annealed beta, update priorities; n-step: the
n-step memory sampled at the same indices), then every agent is evaluated
with ``agent.test``; with a tournament AND a mutation object (as the
reference) the tournament (``TournamentSelection.select``, global numpy RNG)
replaces the population and ``mutation.mutation`` mutates it (RL
hyperparameters, Q-network parameters with the target synced).  The replay
trees, TD / C51 losses and Polyak updates run in libagx.  Returns
(pop, pop_fitnesses).

Sharded over ranks (``create_population`` under a process group), each rank
runs its slice of the population on its own env and its own replay (a
documented deviation from the one shared memory, SURVEY §8e option ii); the
generation step is taken once over the global population on every rank:
the host generators are synchronised, the tournament selects over every
agent (hpo/sharded.py) and the mutations draw for every agent in the global
order (hpo/shard.py), each rank keeping its slice."""

from __future__ import annotations

import numpy as np

from ..algorithms.dqn import DQN, RainbowDQN
from ..components.sampler import Sampler
from ..hpo.shard import all_gather_obj, all_ranks, mutate_population, sync_host_rngs, world_rank
from ..hpo.sharded import select_population


def train_off_policy(env, env_name: str, algo: str, pop, memory, INIT_HP=None, MUT_P=None,
                     swap_channels: bool = False, max_steps: int = 1_000_000, evo_steps: int = 10_000,
                     eval_steps=None, eval_loop: int = 1, learning_delay: int = 0, eps_start: float = 1.0,
                     eps_end: float = 0.1, eps_decay: float = 0.995, target: float | None = None, n_step: bool = False,
                     per: bool = False, n_step_memory=None, tournament=None, mutation=None, checkpoint=None,
                     checkpoint_path=None, overwrite_checkpoints: bool = False, save_elite: bool = False,
                     elite_path=None, wb: bool = False, verbose: bool = True, accelerator=None, wandb_api_key=None,
                     wandb_kwargs=None):
    if mutation is not None:  # pre-training mutation (the reference's :238-240 / :204-206)
        pop = mutate_population(mutation, pop, pre_training_mut=True)
    num_envs = env.num_envs if hasattr(env, "num_envs") else 1
    sampler = Sampler(memory=memory)
    n_step_sampler = Sampler(memory=n_step_memory) if n_step_memory is not None else None
    pop_fitnesses: list[list[float]] = []

    def learn_once(agent):
        if per:
            experiences = sampler.sample(agent.batch_size, agent.beta)
            n_exp = n_step_sampler.sample(experiences["idxs"]) if n_step_sampler is not None else None
            loss, idxs, priorities = agent.learn(experiences, n_experiences=n_exp, per=per)
            memory.update_priorities(idxs, priorities)
            return loss
        experiences = sampler.sample(agent.batch_size, return_idx=n_step_memory is not None)
        if n_step_memory is not None:
            loss, *_ = agent.learn(experiences, n_experiences=n_step_sampler.sample(experiences["idxs"]))
            return loss
        out = agent.learn(experiences)
        return out[0] if isinstance(out, tuple) else out

    while np.less([agent.steps[-1] for agent in pop], max_steps).all():
        for agent in pop:
            obs, info = env.reset()
            scores = np.zeros(num_envs)
            if isinstance(agent, DQN):
                epsilon = eps_start
            for idx_step in range(evo_steps // num_envs):
                if isinstance(agent, DQN):
                    action = agent.get_action(obs, epsilon)
                    epsilon = max(eps_end, epsilon * eps_decay)
                elif isinstance(agent, RainbowDQN):
                    action = agent.get_action(obs)
                else:
                    raise NotImplementedError(f"{type(agent).__name__} is outside the agx off-policy path")
                next_obs, reward, done, trunc, info = env.step(action)
                scores += np.asarray(reward)
                for i, (d, t) in enumerate(zip(np.atleast_1d(done), np.atleast_1d(trunc))):
                    if d or t:
                        agent.scores.append(scores[i])
                        scores[i] = 0
                transition = {"obs": obs, "action": np.asarray(action).reshape(num_envs, 1),
                              "reward": np.asarray(reward, dtype=np.float32).reshape(num_envs, 1),
                              "next_obs": next_obs,
                              "done": np.asarray(done, dtype=np.float32).reshape(num_envs, 1)}
                if n_step_memory is not None:
                    one_step = n_step_memory.add(transition)
                    if one_step is not None:
                        memory.add(one_step)
                else:
                    memory.add(transition)
                if per:
                    fraction = min((agent.steps[-1] + idx_step + 1) * num_envs / max_steps, 1.0)
                    agent.beta += fraction * (1.0 - agent.beta)
                ready = len(memory) >= agent.batch_size and memory.size > learning_delay
                if agent.learn_step > num_envs:
                    if idx_step % (agent.learn_step // num_envs) == 0 and ready:
                        learn_once(agent)
                elif ready:
                    for _ in range(num_envs // agent.learn_step):
                        learn_once(agent)
                obs = next_obs
            agent.steps[-1] += (evo_steps // num_envs) * num_envs
        if isinstance(pop[-1], DQN):
            eps_start = epsilon  # train_off_policy.py:456-458: the next generation starts where this one ended
        fitnesses = [agent.test(env, swap_channels=swap_channels, max_steps=eval_steps, loop=eval_loop)
                     for agent in pop]
        world, _ = world_rank()
        if world > 1:  # every global agent's fitness, as the single-process run returns
            import torch.distributed as dist

            box: list = [None] * world
            all_gather_obj(box, fitnesses, tag="fitness")
            pop_fitnesses.append([f for b in box for f in b])
        else:
            pop_fitnesses.append(fitnesses)
        if verbose:
            print(f"--- {env_name} {algo}: steps {[a.steps[-1] for a in pop]}, fitness "
                  f"{[round(f, 2) for f in fitnesses]}")
        for agent in pop:
            agent.steps.append(agent.steps[-1])
        if target is not None and all_ranks(np.all(np.greater([np.mean(a.fitness[-10:]) for a in pop], target))) \
                and len(pop[0].steps) >= 100:
            return pop, pop_fitnesses
        if tournament and mutation is not None:
            # tournament_selection_and_mutation (utils.py:1137-1225, train_off_policy.py:557-565):
            # under an initialised process group each rank holds a shard of the population
            sync_host_rngs()  # every rank draws the selection and mutations from one state
            _, pop = select_population(tournament, pop)
            pop = mutate_population(mutation, pop)
    return pop, pop_fitnesses
