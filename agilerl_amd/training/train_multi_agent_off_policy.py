"""Drop-in ``train_multi_agent_off_policy``
(agilerl/training/train_multi_agent_off_policy.py:33-560) for MADDPG
populations on the HBM ``MultiAgentReplayBuffer``.

Per generation each agent in turn: ``evo_steps // num_envs`` vector steps of
``get_action`` (raw actor outputs saved), ``save_to_memory`` into the shared
memory, learning every ``learn_step`` env steps once ``len(memory) >=
batch_size`` and ``memory.counter > learning_delay``; episode bookkeeping and
OU-noise resets on finished envs; then ``agent.test`` fitness, and tournament
selection of clones and mutations (RL hyperparameters, actor parameters with
the targets synced) when both a tournament and a mutation object are given,
as the reference.  Returns (pop, pop_fitnesses)."""

from __future__ import annotations

import numpy as np

from ..components.sampler import Sampler
from ..hpo.shard import all_ranks, mutate_population, sync_host_rngs
from ..hpo.sharded import select_population


def train_multi_agent_off_policy(env, env_name: str, algo: str, pop, memory, INIT_HP=None, MUT_P=None,
                                 sum_scores: bool = True, swap_channels: bool = False, max_steps: int = 50000,
                                 evo_steps: int = 25, eval_steps=None, eval_loop: int = 1,
                                 learning_delay: int = 0, target: float | None = None, tournament=None,
                                 mutation=None, checkpoint=None, checkpoint_path=None,
                                 overwrite_checkpoints: bool = False, save_elite: bool = False, elite_path=None,
                                 wb: bool = False, verbose: bool = True, accelerator=None, wandb_api_key=None,
                                 wandb_kwargs=None):
    if mutation is not None:  # pre-training mutation (the reference's :238-240 / :204-206)
        pop = mutate_population(mutation, pop, pre_training_mut=True)
    vec = hasattr(env, "num_envs")
    num_envs = env.num_envs if vec else 1
    sampler = Sampler(memory=memory)
    agent_ids = list(env.agents)
    pop_fitnesses: list[list[float]] = []
    while np.less([agent.steps[-1] for agent in pop], max_steps).all():
        for agent in pop:
            agent.set_training_mode(True)
            obs, info = env.reset()
            scores = np.zeros((num_envs, 1)) if sum_scores else np.zeros((num_envs, len(agent_ids)))
            steps = 0
            for idx_step in range(evo_steps // num_envs):
                action, raw_action = agent.get_action(obs=obs, infos=info)
                if not vec:
                    action = {a: act[0] for a, act in action.items()}
                next_obs, reward, termination, truncation, info = env.step(action)
                r = np.array(list(reward.values())).transpose()
                r = np.where(np.isnan(r), 0, r)
                scores += (np.sum(r, axis=-1)[:, None] if vec else np.sum(r, axis=-1)) if sum_scores else r
                steps += num_envs
                memory.save_to_memory(obs, raw_action, reward, next_obs, termination, is_vectorised=vec)
                ready = len(memory) >= agent.batch_size and memory.counter > learning_delay
                if agent.learn_step > num_envs:
                    if idx_step % (agent.learn_step // num_envs) == 0 and ready:
                        agent.learn(sampler.sample(agent.batch_size))
                elif ready:
                    for _ in range(num_envs // agent.learn_step):
                        agent.learn(sampler.sample(agent.batch_size))
                obs = next_obs
                dones = {}
                for a in agent.agent_ids:
                    term = np.where(np.isnan(termination.get(a, True)), True, termination.get(a, True)).astype(bool)
                    trunc = np.where(np.isnan(truncation.get(a, False)), False,
                                     truncation.get(a, False)).astype(bool)
                    dones[a] = term | trunc
                if not vec:
                    dones = {a: np.array([dones[a]]) for a in agent.agent_ids}
                reset_idx = []
                for idx, agent_dones in enumerate(zip(*dones.values())):
                    if all(agent_dones):
                        agent.scores.append(np.asarray(scores[idx]).item() if sum_scores else list(scores[idx]))
                        scores[idx].fill(0)
                        reset_idx.append(idx)
                        if not vec:
                            obs, info = env.reset()
                agent.reset_action_noise(reset_idx)
            agent.steps[-1] += steps
        fitnesses = [agent.test(env, swap_channels=swap_channels, max_steps=eval_steps, loop=eval_loop,
                                sum_scores=sum_scores) for agent in pop]
        pop_fitnesses.append(fitnesses)
        if verbose:
            print(f"--- {env_name} {algo}: steps {[a.steps[-1] for a in pop]}, fitness {fitnesses}")
        for agent in pop:
            agent.steps.append(agent.steps[-1])
        if target is not None and all_ranks(np.all(np.greater([np.mean(a.fitness[-10:]) for a in pop], target))) \
                and len(pop[0].steps) >= 100:
            return pop, pop_fitnesses
        if tournament and mutation is not None:  # tournament_selection_and_mutation (:525-535)
            sync_host_rngs()  # every rank draws the selection and mutations from one state
            _, pop = select_population(tournament, pop)
            pop = mutate_population(mutation, pop)
    return pop, pop_fitnesses
