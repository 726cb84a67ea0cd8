"""Drop-in ``train_on_policy`` (agilerl/training/train_on_policy.py:30-511)
for a PPO population built by ``agilerl_amd.utils.create_population``.

The reference loops over agents, each collecting its own rollout from the
shared env and learning in turn (:210).  Here the population is ONE HBM
engine: every vector step advances all P agents (``env.num_envs`` must be
P x num_envs, agent p owning envs [p*N, (p+1)*N)), and each iteration runs
bootstrap + GAE + the fused learner for all agents at once.  A generation is
``ceil(evo_steps / learn_step)`` iterations per agent (:248-262), followed by
fitness and tournament selection on the device (hpo.population_sync).

Fitness is ``agent.test`` of every agent (train_on_policy.py:363-373: one
finished episode per env, ``eval_steps`` caps a pass, mean over
``eval_loop`` passes), run for the whole population at once by
``PopulationRunner.evaluate``: agent p acts on its own env slice with the
fused policy step; the env is reset per pass, so the next generation's
rollout starts from a reset like the reference's next collect_rollouts.
Training-episode means go to ``agent.scores``.  Selection runs whenever a
tournament is given (the reference also needs a mutation object).
Mutations (architecture / hyper-parameter) are outside the hot path: a
``mutation`` object is ignored with a warning.  Returns (pop, pop_fitnesses)
like the reference.
"""

from __future__ import annotations

import time
import warnings

import numpy as np
import torch.distributed as dist

from ..hpo.population_sync import PopulationSync
from ..population.runner import PopulationRunner


def train_on_policy(env, env_name: str, algo: str, pop, INIT_HP=None, MUT_P=None, swap_channels: bool = False,
                    max_steps: int = 1_000_000, evo_steps: int = 10_000, eval_steps=None, eval_loop: int = 1,
                    target: float | None = None, tournament=None, mutation=None, checkpoint=None,
                    checkpoint_path=None, overwrite_checkpoints: bool = False, save_elite: bool = False,
                    elite_path=None, wb: bool = False, verbose: bool = True, accelerator=None, wandb_api_key=None,
                    wandb_kwargs=None, collect_rollouts_fn=None):
    if collect_rollouts_fn is not None:
        raise NotImplementedError("custom collect_rollouts_fn: the population engine collects on device")
    if mutation is not None:
        warnings.warn("agx train_on_policy: mutations are outside the hot path and are not applied", stacklevel=2)
    population = pop[0].population
    if any(a.population is not population for a in pop):
        raise ValueError("all agents must come from one agilerl_amd.utils.create_population call")
    P, N, T = population.P, population.N, population.T
    if env.num_envs != P * N:
        raise ValueError(f"the env must hold num_envs x population_size = {P * N} environments "
                         f"(agent p owns envs [p*{N}, (p+1)*{N})); got {env.num_envs}")
    runner = PopulationRunner(population, env)
    sync = None
    if tournament is not None:
        world, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)
        sync = PopulationSync(population, runner, world, rank, seed=None, tournament_size=tournament.tournament_size,
                              elitism=tournament.elitism, eval_loop=tournament.eval_loop)
    iters_per_gen = max(1, -(-evo_steps // (T * N)))
    pop_fitnesses: list[list[float]] = []
    t0 = time.time()
    while min(agent.steps[-1] for agent in pop) < max_steps:
        losses = []
        for _ in range(iters_per_gen):
            losses.append(runner.iteration().cpu().numpy())
            for agent in pop:
                agent.steps[-1] += T * N
        # training-episode scores (on_policy.py:147-172 -> agent.scores) ...
        r_sum = runner.episode_return_sum.cpu().numpy()
        r_cnt = runner.episodes.cpu().numpy()
        runner.reset_episode_stats()
        # ... then the population's fitness: agent.test for every agent
        # (train_on_policy.py:363-373), batched on device over the env slices
        fitness = [float(f) for f in runner.evaluate(loop=eval_loop, max_steps=eval_steps)]
        for i, agent in enumerate(pop):
            if r_cnt[i] > 0:
                agent.scores.append(float(r_sum[i] / r_cnt[i]))
            agent.fitness.append(fitness[i])
            agent.steps.append(agent.steps[-1])
        pop_fitnesses.append(fitness)
        if verbose:
            fps = sum(a.steps[-1] for a in pop) / max(time.time() - t0, 1e-9)
            print(f"--- {env_name} {algo}: steps {[a.steps[-1] for a in pop]}, fitness "
                  f"{[round(f, 2) for f in fitness]}, mean loss {np.mean(losses):.4f}, {fps:.0f} env-steps/s")
        if target is not None and np.all(np.greater([np.mean(a.fitness[-10:]) for a in pop], target)) \
                and len(pop[0].steps) >= 100:
            break
        if sync is not None:  # fitness reduced on the host already: hand it over
            sync.fitness_override = np.asarray(fitness)
            sync.generation()
    return pop, pop_fitnesses
