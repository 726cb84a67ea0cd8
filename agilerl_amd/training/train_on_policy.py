"""Drop-in ``train_on_policy`` (agilerl/training/train_on_policy.py:30-511)
for a PPO population built by ``agilerl_amd.utils.create_population``.

The reference loops over agents, each taking its turn on the shared env
(``env.reset()`` at the start of its turn, :210-262) and learning in turn.
Here the population is ONE HBM engine: every vector step advances all P
agents, and each iteration runs bootstrap + GAE + the fused learner for all
agents at once.  The env the reference call site passes (``num_envs`` = N) is
given to the agents as P deep copies side by side (envs.StackedVecEnv, agent
p owning envs [p*N, (p+1)*N)); a vector env of P*N envs, or a StackedVecEnv,
is used as is.  A generation is ``ceil(evo_steps / learn_step)`` iterations
per agent (:248-262).

Per generation, as the reference:
  * fitness = ``agent.test`` of every agent (:363-373: one finished episode
    per env, ``eval_steps`` caps a pass, mean over ``eval_loop`` passes), run
    for the whole population at once by ``PopulationRunner.evaluate``;
  * with a tournament AND a mutation object (:440-452):
    tournament_selection_and_mutation (utils/utils.py:1137-1225) — selection
    on the device (hpo.population_sync: parent rows, Adam state, lr, step and
    per-agent hyperparameters cloned), the clones' host attributes (fitness /
    score / step histories, mutation registry, index: elite keeps its own,
    the others max_id + 1, ...) as TournamentSelection.clone gives them, then
    ``mutation.mutation(pop)`` (hpo.mutation: RL-hyperparameter and
    parameter mutations with the reference's draws), then the elite saved
    when ``save_elite`` (utils.py:1217-1223);
  * a population checkpoint every ``checkpoint`` steps
    (save_population_checkpoint, utils.py:1087-1135): ``{path}_{i}.pt`` or
    ``{path}_{i}_{steps}.pt``.
Returns (pop, pop_fitnesses) like the reference.
"""

from __future__ import annotations

import copy
import time
from datetime import datetime

import numpy as np
import torch.distributed as dist

from ..envs import StackedVecEnv
from ..hpo.population_sync import PopulationSync
from ..population.runner import PopulationRunner


def _population_env(env, P: int, N: int):
    if env.num_envs == P * N:
        return env
    if env.num_envs == N:
        return env if P == 1 else StackedVecEnv.from_shared(env, P)
    raise ValueError(f"env has {env.num_envs} environments; the population needs num_envs = {N} (the reference's "
                     f"shared env, cloned per agent) or population_size x num_envs = {P * N}")


def _clone_host_attributes(pop, parents: list[int], elitism: bool, fitness_of=None) -> None:
    """The attributes TournamentSelection._select_standard_agents gives the
    clones (tournament.py:71-119 + clone/copy_attributes, core/base.py:
    444-503, 871-937): new agent j is a copy of old agent parents[j]; the
    elite keeps its index, every other clone gets max_id + 1, + 2, ...  With
    several ranks a parent may live elsewhere: its fitness history comes
    from the gathered record (``fitness_of``), the rest stays local."""
    P = len(pop)
    old = [dict(index=a.index, fitness=list(a.fitness), scores=list(a.scores), steps=list(a.steps),
                registry=a.registry, mut=a.mut) for a in pop]
    max_id = max(o["index"] for o in old)
    for j, q in enumerate(parents):
        a = pop[j]
        src = old[q] if q < P and fitness_of is None else None
        if src is not None:
            a.fitness, a.scores, a.steps = (copy.deepcopy(src[k]) for k in ("fitness", "scores", "steps"))
            a.registry, a.mut = copy.deepcopy(src["registry"]), src["mut"]
        elif fitness_of is not None:
            a.fitness = list(fitness_of(q))
        if elitism and j == 0:
            a.index = old[q]["index"] if src is not None else a.index
        else:
            max_id += 1
            a.index = max_id


def train_on_policy(env, env_name: str, algo: str, pop, INIT_HP=None, MUT_P=None, swap_channels: bool = False,
                    max_steps: int = 1_000_000, evo_steps: int = 10_000, eval_steps=None, eval_loop: int = 1,
                    target: float | None = None, tournament=None, mutation=None, checkpoint=None,
                    checkpoint_path=None, overwrite_checkpoints: bool = False, save_elite: bool = False,
                    elite_path=None, wb: bool = False, verbose: bool = True, accelerator=None, wandb_api_key=None,
                    wandb_kwargs=None, collect_rollouts_fn=None):
    if collect_rollouts_fn is not None:
        raise NotImplementedError("custom collect_rollouts_fn: the population engine collects on device "
                                  "(PopulationRunner); pass None")
    population = pop[0].population
    if any(a.population is not population for a in pop):
        raise ValueError("all agents must come from one agilerl_amd.utils.create_population call")
    P, N, T = population.P, population.N, population.T
    env = _population_env(env, P, N)
    runner = PopulationRunner(population, env)
    world, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)
    sync = None
    if tournament is not None and mutation is not None:  # the reference selects only with both (:440)
        sync = PopulationSync(population, runner, world, rank, seed=None, tournament_size=tournament.tournament_size,
                              elitism=tournament.elitism, eval_loop=tournament.eval_loop)
    save_path = (checkpoint_path.split(".pt")[0] if checkpoint_path is not None
                 else f"{env_name}-EvoHPO-{algo}-{datetime.now().strftime('%m%d%Y%H%M%S')}")
    checkpoint_count = 0
    if mutation is not None:  # pre-training mutation (:200-201)
        pop = mutation.mutation(pop, pre_training_mut=True)
    iters_per_gen = max(1, -(-evo_steps // (T * N)))
    pop_fitnesses: list[list[float]] = []
    t0 = time.time()
    while min(agent.steps[-1] for agent in pop) < max_steps:
        losses = []
        for _ in range(iters_per_gen):
            losses.append(runner.iteration().cpu().numpy())
            population.check_errors()
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
        if target is not None and np.all(np.greater([np.mean(a.fitness[-10:]) for a in pop], target)) \
                and len(pop[0].steps) >= 100:
            return pop, pop_fitnesses
        if sync is not None:  # tournament_selection_and_mutation (utils.py:1137-1225)
            sync.fitness_override = np.asarray(fitness)  # reduced on the host already: hand it over
            parents = sync.generation()
            mine = parents[rank * P:(rank + 1) * P]
            hist = sync.history
            fit_of = None if world == 1 else (lambda q: [h[q] for h in hist])
            _clone_host_attributes(pop, [q % P if world == 1 else q for q in mine], tournament.elitism, fit_of)
            if save_elite and tournament.elitism and rank == 0:
                # the reference saves ``elite``, the unmutated clone of the best agent
                # (utils.py:1214-1223): slot 0 holds exactly that until mutation runs
                elite_save_path = elite_path.split(".pt")[0] if elite_path is not None else f"{env_name}-elite_{algo}"
                pop[0].save_checkpoint(f"{elite_save_path}.pt")
            pop = mutation.mutation(pop)
        if verbose:
            fps = sum(a.steps[-1] for a in pop) / max(time.time() - t0, 1e-9)
            print(f"--- {env_name} {algo}: steps {[a.steps[-1] for a in pop]}, fitness "
                  f"{[round(f, 2) for f in fitness]}, mean loss {np.mean(losses):.4f}, "
                  f"mutations {[a.mut for a in pop]}, {fps:.0f} env-steps/s")
        if checkpoint is not None and pop[0].steps[-1] // checkpoint > checkpoint_count:
            for i, agent in enumerate(pop):  # save_population_checkpoint (utils.py:1126-1135)
                agent.save_checkpoint(f"{save_path}_{i}.pt" if overwrite_checkpoints
                                      else f"{save_path}_{i}_{agent.steps[-1]}.pt")
            checkpoint_count += 1
    return pop, pop_fitnesses

