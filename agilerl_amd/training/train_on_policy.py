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

Sharded over ranks (``create_population`` under a process group of G > 1:
rank r holds global agents r*P ..), the run is the single-process run of the
G*P-agent population: each agent samples its global env's stream, learns
from its global shuffles, and the generation step (fitness all-gather,
tournament, host attributes of the clones, mutations) is taken once over the
global population on every rank (hpo/shard.py), each rank keeping its slice.
``pop_fitnesses`` holds every global agent's fitness.
"""

from __future__ import annotations

import copy
import time
from datetime import datetime

import numpy as np
import torch.distributed as dist

from ..envs import StackedVecEnv
from ..hpo.population_sync import PopulationSync
from ..hpo.shard import all_ranks, gather_records, mutate_population
from ..population.runner import PopulationRunner


def _population_env(env, P: int, N: int, offset: int = 0):
    if env.num_envs == P * N:
        return env
    if env.num_envs == N:
        return env if P == 1 and offset == 0 else StackedVecEnv.from_shared(env, P, offset)
    raise ValueError(f"env has {env.num_envs} environments; the population needs num_envs = {N} (the reference's "
                     f"shared env, cloned per agent) or population_size x num_envs = {P * N}")


def _clone_host_attributes(pop, parents: list[int], elitism: bool, records: list[dict], rank: int = 0) -> None:
    """The attributes TournamentSelection._select_standard_agents gives the
    clones (tournament.py:71-119 + clone/copy_attributes, core/base.py:
    444-503, 871-937), over the GLOBAL population: new agent g is a copy of
    old agent parents[g] (``records``: every global agent's host record,
    taken before the clone); the elite keeps its index, every other clone
    gets max_id + 1, + 2, ... in global slot order.  This rank applies its
    own slots."""
    import copy as _copy

    P = len(pop)
    max_id = max(r["index"] for r in records)
    for g, q in enumerate(parents):
        if elitism and g == 0:
            new_index = records[q]["index"]
        else:
            max_id += 1
            new_index = max_id
        if g // P != rank:
            continue
        a, src = pop[g % P], records[q]
        a.fitness, a.scores, a.steps = (_copy.deepcopy(src[k]) for k in ("fitness", "scores", "steps"))
        a.registry, a.mut = _copy.deepcopy(src["_registry"]), src.get("mut")
        a.index = new_index
        # the device rows (PopulationSync) carry the hyperparameters as f32 /
        # int32; the host keeps the parent's exact values
        hp = src.get("_hp", {})
        a.population.set_host_hparams(a.row, lr=hp.get("lr"), batch_size=hp.get("batch_size"),
                                      update_epochs=hp.get("update_epochs"), ent_coef=hp.get("ent_coef"))


def _sync_global_epochs(population) -> None:
    """Every global agent's update_epochs (the shuffles each draws) and batch
    size (the learner's partner split) after a mutation may have changed
    another shard's."""
    if population.global_P == population.P:
        return
    box: list = [None] * dist.get_world_size()
    dist.all_gather_object(box, (list(population.agent_epochs), list(population.agent_batch)))
    population.global_epochs = [int(e) for b in box for e in b[0]]
    population.global_batch = [int(x) for b in box for x in b[1]]


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
    world, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)
    if population.global_P not in (P, P * world) or population.agent_offset not in (0, rank * P):
        raise ValueError("the population's shard does not match this process group")
    env = _population_env(env, P, N, population.agent_offset)
    runner = PopulationRunner(population, env)
    sync = None
    if tournament is not None and mutation is not None:  # the reference selects only with both (:440)
        sync = PopulationSync(population, runner, world, rank, seed=None, tournament_size=tournament.tournament_size,
                              elitism=tournament.elitism, eval_loop=tournament.eval_loop)
    save_path = (checkpoint_path.split(".pt")[0] if checkpoint_path is not None
                 else f"{env_name}-EvoHPO-{algo}-{datetime.now().strftime('%m%d%Y%H%M%S')}")
    checkpoint_count = 0
    if mutation is not None:  # pre-training mutation (:200-201)
        pop = mutate_population(mutation, pop, pre_training_mut=True)
        _sync_global_epochs(population)
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
        if world > 1:
            box: list = [None] * world
            dist.all_gather_object(box, fitness)
            pop_fitnesses.append([f for b in box for f in b])
        else:
            pop_fitnesses.append(fitness)
        if target is not None and all_ranks(np.all(np.greater([np.mean(a.fitness[-10:]) for a in pop], target))) \
                and len(pop[0].steps) >= 100:
            return pop, pop_fitnesses
        if sync is not None:  # tournament_selection_and_mutation (utils.py:1137-1225)
            records = gather_records(pop)  # every global agent's host attributes, before the clone
            sync.fitness_override = np.asarray(fitness)  # reduced on the host already: hand it over
            parents = sync.generation()
            _clone_host_attributes(pop, parents, tournament.elitism, records, rank)
            if save_elite and tournament.elitism and rank == 0:
                # the reference saves ``elite``, the unmutated clone of the best agent
                # (utils.py:1214-1223): slot 0 holds exactly that until mutation runs
                elite_save_path = elite_path.split(".pt")[0] if elite_path is not None else f"{env_name}-elite_{algo}"
                pop[0].save_checkpoint(f"{elite_save_path}.pt")
            pop = mutate_population(mutation, pop)
            _sync_global_epochs(population)
        if verbose:
            fps = sum(a.steps[-1] for a in pop) / max(time.time() - t0, 1e-9)
            print(f"--- {env_name} {algo}: steps {[a.steps[-1] for a in pop]}, fitness "
                  f"{[round(f, 2) for f in fitness]}, mean loss {np.mean(losses):.4f}, "
                  f"mutations {[a.mut for a in pop]}, {fps:.0f} env-steps/s")
        if checkpoint is not None and pop[0].steps[-1] // checkpoint > checkpoint_count:
            for j, agent in enumerate(pop):  # save_population_checkpoint (utils.py:1126-1135)
                i = population.agent_offset + j  # the global slot
                agent.save_checkpoint(f"{save_path}_{i}.pt" if overwrite_checkpoints
                                      else f"{save_path}_{i}_{agent.steps[-1]}.pt")
            checkpoint_count += 1
    return pop, pop_fitnesses

