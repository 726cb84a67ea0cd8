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
from ..hpo.shard import all_gather_obj, all_ranks, gather_fitness_records, mutate_population
from ..population.engine import PopulationEngine


#: host wall seconds per phase of the generation loop, accumulated over calls
#: (diagnostic; bench.py reads and clears it): "train" (collect + learn
#: iterations), "evaluate" (agent.test of every agent), "select" (tournament,
#: parent clone, host attributes), "mutate" (mutations), "regroup" (moving
#: mutated agents to their groups)
PHASE_TIMES: dict[str, float] = {}


class _Phase:
    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        PHASE_TIMES[self.name] = PHASE_TIMES.get(self.name, 0.0) + time.perf_counter() - self.t0
        return False


def _population_env(env, P: int, N: int, offset: int = 0):
    if env.num_envs == P * N:
        return env
    if env.num_envs == N:
        return env if P == 1 and offset == 0 else StackedVecEnv.from_shared(env, P, offset)
    raise ValueError(f"env has {env.num_envs} environments; the population needs num_envs = {N} (the reference's "
                     f"shared env, cloned per agent) or population_size x num_envs = {P * N}")


def _check_env_allows_mutations(engine, mutation, pop) -> None:
    """Architecture and learn_step mutations give agents their own networks /
    rollout lengths, and such agents need an env each (the reference's
    shared N-env, cloned per agent, or a StackedVecEnv).  One undivided
    vector env of P x N envs keeps the whole population in one group: refuse
    it at start-up rather than after the first such mutation."""
    if mutation is None or engine.slot_envs is not None or engine.P == 1:
        return
    arch = float(getattr(mutation, "architecture_mut", 0.0) or 0.0) > 0
    hp = getattr(getattr(pop[0], "registry", None), "hp_config", None)
    ls = bool(hp) and "learn_step" in hp.names() and float(getattr(mutation, "rl_hp_mut", 0.0) or 0.0) > 0
    if arch or ls:
        raise ValueError("architecture / learn_step mutations need one env per agent: pass the reference's "
                         f"num_envs = {engine.N} env (cloned per agent) or a StackedVecEnv of "
                         f"{engine.P} envs, not one vector env of {engine.P * engine.N}")


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


def _all_one_group(engine) -> bool:
    """Every rank holds one group, and all ranks the same (shape, learn_step):
    the device-row clone of PopulationSync applies."""
    mine = (engine.single_group, engine.groups[0].pop.spec.shape_key(), engine.groups[0].learn_step)
    if engine.world == 1:
        return mine[0]
    box: list = [None] * engine.world
    all_gather_obj(box, mine, tag="group_shapes")
    return all(b[0] for b in box) and len({(b[1], b[2]) for b in box}) == 1


def _apply_mutations(engine) -> None:
    """After mutations: agents whose architecture or learn_step changed move to
    their group (regroup); every rank learns every global agent's plan."""
    changed = engine.pending()
    if engine.world > 1:
        box: list = [None] * engine.world
        all_gather_obj(box, changed, tag="mutated_flags")
        changed = any(box)
    if changed:
        engine.regroup(engine.local_states())
    else:
        engine.refresh_plan()


def _train_with_collector(engine, pop, env, evo_steps: int, collect_fn) -> list:
    """train_on_policy.py:216-248 with a custom ``collect_rollouts_fn``: agent
    after agent on the caller's env, ``ceil(evo_steps / learn_step)`` times
    ``collect_fn(agent, env, n_steps=..., last_obs=..., last_done=...,
    last_scores=..., last_info=...)`` (filling ``agent.rollout_buffer``) then
    ``agent.learn()``; the collector's completed episode scores become the
    agent's training score."""
    losses = []
    for j, agent in enumerate(pop):
        g, _ = engine.group_of(j)
        n_steps = -(int(g.learn_step) // -engine.N)
        last = {"last_obs": None, "last_done": None, "last_scores": None, "last_info": None}
        completed: list[float] = []
        for _ in range(engine.iterations(evo_steps, g.learn_step)):
            out = collect_fn(agent, env, n_steps=n_steps, **last)
            if isinstance(out, tuple) and len(out) == 5:
                scores, last["last_obs"], last["last_done"], last["last_scores"], last["last_info"] = out
                completed += [float(x) for x in scores]
            losses.append(np.asarray([agent.learn()]))
        if completed:
            agent.scores.append(float(np.mean(completed)))
    return losses


def train_on_policy(env, env_name: str, algo: str, pop, INIT_HP=None, MUT_P=None, swap_channels: bool = False,
                    max_steps: int = 1_000_000, evo_steps: int = 10_000, eval_steps=None, eval_loop: int = 1,
                    target: float | None = None, tournament=None, mutation=None, checkpoint=None,
                    checkpoint_path=None, overwrite_checkpoints: bool = False, save_elite: bool = False,
                    elite_path=None, wb: bool = False, verbose: bool = True, accelerator=None, wandb_api_key=None,
                    wandb_kwargs=None, collect_rollouts_fn=None):
    population = pop[0].population
    user_env = env
    if any(a.population is not population for a in pop):
        raise ValueError("all agents must come from one agilerl_amd.utils.create_population call")
    P, N = population.P, population.N
    world, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)
    if population.global_P not in (P, P * world) or population.agent_offset not in (0, rank * P):
        raise ValueError("the population's shard does not match this process group")
    env = _population_env(env, P, N, population.agent_offset)
    # agents grouped by (network shape, learn_step): one group until a mutation splits them
    # a custom collector fills one agent's rollout at a time (the reference's
    # per-agent loop, :216-248): every agent then learns in a group of its own
    engine = PopulationEngine(population, pop, env, world, rank, singleton=collect_rollouts_fn is not None)
    _check_env_allows_mutations(engine, mutation, pop)
    sync = None
    if tournament is not None and mutation is not None:  # the reference selects only with both (:440)
        sync = PopulationSync(population, engine.groups[0].runner, world, rank, seed=None,
                              tournament_size=tournament.tournament_size, elitism=tournament.elitism,
                              eval_loop=tournament.eval_loop)
    save_path = (checkpoint_path.split(".pt")[0] if checkpoint_path is not None
                 else f"{env_name}-EvoHPO-{algo}-{datetime.now().strftime('%m%d%Y%H%M%S')}")
    checkpoint_count = 0
    if mutation is not None:  # pre-training mutation (:200-201)
        pop = mutate_population(mutation, pop, pre_training_mut=True)
        _apply_mutations(engine)
    pop_fitnesses: list[list[float]] = []
    t0 = time.time()
    # np.less([...], max_steps).all() (:204): every agent of every rank still below max_steps
    while all_ranks(all(agent.steps[-1] < max_steps for agent in pop)):
        # the generation's minibatch shuffles, agent after agent as the reference's
        # agents learn (train_on_policy.py:210-248 -> ppo.py:836-842)
        with _Phase("train"):
            engine.draw_generation_perms(evo_steps)
            if collect_rollouts_fn is None:
                losses = engine.train(evo_steps)
            else:
                losses = _train_with_collector(engine, pop, user_env, evo_steps, collect_rollouts_fn)
        for j, agent in enumerate(pop):
            agent.steps[-1] += engine.steps_per_generation(j, evo_steps)
        engine.resync_numpy_after_generation(evo_steps)
        # training-episode scores (on_policy.py:147-172 -> agent.scores) ...
        r_sum, r_cnt = engine.episode_stats()
        # ... then the population's fitness: agent.test for every agent
        # (train_on_policy.py:363-373), batched on device over the env slices
        with _Phase("evaluate"):
            fitness = engine.evaluate(eval_loop, eval_steps)
        for i, agent in enumerate(pop):
            if r_cnt[i] > 0 and collect_rollouts_fn is None:
                agent.scores.append(float(r_sum[i] / r_cnt[i]))
            agent.fitness.append(fitness[i])
            agent.steps.append(agent.steps[-1])
        # the fitness scalars and, when a generation step follows, the agents'
        # host records it clones from: one exchange
        global_fit, gathered = gather_fitness_records(pop, fitness, sync is not None)
        pop_fitnesses.append(global_fit if world > 1 else fitness)
        if target is not None and all_ranks(np.all(np.greater([np.mean(a.fitness[-10:]) for a in pop], target))) \
                and len(pop[0].steps) >= 100:
            return pop, pop_fitnesses
        if sync is not None:  # tournament_selection_and_mutation (utils.py:1137-1225)
            with _Phase("select"):
                records = gathered  # every global agent's host attributes, before the clone
                sync.fitness_override = np.asarray(fitness)  # reduced on the host already: hand it over
                if _all_one_group(engine):
                    # one network shape and rollout length everywhere: parent rows move in HBM
                    sync.pop, sync.runner = engine.groups[0].pop, engine.groups[0].runner
                    parents = sync.generation()
                else:
                    parents = sync.select()
                    engine.regroup(engine.clone_states(parents, records))
                _clone_host_attributes(pop, parents, tournament.elitism, records, rank)
            if save_elite and tournament.elitism and rank == 0:
                # the reference saves ``elite``, the unmutated clone of the best agent
                # (utils.py:1214-1223): slot 0 holds exactly that until mutation runs
                elite_save_path = elite_path.split(".pt")[0] if elite_path is not None else f"{env_name}-elite_{algo}"
                pop[0].save_checkpoint(f"{elite_save_path}.pt")
            with _Phase("mutate"):
                pop = mutate_population(mutation, pop)
            with _Phase("regroup"):
                _apply_mutations(engine)
        if verbose:
            fps = sum(a.steps[-1] for a in pop) / max(time.time() - t0, 1e-9)
            print(f"--- {env_name} {algo}: steps {[a.steps[-1] for a in pop]}, fitness "
                  f"{[round(f, 2) for f in fitness]}, mean loss {np.mean([np.mean(x) for x in losses]):.4f}, "
                  f"mutations {[a.mut for a in pop]}, {fps:.0f} env-steps/s")
        if checkpoint is not None and pop[0].steps[-1] // checkpoint > checkpoint_count:
            for j, agent in enumerate(pop):  # save_population_checkpoint (utils.py:1126-1135)
                i = population.agent_offset + j  # the global slot
                agent.save_checkpoint(f"{save_path}_{i}.pt" if overwrite_checkpoints
                                      else f"{save_path}_{i}_{agent.steps[-1]}.pt")
            checkpoint_count += 1
    return pop, pop_fitnesses
