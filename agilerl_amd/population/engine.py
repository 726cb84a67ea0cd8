"""The population engine of train_on_policy: agents with different networks
and rollout lengths, as architecture and ``learn_step`` mutations make them.

The reference trains the agents of a population one after another, each
with its own networks and its own rollout length (train_on_policy.py:
210-262: ``-(evo_steps // -agent.learn_step)`` collect + learn iterations of
``ceil(learn_step / num_envs)`` vector steps per agent and generation).
Here the agents are SLOTS (local slot j = global agent rank * P + j, which
owns its env copy and its sampling streams) grouped by (network shape,
learn_step): every group is one :class:`PPOPopulation` (stacked parameters,
Adam state and rollout SoA in HBM; the fused HIP learner and rollout when the
shape is instantiated, the autograd learner with the HIP loss / clip + Adam
kernels otherwise) with its own :class:`PopulationRunner` over its slots'
envs.  An unmutated population is ONE group: exactly the lock-step engine.

Per generation:
  * ``draw_generation_perms``: the minibatch shuffles of the whole
    generation from numpy's global stream, agent after agent over the GLOBAL
    population (each agent's K learns of E shuffles, ppo.py:836-842), each
    group taking its agents' rows — the reference's draw order;
  * ``train``: every group runs its agents' K iterations;
  * fitness / episode scores per slot;
  * the clone (tournament): a single unchanged group keeps PopulationSync's
    device-row clone; otherwise every slot's full state (``AgentState``:
    network shape, learn_step, parameters, Adam moments and step,
    hyperparameters) is copied from its parent's (local: on device; another
    rank's: one packed message per (source, destination) pair);
  * mutations (hpo/shard.py over the global population): RL-hyperparameter
    and parameter mutations act on the group rows; an architecture or
    learn_step mutation leaves the view with a pending state;
  * ``regroup``: groups rebuilt from the slots' states when anything moved.
"""

from __future__ import annotations

import copy
import math
import os
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from ..envs import StackedVecEnv
from ..hpo.shard import all_gather_obj
from ..rng import numpy_shuffle_perms
from .ppo_pop import PPOPopulation
from .runner import PopulationRunner


@dataclass
class AgentState:
    """Everything one agent's learner carries between generations."""
    spec: object
    learn_step: int
    params: torch.Tensor      # [n] f32 (device or host)
    exp_avg: torch.Tensor     # [n]
    exp_avg_sq: torch.Tensor  # [n]
    step: int
    lr: float
    batch_size: int
    update_epochs: int
    ent_coef: float

    # A network spec is never changed in place (an architecture mutation makes a
    # new one: population/arch.py, image_arch.py), so states share it.
    def clone(self) -> "AgentState":
        return AgentState(self.spec, self.learn_step, self.params.clone(), self.exp_avg.clone(),
                          self.exp_avg_sq.clone(), self.step, self.lr, self.batch_size, self.update_epochs,
                          self.ent_coef)


def export_state(pop: PPOPopulation, row: int, learn_step: int, steps: list | None = None) -> AgentState:
    """``steps``: the population's Adam step counts read once (host list) by
    a caller exporting several rows; else this row's is read (a device sync)."""
    n = pop.spec.n_params
    return AgentState(pop.spec, int(learn_step), pop.params.data[row, :n].clone(),
                      pop.opt.exp_avg[row, :n].clone(), pop.opt.exp_avg_sq[row, :n].clone(),
                      int(steps[row] if steps is not None else pop.opt.steps[row]), float(pop.agent_lr[row]),
                      int(pop.agent_batch[row]), int(pop.agent_epochs[row]), float(pop.agent_ent[row]))


class _Group:
    def __init__(self, pop: PPOPopulation, runner: PopulationRunner, slots: list[int], learn_step: int):
        self.pop, self.runner, self.slots, self.learn_step = pop, runner, list(slots), int(learn_step)


class PopulationEngine:
    def __init__(self, population: PPOPopulation, views: list, env, world: int = 1, rank: int = 0,
                 singleton: bool = False):
        """``singleton``: every agent in a group of its own (custom collectors
        fill one agent's rollout at a time, as the reference's per-agent loop)."""
        self.views = list(views)
        self.singleton = bool(singleton)
        self.P, self.N = population.P, population.N
        self.world, self.rank = world, rank
        self.device = population.device
        learn_step = int(views[0].learn_step)
        # per-slot envs: a StackedVecEnv splits into its agents' envs; one
        # undivided vector env of P*N envs keeps the population in one group
        self.slot_envs = list(env.envs) if isinstance(env, StackedVecEnv) and len(env.envs) == self.P else None
        self._template = population
        self.groups = [_Group(population, PopulationRunner(population, env), list(range(self.P)), learn_step)]
        for j, v in enumerate(self.views):
            v.population, v.row = population, j
        # every global slot's (S, E, K-defining learn_step): refreshed after mutations
        self.global_plan = [(population.S, population.update_epochs, learn_step)] * (self.P * world)
        self._gen_state = None  # numpy state before the generation's shuffles (target_kl re-sync)
        # Sampling-noise counters.  A slot's Philox / Gumbel key is (seed_base,
        # global env index, counter); a group built by regroup() starts at
        # counter 0, so the counters are set from engine-level counts that every
        # rank shares: generation g's rollouts use counters from g << 24 (a
        # generation's vector steps stay far below 2^24), and the k-th
        # evaluation of the run its own round.  Neither depends on how slots are
        # grouped, so a sharded run and the single-process run draw alike.
        self._generation = 0
        self._eval_calls = getattr(population, "eval_rounds", 0)
        self._counter0 = -(-int(population.act_counter) // (1 << 24)) << 24  # past any earlier use
        self.refresh_plan()
        if self.singleton and self.P > 1:
            self.regroup(self.local_states())

    # ------------------------------------------------------------------ #
    @property
    def single_group(self) -> bool:
        return len(self.groups) == 1

    def group_of(self, slot: int) -> tuple[_Group, int]:
        for g in self.groups:
            if slot in g.slots:
                return g, g.slots.index(slot)
        raise KeyError(slot)

    def iterations(self, evo_steps: int, learn_step: int) -> int:
        """collect + learn iterations per generation (train_on_policy.py:231)."""
        return max(1, -(int(evo_steps) // -int(learn_step)))

    # ------------------------------------------------------------------ #
    def refresh_plan(self) -> None:
        """Every global slot's (rollout samples S, update epochs, learn_step)
        — each rank knows its own; one gather when sharded."""
        local = []
        for j in range(self.P):
            g, r = self.group_of(j)
            local.append((g.pop.S, int(g.pop.agent_epochs[r]), g.learn_step, int(g.pop.agent_batch[r])))
        if self.world > 1:
            box: list = [None] * self.world
            all_gather_obj(box, local, tag="population_plan")
            plan = [tuple(x) for b in box for x in b]
        else:
            plan = local
        self.global_plan = [x[:3] for x in plan]
        gmax = max(x[3] for x in plan)
        for g in self.groups:  # every group splits minibatches like the whole population
            g.pop.global_batch_max = gmax

    def draw_generation_perms(self, evo_steps: int) -> None:
        """The generation's minibatch shuffles from numpy's global stream in
        the reference's order: global agent after global agent, each its K
        learns of E shuffles of arange(S) (cumulative within a learn), every
        group taking the rows of its own agents."""
        pops = [g.pop for g in self.groups]
        if any(p.perm_source != "numpy" for p in pops):
            return
        for p in pops:
            p.discard_prefetch()
        self._gen_state = np.random.get_state(legacy=True)
        blocks = {}
        for g in self.groups:
            K = self.iterations(evo_steps, g.learn_step)
            blocks[id(g)] = np.zeros((K, g.pop.update_epochs, g.pop.P, g.pop.S), dtype=np.int64)
        where = {self.rank * self.P + j: self.group_of(j) for j in range(self.P)}
        # consecutive global agents with the same (S, E, K) draw in one native
        # call: agent after agent, learn after learn, each learn a fresh
        # arange(S) shuffled E times -- the same order as one call per learn
        plan = [(S, E, self.iterations(evo_steps, ls)) for S, E, ls in self.global_plan]
        i = 0
        while i < len(plan):
            j = i + 1
            while j < len(plan) and plan[j] == plan[i]:
                j += 1
            S, E, K = plan[i]
            if K > 0:
                buf = numpy_shuffle_perms((j - i) * K, E, S)  # [E, (j-i)*K, S]
                for gid in range(i, j):
                    if gid in where:
                        g, r = where[gid]
                        o = (gid - i) * K
                        blocks[id(g)][:, :E, r] = buf[:, o:o + K].transpose(1, 0, 2)
            i = j
        for g in self.groups:
            g.pop.set_generation_perms(blocks[id(g)])

    def resync_numpy_after_generation(self, evo_steps: int) -> None:
        """target_kl: the reference draws one shuffle per epoch an agent
        actually runs; re-advance the global stream from the generation's
        start by exactly those, over the global population (every rank
        replays the same re-advance; see PPOPopulation)."""
        pops = [g.pop for g in self.groups]
        if self._gen_state is None or all(p.target_kl is None for p in pops):
            return
        ran_local = [None] * self.P
        for g in self.groups:
            rows = [t.cpu().numpy() for t in g.pop._gen_ran]
            for r, slot in enumerate(g.slots):
                ran_local[slot] = [int(x[r]) for x in rows]
        if self.world > 1:
            # every rank replays the GLOBAL re-advance: each slot's epochs run
            # (a few ints per agent) gathered like refresh_plan's plan
            box: list = [None] * self.world
            all_gather_obj(box, ran_local, tag="epochs_run")
            ran_of = [x for b in box for x in b]
        else:
            ran_of = ran_local
        full = all(ran_of[j] == [self.global_plan[j][1]] * len(ran_of[j]) for j in range(len(ran_of)))
        if full:
            return
        np.random.set_state(self._gen_state)
        for j, (S, E, ls) in enumerate(self.global_plan):
            for ran in ran_of[j]:
                if ran:
                    numpy_shuffle_perms(1, ran, S)
        self._gen_state = None

    # ------------------------------------------------------------------ #
    def train(self, evo_steps: int, on_iteration=None) -> list:
        """Every group runs its agents' iterations of the generation; ->
        per-iteration mean losses (host arrays, group by group, slot order
        where known).

        The groups' iterations interleave, each group on a stream of its own
        (the host paces next the group with the most iterations left among
        those whose learner has finished): a group's learner (enqueued behind
        its rollout) runs on the device while the host paces ANOTHER group's
        rollout, and the groups' learners overlap one another.  At most one persistent launch is ever paced, and the
        host waits only for the launch it paces (the other streams hold finite
        kernels), so no hardware-queue ordering can stall it.  No host sync
        inside the loop: errors and losses are read once every group's
        iterations are queued (the learner reuses its loss buffer, hence the
        device-side copies)."""
        base = self._counter0 + (self._generation << 24)
        self._generation += 1
        main = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        iters, pending = [], []
        for k, g in enumerate(self.groups):
            if g.pop.act_counter > base:
                raise RuntimeError(f"rollout counter {g.pop.act_counter} overran generation {self._generation - 2}")
            g.pop.act_counter = base
            iters.append(self.iterations(evo_steps, g.learn_step))
            pending.append([])
        streams = [_train_stream(k) for k in range(len(self.groups))] if main is not None else None
        if streams is not None:
            for st in set(streams):  # parameters / buffers written by selection, mutation, regrouping
                st.wait_stream(main)
        # which group's next iteration the host paces: among the groups whose
        # previous learner has finished (its event), the one with the most
        # iterations left — the longest chain first; if none has finished, the
        # one with the most left anyway (its rollout starts when its learner
        # ends).  Each group's own iterations keep their order.
        left = list(iters)
        done_ev = [None] * len(self.groups)
        if streams is not None and len(self.groups) > 1 and self._paced_together():
            try:
                self._train_paced_together(left, streams, pending, on_iteration)
            finally:
                for st in set(streams):
                    main.wait_stream(st)
            losses = []
            for k, g in enumerate(self.groups):
                g.pop.check_errors()
                losses += [x.cpu().numpy() for x in pending[k]]
            return losses
        try:
            while any(left):
                cands = [k for k in range(len(self.groups)) if left[k]]
                ready = [k for k in cands if done_ev[k] is None or done_ev[k].query()]
                k = max(ready or cands, key=lambda c: (left[c], -c))
                g = self.groups[k]
                if streams is not None:
                    with torch.cuda.stream(streams[k]):
                        pending[k].append(g.runner.iteration().clone())
                        done_ev[k] = torch.cuda.Event()
                        done_ev[k].record()
                else:
                    pending[k].append(g.runner.iteration().clone())
                left[k] -= 1
                if on_iteration is not None:
                    on_iteration(g)
        finally:
            if streams is not None:
                for st in set(streams):
                    main.wait_stream(st)
        losses = []
        for k, g in enumerate(self.groups):
            g.pop.check_errors()
            losses += [x.cpu().numpy() for x in pending[k]]
        return losses


    def _paced_together(self) -> bool:
        """Every group runs the pipelined persistent iteration (a device-free
        env and a HIP policy step), so their rollouts can be paced together
        (AGX_TRAIN_TOGETHER=0 turns it off)."""
        if os.environ.get("AGX_TRAIN_TOGETHER", "1") == "0":
            return False
        # target-KL learns: drawing the next shuffles waits for a learner's epochs
        # run (a device sync), which must not happen while launches are resident
        if not all(((g.runner.persistent and g.pop.fused_descriptor() is not None) or g.runner.graph_persistent)
                   and g.pop.target_kl is None for g in self.groups):
            return False
        return self.co_resident_demand() <= self._cu_count()

    # partner workgroups per agent of either learner, at most (learner.hip kMaxK,
    # graph_learner.hip kMaxGK): an agent's learn holds at most this many CUs
    _MAX_PARTNERS = 16

    def co_resident_demand(self) -> int:
        """Workgroups that may have to be resident at the same time when the
        groups run together: every group's persistent rollout (all of whose
        workgroups wait on the host) and every group's partnered learner (whose
        partners spin on each other), one CU each at most.  Within the CU count,
        every such workgroup finds a CU however the launches interleave (the
        other kernels all finish); above it a rollout partly resident and a
        learner whose partners wait for its CUs could wait on each other, so
        the groups then run one after another."""
        return sum(int(g.runner.n_wg) + self._MAX_PARTNERS * g.pop.P for g in self.groups)

    def _cu_count(self) -> int:
        if not hasattr(self, "_cus"):
            self._cus = int(torch.cuda.get_device_properties(self.groups[0].pop.device).multi_processor_count)
        return self._cus

    def _train_paced_together(self, left: list, streams: list, pending: list, on_iteration) -> None:
        """The groups' iterations with their rollouts paced TOGETHER: each
        round of the loop releases the next step of every running rollout
        (each group's persistent launch computes its policy step meanwhile),
        then waits for each in turn and steps its envs; a group whose rollout
        has ended starts its next iteration at once (rollout + GAE + learner
        enqueued on its stream; the launch starts when its learner is done).

        Only launches seen running (agx_rollout_ctl.started) are paced, and the
        host never waits for one that is not: a launch queued in a hardware
        queue behind another group's resident launch (a process has few, see
        GPU_MAX_HW_QUEUES) starts once that one ends, so the loop cannot stall.
        Each group's env steps, releases and launches are those of its own
        iteration() loop, in order."""
        G = len(self.groups)
        ctx = [None] * G
        running = [False] * G
        # first-use work (learner workspaces, pinned staging, the act workspace of
        # a runtime shape) while no launch is resident: a fresh group (after a
        # regroup) runs its first iteration alone, the others get their learner
        # and staging ready; nothing in the loop below may then wait for the device
        for k, g in enumerate(self.groups):
            with torch.cuda.stream(streams[k]):
                if not getattr(g.runner, "_paced_before", False):
                    if left[k]:
                        pending[k].append(g.runner.iteration().clone())
                        left[k] -= 1
                        if on_iteration is not None:
                            on_iteration(g)
                    g.runner._paced_before = True
                g.pop.prepare_learn()
        try:
            while True:
                for k in range(G):
                    if ctx[k] is None and left[k]:
                        with torch.cuda.stream(streams[k]):
                            ctx[k] = self.groups[k].runner.begin_iteration()
                        running[k] = False
                        left[k] -= 1
                live = [k for k in range(G) if ctx[k] is not None]
                if not live:
                    return
                for k in live:
                    if not running[k]:
                        running[k] = self.groups[k].runner.launch_running()
                go = [k for k in live if running[k]]
                if not go:
                    # every launch still waits for its learner (or queue): yield the core
                    # (env worker threads may need it) and poll again
                    time.sleep(0)
                    continue
                for k in go:
                    self.groups[k].runner.pace_release(ctx[k])
                for k in go:
                    g = self.groups[k]
                    g.runner.pace_wait_step(ctx[k])
                    if ctx[k].t == g.pop.T:
                        with torch.cuda.stream(streams[k]):
                            pending[k].append(g.runner.end_iteration(ctx[k]).clone())
                        ctx[k] = None
                        if on_iteration is not None:
                            on_iteration(g)
        except BaseException:
            # every launch released with the abort word first (one queued behind
            # another's would otherwise keep that one waiting), then each drained
            for k in range(G):
                if ctx[k] is not None:
                    ctx[k].lib.agx_host_signal(ctx[k].ctl, 0xFFFFFFFF)
            for k in range(G):
                if ctx[k] is not None:
                    with torch.cuda.stream(streams[k]):
                        self.groups[k].runner.abort_iteration(ctx[k])
            raise

    def steps_per_generation(self, slot: int, evo_steps: int) -> int:
        g, _ = self.group_of(slot)
        return self.iterations(evo_steps, g.learn_step) * g.pop.T * self.N

    def episode_stats(self) -> tuple[np.ndarray, np.ndarray]:
        r_sum, r_cnt = np.zeros(self.P), np.zeros(self.P)
        for g in self.groups:
            s, c = g.runner.episode_return_sum.cpu().numpy(), g.runner.episodes.cpu().numpy()
            g.runner.reset_episode_stats()
            for r, slot in enumerate(g.slots):
                r_sum[slot], r_cnt[slot] = s[r], c[r]
        return r_sum, r_cnt

    def evaluate(self, loop: int, max_steps) -> list[float]:
        """agent.test for every agent (train_on_policy.py:363-373).  Where
        every group paces persistent launches and every network has an
        evaluation layer list (runner.population_eval_ok), ALL agents run one
        pass together: ONE persistent launch (agx_ppo_eval_multi_persistent),
        each agent on its own network, over one stack of all the agents' envs.
        Otherwise each group's pass as PopulationRunner.evaluate — a
        persistent launch per pass where the group's policy step is a HIP
        kernel — one group after another, and groups on the PyTorch policy
        step stepped together (runner.run_lockstep).  A group's samples depend
        only on its agents' counters, so neither form changes any result."""
        from .runner import _EvalDriver, population_eval_ok, run_lockstep

        self._eval_calls += 1
        acc = {id(g): np.zeros(g.pop.P) for g in self.groups}
        for g in self.groups:
            g.pop.eval_rounds = self._eval_calls
        runners = [g.runner for g in self.groups]
        if population_eval_ok(runners) and (len(self.groups) == 1 or self.slot_envs is not None):
            # every agent of every group in ONE persistent launch per pass
            # (agx_ppo_eval_multi_persistent) on one stack of all their envs
            if len(self.groups) == 1:
                env, staging = runners[0].env, None
            else:
                env = StackedVecEnv([self.slot_envs[j] for g in self.groups for j in g.slots])
                staging = self._eval_staging(sum(g.pop.P for g in self.groups))
            for k in range(loop):
                d = _EvalDriver(runners[0], k, max_steps, runners=runners, env=env, staging=staging)
                if d.can_pipeline():
                    d.run_pipelined()
                else:
                    run_lockstep([d])
                res, off = d.result(), 0
                for g in self.groups:
                    acc[id(g)] += res[off:off + g.pop.P]
                    off += g.pop.P
            return self._fitness(acc, loop)
        # Groups with a HIP policy step run their passes as persistent launches,
        # ONE resident at a time: a process has few hardware queues
        # (GPU_MAX_HW_QUEUES, 4 by default), so two resident launches — or a
        # resident launch and another group's per-step kernels — can share one
        # queue, the later one waiting behind a launch that waits for the host.
        # The remaining groups (the PyTorch policy step) step together in lock
        # step with per-step launches, after the persistent passes.
        paced = [g for g in self.groups if g.runner.persistent or g.runner.graph_persistent]
        stepped = [g for g in self.groups if g not in paced]
        for k in range(loop):
            batches = [[g] for g in paced] + ([stepped] if stepped else [])
            for batch in batches:
                drivers = [(g, _EvalDriver(g.runner, k, max_steps, allow_persistent=len(batch) == 1))
                           for g in batch]
                run_lockstep([d for _, d in drivers])
                for g, d in drivers:
                    acc[id(g)] += d.result()
        return self._fitness(acc, loop)

    def _fitness(self, acc: dict, loop: int) -> list[float]:
        out = [0.0] * self.P
        for g in self.groups:
            g.runner.after_evaluation()
            f = acc[id(g)] / loop
            for r, slot in enumerate(g.slots):
                out[slot] = float(f[r])
        return out

    def _eval_staging(self, P: int):
        """Coherent host staging of the population-wide evaluation pass (obs /
        reward / done, actions, control block, per-agent plan table), kept
        for the population size it was made for."""
        from .runner import _coherent, _packed

        bufs = getattr(self, "_eval_bufs", None)
        if bufs is None or bufs[0] != P:
            from .. import _lib

            lib = _lib.load()
            pop = self.groups[0].pop
            N, D = pop.N, pop.spec.obs_dim
            _, obs, rew, done = _packed(P, N, D, owner=self)
            act = _coherent(self, P * N * 8).view(torch.int64)
            ctl = _coherent(self, int(lib.agx_ppo_rollout_graph_ctl_bytes(P, N)))
            agents = _coherent(self, int(lib.agx_ppo_eval_multi_bytes(P)))
            bufs = self._eval_bufs = (P, (obs, rew, done, act, ctl, None, agents))
        return bufs[1]

    # ------------------------------------------------------------------ #
    def local_states(self) -> list[AgentState]:
        out = []
        steps = {}  # each group's Adam step counts: one device read per group
        for j in range(self.P):
            v = self.views[j]
            pending = getattr(v, "_pending_state", None)
            if pending is not None:
                out.append(pending)
                continue
            g, r = self.group_of(j)
            if id(g) not in steps:
                steps[id(g)] = g.pop.opt.steps.tolist()
            out.append(export_state(g.pop, r, getattr(v, "_pending_learn_step", None) or g.learn_step,
                                    steps[id(g)]))
        return out

    def clone_states(self, parents: list[int], records: list[dict]) -> list[AgentState]:
        """New slot j <- the state of global agent parents[rank * P + j];
        parents on other ranks cross once per (source, destination) pair."""
        P, me = self.P, self.rank
        mine = self.local_states()
        new = [None] * P
        if self.world > 1:
            comm = torch.device("cpu") if dist.get_backend() == "gloo" else self.device
            need = [[sorted({q % P for q in parents[r * P:(r + 1) * P] if q // P == src}) if src != r else []
                     for src in range(self.world)] for r in range(self.world)]
            ops, recv, sends = [], {}, []
            for dst in range(self.world):
                rows = need[dst][me]
                if rows:
                    msg = torch.cat([torch.cat([mine[q].params, mine[q].exp_avg, mine[q].exp_avg_sq]) for q in rows])
                    sends.append(msg.to(comm))
                    ops.append(dist.P2POp(dist.isend, sends[-1], dst))
            for src in range(self.world):
                rows = need[me][src]
                if rows:
                    n = sum(3 * records[src * P + q]["_spec"].n_params for q in rows)
                    recv[src] = torch.empty(n, dtype=torch.float32, device=comm)
                    ops.append(dist.P2POp(dist.irecv, recv[src], src))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            remote = {}
            for src, buf in recv.items():
                off = 0
                for q in need[me][src]:
                    rec = records[src * P + q]
                    n = rec["_spec"].n_params
                    t = buf[off:off + 3 * n].to(self.device)
                    hp = rec["_hp"]
                    remote[src * P + q] = AgentState(copy.deepcopy(rec["_spec"]), int(hp["learn_step"]), t[:n].clone(),
                                                     t[n:2 * n].clone(), t[2 * n:].clone(), int(rec["_adam_step"]),
                                                     float(hp["lr"]), int(hp["batch_size"]),
                                                     int(hp["update_epochs"]), float(hp["ent_coef"]))
                    off += 3 * n
        for j in range(P):
            q = parents[me * P + j]
            new[j] = mine[q % P].clone() if q // P == me else remote[q].clone()
        return new

    def regroup(self, states: list[AgentState]) -> None:
        """Groups rebuilt from every slot's state: slots with equal (network
        shape, learn_step) share a PPOPopulation, in slot order."""
        key = (lambda j, s: (j, s.spec.shape_key(), s.learn_step)) if self.singleton else \
            (lambda j, s: (s.spec.shape_key(), s.learn_step))
        if self.slot_envs is None and len({key(j, s) for j, s in enumerate(states)}) > 1:
            raise NotImplementedError("agents with different networks or learn_step need one env per agent: pass "
                                      "the reference's num_envs env (cloned per agent) or a StackedVecEnv")
        order: dict[tuple, list[int]] = {}
        for j, s in enumerate(states):
            order.setdefault(key(j, s), []).append(j)
        t = self._template
        groups = []
        for k, slots in order.items():
            learn_step = k[-1]
            st = [states[j] for j in slots]
            spec = st[0].spec
            pop = PPOPopulation(spec, len(slots), self.N, learn_step=learn_step,
                                batch_size=max(s.batch_size for s in st), lr=[s.lr for s in st], gamma=t.gamma,
                                gae_lambda=t.gae_lambda, clip_coef=t.clip_coef, ent_coef=st[0].ent_coef,
                                vf_coef=t.vf_coef, max_grad_norm=t.max_grad_norm,
                                update_epochs=max(s.update_epochs for s in st), target_kl=t.target_kl,
                                device=self.device, fused=t.fused, perm_source=t.perm_source,
                                action_masks=t.use_action_masks, global_pop_size=t.global_P, seed_base=t.seed_base,
                                agent_ids=[self.rank * self.P + j for j in slots], init_params=False)
            n = spec.n_params
            with torch.no_grad():
                for r, s in enumerate(st):
                    pop.params.data[r, :n].copy_(s.params)
                    pop.opt.exp_avg[r, :n].copy_(s.exp_avg)
                    pop.opt.exp_avg_sq[r, :n].copy_(s.exp_avg_sq)
                    pop.opt.steps[r] = s.step
                    pop.opt.lr[r] = s.lr
                    pop.set_agent_hparam(r, "batch_size", s.batch_size)
                    pop.set_agent_hparam(r, "update_epochs", s.update_epochs)
                    pop.set_agent_hparam(r, "ent_coef", s.ent_coef)
                    pop.set_host_hparams(r, lr=s.lr)
            env = (StackedVecEnv([self.slot_envs[j] for j in slots]) if self.slot_envs is not None
                   else self.groups[0].runner.env)
            groups.append(_Group(pop, PopulationRunner(pop, env), slots, learn_step))
        self.groups = groups
        for g in groups:
            for r, slot in enumerate(g.slots):
                v = self.views[slot]
                v.population, v.row = g.pop, r
                v._pending_state = None
                v._pending_learn_step = None
                v._learn_step = g.learn_step
        self.refresh_plan()

    def pending(self) -> bool:
        return any(getattr(v, "_pending_state", None) is not None or getattr(v, "_pending_learn_step", None)
                   for v in self.views)



# The groups' training streams: non-blocking streams (agx_stream_create) made
# once per process, as many as the process has hardware queues
# (GPU_MAX_HW_QUEUES, 4 by default): streams are given hardware queues in
# turn, so consecutive groups land on different queues and a group's rollout
# does not wait in a queue behind another group's learner.  Group k trains on
# stream k mod that count.
_TRAIN_STREAMS: list = []


def _train_stream(k: int):
    from .. import _lib

    n = max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    while len(_TRAIN_STREAMS) < n:
        h = _lib.load().agx_stream_create()
        if not h:
            raise _lib.AgxError(_lib.load().agx_last_error().decode(errors="replace"))
        _TRAIN_STREAMS.append(torch.cuda.ExternalStream(h))
    return _TRAIN_STREAMS[k % n]
