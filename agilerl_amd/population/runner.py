"""Host env workers <-> HBM rollout SoA for a whole population.

Reference: agilerl/rollouts/on_policy.py:23-203 (one agent at a time, CPU
TensorDicts, a forward + ``.cpu()`` sync per step).  Here one vector step of
EVERY agent is, on the fused path (agx_ppo_rollout_step):

  1. ONE launch: scatter the staged obs into rollout slot t, the staged
     reward/done of step t-1 into slot t-1 (+ episode accounting), and the
     policy step (MFMA forward, Gumbel-max sample) writing action / log-prob /
     value into slot t and the P*N actions;
  2. an event wait (the only synchronisation);
  3. the host env step, writing obs / reward / done straight into ONE packed
     pinned staging buffer.
The staging buffer and the action buffer are pinned host memory that the
kernel reads / writes directly (zero-copy over the host link: 40 KB in and
8 KB out per step at config 2), so a step is one launch and one wait; with
AGX_ZERO_COPY=0 the staging goes through one H2D and one D2H copy instead.

Persistent mode (AGX_PERSISTENT_ROLLOUT: "auto" default, "1" always, "0"
never): the whole
rollout is ONE launch (agx_ppo_rollout_persistent) whose workgroups keep the
parameters in LDS and are paced step by step through a control block in
coherent host memory — the host releases step t after the env step
(agx_host_signal) and spins on the workgroups' done words (agx_host_wait),
so a vector step costs no launch and no event wait.  Staging, actions and
the control block then live in coherent (fine-grained) host memory, which
the device re-reads within one launch.

From the persistent launch to the host's final release the device waits
for the host thread, so nothing the env does in its step may wait for the
device (``torch.cuda.synchronize()``, a ``.item()`` on a CUDA tensor, a
blocking copy, ``hipHostFree``): it would stall the rollout until its
timeout.  "auto" therefore paces a persistent rollout only for envs that
declare ``agx_device_free = True`` (the synthetic envs, and a StackedVecEnv
whose every env declares it); any other env gets one launch per vector step,
where its step may use the device freely.  A gymnasium env that does not touch
the GPU can opt in by setting the attribute.

Architectures outside the fused kernels use the plain-PyTorch policy step
with per-field copies (``_collect_torch``).
"""

from __future__ import annotations

import ctypes
import os
import weakref

import numpy as np
import torch

from .. import _lib
from .ppo_pop import PPOPopulation


class AgxRolloutIO(ctypes.Structure):
    """Mirror of ``agx_rollout_io`` (include/agx.h)."""

    _fields_ = [
        ("stage_obs", ctypes.c_void_p), ("stage_rew", ctypes.c_void_p), ("stage_done", ctypes.c_void_p),
        ("obs_slot", ctypes.c_void_p), ("obs_agent_stride", ctypes.c_int64),
        ("rewards_prev", ctypes.c_void_p), ("dones_prev", ctypes.c_void_p), ("prev_agent_stride", ctypes.c_int64),
        ("actions", ctypes.c_void_p), ("log_probs", ctypes.c_void_p), ("values", ctypes.c_void_p),
        ("slot_agent_stride", ctypes.c_int64), ("actions_flat", ctypes.c_void_p),
        ("scores", ctypes.c_void_p), ("return_sum", ctypes.c_void_p), ("episodes", ctypes.c_void_p),
        ("stage_mask", ctypes.c_void_p), ("mask_slot", ctypes.c_void_p), ("mask_agent_stride", ctypes.c_int64),
        ("agent_env_base", ctypes.c_void_p),
    ]


class AgxEvalTally(ctypes.Structure):
    """Mirror of ``agx_eval_tally`` (include/agx_graph.h)."""

    _fields_ = [("stage_rew", ctypes.c_void_p), ("stage_done", ctypes.c_void_p), ("scores", ctypes.c_void_p),
                ("completed", ctypes.c_void_p), ("finished", ctypes.c_void_p), ("fin_words", ctypes.c_void_p),
                ("prev", ctypes.c_int)]


# hipHostFree waits for the whole device.  A persistent rollout of this
# process waits for the host from its launch until the host's final release,
# so a free in that window (a garbage-collected runner's buffers, finalised in
# the middle of another runner's env step) stalls the rollout until its
# timeout.  Frees that come while a rollout is being paced are deferred to
# the end of the pacing.
_PACING = 0
_DEFERRED_FREES: list[int] = []
# Coherent buffers of retired runners, by size: the population engine rebuilds
# its groups every generation with the same staging sizes, so a buffer goes
# back to this pool instead of hipHostFree (which waits for the device) and the
# next runner of that size takes it instead of a fresh hipHostMalloc.
_HOST_POOL: dict[int, list[int]] = {}
_HOST_POOL_MAX = 64  # buffers kept per size; the rest are freed


def _host_free(p: int, nbytes: int | None = None) -> None:
    if nbytes is not None:
        pool = _HOST_POOL.setdefault(nbytes, [])
        if len(pool) < _HOST_POOL_MAX:
            pool.append(p)
            return
    if _PACING:
        _DEFERRED_FREES.append(p)
    else:
        _lib.load().agx_host_free(p)


def _pacing_begin() -> None:
    global _PACING
    _PACING += 1


def _pacing_end() -> None:
    global _PACING
    _PACING -= 1
    if not _PACING:
        lib = _lib.load()
        while _DEFERRED_FREES:
            lib.agx_host_free(_DEFERRED_FREES.pop())


def _device_sync() -> None:
    torch.cuda.synchronize()


def _coherent(owner, nbytes: int) -> torch.Tensor:
    """Zeroed uint8 CPU tensor over agx_host_alloc memory (coherent,
    device-accessible at the same address), returned to the size pool when its
    owner is collected (see _host_free).

    A pooled buffer's previous owner may still have device work queued that
    reads or writes it (a launch's control words, a learner's skip word, a
    tally's fin words): it is reused only after the device has drained, and
    never inside a pacing window (where the device waits for this thread), in
    which case a fresh buffer is allocated instead."""
    pool = _HOST_POOL.get(nbytes) if not _PACING else None
    if pool:
        _device_sync()
        p = pool.pop()
        ctypes.memset(p, 0, nbytes)
    else:
        lib = _lib.load()
        p = lib.agx_host_alloc(nbytes)
        if not p:
            raise _lib.AgxError(lib.agx_last_error().decode(errors="replace"))
        ctypes.memset(p, 0, nbytes)
    weakref.finalize(owner, _host_free, p, nbytes)
    return torch.from_numpy(np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)))


def _packed(P: int, N: int, D: int, owner=None, obs_dtype=torch.float32, **kw):
    """One byte buffer [obs P*N*D (f32, or uint8 frames) | reward f32 P*N |
    done u8 P*N] + views (the reward stays 4-byte aligned)."""
    isz = torch.empty(0, dtype=obs_dtype).element_size()
    n_obs, n_rew = (P * N * D * isz + 15) // 16 * 16, P * N * 4
    nbytes = (n_obs + n_rew + P * N + 15) // 16 * 16
    buf = _coherent(owner, nbytes) if owner is not None else torch.zeros(nbytes, dtype=torch.uint8, **kw)
    obs = buf[:P * N * D * isz].view(obs_dtype).view(P * N, D)
    rew = buf[n_obs:n_obs + n_rew].view(torch.float32)
    done = buf[n_obs + n_rew:n_obs + n_rew + P * N].view(torch.bool)
    return buf, obs, rew, done


class PopulationRunner:
    def __init__(self, pop: PPOPopulation, env):
        if env.num_envs != pop.P * pop.N:
            raise ValueError(f"env has {env.num_envs} envs, population needs P*N = {pop.P * pop.N}")
        self.pop, self.env = pop, env
        P, N, D = pop.P, pop.N, pop.spec.obs_dim
        dev = pop.device
        self.zero_copy = os.environ.get("AGX_ZERO_COPY", "1") != "0"
        desc = pop.fused_descriptor()
        gdesc = pop.learn_descriptor() if desc is None else None  # a mutated (runtime-shape) network
        mode = os.environ.get("AGX_PERSISTENT_ROLLOUT", "auto")
        paced = self.zero_copy and mode != "0" and (mode == "1" or bool(getattr(env, "agx_device_free", False)))
        # every workgroup of a persistent launch must be co-resident (the host
        # paces them in lock step); larger grids take per-step launches
        lib = _lib.load()
        self.persistent = bool(paced and desc is not None and
                               lib.agx_rollout_workgroups(P, N) <= lib.agx_rollout_max_workgroups(ctypes.byref(desc)))
        self.graph_persistent = bool(paced and gdesc is not None and pop.obs.dtype == torch.float32 and
                                     lib.agx_ppo_rollout_graph_workgroups(P, N) <=
                                     lib.agx_ppo_rollout_graph_max_workgroups())
        if self.persistent or self.graph_persistent:
            self.stage_h, self.obs_h, self.rew_h, self.done_h = _packed(P, N, D, owner=self)
            self.act_h = _coherent(self, P * N * 8).view(torch.int64)
            self.n_wg = int(lib.agx_ppo_rollout_graph_workgroups(P, N) if self.graph_persistent
                            else lib.agx_rollout_workgroups(P, N))
            self.ctl_h = _coherent(self, self._ctl_bytes())
            self.args_h = _coherent(self, int(lib.agx_rollout_args_bytes(pop.T + 1)))
            self.seq_base = 0
            self.timeout_s = float(os.environ.get("AGX_ROLLOUT_TIMEOUT", "20"))
        else:
            self.stage_h, self.obs_h, self.rew_h, self.done_h = _packed(P, N, D, obs_dtype=pop.obs.dtype,
                                                                        pin_memory=True)
            self.act_h = torch.zeros(P * N, dtype=torch.int64, pin_memory=True)
        self.stage_d, self.obs_d, self.rew_d, self.done_d = _packed(P, N, D, obs_dtype=pop.obs.dtype, device=dev)
        self.term_h = torch.zeros(P * N, dtype=torch.bool, pin_memory=True)
        self.act_d = torch.zeros(P * N, dtype=torch.int64, device=dev)
        self.last_obs = torch.zeros(P, N, D, dtype=pop.obs.dtype, device=dev)
        self.last_done = torch.zeros(P, N, dtype=torch.uint8, device=dev)
        self.last_value = torch.zeros(P, N, dtype=torch.float32, device=dev)
        self.last_value_valid = False
        self.ev = torch.cuda.Event()
        self.started = False
        self.env_steps = 0
        # per-env episode accounting (on_policy.py:147-172), reduced per agent on demand
        self.scores = torch.zeros(P * N, dtype=torch.float32, device=dev)
        self.ret_sum_env = torch.zeros(P * N, dtype=torch.float64, device=dev)
        self.episodes_env = torch.zeros(P * N, dtype=torch.int64, device=dev)
        self._ios = None
        self._np = None
        self._ctl_words = None
        self.stats_event = None

    def _ctl_bytes(self) -> int:
        lib, P, N = _lib.load(), self.pop.P, self.pop.N
        return int(lib.agx_ppo_rollout_graph_ctl_bytes(P, N) if self.graph_persistent
                   else lib.agx_rollout_ctl_bytes(P, N))

    # ------------------------------------------------------------------ #
    @property
    def episode_return_sum(self) -> torch.Tensor:
        return self.ret_sum_env.view(self.pop.P, self.pop.N).sum(1)

    @property
    def episodes(self) -> torch.Tensor:
        return self.episodes_env.view(self.pop.P, self.pop.N).sum(1)

    def reset_episode_stats(self) -> None:
        self.ret_sum_env.zero_()
        self.episodes_env.zero_()

    # ------------------------------------------------------------------ #
    def _build_ios(self):
        """agx_rollout_io for every step t = 0..T (t = T: final scatter only)."""
        pop = self.pop
        T, N, D = pop.T, pop.N, pop.spec.obs_dim
        ios = (AgxRolloutIO * (T + 1))()
        for t in range(T + 1):
            io = AgxRolloutIO()
            src_obs, src_rew, src_done = ((self.obs_h, self.rew_h, self.done_h) if self.zero_copy
                                          else (self.obs_d, self.rew_d, self.done_d))
            io.stage_obs = src_obs.data_ptr()
            if t > 0:
                io.stage_rew = src_rew.data_ptr()
                io.stage_done = src_done.data_ptr()
                io.rewards_prev = pop.rewards[:, t - 1].data_ptr()
                io.dones_prev = pop.dones[:, t - 1].data_ptr()
                io.scores = self.scores.data_ptr()
                io.return_sum = self.ret_sum_env.data_ptr()
                io.episodes = self.episodes_env.data_ptr()
            if t < T:
                io.obs_slot = pop.obs[:, t].data_ptr()
                io.obs_agent_stride = T * N * D
                io.actions = pop.actions[:, t].data_ptr()
                io.log_probs = pop.log_probs[:, t].data_ptr()
                io.values = pop.values[:, t].data_ptr()
                io.actions_flat = (self.act_h if self.zero_copy else self.act_d).data_ptr()
                io.slot_agent_stride = T * N
            else:  # final obs -> last_obs + bootstrap value
                io.obs_slot = self.last_obs.data_ptr()
                io.obs_agent_stride = N * D
                io.values = self.last_value.data_ptr()
                io.slot_agent_stride = N
            io.prev_agent_stride = T * N
            io.agent_env_base = pop.env_base_d.data_ptr()  # each agent samples its global envs' streams
            ios[t] = io
        self._ios = ios

    def _env_step(self) -> None:
        # numpy views of the staging made once (Tensor.numpy() costs ~1-3 us a call)
        if self._np is None:
            self._np = (self.act_h.numpy(), self.obs_h.numpy(), self.rew_h.numpy(), self.done_h.numpy(),
                        self.term_h.numpy())
        act, obs, rew, done, term_np = self._np
        _, _, term, trunc, _ = self.env.step(act, out_obs=obs, out_rew=rew, out_done=done)
        if trunc is not None and np.count_nonzero(trunc):  # done = term | trunc (on_policy.py:121-126)
            done |= trunc
        np.copyto(term_np, term)

    @torch.no_grad()
    def collect(self) -> None:
        pop, env = self.pop, self.env
        desc = pop.fused_descriptor()
        if desc is None and not self.graph_persistent:
            return self._collect_torch()
        P, N, T = pop.P, pop.N, pop.T
        if self._ios is None:
            self._build_ios()
        if not self.started:
            env.reset(out_obs=self.obs_h.numpy())
            if not self.zero_copy:
                self.stage_d.copy_(self.stage_h, non_blocking=True)
            self.started = True
        if self.persistent or self.graph_persistent:
            return self._collect_persistent(desc)
        lib = _lib.load()
        fn = lib.agx_ppo_rollout_step
        dref = ctypes.byref(desc)
        params = pop.params.data.data_ptr()
        s = _lib.stream()
        for t in range(T):
            pop.act_counter += 1
            _lib.check(fn(dref, P, N, params, ctypes.byref(self._ios[t]), 1, 1, pop.act_seed, pop.act_counter, s),
                       "agx_ppo_rollout_step")
            if not self.zero_copy:
                self.act_h.copy_(self.act_d, non_blocking=True)
            self.ev.record()
            self.ev.synchronize()
            self._env_step()
            if not self.zero_copy:
                self.stage_d.copy_(self.stage_h, non_blocking=True)
        # reward/done of the last step -> slot T-1; final obs -> last_obs + bootstrap value
        _lib.check(fn(dref, P, N, params, ctypes.byref(self._ios[T]), 1, 0, pop.act_seed, 0, s),
                   "agx_ppo_rollout_step")
        self._mark_stats()
        self.last_value_valid = True
        self.last_done.view(-1).copy_(self.term_h.view(torch.uint8), non_blocking=True)  # last_done = term (:196)
        self.env_steps += P * N * T

    def _collect_persistent(self, desc) -> None:
        """One launch for the whole rollout; the host paces it step by step."""
        _pacing_begin()
        try:
            lib, ctl, base = self._launch_persistent(desc)
            self._pace_persistent(lib, ctl, base)
        finally:
            _pacing_end()
        self._finish_persistent()

    def _launch_persistent(self, desc):
        pop = self.pop
        P, N, T = pop.P, pop.N, pop.T
        lib = _lib.load()
        ctl = self.ctl_h.data_ptr()
        base = self.seq_base
        if base + T + 1 >= 0xFFFFFFF0:  # never in practice: 2^32 / (T + 1) rollouts
            torch.cuda.current_stream().synchronize()
            self.ctl_h.zero_()
            base = 0
        if self.graph_persistent:  # a mutated shape: the runtime-shape policy step in the same loop
            from .learner import graph_act_workspace

            gdesc = pop.learn_descriptor()
            ws = graph_act_workspace(pop, gdesc)[1]
            _lib.check(lib.agx_ppo_rollout_graph_persistent(ctypes.byref(gdesc), P, N, pop.params.data.data_ptr(),
                                                            self._ios, T + 1, base, pop.act_seed, pop.act_counter,
                                                            self.args_h.data_ptr(), ctl, self.timeout_s,
                                                            ws.data_ptr(), _lib.stream()),
                       "agx_ppo_rollout_graph_persistent")
        else:
            _lib.check(lib.agx_ppo_rollout_persistent(ctypes.byref(desc), P, N, pop.params.data.data_ptr(),
                                                      self._ios, T + 1, base, pop.act_seed, pop.act_counter,
                                                      self.args_h.data_ptr(), ctl, self.timeout_s, _lib.stream()),
                       "agx_ppo_rollout_persistent")
        self.seq_base = base + T + 1
        self._mark_stats()
        return lib, ctl, base

    def _mark_stats(self) -> None:
        """Event after the rollout's last episode-accounting write: the
        generation step reads the episode statistics behind it (on a side
        stream) instead of behind everything queued after the rollout."""
        if self.stats_event is None:
            self.stats_event = torch.cuda.Event()
        self.stats_event.record()

    def _pace_persistent(self, lib, ctl, base) -> None:
        T = self.pop.T
        try:
            for t in range(T):
                lib.agx_host_signal(ctl, base + t + 1)
                _lib.check(lib.agx_host_wait(ctl, self.n_wg, base + t + 1, self.timeout_s), "agx_host_wait")
                self._env_step()
            lib.agx_host_signal(ctl, base + T + 1)  # reward/done of step T-1, final obs, bootstrap value
        except BaseException:
            lib.agx_host_signal(ctl, 0xFFFFFFFF)  # release the workgroups, then reset the block
            torch.cuda.current_stream().synchronize()
            self.ctl_h.zero_()
            self.seq_base = 0
            raise
        self.pop.act_counter += T
        self.env_steps += self.pop.P * self.pop.N * T

    def _finish_persistent(self) -> None:
        # stream-ordered after the rollout kernel, which ends only after the
        # host's final release — by then the last env step has written term_h
        self.last_value_valid = True
        v = self.__dict__.get("_done_views")
        if v is None:
            v = self._done_views = (self.last_done.view(-1), self.term_h.view(torch.uint8))
        v[0].copy_(v[1], non_blocking=True)  # last_done = term (:196)

    @torch.no_grad()
    def _collect_torch(self) -> None:
        pop, env = self.pop, self.env
        P, N, T = pop.P, pop.N, pop.T
        if not self.started:
            env.reset(out_obs=self.obs_h.numpy())
            self.last_obs.copy_(self.obs_h.view(P, N, -1), non_blocking=True)
            self.started = True
        self.last_value_valid = False
        pop.obs[:, 0].copy_(self.last_obs)
        for t in range(T):
            pop.act_into(t, self.act_d)
            self.act_h.copy_(self.act_d, non_blocking=True)
            self.ev.record()
            self.ev.synchronize()
            self._env_step()
            pop.rewards[:, t].copy_(self.rew_h.view(P, N), non_blocking=True)
            pop.dones[:, t].copy_(self.done_h.view(torch.uint8).view(P, N), non_blocking=True)
            nxt = pop.obs[:, t + 1] if t + 1 < T else self.last_obs
            nxt.copy_(self.obs_h.view(P, N, -1), non_blocking=True)
            r = pop.rewards[:, t].reshape(-1)
            d = pop.dones[:, t].reshape(-1).bool()
            self.scores += r
            self.ret_sum_env += torch.where(d, self.scores, 0.0).double()
            self.episodes_env += d.long()
            self.scores.masked_fill_(d, 0.0)
        gdesc = pop.learn_descriptor()
        if gdesc is not None:  # a mutated shape: the bootstrap value from the runtime-shape kernel too
            from .learner import policy_step_graph

            policy_step_graph(pop, gdesc, self.last_obs, N * pop.spec.obs_dim, sample=False, counter=0,
                              values=self.last_value, out_agent_stride=N)
            self.last_value_valid = True
        self._mark_stats()
        self.last_done.view(-1).copy_(self.term_h.view(torch.uint8), non_blocking=True)
        self.env_steps += P * N * T

    @torch.no_grad()
    def evaluate(self, loop: int = 1, max_steps: int | None = None) -> np.ndarray:
        """Fitness of every agent at once: PPO.test (ppo.py:1113-1289) run for
        the whole population on its env slices — agent p acts on envs
        [p*N, (p+1)*N) with the sampled policy step; each env's first finished
        episode score counts, ``max_steps`` ends the pass; mean over envs, then
        over ``loop`` passes.  The env is reset per pass (as test() does), so
        the next rollout starts from a fresh reset like the reference's next
        collect_rollouts (on_policy.py:50-56).  -> float64 [P].

        Compiled shapes on a device-free env run the pass as ONE persistent
        launch (agx_ppo_eval_persistent, paced like the rollout); other
        shapes launch the policy step per vector step (_EvalDriver)."""
        pop = self.pop
        pop.eval_rounds = getattr(pop, "eval_rounds", 0) + 1
        out = np.zeros((loop, pop.P))
        for k in range(loop):
            d = _EvalDriver(self, k, max_steps)
            if d.can_pipeline():
                d.run_pipelined()
            else:
                run_lockstep([d])
            out[k] = d.result()
        self.after_evaluation()
        return out.mean(0)

    def _eval_staging(self):
        """Coherent host buffers of the persistent evaluation (allocated on
        first use): packed obs / reward / done staging, actions, a control
        block of its own and the per-step arguments of one launch, plus the
        stream is assigned by run_lockstep)."""
        if getattr(self, "_eval_bufs", None) is None:
            pop = self.pop
            P, N, D = pop.P, pop.N, pop.spec.obs_dim
            lib = _lib.load()
            _, obs, rew, done = _packed(P, N, D, owner=self)
            act = _coherent(self, P * N * 8).view(torch.int64)
            # room for the group's own evaluation launch and the population-wide one
            ctl = _coherent(self, max(self._ctl_bytes(), int(lib.agx_ppo_rollout_graph_ctl_bytes(P, N))))
            args = _coherent(self, int(lib.agx_rollout_args_bytes(_EVAL_CHUNK)))
            agents = _coherent(self, int(lib.agx_ppo_eval_multi_bytes(P)))
            self._eval_bufs = (obs, rew, done, act, ctl, args, agents)
        return self._eval_bufs

    def after_evaluation(self) -> None:
        self.started = False  # the next collect() starts from env.reset()
        self.last_value_valid = False
        self.scores.zero_()

    def iteration(self) -> torch.Tensor:
        """collect -> bootstrap + GAE -> learn; returns per-agent mean loss (device)."""
        desc = self.pop.fused_descriptor()
        if (self.persistent and desc is not None) or self.graph_persistent:
            return self._iteration_pipelined(desc)
        self.collect()
        self.pop.finish_rollout(self.last_obs, self.last_done,
                                self.last_value if self.last_value_valid else None)
        return self.pop.learn()

    @torch.no_grad()
    def _iteration_pipelined(self, desc) -> torch.Tensor:
        """The persistent rollout, the last_done copy, GAE and the learner are
        all enqueued on the stream BEFORE the host paces the rollout: the GPU
        runs rollout -> GAE -> learner back to back with no host launch gap
        (the host-side launch work overlaps the rollout instead of sitting
        between it and the learner).  Same launches, same order, same data as
        collect() + finish_rollout() + learn().  If the host loop raises (or
        the pacing times out), the workgroups are released with the abort /
        timeout word set in the control block; the queued learner reads that
        word first (``skip_if_set``) and returns without touching parameters
        or Adam state, and the exception propagates."""
        c = self.begin_iteration()
        try:
            while c.t < self.pop.T:
                self.pace_release(c)
                self.pace_wait_step(c)
        except BaseException:
            self.abort_iteration(c)
            raise
        return self.end_iteration(c)

    # -- an iteration in parts: a host pacing several groups' rollouts at once
    # (PopulationEngine.train) interleaves their pace_release / pace_wait_step
    def begin_iteration(self) -> "_IterCtx":
        """Everything of the pipelined iteration but the pacing: the persistent
        rollout launch (its control block's ``started`` word cleared first), the
        last_done copy, GAE and the learner, enqueued on the current stream.
        Nothing here waits for the device."""
        desc = self.pop.fused_descriptor()
        if self._ios is None:
            self._build_ios()
        if not self.started:
            self.env.reset(out_obs=self.obs_h.numpy())
            self.started = True
        self.pop.prepare_learn()  # nothing between the launch and the pacing may wait for the device
        if self._ctl_words is None:
            self._ctl_words = self.ctl_h.numpy().view(np.uint32)
        self._ctl_words[3] = 0  # agx_rollout_ctl.started
        _pacing_begin()
        try:
            lib, ctl, base = self._launch_persistent(desc)
            self._finish_persistent()
            self.pop.finish_rollout(self.last_obs, self.last_done, self.last_value)
            # the learner reads the control block's timeout word when it starts:
            # set by an aborted (host exception) or timed-out rollout, so the
            # partial rollout never updates the parameters or Adam state
            loss = self.pop.learn(prefetch=False, skip_if_set=ctl + 4)
        except BaseException:
            _pacing_end()
            raise
        return _IterCtx(lib, ctl, base, loss)

    def launch_running(self) -> bool:
        """Every workgroup of the current persistent rollout launch is resident
        (agx_rollout_ctl.started counts them): a launch only partly resident is
        not paced, so the host never waits on workgroups that cannot start."""
        return int(self._ctl_words[3]) >= self.n_wg

    def pace_release(self, c: "_IterCtx") -> None:
        c.lib.agx_host_signal(c.ctl, c.base + c.t + 1)

    def pace_wait_step(self, c: "_IterCtx") -> None:
        """Wait for released step c.t, step the env; after the last step the
        release of the final obs / bootstrap value."""
        _lib.check(c.lib.agx_host_wait(c.ctl, self.n_wg, c.base + c.t + 1, self.timeout_s), "agx_host_wait")
        self._env_step()
        c.t += 1
        if c.t == self.pop.T:
            c.lib.agx_host_signal(c.ctl, c.base + self.pop.T + 1)  # reward/done of step T-1, final obs, bootstrap value

    def abort_iteration(self, c: "_IterCtx") -> None:
        """Release the workgroups with the abort word (the queued learner then
        skips), wait for the stream, reset the control block."""
        try:
            c.lib.agx_host_signal(c.ctl, 0xFFFFFFFF)
            torch.cuda.current_stream().synchronize()
            self.ctl_h.zero_()
            self.seq_base = 0
        finally:
            _pacing_end()

    def end_iteration(self, c: "_IterCtx") -> torch.Tensor:
        self.pop.act_counter += self.pop.T
        self.env_steps += self.pop.P * self.pop.N * self.pop.T
        _pacing_end()
        if self.pop.prefetch_perms:  # next learn's minibatch orders: host work while the GPU learns
            self.pop.prefetch_permutations()
        return c.loss


class _IterCtx:
    """An enqueued pipelined iteration being paced: its control block, release
    base, the learner's loss tensor and the next step to release."""

    __slots__ = ("lib", "ctl", "base", "loss", "t")

    def __init__(self, lib, ctl, base, loss):
        self.lib, self.ctl, self.base, self.loss, self.t = lib, ctl, base, loss, 0


# ---------------------------------------------------------------------- #
# evaluation (PPO.test, ppo.py:1113-1289) for one group, steppable in lock
# step with other groups' passes
# ---------------------------------------------------------------------- #
#: vector steps per persistent evaluation launch (a pass that needs more takes
#: another launch); the per-step arguments of a launch sit in coherent host memory
_EVAL_CHUNK = 1024


def _eval_nets(runners: list) -> tuple | None:
    """(per-agent ctypes array of agx_ppo_graph pointers, [edesc per runner])
    when every runner's network has an evaluation layer list, else None."""
    descs = [r.pop.eval_descriptor() for r in runners]
    if any(d is None for d in descs):
        return None
    ptrs = [ctypes.cast(ctypes.pointer(d), ctypes.c_void_p).value for r, d in zip(runners, descs) for _ in range(r.pop.P)]
    return (ctypes.c_void_p * len(ptrs))(*ptrs), descs


def population_eval_ok(runners: list, paced: bool = True) -> bool:
    """Whether the runners' agents can be evaluated together in ONE persistent
    launch (agx_ppo_eval_multi_persistent): every runner paces persistent
    launches (a device-free env; not asked with paced=False), every network
    has an evaluation layer list, one env width, and the kernel takes the
    whole grid."""
    if not runners or (paced and not all(r.persistent or r.graph_persistent for r in runners)):
        return False
    pops = [r.pop for r in runners]
    if len({(p.N, p.spec.obs_dim, p.spec.n_actions) for p in pops}) != 1:
        return False
    if any(p.obs.dtype != torch.float32 for p in pops):
        return False
    nets = _eval_nets(runners)
    if nets is None:
        return False
    P = sum(p.P for p in pops)
    return bool(_lib.load().agx_ppo_eval_multi_supported(nets[0], P, pops[0].N))


class _EvalDriver:
    """One evaluation pass of one group — or of several groups together
    (``runners``: the population engine's groups, on the stacked ``env``
    holding their envs in order): reset, then per vector step the sampled
    policy step of every agent (evaluation counters ``(1 << 41) +
    (eval_round << 24) + (k << 20) + step``, the agent's own Philox stream),
    the env step, and each env's first finished episode score.  Persistent
    mode keeps ONE launch resident for the pass and paces it through its own
    control block: agx_ppo_eval_multi_persistent (every agent on its own
    network, all groups at once) where population_eval_ok holds, else the
    group's agx_ppo_eval_persistent / agx_ppo_eval_graph_persistent;
    otherwise one policy-step launch + event wait per step (the evaluation
    layer list when the multi form is available, so both give the same
    samples)."""

    def __init__(self, runner: "PopulationRunner", k: int, max_steps: int | None, allow_persistent: bool = True,
                 runners: list | None = None, env=None, staging=None):
        self.runners = list(runners) if runners else [runner]
        self.runner, self.pop = runner, runner.pop
        self.env = env if env is not None else runner.env
        pops = [r.pop for r in self.runners]
        pop = self.pop
        P, N, D = sum(p.P for p in pops), pop.N, pop.spec.obs_dim
        self.P, self.N, self.D = P, N, D
        self.max_steps = max_steps
        self.counter0s = [(1 << 41) + (int(p.eval_rounds) << 24) + (k << 20) for p in pops]
        self.counter0 = self.counter0s[0]
        capable = population_eval_ok(self.runners, paced=False)
        self.multi = bool(allow_persistent and capable and population_eval_ok(self.runners))
        self.device_tally = False
        if len(self.runners) > 1 and not self.multi:
            raise ValueError("several groups evaluate together only in the population-wide launch")
        self.desc = pop.fused_descriptor()
        self.gdesc = pop.learn_descriptor() if self.desc is None else None
        # the evaluation layer list wherever the multi form can run, per-step
        # launches included: persistent and per-step passes then sample alike
        self.edescs = _eval_nets(self.runners)[1] if capable else None
        self.persistent = bool(self.multi or (allow_persistent and (
            (runner.persistent and self.desc is not None) or (runner.graph_persistent and self.gdesc is not None))))
        self.step = 0
        self.scores = np.zeros(P * N)
        self.completed = np.zeros(P * N)
        self.finished = np.zeros(P * N, dtype=bool)
        self.n_finished = 0
        lib = _lib.load()
        if self.persistent:
            st = staging if staging is not None else runner._eval_staging()
            self.obs_h, self.rew_h, self.done_h, self.act_h, self.ctl_h, self.args_h = st[:6]
            self.launched_to = 0  # steps covered by launches so far (0: no launch resident)
            # per-step host work kept to the env step: numpy views of the staging
            # and the control-block entry points, taken once
            self._views = (self.obs_h.numpy(), self.rew_h.numpy(), self.done_h.numpy(), self.act_h.numpy())
            self._signal, self._wait_fn, self._ctl = lib.agx_host_signal, lib.agx_host_wait, self.ctl_h.data_ptr()
            if self.multi:
                self.n_wg = int(lib.agx_ppo_rollout_graph_workgroups(P, N))
                nets = _eval_nets(self.runners)
                self._nets = nets[0]
                self._params = (ctypes.c_void_p * P)(*[r.pop.params.data[a].data_ptr()
                                                       for r in self.runners for a in range(r.pop.P)])
                self._env_base = (ctypes.c_int64 * P)(*[int(i) * N for r in self.runners for i in r.pop.agent_ids])
                self._seeds = (ctypes.c_uint64 * P)(*[r.pop.act_seed for r in self.runners for _ in range(r.pop.P)])
                self._ctr0 = [c for r, c in zip(self.runners, self.counter0s) for _ in range(r.pop.P)]
                nb = int(lib.agx_ppo_eval_multi_bytes(P))
                self._agents_h = st[6] if len(st) > 6 else _coherent(self, nb)
                self._agents_d = torch.empty(nb, dtype=torch.uint8, device=pop.device)  # before any launch
                # the episode tally on the device (a pass to the end of every episode):
                # the host then only sums the workgroups' finished counts
                self.device_tally = max_steps is None and os.environ.get("AGX_EVAL_DEVICE_TALLY", "1") != "0"
                if self.device_tally:
                    dev = pop.device
                    self._t_scores = torch.zeros(P * N, dtype=torch.float64, device=dev)
                    self._t_completed = torch.zeros(P * N, dtype=torch.float64, device=dev)
                    self._t_finished = torch.zeros(P * N, dtype=torch.uint8, device=dev)
                    self._t_fin = _coherent(self, 4 * self.n_wg).view(torch.int32)
                    self._t_fin_np = self._t_fin.numpy()
                    # every workgroup's env count: the pass ends when the counts reach
                    # them (one byte compare per step instead of a numpy sum)
                    gx = self.n_wg // P
                    self._fin_all = np.array([min(16, N - 16 * x) for x in range(gx)] * P, dtype=np.int32).tobytes()
                    self._tally = AgxEvalTally(self.rew_h.data_ptr(), self.done_h.data_ptr(),
                                               self._t_scores.data_ptr(), self._t_completed.data_ptr(),
                                               self._t_finished.data_ptr(), self._t_fin.data_ptr(), 0)
            else:
                self.n_wg = runner.n_wg
        else:
            self.act_d = torch.empty(P * N, dtype=torch.int64, device=pop.device)
            self.act_h = torch.empty(P * N, dtype=torch.int64, pin_memory=True)
            self.obs_h = torch.empty(P * N * D, dtype=pop.obs.dtype, pin_memory=True)
            self.obs_d = torch.empty(P, N, D, dtype=pop.obs.dtype, device=pop.device)
            self.ev = torch.cuda.Event()
        if self.edescs is not None and not self.multi:  # per-step launches of the evaluation layer list
            from .learner import graph_act_workspace

            graph_act_workspace(self.pop, self.edescs[0])
        elif self.gdesc is not None:  # its scratch now: nothing may allocate while a persistent launch waits
            from .learner import graph_act_workspace

            graph_act_workspace(self.pop, self.gdesc)
        self.obs = None
        self.stream = None  # a dedicated non-blocking stream, assigned by run_lockstep
        self._pipelined = False

    # -- lock-step protocol -------------------------------------------------
    def begin(self) -> None:
        # the driver's stream starts after everything queued so far (the learner
        # that wrote the parameters).  Ordered here, before any group's
        # persistent launch is resident: nothing after a launch may wait for
        # the device while the host is pacing it
        self.stream.wait_stream(torch.cuda.current_stream(self.pop.device))
        if self.persistent:
            self.env.reset(out_obs=self.obs_h.numpy())
        else:
            self.obs, _ = self.env.reset()

    def _launch(self) -> None:
        """A persistent launch covering the next chunk of steps.  Each launch
        starts on a freshly zeroed control block (the previous launch has
        exited: it either ran all its steps or was stopped and synchronised)."""
        lib = _lib.load()
        pop = self.pop
        n = _EVAL_CHUNK if self.max_steps is None else min(_EVAL_CHUNK, int(self.max_steps) - self.step)
        self.ctl_h.zero_()
        if self.multi:  # every agent of every group on its own network
            ctr = (ctypes.c_uint64 * self.P)(*[c + self.step for c in self._ctr0])
            tally = None
            if self.device_tally and self._pipelined:
                self._tally.prev = 1 if self.step > 0 else 0
                tally = ctypes.byref(self._tally)
            _lib.check(lib.agx_ppo_eval_multi_persistent(self._nets, self._params, self._env_base, self._seeds, ctr,
                                                         self.P, self.N, self.obs_h.data_ptr(), self.act_h.data_ptr(),
                                                         n, 0, self._agents_h.data_ptr(), self._agents_d.data_ptr(),
                                                         self.ctl_h.data_ptr(), self.runner.timeout_s, tally,
                                                         self.stream.cuda_stream),
                       "agx_ppo_eval_multi_persistent")
        elif self.desc is not None:
            _lib.check(lib.agx_ppo_eval_persistent(ctypes.byref(self.desc), self.P, self.N,
                                                   pop.params.data.data_ptr(), self.obs_h.data_ptr(), None,
                                                   self.act_h.data_ptr(), pop.env_base_d.data_ptr(), n, 0, pop.act_seed,
                                                   self.counter0 + self.step, self.args_h.data_ptr(),
                                                   self.ctl_h.data_ptr(), self.runner.timeout_s,
                                                   self.stream.cuda_stream),
                       "agx_ppo_eval_persistent")
        else:  # a mutated shape (its act workspace was taken at construction)
            _lib.check(lib.agx_ppo_eval_graph_persistent(ctypes.byref(self.gdesc), self.P, self.N,
                                                         pop.params.data.data_ptr(), self.obs_h.data_ptr(), None,
                                                         self.act_h.data_ptr(), pop.env_base_d.data_ptr(), n, 0,
                                                         pop.act_seed, self.counter0 + self.step,
                                                         self.args_h.data_ptr(), self.ctl_h.data_ptr(),
                                                         self.runner.timeout_s, pop._act_ws[1].data_ptr(),
                                                         self.stream.cuda_stream),
                       "agx_ppo_eval_graph_persistent")
        _pacing_begin()
        self.launch_step0 = self.step
        self.launched_to = self.step + n

    def request(self) -> None:
        """Start the policy step of vector step self.step."""
        if self.persistent:
            if self.step >= self.launched_to:
                if self.launched_to > 0:  # the previous launch ran all its steps and ends by itself
                    self._drain()
                self._launch()
            self._signal(self._ctl, self.step - self.launch_step0 + 1)
            return
        with torch.cuda.stream(self.stream):  # never the NULL stream: it would wait for resident launches
            self._request_step()

    def _request_step(self) -> None:
        pop, P, N, D = self.pop, self.P, self.N, self.D
        self.obs_h.numpy()[:] = np.asarray(self.obs).reshape(-1)
        self.obs_d.view(-1).copy_(self.obs_h, non_blocking=True)
        counter = self.counter0 + self.step
        if self.edescs is not None:  # the evaluation layer list (as the multi launch samples)
            from .learner import policy_step_graph

            policy_step_graph(pop, self.edescs[0], self.obs_d, N * D, sample=True, counter=counter,
                              out_agent_stride=N, actions_flat=self.act_d)
        elif self.desc is not None:
            from .learner import policy_step

            policy_step(pop, self.desc, self.obs_d, N * D, sample=True, counter=counter, out_agent_stride=N,
                        actions_flat=self.act_d)
        elif self.gdesc is not None:  # a mutated shape: agx_ppo_act_graph, same counters
            from .learner import policy_step_graph

            policy_step_graph(pop, self.gdesc, self.obs_d, N * D, sample=True, counter=counter,
                              out_agent_stride=N, actions_flat=self.act_d)
        else:
            self.act_d.copy_(pop.act(self.obs_d, counter=counter)[0].view(-1))
        self.act_h.copy_(self.act_d, non_blocking=True)
        self.ev.record()

    def wait(self) -> None:
        if self.persistent:
            t = self.step - self.launch_step0 + 1
            rc = self._wait_fn(self._ctl, self.n_wg, t, self.runner.timeout_s)
            if rc != 0:
                msg = _lib.load().agx_last_error().decode(errors="replace")
                words = self.ctl_h.view(torch.int32)
                done = words[4:4 + self.n_wg].tolist()
                kind = "population" if self.multi else ("graph" if self.desc is None else "compiled")
                state = (f"{kind} pass P={self.P} N={self.N}: step "
                         f"{self.step} (launch from {self.launch_step0} to {self.launched_to}), waiting for "
                         f"{t}; control block seq {int(words[0])} timeout {int(words[1])} nwg {int(words[2])} "
                         f"(driver {self.n_wg}); done words {done}")
                self.abort()
                raise _lib.AgxError(f"agx_host_wait failed ({rc}): {msg}; evaluation {state}")
            return
        self.ev.synchronize()

    def env_step(self) -> bool:
        """The env step on the actions; -> True once every env has finished."""
        if self.persistent:
            obs_n, rew_n, done_n, act_n = self._views
            try:
                _, _, term, trunc, _ = self.env.step(act_n, out_obs=obs_n, out_rew=rew_n, out_done=done_n)
            except BaseException:
                self.abort()
                raise
            reward = rew_n
        else:
            self.obs, reward, term, trunc, _ = self.env.step(self.act_h.numpy().copy())
        self.step += 1
        self.scores += np.asarray(reward).reshape(-1)
        done = np.asarray(term, dtype=bool).reshape(-1)
        if trunc is not None:
            done = done | np.asarray(trunc, dtype=bool).reshape(-1)
        if self.max_steps is not None and self.step == self.max_steps:
            done = np.ones(self.P * self.N, dtype=bool)
        new = done & ~self.finished
        if new.any():
            self.completed[new] = self.scores[new]
            self.finished |= new
            self.n_finished = int(self.finished.sum())
        return self.n_finished == self.finished.size

    def _drain(self) -> None:
        _pacing_end()
        self.stream.synchronize()  # only this pass's launch: other groups' stay resident
        self.launched_to = 0

    def end(self) -> None:
        """The pass is over: a persistent launch still waiting for its next
        step is stopped cleanly (AGX_ROLLOUT_STOP) and drained."""
        if self.persistent and self.launched_to > 0:
            if self.step < self.launched_to:
                _lib.load().agx_host_signal(self.ctl_h.data_ptr(), AGX_ROLLOUT_STOP)
            self._drain()

    def abort(self) -> None:
        if self.persistent and self.launched_to > 0:
            _lib.load().agx_host_signal(self.ctl_h.data_ptr(), AGX_ROLLOUT_STOP)
            self._drain()

    def result(self) -> np.ndarray:
        return self.completed.reshape(self.P, self.N).mean(1)

    # -- the pass in two halves ---------------------------------------------
    def can_pipeline(self) -> bool:
        """A population-wide launch over a stack of one env per agent can
        run in two halves (AGX_EVAL_PIPELINE=0 turns it off)."""
        from ..envs import StackedVecEnv

        return bool(self.multi and self.P >= 2 and isinstance(self.env, StackedVecEnv) and
                    len(self.env.envs) == self.P and all(int(e.num_envs) == self.N for e in self.env.envs) and
                    os.environ.get("AGX_EVAL_PIPELINE", "1") != "0")

    def _half_env_step(self, h: int) -> None:
        """One part's env step and episode tally, on views of the staging and
        of the tallies made once per pass (run_pipelined)."""
        obs, rew, done_st, act, sc, fin, comp, buf = self._part_views[h]
        try:
            _, _, term, trunc, _ = self._half_envs[h].step(act, out_obs=obs, out_rew=rew, out_done=done_st)
        except BaseException:
            self.abort()
            raise
        if self.device_tally:  # the launch tallies this step's reward / done at its next step
            if trunc is not None and np.count_nonzero(trunc):
                np.logical_or(done_st, trunc, out=done_st)  # done = term | trunc
            return
        sc += rew
        if self.max_steps is not None and self.step + 1 == self.max_steps:
            buf[:] = True
        elif trunc is not None:
            np.logical_or(term, trunc, out=buf)
        else:
            np.copyto(buf, term)
        np.logical_and(buf, ~fin, out=buf)
        if buf.any():
            comp[buf] = sc[buf]
            fin |= buf
            self.n_finished = int(self.finished.sum())

    def run_pipelined(self) -> None:
        """The whole pass with the agents in n parts (AGX_EVAL_PARTS, default
        2: more parts cost more host work than they hide, r5 tools/gpu_eval_parts.sh), each a step ahead of the next: while
        one part's workgroups compute their policy step, the host steps the
        other parts' envs (agx_host_signal_range / agx_host_wait_range).  Same
        launch, counters, releases and samples as the lock-step loop
        (run_lockstep); the device latency hides behind the other parts' env
        work."""
        from ..envs import StackedVecEnv

        lib = _lib.load()
        P, N = self.P, self.N
        n = max(2, min(P, int(os.environ.get("AGX_EVAL_PARTS", "2"))))
        gx = self.n_wg // P
        cut = [round(i * P / n) for i in range(n + 1)]
        self._halves = [(cut[i] * N, cut[i + 1] * N) for i in range(n)]
        blocks = [(cut[i] * gx, cut[i + 1] * gx) for i in range(n)]
        self._half_envs = [StackedVecEnv(self.env.envs[cut[i]:cut[i + 1]]) for i in range(n)]
        obs_n, rew_n, done_n, act_n = self._views
        self._part_views = [(obs_n[a:b], rew_n[a:b], done_n[a:b], act_n[a:b], self.scores[a:b], self.finished[a:b],
                             self.completed[a:b], np.zeros(b - a, dtype=bool)) for a, b in self._halves]
        sig, wait, sigwait = lib.agx_host_signal_range, lib.agx_host_wait_range, lib.agx_host_signal_wait_range
        tmo = self.runner.timeout_s
        self.stream = _eval_stream(0)
        self._pipelined = True
        self.begin()

        def _failed(rc, h):
            msg = lib.agx_last_error().decode(errors="replace")
            self.abort()
            raise _lib.AgxError(f"agx_host_wait_range failed ({rc}): {msg}; evaluation part {h} of "
                                f"{n}, P={P} N={N} at step {self.step}")

        waited0 = False  # part 0's wait for this step done by the previous step's last hand-over
        try:
            while True:
                if self.step >= self.launched_to:
                    if self.launched_to > 0:  # the previous launch ran all its steps and ends by itself
                        self._drain()
                    self._launch()
                    for w0, w1 in blocks:
                        sig(self._ctl, w0, w1, 1)
                    waited0 = False
                rel = self.step - self.launch_step0 + 1
                more = self.step + 1 < self.launched_to  # the launch covers the next step
                if not waited0:
                    rc = wait(self._ctl, blocks[0][0], blocks[0][1], rel, tmo)
                    if rc != 0:
                        _failed(rc, 0)
                waited0 = False
                for h in range(n):
                    self._half_env_step(h)
                    if h + 1 < n:
                        # this part's next step released, then the next part's wait: one call
                        rc = (sigwait(self._ctl, blocks[h][0], blocks[h][1], rel + 1, blocks[h + 1][0],
                                      blocks[h + 1][1], rel, tmo) if more
                              else wait(self._ctl, blocks[h + 1][0], blocks[h + 1][1], rel, tmo))
                        if rc != 0:
                            _failed(rc, h + 1)
                self.step += 1
                if self.device_tally and self._t_fin_np.tobytes() == self._fin_all:  # tallied by the launch
                    self.n_finished = P * N
                done = self.n_finished == P * N or (self.max_steps is not None and self.step >= self.max_steps)
                if more:  # the last part's next step, and (going on) part 0's wait for it
                    if done:
                        sig(self._ctl, blocks[-1][0], blocks[-1][1], rel + 1)
                    else:
                        rc = sigwait(self._ctl, blocks[-1][0], blocks[-1][1], rel + 1, blocks[0][0], blocks[0][1],
                                     rel + 1, tmo)
                        if rc != 0:
                            _failed(rc, 0)
                        waited0 = True
                if done:
                    break
            self.end()
        except BaseException:
            self.abort()
            raise
        if self.device_tally:
            self.completed = self._t_completed.cpu().numpy()


AGX_ROLLOUT_STOP = 0xFFFFFFFE  # include/agx.h

# Dedicated non-blocking streams for the evaluation passes, one per
# lock-stepped group, created once per process (agx_stream_create).  Not from
# torch's stream pool: its round-robin could hand two groups the same stream,
# and one resident persistent launch would then hold the other's back; and not
# the legacy NULL stream, whose work waits for every blocking stream.
_EVAL_STREAMS: list = []


def _eval_stream(i: int):
    while len(_EVAL_STREAMS) <= i:
        h = _lib.load().agx_stream_create()
        if not h:
            raise _lib.AgxError(_lib.load().agx_last_error().decode(errors="replace"))
        _EVAL_STREAMS.append(torch.cuda.ExternalStream(h))
    return _EVAL_STREAMS[i]


def run_lockstep(drivers: list) -> None:
    """Step several groups' evaluation passes together: every vector step
    releases all groups' policy steps, waits for all, then steps all envs, so
    the groups' device work and host env steps overlap instead of running
    one pass after another."""
    active = list(drivers)
    # every driver on a stream of its own, none on the legacy NULL stream (work
    # there would wait for the other groups' resident persistent launches)
    for k, d in enumerate(active):
        d.stream = _eval_stream(k)
    try:
        for d in active:  # every group's stream ordering first, then the launches
            d.begin()
        while active:
            for d in active:
                d.request()
            for d in active:
                d.wait()
            still = []
            for d in active:
                if d.env_step():
                    d.end()
                else:
                    still.append(d)
            active = still
    except BaseException:
        for d in active:
            d.abort()
        raise
