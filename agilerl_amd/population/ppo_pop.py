"""A PPO population resident in HBM: stacked networks, SoA rollout storage,
batched rollout inference and a batched learner.

Reference behaviour mirrored per agent:
  * rollout collection  agilerl/rollouts/on_policy.py:23-203 (done = term|trunc
    of THIS step; bootstrap with last_done = term, :184-196)
  * rollout storage     agilerl/components/rollout_buffer.py:137-411 (time-major
    (T, N) SoA; here (P, T, N) on the GPU instead of CPU TensorDicts)
  * GAE                 rollout_buffer.py:413-481 -> agx_gae (bit-exact)
  * learner             agilerl/algorithms/ppo.py:814-921: global advantage
    normalisation, E epochs of shuffled minibatches, clipped surrogate +
    clipped value loss - entropy, per-group grad clip, Adam;
    returns sum(loss)/(num_samples*epochs) (:920)

The population axis replaces the reference's sequential agent loop
(train_on_policy.py:210): every kernel processes all P agents at once.
Sampling uses an on-device Gumbel-max draw (the reference's torch.multinomial
stream cannot be reproduced on a GPU generator anyway).  Minibatch order is
the reference's: by default the permutations come from numpy's global
legacy MT19937 exactly as PPO.learn's ``np.random.shuffle`` draws them
(``perm_source="numpy"``, agilerl_amd/rng.py); ``perm_source="device"``
draws them on the GPU instead (no host work, not reproducible against the
reference).

Two learner back ends share this state:
  * ``fused=True``  one persistent HIP workgroup per agent runs all E x M
                    minibatch updates (agx_ppo_learn, f32 MFMA GEMMs) —
                    the production path;
  * ``fused=False`` plain-PyTorch fp32 autograd over the stacked networks with
                    the HIP loss / clip+Adam kernels — the numerics reference
                    for the fused kernel and the path for architectures it does
                    not cover.
"""

from __future__ import annotations

import math
import os

import numpy as np
import torch

from .. import _lib
from .. import kernels as K
from ..rng import numpy_shuffle_perms, numpy_shuffle_perms_shard
from .nets import ActorCriticSpec, categorical


class _PPOLossFn(torch.autograd.Function):
    """Clipped surrogate loss for P minibatches at once (HIP fwd+bwd)."""

    @staticmethod
    def forward(ctx, logp, value, entropy, old_logp, adv, ret, old_v, gidx, b, clip, vf, ent):
        g1, g2, g3, stats = K.ppo_loss_fwd_bwd(
            logp.contiguous().view(-1), old_logp, adv, ret, old_v, value.contiguous().view(-1),
            entropy.contiguous().view(-1), b, clip, vf, ent, index=gidx)
        ctx.save_for_backward(g1, g2, g3)
        ctx.shape = logp.shape
        ctx.mark_non_differentiable(stats)
        return stats[:, 0].sum(), stats

    @staticmethod
    def backward(ctx, gl, _gs):
        g1, g2, g3 = ctx.saved_tensors
        s = ctx.shape
        return (g1.view(s) * gl, g2.view(s) * gl, g3.view(s) * gl) + (None,) * 9


class PPOPopulation:
    def __init__(self, spec: ActorCriticSpec, pop_size: int, num_envs: int, *, learn_step=2048,
                 batch_size=128, lr=1e-3, gamma=0.99, gae_lambda=0.95, clip_coef=0.2, ent_coef=0.01,
                 vf_coef=0.5, max_grad_norm=0.5, update_epochs=4, target_kl=None, seeds=None,
                 device="cuda", fused=True, perm_source="numpy", action_masks=False, agent_offset=0,
                 global_pop_size=None, seed_base=None, agent_ids=None, init_params=True):
        self.spec = spec
        self.P, self.N = int(pop_size), int(num_envs)
        # a shard of a population spread over ranks: these P agents are global
        # agents agent_offset .. agent_offset + P of global_pop_size (their
        # sampling streams, env copies and minibatch shuffles are the global
        # agents' own, so the sharded run draws what one process would)
        self.agent_offset = int(agent_offset)
        self.global_P = self.P if global_pop_size is None else int(global_pop_size)
        if self.agent_offset < 0 or self.agent_offset + self.P > self.global_P:
            raise ValueError("agent_offset / global_pop_size do not contain this shard")
        # global index of each local agent (a contiguous shard by default; a
        # group of the population engine holds any subset): keys its env
        # copies' sampling streams
        self.agent_ids = (list(range(self.agent_offset, self.agent_offset + self.P)) if agent_ids is None
                          else [int(i) for i in agent_ids])
        if len(self.agent_ids) != self.P:
            raise ValueError("agent_ids must name every agent")
        self.T = -(learn_step // -self.N)  # capacity = ceil(learn_step / num_envs), ppo.py:363
        self.S = self.T * self.N
        self.batch_size = int(batch_size)
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        self.clip_coef, self.ent_coef, self.vf_coef = float(clip_coef), float(ent_coef), float(vf_coef)
        self.max_grad_norm = float(max_grad_norm)
        self.update_epochs = int(update_epochs)
        self.target_kl = target_kl
        self.device = torch.device(device)
        seeds = list(range(self.agent_offset, self.agent_offset + self.P)) if seeds is None else list(seeds)
        self.seeds = seeds
        # population-level streams key off the global population's first seed
        seed_base = int(seeds[0]) if seed_base is None else int(seed_base)
        self.seed_base = seed_base
        # init_params=False: zeros, for a caller that copies every row in (the
        # population engine's regrouping; the orthogonal init is a host QR per layer)
        self.params = torch.nn.Parameter(spec.init_params(self.P, seeds, self.device) if init_params else
                                         torch.zeros(self.P, spec.n_params, dtype=torch.float32, device=self.device))
        self.params.grad = torch.zeros_like(self.params)
        lr_list = [float(lr)] * self.P if not isinstance(lr, (list, tuple)) else [float(x) for x in lr]
        self.opt = K.ClipAdam(self.params.data, spec.group_offsets, lr_list, max_norm=self.max_grad_norm,
                              grads=self.params.grad)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed_base * 7919 + 17)
        if perm_source not in ("numpy", "device"):
            raise ValueError("perm_source must be 'numpy' or 'device'")
        self.perm_source = perm_source
        self.use_action_masks = bool(action_masks)
        # sticky device error word of the fused learner (partner timeout); checked at host sync points
        self.err_word = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.last_kl = None
        # per-agent RL hyperparameters (mutation.py:413-453 mutates them agent by
        # agent); batch_size / update_epochs above are the population maxima
        self.agent_batch = [self.batch_size] * self.P
        self.agent_epochs = [self.update_epochs] * self.P
        self.agent_ent = [self.ent_coef] * self.P
        self.agent_lr = list(lr_list)  # exact host values (the device table is f32)
        # device copies (the learner reads them once the population is heterogeneous;
        # PopulationSync moves them with the parent rows)
        self.hp_batch_d = torch.full((self.P,), self.batch_size, dtype=torch.int32, device=self.device)
        self.hp_epochs_d = torch.full((self.P,), self.update_epochs, dtype=torch.int32, device=self.device)
        self.hp_ent_d = torch.full((self.P,), self.ent_coef, dtype=torch.float32, device=self.device)
        self._hetero = False
        self.fused = fused
        self.act_seed = (seed_base * 0x9E3779B97F4A7C15 + 0x5851F42D) & 0xFFFFFFFFFFFFFFFF
        # every global agent's update_epochs (the shuffles each draws; ranks
        # refresh the other shards' entries after a mutation)
        self.global_epochs = [self.update_epochs] * self.global_P
        self.global_batch_max = None
        self._shard_scratch: dict = {}
        self.act_counter = 0
        self._desc = None
        self._gdesc = None
        self._edesc = None
        self._alloc_rollout()
        self.env_base_d = torch.tensor([i * self.N for i in self.agent_ids], dtype=torch.int64, device=self.device)
        self.learn_steps = 0
        self.rollout_id = 0
        self.prefetch_perms = os.environ.get("AGX_PREFETCH_PERMS", "1") != "0"
        self._perm_next = None
        self._perm_stream = None
        self._perm_host = None
        self._perm_k = 0
        self._gae_launch = None
        # target-KL runs: numpy state before the current learn's shuffles, and
        # the correction owed to the global stream once its epochs_run is known
        self._perm_drawn_state = None
        self._kl_pending = None
        # a generation's shuffles drawn ahead by the population engine, agent by
        # agent (set_generation_perms): [K, E, P, S], learn k reads row k
        self._gen_block = None
        self._gen_block_d = None
        self._gen_k = 0
        self._gen_ran: list[torch.Tensor] = []

    # ------------------------------------------------------------------ #
    def _alloc_rollout(self):
        P, T, N, D, dev = self.P, self.T, self.N, self.spec.obs_dim, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        # image specs keep uint8 frames (normalised inside the first conv's load)
        self.obs = torch.zeros(P, T, N, D, dtype=getattr(self.spec, "obs_dtype", torch.float32), device=dev)
        self.actions = torch.zeros(P, T, N, dtype=torch.int64, device=dev)
        self.rewards = torch.zeros(P, T, N, **f32)
        self.dones = torch.zeros(P, T, N, dtype=torch.uint8, device=dev)
        self.values = torch.zeros(P, T, N, **f32)
        self.log_probs = torch.zeros(P, T, N, **f32)
        self.advantages = torch.zeros(P, T, N, **f32)
        self.returns = torch.zeros(P, T, N, **f32)
        self.adv_stats = torch.zeros(P, 2, dtype=torch.float64, device=dev)
        # legal-action masks (1 = legal) stored with the rollout when the env provides them
        self.action_masks = (torch.ones(P, T, N, self.spec.n_actions, dtype=torch.uint8, device=dev)
                             if self.use_action_masks else None)
        self.gae_ws = torch.empty(max(16, K._lib.load().agx_gae_workspace_bytes(P, T, N)), dtype=torch.uint8,
                                  device=dev)

    # ------------------------------------------------------------------ #
    @torch.no_grad()
    def act(self, obs: torch.Tensor, counter: int | None = None):
        """obs [P, N, D] (device) -> action, log_prob, entropy, value, each [P, N].
        Gumbel-max sampling; with ``counter`` every agent draws from its own
        generator keyed by (population seed, global agent id, counter), so an
        agent's draws do not depend on which other agents share its population."""
        logits, value = self.spec.forward(self.params.data, obs)
        logp_all, ent = categorical(logits)
        if counter is None:
            u = torch.rand(logits.shape, generator=self.gen, device=self.device)
        else:
            u = torch.empty(logits.shape, device=self.device)
            g = torch.Generator(device=self.device)
            for p, aid in enumerate(self.agent_ids):
                g.manual_seed(((self.seed_base * 1_000_003 + aid) * 2_097_152 + int(counter)) & 0x7FFFFFFFFFFFFFFF)
                u[p] = torch.rand(logits.shape[1:], generator=g, device=self.device)
        u.clamp_(min=1e-20)
        action = torch.argmax(logits - torch.log(-torch.log(u)), dim=-1)
        logp = logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1)
        return action, logp, ent, value

    def fused_descriptor(self):
        """agx_ppo_net for this architecture, or None when the fused kernels do
        not cover it (then the plain-PyTorch forward / learner run)."""
        if not self.fused or not isinstance(self.spec, ActorCriticSpec):
            return None  # the fused kernels take the MLP actor-critic shapes only
        if self._desc is None:
            from .learner import net_descriptor

            self._desc = net_descriptor(self.spec) or False
        return self._desc or None

    def learn_descriptor(self):
        """The network the fused learn() runs: agx_ppo_net for the compiled
        shapes, else agx_ppo_graph (agx_ppo_learn_graph: any MLP actor-critic
        an architecture mutation produces); None: the plain-PyTorch learner."""
        desc = self.fused_descriptor()
        if desc is not None or not self.fused or not isinstance(self.spec, ActorCriticSpec):
            return desc
        if self._gdesc is None:
            from .learner import graph_descriptor

            self._gdesc = graph_descriptor(self.spec) or False
        return self._gdesc or None

    def eval_descriptor(self):
        """agx_ppo_graph of this network for the evaluation passes: every MLP
        actor-critic, the compiled shapes included, so that a population's
        agents are evaluated together in one launch whatever kernels they train
        on (agx_ppo_eval_multi_persistent).  None: the PyTorch policy step."""
        if not self.fused or not isinstance(self.spec, ActorCriticSpec):
            return None
        if self.fused_descriptor() is None:
            return self.learn_descriptor()  # already the runtime layer list
        if self._edesc is None:
            from .learner import graph_descriptor

            self._edesc = graph_descriptor(self.spec) or False
        return self._edesc or None

    @torch.no_grad()
    def act_into(self, t: int, actions_flat: torch.Tensor | None = None) -> None:
        """Rollout policy step for slot t: reads obs[:, t], writes actions /
        log_probs / values[:, t] in place (and a contiguous [P*N] copy of the
        actions for the host env step)."""
        desc = self.fused_descriptor()
        if desc is None and self.learn_descriptor() is not None:  # a mutated shape: the runtime-shape kernel
            from .learner import policy_step_graph

            self.act_counter += 1
            TN = self.T * self.N
            policy_step_graph(self, self.learn_descriptor(), self.obs[:, t], TN * self.spec.obs_dim, sample=True,
                              counter=self.act_counter, actions=self.actions[:, t], log_probs=self.log_probs[:, t],
                              values=self.values[:, t], out_agent_stride=TN, actions_flat=actions_flat)
            return
        if desc is None:
            self.act_counter += 1
            action, logp, _ent, value = self.act(self.obs[:, t], counter=self.act_counter)
            self.actions[:, t].copy_(action)
            self.values[:, t].copy_(value)
            self.log_probs[:, t].copy_(logp)
            if actions_flat is not None:
                actions_flat.copy_(action.view(-1))
            return
        from .learner import policy_step

        self.act_counter += 1
        TN = self.T * self.N
        policy_step(self, desc, self.obs[:, t], TN * self.spec.obs_dim, sample=True, counter=self.act_counter,
                    actions=self.actions[:, t], log_probs=self.log_probs[:, t], values=self.values[:, t],
                    out_agent_stride=TN, actions_flat=actions_flat)

    @torch.no_grad()
    def store(self, t: int, obs, action, reward, done, value, logp):
        self.obs[:, t].copy_(obs, non_blocking=True)
        self.actions[:, t].copy_(action, non_blocking=True)
        self.rewards[:, t].copy_(reward, non_blocking=True)
        self.dones[:, t].copy_(done, non_blocking=True)
        self.values[:, t].copy_(value, non_blocking=True)
        self.log_probs[:, t].copy_(logp, non_blocking=True)

    def finish_rollout(self, last_obs: torch.Tensor, last_done: torch.Tensor,
                       last_value: torch.Tensor | None = None):
        """Bootstrap value + GAE (+ per-agent advantage statistics).  The fused
        runner computes last_value in its final rollout-step launch."""
        self.rollout_id += 1
        if last_value is None:
            with torch.no_grad():
                _, last_value = self.spec.forward(self.params.data, last_obs)
        if not last_value.is_contiguous():
            last_value = last_value.contiguous()
        if not last_done.is_contiguous():
            last_done = last_done.contiguous()
        key = (last_value.data_ptr(), last_done.data_ptr(), last_value.shape, last_done.dtype,
               *(t.data_ptr() for t in (self.rewards, self.dones, self.values, self.advantages, self.returns,
                                        self.adv_stats, self.gae_ws)))
        if self._gae_launch is not None and self._gae_launch[0] == key:
            self._gae_launch[1](_lib.stream())  # the runner's steady state: one cached launch
            return
        launch = K.gae_launcher(self.rewards, self.dones, self.values, last_value, last_done, self.gamma,
                                self.gae_lambda, True, self.advantages, self.returns, self.adv_stats, self.gae_ws)
        # keep a launcher only for the runner's persistent last_value / last_done
        self._gae_launch = (key, launch, last_value, last_done)

    # ------------------------------------------------------------------ #
    def learn(self, prefetch: bool = True, skip_if_set: int | None = None) -> torch.Tensor:
        """One PPO update of every agent; returns the reference's mean_loss per
        agent (device tensor [P], no host sync).  ``prefetch``: draw the next
        learn's permutations right away (the pipelined runner passes False and
        prefetches after pacing the rollout instead)."""
        self.learn_steps += 1
        if self.learn_descriptor() is not None:
            from .learner import fused_learn

            loss = fused_learn(self, skip_if_set=skip_if_set)
            self.last_kl = self._fused.kl
            self._record_kl_pending(self._fused.epochs_run)
            # with target_kl the next learn's shuffles depend on this one's stops
            if prefetch and self.prefetch_perms and self.target_kl is None:
                self.prefetch_permutations()
            return loss
        loss = self._learn_torch()
        self._record_kl_pending(self.last_epochs_run)
        return loss

    # ------------------------------------------------------------------ #
    # target_kl and the global numpy stream (ppo.py:836-842, 917-918)
    #
    # The reference's agents learn one after another, each drawing one
    # np.random.shuffle per epoch it actually runs; an agent that stops early
    # on target_kl draws fewer.  The engine draws every agent's E shuffles
    # before the learn (all agents run at once), so after an early stop:
    #   * agents after the first early-stopping agent learn from shuffles
    #     that are shifted against the reference's (agent p's would start at
    #     shuffle sum(epochs_run[:p]), which is only known once every agent
    #     before it has finished — a serial dependency the population breaks);
    #   * the GLOBAL stream is put back in step: once the learn's epochs_run
    #     is known, the state is rewound to before the draw and advanced by
    #     exactly sum(epochs_run) shuffles, the reference's count, so every
    #     later consumer (tournament and mutation draws, the next learn) sees
    #     the state the reference would.
    # Without target_kl every agent runs all its epochs and both are exact.
    def _record_kl_pending(self, epochs_run) -> None:
        if self.target_kl is not None and self._gen_block is not None:
            self._gen_ran.append(torch.as_tensor(epochs_run).detach().clone())  # the engine re-syncs the stream
            return
        if self.target_kl is None or self.perm_source != "numpy" or self._perm_drawn_state is None:
            return
        planned = list(self.agent_epochs) if self.heterogeneous else [self.update_epochs] * self.P
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        self._kl_pending = (self._perm_drawn_state, planned, epochs_run, ev)
        self._perm_drawn_state = None

    def sync_numpy_stream(self) -> None:
        """Apply the correction a target-KL learn owes the global numpy stream
        (waits for that learn's epochs_run; see above).  Called before anything
        draws from the stream: the next permutation draw, tournament and
        mutation draws (discard_prefetch)."""
        if self._kl_pending is None:
            return
        state, planned, epochs_run, ev = self._kl_pending
        self._kl_pending = None
        if ev is not None:
            ev.synchronize()
        ran = [int(x) for x in torch.as_tensor(epochs_run).cpu().tolist()]
        if ran == planned:
            return
        np.random.set_state(state)
        total = int(sum(ran))
        if total:
            numpy_shuffle_perms(1, total, self.S)

    def check_errors(self) -> None:
        """Raise AgxError if a fused learn() since the last check left an agent's
        update incomplete (a partner workgroup timed out); resets the word.
        Synchronises with the device."""
        w = int(self.err_word.item())
        if w != 0:
            self.err_word.zero_()
            why = []
            if w & 1:  # AGX_LEARN_ERR_TIMEOUT
                why.append("a partner workgroup timed out; the population's parameters are incomplete for this "
                           "learn()")
            if w & 2:  # AGX_LEARN_ERR_PERM
                why.append("a minibatch permutation index was outside [0, S) (the gather prologue substituted "
                           "row 0; this learn() is invalid)")
            raise _lib.AgxError("agx_ppo_learn: " + "; ".join(why or [f"error word {w:#x}"]))

    # ------------------------------------------------------------------ #
    @property
    def heterogeneous(self) -> bool:
        return self._hetero

    @property
    def _hp_dev(self):
        """(batch i32 [P], epochs i32 [P], ent f32 [P]) for the learner, or None
        while every agent shares the population's values (and the partner
        split is sized by that batch: a group split like a larger global
        batch passes its agents' own sizes)."""
        if self._hetero or self.split_batch != self.batch_size:
            return (self.hp_batch_d, self.hp_epochs_d, self.hp_ent_d)
        return None

    def set_agent_hparam(self, p: int, name: str, value) -> None:
        """Set one agent's RL hyperparameter (the HPO mutation of
        mutation.py:413-453 on agent p).  ``learn_step`` would change the
        agent's rollout length, which the lock-step population engine shares
        across agents: it raises NotImplementedError."""
        p = int(p)
        if name == "lr":
            self.opt.lr[p] = float(value)
            self.agent_lr[p] = float(value)
            return
        if name == "batch_size":
            if int(value) < 1:
                raise ValueError("batch_size must be >= 1")
            # a minibatch larger than the rollout is the whole rollout (the
            # reference's indices[start:start + batch_size] slice, ppo.py:843-845):
            # the learner tables hold min(batch, S), the agent keeps its value
            self.agent_batch[p] = int(value)
            self.hp_batch_d[p] = min(int(value), self.S)
        elif name == "update_epochs":
            if int(value) < 1:
                raise ValueError("update_epochs must be >= 1")
            self.agent_epochs[p] = int(value)
            self.hp_epochs_d[p] = int(value)
        elif name == "ent_coef":
            self.agent_ent[p] = float(value)
            self.hp_ent_d[p] = float(value)
        elif name == "learn_step":
            raise NotImplementedError("learn_step is the rollout length every agent of the population engine shares")
        else:
            raise KeyError(f"no per-agent hyperparameter {name!r}")
        self._rederive()

    @property
    def split_batch(self) -> int:
        """The minibatch size that sizes the fused learner's partner split:
        the largest of the GLOBAL population (``global_batch_max``, set by the
        population engine; a shard or a group splits like the whole
        population, so its agents' sums run in the same order)."""
        return min(max(max(self.agent_batch), self.global_batch_max or 0), self.S)

    def set_host_hparams(self, p: int, lr=None, batch_size=None, update_epochs=None, ent_coef=None) -> None:
        """Exact host values of agent p's hyperparameters after a clone whose
        device rows already hold them (a parent from another rank: the
        device tables are f32 / int32, the host lists keep Python floats)."""
        if lr is not None:
            self.agent_lr[p] = float(lr)
        if batch_size is not None:
            self.agent_batch[p] = int(batch_size)
        if update_epochs is not None:
            self.agent_epochs[p] = int(update_epochs)
        if ent_coef is not None:
            self.agent_ent[p] = float(ent_coef)
        self._rederive()

    def reinit_agent_optimizer(self, p: int) -> None:
        """reinit_optimizers for agent p (core/base.py:654-710): a fresh Adam,
        zero moments and step count, the agent's current learning rate."""
        self.opt.exp_avg[p].zero_()
        self.opt.exp_avg_sq[p].zero_()
        self.opt.steps[p] = 0

    def _rederive(self) -> None:
        """Population maxima (they size the learner's workspace and partner
        split) and the heterogeneity flag, from the per-agent lists."""
        self.batch_size = min(max(self.agent_batch), self.S)
        if max(self.agent_epochs) != self.update_epochs:
            self.update_epochs = max(self.agent_epochs)
            self._fused = None      # workspace is sized by the epochs
            self._perm_host = None  # pinned [E, P, S] staging
            self.discard_prefetch()
            self._perm_next = None
        self._hetero = not (len(set(self.agent_batch)) == 1 and len(set(self.agent_epochs)) == 1
                            and len(set(self.agent_ent)) == 1)

    def after_clone(self, local_parents: list[int] | None) -> None:
        """PopulationSync has copied every cloned row (params, Adam state, lr,
        step, and the per-agent hyperparameter rows).  Single rank: the new
        agent j took local row local_parents[j], mirrored on the host lists;
        several ranks (parents may be remote): re-read the device rows."""
        if local_parents is not None:
            b, e, h, r = list(self.agent_batch), list(self.agent_epochs), list(self.agent_ent), list(self.agent_lr)
            self.agent_batch = [b[q] for q in local_parents]
            self.agent_epochs = [e[q] for q in local_parents]
            self.agent_ent = [h[q] for q in local_parents]
            self.agent_lr = [r[q] for q in local_parents]
        else:
            self.agent_batch = [int(x) for x in self.hp_batch_d.cpu()]
            self.agent_epochs = [int(x) for x in self.hp_epochs_d.cpu()]
            self.agent_ent = [float(x) for x in self.hp_ent_d.cpu()]
            self.agent_lr = [float(x) for x in self.opt.lr.cpu()]
        self._rederive()

    def minibatch_plan(self):
        b = self.batch_size
        return [(s, min(s + b, self.S)) for s in range(0, self.S, b)]

    def permutations(self) -> torch.Tensor:
        """[E, P, S] int64 per-agent minibatch orders for the next learn():
        numpy's global np.random.shuffle stream (default, ppo.py:836-842) or a
        device draw.  Returns the draw made ahead by prefetch_permutations()
        if there is one (the same draw, in the same order, as drawing here)."""
        if self._perm_next is not None:
            perms, ev, state = self._perm_next[:3]
            self._perm_next = None
            self._perm_drawn_state = state
            main = torch.cuda.current_stream()
            if ev is not None:
                main.wait_event(ev)
            perms.record_stream(main)  # (a block row: the block stays allocated until this stream is past it)
            return perms
        if self.perm_source == "numpy" and self._gen_block_d is not None:
            perms = self._next_block_row()
            perms.record_stream(torch.cuda.current_stream(self.device))
            return perms
        if self.perm_source == "numpy":
            host = self._host_perm_buffer()
            self._perm_drawn_state = self._fill_numpy_perms(host.numpy())
            perms = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._perm_host[self._perm_k ^ 1][1] = ev
            return perms
        keys = torch.rand(self.update_epochs, self.P, self.S, generator=self.gen, device=self.device)
        return torch.argsort(keys, dim=-1)

    def set_generation_perms(self, block: np.ndarray | None) -> None:
        """The population engine's draw of this population's shuffles for a
        whole generation ([K, E, P, S] int64: learn k of local agent p visits
        block[k, e, p] in epoch e), drawn agent by agent over the global
        population as the reference's agents learn one after another
        (train_on_policy.py:210-248 -> ppo.py:836-842).  None: draw per learn."""
        self.discard_prefetch()
        if block is not None:
            if block.ndim != 4 or block.shape[1:] != (self.update_epochs, self.P, self.S):
                raise ValueError(f"generation shuffles {block.shape}, expected [K, {self.update_epochs}, {self.P}, "
                                 f"{self.S}]")
        self._gen_block, self._gen_k, self._gen_ran = block, 0, []
        # the whole block in HBM once (one copy at the generation's start, before
        # any launch): each learn then takes its row without host work
        self._gen_block_d = (torch.from_numpy(block).to(self.device)
                             if block is not None and self.device.type == "cuda" else None)

    def _next_block_row(self) -> torch.Tensor:
        """The next learn's [E, P, S] row of the generation block in HBM."""
        if self._gen_k >= self._gen_block.shape[0]:
            raise RuntimeError("more learns than the generation's shuffles were drawn for")
        row = self._gen_block_d[self._gen_k]
        self._gen_k += 1
        return row

    def _fill_numpy_perms(self, out: np.ndarray):
        """The next learn's [E, P, S] numpy-stream permutations into ``out``;
        -> the global numpy state before the draw (None when they come from
        the engine's generation block, which owns the stream)."""
        if self._gen_block is not None:
            if self._gen_k >= self._gen_block.shape[0]:
                raise RuntimeError("more learns than the generation's shuffles were drawn for")
            np.copyto(out, self._gen_block[self._gen_k])
            self._gen_k += 1
            return None
        self.sync_numpy_stream()
        state = np.random.get_state(legacy=True)
        self._draw_numpy_perms(out)
        return state

    def _draw_numpy_perms(self, out: np.ndarray) -> None:
        """[E, P, S] from the global numpy stream: this shard's agents' shuffles
        in the global agent order (rng.py).  An agent with fewer epochs than E
        draws fewer shuffles; its rows beyond get arange(S), so no row of the
        (reused, uninitialised pinned) buffer ever holds an out-of-range index
        — the gather prologue and the PyTorch learner index with every row."""
        if self.global_P == self.P:
            numpy_shuffle_perms(self.P, self.update_epochs, self.S, out=out,
                                epochs_per_agent=self.agent_epochs if self.heterogeneous else None)
        else:
            eg = list(self.global_epochs)
            eg[self.agent_offset:self.agent_offset + self.P] = self.agent_epochs
            numpy_shuffle_perms_shard(out, self.agent_offset, self.global_P, eg, self._shard_scratch)
        E = out.shape[0]
        for p, e in enumerate(self.agent_epochs):
            if e < E:
                out[e:, p, :] = np.arange(self.S, dtype=np.int64)

    def _host_perm_buffer(self) -> torch.Tensor:
        """One of two pinned [E, P, S] int64 host buffers, alternating (the H2D
        copy that last read a buffer finished long before it is reused: it
        precedes a whole learn() on the stream; checked by its event)."""
        self._alloc_perm_host()
        slot = self._perm_host[self._perm_k]
        self._perm_k ^= 1
        if slot[1] is not None:
            slot[1].synchronize()
        return slot[0]

    def _alloc_perm_host(self) -> None:
        if self._perm_host is None:
            shape = (self.update_epochs, self.P, self.S)
            self._perm_host = [[torch.empty(shape, dtype=torch.int64, pin_memory=True), None] for _ in range(2)]

    def prepare_learn(self) -> None:
        """Do now what the next learn() would otherwise do on first use: build
        the fused learner (device workspace) and the pinned permutation
        staging, and draw the permutations.  The pipelined runner calls this
        before launching a persistent rollout: between that launch and the
        host pacing it, the device is waiting for this thread, so nothing
        there may wait for the device — and a hipMalloc / hipHostMalloc, or an
        event sync, can."""
        if self.learn_descriptor() is not None:
            from .learner import learner_stale, make_learner

            if learner_stale(self):
                self._fused = make_learner(self)
        if self.perm_source == "numpy":
            self._alloc_perm_host()
        if self.prefetch_perms:
            self.prefetch_permutations()

    def prefetch_permutations(self) -> None:
        """Draw the next learn's permutations now, off the critical path:
        device mode enqueues rand + a radix sort on a side stream (beside the
        learner and the next rollout); numpy mode runs the native host shuffle
        (~0.5 ms of host time while the GPU learns) and an async H2D copy.
        Anything else that draws from the global numpy generator in between
        (tournament selection, mutations) must call discard_prefetch() first,
        so the draws stay in the reference's order."""
        if self._perm_next is not None or self.device.type != "cuda":
            return
        if self._gen_block is not None and self._gen_k >= self._gen_block.shape[0]:
            return  # the generation's learns are all served: the next block is drawn with the next generation
        if self._perm_stream is None:
            self._perm_stream = torch.cuda.Stream(device=self.device)
        side = self._perm_stream
        state = None
        from_block = False
        if self.perm_source == "numpy" and self._gen_block_d is not None:
            self._perm_next = (self._next_block_row(), None, None, True)
            return
        if self.perm_source == "numpy":
            # waits for a target-KL learn's epochs_run (before any rollout launch)
            from_block = self._gen_block is not None
            host = self._host_perm_buffer()
            state = self._fill_numpy_perms(host.numpy())
            with torch.cuda.stream(side):
                perms = host.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            self._perm_host[self._perm_k ^ 1][1] = ev
        else:
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                keys = torch.rand(self.update_epochs, self.P, self.S, generator=self.gen, device=self.device)
                perms = torch.argsort(keys, dim=-1)
                ev = torch.cuda.Event()
                ev.record(side)
        self._perm_next = (perms, ev, state, from_block)

    def discard_prefetch(self) -> None:
        """Undo a prefetched numpy draw: the global numpy state goes back to
        before it, so the next consumer of the stream draws what it would have
        drawn without the prefetch (the permutations are re-drawn later)."""
        if self._perm_next is not None and len(self._perm_next) > 3 and self._perm_next[3]:
            self._perm_next = None  # a generation-block row: served again by the next permutations()
            self._gen_k -= 1
            return
        if self._perm_next is None or self._perm_next[2] is None:
            self.sync_numpy_stream()
            return  # nothing drawn ahead from numpy (device draws use the pop's own generator)
        perms, ev, state = self._perm_next[:3]
        self._perm_next = None
        np.random.set_state(state)

    def _learn_torch(self, perms: torch.Tensor | None = None) -> torch.Tensor:
        """Plain-PyTorch fp32 autograd learner over the stacked networks (HIP
        loss and clip + Adam kernels): the numerics cross-check of the fused
        kernel and the path for architectures it does not cover.  Same
        semantics, including target-KL early stop per agent (stopped agents'
        rows are left untouched) and action masks."""
        if perms is None:
            perms = self.permutations()
        K.adv_normalize_(self.advantages, self.adv_stats)
        if not self.heterogeneous:
            return self._learn_torch_group(perms, None, self.batch_size, self.update_epochs, self.ent_coef)
        # per-agent batch / epochs / entropy (HPO mutations): agents sharing all
        # three learn together; the others' rows are left untouched (active mask)
        groups: dict[tuple, list[int]] = {}
        for p in range(self.P):
            groups.setdefault((self.agent_batch[p], self.agent_epochs[p], self.agent_ent[p]), []).append(p)
        out = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        kl = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        ran = torch.zeros(self.P, dtype=torch.int32, device=self.device)
        for (b, e, ent), rows in groups.items():
            loss = self._learn_torch_group(perms, rows, b, e, ent)
            idx = torch.tensor(rows, device=self.device)
            out[idx] = loss[idx]
            kl[idx] = self.last_kl[idx]
            ran[idx] = self.last_epochs_run[idx]
        self.last_kl = kl
        self.last_epochs_run = ran
        return out

    def _learn_torch_group(self, perms, rows, batch_size, epochs, ent_coef) -> torch.Tensor:
        """E epochs x minibatches of ``batch_size`` for the agents in ``rows``
        (None: all agents); -> the reference's mean loss per agent [P]."""
        P, S, D = self.P, self.S, self.spec.obs_dim
        image = not isinstance(self.spec, ActorCriticSpec)
        obs = self.obs.view(P, S, D)
        act = self.actions.view(P, S)
        masks = None if self.action_masks is None else self.action_masks.view(P, S, -1)
        old_logp = self.log_probs.view(-1)
        adv = self.advantages.view(-1)
        ret = self.returns.view(-1)
        old_v = self.values.view(-1)
        base = (torch.arange(P, device=self.device) * S).unsqueeze(1)
        total = torch.zeros(P, dtype=torch.float32, device=self.device)
        kl_sum = torch.zeros(P, dtype=torch.float64, device=self.device)
        n_mb = 0
        member = None
        if rows is not None:
            member = torch.zeros(P, dtype=torch.uint8, device=self.device)
            member[torch.tensor(rows, device=self.device)] = 1
        active = member  # all (member) agents until one stops (u8 [P])
        plan = [(s, min(s + batch_size, S)) for s in range(0, S, batch_size)]
        ran = torch.zeros(P, dtype=torch.int32, device=self.device)  # epochs each agent runs
        for e in range(epochs):
            ran += 1 if active is None else active.int()
            for s0, s1 in plan:
                idx = perms[e][:, s0:s1]  # [P, b]
                ob = torch.gather(obs, 1, idx.unsqueeze(-1).expand(-1, -1, D))
                ac = torch.gather(act, 1, idx)
                logits, value = (self.spec.forward(self.params, ob, rows=rows) if image
                                 else self.spec.forward(self.params, ob))
                if masks is not None:
                    mk = torch.gather(masks, 1, idx.unsqueeze(-1).expand(-1, -1, masks.shape[-1]))
                    logits = torch.where(mk.bool(), logits, torch.full_like(logits, -1e8))
                logp_all, ent = categorical(logits)
                logp = logp_all.gather(-1, ac.unsqueeze(-1)).squeeze(-1)
                gidx = (idx + base).reshape(-1).contiguous()
                loss, stats = _PPOLossFn.apply(logp, value, ent, old_logp, adv, ret, old_v, gidx,
                                               s1 - s0, self.clip_coef, self.vf_coef, ent_coef)
                self.params.grad.zero_()
                loss.backward()
                self.opt.step(active)
                on = 1.0 if active is None else active.float()
                total += stats[:, 0] * on
                kl_sum += stats[:, 4].double() * (1.0 if active is None else active.double())
                n_mb += 1
            if self.target_kl is not None:
                # np.mean(approx_kl_divs) over every minibatch so far (ppo.py:917-918)
                stop = (kl_sum / n_mb > float(self.target_kl)).to(torch.uint8)
                now = (1 - stop) if active is None else active * (1 - stop)
                if int(now.sum()) == P and active is None:
                    continue
                active = now.contiguous()
                if int(active.sum()) == 0:
                    break
        self.last_kl = (kl_sum / max(n_mb, 1)).float()
        self.last_epochs_run = ran
        return total / (S * epochs)

    # ------------------------------------------------------------------ #
    @torch.no_grad()
    def evaluate(self, obs: torch.Tensor) -> torch.Tensor:
        """Greedy actions (mode of the categorical) for fitness evaluation."""
        logits, _ = self.spec.forward(self.params.data, obs)
        return torch.argmax(logits, dim=-1)

    def n_minibatches(self) -> int:
        return math.ceil(self.S / self.batch_size)

    def n_updates(self) -> int:
        """Minibatch updates of one learn() over the whole population (no early stop)."""
        return sum(e * math.ceil(self.S / b) for b, e in zip(self.agent_batch, self.agent_epochs))
