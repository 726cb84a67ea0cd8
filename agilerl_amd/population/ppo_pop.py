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
stream cannot be reproduced on a GPU generator anyway).

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

import torch

from .. import kernels as K
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
                 device="cuda", fused=True):
        self.spec = spec
        self.P, self.N = int(pop_size), int(num_envs)
        self.T = -(learn_step // -self.N)  # capacity = ceil(learn_step / num_envs), ppo.py:363
        self.S = self.T * self.N
        self.batch_size = int(batch_size)
        self.gamma, self.gae_lambda = float(gamma), float(gae_lambda)
        self.clip_coef, self.ent_coef, self.vf_coef = float(clip_coef), float(ent_coef), float(vf_coef)
        self.max_grad_norm = float(max_grad_norm)
        self.update_epochs = int(update_epochs)
        self.target_kl = target_kl
        self.device = torch.device(device)
        seeds = list(range(self.P)) if seeds is None else list(seeds)
        self.seeds = seeds
        self.params = torch.nn.Parameter(spec.init_params(self.P, seeds, self.device))
        self.params.grad = torch.zeros_like(self.params)
        lr_list = [float(lr)] * self.P if not isinstance(lr, (list, tuple)) else [float(x) for x in lr]
        self.opt = K.ClipAdam(self.params.data, spec.group_offsets, lr_list, max_norm=self.max_grad_norm,
                              grads=self.params.grad)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seeds[0]) * 7919 + 17)
        self.fused = fused
        self.act_seed = (int(seeds[0]) * 0x9E3779B97F4A7C15 + 0x5851F42D) & 0xFFFFFFFFFFFFFFFF
        self.act_counter = 0
        self._desc = None
        self._alloc_rollout()
        self.learn_steps = 0
        self.rollout_id = 0
        self.prefetch_perms = os.environ.get("AGX_PREFETCH_PERMS", "1") != "0"
        self._perm_next = None
        self._perm_stream = None
        self._gae_launch = None

    # ------------------------------------------------------------------ #
    def _alloc_rollout(self):
        P, T, N, D, dev = self.P, self.T, self.N, self.spec.obs_dim, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.obs = torch.zeros(P, T, N, D, **f32)
        self.actions = torch.zeros(P, T, N, dtype=torch.int64, device=dev)
        self.rewards = torch.zeros(P, T, N, **f32)
        self.dones = torch.zeros(P, T, N, dtype=torch.uint8, device=dev)
        self.values = torch.zeros(P, T, N, **f32)
        self.log_probs = torch.zeros(P, T, N, **f32)
        self.advantages = torch.zeros(P, T, N, **f32)
        self.returns = torch.zeros(P, T, N, **f32)
        self.adv_stats = torch.zeros(P, 2, dtype=torch.float64, device=dev)
        self.gae_ws = torch.empty(max(16, K._lib.load().agx_gae_workspace_bytes(P, T, N)), dtype=torch.uint8,
                                  device=dev)

    # ------------------------------------------------------------------ #
    @torch.no_grad()
    def act(self, obs: torch.Tensor):
        """obs [P, N, D] (device) -> action, log_prob, entropy, value, each [P, N]."""
        logits, value = self.spec.forward(self.params.data, obs)
        logp_all, ent = categorical(logits)
        u = torch.rand(logits.shape, generator=self.gen, device=self.device).clamp_(min=1e-20)
        action = torch.argmax(logits - torch.log(-torch.log(u)), dim=-1)
        logp = logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1)
        return action, logp, ent, value

    def fused_descriptor(self):
        """agx_ppo_net for this architecture, or None when the fused kernels do
        not cover it (then the plain-PyTorch forward / learner run)."""
        if not self.fused:
            return None
        if self._desc is None:
            from .learner import net_descriptor

            self._desc = net_descriptor(self.spec) or False
        return self._desc or None

    @torch.no_grad()
    def act_into(self, t: int, actions_flat: torch.Tensor | None = None) -> None:
        """Rollout policy step for slot t: reads obs[:, t], writes actions /
        log_probs / values[:, t] in place (and a contiguous [P*N] copy of the
        actions for the host env step)."""
        desc = self.fused_descriptor()
        if desc is None:
            action, logp, _ent, value = self.act(self.obs[:, t])
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

    @torch.no_grad()
    def finish_rollout(self, last_obs: torch.Tensor, last_done: torch.Tensor,
                       last_value: torch.Tensor | None = None):
        """Bootstrap value + GAE (+ per-agent advantage statistics).  The fused
        runner computes last_value in its final rollout-step launch."""
        self.rollout_id += 1
        if last_value is None:
            _, last_value = self.spec.forward(self.params.data, last_obs)
        last_value, last_done = last_value.contiguous(), last_done.contiguous()
        key = (last_value.data_ptr(), last_done.data_ptr(), last_value.shape, last_done.dtype,
               *(t.data_ptr() for t in (self.rewards, self.dones, self.values, self.advantages, self.returns,
                                        self.adv_stats, self.gae_ws)))
        if self._gae_launch is not None and self._gae_launch[0] == key:
            self._gae_launch[1](torch.cuda.current_stream(self.device).cuda_stream)
            return
        launch = K.gae_launcher(self.rewards, self.dones, self.values, last_value, last_done, self.gamma,
                                self.gae_lambda, True, self.advantages, self.returns, self.adv_stats, self.gae_ws)
        # keep a launcher only for the runner's persistent last_value / last_done
        self._gae_launch = (key, launch, last_value, last_done)

    # ------------------------------------------------------------------ #
    def learn(self) -> torch.Tensor:
        """One PPO update of every agent; returns the reference's mean_loss per
        agent (device tensor [P], no host sync)."""
        self.learn_steps += 1
        if self.target_kl is None and self.fused_descriptor() is not None:
            from .learner import fused_learn

            loss = fused_learn(self)
            if self.prefetch_perms:
                self.prefetch_permutations()
            return loss
        return self._learn_torch()

    def minibatch_plan(self):
        b = self.batch_size
        return [(s, min(s + b, self.S)) for s in range(0, self.S, b)]

    def permutations(self) -> torch.Tensor:
        """[E, P, S] int64 per-agent shuffles (the reference's np.random.shuffle
        per epoch, ppo.py:842), drawn on the device.  Returns the draw made
        ahead by prefetch_permutations() if there is one (the same draw, in
        the same order, as drawing here)."""
        if self._perm_next is not None:
            perms, ev = self._perm_next
            self._perm_next = None
            main = torch.cuda.current_stream(self.device)
            main.wait_event(ev)
            perms.record_stream(main)
            return perms
        keys = torch.rand(self.update_epochs, self.P, self.S, generator=self.gen, device=self.device)
        return torch.argsort(keys, dim=-1)

    def prefetch_permutations(self) -> None:
        """Draw the next permutations on a side stream now (rand + a radix
        sort, ~35 us of small launches), so they run beside the learner and
        the next rollout instead of between them.  Only the fused path calls
        it: there the generator draws nothing else, so the sequence of draws
        is unchanged."""
        if self._perm_next is not None or self.device.type != "cuda":
            return
        if self._perm_stream is None:
            self._perm_stream = torch.cuda.Stream(device=self.device)
        side = self._perm_stream
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            keys = torch.rand(self.update_epochs, self.P, self.S, generator=self.gen, device=self.device)
            perms = torch.argsort(keys, dim=-1)
            ev = torch.cuda.Event()
            ev.record(side)
        self._perm_next = (perms, ev)

    def _learn_torch(self, perms: torch.Tensor | None = None) -> torch.Tensor:
        P, S, D = self.P, self.S, self.spec.obs_dim
        K.adv_normalize_(self.advantages, self.adv_stats)
        obs = self.obs.view(P, S, D)
        act = self.actions.view(P, S)
        old_logp = self.log_probs.view(-1)
        adv = self.advantages.view(-1)
        ret = self.returns.view(-1)
        old_v = self.values.view(-1)
        base = (torch.arange(P, device=self.device) * S).unsqueeze(1)
        if perms is None:
            perms = self.permutations()
        total = torch.zeros(P, dtype=torch.float32, device=self.device)
        for e in range(self.update_epochs):
            for s0, s1 in self.minibatch_plan():
                idx = perms[e][:, s0:s1]  # [P, b]
                ob = torch.gather(obs, 1, idx.unsqueeze(-1).expand(-1, -1, D))
                ac = torch.gather(act, 1, idx)
                logits, value = self.spec.forward(self.params, ob)
                logp_all, ent = categorical(logits)
                logp = logp_all.gather(-1, ac.unsqueeze(-1)).squeeze(-1)
                gidx = (idx + base).reshape(-1).contiguous()
                loss, stats = _PPOLossFn.apply(logp, value, ent, old_logp, adv, ret, old_v, gidx,
                                               s1 - s0, self.clip_coef, self.vf_coef, self.ent_coef)
                self.params.grad.zero_()
                loss.backward()
                self.opt.step()
                total += stats[:, 0]
        return total / (S * self.update_epochs)

    # ------------------------------------------------------------------ #
    @torch.no_grad()
    def evaluate(self, obs: torch.Tensor) -> torch.Tensor:
        """Greedy actions (mode of the categorical) for fitness evaluation."""
        logits, _ = self.spec.forward(self.params.data, obs)
        return torch.argmax(logits, dim=-1)

    def n_minibatches(self) -> int:
        return math.ceil(self.S / self.batch_size)
