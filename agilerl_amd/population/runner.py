"""Host env workers <-> HBM rollout SoA for a whole population.

One vector step of every agent = one batched inference launch sequence on the
GPU, one pinned D2H of the actions (the only synchronisation), the host env
step writing straight into pinned staging buffers, and async H2D copies into
the (P, T, N) rollout arrays (reference: agilerl/rollouts/on_policy.py:23-203,
one agent at a time through CPU TensorDicts).
"""

from __future__ import annotations

import torch

from .ppo_pop import PPOPopulation


class PopulationRunner:
    def __init__(self, pop: PPOPopulation, env):
        if env.num_envs != pop.P * pop.N:
            raise ValueError(f"env has {env.num_envs} envs, population needs P*N = {pop.P * pop.N}")
        self.pop, self.env = pop, env
        P, N, D = pop.P, pop.N, pop.spec.obs_dim
        pin = dict(pin_memory=True)
        self.obs_h = torch.zeros(P * N, D, dtype=torch.float32, **pin)
        self.rew_h = torch.zeros(P * N, dtype=torch.float32, **pin)
        self.done_h = torch.zeros(P * N, dtype=torch.bool, **pin)
        self.term_h = torch.zeros(P * N, dtype=torch.bool, **pin)
        self.act_h = torch.zeros(P * N, dtype=torch.int64, **pin)
        self.act_d = torch.zeros(P * N, dtype=torch.int64, device=pop.device)
        self.last_obs = torch.zeros(P, N, D, dtype=torch.float32, device=pop.device)
        self.last_done = torch.zeros(P, N, dtype=torch.uint8, device=pop.device)
        self.ev = torch.cuda.Event()
        self.started = False
        self.env_steps = 0
        self.scores = torch.zeros(P, N, dtype=torch.float32, device=pop.device)
        self.episode_return_sum = torch.zeros(P, dtype=torch.float64, device=pop.device)
        self.episodes = torch.zeros(P, dtype=torch.int64, device=pop.device)

    def _h2d(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        dst.copy_(src.view(dst.shape), non_blocking=True)

    @torch.no_grad()
    def collect(self) -> None:
        pop, env = self.pop, self.env
        P, N, T = pop.P, pop.N, pop.T
        if not self.started:
            env.reset(out_obs=self.obs_h.numpy())
            self._h2d(self.last_obs, self.obs_h)
            self.started = True
        pop.obs[:, 0].copy_(self.last_obs)
        for t in range(T):
            pop.act_into(t, self.act_d)
            self.act_h.copy_(self.act_d, non_blocking=True)
            self.ev.record()
            self.ev.synchronize()
            _, _, term, trunc, _ = env.step(self.act_h.numpy(), out_obs=self.obs_h.numpy(),
                                            out_rew=self.rew_h.numpy(), out_done=self.done_h.numpy())
            if trunc is not None and trunc.any():  # done = term | trunc (on_policy.py:121-126)
                self.done_h.numpy()[:] |= trunc
            self.term_h.numpy()[:] = term
            self._h2d(pop.rewards[:, t], self.rew_h)
            self._h2d(pop.dones[:, t], self.done_h.view(torch.uint8))
            nxt = pop.obs[:, t + 1] if t + 1 < T else self.last_obs
            self._h2d(nxt, self.obs_h)
            # running episode scores for fitness (on_policy.py:147-172)
            self.scores += pop.rewards[:, t]
            d = pop.dones[:, t].bool()
            self.episode_return_sum += torch.where(d, self.scores, 0.0).sum(1).double()
            self.episodes += d.sum(1)
            self.scores.masked_fill_(d, 0.0)
        self._h2d(self.last_done, self.term_h.view(torch.uint8))  # last_done = term only (:196)
        self.env_steps += P * N * T

    def iteration(self) -> torch.Tensor:
        """collect -> bootstrap + GAE -> learn; returns per-agent mean loss (device)."""
        self.collect()
        self.pop.finish_rollout(self.last_obs, self.last_done)
        return self.pop.learn()
