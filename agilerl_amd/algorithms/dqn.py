"""Drop-in ``DQN`` (agilerl/algorithms/dqn.py:61-380) with the TD target,
MSE loss and its gradient in one HIP kernel (agx_td_target) and the soft
target update in agx_polyak.

The Q network is the reference's MLP (create_mlp, utils/evolvable_networks.py:
527-644: [Linear -> LayerNorm -> ReLU] x L -> Linear, orthogonal init gain
sqrt(2), output layer x0.1), as plain PyTorch modules on the GPU; ``learn``
takes the reference's experience mapping (obs, action, reward, next_obs,
done) and returns the loss as a float.  Supported: Box observations,
Discrete actions, ``net_config`` ``encoder_config`` / ``head_config``
``hidden_size`` lists.
"""

from __future__ import annotations

import math
from typing import Any

import numpy as np
import torch
from torch import nn

from .. import kernels as K


def _hidden(cfg, default):
    if cfg is None:
        return list(default)
    return list(getattr(cfg, "hidden_size", None) or cfg.get("hidden_size", default))


def build_q_mlp(obs_dim: int, n_actions: int, net_config: dict | None, seed: int | None = None) -> nn.Sequential:
    net_config = dict(net_config or {})
    hidden = _hidden(net_config.get("encoder_config"), [64])
    latent = int(net_config.get("latent_dim", 64))
    head = _hidden(net_config.get("head_config"), [64])
    dims = [obs_dim, *hidden, latent, *head]
    gen = torch.Generator().manual_seed(seed) if seed is not None else None
    layers: list[nn.Module] = []
    for i in range(len(dims) - 1):
        lin = nn.Linear(dims[i], dims[i + 1])
        nn.init.orthogonal_(lin.weight, math.sqrt(2), generator=gen)
        nn.init.zeros_(lin.bias)
        layers += [lin, nn.LayerNorm(dims[i + 1]), nn.ReLU()]
    out = nn.Linear(dims[-1], n_actions)
    nn.init.orthogonal_(out.weight, math.sqrt(2), generator=gen)
    nn.init.zeros_(out.bias)
    with torch.no_grad():
        out.weight.mul_(0.1)  # output_vanish (evolvable_networks.py:621-629)
    layers.append(out)
    return nn.Sequential(*layers)


class _TDLoss(torch.autograd.Function):
    """MSE(Q(s)[a], r + gamma * q_t * (1 - d)) with the HIP kernel computing
    y, the loss and dLoss/dQ(s) in one pass."""

    @staticmethod
    def forward(ctx, q_cur, q_next_target, q_next_online, actions, rewards, dones, gamma, double):
        _, g_q, loss = K.td_target(q_next_target.contiguous(), rewards, dones, gamma,
                                   q_next_online=q_next_online.contiguous() if double else None, double=double,
                                   q_cur=q_cur.contiguous(), actions=actions)
        ctx.save_for_backward(g_q)
        return loss.view(())

    @staticmethod
    def backward(ctx, gl):
        (g_q,) = ctx.saved_tensors
        return (g_q * gl,) + (None,) * 7


class DQN:
    algo = "DQN"

    def __init__(self, observation_space, action_space, index: int = 0, hp_config=None, net_config=None,
                 batch_size: int = 64, lr: float = 1e-4, learn_step: int = 5, gamma: float = 0.99,
                 tau: float = 1e-3, mut=None, normalize_images: bool = True, double: bool = False,
                 actor_network=None, device="cuda", accelerator=None, cudagraphs: bool = False, wrap: bool = True):
        if not hasattr(action_space, "n"):
            raise NotImplementedError("agx DQN supports Discrete action spaces")
        if actor_network is not None:
            raise NotImplementedError("custom actor modules: use net_config (MLP) networks")
        assert isinstance(batch_size, int) and batch_size >= 1, "Batch size must be an integer greater than or equal to one."
        assert lr > 0, "Learning rate must be greater than zero."
        self.observation_space, self.action_space = observation_space, action_space
        self.index, self.net_config, self.mut = index, net_config, mut
        self.batch_size, self.lr, self.learn_step = batch_size, lr, learn_step
        self.gamma, self.tau, self.double = gamma, tau, double
        self.device = torch.device(device)
        self.action_dim = int(action_space.n)
        self.obs_dim = int(np.prod(observation_space.shape))
        self.actor = build_q_mlp(self.obs_dim, self.action_dim, net_config, seed=index).to(self.device)
        self.actor_target = build_q_mlp(self.obs_dim, self.action_dim, net_config).to(self.device)
        self.actor_target.load_state_dict(self.actor.state_dict())
        self.optimizer = torch.optim.Adam(self.actor.parameters(), lr=lr)
        self.scores: list[float] = []
        self.fitness: list[float] = []
        self.steps: list[int] = [0]

    @classmethod
    def from_init_hp(cls, observation_space, action_space, net_config, INIT_HP, index=0, device="cuda", **kw):
        return cls(observation_space, action_space, index=index, net_config=net_config,
                   batch_size=INIT_HP.get("BATCH_SIZE", 64), lr=INIT_HP.get("LR", 1e-4),
                   learn_step=INIT_HP.get("LEARN_STEP", 5), gamma=INIT_HP.get("GAMMA", 0.99),
                   tau=INIT_HP.get("TAU", 1e-3), double=INIT_HP.get("DOUBLE", False), device=device, **kw)

    def _obs(self, obs) -> torch.Tensor:
        return torch.as_tensor(np.asarray(obs) if not isinstance(obs, torch.Tensor) else obs,
                               dtype=torch.float32).to(self.device).reshape(-1, self.obs_dim)

    @torch.no_grad()
    def get_action(self, obs, epsilon: float = 0.0, action_mask=None, *args: Any, **kwargs: Any) -> np.ndarray:
        """Epsilon-greedy action(s) (dqn.py:188-250)."""
        o = self._obs(obs)
        q = self.actor(o)
        if action_mask is not None:
            m = torch.as_tensor(np.asarray(action_mask), device=self.device).reshape(q.shape).bool()
            q = q.masked_fill(~m, -float("inf"))
        greedy = q.argmax(dim=1)
        if epsilon > 0:
            rand = torch.rand(o.shape[0], device=self.device) < epsilon
            if action_mask is not None:
                random_a = torch.multinomial(m.float(), 1).view(-1)
            else:
                random_a = torch.randint(0, self.action_dim, (o.shape[0],), device=self.device)
            greedy = torch.where(rand, random_a, greedy)
        return greedy.cpu().numpy()

    def update(self, obs, actions, rewards, next_obs, dones) -> torch.Tensor:
        with torch.no_grad():
            q_next_target = self.actor_target(next_obs)
            q_next_online = self.actor(next_obs) if self.double else None
        q_cur = self.actor(obs)
        loss = _TDLoss.apply(q_cur, q_next_target, q_next_online, actions.reshape(-1).long().contiguous(),
                             rewards.reshape(-1).float().contiguous(), dones.reshape(-1).float().contiguous(),
                             float(self.gamma), bool(self.double))
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
        return loss.detach()

    def learn(self, experiences) -> float:
        """experiences: mapping with obs, action, reward, next_obs, done (dqn.py:326-348)."""
        get = experiences.get if hasattr(experiences, "get") else (lambda k: experiences[k])
        obs = self._obs(get("obs"))
        next_obs = self._obs(get("next_obs"))
        to = lambda x: torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x).to(self.device)
        loss = self.update(obs, to(get("action")), to(get("reward")), next_obs, to(get("done")))
        self.soft_update()
        return float(loss.item())

    @torch.no_grad()
    def soft_update(self) -> None:
        """target <- tau * online + (1 - tau) * target (dqn.py:349-358), one
        agx_polyak launch per parameter tensor."""
        for t, o in zip(self.actor_target.parameters(), self.actor.parameters()):
            K.polyak_(t.data.view(-1), o.data.reshape(-1), float(self.tau))

    @torch.no_grad()
    def test(self, env, swap_channels: bool = False, max_steps: int | None = None, loop: int = 3) -> float:
        rewards = []
        num_envs = env.num_envs if hasattr(env, "num_envs") else 1
        for _ in range(loop):
            obs, _ = env.reset()
            scores = np.zeros(num_envs)
            completed = np.zeros(num_envs)
            finished = np.zeros(num_envs, dtype=bool)
            step = 0
            while not np.all(finished):
                obs, r, term, trunc, _ = env.step(self.get_action(obs, epsilon=0.0))
                step += 1
                scores += np.asarray(r).reshape(num_envs)
                done = np.logical_or(term, trunc).reshape(num_envs)
                if max_steps is not None and step == max_steps:
                    done[:] = True
                for i in range(num_envs):
                    if done[i] and not finished[i]:
                        completed[i] = scores[i]
                        finished[i] = True
            rewards.append(float(np.mean(completed)))
        f = float(np.mean(rewards))
        self.fitness.append(f)
        return f


class RainbowDQN:
    """Placeholder kept for create_population's dispatch: the Rainbow
    projection + loss is available as ``agilerl_amd.kernels.c51_project_loss``
    (agx_c51_project_loss, bit-exact to dqn_rainbow.py:284-367); the noisy
    dueling distributional network around it is outside this round's scope."""

    @classmethod
    def from_init_hp(cls, *a, **k):
        raise NotImplementedError("RainbowDQN agent: use agilerl_amd.kernels.c51_project_loss for the loss")
