"""Drop-in ``DQN`` (agilerl/algorithms/dqn.py:61-380) with the TD target,
MSE loss and its gradient in one HIP kernel (agx_td_target) and the soft
target update in agx_polyak.

The Q networks are the reference's ``QNetwork`` / ``RainbowQNetwork``
(agilerl_amd.networks: EvolvableMLP encoder + head with the reference's
defaults, initialisation and state-dict keys) on the GPU; ``learn`` takes the reference's experience mapping (obs, action, reward, next_obs,
done) and returns the loss as a float.  Supported: Box observations (vectors, or
image frames through EvolvableCNN encoders on the HIP conv kernels),
Discrete actions, ``net_config`` ``encoder_config`` / ``head_config``
``hidden_size`` lists.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .. import kernels as K
from . import checkpoint as C
from .evolvable import EvolvableAgentMixin
from . import learn_graph
from .flat_state import flat_state
from ..modules.custom_components import noisy_scope
from ..networks import QNetwork, RainbowQNetwork
from ..networks.base import image_norm_bounds, is_image_space, mlp_net_config


def _setup_image_input(agent, normalize_images: bool) -> None:
    """Image Box spaces: the networks get EvolvableCNN encoders; with
    normalize_images and finite [low, high] != [0, 1] the frames stay uint8
    up to the first convolution, which normalises them in its load
    (preprocess_observation -> apply_image_normalization, algo_utils.py:
    996-1022, 1134-1183)."""
    agent.normalize_images = normalize_images
    agent._image = is_image_space(agent.observation_space)
    agent._img_norm = image_norm_bounds(agent.observation_space) if agent._image and normalize_images else None
    for net in (agent.actor, agent.actor_target):
        net.set_image_norm(agent._img_norm)


def _obs_tensor(agent, obs) -> torch.Tensor:
    x = obs if isinstance(obs, torch.Tensor) else torch.as_tensor(np.asarray(obs))
    x = x.to(agent.device)
    if not agent._image:
        return x.to(torch.float32).reshape(-1, agent.obs_dim)
    x = x.reshape(-1, *agent.observation_space.shape)
    if x.dtype == torch.uint8 and agent._img_norm is not None:
        return x  # normalised inside the first convolution
    x = x.to(torch.float32)
    if agent._img_norm is not None:  # float frames: the reference's (x - low) / (high - low) in f32
        lo, hi = agent._img_norm
        x = (x - lo) / float(np.float32(hi) - np.float32(lo))
    return x


def _net_kwargs(net_config) -> dict:
    return {k: (dict(v) if isinstance(v, dict) else v) for k, v in dict(net_config or {}).items()}


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


class DQN(EvolvableAgentMixin, C.TorchCheckpointMixin):
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
        # QNetwork with the reference's defaults and state-dict keys (dqn.py:133-146)
        self.actor = QNetwork(observation_space, action_space, device=self.device, **_net_kwargs(net_config))
        self.actor_target = QNetwork(observation_space, action_space, device=self.device, **_net_kwargs(net_config))
        self.actor_target.load_state_dict(self.actor.state_dict())
        _setup_image_input(self, normalize_images)
        self.optimizer = torch.optim.Adam(self.actor.parameters(), lr=lr)
        self._init_registry(hp_config)
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
        return _obs_tensor(self, obs)

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
        fs = flat_state(self)
        if fs is None or not fs.step(0.0):  # Adam over the flat buffers: one launch (flat_state.py)
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

    def _fresh_optimizer(self, lr_name: str):
        return torch.optim.Adam(self.actor.parameters(), lr=self.lr)

    def clone(self, index: int | None = None, wrap: bool = True):
        """Deep copy with a new index (EvolvableAlgorithm.clone, core/base.py)."""
        import copy

        c = copy.deepcopy(self)
        if index is not None:
            c.index = index
        return c

    @torch.no_grad()
    def soft_update(self) -> None:
        """target <- tau * online + (1 - tau) * target (dqn.py:349-358): one
        agx_polyak launch over the flat buffers (flat_state.py), else one per
        parameter tensor."""
        fs = flat_state(self)
        if fs is not None:
            fs.polyak(self.tau)
            return
        for t, o in zip(self.actor_target.parameters(), self.actor.parameters()):
            K.polyak_(t.data.view(-1), o.data.reshape(-1), float(self.tau))

    @torch.no_grad()
    def test(self, env, swap_channels: bool = False, max_steps: int | None = None, loop: int = 3) -> float:
        return _evaluate(self, env, lambda o: self.get_action(o, epsilon=0.0), max_steps, loop)


def _evaluate(agent, env, act, max_steps, loop) -> float:
    """Mean over ``loop`` passes of the score of every env's first finished
    episode (the reference algorithms' ``test``); appended to agent.fitness."""
    rewards = []
    num_envs = env.num_envs if hasattr(env, "num_envs") else 1
    for _ in range(loop):
        obs, _ = env.reset()
        scores = np.zeros(num_envs)
        completed = np.zeros(num_envs)
        finished = np.zeros(num_envs, dtype=bool)
        step = 0
        while not np.all(finished):
            obs, r, term, trunc, _ = env.step(act(obs))
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
    agent.fitness.append(f)
    return f


class _C51Loss(torch.autograd.Function):
    """Elementwise C51 cross entropy with the projection in agx_c51_project_loss
    (bit-exact to the serial index_add_, dqn_rainbow.py:313-367); the gradient
    w.r.t. log_p[i, a_i, :] is -proj[i, :]."""

    @staticmethod
    def forward(ctx, logp_cur, q_next_online, target_dist, actions, rewards, dones, support, v_min, v_max, gamma):
        loss, proj = K.c51_project_loss(q_next_online.contiguous(), target_dist.contiguous(), logp_cur.contiguous(),
                                        actions, rewards, dones, support, v_min, v_max, gamma, with_proj=True)
        ctx.save_for_backward(proj, actions)
        ctx.shape = logp_cur.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        proj, actions = ctx.saved_tensors
        grad = torch.zeros(ctx.shape, dtype=proj.dtype, device=proj.device)
        grad[torch.arange(proj.shape[0], device=proj.device), actions] = -proj * g.unsqueeze(1)
        return (grad,) + (None,) * 9


class _C51RowsLoss(torch.autograd.Function):
    """The same loss on the selected rows (agx_c51_project_loss_rows): log p
    of the taken action [B, Z] and the target distribution of a* [B, Z], as
    the dueling head emits them; d loss / d logp_rows = -proj."""

    @staticmethod
    def forward(ctx, logp_rows, target_rows, rewards, dones, support, v_min, v_max, gamma):
        loss, proj = K.c51_project_loss_rows(target_rows.contiguous(), logp_rows.contiguous(), rewards, dones, support,
                                             v_min, v_max, gamma, with_proj=True)
        ctx.save_for_backward(proj)
        return loss

    @staticmethod
    def backward(ctx, g):
        (proj,) = ctx.saved_tensors
        return (-proj * g.unsqueeze(1),) + (None,) * 7


@torch.no_grad()
def _next_pair(agent, next_obs):
    """The two no-grad forwards of a Rainbow update on s' (dqn_rainbow.py:
    284-367: a* = argmax_a Q_online(s'), then the target network's
    distribution of a*) with both networks in one launch per layer: the flat
    state keeps online and target parameters as the two rows of one buffer,
    so every convolution is a grouped launch over (online, target) reading
    the same frames, the encoder's Linear one batched GEMM, and the four head
    streams one agx_noisy_streams_forward_each launch per depth.  -> (a*,
    target rows [B, Z]), or None where the network is not the CNN + dueling
    head this covers (the caller runs the reference's two forwards)."""
    import ctypes

    from torch import nn

    from .. import _lib
    from ..modules.cnn import AgxConv2d, EvolvableCNN, _FusedIdentity, _shape
    from ..modules.noisy_streams import head_streams_each
    from ..networks.q_networks import DuelingDistributionalMLP, DuelingHeadFn, DuelingRowsFn
    from .learn_graph import _hooked

    actor, target = agent.actor, agent.actor_target
    enc = getattr(actor, "encoder", None)
    if (not isinstance(enc, EvolvableCNN) or not isinstance(getattr(actor, "head_net", None), DuelingDistributionalMLP)
            or getattr(actor, "flatten_obs", False) or not isinstance(next_obs, torch.Tensor) or not next_obs.is_cuda
            or next_obs.dim() != 4 or agent.num_atoms > 64 or _hooked(actor, target)):
        return None
    fs = flat_state(agent)
    if fs is None:
        return None
    B = next_obs.shape[0]
    x, first = next_obs.contiguous(), True
    for _, mod in enc.model.named_children():
        if type(mod) is AgxConv2d:
            u8 = x.dtype == torch.uint8
            if (u8 and mod.image_norm is None) or (not u8 and x.dtype != torch.float32) or mod.bias is None:
                return None
            xs = x if first else x[0]
            sh = _shape(xs, mod.weight, int(mod.stride[0]))
            OH = (sh.height - sh.kernel_h) // sh.stride + 1
            OW = (sh.width - sh.kernel_w) // sh.stride + 1
            y = torch.empty(2, B, mod.out_channels, OH, OW, dtype=torch.float32, device=x.device)
            w2, b2 = fs.pair_view(mod.weight), fs.pair_view(mod.bias)
            lo, hi = (float(mod.image_norm[0]), float(mod.image_norm[1])) if u8 else (0.0, 1.0)
            _lib.call("agx_conv2d_forward_grouped", ctypes.byref(sh), 2, x.data_ptr(), 0 if first else x[0].numel(),
                      int(u8), lo, hi, w2.data_ptr(), w2.stride(0), b2.data_ptr(), b2.stride(0), int(mod.fuse_relu),
                      y.data_ptr(), y[0].numel(), _lib.stream())
            x, first = y, False
        elif type(mod) is _FusedIdentity or type(mod) is nn.Identity:
            pass
        elif type(mod) is nn.ReLU:
            x = torch.relu(x)
        elif type(mod) is nn.Flatten and not first:
            x = x.reshape(2, B, -1)
        elif type(mod) is nn.Linear and not first and x.dim() == 3 and mod.bias is not None:
            w2, b2 = fs.pair_view(mod.weight), fs.pair_view(mod.bias)
            x = torch.baddbmm(b2.unsqueeze(1), x, w2.transpose(1, 2))
        else:
            return None
    if first or x.dim() != 3:
        return None
    ha, ht = actor.head_net, target.head_net
    out = head_streams_each([ha.model, ha.advantage_net, ht.model, ht.advantage_net], [x[0], x[0], x[1], x[1]])
    if out is None:
        return None
    v_on, a_on, v_tg, a_tg = out
    A, Z = agent.action_dim, agent.num_atoms
    q = DuelingHeadFn.apply(v_on, a_on, ha.support, A, Z, 0)
    a_star = q.argmax(1)  # first maximum, as the reference's argmax
    return a_star, DuelingRowsFn.apply(v_tg, a_tg, a_star, A, Z, 1)


class _TripleConvFn(torch.autograd.Function):
    """One encoder layer of a Rainbow update's three forwards in one launch
    (agx_conv2d_forward_grouped2, group g = g1 + 2 g2): g = 0 the online
    network on s', 1 the online network on s (the one the loss
    differentiates), 2 the target network on s'; g1 picks the frames, g2 the
    network (online and target parameters are the rows of the flat state's
    pair buffer, n elements apart).  -> (y3 [3, B, C, OH, OW] without
    gradient, y3[1] with it); the backward is group 1's convolution backward
    alone (Conv2dFn.backward)."""

    @staticmethod
    def forward(ctx, x1, w, b, x3, x_strides, n, stride, relu, norm):
        import ctypes

        from .. import _lib
        from ..modules.cnn import _shape

        u8 = x1.dtype == torch.uint8
        sh = _shape(x1, w, stride)
        OH = (sh.height - sh.kernel_h) // stride + 1
        OW = (sh.width - sh.kernel_w) // stride + 1
        B = x1.shape[0]
        y3 = torch.empty(3, B, w.shape[0], OH, OW, dtype=torch.float32, device=x1.device)
        Y = y3[0].numel()
        lo, hi = (float(norm[0]), float(norm[1])) if u8 else (0.0, 1.0)
        _lib.call("agx_conv2d_forward_grouped2", ctypes.byref(sh), 3, 2, x3.data_ptr(), x_strides[0], x_strides[1],
                  int(u8), lo, hi, w.data_ptr(), 0, n, b.data_ptr(), 0, n, int(relu), y3.data_ptr(), Y, 2 * Y,
                  _lib.stream())
        y1 = y3[1]
        ctx.save_for_backward(x1, w, y1 if relu else None)
        ctx.meta = (stride, relu, u8, lo, hi)
        ctx.mark_non_differentiable(y3)
        ctx.set_materialize_grads(False)  # no zero-filled [3, B, C, OH, OW] gradient for y3
        return y3, y1

    @staticmethod
    def backward(ctx, _g3, dy):
        import ctypes

        from .. import _lib
        from ..modules.cnn import _shape

        x, w, y = ctx.saved_tensors
        stride, relu, u8, lo, hi = ctx.meta
        if dy is None:
            return (None,) * 9
        sh = _shape(x, w, stride)
        dy = dy.contiguous()
        dw = torch.empty_like(w)
        db = torch.empty(w.shape[0], dtype=torch.float32, device=w.device)
        dx = torch.empty_like(x) if (ctx.needs_input_grad[0] and not u8) else None
        ws = torch.empty(max(16, _lib.load().agx_conv2d_wgrad_workspace_bytes(ctypes.byref(sh))), dtype=torch.uint8,
                         device=w.device)
        _lib.call("agx_conv2d_backward", ctypes.byref(sh), x.data_ptr(), int(u8), lo, hi, w.data_ptr(), _lib.ptr(y),
                  dy.data_ptr(), _lib.ptr(dx), dw.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), _lib.stream())
        return dx, dw, db, None, None, None, None, None, None


def _triple_pass(agent, obs, acts, next_obs):
    """A Rainbow update's three network passes (dqn_rainbow.py:284-367: the
    online network on s' for a*, the target network on s' for the target
    distribution, the online network on s for log p) with every encoder layer
    one grouped launch over all three (_TripleConvFn), the pair's Linear one
    batched GEMM, the pair's four head streams one launch per depth and the
    online head on s the autograd head streams.  -> (log p rows [B, Z] with
    gradient, target rows [B, Z]), or None where the network is not the CNN +
    dueling head this covers (the caller runs the three forwards)."""
    from torch import nn
    from torch.nn import functional as F

    from ..modules.cnn import AgxConv2d, EvolvableCNN, _FusedIdentity
    from ..modules.noisy_streams import head_streams_each, mixed_streams
    from ..networks.q_networks import DuelingDistributionalMLP, DuelingHeadFn, DuelingRowsFn
    from .learn_graph import _hooked

    actor, target = agent.actor, agent.actor_target
    enc = getattr(actor, "encoder", None)
    if (not isinstance(enc, EvolvableCNN) or not isinstance(getattr(actor, "head_net", None), DuelingDistributionalMLP)
            or getattr(actor, "flatten_obs", False) or not isinstance(next_obs, torch.Tensor)
            or not isinstance(obs, torch.Tensor) or not next_obs.is_cuda or next_obs.dim() != 4
            or obs.shape != next_obs.shape or obs.dtype != next_obs.dtype or agent.num_atoms > 64
            or _hooked(actor, target) or not torch.is_grad_enabled()):
        return None
    fs = flat_state(agent)
    if fs is None:
        return None
    mods = list(enc.model.children())
    convs = [m for m in mods if type(m) is AgxConv2d]
    if not convs or any(m.bias is None for m in convs):
        return None
    if obs.dtype == torch.uint8 and convs[0].image_norm is None:
        return None
    if obs.dtype not in (torch.uint8, torch.float32):
        return None
    B = obs.shape[0]
    frames = torch.stack([next_obs, obs])  # g1 = 0: s', g1 = 1: s
    x1, x3, xs, first = frames[1], frames, (frames[0].numel(), 0), True
    y3 = None
    lat_pair = lat_s = None
    for mod in mods:
        if type(mod) is AgxConv2d:
            y3, x1 = _TripleConvFn.apply(x1, mod.weight, mod.bias, x3, xs, fs.n, int(mod.stride[0]), mod.fuse_relu,
                                         mod.image_norm if x1.dtype == torch.uint8 else None)
            x3, xs, first = y3, (y3[0].numel(), 2 * y3[0].numel()), False
        elif type(mod) is _FusedIdentity or type(mod) is nn.Identity:
            pass
        elif type(mod) is nn.Flatten and not first and lat_pair is None:
            pass  # flattened below with the Linear
        elif type(mod) is nn.Linear and not first and lat_pair is None and mod.bias is not None:
            F_ = y3[0].numel() // B
            pair = y3.reshape(3, B, F_)[0::2]  # online and target on s'
            w2, b2 = fs.pair_view(mod.weight), fs.pair_view(mod.bias)
            with torch.no_grad():
                lat_pair = torch.baddbmm(b2.unsqueeze(1), pair, w2.transpose(1, 2))
            lat_s = F.linear(x1.reshape(B, F_), mod.weight, mod.bias)
        elif type(mod) is nn.ReLU and lat_pair is not None:
            with torch.no_grad():
                lat_pair = torch.relu(lat_pair)
            lat_s = torch.relu(lat_s)
        else:
            return None
    if lat_pair is None:
        return None
    ha, ht = actor.head_net, target.head_net
    A, Z = agent.action_dim, agent.num_atoms
    # the pair's four streams (no gradient) and the online head on s (with
    # it) in one launch per depth
    out = mixed_streams([ha.model, ha.advantage_net, ht.model, ht.advantage_net],
                        [lat_pair[0], lat_pair[0], lat_pair[1], lat_pair[1]], [ha.model, ha.advantage_net], lat_s)
    if out is not None:
        v_on, a_on, v_tg, a_tg, v_s, a_s = out
        logp_rows = DuelingRowsFn.apply(v_s, a_s, acts, A, Z, 2)
    else:
        with torch.no_grad():
            out = head_streams_each([ha.model, ha.advantage_net, ht.model, ht.advantage_net],
                                    [lat_pair[0], lat_pair[0], lat_pair[1], lat_pair[1]])
        if out is None:
            return None
        v_on, a_on, v_tg, a_tg = out
        logp_rows = actor.head_net(lat_s, q=False, log=True, rows=acts)
    with torch.no_grad():
        a_star = DuelingHeadFn.apply(v_on, a_on, ha.support, A, Z, 0).argmax(1)  # first maximum, as the reference
        target_rows = DuelingRowsFn.apply(v_tg, a_tg, a_star, A, Z, 1)
    return logp_rows, target_rows


class RainbowDQN(EvolvableAgentMixin, C.TorchCheckpointMixin):
    """Drop-in RainbowDQN (agilerl/algorithms/dqn_rainbow.py:77-501) with the
    C51 projection + loss in agx_c51_project_loss and Polyak in agx_polyak."""

    algo = "Rainbow DQN"

    def __init__(self, observation_space, action_space, index: int = 0, hp_config=None, net_config=None,
                 batch_size: int = 64, lr: float = 1e-4, learn_step: int = 5, gamma: float = 0.99, tau: float = 1e-3,
                 beta: float = 0.4, prior_eps: float = 1e-6, num_atoms: int = 51, v_min: float = 0,
                 v_max: float = 200, noise_std: float = 0.5, n_step: int = 3, mut=None,
                 normalize_images: bool = True, combined_reward: bool = False, actor_network=None, device="cuda",
                 accelerator=None, wrap: bool = True):
        if not hasattr(action_space, "n"):
            raise NotImplementedError("agx RainbowDQN supports Discrete action spaces")
        if actor_network is not None:
            raise NotImplementedError("custom actor modules: use net_config (MLP) networks")
        assert isinstance(batch_size, int) and batch_size >= 1, "Batch size must be an integer greater than or equal to one."
        assert lr > 0, "Learning rate must be greater than zero."
        self.observation_space, self.action_space = observation_space, action_space
        self.index, self.net_config, self.mut = index, net_config, mut
        self.batch_size, self.lr, self.learn_step = batch_size, lr, learn_step
        self.gamma, self.tau, self.beta, self.prior_eps = gamma, tau, beta, prior_eps
        self.num_atoms, self.v_min, self.v_max, self.noise_std = num_atoms, v_min, v_max, noise_std
        self.n_step, self.combined_reward = n_step, combined_reward
        self.device = torch.device(device)
        self.action_dim = int(action_space.n)
        self.obs_dim = int(np.prod(observation_space.shape))
        self.support = torch.linspace(v_min, v_max, num_atoms, device=self.device)
        self.delta_z = (v_max - v_min) / (num_atoms - 1)
        # dqn_rainbow.py:190-215: head defaults hidden [64], noisy, output activation ReLU -> None
        self.actor = RainbowQNetwork(observation_space, action_space, support=self.support, num_atoms=num_atoms,
                                     noise_std=noise_std, device=self.device, **self._net_kwargs(net_config))
        self.actor_target = RainbowQNetwork(observation_space, action_space, support=self.support,
                                            num_atoms=num_atoms, noise_std=noise_std, device=self.device,
                                            **self._net_kwargs(net_config))
        self.actor_target.load_state_dict(self.actor.state_dict())
        _setup_image_input(self, normalize_images)
        self.optimizer = torch.optim.Adam(self.actor.parameters(), lr=lr)
        self._init_registry(hp_config)
        self.scores: list[float] = []
        self.fitness: list[float] = []
        self.steps: list[int] = [0]

    def _net_kwargs(self, net_config) -> dict:
        kw = _net_kwargs(net_config)
        head = dict(kw.get("head_config") or {})
        kw["head_config"] = mlp_net_config(head.get("hidden_size", [64]), noise_std=self.noise_std,
                                           output_activation="ReLU", min_mlp_nodes=head.get("min_mlp_nodes", 16),
                                           max_mlp_nodes=head.get("max_mlp_nodes", 500))
        return kw

    @classmethod
    def from_init_hp(cls, observation_space, action_space, net_config, INIT_HP, index=0, device="cuda", **kw):
        return cls(observation_space, action_space, index=index, net_config=net_config,
                   batch_size=INIT_HP.get("BATCH_SIZE", 64), lr=INIT_HP.get("LR", 1e-4),
                   learn_step=INIT_HP.get("LEARN_STEP", 5), gamma=INIT_HP.get("GAMMA", 0.99),
                   tau=INIT_HP.get("TAU", 1e-3), beta=INIT_HP.get("BETA", 0.4),
                   prior_eps=INIT_HP.get("PRIOR_EPS", 1e-5), num_atoms=INIT_HP.get("NUM_ATOMS", 51),
                   v_min=INIT_HP.get("V_MIN", -100), v_max=INIT_HP.get("V_MAX", 100),  # utils.py:454-457
                   n_step=INIT_HP.get("N_STEP", 3), device=device, **kw)

    def _obs(self, obs) -> torch.Tensor:
        return _obs_tensor(self, obs)

    @torch.no_grad()
    def get_action(self, obs, action_mask=None, training: bool = True, *args, **kwargs) -> np.ndarray:
        self.actor.train(mode=training)
        q = self.actor(self._obs(obs)).cpu().numpy()
        self.actor.train()
        if action_mask is None:
            return np.argmax(q, axis=-1)
        return np.argmax(np.ma.array(q, mask=1 - np.asarray(action_mask)), axis=-1)

    def _dqn_loss(self, obs, actions, rewards, next_obs, dones, gamma) -> torch.Tensor:
        acts = actions.reshape(-1).long().contiguous()
        rew = rewards.reshape(-1).float().contiguous()
        done = dones.reshape(-1).float().contiguous()
        if self.num_atoms == 51 and self.device.type == "cuda":
            # the heads emit only the selected rows (target_dist[range(B), a*],
            # log_p[range(B), action]); the C51 step streams them contiguously
            fused = _triple_pass(self, obs, acts, next_obs)
            if fused is not None:
                logp_rows, target_rows = fused
                return _C51RowsLoss.apply(logp_rows, target_rows, rew, done, self.support, float(self.v_min),
                                          float(self.v_max), float(gamma))
            with torch.no_grad():
                pair = _next_pair(self, next_obs)
                if pair is not None:
                    a_star, target_rows = pair
                else:
                    a_star = self.actor(next_obs).argmax(1)     # first maximum, as the reference's argmax
                    target_rows = self.actor_target(next_obs, q=False, rows=a_star)
            logp_rows = self.actor(obs, q=False, log=True, rows=acts)
            return _C51RowsLoss.apply(logp_rows, target_rows, rew, done, self.support, float(self.v_min),
                                      float(self.v_max), float(gamma))
        with torch.no_grad():
            q_next = self.actor(next_obs)                   # a* = argmax online Q(s')
            target_dist = self.actor_target(next_obs, q=False)
        logp = self.actor(obs, q=False, log=True)
        return _C51Loss.apply(logp, q_next, target_dist, acts, rew, done, self.support, float(self.v_min),
                              float(self.v_max), float(gamma))

    @torch.no_grad()
    def test(self, env, swap_channels: bool = False, max_steps: int | None = None, loop: int = 3) -> float:
        return _evaluate(self, env, lambda o: self.get_action(o, training=False), max_steps, loop)

    def _losses(self, xs: list, n_step: bool, per: bool):
        """The update's loss and backward pass over xs = [obs, action, reward,
        next_obs, done] (+ the n-step batch's five) (+ PER weights)."""
        el = None
        with noisy_scope():  # each noisy layer's mu + sigma * eps formed once for the update's forwards
            if self.combined_reward or not n_step:
                el = self._dqn_loss(*xs[:5], self.gamma)
            if n_step:
                nl = self._dqn_loss(*xs[5:10], self.gamma ** self.n_step)
                el = el + nl if self.combined_reward else nl
        if per:
            # (B,) * (B,1) broadcasts to (B,B) in the reference: mean = mean(loss) * mean(w)
            loss = torch.mean(el * xs[-1])
        else:
            loss = torch.mean(el)
        self.optimizer.zero_grad()
        loss.backward()
        return loss, el

    def learn(self, experiences, n_experiences=None, per: bool = False):
        """-> (loss, idxs, new_priorities) (dqn_rainbow.py:369-490).  The
        device work is replayed from a captured graph from the second update
        of a given shape on (learn_graph.py)."""
        to = lambda x: torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x).to(self.device)
        get = lambda e, k: e[k]
        n_step = n_experiences is not None
        xs = [self._obs(get(experiences, "obs")), to(get(experiences, "action")), to(get(experiences, "reward")),
              self._obs(get(experiences, "next_obs")), to(get(experiences, "done"))]
        if n_step:
            xs += [self._obs(get(n_experiences, "obs")), to(get(n_experiences, "action")),
                   to(get(n_experiences, "reward")), self._obs(get(n_experiences, "next_obs")),
                   to(get(n_experiences, "done"))]
        if per:
            xs.append(to(get(experiences, "weights")))
        idxs = get(experiences, "idxs") if (per or n_step) else None
        fs = flat_state(self)
        nets = (self.actor, self.actor_target)
        g = self.optimizer.param_groups[0]
        key = ("rainbow", n_step, per, bool(self.combined_reward), float(self.gamma), int(self.n_step),
               float(self.v_min), float(self.v_max), int(self.num_atoms), float(self.tau), tuple(g["betas"]),
               float(g["eps"]))
        out = learn_graph.run(fs, key, xs, lambda s: self._losses(s, n_step, per), nets, 10.0, self.tau)
        if out is None:
            loss, el = self._losses(xs, n_step, per)
            flat_ok = fs is not None and fs.step(10.0)  # clip_grad_norm_(10) + Adam: one launch (flat_state.py)
            if flat_ok:
                fs.polyak(self.tau)
            else:
                torch.nn.utils.clip_grad_norm_(self.actor.parameters(), 10.0)
                self.optimizer.step()
                self.soft_update()
            self.actor.reset_noise()
            self.actor_target.reset_noise()
            learn_graph.note_eager(fs, key, xs, nets, flat_ok)
        else:
            loss, el = out
        new_priorities = el.detach().cpu().numpy() + self.prior_eps if per else None
        return loss.item(), idxs, new_priorities

    def _fresh_optimizer(self, lr_name: str):
        return torch.optim.Adam(self.actor.parameters(), lr=self.lr)

    def clone(self, index: int | None = None, wrap: bool = True):
        """Deep copy with a new index (EvolvableAlgorithm.clone, core/base.py)."""
        import copy

        c = copy.deepcopy(self)
        if index is not None:
            c.index = index
        return c

    @torch.no_grad()
    def soft_update(self) -> None:
        fs = flat_state(self)
        if fs is not None:
            fs.polyak(self.tau)
            return
        for t, o in zip(self.actor_target.parameters(), self.actor.parameters()):
            K.polyak_(t.data.view(-1), o.data.reshape(-1), float(self.tau))
