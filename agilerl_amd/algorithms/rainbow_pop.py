"""Population-batched Rainbow / DQN learner: one launch chain for all P agents.

The reference learns agent after agent (train_off_policy.py:249 ->
RainbowDQN.learn, dqn_rainbow.py:369-490): per agent a forward of the online
net on s' (a* = argmax Q), of the target net on s', of the online net on s,
the C51 projection + cross entropy, backward, clip_grad_norm_(10), Adam,
the Polyak soft update and a noise reset.  Here the P agents' networks live
as rows of flat ``[P, n]`` buffers (parameters, gradients, Adam moments,
target parameters, noise epsilons) and each agent's ``nn.Module`` tensors
are views into its row, so the agents stay ordinary ``RainbowDQN`` objects
(``get_action``, checkpoints, ``agent.learn`` all see the same storage).
One ``learn`` over P agents' batches is then:

  * every layer of all P networks in one launch: grouped implicit-GEMM
    convolutions reading each agent's filters in place from its row
    (agx_conv2d_*_grouped), batched GEMMs over the stacked ``[P, out, in]``
    row views for the Linear / NoisyLinear layers (noisy weights mu + sigma
    * eps formed once for all agents), LayerNorm over ``[P, B, F]``;
  * the dueling head on P*B rows emitting only the selected rows
    (agx_dueling_head_forward_rows: target distribution of a*, log p of the
    taken action) and the C51 projection + loss on P*B rows
    (agx_c51_project_loss_rows);
  * the per-agent PER-weighted mean (the reference's ``(B,) * (B, 1)``
    broadcast), one backward for all agents (their parameters are disjoint);
  * one fused clip + Adam launch over ``[P, n]`` (agx_clip_adam: per-agent
    norm, lr and step count) and one Polyak launch over ``[P, n]``;
  * the agents' noise resets in agent order (the reference's torch draws).

DQN agents (dqn.py:274-348) take the same chain with their Q head, the
TD target + MSE (agx_td_target, per agent) and Adam without clipping.
Agents whose hyperparameters differ in a way the batched chain does not
carry (batch size, gamma, tau, n-step / combined-reward settings) are
learned in groups of equal settings.
"""

from __future__ import annotations

import warnings
import weakref

import numpy as np
import torch
from torch import nn
from torch.nn import functional as F

from .. import kernels as K
from ..modules.cnn import AgxConv2d, Conv2dGroupedFn, _FusedIdentity
from ..modules.custom_components import NoisyLinear
from ..modules.mlp import EvolvableMLP
from ..modules.cnn import EvolvableCNN
from ..population.image_nets import BatchedLinearFn


class _Rows:
    """A ``[P, n]`` buffer and the per-tensor offsets of one module tree."""

    def __init__(self, P: int, shapes: list[tuple[str, torch.Size]], device):
        self.offsets: dict[str, tuple[int, torch.Size]] = {}
        off = 0
        for name, shape in shapes:
            self.offsets[name] = (off, shape)
            off += int(np.prod(shape)) if len(shape) else 1
        self.n = off
        self.data = torch.zeros(P, max(off, 1), dtype=torch.float32, device=device)

    def view(self, name: str, buf: torch.Tensor | None = None) -> torch.Tensor:
        off, shape = self.offsets[name]
        b = self.data if buf is None else buf
        k = int(np.prod(shape)) if len(shape) else 1
        return b[:, off:off + k].view(b.shape[0], *shape)

    def row_view(self, p: int, name: str, buf: torch.Tensor | None = None) -> torch.Tensor:
        off, shape = self.offsets[name]
        b = self.data if buf is None else buf
        k = int(np.prod(shape)) if len(shape) else 1
        return b[p, off:off + k].view(shape)


def _backward(loss: torch.Tensor) -> None:
    """loss.backward() with autograd's gradient-layout notice silenced: the
    stacked leaves are strided row views whose preset .grad is a strided view
    of the flat gradient rows by design (AccumulateGrad adds into it in place,
    no copy).  Scoped to this call, so the notice stays on for other modules."""
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", message="grad and param do not obey the gradient layout contract")
        loss.backward()


def _module_ops(net: nn.Module) -> list[tuple[str, nn.Module]]:
    """(qualified name prefix, leaf module) in execution order of a
    RainbowQNetwork's encoder (EvolvableCNN / EvolvableMLP)."""
    enc = net.encoder
    if not isinstance(enc, (EvolvableCNN, EvolvableMLP)):
        raise NotImplementedError("population Rainbow learner: CNN or MLP encoders")
    return [(f"encoder.model.{k}", m) for k, m in enc.model.named_children()]


class RainbowPopulationLearner:
    """Batched learner over ``agents`` (RainbowDQN or DQN objects of one
    architecture).

    Construction moves every agent's online / target parameters, noise
    buffers and Adam state into rows of flat device buffers and leaves the
    agents' tensors as views of those rows.  ``learn(experiences)`` takes one
    experience dict per agent (the reference's ``agent.learn`` argument) and
    returns one ``(loss, idxs, new_priorities)`` tuple per agent."""

    def __init__(self, agents: list):
        if not agents:
            raise ValueError("no agents")
        a0 = agents[0]
        keys = [(k, v.shape) for k, v in a0.actor.state_dict().items()]
        for a in agents[1:]:
            if [(k, v.shape) for k, v in a.actor.state_dict().items()] != keys:
                raise ValueError("population learner: every agent needs the same network shapes")
        if a0.device.type != "cuda":
            raise NotImplementedError("population learner runs on the GPU")
        self.agents = list(agents)
        self.rainbow = hasattr(a0, "num_atoms")
        if any(hasattr(a, "num_atoms") != self.rainbow for a in agents):
            raise ValueError("population learner: one algorithm per population")
        self.P = P = len(agents)
        self.device = a0.device
        pnames = [(k, p.shape) for k, p in a0.actor.named_parameters()]
        bnames = [(k, b.shape) for k, b in a0.actor.named_buffers() if k.endswith("_epsilon")]
        self.pnames = [k for k, _ in pnames]
        self.prm = _Rows(P, pnames, self.device)
        self.tgt = _Rows(P, pnames, self.device)
        self.noise = _Rows(P, bnames, self.device)
        self.tnoise = _Rows(P, bnames, self.device)
        self.grad = torch.zeros_like(self.prm.data)
        self.m = torch.zeros_like(self.prm.data)
        self.v = torch.zeros_like(self.prm.data)
        self.steps = torch.zeros(P, dtype=torch.int64, device=self.device)
        n = self.prm.n
        with torch.no_grad():
            for p, a in enumerate(agents):
                self._adopt(p, a)
        self.workspace = torch.empty(max(16, K._lib.load().agx_adam_workspace_bytes(P, n)), dtype=torch.uint8,
                                     device=self.device)
        self.offsets = torch.tensor([0, n], dtype=torch.int64)
        # stacked leaf views ([P, *shape]) of the online parameters, their
        # gradients accumulating in place into the flat gradient rows (the
        # layout-contract notice this raises is silenced around backward only,
        # _backward)
        self.leaf: dict[str, torch.Tensor] = {}
        for k in self.pnames:
            t = self.prm.view(k).detach().requires_grad_(True)
            t.grad = self.prm.view(k, self.grad)
            self.leaf[k] = t
        self._enc_ops = _module_ops(a0.actor)
        self.image_norm = None
        if isinstance(a0.actor.encoder, EvolvableCNN):
            first = next(m for _, m in self._enc_ops if isinstance(m, AgxConv2d))
            self.image_norm = first.image_norm

    # ------------------------------------------------------------------ #
    def _adopt(self, p: int, a) -> None:
        """Agent p's tensors -> row p; its tensors become views of the row."""
        for net, rows, nrows in ((a.actor, self.prm, self.noise), (a.actor_target, self.tgt, self.tnoise)):
            for k, prm in net.named_parameters():
                v = rows.row_view(p, k)
                v.copy_(prm.data)
                prm.data = v
            for k, buf in net.named_buffers():
                if k in nrows.offsets:
                    v = nrows.row_view(p, k)
                    v.copy_(buf)
                    mod, _, attr = k.rpartition(".")
                    owner = net.get_submodule(mod) if mod else net
                    owner._buffers[attr] = v
        opt = a.optimizer
        step = 0
        for k, prm in a.actor.named_parameters():
            st = opt.state.get(prm)
            if st and "exp_avg" in st:
                self.m[p].narrow(0, self.prm.offsets[k][0], prm.numel()).copy_(st["exp_avg"].reshape(-1))
                self.v[p].narrow(0, self.prm.offsets[k][0], prm.numel()).copy_(st["exp_avg_sq"].reshape(-1))
                step = int(st["step"])
            opt.state[prm] = {"step": torch.tensor(float(step)),
                              "exp_avg": self.prm.row_view(p, k, self.m),
                              "exp_avg_sq": self.prm.row_view(p, k, self.v)}
        self.steps[p] = step
        # the agent's own flat learner state (flat_state.py) stands aside while its
        # tensors are rows here
        a.__dict__["_pop_rows"] = (weakref.ref(self), tuple(q.data_ptr() for q in a.actor.parameters()))

    def sync_optimizers(self) -> None:
        """Write the device step counts into the agents' torch Adam states
        (their moments are already views of the flat rows)."""
        steps = self.steps.cpu().tolist()
        for a, s in zip(self.agents, steps):
            for prm in a.actor.parameters():
                a.optimizer.state[prm]["step"] = torch.tensor(float(s))

    # ------------------------------------------------------------------ #
    def _linear(self, x, name, noisy: bool, params: dict | None, rows: _Rows, noise: _Rows):
        def P_(k):
            return params[k] if params is not None else rows.view(k)

        if noisy:
            w = P_(f"{name}.weight_mu") + P_(f"{name}.weight_sigma") * noise.view(f"{name}.weight_epsilon")
            b = P_(f"{name}.bias_mu") + P_(f"{name}.bias_sigma") * noise.view(f"{name}.bias_epsilon")
        else:
            w, b = P_(f"{name}.weight"), P_(f"{name}.bias")
        return BatchedLinearFn.apply(x, w, b)

    def _seq(self, x, ops, params, rows, noise):
        for name, mod in ops:
            if isinstance(mod, AgxConv2d):
                x = Conv2dGroupedFn.apply(x, params[f"{name}.weight"] if params is not None else rows.view(
                    f"{name}.weight"), params[f"{name}.bias"] if params is not None else rows.view(f"{name}.bias"),
                    int(mod.stride[0]), mod.fuse_relu, mod.image_norm if x.dtype == torch.uint8 else None)
            elif isinstance(mod, _FusedIdentity):
                pass
            elif isinstance(mod, nn.Flatten):
                x = x.reshape(x.shape[0], x.shape[1], -1)
            elif isinstance(mod, NoisyLinear):
                x = self._linear(x, name, mod.training, params, rows, noise)
            elif isinstance(mod, nn.Linear):
                x = self._linear(x, name, False, params, rows, noise)
            elif isinstance(mod, nn.LayerNorm):
                x = F.layer_norm(x, mod.normalized_shape, None, None, mod.eps)
                if mod.elementwise_affine:
                    g = params[f"{name}.weight"] if params is not None else rows.view(f"{name}.weight")
                    bb = params[f"{name}.bias"] if params is not None else rows.view(f"{name}.bias")
                    x = x * g.unsqueeze(1) + bb.unsqueeze(1)
            else:  # stateless activation
                x = mod(x)
        return x

    def _head_streams(self, net, x, params, rows, noise):
        """RainbowQNetwork over [P, B, ...] -> value [P*B, Z], advantage [P*B, A*Z]."""
        P, B = x.shape[0], x.shape[1]
        if self._flatten_obs(net):
            x = x.reshape(P, B, -1)
        lat = self._seq(x, _module_ops(net), params, rows, noise)
        head = net.head_net
        v = self._seq(lat, [(f"head_net.model.{k}", m) for k, m in head.model.named_children()], params, rows, noise)
        if not self.rainbow:  # QNetwork: the "value" head is Q [P, B, A]
            return v
        a = self._seq(lat, [(f"head_net.advantage_net.{k}", m) for k, m in head.advantage_net.named_children()],
                      params, rows, noise)
        return v.reshape(P * B, -1), a.reshape(P * B, -1)

    @staticmethod
    def _flatten_obs(net) -> bool:
        return bool(getattr(net, "flatten_obs", False))

    # ------------------------------------------------------------------ #
    def _td_losses(self, obs, acts, rew, done, next_obs, gamma):
        """DQN: per-agent TD target + MSE (dqn.py:274-324) -> loss [P]."""
        from .dqn import _TDLoss

        a0 = self.agents[0]
        with torch.no_grad():
            q_next_t = self._head_streams(a0.actor_target, next_obs, None, self.tgt, self.tnoise)
            q_next_o = self._head_streams(a0.actor, next_obs, None, self.prm, self.noise) if a0.double else None
        q_cur = self._head_streams(a0.actor, obs, self.leaf, self.prm, self.noise)
        return torch.stack([_TDLoss.apply(q_cur[p], q_next_t[p].contiguous(),
                                          q_next_o[p].contiguous() if q_next_o is not None else None,
                                          acts[p].contiguous(), rew[p].contiguous(), done[p].contiguous(),
                                          float(gamma), bool(a0.double)) for p in range(self.P)])

    def _loss(self, obs, acts, rew, done, next_obs, gamma):
        """Elementwise C51 loss [P, B] of every agent (dqn_rainbow.py:313-367)."""
        from ..networks.q_networks import DuelingHeadFn, DuelingRowsFn

        a0 = self.agents[0]
        P, B = obs.shape[0], obs.shape[1]
        A, Z = a0.action_dim, a0.num_atoms
        with torch.no_grad():
            v, adv = self._head_streams(a0.actor, next_obs, None, self.prm, self.noise)
            q = DuelingHeadFn.apply(v, adv, a0.support, A, Z, 0)          # [P*B, A]
            a_star = q.argmax(1)                                            # first maximum
            v, adv = self._head_streams(a0.actor_target, next_obs, None, self.tgt, self.tnoise)
            target_rows = DuelingRowsFn.apply(v, adv, a_star, A, Z, 1)     # [P*B, Z]
        v, adv = self._head_streams(a0.actor, obs, self.leaf, self.prm, self.noise)
        logp_rows = DuelingRowsFn.apply(v, adv, acts.reshape(-1), A, Z, 2)
        from .dqn import _C51RowsLoss

        el = _C51RowsLoss.apply(logp_rows, target_rows, rew.reshape(-1), done.reshape(-1), a0.support,
                                float(a0.v_min), float(a0.v_max), float(gamma))
        return el.view(P, B)

    def _stack(self, exps, key, obs=False):
        a0 = self.agents[0]
        xs = []
        for e in exps:
            x = e[key]
            if obs:
                xs.append(a0._obs(x))
            else:
                t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
                xs.append(t.to(self.device))
        return torch.stack(xs)

    def _adam(self, max_norm: float) -> None:
        """One agx_clip_adam launch over [P, n]: per-agent norm clip (max_norm
        <= 0: none), per-agent lr and step count."""
        lr = torch.tensor([float(a.lr) for a in self.agents], dtype=torch.float32).to(self.device)
        K._lib.call("agx_clip_adam", self.prm.data.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(),
                    self.v.data_ptr(), self.P, self.prm.n, self.offsets.data_ptr(), 1, float(max_norm),
                    lr.data_ptr(), 0.9, 0.999, 1e-8, self.steps.data_ptr(), None, self.workspace.data_ptr(),
                    K._lib.stream())

    def _learn_dqn(self, experiences: list) -> list:
        """DQN.learn per agent (dqn.py:326-348): TD loss, Adam (no clipping),
        Polyak -> [loss] per agent."""
        a0 = self.agents[0]
        for a in self.agents[1:]:
            for attr in ("gamma", "tau", "double"):
                if getattr(a, attr) != getattr(a0, attr):
                    raise NotImplementedError(f"population learner: agents differ in {attr}")
        obs, next_obs = self._stack(experiences, "obs", True), self._stack(experiences, "next_obs", True)
        acts = self._stack(experiences, "action").reshape(self.P, -1).long()
        rew = self._stack(experiences, "reward").reshape(self.P, -1).float()
        done = self._stack(experiences, "done").reshape(self.P, -1).float()
        self.grad.zero_()
        loss = self._td_losses(obs, acts, rew, done, next_obs, a0.gamma)
        _backward(loss.sum())
        self._adam(0.0)
        K.polyak_(self.tgt.data.view(-1), self.prm.data.view(-1), float(a0.tau))
        return [float(x) for x in loss.detach().cpu().tolist()]

    def learn(self, experiences: list, n_experiences: list | None = None, per: bool = False) -> list:
        """-> [(loss, idxs, new_priorities)] per agent, as ``agent.learn``."""
        a0 = self.agents[0]
        if len(experiences) != self.P:
            raise ValueError(f"need one experience batch per agent ({self.P})")
        if not self.rainbow:
            return self._learn_dqn(experiences)
        for a in self.agents[1:]:
            for attr in ("gamma", "tau", "n_step", "combined_reward", "v_min", "v_max", "num_atoms", "prior_eps"):
                if getattr(a, attr) != getattr(a0, attr):
                    raise NotImplementedError(f"population learner: agents differ in {attr}")
        n_step = n_experiences is not None

        def batch(exps):
            return (self._stack(exps, "obs", True), self._stack(exps, "action").reshape(self.P, -1).long(),
                    self._stack(exps, "reward").reshape(self.P, -1).float(), self._stack(exps, "done").reshape(
                        self.P, -1).float(), self._stack(exps, "next_obs", True))

        self.grad.zero_()
        el = None
        if a0.combined_reward or not n_step:
            el = self._loss(*batch(experiences), a0.gamma)
        if n_step:
            nl = self._loss(*batch(n_experiences), a0.gamma ** a0.n_step)
            el = el + nl if a0.combined_reward else nl
        if per:
            w = self._stack(experiences, "weights").float()
            if w.dim() == 3:  # (B, 1) weights: the reference's (B,) * (B, 1) broadcast, a mean over (B, B)
                loss = (el.unsqueeze(1) * w).mean((1, 2))
            else:
                loss = (el * w.reshape(self.P, -1)).mean(1)
        else:
            loss = el.mean(1)
        _backward(loss.sum())
        self._adam(10.0)
        K.polyak_(self.tgt.data.view(-1), self.prm.data.view(-1), float(a0.tau))
        for a in self.agents:  # the reference's per-agent noise draws, in agent order
            a.actor.reset_noise()
            a.actor_target.reset_noise()
        losses = loss.detach().cpu().tolist()
        el_h = el.detach().cpu().numpy() if per else None
        out = []
        for p, a in enumerate(self.agents):
            idxs = experiences[p]["idxs"] if (per or n_step) else None
            pri = el_h[p] + a.prior_eps if per else None
            out.append((losses[p], idxs, pri))
        return out
