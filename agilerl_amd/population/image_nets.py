"""Population-stacked CNN actor-critics over ONE flat parameter buffer [P, n]
— the image-observation counterpart of ``nets.ActorCriticSpec`` (Atari PPO,
BASELINE config 5).

Architecture (what the reference's PPO builds for an image Box space with a
shared encoder, algorithms/ppo.py:286-320 -> networks/base.py:521-530):

  encoder : EvolvableCNN (modules/cnn.py:224-552): per layer Conv2d(k, stride)
            -> ReLU, flatten, Linear(-> latent) -> output activation (ReLU:
            base.py:226-230 takes the encoder's activation when none is set)
  actor   : MLP head on the latent (create_mlp, evolvable_networks.py:527-644):
            [Linear (-> LayerNorm) -> ReLU] per hidden size, Linear(-> A) x0.1
  critic  : the same head shape on the same latent, Linear(-> 1) x0.1

Parameters of agent p are row p of ``flat[P, n]`` in state-dict order
[conv layers | linear_output | actor head | critic head]; the two clip groups
of ppo.py:910-911 are [0, actor_end) (shared encoder + actor head) and
[actor_end, n) (critic head), as for the MLP spec.

Forward: the convolutions run on the HIP implicit-GEMM kernels
(modules/cnn.py ``Conv2dGroupedFn``: f32 MFMA, ReLU fused in the epilogue; uint8
frames are normalised to (x - low) / (high - low) inside the first layer's
load, so the uint8 rollout SoA is read as is).  Every layer is ONE
population-batched launch (agx_conv2d_*_grouped: each agent its own
filters, read in place from its row of the flat buffer); the linear_output
layer and the heads are batched over the population too (one bmm each).  The
flat buffer is split into per-parameter chunks once per forward (``split``:
its backward is one cat, not a full-size scatter per view).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from ..modules.cnn import Conv2dGroupedFn
from .nets import ActorCriticSpec, Layer


class BatchedLinearFn(torch.autograd.Function):
    """y [P, B, out] = x [P, B, in] @ W[p]^T + b[p] for every agent p (the
    population's Linear layers, one batched GEMM), with the backward's weight
    gradient formed directly in W's own [P, out, in] layout (dy^T x): autograd
    of ``baddbmm(b, x, W.transpose(1, 2))`` builds it as the transpose of
    x^T dy and copies it back into the parameter chunk's layout."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        return torch.baddbmm(b.unsqueeze(1), x, W.transpose(1, 2))

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dx = torch.bmm(dy, W) if ctx.needs_input_grad[0] else None
        dW = torch.bmm(dy.transpose(1, 2), x) if ctx.needs_input_grad[1] else None
        db = dy.sum(1) if ctx.needs_input_grad[2] else None
        return dx, dW, db


@dataclass
class ImageActorCriticSpec:
    obs_shape: tuple[int, int, int]
    n_actions: int
    channel_size: list[int] = field(default_factory=lambda: [32, 64, 64])
    kernel_size: list[int] = field(default_factory=lambda: [8, 4, 3])
    stride_size: list[int] = field(default_factory=lambda: [4, 2, 1])
    latent_dim: int = 256
    actor_hidden: list[int] = field(default_factory=lambda: [256])
    critic_hidden: list[int] = field(default_factory=lambda: [256])
    head_layer_norm: bool = False
    encoder_name: str = "shared_encoder"
    obs_dtype: torch.dtype = torch.uint8
    image_norm: tuple[float, float] | None = (0.0, 255.0)
    # architecture-mutation limits (population/image_arch.py): the CNN's
    # (min / max hidden layers, min / max channels; CnnNetConfig's defaults
    # 1, 6, 16, 256), the heads' (min / max hidden layers, min / max nodes)
    # and the latent's (min, max) (EvolvableNetwork: 8, 128)
    cnn_limits: tuple = (1, 6, 16, 256)
    actor_limits: tuple = (1, 3, 16, 500)
    critic_limits: tuple = (1, 3, 16, 500)
    latent_limits: tuple = (8, 128)

    def __post_init__(self) -> None:
        if not (len(self.channel_size) == len(self.kernel_size) == len(self.stride_size)):
            raise ValueError("channel_size, kernel_size and stride_size must have the same length")
        self.obs_shape = tuple(int(x) for x in self.obs_shape)
        self.kernel_size = [int(k[0] if isinstance(k, (tuple, list)) else k) for k in self.kernel_size]
        self.obs_dim = int(math.prod(self.obs_shape))
        c, h, w = self.obs_shape
        self.convs = []  # (name, cin, cout, k, stride, w_off, b_off)
        off = 0
        for i, (co, k, s) in enumerate(zip(self.channel_size, self.kernel_size, self.stride_size), 1):
            name = f"{self.encoder_name}_conv_layer_{i}"
            self.convs.append((name, c, int(co), k, int(s), off, off + int(co) * c * k * k))
            off += int(co) * c * k * k + int(co)
            h, w, c = (h - k) // s + 1, (w - k) // s + 1, int(co)
            if h < 1 or w < 1:
                raise ValueError(f"input {self.obs_shape} is too small for the conv stack")
        self.feat_dim = c * h * w
        self.conv_out = (c, h, w)
        self.lin_out = Layer(f"{self.encoder_name}_linear_output", self.feat_dim, self.latent_dim, None, True)
        self.lin_out.w, self.lin_out.b = off, off + self.feat_dim * self.latent_dim
        off += self.feat_dim * self.latent_dim + self.latent_dim
        ln = "affine" if self.head_layer_norm else None
        self.actor = ActorCriticSpec._head(self, "actor", self.actor_hidden, self.n_actions, ln)
        self.critic = ActorCriticSpec._head(self, "value", self.critic_hidden, 1, ln)
        for lay in self.actor + self.critic:
            lay.w = off
            off += lay.fin * lay.fout
            lay.b = off
            off += lay.fout
            if lay.ln == "affine":
                lay.g = off
                off += lay.fout
                lay.beta = off
                off += lay.fout
            if lay is self.actor[-1]:
                self.actor_end = off
        self.n_params = off
        self.group_offsets = [0, self.actor_end, self.n_params]
        # contiguous parameter chunks in row order: (offset, size, shape)
        chunks = []
        for name, ci, co, k, s, wo, bo in self.convs:
            chunks += [(wo, co * ci * k * k, (co, ci, k, k)), (bo, co, (co,))]
        chunks += [(self.lin_out.w, self.feat_dim * self.latent_dim, (self.latent_dim, self.feat_dim)),
                   (self.lin_out.b, self.latent_dim, (self.latent_dim,))]
        for lay in self.actor + self.critic:
            chunks += [(lay.w, lay.fin * lay.fout, (lay.fout, lay.fin)), (lay.b, lay.fout, (lay.fout,))]
            if lay.ln == "affine":
                chunks += [(lay.g, lay.fout, (lay.fout,)), (lay.beta, lay.fout, (lay.fout,))]
        assert [c[0] for c in chunks] == sorted(c[0] for c in chunks)
        self._chunks = chunks
        self._index = {c[0]: i for i, c in enumerate(chunks)}

    def shape_key(self) -> tuple:
        """Agents with equal keys share a network layout (population groups)."""
        return (self.obs_shape, self.n_actions, tuple(self.channel_size), tuple(self.kernel_size),
                tuple(self.stride_size), self.latent_dim, tuple(self.actor_hidden), tuple(self.critic_hidden),
                self.head_layer_norm, self.encoder_name, self.obs_dtype, self.image_norm, tuple(self.cnn_limits),
                tuple(self.actor_limits), tuple(self.critic_limits), tuple(self.latent_limits))

    # ------------------------------------------------------------------ #
    def init_params(self, P: int, seeds: list[int] | None = None, device="cpu") -> torch.Tensor:
        """Per agent, in module order: conv layers orthogonal (gain sqrt 2),
        zero bias (layer_init, evolvable_networks.py:410-441); linear_output
        torch's default nn.Linear init (cnn.py:536-540); head layers
        orthogonal sqrt 2 with the output layer x0.1 (output_vanish)."""
        flat = torch.zeros(P, self.n_params, dtype=torch.float32)
        for p in range(P):
            gen = torch.Generator().manual_seed(int(seeds[p]) if seeds is not None else p)
            for _name, ci, co, k, _s, wo, _bo in self.convs:
                w = torch.empty(co, ci, k, k)
                torch.nn.init.orthogonal_(w, math.sqrt(2), generator=gen)
                flat[p, wo:wo + w.numel()] = w.reshape(-1)
            lo = self.lin_out
            w = torch.empty(lo.fout, lo.fin)
            torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=gen)
            bound = 1.0 / math.sqrt(lo.fin)
            b = torch.empty(lo.fout).uniform_(-bound, bound, generator=gen)
            flat[p, lo.w:lo.w + w.numel()] = w.reshape(-1)
            flat[p, lo.b:lo.b + lo.fout] = b
            for lay in self.actor + self.critic:
                w = torch.empty(lay.fout, lay.fin)
                torch.nn.init.orthogonal_(w, math.sqrt(2), generator=gen)
                if lay.vanish:
                    w.mul_(0.1)
                flat[p, lay.w:lay.w + w.numel()] = w.reshape(-1)
                if lay.ln == "affine":
                    flat[p, lay.g:lay.g + lay.fout] = 1.0
        return flat.to(device)

    # ------------------------------------------------------------------ #
    def _split(self, flat: torch.Tensor) -> list[torch.Tensor]:
        return list(flat.split([c[1] for c in self._chunks], dim=1))

    def _chunk(self, parts, off: int, P: int) -> torch.Tensor:
        i = self._index[off]
        return parts[i].view(P, *self._chunks[i][2])

    def _head(self, parts, x: torch.Tensor, layers: list[Layer]) -> torch.Tensor:
        P = x.shape[0]
        for lay in layers:
            W, b = self._chunk(parts, lay.w, P), self._chunk(parts, lay.b, P)
            x = BatchedLinearFn.apply(x, W, b)
            if lay.ln is not None:
                x = F.layer_norm(x, (lay.fout,), eps=1e-5)
                if lay.ln == "affine":
                    x = x * self._chunk(parts, lay.g, P).unsqueeze(1) + self._chunk(parts, lay.beta, P).unsqueeze(1)
            if lay.act:
                x = torch.relu(x)
        return x

    def features(self, flat: torch.Tensor, obs: torch.Tensor, parts=None, rows=None) -> torch.Tensor:
        """Conv stack of every agent -> flattened features [P, B, feat_dim]:
        one population-batched launch per layer and direction
        (agx_conv2d_*_grouped, each agent its own filters).  ``rows`` (the
        agents a heterogeneous learner group updates) does not narrow it: the
        other agents' outputs are computed and left unused."""
        P, B = obs.shape[0], obs.shape[1]
        parts = self._split(flat) if parts is None else parts
        x = obs.reshape(P, B, *self.obs_shape)
        u8 = x.dtype == torch.uint8
        if u8 and self.image_norm is None:
            x = x.float()
            u8 = False
        elif not u8:
            x = x.float()
            if self.image_norm is not None:  # preprocess_observation (algo_utils.py:1134-1183)
                lo, hi = self.image_norm
                x = (x - lo) / (hi - lo)
        h = x
        for j, (_name, ci, co, k, s, wo, bo) in enumerate(self.convs):
            w = parts[self._index[wo]].view(P, co, ci, k, k)
            b = parts[self._index[bo]]
            h = Conv2dGroupedFn.apply(h, w, b, s, True, self.image_norm if (j == 0 and u8) else None)
        return h.reshape(P, B, self.feat_dim)

    def forward(self, flat: torch.Tensor, obs: torch.Tensor, rows=None):
        """obs [P, B, obs_dim] (uint8 frames or f32) -> (logits [P, B, A], value [P, B])."""
        P = obs.shape[0]
        parts = self._split(flat)
        feat = self.features(flat, obs, parts, rows)
        lo = self.lin_out
        lat = torch.relu(BatchedLinearFn.apply(feat, self._chunk(parts, lo.w, P), self._chunk(parts, lo.b, P)))
        logits = self._head(parts, lat, self.actor)
        value = self._head(parts, lat, self.critic).squeeze(-1)
        return logits, value

    def state_dict_keys(self) -> dict[str, tuple[int, tuple[int, ...]]]:
        """Reference-compatible parameter names -> (offset, shape)."""
        out = {}
        for net in ("actor.encoder.model", "critic.encoder.model"):
            for name, ci, co, k, _s, wo, bo in self.convs:
                out[f"{net}.{name}.weight"] = (wo, (co, ci, k, k))
                out[f"{net}.{name}.bias"] = (bo, (co,))
            out[f"{net}.{self.lin_out.name}.weight"] = (self.lin_out.w, (self.latent_dim, self.feat_dim))
            out[f"{net}.{self.lin_out.name}.bias"] = (self.lin_out.b, (self.latent_dim,))
        for net, layers in (("actor.head_net._wrapped.model", self.actor), ("critic.head_net.model", self.critic)):
            for lay in layers:
                out[f"{net}.{lay.name}.weight"] = (lay.w, (lay.fout, lay.fin))
                out[f"{net}.{lay.name}.bias"] = (lay.b, (lay.fout,))
                if lay.ln == "affine":
                    ln_name = lay.name.replace("linear_layer", "layer_norm")
                    out[f"{net}.{ln_name}.weight"] = (lay.g, (lay.fout,))
                    out[f"{net}.{ln_name}.bias"] = (lay.beta, (lay.fout,))
        return out
