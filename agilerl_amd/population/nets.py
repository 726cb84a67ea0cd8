"""Population-stacked actor-critic MLPs over ONE flat parameter buffer [P, n].

Architecture (what the reference builds for PPO with a shared MLP encoder,
agilerl/utils/evolvable_networks.py:527-644 ``create_mlp`` via
agilerl/networks/base.py:541-561, ``StochasticActor`` / ``ValueNetwork``):

  encoder : [Linear -> LayerNorm(affine) -> act] per hidden size,
            Linear(-> latent) -> LayerNorm(no affine) -> act    (output_layernorm, output_vanish off)
  actor   : [Linear -> LayerNorm(affine) -> act] per hidden size, Linear(-> A)  (x0.1 init)
  critic  : same on the actor's latent (share_encoders, ppo.py:487-491), Linear(-> 1)

Every agent's parameters are one contiguous row of ``flat[P, n]`` laid out
[encoder | actor head | critic head] in state-dict order (weight, bias,
LN weight, LN bias per layer), so one kernel launch updates the whole
population and the two clip groups of ppo.py:910-911 are the contiguous
ranges [0, enc+actor) and [enc+actor, n).  Weights use the nn.Linear [out, in]
layout.  Initialisation: orthogonal (gain sqrt 2), zero bias, output layers
x0.1 (``layer_init`` / ``output_vanish``, evolvable_networks.py:410-441, 621-629).

``forward`` is the plain-PyTorch fp32 path (batched over the population with
bmm); it is the numerics reference for the fused HIP learner and the path
for architectures the fused kernel does not cover.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F


@dataclass
class Layer:
    name: str
    fin: int
    fout: int
    ln: str | None  # None | "affine" | "plain"
    act: bool
    w: int = 0
    b: int = 0
    g: int = -1
    beta: int = -1
    vanish: bool = False


@dataclass
class ActorCriticSpec:
    obs_dim: int
    n_actions: int
    encoder_hidden: list[int] = field(default_factory=lambda: [64])
    latent_dim: int = 64
    actor_hidden: list[int] = field(default_factory=lambda: [64])
    critic_hidden: list[int] = field(default_factory=lambda: [64])
    layer_norm: bool = True
    # ppo.py:308: the actor's encoder is named "shared_encoder" when the critic
    # shares it (the reference default), so its layers are
    # shared_encoder_linear_layer_1, ... in the state dict
    encoder_name: str = "shared_encoder"
    # architecture-mutation limits (population/arch.py): per MLP (min / max
    # hidden layers, min / max nodes; EvolvableMLP's defaults 1, 3, 32, 500, or
    # MlpNetConfig's 1, 3, 16, 500) and the latent's (min, max)
    # (EvolvableNetwork: 8, 128)
    encoder_limits: tuple = (1, 3, 32, 500)
    actor_limits: tuple = (1, 3, 32, 500)
    critic_limits: tuple = (1, 3, 32, 500)
    latent_limits: tuple = (8, 128)
    # share_encoders=False (ppo.py:292-320): the critic has its own encoder
    # ("critic_encoder", the actor's is then "actor_encoder"), laid out after
    # the actor head in the reference's state-dict order
    share_encoders: bool = True
    critic_encoder_name: str = "critic_encoder"

    def shape_key(self) -> tuple:
        """Agents with equal keys share a network layout (population groups)."""
        return (self.obs_dim, self.n_actions, tuple(self.encoder_hidden), self.latent_dim, tuple(self.actor_hidden),
                tuple(self.critic_hidden), self.layer_norm, self.encoder_name, tuple(self.encoder_limits),
                tuple(self.actor_limits), tuple(self.critic_limits), tuple(self.latent_limits), self.share_encoders,
                self.critic_encoder_name)

    def __post_init__(self) -> None:
        ln = "affine" if self.layer_norm else None
        enc = [self.obs_dim, *self.encoder_hidden]
        def encoder(e):
            layers = [Layer(f"{e}_linear_layer_{i}", enc[i - 1], enc[i], ln, True) for i in range(1, len(enc))]
            layers.append(Layer(f"{e}_linear_layer_output", enc[-1], self.latent_dim,
                                "plain" if self.layer_norm else None, True))
            return layers

        self.encoder = encoder(self.encoder_name)
        self.critic_encoder = [] if self.share_encoders else encoder(self.critic_encoder_name)
        self.actor = self._head("actor", self.actor_hidden, self.n_actions, ln)
        self.critic = self._head("value", self.critic_hidden, 1, ln)  # ValueNetwork head name (value_networks.py:96)
        off = 0
        for lay in self.encoder + self.actor + self.critic_encoder + self.critic:
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

    def _head(self, name, hidden, nout, ln):
        dims = [self.latent_dim, *hidden]
        layers = [Layer(f"{name}_linear_layer_{i}", dims[i - 1], dims[i], ln, True)
                  for i in range(1, len(dims))]
        layers.append(Layer(f"{name}_linear_layer_output", dims[-1], nout, None, False, vanish=True))
        return layers

    @property
    def layers(self) -> list[Layer]:
        return self.encoder + self.actor + self.critic_encoder + self.critic

    def aliased(self, key: str) -> bool:
        """A state-dict key whose tensor is another key's (the shared
        encoder's critic copy)."""
        return self.share_encoders and key.startswith("critic.encoder.")

    # ------------------------------------------------------------------ #
    def init_params(self, P: int, seeds: list[int] | None = None, device="cpu") -> torch.Tensor:
        flat = torch.zeros(P, self.n_params, dtype=torch.float32)
        for p in range(P):
            gen = torch.Generator().manual_seed(int(seeds[p]) if seeds is not None else p)
            for lay in self.layers:
                w = torch.empty(lay.fout, lay.fin)
                torch.nn.init.orthogonal_(w, math.sqrt(2), generator=gen)
                if lay.vanish:
                    w.mul_(0.1)
                flat[p, lay.w: lay.w + w.numel()] = w.reshape(-1)
                if lay.ln == "affine":
                    flat[p, lay.g: lay.g + lay.fout] = 1.0
        return flat.to(device)

    def views(self, flat: torch.Tensor, lay: Layer):
        P = flat.shape[0]
        W = flat[:, lay.w: lay.w + lay.fin * lay.fout].view(P, lay.fout, lay.fin)
        b = flat[:, lay.b: lay.b + lay.fout]
        g = flat[:, lay.g: lay.g + lay.fout] if lay.ln == "affine" else None
        be = flat[:, lay.beta: lay.beta + lay.fout] if lay.ln == "affine" else None
        return W, b, g, be

    def _run(self, flat, x, layers):
        """Agent by agent: 2-D GEMMs whose kernel choice (and so rounding)
        depends only on the agent's own shapes, never on how many agents the
        population holds — a population split into groups or sharded over
        ranks computes exactly what the whole one does."""
        outs = []
        for p in range(flat.shape[0]):
            h = x[p]
            for lay in layers:
                W, b, g, be = self.views(flat[p:p + 1], lay)
                h = torch.addmm(b[0], h, W[0].t())
                if lay.ln is not None:
                    h = F.layer_norm(h, (lay.fout,), eps=1e-5)
                    if g is not None:
                        h = h * g[0] + be[0]
                if lay.act:
                    h = torch.relu(h)
            outs.append(h)
        return torch.stack(outs)

    def forward(self, flat: torch.Tensor, obs: torch.Tensor):
        """obs [P, B, obs_dim] -> (logits [P, B, A], value [P, B])."""
        lat = self._run(flat, obs, self.encoder)
        logits = self._run(flat, lat, self.actor)
        lat_c = lat if self.share_encoders else self._run(flat, obs, self.critic_encoder)
        value = self._run(flat, lat_c, self.critic).squeeze(-1)
        return logits, value

    def state_dict_keys(self) -> dict[str, tuple[int, tuple[int, ...]]]:
        """Reference-compatible parameter names -> (offset, shape)."""
        out = {}
        # critic.encoder is the reference's detached copy of the shared actor encoder
        # (share_encoders, algo_utils.py:164-187): same offsets as actor.encoder
        # the actor's head is an EvolvableDistribution wrapping the MLP
        # (networks/actors.py:330-336, modules/base.py:740-760): its
        # parameters sit under head_net._wrapped in the reference's state dict
        for net, layers in (("actor.encoder.model", self.encoder), ("actor.head_net._wrapped.model", self.actor),
                            ("critic.encoder.model", self.encoder if self.share_encoders else self.critic_encoder),
                            ("critic.head_net.model", self.critic)):
            for lay in layers:
                out[f"{net}.{lay.name}.weight"] = (lay.w, (lay.fout, lay.fin))
                out[f"{net}.{lay.name}.bias"] = (lay.b, (lay.fout,))
                if lay.ln == "affine":
                    ln_name = lay.name.replace("linear_layer", "layer_norm")
                    out[f"{net}.{ln_name}.weight"] = (lay.g, (lay.fout,))
                    out[f"{net}.{ln_name}.bias"] = (lay.beta, (lay.fout,))
        return out


def categorical(logits: torch.Tensor):
    """log-softmax and entropy as ``agilerl/utils/torch_utils.py:142-199``:
    H = -sum p * log(p + 1e-8)."""
    logp_all = torch.log_softmax(logits, dim=-1)
    p = torch.softmax(logits, dim=-1)
    ent = -(p * torch.log(p + 1e-8)).sum(-1)
    return logp_all, ent
