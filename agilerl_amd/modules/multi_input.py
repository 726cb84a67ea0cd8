"""``EvolvableMultiInput`` (agilerl/modules/multi_input.py:22-535) for Dict
observation spaces of vector (1-D Box) subspaces — the shared MADDPG critic's
input: the vector observations are concatenated in the space's key order and
mapped by ``final_dense`` (nn.Linear, default init) -> optional non-affine
``final_layernorm`` -> output activation.  CNN / nested / vector-MLP feature
extractors are outside the hot path (NotImplementedError)."""

from __future__ import annotations

import numpy as np
import torch
from torch import nn

from .mlp import get_activation


class EvolvableMultiInput(nn.Module):
    def __init__(self, observation_space, num_outputs: int, latent_dim: int | None = None,
                 vector_space_mlp: bool = False, cnn_config=None, mlp_config=None, init_dicts=None,
                 output_activation: str | None = None, output_layernorm: bool = False, min_latent_dim: int = 8,
                 max_latent_dim: int = 128, device="cpu", name: str = "multi_input", random_seed=None,
                 **_ignored) -> None:
        super().__init__()
        if vector_space_mlp:
            raise NotImplementedError("vector_space_mlp=True is outside the agx hot path")
        for key, space in observation_space.items():
            if not hasattr(space, "shape") or hasattr(space, "n") or len(space.shape) > 1:
                raise NotImplementedError(f"multi-input subspace {key!r}: only 1-D Box subspaces are supported")
        self.observation_space = observation_space
        self.keys = list(observation_space.keys())
        self.dims = [int(np.prod(observation_space[k].shape)) for k in self.keys]
        self.total_vector_dims = int(sum(self.dims))
        self.num_outputs, self.name, self.device = num_outputs, name, device
        self.vector_space_mlp, self.output_activation = False, output_activation
        self.output_layernorm = output_layernorm
        self.feature_net = nn.ModuleDict()
        self.final_dense = nn.Linear(self.total_vector_dims, num_outputs, device=device)
        self.final_layernorm = nn.LayerNorm(num_outputs, device=device, elementwise_affine=False) \
            if output_layernorm else None
        self.output = get_activation(output_activation)
        self.rng = np.random.default_rng(seed=random_seed)
        self.last_mutation_attr: str | None = None
        self.disabled: set[str] = set()

    def disable_mutations(self, kind: str | None = None) -> None:
        self.disabled.update(("add_latent_node", "remove_latent_node") if kind in (None, "node") else ())

    def recreate_network(self) -> None:
        """recreate_encoder (networks/base.py:493-503) for this encoder: a new
        ``final_dense`` for the current ``num_outputs`` (torch's default
        nn.Linear init, the module's only random draw), parameters kept where
        the shapes overlap (preserve_parameters, modules/base.py:472-502)."""
        old = self.final_dense
        dev = old.weight.device
        new = nn.Linear(self.total_vector_dims, self.num_outputs, device=dev)
        with torch.no_grad():
            for name in ("weight", "bias"):
                o, n = getattr(old, name), getattr(new, name)
                if o.shape == n.shape:
                    setattr(new, name, o)
                else:
                    sl = tuple(slice(0, min(a, b)) for a, b in zip(o.shape, n.shape))
                    n.data[sl] = o.data[sl]
        self.final_dense = new
        if self.final_layernorm is not None:
            self.final_layernorm = nn.LayerNorm(self.num_outputs, device=dev, elementwise_affine=False)

    def forward(self, x) -> torch.Tensor:
        if isinstance(x, (tuple, list)):
            x = dict(zip(self.keys, x))
        parts = []
        for k in self.keys:
            o = x[k] if isinstance(x[k], torch.Tensor) else torch.tensor(x[k], dtype=torch.float32,
                                                                          device=self.device)
            parts.append(o.unsqueeze(0) if o.dim() == 1 else o)
        latent = self.final_dense(torch.cat(parts, dim=1))
        if self.final_layernorm is not None:
            latent = self.final_layernorm(latent)
        return self.output(latent)
