"""MLP-encoder part of ``EvolvableNetwork`` (agilerl/networks/base.py:150-560).

The hot path covers Box observations with EvolvableMLP encoders; image / dict
/ recurrent / SimBa encoders are outside it and raise NotImplementedError.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch
from torch import nn

from ..modules.mlp import EvolvableMLP, preserve_parameters


def mlp_net_config(hidden_size, **overrides) -> dict[str, Any]:
    """``asdict(MlpNetConfig(...))`` (modules/configs.py:56-70)."""
    cfg = dict(hidden_size=list(hidden_size), activation="ReLU", output_activation=None, min_hidden_layers=1,
               max_hidden_layers=3, min_mlp_nodes=16, max_mlp_nodes=500, layer_norm=True, output_vanish=True,
               output_layernorm=False, init_layers=True, noisy=False, noise_std=0.5)
    cfg.update(overrides)
    return cfg


def as_config(cfg) -> dict[str, Any] | None:
    if cfg is None:
        return None
    if hasattr(cfg, "__dataclass_fields__"):
        from dataclasses import asdict

        return asdict(cfg)
    return dict(cfg)


def flatdim(space) -> int:
    if hasattr(space, "n"):
        return int(space.n)
    return int(np.prod(space.shape))


class EvolvableNetwork(nn.Module):
    def __init__(self, observation_space, encoder_cls=None, encoder_config=None, action_space=None,
                 min_latent_dim: int = 8, max_latent_dim: int = 128, latent_dim: int = 32, simba: bool = False,
                 recurrent: bool = False, device="cpu", random_seed: int | None = None,
                 encoder_name: str = "encoder") -> None:
        super().__init__()
        if encoder_cls is not None or simba or recurrent:
            raise NotImplementedError("agx networks build EvolvableMLP encoders (Box observations)")
        multi = hasattr(observation_space, "spaces")
        if not multi and (not hasattr(observation_space, "shape") or hasattr(observation_space, "n")):
            raise NotImplementedError("agx networks take Box or Dict-of-Box observation spaces")
        assert latent_dim <= max_latent_dim, "Latent dimension must be less than or equal to max latent dimension."
        assert latent_dim >= min_latent_dim, "Latent dimension must be greater than or equal to min latent dimension."
        self.observation_space, self.action_space = observation_space, action_space
        self.latent_dim, self.min_latent_dim, self.max_latent_dim = latent_dim, min_latent_dim, max_latent_dim
        self.device, self.random_seed, self.encoder_name = device, random_seed, encoder_name
        encoder_config = as_config(encoder_config)
        if encoder_config is None:  # get_default_encoder_config (utils/evolvable_networks.py:168-216)
            encoder_config = {"output_activation": "ReLU"} if multi else \
                mlp_net_config([64, 64], output_activation="ReLU", output_vanish=False)
        if encoder_config.get("output_activation") is None:  # base.py:226-230
            encoder_config["output_activation"] = encoder_config.get("activation", "ReLU")
        self.flatten_obs = False
        if multi:  # EvolvableMultiInput encoder (base.py:500-520)
            from ..modules.multi_input import EvolvableMultiInput

            encoder_config.pop("num_outputs", None)
            self.encoder_config = encoder_config
            self.encoder = EvolvableMultiInput(observation_space, num_outputs=latent_dim, device=device,
                                               name=encoder_name, **encoder_config)
            return
        # MLP encoders: output LayerNorm follows layer_norm, no output vanish (base.py:547-554)
        encoder_config["output_layernorm"] = encoder_config.get("layer_norm", True)
        encoder_config["output_vanish"] = False
        encoder_config.pop("num_outputs", None)
        self.encoder_config = encoder_config
        self.flatten_obs = len(observation_space.shape) > 1
        self.encoder = EvolvableMLP(num_inputs=int(np.prod(observation_space.shape)), num_outputs=latent_dim,
                                    device=device, name=encoder_name, **encoder_config)

    def extract_features(self, x: torch.Tensor, hidden_state=None) -> torch.Tensor:
        if self.flatten_obs:
            x = x.flatten(1)
        return self.encoder(x)

    def forward_head(self, latent: torch.Tensor, *args, **kwargs) -> torch.Tensor:
        return self.head_net(latent, *args, **kwargs)

    def create_mlp(self, num_inputs: int, num_outputs: int, name: str, net_config: dict[str, Any]) -> EvolvableMLP:
        return EvolvableMLP(num_inputs=num_inputs, num_outputs=num_outputs, device=self.device, name=name,
                            **net_config)

    def recreate_encoder(self) -> None:
        cfg = dict(self.encoder.net_config)
        new = EvolvableMLP(num_inputs=self.encoder.num_inputs, num_outputs=self.latent_dim, device=self.device,
                           name=self.encoder_name, **cfg)
        self.encoder = preserve_parameters(self.encoder, new)

    def reset_noise(self) -> None:
        from ..modules.custom_components import NoisyLinear

        for m in self.modules():
            if isinstance(m, NoisyLinear):
                m.reset_noise()
