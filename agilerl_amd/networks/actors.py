"""``DeterministicActor`` (agilerl/networks/actors.py:49-230): EvolvableMLP
encoder + head named "actor"; output activation GumbelSoftmax for Discrete
action spaces, Tanh for Box (or a user choice among the allowed ones)."""

from __future__ import annotations

import warnings

import torch

from .base import EvolvableNetwork, as_config, flatdim, mlp_net_config

_ALLOWED = ("Tanh", "Softsign", "Sigmoid", "Softmax", "GumbelSoftmax")


def get_output_bounds(output_activation: str):
    if output_activation in ("Tanh", "Softsign"):
        return -1.0, 1.0
    if output_activation in ("Sigmoid", "Softmax", "GumbelSoftmax"):
        return 0.0, 1.0
    return None, None


class DeterministicActor(EvolvableNetwork):
    def __init__(self, observation_space, action_space, encoder_cls=None, encoder_config=None, head_config=None,
                 min_latent_dim: int = 8, max_latent_dim: int = 128, latent_dim: int = 32, simba: bool = False,
                 recurrent: bool = False, device="cpu", random_seed: int | None = None,
                 encoder_name: str = "encoder") -> None:
        super().__init__(observation_space, encoder_cls=encoder_cls, encoder_config=encoder_config,
                         action_space=action_space, min_latent_dim=min_latent_dim, max_latent_dim=max_latent_dim,
                         latent_dim=latent_dim, simba=simba, recurrent=recurrent, device=device,
                         random_seed=random_seed, encoder_name=encoder_name)
        discrete = hasattr(action_space, "n")
        if discrete:
            self.action_low = self.action_high = None
            output_activation = "GumbelSoftmax"
        else:
            self.action_low = torch.as_tensor(action_space.low, dtype=torch.float32)
            self.action_high = torch.as_tensor(action_space.high, dtype=torch.float32)
            output_activation = "Tanh"
        head_config = as_config(head_config)
        if head_config is not None and "output_activation" in head_config:
            user = head_config["output_activation"]
            if user in _ALLOWED:
                output_activation = user
            else:
                warnings.warn(f"Output activation must be one of the following: {', '.join(_ALLOWED)}. Got {user} "
                              "instead. Using default output activation.", stacklevel=2)
        self.output_activation = output_activation
        if head_config is None:
            head_config = mlp_net_config([32], output_activation=output_activation)
        else:
            head_config["output_activation"] = output_activation
        self.output_size = flatdim(action_space)
        self.head_net = self.create_mlp(self.latent_dim, self.output_size, "actor", head_config)

    @staticmethod
    def rescale_action(action: torch.Tensor, low: torch.Tensor, high: torch.Tensor,
                       output_activation: str) -> torch.Tensor:
        """[min_out, max_out] -> [low, high] (actors.py:153-188)."""
        lo, hi = get_output_bounds(output_activation)
        if lo is None or hi is None or low.isinf().any() or high.isinf().any():
            return action
        return (low + (high - low) * ((action - lo) / (hi - lo))).to(low.dtype)

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        return self.head_net(self.extract_features(obs))
