"""``QNetwork`` and ``RainbowQNetwork`` (agilerl/networks/q_networks.py:20-290)
with ``DuelingDistributionalMLP`` (agilerl/networks/custom_modules.py:20-162):
same module tree and state-dict keys as the reference (``encoder.model.
encoder_linear_layer_1.weight``, ``head_net.model.value_linear_layer_output.
weight_mu``, ``head_net.advantage_net.advantage_linear_layer_1.weight_mu`` ...).
"""

from __future__ import annotations

import warnings
from typing import Any

import torch
from torch.nn import functional as F

from ..modules.mlp import EvolvableMLP, create_mlp
from ..modules.noisy_streams import head_streams
from .base import EvolvableNetwork, as_config, flatdim, is_image_space, mlp_net_config


class QNetwork(EvolvableNetwork):
    def __init__(self, observation_space, action_space, encoder_cls=None, encoder_config=None, head_config=None,
                 min_latent_dim: int = 8, max_latent_dim: int = 128, latent_dim: int = 32, simba: bool = False,
                 recurrent: bool = False, device="cpu", random_seed: int | None = None) -> None:
        super().__init__(observation_space, encoder_cls=encoder_cls, encoder_config=encoder_config,
                         action_space=action_space, min_latent_dim=min_latent_dim, max_latent_dim=max_latent_dim,
                         latent_dim=latent_dim, simba=simba, recurrent=recurrent, device=device,
                         random_seed=random_seed)
        if not hasattr(action_space, "n") and not hasattr(action_space, "nvec"):
            raise ValueError("Action space must be either Discrete or MultiDiscrete")
        head_config = as_config(head_config)
        if head_config is None:
            head_config = mlp_net_config([32], output_activation=None)
        else:
            head_config["output_activation"] = None
        self.num_actions = flatdim(action_space)
        self.head_net = self.create_mlp(self.latent_dim, self.num_actions, "value", head_config)

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        return self.head_net(self.extract_features(obs))


class DuelingHeadFn(torch.autograd.Function):
    """(value [B, Z], advantage [B, A*Z]) -> the head output of ``mode``
    (0: q [B, A], 1: clamped probabilities [B, A, Z], 2: log-probabilities
    [B, A, Z]) on agx_dueling_head_forward / _backward (csrc/heads.hip)."""

    @staticmethod
    def forward(ctx, value, adv, support, A: int, Z: int, mode: int):
        from .. import _lib

        value, adv = value.contiguous(), adv.contiguous()
        B = value.shape[0]
        sup = support.to(device=value.device, dtype=torch.float32).contiguous() if mode == 0 else None
        shape = (B, A) if mode == 0 else (B, A, Z)
        out = torch.empty(shape, dtype=torch.float32, device=value.device)
        _lib.call("agx_dueling_head_forward", value.data_ptr(), adv.data_ptr(), _lib.ptr(sup), B, A, Z, mode,
                  out.data_ptr(), _lib.stream())
        ctx.save_for_backward(value, adv, sup if sup is not None else value.new_empty(0))
        ctx.meta = (A, Z, mode)
        return out

    @staticmethod
    def backward(ctx, g):
        from .. import _lib

        value, adv, sup = ctx.saved_tensors
        A, Z, mode = ctx.meta
        g = g.contiguous()
        dv, da = torch.empty_like(value), torch.empty_like(adv)
        _lib.call("agx_dueling_head_backward", value.data_ptr(), adv.data_ptr(), _lib.ptr(sup if mode == 0 else None),
                  g.data_ptr(), value.shape[0], A, Z, mode, dv.data_ptr(), da.data_ptr(), _lib.stream())
        return dv, da, None, None, None, None


class DuelingRowsFn(torch.autograd.Function):
    """(value [B, Z], advantage [B, A*Z], rows [B]) -> the clamped
    probabilities (mode 1) or log-probabilities (mode 2) of action rows[b]
    only, [B, Z] (agx_dueling_head_forward_rows / _backward_rows): the
    reference's ``out[range(B), rows]`` gather fused into the head."""

    @staticmethod
    def forward(ctx, value, adv, rows, A: int, Z: int, mode: int):
        from .. import _lib

        value, adv = value.contiguous(), adv.contiguous()
        rows = rows.reshape(-1).to(torch.int64).contiguous()
        B = value.shape[0]
        if rows.shape[0] != B:
            raise ValueError(f"rows: expected {B} action indices, got {rows.shape[0]}")
        out = torch.empty((B, Z), dtype=torch.float32, device=value.device)
        _lib.call("agx_dueling_head_forward_rows", value.data_ptr(), adv.data_ptr(), rows.data_ptr(), B, A, Z, mode,
                  out.data_ptr(), _lib.stream())
        ctx.save_for_backward(value, adv, rows)
        ctx.meta = (A, Z, mode)
        return out

    @staticmethod
    def backward(ctx, g):
        from .. import _lib

        value, adv, rows = ctx.saved_tensors
        A, Z, mode = ctx.meta
        if mode != 2:
            raise NotImplementedError("selected-row gradient: log mode only (the target distribution is no_grad)")
        g = g.contiguous()
        dv, da = torch.empty_like(value), torch.empty_like(adv)
        _lib.call("agx_dueling_head_backward_rows", value.data_ptr(), adv.data_ptr(), rows.data_ptr(), g.data_ptr(),
                  value.shape[0], A, Z, dv.data_ptr(), da.data_ptr(), _lib.stream())
        return dv, da, None, None, None, None


class DuelingDistributionalMLP(EvolvableMLP):
    """value stream = self.model (name "value"), advantage stream =
    self.advantage_net (name "advantage"); x = V + A - mean_a A; log-softmax
    or softmax clamped at 1e-3 (not renormalised); q = sum_z p z."""

    def __init__(self, num_inputs: int, num_outputs: int, hidden_size: list[int], num_atoms: int,
                 support: torch.Tensor, layer_norm: bool = True, output_layernorm: bool = False,
                 output_vanish: bool = True, init_layers: bool = False, noisy: bool = True, noise_std: float = 0.5,
                 activation: str = "ReLU", output_activation: str | None = None, min_hidden_layers: int = 1,
                 max_hidden_layers: int = 3, min_mlp_nodes: int = 64, max_mlp_nodes: int = 500,
                 new_gelu: bool = False, device="cpu", random_seed: int | None = None) -> None:
        super().__init__(num_inputs, num_atoms, hidden_size, activation, output_activation, min_hidden_layers,
                         max_hidden_layers, min_mlp_nodes, max_mlp_nodes, layer_norm=layer_norm,
                         output_layernorm=output_layernorm, output_vanish=output_vanish, init_layers=init_layers,
                         noisy=noisy, noise_std=noise_std, new_gelu=new_gelu, device=device, name="value",
                         random_seed=random_seed)
        self.num_atoms, self.num_actions = num_atoms, num_outputs
        self.support = support  # plain attribute, not a state-dict entry (custom_modules.py:96)
        self.advantage_net = self._advantage()

    def _advantage(self):
        return create_mlp(input_size=self.num_inputs, output_size=self.num_actions * self.num_atoms,
                          hidden_size=self.hidden_size, output_vanish=self.output_vanish,
                          output_activation=self.output_activation, noisy=self.noisy, init_layers=self.init_layers,
                          layer_norm=self.layer_norm, activation=self.activation, noise_std=self.noise_std,
                          device=self.device, new_gelu=self.new_gelu, name="advantage")

    @property
    def net_config(self) -> dict[str, Any]:
        return super().net_config

    def forward(self, x: torch.Tensor, q: bool = True, log: bool = False, rows: torch.Tensor | None = None):
        """rows (int64 [B], q=False): only action rows[b]'s distribution, [B, Z]."""
        fused = head_streams([self.model, self.advantage_net], x)  # both streams, one launch per depth
        if fused is not None:
            value, advantage = fused
        else:
            value = self.model(x)
            advantage = self.advantage_net(x)
        if rows is not None and q:
            raise ValueError("rows selects distributions: pass q=False")
        if rows is not None and value.is_cuda and self.num_atoms <= 64 and value.dtype == torch.float32:
            return DuelingRowsFn.apply(value, advantage, rows, self.num_actions, self.num_atoms, 2 if log else 1)
        if value.is_cuda and self.num_atoms <= 64 and value.dtype == torch.float32 and rows is None:
            # the combine, softmax, clamp and support dot in one HIP launch (csrc/heads.hip)
            mode = 2 if log else (0 if q else 1)
            return DuelingHeadFn.apply(value, advantage, self.support, self.num_actions, self.num_atoms, mode)
        out = self._combine(value, advantage, q, log)
        if rows is not None:
            return out[torch.arange(out.shape[0], device=out.device), rows.reshape(-1).long()]
        return out

    def _combine(self, value: torch.Tensor, advantage: torch.Tensor, q: bool, log: bool) -> torch.Tensor:
        b = value.size(0)
        x = value.view(b, 1, self.num_atoms) + advantage.view(b, self.num_actions, self.num_atoms)
        x = x - advantage.view(b, self.num_actions, self.num_atoms).mean(1, keepdim=True)
        if log:
            return F.log_softmax(x.view(-1, self.num_atoms), dim=-1).view(-1, self.num_actions, self.num_atoms)
        x = F.softmax(x.view(-1, self.num_atoms), dim=-1).view(-1, self.num_actions, self.num_atoms).clamp(min=1e-3)
        return torch.sum(x * self.support, dim=2) if q else x

    def recreate_network(self) -> None:
        from ..modules.mlp import preserve_parameters

        super().recreate_network()
        self.advantage_net = preserve_parameters(self.advantage_net, self._advantage())


class RainbowQNetwork(EvolvableNetwork):
    def __init__(self, observation_space, action_space, support: torch.Tensor, num_atoms: int = 51,
                 noise_std: float = 0.5, encoder_config=None, head_config=None, min_latent_dim: int = 8,
                 max_latent_dim: int = 128, latent_dim: int = 32, device="cpu",
                 random_seed: int | None = None) -> None:
        encoder_config = as_config(encoder_config)
        if not is_image_space(observation_space):  # q_networks.py:189-206: MLP encoders only
            if encoder_config is None:
                encoder_config = mlp_net_config([64, 64], output_activation="ReLU", output_vanish=False)
            # plain (non-noisy) encoder, default init, LayerNorm
            encoder_config["noise_std"] = noise_std
            encoder_config["output_activation"] = encoder_config.get("activation", "ReLU")
            encoder_config["output_vanish"] = False
            encoder_config["init_layers"] = False
            encoder_config["layer_norm"] = True
        super().__init__(observation_space, encoder_config=encoder_config, action_space=action_space,
                         min_latent_dim=min_latent_dim, max_latent_dim=max_latent_dim, latent_dim=latent_dim,
                         device=device, random_seed=random_seed)
        if not hasattr(action_space, "n") and not hasattr(action_space, "nvec"):
            raise ValueError("Action space must be either Discrete or MultiDiscrete")
        head_config = as_config(head_config)
        if head_config is None:
            head_config = mlp_net_config([16], output_activation=None, noise_std=noise_std)
        head_config["output_activation"] = None  # q_networks.py:243-248
        for arg in ("noisy", "init_layers", "layer_norm", "output_vanish"):
            head_config.pop(arg, None)
        self.num_actions, self.num_atoms, self.noise_std = flatdim(action_space), num_atoms, noise_std
        self.head_net = DuelingDistributionalMLP(num_inputs=self.latent_dim, num_outputs=self.num_actions,
                                                 num_atoms=num_atoms, support=support, device=device,
                                                 **head_config)

    @property
    def support(self) -> torch.Tensor:
        return self.head_net.support

    def forward(self, obs: torch.Tensor, q: bool = True, log: bool = False, rows: torch.Tensor | None = None):
        if rows is None:
            return self.head_net(self.extract_features(obs), q=q, log=log)
        return self.head_net(self.extract_features(obs), q=q, log=log, rows=rows)


class ContinuousQNetwork(EvolvableNetwork):
    """Q(s, a) (q_networks.py:302-430): encoder without LayerNorm (actions are
    concatenated to the latent unscaled), head "value" on [latent, a] -> 1."""

    def __init__(self, observation_space, action_space, encoder_cls=None, encoder_config=None, head_config=None,
                 min_latent_dim: int = 8, max_latent_dim: int = 128, latent_dim: int = 32, simba: bool = False,
                 recurrent: bool = False, device="cpu", random_seed: int | None = None) -> None:
        encoder_config = as_config(encoder_config)
        if not hasattr(observation_space, "spaces"):
            if encoder_config is None:
                encoder_config = mlp_net_config([64, 64], output_activation="ReLU", output_vanish=False,
                                                layer_norm=False)
            elif "hidden_size" in encoder_config:
                if encoder_config.get("layer_norm", False):
                    warnings.warn("Layer normalization is not supported for the encoder of DDPG networks. "
                                  "Disabling it.", stacklevel=2)
                encoder_config["layer_norm"] = False
        super().__init__(observation_space, encoder_cls=encoder_cls, encoder_config=encoder_config,
                         action_space=action_space, min_latent_dim=min_latent_dim, max_latent_dim=max_latent_dim,
                         latent_dim=latent_dim, simba=simba, recurrent=recurrent, device=device,
                         random_seed=random_seed)
        head_config = as_config(head_config)
        if head_config is None:
            head_config = mlp_net_config([32], output_activation=None)
        else:
            head_config["output_activation"] = None
        self.num_actions = action_space_flatdim(action_space)
        self.head_net = self.create_mlp(self.latent_dim + self.num_actions, 1, "value", head_config)

    def forward(self, obs, actions) -> torch.Tensor:
        if not isinstance(actions, torch.Tensor):
            actions = torch.as_tensor(actions, dtype=torch.float32)
        if actions.dim() == 1:
            actions = actions.unsqueeze(0)
        return self.head_net(torch.cat([self.extract_features(obs), actions], dim=-1))


def action_space_flatdim(space) -> int:
    if isinstance(space, (list, tuple)):
        return sum(action_space_flatdim(s) for s in space)
    return flatdim(space)
