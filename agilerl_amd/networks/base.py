"""Encoder part of ``EvolvableNetwork`` (agilerl/networks/base.py:150-560).

Box observations get EvolvableMLP encoders, image Box spaces (3-D shape,
utils/evolvable_networks.py:74-84) EvolvableCNN encoders on the HIP conv
kernels (modules/cnn.py), Dict/Tuple spaces EvolvableMultiInput; recurrent
and SimBa encoders are outside the hot path and raise NotImplementedError.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch
from torch import nn

from ..modules.cnn import EvolvableCNN
from ..modules.mlp import EvolvableMLP, preserve_parameters


def mlp_net_config(hidden_size, **overrides) -> dict[str, Any]:
    """``asdict(MlpNetConfig(...))`` (modules/configs.py:56-70)."""
    cfg = dict(hidden_size=list(hidden_size), activation="ReLU", output_activation=None, min_hidden_layers=1,
               max_hidden_layers=3, min_mlp_nodes=16, max_mlp_nodes=500, layer_norm=True, output_vanish=True,
               output_layernorm=False, init_layers=True, noisy=False, noise_std=0.5)
    cfg.update(overrides)
    return cfg


def cnn_net_config(**overrides) -> dict[str, Any]:
    """``asdict(CnnNetConfig(channel_size=[32, 32], kernel_size=[3, 3],
    stride_size=[1, 1], output_activation="ReLU"))`` — the default image
    encoder (evolvable_networks.py:190-196, configs.py:114-127)."""
    cfg = dict(channel_size=[32, 32], kernel_size=[3, 3], stride_size=[1, 1], sample_input=None, activation="ReLU",
               output_activation="ReLU", block_type="Conv2d", min_hidden_layers=1, max_hidden_layers=6,
               min_channel_size=16, max_channel_size=256, layer_norm=False, init_layers=True)
    cfg.update(overrides)
    return cfg


def is_image_space(space) -> bool:
    """evolvable_networks.py:74-84: a Box with a 3-D shape."""
    return hasattr(space, "shape") and not hasattr(space, "n") and not hasattr(space, "spaces") \
        and space.shape is not None and len(space.shape) == 3


def image_norm_bounds(space) -> tuple[float, float] | None:
    """(low, high) of apply_image_normalization (algo_utils.py:1134-1183) when
    the kernel can fold it into its load: finite, uniform bounds other than
    [0, 1].  None when the reference leaves the frames as they are (infinite
    or [0, 1] bounds); ValueError for per-pixel bounds, which the agx path
    does not normalise."""
    low, high = np.asarray(space.low, dtype=np.float64), np.asarray(space.high, dtype=np.float64)
    if np.isinf(high).any() or np.isinf(low).any():
        return None
    if np.all(high == 1) and np.all(low == 0):
        return None
    if low.min() != low.max() or high.min() != high.max():
        raise ValueError("agx image inputs: per-pixel observation bounds are not supported (uniform low/high)")
    return float(np.float32(low.flat[0])), float(np.float32(high.flat[0]))


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


def mutation_probs(table: list[str], new_layer_prob: float) -> list[float]:
    """EvolvableModule.get_mutation_probs (modules/base.py:661-685) over a
    table of method names."""
    layer = [m for m in table if m.split(".")[-1] in ("add_layer", "remove_layer")]
    nl, nn_ = len(layer), len(table) - len(layer)
    if nl == 0 or nn_ == 0:
        return [1 / len(table)] * len(table)
    return [new_layer_prob / nl if m in layer else (1 - new_layer_prob) / nn_ for m in table]


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
        self.rng = np.random.default_rng(seed=random_seed)  # latent-node draws (EvolvableModule.rng)
        encoder_config = as_config(encoder_config)
        image = not multi and is_image_space(observation_space)
        if encoder_config is None:  # get_default_encoder_config (utils/evolvable_networks.py:168-216)
            encoder_config = {"output_activation": "ReLU"} if multi else cnn_net_config() if image else \
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
        if image:  # EvolvableCNN encoder (base.py:521-530)
            encoder_config.pop("num_outputs", None)
            self.encoder_config = encoder_config
            self.encoder = EvolvableCNN(input_shape=list(observation_space.shape), num_outputs=latent_dim,
                                        device=device, name=encoder_name, **encoder_config)
            # the encoder's LAYER mutations are disabled (networks/base.py:266-268)
            self.encoder.disable_mutations("layer")
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

    def set_image_norm(self, bounds: tuple[float, float] | None) -> None:
        """uint8 frames are normalised inside the first convolution's load."""
        if not isinstance(self.encoder, EvolvableCNN):
            return
        if bounds is None:
            self.encoder.clear_image_norm()
        else:
            self.encoder.set_image_norm(*bounds)

    def recreate_encoder(self) -> None:
        """networks/base.py:493-503: the encoder rebuilt for the current latent,
        parameters kept where the shapes overlap."""
        if isinstance(self.encoder, EvolvableCNN):
            self.encoder.num_outputs = self.latent_dim
            self.encoder.recreate_network()
            return
        cfg = dict(self.encoder.net_config)
        new = EvolvableMLP(num_inputs=self.encoder.num_inputs, num_outputs=self.latent_dim, device=self.device,
                           name=self.encoder_name, **cfg)
        self.encoder = preserve_parameters(self.encoder, new)

    # ---- architecture mutations (networks/base.py:457-491, modules/mlp.py:213-312)
    def add_latent_node(self, numb_new_nodes: int | None = None) -> dict:
        if numb_new_nodes is None:
            numb_new_nodes = int(self.rng.choice([8, 16, 32]))
        old = self.latent_dim
        if self.latent_dim + numb_new_nodes < self.max_latent_dim:
            self.latent_dim += numb_new_nodes
        self.recreate_network(old)
        return {"numb_new_nodes": numb_new_nodes}

    def remove_latent_node(self, numb_new_nodes: int | None = None) -> dict:
        if numb_new_nodes is None:
            numb_new_nodes = int(self.rng.choice([8, 16, 32]))
        old = self.latent_dim
        if self.latent_dim - numb_new_nodes > self.min_latent_dim:
            self.latent_dim -= numb_new_nodes
        self.recreate_network(old)
        return {"numb_new_nodes": numb_new_nodes}

    def recreate_network(self, old_latent: int | None = None) -> None:
        """Encoder (output = latent) and head (input = latent [+ whatever the
        head concatenates]) rebuilt with their parameters kept where the
        shapes overlap (preserve_parameters)."""
        old_latent = self.latent_dim if old_latent is None else old_latent
        self.encoder.num_outputs = self.latent_dim
        self.encoder.recreate_network()
        head = getattr(self, "head_net", None)
        if head is not None:
            head.num_inputs = head.num_inputs - old_latent + self.latent_dim
            head.recreate_network()

    # a multi-input encoder's (the MADDPG critic's) table, in the reference's
    # order under PYTHONHASHSEED=0 (tests/golden maddpgarch*: critic_methods)
    MULTI_INPUT_METHODS = ["head_net.remove_layer", "head_net.add_layer", "remove_latent_node", "add_latent_node",
                           "encoder.remove_latent_node", "encoder.add_latent_node", "head_net.add_node",
                           "head_net.remove_node"]

    @property
    def mutation_methods(self) -> list[str]:
        """The network's mutation table in the reference's order under
        PYTHONHASHSEED=0 (population/arch.py for MLP encoders,
        population/image_arch.py for CNN encoders), without the methods its
        modules disabled (EvolvableModule.disable_mutations)."""
        from ..population import arch, image_arch
        from ..modules.multi_input import EvolvableMultiInput

        if isinstance(self.encoder, EvolvableCNN):
            table = image_arch.METHODS
        elif isinstance(self.encoder, EvolvableMultiInput):
            table = self.MULTI_INPUT_METHODS
        else:
            table = arch.METHODS

        def on(m: str) -> bool:
            if "." not in m:
                return True
            owner, name = m.split(".", 1)
            return name not in getattr(getattr(self, owner, None), "disabled", ())

        return [m for m in table if on(m)]

    @staticmethod
    def is_layer_method(method: str) -> bool:
        return method.split(".")[-1] in ("add_layer", "remove_layer")

    def sample_mutation_method(self, new_layer_prob: float, rng) -> str:
        """EvolvableModule.sample_mutation_method (modules/base.py:661-711):
        layer methods share new_layer_prob, node methods the rest (uniform
        when one kind is empty)."""
        table = self.mutation_methods
        return str(rng.choice(table, p=mutation_probs(table, new_layer_prob), size=1)[0])

    def share_rng(self) -> None:
        """ModuleMeta (modules/base.py:253-255): a network's evolvable modules
        draw from the network's generator (a CNN's kernel-size helper keeps
        its own)."""
        for name in ("encoder", "head_net"):
            mod = getattr(self, name, None)
            if mod is not None and hasattr(mod, "rng"):
                mod.rng = self.rng

    def apply_mutation(self, method: str) -> str | None:
        """One method of the mutation table on this network -> the method
        actually applied (layer mutations at a limit fall back to add_node,
        mlp.py:227-252; a CNN falls back as modules/cnn.py does), or None when
        the fallback is a disabled method (MutationContext, base.py:181-190)."""
        return self.apply_mutation_dict(method)[0]

    def apply_mutation_dict(self, method: str, mut_dict: dict | None = None) -> tuple[str | None, dict]:
        """_apply_arch_mutation (hpo/mutation.py:1013-1070) on this network:
        ``method`` called with ``mut_dict`` as its arguments -> (the method
        actually applied or None, the mutation dict it returned)."""
        self.share_rng()
        kw = dict(mut_dict or {})
        if method in ("add_latent_node", "remove_latent_node"):
            d = getattr(self, method)(**kw)
            return method, d or {}
        owner, name = method.split(".")
        mod = getattr(self, owner)
        d = getattr(mod, name)(**kw)
        if mod.last_mutation_attr is None:
            return None, d or {}
        return f"{owner}.{mod.last_mutation_attr}", d or {}

    @property
    def activation(self) -> str | None:
        """networks/base.py:298-305: the encoder's activation."""
        return getattr(self.encoder, "activation", None)

    def change_activation(self, activation: str, output: bool = False) -> None:
        """networks/base.py:445-455: every evolvable module of the network
        takes the activation; the encoder's output activation too."""
        for name in ("encoder", "head_net"):
            mod = getattr(self, name, None)
            if mod is not None and hasattr(mod, "change_activation"):
                mod.change_activation(activation, output=True if name == "encoder" else output)

    def reset_noise(self) -> None:
        from ..modules.custom_components import NoisyLinear, reset_noise_layers

        reset_noise_layers([m for m in self.modules() if isinstance(m, NoisyLinear)])
