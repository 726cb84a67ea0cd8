"""Drop-in ``EvolvableMLP`` (agilerl/modules/mlp.py:10-336) and ``create_mlp``
(agilerl/utils/evolvable_networks.py:527-644).

Same constructor, module names (``{name}_linear_layer_{i}``,
``{name}_layer_norm_{i}``, ``{name}_activation_{i}``,
``{name}_linear_layer_output``, ``{name}_layer_norm_output``,
``{name}_activation_output``) and therefore the same state-dict keys, the
same initialisation (orthogonal gain sqrt(2), bias 0; output x0.1 when
``output_vanish``) and the same architecture mutations (add/remove layer or
nodes, parameters preserved by overlapping slices).  The PPO population
engine flattens exactly this layout into its HBM parameter rows
(population/nets.py ``state_dict_keys``), so reference checkpoints map onto
the fused kernels key by key.
"""

from __future__ import annotations

import copy
from collections import OrderedDict
from typing import Any

import numpy as np
import torch
from torch import nn

from .custom_components import GumbelSoftmax, NoisyLinear, reset_noise_layers


class NewGELU(nn.Module):
    """tanh-approximated GELU (the reference's ``NewGELU``)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return 0.5 * x * (1.0 + torch.tanh(np.sqrt(2.0 / np.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def get_activation(activation_name: str | None, new_gelu: bool = False) -> nn.Module:
    """Activation module by name (evolvable_networks.py:348-374); None -> Identity."""
    table = {"Tanh": nn.Tanh, "ReLU": nn.ReLU, "ELU": nn.ELU, "Softsign": nn.Softsign, "Sigmoid": nn.Sigmoid,
             "GumbelSoftmax": GumbelSoftmax, "Softplus": nn.Softplus, "Softmax": nn.Softmax,
             "LeakyReLU": nn.LeakyReLU, "PReLU": nn.PReLU, "GELU": NewGELU if new_gelu else nn.GELU,
             "Identity": nn.Identity}
    name = activation_name if activation_name is not None else "Identity"
    return table[name](dim=-1) if name == "Softmax" else table[name]()


def layer_init(layer: nn.Module, std: float = float(np.sqrt(2)), bias_const: float = 0.0) -> nn.Module:
    """Orthogonal weights (gain ``std``), constant bias (evolvable_networks.py:410-441)."""
    if hasattr(layer, "weight"):
        nn.init.orthogonal_(layer.weight, std)
    elif hasattr(layer, "weight_mu") and hasattr(layer, "weight_sigma"):
        nn.init.orthogonal_(layer.weight_mu, std)
        nn.init.orthogonal_(layer.weight_sigma, std)
    if hasattr(layer, "bias"):
        nn.init.constant_(layer.bias, bias_const)
    elif hasattr(layer, "bias_mu"):
        nn.init.constant_(layer.bias_mu, bias_const)
    return layer


def create_mlp(input_size: int, output_size: int, hidden_size: list[int], output_vanish: bool,
               output_activation: str | None = None, noisy: bool = False, init_layers: bool = True,
               layer_norm: bool = False, output_layernorm: bool = False, activation: str = "ReLU",
               noise_std: float = 0.1, device="cpu", new_gelu: bool = False, name: str = "mlp") -> nn.Sequential:
    net: OrderedDict[str, nn.Module] = OrderedDict()
    dims = [input_size, *hidden_size]
    for i in range(1, len(dims)):
        lin = NoisyLinear(dims[i - 1], dims[i], noise_std, device=device) if noisy else \
            nn.Linear(dims[i - 1], dims[i], device=device)
        net[f"{name}_linear_layer_{i}"] = layer_init(lin) if init_layers else lin
        if layer_norm:
            net[f"{name}_layer_norm_{i}"] = nn.LayerNorm(dims[i], device=device)
        net[f"{name}_activation_{i}"] = get_activation(activation, new_gelu)
    out = NoisyLinear(dims[-1], output_size, noise_std, device=device) if noisy else \
        nn.Linear(dims[-1], output_size, device=device)
    if init_layers:
        out = layer_init(out)
    if output_vanish:
        with torch.no_grad():
            for t in ((out.weight_mu, out.bias_mu, out.weight_sigma, out.bias_sigma) if noisy
                      else (out.weight, out.bias)):
                t.mul_(0.1)
    net[f"{name}_linear_layer_output"] = out
    if output_layernorm:
        net[f"{name}_layer_norm_output"] = nn.LayerNorm(output_size, device=device, elementwise_affine=False)
    net[f"{name}_activation_output"] = get_activation(output_activation, new_gelu)
    return nn.Sequential(net)


def preserve_parameters(old_net: nn.Module, new_net: nn.Module) -> nn.Module:
    """Copy parameters of equal name; differing shapes copy the overlapping
    slice, except norms (modules/base.py:472-502)."""
    old = dict(old_net.named_parameters())
    for key, param in new_net.named_parameters():
        if key in old:
            o = old[key]
            if o.data.size() == param.data.size():
                param.data = o.data
            elif "norm" not in key:
                sl = tuple(slice(0, min(a, b)) for a, b in zip(o.data.size(), param.data.size()))
                param.data[sl] = o.data[sl]
    return new_net


class EvolvableMLP(nn.Module):
    def __init__(self, num_inputs: int, num_outputs: int, hidden_size: list[int], activation: str = "ReLU",
                 output_activation: str | None = None, min_hidden_layers: int = 1, max_hidden_layers: int = 3,
                 min_mlp_nodes: int = 32, max_mlp_nodes: int = 500, layer_norm: bool = True,
                 output_layernorm: bool = False, output_vanish: bool = True, init_layers: bool = True,
                 noisy: bool = False, noise_std: float = 0.5, new_gelu: bool = False, device="cpu",
                 name: str = "mlp", random_seed: int | None = None) -> None:
        super().__init__()
        assert num_inputs > 0, "'num_inputs' cannot be less than or equal to zero, please enter a valid integer."
        assert num_outputs > 0, "'num_outputs' cannot be less than or equal to zero, please enter a valid integer."
        for num in hidden_size:
            assert num > 0, "'hidden_size' cannot contain zero, please enter a valid integer."
        assert len(hidden_size) != 0, "MLP must contain at least one hidden layer."
        assert min_hidden_layers < max_hidden_layers, "'min_hidden_layers' must be less than 'max_hidden_layers."
        assert min_mlp_nodes < max_mlp_nodes, "'min_mlp_nodes' must be less than 'max_mlp_nodes."
        self.device = device
        self.random_seed = random_seed
        self.rng = np.random.default_rng(seed=random_seed)
        self.name = name
        self.num_inputs, self.num_outputs = num_inputs, num_outputs
        self._activation, self.new_gelu, self.output_activation = activation, new_gelu, output_activation
        self.min_hidden_layers, self.max_hidden_layers = min_hidden_layers, max_hidden_layers
        self.min_mlp_nodes, self.max_mlp_nodes = min_mlp_nodes, max_mlp_nodes
        self.layer_norm, self.output_vanish, self.output_layernorm = layer_norm, output_vanish, output_layernorm
        self.init_layers, self.hidden_size = init_layers, list(hidden_size)
        self.noisy, self.noise_std = noisy, noise_std
        self.last_mutation_attr: str | None = None
        self.disabled: set[str] = set()
        self.model = self._create()

    def _create(self) -> nn.Sequential:
        return create_mlp(input_size=self.num_inputs, output_size=self.num_outputs, hidden_size=self.hidden_size,
                          output_vanish=self.output_vanish, output_activation=self.output_activation,
                          noisy=self.noisy, init_layers=self.init_layers, layer_norm=self.layer_norm,
                          output_layernorm=self.output_layernorm, activation=self.activation,
                          noise_std=self.noise_std, device=self.device, new_gelu=self.new_gelu, name=self.name)

    @property
    def activation(self) -> str:
        return self._activation

    @activation.setter
    def activation(self, activation: str) -> None:
        self._activation = activation

    @property
    def net_config(self) -> dict[str, Any]:
        """Constructor arguments minus num_inputs / num_outputs / device / name (mlp.py:137-150)."""
        return dict(hidden_size=list(self.hidden_size), activation=self.activation,
                    output_activation=self.output_activation, min_hidden_layers=self.min_hidden_layers,
                    max_hidden_layers=self.max_hidden_layers, min_mlp_nodes=self.min_mlp_nodes,
                    max_mlp_nodes=self.max_mlp_nodes, layer_norm=self.layer_norm,
                    output_layernorm=self.output_layernorm, output_vanish=self.output_vanish,
                    init_layers=self.init_layers, noisy=self.noisy, noise_std=self.noise_std,
                    new_gelu=self.new_gelu, random_seed=self.random_seed)

    def forward(self, x) -> torch.Tensor:
        if not isinstance(x, torch.Tensor):
            x = torch.tensor(np.asarray(x), dtype=torch.float32, device=self.device)
        if x.dim() == 1:
            x = x.unsqueeze(0)
        return self.model(x)

    def get_output_dense(self) -> nn.Module:
        return getattr(self.model, f"{self.name}_linear_layer_output")

    def reset_noise(self) -> None:
        reset_noise_layers([m for m in self.modules() if isinstance(m, NoisyLinear)])

    @staticmethod
    def _init_gaussian(module: nn.Module, std_coeff: float) -> None:
        for m in ([module] if isinstance(module, nn.Linear) else list(module.modules())):
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, mean=0, std=std_coeff / m.weight.size(1))
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def init_weights_gaussian(self, std_coeff: float = 4, output_coeff: float = 4) -> None:
        self._init_gaussian(self.model, std_coeff)
        self._init_gaussian(self.get_output_dense(), output_coeff)

    # ---- architecture mutations (mlp.py:214-336) ---------------------------
    LAYER_METHODS = ("add_layer", "remove_layer")
    NODE_METHODS = ("add_node", "remove_node")

    def disable_mutations(self, kind: str | None = None) -> None:
        """EvolvableModule.disable_mutations: "layer", "node" or both (None);
        a disabled method leaves the owner's mutation table (networks/base.py
        filters it)."""
        if kind in (None, "layer"):
            self.disabled.update(self.LAYER_METHODS)
        if kind in (None, "node"):
            self.disabled.update(self.NODE_METHODS)

    def change_activation(self, activation: str, output: bool = False) -> None:
        if output:
            self.output_activation = activation
        self.activation = activation
        self.recreate_network()

    def add_layer(self) -> dict[str, int] | None:
        self.last_mutation_attr = "add_layer"
        if len(self.hidden_size) < self.max_hidden_layers:
            self.hidden_size += [self.hidden_size[-1]]
            self.recreate_network()
            return None
        return self.add_node()

    def remove_layer(self) -> dict[str, int] | None:
        self.last_mutation_attr = "remove_layer"
        if len(self.hidden_size) > self.min_hidden_layers:
            self.hidden_size = self.hidden_size[:-1]
            self.recreate_network()
            return None
        return self.add_node()

    def add_node(self, hidden_layer: int | None = None, numb_new_nodes: int | None = None) -> dict[str, int]:
        self.last_mutation_attr = "add_node"
        hidden_layer = int(self.rng.integers(0, len(self.hidden_size))) if hidden_layer is None else \
            min(hidden_layer, len(self.hidden_size) - 1)
        if numb_new_nodes is None:
            numb_new_nodes = int(self.rng.choice([16, 32, 64]))
        if self.hidden_size[hidden_layer] + numb_new_nodes <= self.max_mlp_nodes:
            self.hidden_size[hidden_layer] += numb_new_nodes
        self.recreate_network()
        return {"hidden_layer": hidden_layer, "numb_new_nodes": numb_new_nodes}

    def remove_node(self, hidden_layer: int | None = None, numb_new_nodes: int | None = None) -> dict[str, int]:
        self.last_mutation_attr = "remove_node"
        hidden_layer = int(self.rng.integers(0, len(self.hidden_size))) if hidden_layer is None else \
            min(hidden_layer, len(self.hidden_size) - 1)
        if numb_new_nodes is None:
            numb_new_nodes = int(self.rng.choice([16, 32, 64]))
        if self.hidden_size[hidden_layer] - numb_new_nodes > self.min_mlp_nodes:
            self.hidden_size[hidden_layer] -= numb_new_nodes
        self.recreate_network()
        return {"hidden_layer": hidden_layer, "numb_new_nodes": numb_new_nodes}

    def recreate_network(self) -> None:
        self.model = preserve_parameters(self.model, self._create())

    def clone(self) -> "EvolvableMLP":
        return copy.deepcopy(self)
