from .cnn import EvolvableCNN
from .custom_components import GumbelSoftmax, NoisyLinear
from .mlp import EvolvableMLP, create_mlp, get_activation, layer_init, preserve_parameters

__all__ = ["EvolvableCNN", "EvolvableMLP", "create_mlp", "get_activation", "layer_init", "preserve_parameters", "NoisyLinear",
           "GumbelSoftmax"]
