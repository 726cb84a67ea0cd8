from .base import EvolvableNetwork
from .q_networks import DuelingDistributionalMLP, QNetwork, RainbowQNetwork

__all__ = ["EvolvableNetwork", "QNetwork", "RainbowQNetwork", "DuelingDistributionalMLP"]
