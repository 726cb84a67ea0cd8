from .actors import DeterministicActor
from .base import EvolvableNetwork
from .q_networks import ContinuousQNetwork, DuelingDistributionalMLP, QNetwork, RainbowQNetwork

__all__ = ["EvolvableNetwork", "QNetwork", "RainbowQNetwork", "DuelingDistributionalMLP", "ContinuousQNetwork",
           "DeterministicActor"]
