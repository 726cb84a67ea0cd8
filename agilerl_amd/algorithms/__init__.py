"""Drop-in algorithm classes (agilerl.algorithms) on the agx hot path."""

from .dqn import DQN, RainbowDQN
from .maddpg import MADDPG
from .ppo import PPO

__all__ = ["PPO", "DQN", "RainbowDQN", "MADDPG"]
