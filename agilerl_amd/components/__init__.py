"""Drop-in replacements for agilerl.components (segment trees, replay and
rollout buffers) with their storage in HBM and their hot loops in libagx."""

from .multi_agent_replay_buffer import MultiAgentReplayBuffer
from .replay_buffer import MultiStepReplayBuffer, PrioritizedReplayBuffer, ReplayBuffer
from .rollout_buffer import RolloutBuffer
from .sampler import Sampler
from .segment_tree import MinSegmentTree, SegmentTree, SumSegmentTree

__all__ = ["ReplayBuffer", "MultiStepReplayBuffer", "PrioritizedReplayBuffer", "RolloutBuffer", "SegmentTree", "SumSegmentTree",
           "MinSegmentTree", "Sampler",
           "MultiAgentReplayBuffer"]
