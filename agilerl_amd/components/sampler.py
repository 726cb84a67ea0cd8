"""Drop-in ``Sampler`` (agilerl/components/sampler.py:25-202) over the agx
HBM buffers (standard / PER / n-step; the distributed dataloader form is
outside the hot path)."""

from __future__ import annotations


class Sampler:
    def __init__(self, memory=None, dataset=None, dataloader=None) -> None:
        if memory is None:
            raise NotImplementedError("the distributed dataset/dataloader sampler is outside the agx hot path")
        self.memory = memory
        from .replay_buffer import MultiStepReplayBuffer, PrioritizedReplayBuffer

        if isinstance(memory, PrioritizedReplayBuffer):
            self.sample = self.sample_per
        elif isinstance(memory, MultiStepReplayBuffer):
            self.sample = self.sample_n_step
        else:
            self.sample = self.sample_standard

    def sample_standard(self, batch_size: int, return_idx: bool = False):
        return self.memory.sample(batch_size, return_idx)

    def sample_per(self, batch_size: int, beta: float):
        return self.memory.sample(batch_size, beta)

    def sample_n_step(self, idxs):
        return self.memory.sample_from_indices(idxs)
