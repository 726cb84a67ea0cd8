"""agx_replay_gather (csrc/replay_gather.hip): the sampled batch of every
stored field in one launch, bit-exact against torch's index_select of the
same rows — uint8 frames (16-byte units), int64 / f32 scalars (4-byte units)
and an odd-width uint8 field (1-byte units); uniform and prioritized
sampling (replay_buffer.py:97-137, 361-409)."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _fill(buf, n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    buf.add({"obs": torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=DEV, generator=g),
             "action": torch.randint(0, 6, (n,), device=DEV, generator=g),
             "reward": torch.randn(n, device=DEV, generator=g),
             "next_obs": torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=DEV, generator=g),
             "done": (torch.rand(n, device=DEV, generator=g) < 0.1).float(),
             "tag": torch.randint(0, 256, (n, 3), dtype=torch.uint8, device=DEV, generator=g)})


def _same(samples, storage, idx):
    for k, v in storage.items():
        ref = v.index_select(0, idx.reshape(-1).to(torch.int64))
        assert samples[k].dtype == ref.dtype and samples[k].shape == ref.shape, k
        assert torch.equal(samples[k], ref), k


def test_prioritized_sample_gathers_every_field():
    from agilerl_amd.components import PrioritizedReplayBuffer

    torch.manual_seed(0)
    buf = PrioritizedReplayBuffer(5000, alpha=0.6)
    _fill(buf, 3000, 1)
    for B in (1, 64, 257):
        s = buf.sample(B, beta=0.4)
        _same(s, buf.storage, s["idxs"])


def test_uniform_sample_gathers_every_field():
    from agilerl_amd.components import ReplayBuffer

    torch.manual_seed(1)
    buf = ReplayBuffer(4000)
    _fill(buf, 2500, 2)
    s = buf.sample(128, return_idx=True)
    _same(s, buf.storage, s["idxs"])
