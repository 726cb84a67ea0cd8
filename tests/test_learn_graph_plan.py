"""learn_graph._copy_plan: which static-input sets go through the one-launch
batched copy (agx_replay_gather over arange(B)) and which fall back to
torch's per-tensor copies.  Host logic only; the copy itself runs in the
replayed-update GPU tests (test_cnn_gpu.py, test_flat_state_gpu.py)."""
import torch

from agilerl_amd.algorithms.learn_graph import _copy_plan


def test_plan_covers_a_replay_batch():
    B = 64
    xs = [torch.zeros(B, 4, 84, 84, dtype=torch.uint8), torch.zeros(B, dtype=torch.int64), torch.zeros(B),
          torch.zeros(B, 4, 84, 84, dtype=torch.uint8), torch.zeros(B), torch.zeros(B, 1)]
    idx, dsts, rbytes = _copy_plan(xs)
    assert idx.tolist() == list(range(B))
    assert list(rbytes) == [4 * 84 * 84, 8, 4, 4 * 84 * 84, 4, 4]
    assert list(dsts) == [x.data_ptr() for x in xs]


def test_plan_refuses_what_the_gather_cannot_copy():
    B = 8
    assert _copy_plan([]) is False
    assert _copy_plan([torch.zeros(())]) is False  # no batch dimension
    assert _copy_plan([torch.zeros(B), torch.zeros(B + 1)]) is False  # ragged leading dims
    assert _copy_plan([torch.zeros(4, B).t()]) is False  # not contiguous
    assert _copy_plan([torch.zeros(B, 0)]) is False  # empty rows
    assert _copy_plan([torch.zeros(B)] * 9) is False  # more fields than one launch takes
    assert _copy_plan([torch.zeros(1 << 16)]) is False  # batch beyond the launch's grid
