"""Drop-in components on the GPU: SegmentTree / SumSegmentTree /
MinSegmentTree (the reference's own known answers, tests/test_components/
test_segment_tree.py:39-129, plus random batches bit-exact against the
oracle), PrioritizedReplayBuffer (indices bit-exact, weights <= 1 ulp f32 vs
the oracle restatement of replay_buffer.py:261-428 under the same global
torch seed), ReplayBuffer and RolloutBuffer."""

import operator

import numpy as np
import pytest
import torch

from oracle import gae as ogae
from oracle import per as oper

pytestmark = pytest.mark.gpu


def test_segment_tree_creation_and_setitem():
    from agilerl_amd.components.segment_tree import SegmentTree

    t = SegmentTree(8, operator.add, 0.0)
    assert t.capacity == 8 and t.operation is operator.add
    assert t.tree.cpu().tolist() == [0.0] * 16
    t[3] = 5.0
    assert t[3] == 5.0
    with pytest.raises(AssertionError):
        SegmentTree(6, operator.add, 0.0)


def test_sum_tree_known_answers():
    from agilerl_amd.components.segment_tree import SumSegmentTree

    tree = SumSegmentTree(4)
    tree[2] = 1.0
    tree[3] = 3.0
    assert np.isclose(tree.sum(), 4.0)
    assert np.isclose(tree.sum(0, 2), 0.0)
    assert np.isclose(tree.sum(0, 3), 1.0)
    assert np.isclose(tree.sum(2, 3), 1.0)
    assert np.isclose(tree.sum(2, -1), 1.0)
    assert np.isclose(tree.sum(2, 4), 4.0)
    for ub, want in [(0.0, 2), (0.5, 2), (0.99, 2), (1.01, 3), (3.0, 3), (4.0, 3)]:
        assert tree.retrieve(ub) == want
    tree2 = SumSegmentTree(4)
    tree2[2] = 1.0
    tree2[2] = 3.0
    assert np.isclose(tree2.sum(), 3.0) and np.isclose(tree2.sum(1, 2), 0.0) and np.isclose(tree2.sum(2, 4), 3.0)
    tree3 = SumSegmentTree(4)
    for i, v in enumerate([0.5, 1.0, 1.0, 3.0]):
        tree3[i] = v
    for ub, want in [(0.0, 0), (0.55, 1), (0.99, 1), (1.51, 2), (3.0, 3), (5.5, 3)]:
        assert tree3.retrieve(ub) == want
    with pytest.raises(AssertionError):
        tree3.retrieve(5.6)


def test_min_tree_known_answers():
    from agilerl_amd.components.segment_tree import MinSegmentTree

    tree = MinSegmentTree(4)
    tree[0] = 1.0
    tree[2] = 0.5
    tree[3] = 3.0
    for (s, e), want in [((0, 0), 0.5), ((0, 2), 1.0), ((0, 3), 0.5), ((0, -1), 0.5), ((2, 4), 0.5), ((3, 4), 3.0)]:
        assert np.isclose(tree.min(s, e), want)
    tree[2] = 0.7
    for (s, e), want in [((0, 0), 0.7), ((0, 2), 1.0), ((0, 3), 0.7), ((0, -1), 0.7), ((2, 4), 0.7), ((3, 4), 3.0)]:
        assert np.isclose(tree.min(s, e), want)
    tree[2] = 4.0
    for (s, e), want in [((0, 0), 1.0), ((0, 2), 1.0), ((0, 3), 1.0), ((0, -1), 1.0), ((2, 4), 3.0), ((2, 3), 4.0),
                         ((2, -1), 4.0), ((3, 4), 3.0)]:
        assert np.isclose(tree.min(s, e), want)


@pytest.mark.parametrize("cap,n", [(64, 40), (1024, 700), (4096, 3000)])
def test_segment_trees_bit_exact_vs_oracle(cap, n):
    """Random batched writes with duplicates (small one-workgroup and large
    multi-launch paths), random range reductions and retrievals."""
    from agilerl_amd.components.segment_tree import MinSegmentTree, SumSegmentTree

    rng = np.random.default_rng(cap + n)
    idx = rng.integers(0, cap, n)
    val = np.abs(rng.standard_normal(n)) ** 0.6 + 1e-5
    st, mt = SumSegmentTree(cap), MinSegmentTree(cap)
    st.set_batch(idx, val)
    mt.set_batch(idx, val)
    ost, omt = oper.SumSegmentTree(cap), oper.MinSegmentTree(cap)
    for i, v in zip(idx, val):
        ost[int(i)] = float(v)
        omt[int(i)] = float(v)
    np.testing.assert_array_equal(st.tree.cpu().numpy(), np.asarray(ost.tree))
    np.testing.assert_array_equal(mt.tree.cpu().numpy(), np.asarray(omt.tree))
    for _ in range(20):
        a, b = sorted(rng.integers(0, cap, 2))
        b = b + 1
        assert st.sum(int(a), int(b)) == ost.sum(int(a), int(b))
        assert mt.min(int(a), int(b)) == omt.min(int(a), int(b))
    total = ost.sum()
    ubs = rng.random(257) * total
    got = st.retrieve_batch(torch.as_tensor(ubs)).cpu().numpy()
    want = np.array([ost.retrieve(float(u)) for u in ubs])
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("max_size,batches,B", [(1000, [16] * 20 + [300], 64), (100, [7] * 30, 32)])
def test_prioritized_replay_buffer_matches_oracle(max_size, batches, B):
    from agilerl_amd.components.replay_buffer import PrioritizedReplayBuffer

    rng = np.random.default_rng(max_size)
    buf = PrioritizedReplayBuffer(max_size, alpha=0.6)
    ref = oper.PER(max_size, alpha=0.6)
    obs_all = []
    for n in batches:
        obs = rng.standard_normal((n, 4)).astype(np.float32)
        obs_all.append(obs)
        buf.add({"obs": obs, "reward": rng.standard_normal(n).astype(np.float32),
                 "frame": rng.integers(0, 255, (n, 3, 3), dtype=np.uint8)})
        ref.add(n)
    assert len(buf) == min(sum(batches), max_size) == ref.size
    assert buf.storage["frame"].dtype == torch.uint8 and buf.storage["reward"].shape == (max_size, 1)
    for step in range(4):
        torch.manual_seed(step)
        u = torch.rand(B).numpy()
        torch.manual_seed(step)
        s = buf.sample(B, beta=0.4 + 0.1 * step)
        want_idx = ref.sample_indices(u)
        got_idx = s["idxs"].view(-1).cpu().numpy()
        np.testing.assert_array_equal(got_idx, want_idx)
        want_w = ref.weights(want_idx, 0.4 + 0.1 * step)
        np.testing.assert_array_equal(s["weights"].view(-1).cpu().numpy(), want_w)
        assert s["obs"].shape == (B, 4)
        pri = np.abs(rng.standard_normal(B)).astype(np.float32) * (step + 1)
        pri[:3] = 0.0  # floor 1e-5
        buf.update_priorities(s["idxs"], torch.as_tensor(pri))
        ref.update_priorities(want_idx, pri)
        # leaves are p ** alpha by glibc's own pow algorithm (csrc/libm_pow.h):
        # every node bit-identical to the reference's tree
        np.testing.assert_array_equal(buf.sum_tree.tree.cpu().numpy(), np.asarray(ref.sum_tree.tree))
        np.testing.assert_array_equal(buf.min_tree.tree.cpu().numpy(), np.asarray(ref.min_tree.tree))
        assert buf.max_priority == ref.max_priority


def test_replay_buffer_circular_and_uniform_sample():
    from agilerl_amd.components.replay_buffer import ReplayBuffer

    buf = ReplayBuffer(10)
    for k in range(4):
        buf.add({"x": np.arange(3 * k, 3 * k + 3, dtype=np.float32)})
    assert len(buf) == 10 and buf.is_full and buf.counter == 12
    x = buf.storage["x"].view(-1).cpu().numpy()
    np.testing.assert_array_equal(x, [10, 11, 2, 3, 4, 5, 6, 7, 8, 9])
    torch.manual_seed(3)
    want = torch.randperm(10)[:5]
    torch.manual_seed(3)
    s = buf.sample(5, return_idx=True)
    np.testing.assert_array_equal(s["idxs"].cpu().numpy(), want.numpy())
    np.testing.assert_array_equal(s["x"].view(-1).cpu().numpy(), x[want.numpy()])


@pytest.mark.parametrize("use_gae", [True, False])
def test_rollout_buffer_gae_bit_exact(use_gae):
    from agilerl_amd.components.rollout_buffer import RolloutBuffer
    from agilerl_amd.envs import Box, Discrete

    T, N = 24, 7
    rng = np.random.default_rng(1)
    buf = RolloutBuffer(T, Box(-1, 1, (5,)), Discrete(3), num_envs=N, use_gae=use_gae)
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = rng.random((T, N)) < 0.1
    for t in range(T - 4):  # partially filled buffer: GAE over the prefix
        buf.add(rng.standard_normal((N, 5)).astype(np.float32), rng.integers(0, 3, N), r[t], d[t], v[t],
                rng.standard_normal(N).astype(np.float32))
    assert buf.size() == (T - 4) * N
    lv = rng.standard_normal(N).astype(np.float32)
    ld = rng.random(N) < 0.2
    buf.compute_returns_and_advantages(torch.as_tensor(lv), torch.as_tensor(ld))
    adv, ret = ogae.gae(r[:T - 4], v[:T - 4], d[:T - 4], lv, ld, 0.99, 0.95, use_gae)
    np.testing.assert_array_equal(buf.buffer["advantages"][:T - 4].cpu().numpy(), adv)
    np.testing.assert_array_equal(buf.buffer["returns"][:T - 4].cpu().numpy(), ret)
    batch = buf.get_tensor_batch()
    assert batch["observations"].shape == ((T - 4) * N, 5) and batch["actions"].shape == ((T - 4) * N, 1)
    for _ in range(4):
        buf.add(np.zeros((N, 5)), np.zeros(N), r[0], d[0], v[0], r[0])
    with pytest.raises(ValueError):
        buf.add(np.zeros((N, 5)), np.zeros(N), r[0], d[0], v[0], r[0])


def test_multistep_replay_buffer_matches_oracle():
    from agilerl_amd.components.replay_buffer import MultiStepReplayBuffer
    from oracle import dqn as odqn

    rng = np.random.default_rng(4)
    n, N = 3, 5
    buf = MultiStepReplayBuffer(50, n_step=n, gamma=0.9)
    hist = []
    for t in range(12):
        tr = {"obs": rng.standard_normal((N, 2)).astype(np.float32),
              "action": rng.integers(0, 3, (N, 1)),
              "reward": rng.standard_normal((N, 1)).astype(np.float32),
              "next_obs": rng.standard_normal((N, 2)).astype(np.float32),
              "done": (rng.random((N, 1)) < 0.15).astype(np.float32)}
        hist.append(tr)
        out = buf.add(tr)
        assert (out is None) == (t < n - 1)
    assert len(buf) == (12 - n + 1) * N
    for k in range(12 - n + 1):
        want = odqn.nstep_fold(hist[k:k + n], 0.9)
        for key in ("obs", "reward", "next_obs", "done"):
            got = buf.storage[key][k * N:(k + 1) * N].cpu().numpy()
            np.testing.assert_array_equal(got, want[key].reshape(got.shape))


@pytest.mark.parametrize("case", ["nstep0", "nstep1", "nstep2", "nstep3"])
def test_multistep_fold_matches_reference_golden(golden, case):
    """MultiStepReplayBuffer's device n-step fold against the reference's
    own _get_n_step_info output (replay_buffer.py:206-258), bit for bit."""
    from agilerl_amd.components.replay_buffer import MultiStepReplayBuffer

    g = golden(case)
    n = int(g["n_step"])
    dkey = str(g["done_key"])
    buf = MultiStepReplayBuffer(64, n_step=n, gamma=float(g["gamma"]))
    for i in range(n):
        tr = {f: g[f"in{i}.{f}"] for f in ("obs", "reward", "next_obs")}
        tr[dkey] = g[f"in{i}.done"]
        buf.add(tr)
    B = g["in0.obs"].shape[0]
    assert len(buf) == B
    for f, key in (("obs", "obs"), ("reward", "reward"), ("next_obs", "next_obs"), ("done", dkey)):
        got = buf.storage[key][:B].cpu().numpy()
        np.testing.assert_array_equal(got, g[f"out.{f}"].reshape(got.shape), err_msg=f)
