"""Host-side env adapters (CPU): StackedVecEnv's vectorized step over a
lock-step stack of SyntheticVecEnv blocks returns exactly what stepping the
blocks one by one does, through time limits, a block stepped on its own, a
re-synchronised stack and a reseeded block."""

import numpy as np
import pytest

from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv


def _pair(max_steps):
    a = StackedVecEnv.from_shared(SyntheticVecEnv(16, max_episode_steps=max_steps), 4)
    b = StackedVecEnv.from_shared(SyntheticVecEnv(16, max_episode_steps=max_steps), 4)
    b._fusable = lambda: False  # the per-block path
    return a, b


@pytest.mark.parametrize("max_steps", [None, 7])
def test_fused_stack_step_matches_per_block(max_steps):
    a, b = _pair(max_steps)
    n = a.num_envs
    outs = [(np.zeros((n, 8), np.float32), np.zeros(n, np.float32), np.zeros(n, np.uint8)) for _ in range(2)]
    a.reset(out_obs=outs[0][0])
    b.reset(out_obs=outs[1][0])
    act = np.zeros(n, dtype=np.int64)
    fused_steps = 0
    for t in range(250):
        x = a.step(act, *outs[0])
        y = b.step(act, *outs[1])
        fused_steps += a._fz is not None
        for u, v in zip(outs[0], outs[1]):
            np.testing.assert_array_equal(u, v)
        np.testing.assert_array_equal(x[2], y[2])
        np.testing.assert_array_equal(x[3], y[3])
        if t == 60:  # one block stepped on its own: the stack leaves lock-step
            for s in (a, b):
                s.envs[2].step(np.zeros(16, dtype=np.int64))
        if t == 120:  # back in lock-step
            for s in (a, b):
                s.envs[2]._k = s.envs[0]._k
        if t == 180:  # a reseeded block: new episode stream
            for s in (a, b):
                s.envs[1].reseed(1234)
    assert fused_steps > 150
    for ea, eb in zip(a.envs, b.envs):
        assert ea.steps == eb.steps and ea._k == eb._k
        np.testing.assert_array_equal(ea._len, eb._len)


def test_restacked_blocks_keep_their_episode_lengths():
    """Blocks of one stack moved into another (a regroup) keep their
    time-limit counters; the first stack notices and stops using its rings."""
    a, b = _pair(5)
    act = np.zeros(a.num_envs, dtype=np.int64)
    for s in (a, b):
        s.reset()
        for _ in range(3):
            s.step(act)
    a2 = StackedVecEnv(a.envs[2:] + a.envs[:2])
    b2 = StackedVecEnv(b.envs[2:] + b.envs[:2])
    b2._fusable = lambda: False
    for _ in range(9):
        x, y = a2.step(act), b2.step(act)
        np.testing.assert_array_equal(x[3], y[3])
        np.testing.assert_array_equal(x[0], y[0])
    assert not a._fusable() or all(e._len is v for e, v in zip(a.envs, a._fz[4]))


def test_blocks_stepped_directly_in_lock_step_keep_truncations():
    """Every block stepped on its own, all together (ring positions still
    agree, so the stacked rings stay valid): the episode lengths grow in place
    and the fused step's cached length bound must follow, or it would skip the
    time-limit test and miss truncations."""
    a, b = _pair(9)
    n = a.num_envs
    act = np.zeros(n, dtype=np.int64)
    for s in (a, b):
        s.reset()
        s.step(act)
    assert a._fz is not None
    for _ in range(6):
        for s in (a, b):
            for e in s.envs:
                e.step(np.zeros(e.num_envs, dtype=np.int64))
    truncs = 0
    for _ in range(12):
        x, y = a.step(act), b.step(act)
        assert a._fz is not None  # still the fused path
        np.testing.assert_array_equal(x[2], y[2])
        np.testing.assert_array_equal(x[3], y[3])
        truncs += int(np.count_nonzero(y[3]))
    assert truncs > 0
    for ea, eb in zip(a.envs, b.envs):
        np.testing.assert_array_equal(ea._len, eb._len)
