"""MultiAgentReplayBuffer host logic against the deque restatement
(oracle/maddpg.py, following multi_agent_replay_buffer.py:16-300): identical
samples under the same Python ``random`` seed — single and vectorised saves,
ring wrap-around, binary fields with and without NaN.  Storage on the CPU
here; tests/test_maddpg_gpu.py repeats it in HBM."""

import random

import numpy as np
import pytest

from oracle.maddpg import DequeReplay

FIELDS = ["obs", "action", "reward", "next_obs", "done"]
AGENTS = ["speaker_0", "listener_0"]
DIMS = {"speaker_0": (3, 3), "listener_0": (11, 5)}


def _step(rng, n, nan=False):
    obs = {a: rng.standard_normal((n, DIMS[a][0])).astype(np.float32) for a in AGENTS}
    act = {a: rng.random((n, DIMS[a][1])).astype(np.float32) for a in AGENTS}
    rew = {a: rng.standard_normal(n).astype(np.float32) for a in AGENTS}
    nxt = {a: rng.standard_normal((n, DIMS[a][0])).astype(np.float32) for a in AGENTS}
    done = {a: (rng.random(n) < 0.3) for a in AGENTS}
    if nan:
        rew["listener_0"][0] = np.nan
        done["listener_0"] = done["listener_0"].astype(np.float32)
        done["listener_0"][0] = np.nan
    return obs, act, rew, nxt, done


def check_against_oracle(device, memory_size=50, steps=23, n_envs=4, batch=16, seed=3):
    from agilerl_amd.components import MultiAgentReplayBuffer

    rng = np.random.default_rng(seed)
    buf = MultiAgentReplayBuffer(memory_size, FIELDS, AGENTS, device=device)
    ref = DequeReplay(memory_size, FIELDS, AGENTS)
    for t in range(steps):
        tr = _step(rng, n_envs, nan=(t == steps - 1))
        buf.save_to_memory(*tr, is_vectorised=True)
        ref.save(*tr, is_vectorised=True)
        assert len(buf) == len(ref.memory)
        if len(buf) >= batch and t % 3 == 0:
            random.seed(100 + t)
            got = buf.sample(batch)
            random.seed(100 + t)
            exp = ref.sample(batch)
            for f, (g, e) in enumerate(zip(got, exp)):
                for a in AGENTS:
                    gg = g[a].cpu().numpy()
                    assert gg.dtype == np.float32 and gg.shape == e[a].shape, (FIELDS[f], a)
                    np.testing.assert_array_equal(gg, e[a], err_msg=f"{FIELDS[f]}/{a}")
    return buf


def test_vectorised_wraparound_cpu():
    buf = check_against_oracle("cpu")
    assert buf.counter == 23 * 4 and len(buf) == 50


def test_single_env_saves_cpu():
    from agilerl_amd.components import MultiAgentReplayBuffer

    rng = np.random.default_rng(0)
    buf = MultiAgentReplayBuffer(7, FIELDS, AGENTS, device="cpu")
    ref = DequeReplay(7, FIELDS, AGENTS)
    for _ in range(11):
        tr = [{a: v[0] for a, v in f.items()} for f in _step(rng, 1)]
        buf.save_to_memory(*tr)
        ref.save(*tr)
    random.seed(5)
    got = buf.sample(5)
    random.seed(5)
    exp = ref.sample(5)
    for g, e in zip(got, exp):
        for a in AGENTS:
            np.testing.assert_array_equal(g[a].numpy(), e[a])
    assert got[2]["speaker_0"].shape == (5, 1)  # scalar rewards come back (B, 1)


def test_assertions():
    from agilerl_amd.components import MultiAgentReplayBuffer

    with pytest.raises(AssertionError):
        MultiAgentReplayBuffer(0, FIELDS, AGENTS, device="cpu")
    with pytest.raises(AssertionError):
        MultiAgentReplayBuffer(10, [], AGENTS, device="cpu")


def test_critic_target_oracle_nan_rules():
    from oracle.maddpg import critic_target

    q = np.array([1.0, 2.0, 0.5, -1.0], np.float32)
    qn = np.array([3.0, 4.0, 5.0, 6.0], np.float32)
    r = np.array([0.5, np.nan, 1.0, 2.0], np.float32)
    d = np.array([0.0, 0.0, np.nan, 1.0], np.float32)
    y, g, loss = critic_target(q, qn, r, d, 0.95)
    np.testing.assert_array_equal(y, np.array([0.5 + np.float32(0.95) * 3.0, np.float32(0.95) * np.float32(4.0),
                                               1.0, 2.0], np.float32))
    assert np.isclose(loss, np.mean((q - y) ** 2)) and np.allclose(g, 2 * (q - y) / 4)
