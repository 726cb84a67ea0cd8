"""Pins the off-policy oracles to reference-run fixtures
(tests/golden/gen_golden.py):
  * oracle/dqn.py nstep_fold == MultiStepReplayBuffer._get_n_step_info
    (replay_buffer.py:206-258), bit for bit;
  * oracle/maddpg.py DequeReplay == MultiAgentReplayBuffer save / sample
    under the same Python ``random`` seed (multi_agent_replay_buffer.py:
    155-167), bit for bit;
  * oracle/maddpg.py critic_target == MADDPG._learn_individual's TD target,
    loss and dL/dQ (maddpg.py:764-790)."""

import random

import numpy as np
import pytest

from oracle import dqn as odqn
from oracle import maddpg as omaddpg


@pytest.mark.parametrize("case", ["nstep0", "nstep1", "nstep2", "nstep3"])
def test_nstep_fold_matches_reference(golden, case):
    g = golden(case)
    n = int(g["n_step"])
    trs = [{f: g[f"in{i}.{f}"] for f in ("obs", "reward", "next_obs", "done")} for i in range(n)]
    got = odqn.nstep_fold(trs, float(g["gamma"]))
    for f in ("obs", "reward", "next_obs", "done"):
        assert np.array_equal(np.asarray(got[f], np.float32), g[f"out.{f}"]), f


FIELDS = ["obs", "action", "reward", "next_obs", "done"]
AGENTS = ["speaker_0", "listener_0"]


@pytest.mark.parametrize("case", ["marep0", "marep1"])
def test_multi_agent_replay_matches_reference(golden, case):
    g = golden(case)
    ref = omaddpg.DequeReplay(int(g["memory_size"]), FIELDS, AGENTS)
    for t in range(int(g["steps"])):
        args = [{a: g[f"save{t}.{f}.{a}"] for a in AGENTS} for f in FIELDS]
        ref.save(*args, is_vectorised=True)
    for s in range(3):
        random.seed(100 * int(g["seed"]) + s)
        sample = ref.sample(int(g["batch"]))
        for f, per in zip(FIELDS, sample):
            for a in AGENTS:
                want = g[f"sample{s}.{f}.{a}"]
                assert np.array_equal(per[a], want, equal_nan=True), (s, f, a)


@pytest.mark.parametrize("case", ["maddpg0", "maddpg1", "maddpg2"])
def test_maddpg_critic_target_matches_reference(golden, case):
    g = golden(case)
    y, grad, loss = omaddpg.critic_target(g["q"], g["q_next"], g["r"], g["d"], float(g["gamma"]))
    assert np.array_equal(y, g["y"].reshape(-1))
    np.testing.assert_allclose(grad, g["g_q"].reshape(-1), rtol=1e-6, atol=1e-9)
    assert abs(float(loss) - float(g["critic_loss"])) <= 1e-6 * abs(float(g["critic_loss"]))
