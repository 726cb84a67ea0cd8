"""The population-batched Rainbow learner (algorithms/rainbow_pop.py) against
each agent's own ``RainbowDQN.learn`` (itself checked against the reference's
loss on a plain-PyTorch twin, test_dropin_gpu.py) — per agent: loss, online
and target parameters, Adam moments, new priorities and the noise drawn
after the update."""

import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _agents(P, obs_space, act_space, **kw):
    from agilerl_amd.algorithms import RainbowDQN

    out = []
    for p in range(P):
        torch.manual_seed(100 + p)
        out.append(RainbowDQN(obs_space, act_space, **kw))
    return out


def _batch(rng, B, obs_shape, n_act, u8=False, per=True):
    def obs():
        if u8:
            return rng.integers(0, 256, (B, *obs_shape), dtype=np.uint8)
        return rng.standard_normal((B, *obs_shape)).astype(np.float32)

    e = {"obs": obs(), "action": rng.integers(0, n_act, (B, 1)), "reward": rng.standard_normal((B, 1)).astype(
        np.float32), "next_obs": obs(), "done": (rng.random((B, 1)) < 0.2).astype(np.float32)}
    if per:
        e["weights"] = rng.random((B, 1)).astype(np.float32)
        e["idxs"] = np.arange(B).reshape(B, 1)
    return e


def _check(agents, refs, outs, ref_outs, rtol=1e-4, atol=5e-5):
    for p, (a, r) in enumerate(zip(agents, refs)):
        (l1, i1, pr1), (l2, i2, pr2) = outs[p], ref_outs[p]
        assert abs(l1 - l2) <= 1e-5 * abs(l2) + 1e-7, (p, l1, l2)
        if pr2 is not None:
            np.testing.assert_allclose(pr1, pr2, rtol=1e-5, atol=1e-7)
        for (k, x), y in zip(a.actor.named_parameters(), r.actor.parameters()):
            torch.testing.assert_close(x, y, rtol=rtol, atol=atol, msg=lambda m: f"agent {p} {k}: {m}")
        for (k, x), y in zip(a.actor_target.named_parameters(), r.actor_target.parameters()):
            torch.testing.assert_close(x, y, rtol=rtol, atol=atol, msg=lambda m: f"agent {p} target {k}: {m}")
        for (k, x), y in zip(a.actor.named_buffers(), r.actor.buffers()):
            assert torch.equal(x, y), (p, k)  # the same noise draws, in agent order
        for x, y in zip(a.actor.parameters(), r.actor.parameters()):
            sa, sr = a.optimizer.state[x], r.optimizer.state[y]
            torch.testing.assert_close(sa["exp_avg"], sr["exp_avg"], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("per", [True, False])
def test_population_learn_equals_per_agent_learn_mlp(per):
    from agilerl_amd.algorithms.rainbow_pop import RainbowPopulationLearner
    from agilerl_amd.envs import Box, Discrete

    obs_space, act_space = Box(-np.inf, np.inf, (6,)), Discrete(4)
    agents = _agents(3, obs_space, act_space, batch_size=32, lr=1e-3, gamma=0.99, tau=0.01, v_min=-10, v_max=10)
    for i, a in enumerate(agents):
        a.lr = 1e-3 * (i + 1)  # per-agent learning rates
        for g in a.optimizer.param_groups:
            g["lr"] = a.lr
    refs = [copy.deepcopy(a) for a in agents]
    learner = RainbowPopulationLearner(agents)
    rng = np.random.default_rng(7)
    for it in range(3):  # three updates: continued Adam state and noise
        exps = [_batch(rng, 32, (6,), 4, per=per) for _ in agents]
        torch.cuda.manual_seed(it)
        ref_outs = [r.learn(e, per=per) for r, e in zip(refs, exps)]
        torch.cuda.manual_seed(it)
        outs = learner.learn(exps, per=per)
        _check(agents, refs, outs, ref_outs)
    learner.sync_optimizers()
    for a, r in zip(agents, refs):
        for x, y in zip(a.actor.parameters(), r.actor.parameters()):
            assert int(a.optimizer.state[x]["step"]) == int(r.optimizer.state[y]["step"]) == 3
    acts = agents[1].get_action(exps[1]["obs"], training=False)
    assert acts.shape == (32,)


def test_population_learn_equals_per_agent_learn_atari_cnn():
    """Config-3 network (CNN 32/64/128 on 4 x 84 x 84 uint8 frames, latent 256,
    dueling noisy head [256], 6 actions, 51 atoms on +-200), n-step with
    combined reward and PER."""
    from agilerl_amd.algorithms.rainbow_pop import RainbowPopulationLearner
    from agilerl_amd.envs import Box, Discrete

    obs_space, act_space = Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6)
    net = {"encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
           "head_config": {"hidden_size": [256]}, "latent_dim": 256, "min_latent_dim": 128, "max_latent_dim": 512}
    agents = _agents(2, obs_space, act_space, net_config=net, batch_size=16, lr=1e-4, gamma=0.99, tau=1e-3,
                     v_min=-200, v_max=200, combined_reward=True, n_step=3)
    refs = [copy.deepcopy(a) for a in agents]
    learner = RainbowPopulationLearner(agents)
    rng = np.random.default_rng(8)
    for it in range(2):
        exps = [_batch(rng, 16, (4, 84, 84), 6, u8=True) for _ in agents]
        nexps = [_batch(rng, 16, (4, 84, 84), 6, u8=True, per=False) for _ in agents]
        torch.cuda.manual_seed(10 + it)
        ref_outs = [r.learn(e, n, per=True) for r, e, n in zip(refs, exps, nexps)]
        torch.cuda.manual_seed(10 + it)
        outs = learner.learn(exps, nexps, per=True)
        _check(agents, refs, outs, ref_outs, rtol=2e-4, atol=1e-4)


@pytest.mark.parametrize("double", [False, True])
def test_population_learn_equals_per_agent_learn_dqn(double):
    """DQN agents (dqn.py:274-348) through the same batched chain: TD target +
    MSE per agent, Adam without clipping, one Polyak launch."""
    from agilerl_amd.algorithms import DQN
    from agilerl_amd.algorithms.rainbow_pop import RainbowPopulationLearner
    from agilerl_amd.envs import Box, Discrete

    obs_space, act_space = Box(-np.inf, np.inf, (4,)), Discrete(2)
    agents = []
    for p in range(3):
        torch.manual_seed(200 + p)
        agents.append(DQN(obs_space, act_space, batch_size=16, lr=1e-3 * (p + 1), gamma=0.99, tau=0.01,
                          double=double))
    refs = [copy.deepcopy(a) for a in agents]
    learner = RainbowPopulationLearner(agents)
    rng = np.random.default_rng(3)
    for _ in range(3):
        exps = [_batch(rng, 16, (4,), 2, per=False) for _ in agents]
        ref_l = [r.learn(e) for r, e in zip(refs, exps)]
        got_l = learner.learn(exps)
        for p, (a, r) in enumerate(zip(agents, refs)):
            assert abs(got_l[p] - ref_l[p]) <= 1e-5 * abs(ref_l[p]) + 1e-7, (p, got_l[p], ref_l[p])
            for (k, x), y in zip(a.actor.named_parameters(), r.actor.parameters()):
                torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5, msg=lambda m: f"agent {p} {k}: {m}")
            for x, y in zip(a.actor_target.parameters(), r.actor_target.parameters()):
                torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5)
