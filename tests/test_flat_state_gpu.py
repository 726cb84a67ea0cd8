"""The per-agent DQN / RainbowDQN update tail over flat buffers
(algorithms/flat_state.py: gradient gather, agx_clip_adam, one agx_polyak)
against the torch tail it replaces (clip_grad_norm_, torch.optim.Adam,
per-tensor Polyak) on identical agents; the flat state across clone,
checkpoint round trip and learning-rate mutation; and agx_noisy_reset
against NoisyLinear's torch ops (custom_components.py:116-131), bit for bit."""

import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(rng, B, obs_dim, n_act, per=True):
    e = {"obs": rng.standard_normal((B, obs_dim)).astype(np.float32), "action": rng.integers(0, n_act, (B, 1)),
         "reward": rng.standard_normal((B, 1)).astype(np.float32),
         "next_obs": rng.standard_normal((B, obs_dim)).astype(np.float32),
         "done": (rng.random((B, 1)) < 0.2).astype(np.float32)}
    if per:
        e["weights"] = rng.random((B, 1)).astype(np.float32)
        e["idxs"] = np.arange(B).reshape(B, 1)
    return e


def _torch_tail(monkeypatch):
    """Route learn() through the torch optimizer tail (no flat state)."""
    from agilerl_amd.algorithms import dqn

    monkeypatch.setattr(dqn, "flat_state", lambda agent: None)


@pytest.mark.parametrize("sizes", [[(5, 7)], [(64, 64), (64, 4), (512, 512), (1, 1)],
                                   [(3 + i, 2 * i + 1) for i in range(19)]])
def test_noisy_reset_bit_exact(sizes):
    from agilerl_amd.modules.custom_components import NoisyLinear, reset_noise_layers

    layers = [NoisyLinear(i, o, device="cuda") for i, o in sizes]
    torch.cuda.manual_seed(123)
    reset_noise_layers(layers)
    got = [(m.weight_epsilon.clone(), m.bias_epsilon.clone()) for m in layers]
    torch.cuda.manual_seed(123)
    for m, (w, b) in zip(layers, got):  # the reference's ops (custom_components.py:116-131)
        x_in = torch.randn(m.in_features, device="cuda")
        x_out = torch.randn(m.out_features, device="cuda")
        e_in, e_out = x_in.sign().mul_(x_in.abs().sqrt_()), x_out.sign().mul_(x_out.abs().sqrt_())
        assert torch.equal(w, e_out.ger(e_in)) and torch.equal(b, e_out)


@pytest.mark.parametrize("per", [True, False])
def test_rainbow_flat_tail_matches_torch_tail(per, monkeypatch):
    from agilerl_amd.algorithms import RainbowDQN
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(5)
    a = RainbowDQN(Box(-np.inf, np.inf, (6,)), Discrete(4), batch_size=32, lr=1e-3, gamma=0.99, tau=0.01,
                   v_min=-10, v_max=10)
    r = copy.deepcopy(a)
    rng = np.random.default_rng(1)
    for it in range(4):
        e = _batch(rng, 32, 6, 4, per=per)
        e["reward"] *= 50.0  # gradient norms above 10: the clip is exercised
        torch.cuda.manual_seed(it)
        l1, _, p1 = a.learn(e, per=per)
        with monkeypatch.context() as mp:
            _torch_tail(mp)
            torch.cuda.manual_seed(it)
            l2, _, p2 = r.learn(e, per=per)
        assert abs(l1 - l2) <= 1e-5 * abs(l2) + 1e-7, (it, l1, l2)
        if per:
            np.testing.assert_allclose(p1, p2, rtol=1e-5, atol=1e-7)
    assert a.__dict__.get("_flat") is not None and r.__dict__.get("_flat") is None
    for (k, x), y in zip(a.actor.named_parameters(), r.actor.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5, msg=lambda m: f"{k}: {m}")
        sa, sr = a.optimizer.state[x], r.optimizer.state[y]
        torch.testing.assert_close(sa["exp_avg"], sr["exp_avg"], rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(sa["exp_avg_sq"], sr["exp_avg_sq"], rtol=1e-4, atol=1e-9)
        assert int(sa["step"]) == int(sr["step"]) == 4
    for x, y in zip(a.actor_target.parameters(), r.actor_target.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5)
    for x, y in zip(a.actor.buffers(), r.actor.buffers()):
        assert torch.equal(x, y)  # the same noise draws


def test_dqn_flat_tail_matches_torch_tail(monkeypatch):
    from agilerl_amd.algorithms import DQN
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(6)
    a = DQN(Box(-np.inf, np.inf, (4,)), Discrete(2), batch_size=16, lr=1e-3, gamma=0.99, tau=0.01, double=True)
    r = copy.deepcopy(a)
    rng = np.random.default_rng(2)
    for _ in range(3):
        e = _batch(rng, 16, 4, 2, per=False)
        l1 = a.learn(e)
        with monkeypatch.context() as mp:
            _torch_tail(mp)
            l2 = r.learn(e)
        assert abs(l1 - l2) <= 1e-5 * abs(l2) + 1e-7
    for x, y in zip(a.actor.parameters(), r.actor.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5)
        assert int(a.optimizer.state[x]["step"]) == int(r.optimizer.state[y]["step"]) == 3
    for x, y in zip(a.actor_target.parameters(), r.actor_target.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5)


def test_flat_state_across_clone_checkpoint_and_lr_change(tmp_path, monkeypatch):
    """A torch optimizer step taken outside learn is followed; a clone
    continues from its parent's Adam state; a checkpoint carries the
    current moments and step count; a mutated learning rate takes effect on
    the next update — each matching the torch tail on a twin."""
    from agilerl_amd.algorithms import RainbowDQN
    from agilerl_amd.envs import Box, Discrete

    obs_space, act_space = Box(-np.inf, np.inf, (6,)), Discrete(4)
    torch.manual_seed(9)
    a = RainbowDQN(obs_space, act_space, batch_size=32, lr=1e-3, gamma=0.99, tau=0.01, v_min=-10, v_max=10)
    r = copy.deepcopy(a)
    rng = np.random.default_rng(4)

    def both(x, y, seed):
        e = _batch(rng, 32, 6, 4)
        torch.cuda.manual_seed(seed)
        x.learn(e, per=True)
        with monkeypatch.context() as mp:
            _torch_tail(mp)
            torch.cuda.manual_seed(seed)
            y.learn(e, per=True)

    both(a, r, 0)
    for x in (a, r):  # a torch optimizer step outside learn (zero gradients): the flat state follows it
        x.optimizer.zero_grad(set_to_none=False)
        x.optimizer.step()
    both(a, r, 1)
    c, rc = a.clone(index=3), r.clone(index=3)
    both(c, rc, 2)
    assert int(c.optimizer.state[next(c.actor.parameters())]["step"]) == 4
    assert int(a.optimizer.state[next(a.actor.parameters())]["step"]) == 3  # the parent untouched
    for g in c.optimizer.param_groups:  # a learning-rate mutation
        g["lr"] = 3e-4
    for g in rc.optimizer.param_groups:
        g["lr"] = 3e-4
    both(c, rc, 3)
    path = str(tmp_path / "c.pt")
    c.save_checkpoint(path)
    d = RainbowDQN(obs_space, act_space, batch_size=32, lr=1e-3, gamma=0.99, tau=0.01, v_min=-10, v_max=10)
    d.load_checkpoint(path)
    for x, y in zip(d.actor.parameters(), c.actor.parameters()):
        assert torch.equal(x, y)
        assert int(d.optimizer.state[x]["step"]) == 5
        assert torch.equal(d.optimizer.state[x]["exp_avg"], c.optimizer.state[y]["exp_avg"])
    both(d, rc, 4)
    for x, y in zip(d.actor.parameters(), rc.actor.parameters()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=5e-5)
        assert int(d.optimizer.state[x]["step"]) == int(rc.optimizer.state[y]["step"]) == 6


@pytest.mark.parametrize("per,n_step", [(True, True), (False, False)])
def test_rainbow_cnn_update_replayed_from_graph_equals_eager(per, n_step, monkeypatch):
    """The config-3 network (uint8 84x84x4 frames, CNN 32/64/128, dueling noisy
    heads): updates replayed from the captured graph (learn_graph.py) equal the
    eager updates of a twin agent bit for bit — losses, priorities,
    parameters, Adam moments and step counts, target parameters and the noise
    buffers — across a learning-rate mutation and a torch optimizer step
    taken outside learn (both applied around the replay)."""
    from agilerl_amd.algorithms import RainbowDQN, learn_graph
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(3)
    net = {"latent_dim": 64, "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3],
                                                "stride_size": [4, 2, 1]}, "head_config": {"hidden_size": [64]}}
    a = RainbowDQN(Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6), batch_size=16, lr=1e-4, gamma=0.99,
                   tau=1e-3, v_min=-10, v_max=10, n_step=3, net_config=net)
    r = copy.deepcopy(a)
    rng = np.random.default_rng(8)
    B = 16

    def batch():
        e = {"obs": torch.as_tensor(rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8), device="cuda"),
             "action": torch.as_tensor(rng.integers(0, 6, (B, 1)), device="cuda"),
             "reward": torch.as_tensor(rng.standard_normal((B, 1)).astype(np.float32), device="cuda"),
             "next_obs": torch.as_tensor(rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8), device="cuda"),
             "done": torch.as_tensor((rng.random((B, 1)) < 0.2).astype(np.float32), device="cuda")}
        if per:
            e["weights"] = torch.as_tensor(rng.random((B, 1)).astype(np.float32), device="cuda")
        e["idxs"] = np.arange(B)
        return e

    for it in range(5):
        e, ne = batch(), (batch() if n_step else None)
        if it == 3:  # a learning-rate mutation and a torch step outside learn
            for x in (a, r):
                for g in x.optimizer.param_groups:
                    g["lr"] = 3e-4
                x.optimizer.zero_grad(set_to_none=False)
                x.optimizer.step()
        torch.cuda.manual_seed(100 + it)
        l1, _, p1 = a.learn(e, ne, per=per)
        with monkeypatch.context() as mp:
            mp.setenv("AGX_LEARN_GRAPH", "0")
            torch.cuda.manual_seed(100 + it)
            l2, _, p2 = r.learn(e, ne, per=per)
        assert l1 == l2, (it, l1, l2)
        if per:
            np.testing.assert_array_equal(p1, p2)
    fs = a.__dict__["_flat"]
    assert any(ent.graph is not None for ent in learn_graph._GRAPHS.get(fs, {}).values())  # replayed
    for (k, x), y in zip(a.actor.named_parameters(), r.actor.parameters()):
        assert torch.equal(x, y), k
        assert torch.equal(x.grad, y.grad), k
        sa, sr = a.optimizer.state[x], r.optimizer.state[y]
        assert torch.equal(sa["exp_avg"], sr["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sr["exp_avg_sq"]), k
        assert int(sa["step"]) == int(sr["step"]) == 6
    for x, y in zip(a.actor_target.parameters(), r.actor_target.parameters()):
        assert torch.equal(x, y)
    for x, y in zip(list(a.actor.buffers()) + list(a.actor_target.buffers()),
                    list(r.actor.buffers()) + list(r.actor_target.buffers())):
        assert torch.equal(x, y)  # the same noise draws
