"""agx_noisy_streams_forward / _backward (csrc/noisy_mlp.hip): Rainbow's
dueling head streams (create_mlp stacks NoisyLinear -> LayerNorm -> ReLU ...
-> NoisyLinear, agilerl/modules/mlp.py; DuelingDistributionalMLP,
agilerl/networks/custom_modules.py:20-162) against the same torch modules in
float64 — outputs, every parameter gradient (d mu, d sigma, LayerNorm affine)
and the latent's gradient — plus determinism, the structures that fall back
to the torch modules, and the head's selected-row log-probabilities with and
without the fused streams."""

import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _streams(latent, hidden, out_v, out_a, noisy=True, seed=0):
    from agilerl_amd.modules.mlp import create_mlp

    torch.manual_seed(seed)
    kw = dict(output_vanish=True, noisy=noisy, init_layers=False, layer_norm=True, noise_std=0.5, device=DEV)
    v = create_mlp(latent, out_v, hidden, name="value", **kw)
    a = create_mlp(latent, out_a, hidden, name="advantage", **kw)
    with torch.no_grad():  # LayerNorm affine away from identity: its gradients are exercised
        for m in list(v.modules()) + list(a.modules()):
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    return v, a


def _row_margins(streams, x):
    """Per row: the smallest |LayerNorm output| of every hidden layer of the
    reference (its distance from the ReLU kink)."""
    ys = []
    hooks = [m.register_forward_hook(lambda mod, i, o: ys.append(o.detach().abs().amin(1)))
             for s in streams for m in s.modules() if isinstance(m, torch.nn.LayerNorm)]
    with torch.no_grad():
        for s in streams:
            s(x)
    for h in hooks:
        h.remove()
    return torch.stack(ys).amin(0) if ys else torch.full((x.shape[0],), float("inf"), device=x.device)


def _inputs(streams, B, latent, g, margin=2e-4):
    """B latent rows whose hidden activations all stay away from the ReLU
    kink by more than the fp32 rounding of the two paths (otherwise a gate
    could legitimately differ between them): rows drawn and kept if so."""
    rows = []
    n = 0
    while n < B:
        cand = torch.randn(2 * B + 16, latent, device=DEV, generator=g)
        ok = _row_margins(streams, cand.double()) > margin
        rows.append(cand[ok])
        n += int(ok.sum())
    return torch.cat(rows)[:B].contiguous()


def _scale(t):
    return max(float(t.detach().abs().max()), 1e-30)


def _check(ours, ref, tol, what):
    err = float((ours.detach().double() - ref.detach().double()).abs().max())
    assert err <= tol * _scale(ref), f"{what}: max err {err:.3e} vs scale {_scale(ref):.3e}"


def _run_case(latent, hidden, out_v, out_a, B, noisy=True, train=True, seed=0):
    from agilerl_amd.modules.noisy_streams import head_streams

    v, a = _streams(latent, hidden, out_v, out_a, noisy=noisy, seed=seed)
    v.train(train)
    a.train(train)
    g = torch.Generator(device=DEV).manual_seed(1000 + seed)
    vd, ad = copy.deepcopy(v).double(), copy.deepcopy(a).double()
    x = _inputs([vd, ad], B, latent, g)
    gv = torch.randn(B, out_v, device=DEV, generator=g)
    ga = torch.randn(B, out_a, device=DEV, generator=g)

    xo = x.clone().requires_grad_(True)
    out = head_streams([v, a], xo)
    assert out is not None, "the fused streams did not take the stack"
    vo, ao = out
    ((vo * gv).sum() + (ao * ga).sum()).backward()

    xr = x.double().requires_grad_(True)
    vr, ar = vd(xr), ad(xr)
    ((vr * gv.double()).sum() + (ar * ga.double()).sum()).backward()

    _check(vo, vr, 2e-5, "value stream output")
    _check(ao, ar, 2e-5, "advantage stream output")
    _check(xo.grad, xr.grad, 5e-5, "d latent")
    for (n, p), q in zip(list(v.named_parameters()) + list(a.named_parameters()),
                         list(vd.parameters()) + list(ad.parameters())):
        if q.grad is None:
            assert p.grad is None, n
            continue
        assert p.grad is not None, n
        _check(p.grad, q.grad, 5e-5, n)
    return v, a, x, gv, ga


def test_config3_head_shape():
    """latent 256, head [256], A = 6, Z = 51, B = 64 (bench config 3)."""
    _run_case(256, [256], 51, 6 * 51, 64)


def test_ragged_two_hidden_layers():
    """Sizes that are not multiples of the 16-wide tiles, fewer rows than a tile."""
    _run_case(72, [37, 20], 11, 33, 5, seed=1)


def test_eval_mode_uses_mu():
    """NoisyLinear in eval mode: weight_mu / bias_mu only (custom_components.py:124-131)."""
    _run_case(64, [64], 51, 102, 64, train=False, seed=2)


def test_large_batch_and_plain_linear():
    _run_case(128, [128], 51, 153, 1000, seed=3)
    _run_case(48, [64], 7, 21, 33, noisy=False, seed=4)


def test_three_hidden_layers():
    _run_case(96, [80, 64, 48], 13, 26, 40, seed=5)


def test_deterministic_bits():
    from agilerl_amd.modules.noisy_streams import head_streams

    v, a = _streams(256, [256], 51, 306, seed=6)
    x = torch.randn(64, 256, device=DEV)
    res = []
    for _ in range(2):
        for p in list(v.parameters()) + list(a.parameters()):
            p.grad = None
        xo = x.clone().requires_grad_(True)
        vo, ao = head_streams([v, a], xo)
        (vo.square().sum() + ao.sin().sum()).backward()
        res.append([vo.detach().clone(), ao.detach().clone(), xo.grad.clone()] +
                   [p.grad.clone() for p in list(v.parameters()) + list(a.parameters())])
    for t1, t2 in zip(*res):
        assert torch.equal(t1, t2)


def test_structures_outside_the_kernel_keep_torch():
    from agilerl_amd.modules.mlp import create_mlp
    from agilerl_amd.modules.noisy_streams import head_streams

    v, a = _streams(32, [32], 5, 10)
    assert head_streams([v, a], torch.randn(1025, 32, device=DEV)) is None  # > 1024 rows
    assert head_streams([v, a], torch.randn(8, 32, device=DEV, dtype=torch.float64)) is None
    tanh = create_mlp(32, 5, [32], output_vanish=True, noisy=True, layer_norm=True, activation="Tanh", device=DEV)
    assert head_streams([tanh, a], torch.randn(8, 32, device=DEV)) is None
    no_ln = create_mlp(32, 5, [32], output_vanish=True, noisy=True, layer_norm=False, device=DEV)
    assert head_streams([no_ln], torch.randn(8, 32, device=DEV)) is None
    h = v[0].register_forward_hook(lambda *args: None)
    assert head_streams([v, a], torch.randn(8, 32, device=DEV)) is None  # hooks only fire in Python
    h.remove()
    assert head_streams([v, a], torch.randn(8, 32, device=DEV)) is not None
    os.environ["AGX_NOISY_STREAMS"] = "0"
    try:
        assert head_streams([v, a], torch.randn(8, 32, device=DEV)) is None
    finally:
        del os.environ["AGX_NOISY_STREAMS"]


def test_dueling_head_rows_with_and_without_fused_streams():
    """DuelingDistributionalMLP.forward(q=False, log=True, rows=a) — the
    learn path's grad-enabled head — on the fused streams vs the torch
    modules (both fp32)."""
    from agilerl_amd.networks.q_networks import DuelingDistributionalMLP

    torch.manual_seed(7)
    A, Z = 6, 51
    support = torch.linspace(-200, 200, Z, device=DEV)
    head = DuelingDistributionalMLP(256, A, [256], Z, support, device=DEV)
    twin = copy.deepcopy(head)
    x = torch.randn(64, 256, device=DEV)
    rows = torch.randint(0, A, (64,), device=DEV)
    g = torch.randn(64, Z, device=DEV)
    x1 = x.clone().requires_grad_(True)
    out = head(x1, q=False, log=True, rows=rows)
    (out * g).sum().backward()
    os.environ["AGX_NOISY_STREAMS"] = "0"
    try:
        x2 = x.clone().requires_grad_(True)
        ref = twin(x2, q=False, log=True, rows=rows)
        (ref * g).sum().backward()
        q2 = twin(x)
    finally:
        del os.environ["AGX_NOISY_STREAMS"]
    q1 = head(x)
    _check(out, ref, 1e-5, "log p rows")
    _check(q1, q2, 1e-5, "q")
    _check(x1.grad, x2.grad, 1e-4, "d latent")
    for (n, p), q in zip(head.named_parameters(), twin.parameters()):
        _check(p.grad, q.grad, 1e-4, n)


def test_rainbow_next_pair_matches_the_two_forwards():
    """RainbowDQN's no-grad forwards on s' (a* from the online network, the
    target network's distribution of a*) as one grouped launch per layer
    (dqn._next_pair) against the two separate forwards of the reference's
    _dqn_loss (dqn_rainbow.py:284-367)."""
    import numpy as np

    from agilerl_amd.algorithms import RainbowDQN
    from agilerl_amd.algorithms.dqn import _next_pair
    from agilerl_amd.algorithms.flat_state import flat_state
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(3)
    net = {"latent_dim": 256, "max_latent_dim": 512, "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3],
                                                 "stride_size": [4, 2, 1]}, "head_config": {"hidden_size": [256]}}
    agent = RainbowDQN(Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6), net_config=net, v_min=-200.0,
                       v_max=200.0)
    assert flat_state(agent) is not None
    with torch.no_grad():  # target != online
        for p in agent.actor_target.parameters():
            p.add_(0.02 * torch.randn_like(p))
    obs = torch.randint(0, 256, (64, 4, 84, 84), dtype=torch.uint8, device=DEV)
    pair = _next_pair(agent, obs)
    assert pair is not None, "the paired forward did not take the config-3 network"
    with torch.no_grad():
        a_ref = agent.actor(obs).argmax(1)
        rows_ref = agent.actor_target(obs, q=False, rows=a_ref)
    assert torch.equal(pair[0], a_ref)
    _check(pair[1], rows_ref, 1e-5, "target rows")


def test_rainbow_triple_pass_matches_the_three_forwards():
    """The update's three passes as one grouped launch per encoder layer
    (dqn._triple_pass: online on s', target on s', online on s with gradient)
    against the reference's three separate forwards: the target rows, the
    taken actions' log-probabilities and the gradient of every online
    parameter."""
    import numpy as np

    from agilerl_amd.algorithms import RainbowDQN
    from agilerl_amd.algorithms.dqn import _triple_pass
    from agilerl_amd.algorithms.flat_state import flat_state
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(4)
    net = {"latent_dim": 256, "max_latent_dim": 512, "encoder_config": {
        "channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
        "head_config": {"hidden_size": [256]}}
    agent = RainbowDQN(Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6), net_config=net, v_min=-200.0,
                       v_max=200.0)
    assert flat_state(agent) is not None
    with torch.no_grad():
        for p in agent.actor_target.parameters():
            p.add_(0.02 * torch.randn_like(p))
    obs = torch.randint(0, 256, (64, 4, 84, 84), dtype=torch.uint8, device=DEV)
    nxt = torch.randint(0, 256, (64, 4, 84, 84), dtype=torch.uint8, device=DEV)
    acts = torch.randint(0, 6, (64,), device=DEV)
    g = torch.randn(64, 51, device=DEV)
    params = list(agent.actor.parameters())

    out = _triple_pass(agent, obs, acts, nxt)
    assert out is not None, "the triple pass did not take the config-3 network"
    logp, trows = out
    grads = torch.autograd.grad((logp * g).sum(), params)

    with torch.no_grad():
        a_ref = agent.actor(nxt).argmax(1)
        trows_ref = agent.actor_target(nxt, q=False, rows=a_ref)
    logp_ref = agent.actor(obs, q=False, log=True, rows=acts)
    grads_ref = torch.autograd.grad((logp_ref * g).sum(), params)
    _check(trows, trows_ref, 1e-5, "target rows")
    _check(logp, logp_ref, 1e-5, "log p rows")
    for (n, _), a, b in zip(agent.actor.named_parameters(), grads, grads_ref):
        _check(a, b, 1e-4, n)
