"""a13: NoisyLinear and the Rainbow dueling distributional head against
fixtures the reference's own code produced (tests/golden/gen_golden.py
gen_dueling: agilerl/modules/custom_components.py:38-131,
agilerl/networks/custom_modules.py:127-162 on create_mlp streams).  CPU, the
same torch ops: bit-exact in the build container; torch's CPU normal draws and
GEMMs take ISA-specific vector paths (a host with other SIMD units can differ
in the last bit), so draws-derived tensors and outputs are compared within
1e-6 relative and the uniform / constant initialisations exactly."""

import numpy as np
import pytest
import torch


def test_noisy_linear_matches_reference(golden):
    from agilerl_amd.modules.custom_components import NoisyLinear

    g = golden("noisy0")
    torch.manual_seed(5)  # the reference's draw order: weight_mu, bias_mu uniforms, then eps_in, eps_out normals
    nl = NoisyLinear(12, 7, std_init=0.4)
    for k, v in nl.state_dict().items():
        if "epsilon" in k:  # normal draws
            _near(v.numpy(), g[f"init.{k}"], k)
        else:
            assert np.array_equal(v.numpy(), g[f"init.{k}"]), k
    x = torch.from_numpy(g["x"])
    _near(nl(x).detach().numpy(), g["y_train"], "train forward")
    nl.eval()
    _near(nl(x).detach().numpy(), g["y_eval"], "eval forward")
    nl.train()
    torch.manual_seed(9)
    nl.reset_noise()
    _near(nl.weight_epsilon.numpy(), g["w_eps2"], "weight_epsilon")
    _near(nl.bias_epsilon.numpy(), g["b_eps2"], "bias_epsilon")


def _near_q(a, b, what, rtol=1e-5):
    """Per element: |a - b| <= rtol * (|b| + rms(b)) — relative to each q
    value, with the population's rms as the floor near zero."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    bound = rtol * (np.abs(b) + np.sqrt(np.mean(b * b)))
    err = np.abs(a - b)
    assert np.all(err <= bound), (what, float(err.max()), float((err / bound).max()))


def _near(a, b, what, rtol=1e-6, scale=None):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = float(np.abs(a - b).max())
    scale = float(np.abs(b).max()) if scale is None else scale
    assert err <= rtol * max(1e-6, scale), (what, err)


@pytest.mark.parametrize("case", ["dueling0", "dueling1"])
def test_dueling_distributional_head_matches_reference(golden, case):
    from agilerl_amd.networks.q_networks import DuelingDistributionalMLP

    g = golden(case)
    L, A, Z = (int(v) for v in g["dims"])
    support = torch.from_numpy(g["support"])
    head = DuelingDistributionalMLP(num_inputs=L, num_outputs=A, hidden_size=[int(h) for h in g["hidden"]],
                                    num_atoms=Z, support=support, noisy=True, layer_norm=True, output_vanish=True,
                                    init_layers=False, noise_std=0.5)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    assert set(sd) == set(head.state_dict()), set(sd) ^ set(head.state_dict())
    head.load_state_dict(sd)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        _near_q(head(x).numpy(), g["q"], "q")
        _near(head(x, q=False).numpy(), g["probs"], "probs")
        _near(head(x, log=True).numpy(), g["logp"], "logp")
    # the clamp(min=1e-3) is applied after the softmax and not renormalised (custom_modules.py:158)
    assert g["probs"].min() >= 1e-3


def _torch_head(value, adv, support, A, Z, mode):
    """The reference's combine (custom_modules.py:145-162) in plain torch ops."""
    b = value.size(0)
    v = value.view(b, 1, Z)
    a = adv.view(b, A, Z)
    x = v + a - a.mean(1, keepdim=True)
    if mode == 2:
        return torch.log_softmax(x.view(-1, Z), dim=-1).view(-1, A, Z)
    x = torch.softmax(x.view(-1, Z), dim=-1).view(-1, A, Z).clamp(min=1e-3)
    return torch.sum(x * support, dim=2) if mode == 0 else x


@pytest.mark.gpu
@pytest.mark.parametrize("A,Z,B", [(6, 51, 37), (18, 51, 256), (3, 11, 5), (4, 64, 9)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_dueling_head_kernel_matches_torch(A, Z, B, mode):
    """agx_dueling_head_forward / _backward vs the reference's tensor ops
    (fp32 within 2e-6 of scale; the exp / sum orders differ)."""
    from agilerl_amd.networks.q_networks import DuelingHeadFn

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(A * 100 + Z + mode)
    value = (torch.randn(B, Z, device=dev, generator=g) * 2).requires_grad_(True)
    adv = (torch.randn(B, A * Z, device=dev, generator=g) * 2).requires_grad_(True)
    support = torch.linspace(-10, 10, Z, device=dev)
    out = DuelingHeadFn.apply(value, adv, support, A, Z, mode)
    v2, a2 = value.detach().clone().requires_grad_(True), adv.detach().clone().requires_grad_(True)
    ref = _torch_head(v2, a2, support, A, Z, mode)
    assert out.shape == ref.shape
    scale = float(ref.detach().abs().max())
    assert float((out - ref).detach().abs().max()) <= 2e-6 * scale + 1e-7
    w = torch.randn(ref.shape, device=dev, generator=g)
    (out * w).sum().backward()
    (ref * w).sum().backward()
    for got, want in ((value.grad, v2.grad), (adv.grad, a2.grad)):
        s = float(want.abs().max()) + 1e-12
        assert float((got - want).abs().max()) <= 5e-6 * s, (float((got - want).abs().max()), s)


@pytest.mark.gpu
@pytest.mark.parametrize("A,Z,B", [(6, 51, 37), (18, 51, 256), (3, 11, 5), (4, 64, 9)])
@pytest.mark.parametrize("mode", [1, 2])
def test_dueling_head_rows_equal_full_head(A, Z, B, mode):
    """agx_dueling_head_forward_rows / _backward_rows: out[range(B), rows] of
    the full HIP head bit for bit, and (log mode) the full head's gradients
    under a gradient that is zero off the selected rows, bit for bit."""
    from agilerl_amd.networks.q_networks import DuelingHeadFn, DuelingRowsFn

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(A * 7 + Z + mode)
    value = (torch.randn(B, Z, device=dev, generator=g) * 2).requires_grad_(True)
    adv = (torch.randn(B, A * Z, device=dev, generator=g) * 2).requires_grad_(True)
    rows = torch.randint(0, A, (B,), device=dev, generator=g)
    out = DuelingRowsFn.apply(value, adv, rows, A, Z, mode)
    v2, a2 = value.detach().clone().requires_grad_(True), adv.detach().clone().requires_grad_(True)
    full = DuelingHeadFn.apply(v2, a2, torch.linspace(-10, 10, Z, device=dev), A, Z, mode)
    idx = torch.arange(B, device=dev)
    assert torch.equal(out, full[idx, rows])
    if mode == 2:
        w = torch.randn(B, Z, device=dev, generator=g)
        (out * w).sum().backward()
        (full[idx, rows] * w).sum().backward()
        assert torch.equal(value.grad, v2.grad) and torch.equal(adv.grad, a2.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["dueling0", "dueling1"])
def test_dueling_head_on_gpu_matches_reference_fixture(golden, case):
    """The module on cuda (the HIP combine) against the reference-run outputs."""
    from agilerl_amd.networks.q_networks import DuelingDistributionalMLP

    g = golden(case)
    L, A, Z = (int(v) for v in g["dims"])
    dev = torch.device("cuda:0")
    support = torch.from_numpy(g["support"]).to(dev)
    head = DuelingDistributionalMLP(num_inputs=L, num_outputs=A, hidden_size=[int(h) for h in g["hidden"]],
                                    num_atoms=Z, support=support, noisy=True, layer_norm=True, output_vanish=True,
                                    init_layers=False, noise_std=0.5, device=dev)
    head.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")})
    x = torch.from_numpy(g["x"]).to(dev)
    with torch.no_grad():
        _near_q(head(x).cpu().numpy(), g["q"], "q")
        for out, key in ((head(x, q=False), "probs"), (head(x, log=True), "logp")):
            want = g[key]
            err = float(np.abs(out.cpu().numpy() - want).max())
            assert err <= 1e-5 * max(1.0, float(np.abs(want).max())), (key, err)
