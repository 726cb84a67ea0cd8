"""Parity of the HIP kernels (through the C ABI) against the CPU oracle and
the reference's golden vectors.  Needs an MI355X."""

from decimal import Decimal, getcontext

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cref  # noqa: E402
from oracle import dqn as odqn  # noqa: E402
from oracle import gae as ogae  # noqa: E402
from oracle import per as oper  # noqa: E402
from oracle import ppo_loss as oppo  # noqa: E402

DEV = torch.device("cuda:0")


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def K():
    from agilerl_amd import kernels

    return kernels


# --------------------------------------------------------------------------- #
# GAE — bit-exact                                                             #
# --------------------------------------------------------------------------- #
@pytest.mark.parametrize("case", [f"gae{i}" for i in range(8)])
def test_gae_golden_bit_exact(golden, case):
    g = golden(case)
    adv, ret = K().gae(T(g["rewards"]), T(g["dones"]), T(g["values"]), T(g["last_value"]),
                       T(g["last_done"]), float(g["gamma"]), float(g["lam"]), bool(g["use_gae"]))
    assert np.array_equal(adv.cpu().numpy().view(np.uint32), g["advantages"].view(np.uint32))
    assert np.array_equal(ret.cpu().numpy().view(np.uint32), g["returns"].view(np.uint32))


@pytest.mark.parametrize("P,Tn,N,pd,use_gae", [(8, 16, 128, 0.01, True), (3, 257, 1000, 0.02, True),
                                               (2, 33, 4099, 0.3, False), (5, 1, 64, 0.5, True),
                                               (1, 9, 1, 0.5, True)])
def test_gae_population_bit_exact_vs_c_oracle(P, Tn, N, pd, use_gae):
    rng = np.random.default_rng(P * 1000 + Tn)
    r = rng.standard_normal((P, Tn, N)).astype(np.float32)
    v = rng.standard_normal((P, Tn, N)).astype(np.float32)
    d = (rng.random((P, Tn, N)) < pd).astype(np.uint8)
    lv = rng.standard_normal((P, N)).astype(np.float32)
    ld = (rng.random((P, N)) < pd).astype(np.uint8)
    adv, ret, stats = K().gae(T(r), T(d), T(v), T(lv), T(ld), 0.99, 0.95, use_gae, with_stats=True)
    ea, er = cref.gae(r, v, d, lv, ld, 0.99, 0.95, use_gae, nthreads=8)
    assert np.array_equal(adv.cpu().numpy(), ea)
    assert np.array_equal(ret.cpu().numpy(), er)
    st = stats.cpu().numpy()
    for p in range(P):
        m, s = ogae.adv_stats(ea[p])
        assert abs(st[p, 0] - m) <= 1e-12 * max(1, abs(m)) + 1e-12
        if Tn * N > 1:
            assert abs(st[p, 1] - s) <= 1e-9 * s


def test_gae_full_size_section8d_bit_exact():
    """The SURVEY §8d roofline shape itself (P=8, T=1024, N=8192: 67.1 M
    transitions, done ~ Bernoulli(0.01)) against the C oracle: every advantage
    and return bit for bit, plus the fused per-agent statistics."""
    P, Tn, N = 8, 1024, 8192
    rng = np.random.default_rng(0)
    r = rng.standard_normal((P, Tn, N), dtype=np.float32)
    v = rng.standard_normal((P, Tn, N), dtype=np.float32)
    d = (rng.random((P, Tn, N), dtype=np.float32) < 0.01).astype(np.uint8)
    lv = rng.standard_normal((P, N), dtype=np.float32)
    ld = (rng.random((P, N)) < 0.01).astype(np.uint8)
    adv, ret, stats = K().gae(T(r), T(d), T(v), T(lv), T(ld), 0.99, 0.95, True, with_stats=True)
    ea, er = cref.gae(r, v, d, lv, ld, 0.99, 0.95, True, nthreads=16)
    ga = adv.cpu().numpy()
    assert np.array_equal(ga.view(np.uint32), ea.view(np.uint32))
    del ga, adv
    assert np.array_equal(ret.cpu().numpy().view(np.uint32), er.view(np.uint32))
    st = stats.cpu().numpy()
    for p in range(P):
        a64 = ea[p].astype(np.float64)
        m = a64.mean()
        assert abs(st[p, 0] - m) <= 1e-9 * max(1.0, abs(m))
        assert abs(st[p, 1] - a64.std(ddof=1)) <= 1e-9 * a64.std(ddof=1)


def test_gae_bool_dones_and_normalize():
    rng = np.random.default_rng(7)
    r = rng.standard_normal((2, 40, 300)).astype(np.float32)
    v = rng.standard_normal((2, 40, 300)).astype(np.float32)
    d = rng.random((2, 40, 300)) < 0.05
    lv = rng.standard_normal((2, 300)).astype(np.float32)
    ld = rng.random((2, 300)) < 0.05
    adv, ret, stats = K().gae(T(r), T(d), T(v), T(lv), T(ld), with_stats=True)
    ea, _ = cref.gae(r, v, d, lv, ld, 0.99, 0.95)
    assert np.array_equal(adv.cpu().numpy(), ea)
    K().adv_normalize_(adv, stats)
    for p in range(2):
        np.testing.assert_allclose(adv[p].cpu().numpy(), ogae.normalize_advantages(ea[p]), rtol=1e-5,
                                   atol=1e-6)


# --------------------------------------------------------------------------- #
# PPO loss                                                                    #
# --------------------------------------------------------------------------- #
def _loss_inputs(S, seed):
    rng = np.random.default_rng(seed)
    old = rng.uniform(-3, -0.05, S).astype(np.float32)
    lp = (old + rng.normal(0, 0.2, S)).astype(np.float32)
    A, R, ov = (rng.standard_normal(S).astype(np.float32) for _ in range(3))
    v = (ov + rng.normal(0, 0.3, S)).astype(np.float32)
    H = rng.uniform(0, 1.3, S).astype(np.float32)
    return lp, old, A, R, ov, v, H


@pytest.mark.parametrize("b,nmb", [(128, 16), (64, 5), (256, 3), (1000, 2), (130, 4), (7, 9)])
def test_ppo_loss_vs_oracle(b, nmb):
    lp, old, A, R, ov, v, H = _loss_inputs(b * nmb, b)
    g1, g2, g3, st = K().ppo_loss_fwd_bwd(*(T(x) for x in (lp, old, A, R, ov, v, H)), b, 0.2, 0.5, 0.01)
    g1, g2, g3, st = (x.cpu().numpy() for x in (g1, g2, g3, st))
    for m in range(nmb):
        s = slice(m * b, (m + 1) * b)
        loss, parts, e1, e2, e3 = oppo.minibatch_loss(lp[s], old[s], A[s], R[s], ov[s], v[s], H[s],
                                                       0.2, 0.5, 0.01)
        tol = 1e-5 * max(1.0, abs(loss))
        assert abs(st[m, 0] - loss) <= tol
        assert abs(st[m, 1] - parts["pg"]) <= 1e-5 * max(1, abs(parts["pg"]))
        assert abs(st[m, 2] - parts["vl"]) <= 1e-5 * max(1, abs(parts["vl"]))
        assert abs(st[m, 4] - parts["kl"]) <= 1e-6
        assert abs(st[m, 5] - parts["clipfrac"]) <= 1e-6
        np.testing.assert_allclose(g1[s], e1, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(g2[s], e2, rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(g3[s], e3, rtol=1e-6)


def test_ppo_loss_golden_with_index_gather(golden):
    """The reference's own schedule: normalised advantages, numpy permutation,
    per-minibatch gradients (ppo0: 2048 samples, b=128, 4 epochs)."""
    g = golden("ppo0")
    S, b = int(g["S"]), int(g["batch"])
    k = K()
    an = T(g["adv_norm"])
    old, R, ov = T(g["old_logp"]), T(g["ret"]), T(g["old_v"])
    nl, nv, H = g["new_logp"], g["new_v"], g["H"]
    snap = 0
    for perm in g["perms"]:
        for s0 in range(0, S, b):
            mb = perm[s0:s0 + b]
            g1, g2, g3, st = k.ppo_loss_fwd_bwd(T(nl[mb]), old, an, R, ov, T(nv[mb]), T(H[mb]), len(mb),
                                                float(g["clip"]), float(g["vf"]), float(g["ent"]),
                                                index=T(mb.astype(np.int64)))
            np.testing.assert_allclose(g1.cpu().numpy(), g["g_logp"][snap][mb], rtol=1e-4, atol=1e-8)
            np.testing.assert_allclose(g2.cpu().numpy(), g["g_v"][snap][mb], rtol=1e-4, atol=1e-8)
            np.testing.assert_allclose(g3.cpu().numpy(), g["g_H"][snap][mb], rtol=1e-5)
            snap += 1
    assert snap == int(g["n_minibatches"])


# --------------------------------------------------------------------------- #
# PER                                                                         #
# --------------------------------------------------------------------------- #
def _trees(cap):
    st = torch.empty(2 * cap, dtype=torch.float64, device=DEV)
    mt = torch.empty(2 * cap, dtype=torch.float64, device=DEV)
    K().per_init(st, mt, cap)
    return st, mt


def _assert_tree_close(dev_tree, ref_tree):
    """Every node bit-identical (leaves by glibc's pow algorithm, internal
    nodes the same f64 adds / mins in the same operand order)."""
    a = dev_tree.cpu().numpy()[1:]
    b = np.asarray(ref_tree)[1:]
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), int((a != b).sum())
    return 1.0


@pytest.mark.parametrize("case", [f"per{i}" for i in range(4)])
def test_per_golden_indices_bit_exact(golden, case):
    g = golden(case)
    ms, alpha, beta, B = int(g["max_size"]), float(g["alpha"]), float(g["beta"]), int(g["B"])
    cap = oper.tree_capacity(ms)
    st, mt = _trees(cap)
    mp = torch.ones(1, dtype=torch.float64, device=DEV)
    k = K()
    k.per_add(st, mt, cap, ms, 0, int(g["n_add"]), alpha, mp)
    ptr = int(g["n_add"]) % ms
    size = min(int(g["n_add"]), ms)
    for rd in range(int(g["rounds"])):
        idx, w = k.per_sample(st, mt, cap, T(g[f"u{rd}"]), size=size, beta=beta)
        assert np.array_equal(idx.cpu().numpy(), g[f"idx{rd}"])
        np.testing.assert_allclose(w.cpu().numpy(), g[f"w{rd}"], rtol=2e-7)
        k.per_update(st, mt, cap, ms, idx, T(g[f"pri{rd}"]), alpha, mp)
        n = int(g[f"extra{rd}"])
        k.per_add(st, mt, cap, ms, ptr, n, alpha, mp)
        ptr = (ptr + n) % ms
        size = min(size + n, ms)
        frac = _assert_tree_close(st, g[f"sum_tree{rd}"])
        _assert_tree_close(mt, g[f"min_tree{rd}"])
        assert frac > 0.95
        assert mp.item() == float(g[f"max_priority{rd}"])


def test_per_large_batches_vs_c_oracle():
    """Multi-launch path (batches > 1024) incl. duplicates, cap 2^17."""
    rng = np.random.default_rng(5)
    ms, alpha, beta = 100_000, 0.6, 0.4
    cap = oper.tree_capacity(ms)
    c = cref.PERTree(ms, alpha)
    st, mt = _trees(cap)
    mp = torch.ones(1, dtype=torch.float64, device=DEV)
    k = K()
    c.add(ms)
    k.per_add(st, mt, cap, ms, 0, ms, alpha, mp)
    for rd in range(3):
        idx = rng.integers(0, ms, 20_000)
        pri = (np.abs(rng.standard_normal(20_000)) * (3 if rd == 1 else 1)).astype(np.float32)
        pri[:50] = 1e-9
        c.update(idx, pri)
        k.per_update(st, mt, cap, ms, T(idx.astype(np.int64)), T(pri), alpha, mp)
        assert mp.item() == c.max_priority
        _assert_tree_close(st, c.sum)
        _assert_tree_close(mt, c.min)
        u = torch.rand(50_000, generator=torch.Generator().manual_seed(rd)).numpy()
        eidx, bad = c.sample(u)
        gidx, w = k.per_sample(st, mt, cap, T(u), size=ms, beta=beta)
        assert bad == 0
        assert np.array_equal(gidx.cpu().numpy(), eidx)
        np.testing.assert_allclose(w.cpu().numpy(), c.weights(eidx, beta), rtol=2e-7)


def test_per_dense_batch_band_rebuild_is_pure_function_of_leaves():
    """Dense batches (n * 32 >= capacity) rebuild whole bands of levels; at the
    §8d shape (cap 2^20, 2^16 updates with duplicates) every internal node
    must equal op(left, right) of its children bit for bit, as the reference's
    per-write ancestor walk leaves them (segment_tree.py:81-95)."""
    rng = np.random.default_rng(8)
    ms, cap = 1_000_000, 1 << 20
    st, mt = _trees(cap)
    mp = torch.ones(1, dtype=torch.float64, device=DEV)
    k = K()
    k.per_add(st, mt, cap, ms, 0, ms, 0.6, mp)
    idx = rng.integers(0, ms, 1 << 16)
    pri = np.abs(rng.standard_normal(1 << 16)).astype(np.float32)
    k.per_update(st, mt, cap, ms, T(idx.astype(np.int64)), T(pri), 0.6, mp)
    s, m = st.cpu().numpy(), mt.cpu().numpy()
    es, em = s.copy(), m.copy()
    for lvl in range(19, -1, -1):
        lo, hi = 1 << lvl, 1 << (lvl + 1)
        es[lo:hi] = es[2 * lo:2 * hi:2] + es[2 * lo + 1:2 * hi:2]
        c, d = em[2 * lo:2 * hi:2], em[2 * lo + 1:2 * hi:2]
        em[lo:hi] = np.where(d < c, d, c)
    assert np.array_equal(s[1:], es[1:]) and np.array_equal(m[1:], em[1:])
    # last duplicate wins on the leaves
    last = {int(i): j for j, i in enumerate(idx)}
    j = np.array(list(last.values()))
    leaves = s[cap + idx[j]]
    np.testing.assert_array_equal(leaves, cref.libm_pow(np.maximum(pri[j].astype(np.float64), 1e-5), 0.6))


def test_per_ring_add_wraps():
    ms, cap = 1000, 1024
    st, mt = _trees(cap)
    mp = torch.full((1,), 2.5, dtype=torch.float64, device=DEV)
    K().per_add(st, mt, cap, ms, 990, 1500, 0.6, mp)  # longer than the ring
    ref = oper.PER(ms, 0.6)
    ref.max_priority, ref.tree_ptr = 2.5, 990
    ref.add(1500)
    _assert_tree_close(st, ref.sum_tree.tree)


def test_libm_pow_bit_exact():
    """The device pow of the PER leaves / IS weights (csrc/libm_pow.h) equals
    the host libm pow — what the reference's Python ``float ** float`` runs —
    bit for bit: 2^21 random inputs over the PER domain (priorities 1e-5 ..
    1e3 at alpha 0.4-0.7, weight bases up to 1e6 at -beta), plus the inputs
    where libm differs from the correctly rounded value (which an exact
    double-double pow would get wrong)."""
    getcontext().prec = 50
    rng = np.random.default_rng(3)
    n = 1 << 21
    x = np.concatenate([np.abs(rng.standard_normal(n // 2)) + 1e-5,
                        np.exp(rng.uniform(np.log(1e-5), np.log(1e6), n // 2))])
    y = rng.choice([0.6, 0.4, 0.7, 0.5, -0.4, -0.5, -0.7, -1.0], size=n)
    got = K().debug_pow(T(x), T(y)).cpu().numpy()
    want = cref.libm_pow(x, y)
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert bad.size == 0, (bad.size, x[bad[:3]], y[bad[:3]], got[bad[:3]], want[bad[:3]])
    # inputs where libm is not correctly rounded: the device must follow libm
    xs = x[:4000]
    cr = np.array([float((Decimal(float(b)) * Decimal(float(a)).ln()).exp()) for a, b in zip(xs, y[:4000])])
    off = cr != want[:4000]
    assert off.any()  # the set exists ...
    assert np.array_equal(got[:4000][off], want[:4000][off])  # ... and the device matches libm on it
    assert float(K().debug_pow(T(np.array([1.1696802377700806])), T(np.array([0.6]))).cpu()[0]) == 1.0986017625035922


# --------------------------------------------------------------------------- #
# DQN TD target / Rainbow C51                                                 #
# --------------------------------------------------------------------------- #
@pytest.mark.parametrize("case", ["dqn0", "dqn1", "dqn2"])
def test_td_target_golden(golden, case):
    g = golden(case)
    y, gq, loss = K().td_target(T(g["q_next_target"]), T(g["r"]), T(g["d"]), float(g["gamma"]),
                                T(g["q_next_online"]), bool(g["double"]), T(g["q_cur"]), T(g["a"]))
    assert np.array_equal(y.cpu().numpy(), g["y"])
    np.testing.assert_allclose(gq.cpu().numpy(), g["g_q"], rtol=1e-5, atol=1e-9)
    assert abs(loss.item() - float(g["loss"])) <= 1e-5 * abs(float(g["loss"]))


@pytest.mark.parametrize("case", [f"c51_{i}" for i in range(4)])
def test_c51_golden(golden, case):
    g = golden(case)
    loss, proj = K().c51_project_loss(T(g["q_next"]), T(g["target_dist"]), T(g["logp_cur"]), T(g["a"]),
                                      T(g["r"]), T(g["d"]), T(g["support"]), float(g["vmin"]),
                                      float(g["vmax"]), float(g["gamma"]), with_proj=True)
    _, eproj = odqn.c51_project(g["q_next"], g["target_dist"], g["r"], g["d"], g["support"],
                                float(g["vmin"]), float(g["vmax"]), float(g["gamma"]))
    assert np.array_equal(proj.cpu().numpy(), eproj)
    np.testing.assert_allclose(loss.cpu().numpy(), g["loss"], rtol=1e-5, atol=1e-6)


def test_c51_large_vs_c_oracle():
    rng = np.random.default_rng(9)
    B, A, Z = 5000, 6, 51
    support = torch.linspace(-200, 200, Z).numpy()
    q = rng.standard_normal((B, A)).astype(np.float32)
    q[:10] = 0.0  # argmax ties -> first index
    td = torch.softmax(torch.randn(B, A, Z), -1).clamp(min=1e-3).numpy()
    lp = torch.log_softmax(torch.randn(B, A, Z), -1).numpy()
    a = rng.integers(0, A, B).astype(np.int64)
    r = (rng.standard_normal(B) * 120).astype(np.float32)
    d = (rng.random(B) < 0.1).astype(np.float32)
    loss, proj = K().c51_project_loss(T(q), T(td), T(lp), T(a), T(r), T(d), T(support), -200, 200,
                                      0.99 ** 4, with_proj=True)
    eloss, eproj = cref.c51(q, td, lp, a, r, d, support, -200.0, 200.0, 0.99 ** 4)
    assert np.array_equal(proj.cpu().numpy(), eproj)
    np.testing.assert_allclose(loss.cpu().numpy(), eloss, rtol=1e-5, atol=1e-5)


def test_c51_full_size_properties():
    """SURVEY §8d shape (2^20 rows, A=6, Z=51, ±200, γ_n = 0.99^4), where the
    CPU oracle is too slow for every row: (1) mass conservation — U = L + 1 for
    every atom, so each projected row sums to its target row's (clamped) mass;
    (2) loss >= 0 (log-probs <= 0); (3) 4096 rows spread over the batch are
    bit-exact against the C oracle."""
    B, A, Z = 1 << 20, 6, 51
    g = torch.Generator(device=DEV).manual_seed(3)
    qn = torch.randn(B, A, device=DEV, generator=g)
    td = torch.softmax(torch.randn(B, A, Z, device=DEV, generator=g), -1).clamp_(min=1e-3)
    lp = torch.log_softmax(torch.randn(B, A, Z, device=DEV, generator=g), -1)
    act = torch.randint(0, A, (B,), device=DEV, generator=g)
    r = torch.randn(B, device=DEV, generator=g) * 50
    d = (torch.rand(B, device=DEV, generator=g) < 0.05).float()
    sup = torch.linspace(-200, 200, Z, device=DEV)
    loss, proj = K().c51_project_loss(qn, td, lp, act, r, d, sup, -200.0, 200.0, 0.99 ** 4, with_proj=True)
    astar = qn.argmax(1)
    mass = td[torch.arange(B, device=DEV), astar].double().sum(1)
    err = (proj.double().sum(1) - mass).abs().max().item()
    assert err < 1e-5, err
    assert loss.min().item() >= 0.0
    rows = torch.linspace(0, B - 1, 4096, device=DEV).long()
    sel = lambda x: x[rows].cpu().numpy()  # noqa: E731
    eloss, eproj = cref.c51(sel(qn), sel(td), sel(lp), sel(act), sel(r), sel(d), sup.cpu().numpy(), -200.0,
                            200.0, 0.99 ** 4)
    assert np.array_equal(proj[rows].cpu().numpy(), eproj)
    np.testing.assert_allclose(loss[rows].cpu().numpy(), eloss, rtol=1e-5, atol=1e-5)


def _lib_error():
    from agilerl_amd._lib import AgxError

    return AgxError


@pytest.mark.parametrize("case", [f"c51_{i}" for i in range(4)])
def test_c51_rows_golden(golden, case):
    """agx_c51_project_loss_rows on the two selected rows gathered from the
    fixture's [B][A][Z] arrays: the same projection bit for bit."""
    g = golden(case)
    B = g["q_next"].shape[0]
    astar = torch.from_numpy(g["q_next"]).argmax(1).numpy()
    td = np.ascontiguousarray(g["target_dist"][np.arange(B), astar])
    lp = np.ascontiguousarray(g["logp_cur"][np.arange(B), g["a"].reshape(-1).astype(np.int64)])
    if td.shape[1] != 51:  # the rows form is Rainbow's 51 atoms only
        with pytest.raises(_lib_error()):
            K().c51_project_loss_rows(T(td), T(lp), T(g["r"]), T(g["d"]), T(g["support"]), float(g["vmin"]),
                                      float(g["vmax"]), float(g["gamma"]))
        return
    loss, proj = K().c51_project_loss_rows(T(td), T(lp), T(g["r"]), T(g["d"]), T(g["support"]), float(g["vmin"]),
                                           float(g["vmax"]), float(g["gamma"]), with_proj=True)
    _, eproj = odqn.c51_project(g["q_next"], g["target_dist"], g["r"], g["d"], g["support"],
                                float(g["vmin"]), float(g["vmax"]), float(g["gamma"]))
    assert np.array_equal(proj.cpu().numpy(), eproj)
    np.testing.assert_allclose(loss.cpu().numpy(), g["loss"], rtol=1e-5, atol=1e-6)


def test_c51_rows_full_size_equals_full_layout():
    """§8d shape (2^20 rows, A=6, Z=51): the selected-rows kernel equals the
    [B][A][Z] kernel bit for bit (loss and projection), incl. argmax ties."""
    B, A, Z = 1 << 20, 6, 51
    g = torch.Generator(device=DEV).manual_seed(5)
    qn = torch.randn(B, A, device=DEV, generator=g)
    qn[:4096] = 0.0  # ties -> the first maximum
    td = torch.softmax(torch.randn(B, A, Z, device=DEV, generator=g), -1).clamp_(min=1e-3)
    lp = torch.log_softmax(torch.randn(B, A, Z, device=DEV, generator=g), -1)
    act = torch.randint(0, A, (B,), device=DEV, generator=g)
    r = torch.randn(B, device=DEV, generator=g) * 50
    d = (torch.rand(B, device=DEV, generator=g) < 0.05).float()
    sup = torch.linspace(-200, 200, Z, device=DEV)
    loss, proj = K().c51_project_loss(qn, td, lp, act, r, d, sup, -200.0, 200.0, 0.99 ** 4, with_proj=True)
    idx = torch.arange(B, device=DEV)
    tr, lr_ = td[idx, qn.argmax(1)].contiguous(), lp[idx, act].contiguous()
    loss2, proj2 = K().c51_project_loss_rows(tr, lr_, r, d, sup, -200.0, 200.0, 0.99 ** 4, with_proj=True)
    assert torch.equal(proj, proj2) and torch.equal(loss, loss2)
    assert torch.equal(loss2, K().c51_project_loss_rows(tr, lr_, r, d, sup, -200.0, 200.0, 0.99 ** 4))


@pytest.mark.parametrize("vmin,vmax,gamma,Z", [(-10.0, 10.0, 0.99 ** 3, 51),   # Δz = 0.4: division path
                                                 (-200.0, 200.0, -0.9, 51),       # L/U decreasing: RMW fallback
                                                 (-100.0, 100.0, 0.99, 41)])      # other Z: row-wave kernel
def test_c51_paths_vs_c_oracle(vmin, vmax, gamma, Z):
    rng = np.random.default_rng(11)
    B, A = 700, 5
    support = torch.linspace(vmin, vmax, Z).numpy()
    q = rng.standard_normal((B, A)).astype(np.float32)
    td = torch.softmax(torch.randn(B, A, Z), -1).clamp(min=1e-3).numpy()
    lp = torch.log_softmax(torch.randn(B, A, Z), -1).numpy()
    a = rng.integers(0, A, B).astype(np.int64)
    r = (rng.standard_normal(B) * (vmax - vmin) / 6).astype(np.float32)
    d = (rng.random(B) < 0.1).astype(np.float32)
    loss, proj = K().c51_project_loss(T(q), T(td), T(lp), T(a), T(r), T(d), T(support), vmin, vmax, gamma,
                                      with_proj=True)
    eloss, eproj = cref.c51(q, td, lp, a, r, d, support, vmin, vmax, gamma)
    assert np.array_equal(proj.cpu().numpy(), eproj)
    np.testing.assert_allclose(loss.cpu().numpy(), eloss, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------- #
# optimiser                                                                   #
# --------------------------------------------------------------------------- #
@pytest.mark.parametrize("P,n,split", [(3, 5000, 3100), (3, 5001, 3101), (2, 40_000, 24_002)],
                         ids=["float4", "scalar", "pre-reduced-norm"])
def test_clip_adam_matches_torch(P, n, split):
    torch.manual_seed(0)
    p0 = torch.randn(P, n)
    grads = [torch.randn(P, n) * (5.0 if s == 0 else 0.01) for s in range(4)]
    lr = [1e-3, 5e-4, 2e-3][:P]
    ref = [torch.nn.Parameter(p0[i, :split].clone()) for i in range(P)]
    ref2 = [torch.nn.Parameter(p0[i, split:].clone()) for i in range(P)]
    opts = [torch.optim.Adam([ref[i], ref2[i]], lr=lr[i]) for i in range(P)]
    params = p0.clone().to(DEV)
    opt = K().ClipAdam(params, [0, split, n], lr, max_norm=0.5)
    for g in grads:
        for i in range(P):
            ref[i].grad = g[i, :split].clone()
            ref2[i].grad = g[i, split:].clone()
            torch.nn.utils.clip_grad_norm_([ref[i]], 0.5)
            torch.nn.utils.clip_grad_norm_([ref2[i]], 0.5)
            opts[i].step()
        opt.grads.copy_(g)
        opt.step()
    got = params.cpu()
    for i in range(P):
        np.testing.assert_allclose(got[i, :split].numpy(), ref[i].detach().numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(got[i, split:].numpy(), ref2[i].detach().numpy(), rtol=1e-5, atol=1e-6)


def test_polyak():
    t = torch.randn(10_001)
    o = torch.randn(10_001)
    exp = 1e-3 * o + (1.0 - 1e-3) * t
    td = t.to(DEV)
    K().polyak_(td, o.to(DEV), 1e-3)
    assert torch.equal(td.cpu(), exp)


def test_rows_gather_matches_index_select():
    """agx_rows_gather (the single-rank generation clone): every buffer's row j
    becomes its old row idx[j], repeats included, bit for bit."""
    import ctypes

    from agilerl_amd import _lib

    dev = torch.device("cuda:0")
    P = 8
    g = torch.Generator(device=dev).manual_seed(9)
    bufs = [torch.randn(P, w, device=dev, generator=g) for w in (13829, 13829, 13829, 1, 2, 1, 1, 1)]
    want = None
    idx_l = [0, 0, 3, 7, 3, 1, 6, 6]
    idx = torch.tensor(idx_l, device=dev)
    want = [b[idx].clone() for b in bufs]
    n = len(bufs)
    widths = (ctypes.c_int64 * n)(*[b.shape[1] for b in bufs])
    ptrs = (ctypes.c_void_p * n)(*[b.data_ptr() for b in bufs])
    ws = torch.empty(int(_lib.load().agx_rows_gather_workspace_bytes(widths, n, P)), dtype=torch.uint8, device=dev)
    _lib.call("agx_rows_gather", ptrs, widths, n, P, idx.data_ptr(), ws.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    for b, w in zip(bufs, want):
        assert torch.equal(b, w)
