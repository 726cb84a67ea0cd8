"""Pin the CPU oracle (numpy + C restatements) to the reference's own outputs.

Fixtures come from tests/golden/gen_golden.py, which executed the reference
source files (agilerl 2.7.0) in place.  CPU only."""

import math

import numpy as np
import pytest

from oracle import cref
from oracle import dqn as odqn
from oracle import gae as ogae
from oracle import per as oper
from oracle import ppo_loss as oppo
from oracle import tournament as otour

GAE_CASES = [f"gae{i}" for i in range(8)]


@pytest.mark.parametrize("case", GAE_CASES)
def test_gae_numpy_bit_exact(golden, case):
    g = golden(case)
    adv, ret = ogae.gae(g["rewards"], g["values"], g["dones"], g["last_value"], g["last_done"],
                        float(g["gamma"]), float(g["lam"]), bool(g["use_gae"]))
    assert np.array_equal(adv.view(np.uint32), g["advantages"].view(np.uint32))
    assert np.array_equal(ret.view(np.uint32), g["returns"].view(np.uint32))


@pytest.mark.parametrize("case", GAE_CASES)
def test_gae_c_bit_exact(golden, case):
    g = golden(case)
    adv, ret = cref.gae(g["rewards"], g["values"], g["dones"], g["last_value"], g["last_done"],
                        float(g["gamma"]), float(g["lam"]), bool(g["use_gae"]))
    assert np.array_equal(adv.view(np.uint32), g["advantages"].view(np.uint32))
    assert np.array_equal(ret.view(np.uint32), g["returns"].view(np.uint32))


def test_gae_c_batched_population_matches_per_agent(golden):
    rng = np.random.default_rng(0)
    P, T, N = 3, 20, 17
    r = rng.standard_normal((P, T, N)).astype(np.float32)
    v = rng.standard_normal((P, T, N)).astype(np.float32)
    d = rng.random((P, T, N)) < 0.1
    lv = rng.standard_normal((P, N)).astype(np.float32)
    ld = rng.random((P, N)) < 0.1
    adv, ret = cref.gae(r, v, d, lv, ld, 0.99, 0.95, nthreads=4)
    for p in range(P):
        a, rt = ogae.gae(r[p], v[p], d[p], lv[p], ld[p])
        assert np.array_equal(a, adv[p]) and np.array_equal(rt, ret[p])


def test_segment_tree_golden(golden):
    g = golden("segtree")
    cap = int(g["cap"])
    s, m = oper.SumSegmentTree(cap), oper.MinSegmentTree(cap)
    for i, x in zip(g["set_idx"], g["set_val"]):
        s[int(i)] = float(x)
        m[int(i)] = float(x)
    assert np.array_equal(np.array(s.tree), g["sum_tree"])
    assert np.array_equal(np.array(m.tree), g["min_tree"])
    got = [s.retrieve(float(q)) for q in g["queries"]]
    assert np.array_equal(got, g["retrieve"])
    for (a, b), es, em in zip(g["ranges"], g["range_sum"], g["range_min"]):
        assert s.sum(int(a), int(b)) == es and m.min(int(a), int(b)) == em


def test_segment_tree_known_answers():
    """Upstream tests/test_components/test_segment_tree.py:39-129."""
    t = oper.SumSegmentTree(4)
    t[2], t[3] = 1.0, 3.0
    assert [t.retrieve(x) for x in (0.0, 0.5, 0.99, 1.01, 3.0, 4.0)] == [2, 2, 2, 3, 3, 3]
    assert math.isclose(t.sum(), 4.0) and math.isclose(t.sum(2, 4), 4.0) and t.sum(0, 2) == 0.0
    t = oper.SumSegmentTree(4)
    t[0], t[1], t[2], t[3] = 0.5, 1.0, 1.0, 3.0
    assert [t.retrieve(x) for x in (0.0, 0.55, 0.99, 1.51, 3.0, 5.5)] == [0, 1, 1, 2, 3, 3]
    m = oper.MinSegmentTree(4)
    m[0], m[2], m[3] = 1.0, 0.5, 3.0
    assert m.min() == 0.5 and m.min(0, 2) == 1.0 and m.min(3, 4) == 3.0
    m[2] = 4.0
    assert m.min() == 1.0 and m.min(2, 4) == 3.0 and m.min(2, 3) == 4.0


def test_per_known_answers():
    """Upstream tests/test_components/test_replay_buffer.py:901-1039."""
    b = oper.PER(100, 0.6)
    b.add(5)
    b.update_priorities(np.arange(3), np.array([2.0, 3.0, 4.0], np.float32))
    for i, p in enumerate([2.0, 3.0, 4.0]):
        assert b.sum_tree[i] == p ** 0.6 and b.min_tree[i] == p ** 0.6
    assert b.max_priority == 4.0
    b2 = oper.PER(10, 0.6)
    b2.add(3)
    b2.update_priorities([0, 1], np.array([1e-10, 1e-10], np.float32))
    assert b2.sum_tree[0] >= 1e-5 ** 0.6
    b3 = oper.PER(100, 0.6)
    b3.add(5)
    pr = [0.5, 1.0, 1.5, 2.0, 2.5]
    for i, p in enumerate(pr):
        b3._update_priority(i, p)
    for i, p in enumerate(pr):
        w = b3.weights([i], 0.4)[0]
        ps = p ** 0.6 / b3.sum_tree.sum()
        pm = b3.min_tree.min() / b3.sum_tree.sum()
        assert np.isclose(w, (ps * 5) ** -0.4 / (pm * 5) ** -0.4, rtol=1e-5)
    with pytest.raises(AssertionError):
        b3._update_priority(100, 1.0)


@pytest.mark.parametrize("case", [f"per{i}" for i in range(4)])
def test_per_golden_python_and_c(golden, case):
    g = golden(case)
    ms, alpha, beta, B = int(g["max_size"]), float(g["alpha"]), float(g["beta"]), int(g["B"])
    py = oper.PER(ms, alpha)
    c = cref.PERTree(ms, alpha)
    py.add(int(g["n_add"]))
    c.add(int(g["n_add"]))
    for rd in range(int(g["rounds"])):
        u = g[f"u{rd}"]
        idx = py.sample_indices(u)
        assert np.array_equal(idx, g[f"idx{rd}"])
        cidx, bad = c.sample(u)
        assert bad == 0 and np.array_equal(cidx, g[f"idx{rd}"])
        assert np.array_equal(py.weights(idx, beta), g[f"w{rd}"])
        assert np.array_equal(c.weights(cidx, beta), g[f"w{rd}"])
        py.update_priorities(idx, g[f"pri{rd}"])
        c.update(cidx, g[f"pri{rd}"])
        py.add(int(g[f"extra{rd}"]))
        c.max_priority = py.max_priority
        c.add(int(g[f"extra{rd}"]))
        assert np.array_equal(np.array(py.sum_tree.tree), g[f"sum_tree{rd}"])
        assert np.array_equal(np.array(py.min_tree.tree), g[f"min_tree{rd}"])
        assert np.array_equal(c.sum, g[f"sum_tree{rd}"]) and np.array_equal(c.min, g[f"min_tree{rd}"])
        assert py.max_priority == g[f"max_priority{rd}"] and c.max_priority == g[f"max_priority{rd}"]
        assert py.tree_ptr == g[f"tree_ptr{rd}"] == int(c.tree_ptr[0])


@pytest.mark.parametrize("case", ["per1", "per2"])
def test_per_bulk_build_equals_path_updates(golden, case):
    g = golden(case)
    st = g["sum_tree0"]
    cap = st.size // 2
    assert np.array_equal(oper.build_tree_from_leaves(st[cap:], cap, "sum")[1:], st[1:])
    mt = g["min_tree0"]
    assert np.array_equal(oper.build_tree_from_leaves(mt[cap:], cap, "min")[1:], mt[1:])


@pytest.mark.parametrize("case", ["ppo0", "ppo1"])
def test_ppo_loss_golden(golden, case):
    g = golden(case)
    an = ogae.normalize_advantages(g["adv"])
    np.testing.assert_allclose(an, g["adv_norm"], rtol=1e-5, atol=1e-6)
    # perms replayed from the global numpy stream
    np.random.seed(int(g["seed"]))
    idx = np.arange(int(g["S"]))
    for e in range(int(g["epochs"])):
        np.random.shuffle(idx)
        assert np.array_equal(idx, g["perms"][e])
    glp, gv, gh, mean_loss = oppo.learn_flat(
        g["old_logp"], g["adv_norm"], g["ret"], g["old_v"], g["new_logp"], g["new_v"], g["H"],
        g["perms"], int(g["batch"]), float(g["clip"]), float(g["vf"]), float(g["ent"]))
    for got, ref in ((glp, g["g_logp"]), (gv, g["g_v"]), (gh, g["g_H"])):
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-9)
    assert abs(mean_loss - float(g["mean_loss"])) <= 1e-5 * abs(float(g["mean_loss"])) + 1e-9


def test_ppo_loss_c_matches_numpy():
    rng = np.random.default_rng(3)
    S, b = 4096, 128
    old = rng.uniform(-3, -0.05, S).astype(np.float32)
    lp = (old + rng.normal(0, 0.1, S)).astype(np.float32)
    adv, ret, ov = (rng.standard_normal(S).astype(np.float32) for _ in range(3))
    v = (ov + rng.normal(0, 0.3, S)).astype(np.float32)
    H = rng.uniform(0, 1.3, S).astype(np.float32)
    loss, g1, g2, g3 = cref.ppo_loss(lp, old, adv, ret, ov, v, H, b, 0.2, 0.5, 0.01)
    for m in range(S // b):
        s = slice(m * b, (m + 1) * b)
        l, _, e1, e2, e3 = oppo.minibatch_loss(lp[s], old[s], adv[s], ret[s], ov[s], v[s], H[s], 0.2, 0.5, 0.01)
        assert abs(loss[m] - l) < 1e-12 * max(1, abs(l))
        np.testing.assert_allclose(g1[s], e1, rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(g2[s], e2, rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(g3[s], e3, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("case", ["dqn0", "dqn1", "dqn2"])
def test_td_target_golden(golden, case):
    g = golden(case)
    y = odqn.td_target(g["q_next_online"], g["q_next_target"], g["r"], g["d"], float(g["gamma"]),
                       bool(g["double"]))
    assert np.array_equal(y, g["y"])
    loss, grad = odqn.td_loss(g["q_cur"], g["a"], y)
    assert abs(loss - float(g["loss"])) <= 1e-5 * abs(float(g["loss"]))
    np.testing.assert_allclose(grad, g["g_q"], rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("case", [f"c51_{i}" for i in range(4)])
def test_c51_golden(golden, case):
    g = golden(case)
    args = (g["q_next"], g["target_dist"], g["logp_cur"], g["a"], g["r"], g["d"], g["support"],
            float(g["vmin"]), float(g["vmax"]), float(g["gamma"]))
    loss, proj = odqn.c51_loss(*args)
    np.testing.assert_allclose(loss, g["loss"], rtol=1e-5, atol=1e-6)
    closs, cproj = cref.c51(*args)
    assert np.array_equal(cproj, proj)
    np.testing.assert_allclose(closs, g["loss"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", [f"tour{i}" for i in range(4)])
def test_tournament_golden(golden, case):
    g = golden(case)
    np.random.seed(int(g["seed"]))
    elite, parents = otour.select(list(g["fitness"]), int(g["tsize"]), bool(g["elitism"]),
                                  int(g["eval_loop"]))
    ind = g["indices"]
    assert ind[elite] == g["elite_parent"]
    assert np.array_equal(ind[np.array(parents)], g["parents"])
