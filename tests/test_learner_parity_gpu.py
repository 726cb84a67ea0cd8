"""Parity of the fused PPO learner (agx_ppo_learn, 79 % of the bench step)
against INDEPENDENT references — neither shares a kernel with it:

  * the reference's own _learn_from_rollout_buffer_flat run end to end on a
    real create_mlp actor-critic (tests/golden/learn*.npz): config-2 shape,
    target-KL early stop + action masks + the default [16] critic head, and a
    continued agent (Adam step > 0);
  * the pure-PyTorch CPU restatement oracle/ppo_learn.py (pinned to those
    goldens by tests/test_ppo_learn_oracle.py) at the exact config-2
    population shape: P=8 agents, N=128 envs, T=16, batch 128, 4 epochs,
    encoder [64] -> 64, heads [64], permutations from the reference's numpy
    shuffle stream.

Tolerance.  One update from the reference's own state (at points along its
trajectory): every parameter entry within 1e-5 x (|ref| + rms(ref)) (Adam
moments 1e-4) except at most 0.01 % of entries, and no entry off by more
than ATOL_MAX.  A whole learn() (64 chained updates): PPO's ratio / value clip
and max() decisions turn last-bit differences into discrete gradient
changes, so two correct fp32 implementations drift apart by as much as the
reference's fp32 run drifts from its own fp64 run (measured: 8e-7 after
epoch 1, 1.7e-3 after epoch 4 on learn0); the whole-learn tests require
|gpu - ref| within 4x that envelope, in max and in mean.
Also: a partner workgroup that never arrives raises AgxError instead of
returning a half-applied update."""

import numpy as np
import pytest
import torch

from oracle.ppo_learn import ActorCritic, reference_learn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
RTOL = 1e-5
ATOL_MAX = 1e-4


def _close_report(a, b, rtol=RTOL):
    """Entry i is close when |a - b| <= rtol * (|b_i| + rms(b)): relative to the
    entry, with near-zero entries measured against the tensor's typical size
    (an Adam update moves every entry by O(lr) whatever its magnitude)."""
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    d = np.abs(a - b)
    rms = float(np.sqrt(np.mean(b * b)))
    bad = d > rtol * (np.abs(b) + rms)
    return bad.mean(), d.max(), np.argmax(d)


def _assert_close(name, a, b, rtol=RTOL, frac=1e-4):
    bad, dmax, i = _close_report(a, b, rtol)
    assert bad <= frac and dmax <= ATOL_MAX, f"{name}: {bad:.2e} of entries beyond rtol {rtol}, max |diff| {dmax:.3e}"


def _names(g, prefix):
    from oracle.ppo_learn import reference_names

    return reference_names({k[len(prefix):]: g[k] for k in g if k.startswith(prefix)})


def _pop(P, N, T, D, A, enc, lat, ah, ch, batch, epochs, lr, target_kl=None, masks=False, seeds=None):
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation

    # the golden networks are create_mlp(..., name="encoder") (gen_golden.py), so
    # the spec takes that encoder name for the state-dict key map
    spec = ActorCriticSpec(obs_dim=D, n_actions=A, encoder_hidden=list(enc), latent_dim=lat,
                           actor_hidden=list(ah), critic_hidden=list(ch), encoder_name="encoder")
    pop = PPOPopulation(spec, P, N, learn_step=T * N, batch_size=batch, lr=lr, update_epochs=epochs,
                        target_kl=target_kl, seeds=seeds, device=DEV, fused=True, action_masks=masks)
    assert pop.fused_descriptor() is not None
    return pop


def _set_stats(pop):
    a = pop.advantages.view(pop.P, -1).double()
    pop.adv_stats[:, 0] = a.mean(1)
    pop.adv_stats[:, 1] = a.std(1)  # unbiased, as agx_gae's stats


def _flat_from_names(spec, sd, n):
    out = np.zeros(n, np.float32)
    for k, (off, shape) in spec.state_dict_keys().items():
        if k.startswith("critic.encoder."):
            continue
        out[off:off + int(np.prod(shape))] = np.asarray(sd[k], np.float32).ravel()
    return out


def _oracle_net(g):
    net = ActorCritic(int(g["obs_dim"]), int(g["n_actions"]), list(g["enc"]), int(g["latent"]),
                      list(g["actor_hidden"]), list(g["critic_hidden"]))
    net.load_reference(_names(g, "init."))
    return net


def _golden_adam(g):
    if int(g["step_in"]) == 0:
        return None
    m, v = _names(g, "init_m."), _names(g, "init_v.")
    adam = {k: (m[k], v[k]) for k in m}
    adam["step"] = int(g["step_in"])
    return adam


def _golden_oracle(g, dtype=torch.float32, on_update=None):
    net = _oracle_net(g)
    adam = _golden_adam(g)
    if dtype == torch.float64:
        net = net.double()
        if adam is not None:
            adam = {k: ((np.asarray(a[0], np.float64), np.asarray(a[1], np.float64)) if k != "step" else a)
                    for k, a in adam.items()}
    tkl = float(g["target_kl"])
    return reference_learn(net, adam, g["obs"], g["actions"], g["old_logp"], g["adv"], g["ret"], g["old_v"],
                           g["perms"], batch_size=int(g["batch"]), epochs=int(g["epochs"]), lr=float(g["lr"]),
                           target_kl=None if tkl <= 0 else tkl, masks=g.get("masks"), dtype=dtype,
                           on_update=on_update)


def _envelope(name, got, ref32, ref64, k_max=4.0):
    """|gpu - ref32| within k x the reference's OWN fp32 rounding sensitivity
    |ref64 - ref32| (PPO's clip / max decisions turn last-bit differences into
    discrete gradient changes late in a learn: two correct fp32
    implementations drift apart exactly as far as fp32 vs fp64 does)."""
    d = np.abs(np.asarray(got, np.float64) - np.asarray(ref32, np.float64))
    e = np.abs(np.asarray(ref64, np.float64) - np.asarray(ref32, np.float64))
    assert d.max() <= k_max * e.max() + 1e-6, f"{name}: max|gpu-ref| {d.max():.3e} vs fp32 envelope {e.max():.3e}"
    assert d.mean() <= k_max * e.mean() + 1e-8, \
        f"{name}: mean|gpu-ref| {d.mean():.3e} vs fp32 envelope {e.mean():.3e}"


def _load_rows(pop, rows, t):
    """rows[p] = dict(obs, act, old_logp, adv (already normalised), ret, old_v, masks|None)."""
    P = pop.P
    pop.obs.copy_(t(np.stack([r["obs"] for r in rows])).view_as(pop.obs))
    pop.actions.copy_(t(np.stack([r["act"] for r in rows])).view_as(pop.actions))
    pop.log_probs.copy_(t(np.stack([r["old_logp"] for r in rows])).view_as(pop.log_probs))
    pop.values.copy_(t(np.stack([r["old_v"] for r in rows])).view_as(pop.values))
    pop.advantages.copy_(t(np.stack([r["adv"] for r in rows])).view_as(pop.advantages))
    pop.returns.copy_(t(np.stack([r["ret"] for r in rows])).view_as(pop.returns))
    if pop.action_masks is not None:
        pop.action_masks.copy_(t(np.stack([r["masks"] for r in rows]).astype(np.uint8)).view_as(pop.action_masks))
    # identity normalisation: (a - 0) * (1 / ((1 - 1e-8) + 1e-8)) == a exactly
    pop.adv_stats[:, 0] = 0.0
    pop.adv_stats[:, 1] = 1.0 - 1e-8
    assert P == len(rows)


@pytest.mark.parametrize("name", ["learn0", "learn1", "learn2"])
def test_fused_single_updates_along_reference_trajectory(golden, name):
    """One fused update from the reference's OWN state at EVERY update of its
    learn() trajectory (each agent of a population starts from a different
    update k of the reference run: parameters, Adam moments, step count, and
    minibatch k as its rollout; populations of 16 agents, the production
    partner split).  Each must land where the reference's update k lands: no
    drift, every layer, at fp32 rounding level."""
    g = golden(name)
    snaps = {}
    out = _golden_oracle(g, on_update=lambda k, sn: snaps.__setitem__(k, sn))
    n_upd = len(out["approx_kl"])
    b = int(g["batch"])
    every = [k for k in range(n_upd) if len(snaps[k]["idx"]) == b]
    after = {k: (snaps[k + 1] if k + 1 in snaps else {"state": out["state"], "exp_avg": out["exp_avg"],
                                                       "exp_avg_sq": out["exp_avg_sq"], "step": out["step"]})
             for k in every}
    assert len(every) >= n_upd - int(g["epochs"])  # only a short last chunk per epoch is skipped
    for c in range(0, len(every), 16):
        _single_updates(g, snaps, after, every[c:c + 16], b)


def _single_updates(g, snaps, after, picks, b):
    P = len(picks)
    pop = _pop(P, b, 1, int(g["obs_dim"]), int(g["n_actions"]), g["enc"], int(g["latent"]), g["actor_hidden"],
               g["critic_hidden"], b, 1, float(g["lr"]), masks="masks" in g)
    spec, n = pop.spec, pop.spec.n_params
    t = lambda x: torch.as_tensor(np.asarray(x)).to(DEV)  # noqa: E731
    rows = []
    for j, k in enumerate(picks):
        sn = snaps[k]
        idx = sn["idx"]
        cv = lambda d: {kk: vv.numpy() for kk, vv in d.items()}  # noqa: E731
        pop.params.data[j] = t(_flat_from_names(spec, cv(sn["state"]), n))
        pop.opt.exp_avg[j] = t(_flat_from_names(spec, cv(sn["exp_avg"]), n))
        pop.opt.exp_avg_sq[j] = t(_flat_from_names(spec, cv(sn["exp_avg_sq"]), n))
        pop.opt.steps[j] = sn["step"]
        rows.append(dict(obs=g["obs"][idx], act=g["actions"][idx], old_logp=g["old_logp"][idx],
                         adv=sn["adv_norm"][idx].astype(np.float32), ret=g["ret"][idx], old_v=g["old_v"][idx],
                         masks=None if "masks" not in g else g["masks"][idx]))
    _load_rows(pop, rows, t)
    from agilerl_amd.population.learner import fused_learn

    perms = torch.arange(b, device=DEV).repeat(1, P, 1).contiguous()
    fused_learn(pop, perms)
    torch.cuda.synchronize()
    pop.check_errors()
    got_p, got_m, got_v = (x.cpu().numpy() for x in (pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq))
    for j, k in enumerate(picks):
        a = after[k]
        cv = lambda d: {kk: vv.numpy() for kk, vv in d.items()}  # noqa: E731
        assert int(pop.opt.steps[j]) == a["step"]
        _assert_close(f"update {k} params", got_p[j], _flat_from_names(spec, cv(a["state"]), n))
        _assert_close(f"update {k} exp_avg", got_m[j], _flat_from_names(spec, cv(a["exp_avg"]), n), rtol=1e-4)
        _assert_close(f"update {k} exp_avg_sq", got_v[j], _flat_from_names(spec, cv(a["exp_avg_sq"]), n),
                      rtol=1e-4)


@pytest.mark.parametrize("name", ["learn0", "learn1", "learn2"])
def test_fused_learner_matches_reference_learn(golden, name):
    """A whole learn() (all epochs, the reference's permutation stream,
    target-KL stop, masks, continued Adam) against the reference run itself:
    same epochs / steps / mean loss, parameters and moments within the
    reference's own fp32 rounding envelope."""
    from agilerl_amd.population.learner import fused_learn

    g = golden(name)
    T, N = int(g["T"]), int(g["N"])
    tkl = float(g["target_kl"])
    pop = _pop(1, N, T, int(g["obs_dim"]), int(g["n_actions"]), g["enc"], int(g["latent"]), g["actor_hidden"],
               g["critic_hidden"], int(g["batch"]), int(g["epochs"]), float(g["lr"]),
               target_kl=None if tkl <= 0 else tkl, masks="masks" in g)
    spec, n = pop.spec, pop.spec.n_params
    t = lambda x: torch.as_tensor(np.asarray(x)).to(DEV)  # noqa: E731
    pop.params.data[0] = t(_flat_from_names(spec, _names(g, "init."), n))
    if int(g["step_in"]) > 0:
        pop.opt.exp_avg[0] = t(_flat_from_names(spec, _names(g, "init_m."), n))
        pop.opt.exp_avg_sq[0] = t(_flat_from_names(spec, _names(g, "init_v."), n))
        pop.opt.steps[0] = int(g["step_in"])
    pop.obs.view(-1)[:] = t(g["obs"]).view(-1)
    pop.actions.view(-1)[:] = t(g["actions"])
    pop.log_probs.view(-1)[:] = t(g["old_logp"])
    pop.values.view(-1)[:] = t(g["old_v"])
    pop.advantages.view(-1)[:] = t(g["adv"])
    pop.returns.view(-1)[:] = t(g["ret"])
    if "masks" in g:
        pop.action_masks.view(-1)[:] = t(g["masks"]).view(-1)
    _set_stats(pop)
    perms = t(g["perms"]).view(int(g["epochs"]), 1, T * N).contiguous()
    loss = fused_learn(pop, perms)
    torch.cuda.synchronize()
    pop.check_errors()
    assert int(pop._fused.epochs_run[0]) == int(g["epochs_run"])
    assert int(pop.opt.steps[0]) == int(g["step_out"])
    assert abs(float(loss[0]) - float(g["mean_loss"])) <= 1e-4 * abs(float(g["mean_loss"])) + 1e-7
    r64 = _golden_oracle(g, torch.float64)
    for key, gold, o64 in (("params", "final.", r64["state"]), ("exp_avg", "m.", r64["exp_avg"]),
                           ("exp_avg_sq", "v.", r64["exp_avg_sq"])):
        got = {"params": pop.params.data, "exp_avg": pop.opt.exp_avg, "exp_avg_sq": pop.opt.exp_avg_sq}[key]
        ref32 = _flat_from_names(spec, _names(g, gold), n)
        ref64 = _flat_from_names(spec, {k: v.numpy() for k, v in o64.items()}, n).astype(np.float64)
        _envelope(key, got[0].cpu().numpy(), ref32, ref64)


def _config2_population(target_kl=None, masks=False, seed=0):
    P, N, T, D, A = 8, 128, 16, 8, 4
    pop = _pop(P, N, T, D, A, [64], 64, [64], [64], 128, 4, 1e-3, target_kl=target_kl, masks=masks,
               seeds=list(range(seed, seed + P)))
    rng = np.random.default_rng(seed + 100)
    S = T * N
    obs = rng.standard_normal((P, S, D)).astype(np.float32)
    mk = None
    if masks:
        mk = rng.random((P, S, A)) < 0.7
        mk[np.arange(P)[:, None], np.arange(S)[None, :], rng.integers(0, A, (P, S))] = True
    nets, data = [], []
    flat0 = pop.params.data.cpu().numpy()
    for p in range(P):
        net = ActorCritic(D, A, [64], 64, [64], [64])
        sd = {k: flat0[p, off:off + int(np.prod(sh))].reshape(sh)
              for k, (off, sh) in pop.spec.state_dict_keys().items() if not k.startswith("critic.encoder.")}
        net.load_reference(sd)
        with torch.no_grad():
            lat = net.encoder(torch.tensor(obs[p]))
            lg = net.actor_head(lat)
            if mk is not None:
                lg = torch.where(torch.tensor(mk[p]), lg, torch.full_like(lg, -1e8))
            pr = torch.softmax(lg, -1).double().numpy()
            pr /= pr.sum(1, keepdims=True)
            act = np.array([rng.choice(A, p=q) for q in pr], np.int64)
            lp = torch.log_softmax(lg, -1).numpy()[np.arange(S), act]
            v = net.critic_head(lat).squeeze(-1).numpy()
        lp = (lp + rng.normal(0, 0.02, S)).astype(np.float32)
        v = (v + rng.normal(0, 0.1, S)).astype(np.float32)
        adv = (rng.standard_normal(S) * 1.5 + 0.2).astype(np.float32)
        ret = (v + rng.standard_normal(S)).astype(np.float32)
        nets.append(net)
        data.append((obs[p], act, lp, v, adv, ret, None if mk is None else mk[p]))
    t = lambda x: torch.as_tensor(np.asarray(x)).to(DEV)  # noqa: E731
    pop.obs.copy_(t(obs).view_as(pop.obs))
    pop.actions.copy_(t(np.stack([d[1] for d in data])).view_as(pop.actions))
    pop.log_probs.copy_(t(np.stack([d[2] for d in data])).view_as(pop.log_probs))
    pop.values.copy_(t(np.stack([d[3] for d in data])).view_as(pop.values))
    pop.advantages.copy_(t(np.stack([d[4] for d in data])).view_as(pop.advantages))
    pop.returns.copy_(t(np.stack([d[5] for d in data])).view_as(pop.returns))
    if mk is not None:
        pop.action_masks.copy_(t(mk.astype(np.uint8)).view_as(pop.action_masks))
    _set_stats(pop)
    return pop, nets, data


@pytest.mark.parametrize("target_kl,masks", [(None, False), (0.0035, True)])
def test_fused_learner_config2_population_vs_oracle(target_kl, masks):
    """The exact config-2 population (P=8, N=128, T=16, B=128, E=4) with the
    reference's numpy permutation stream vs oracle/ppo_learn.py per agent."""
    from agilerl_amd.population.learner import fused_learn

    torch.set_num_threads(4)
    pop, nets, data = _config2_population(target_kl, masks)
    P, S = pop.P, pop.S
    np.random.seed(1234)
    perms_h = pop.permutations().cpu().numpy()  # numpy stream, [E, P, S]
    np.random.seed(1234)
    from agilerl_amd.rng import numpy_shuffle_perms

    assert np.array_equal(perms_h, numpy_shuffle_perms(P, 4, S))
    loss = fused_learn(pop, torch.as_tensor(perms_h).to(DEV))
    torch.cuda.synchronize()
    pop.check_errors()
    got_p = pop.params.data.cpu().numpy()
    got_m, got_v = pop.opt.exp_avg.cpu().numpy(), pop.opt.exp_avg_sq.cpu().numpy()
    epochs = pop._fused.epochs_run.cpu().numpy()
    runs = []
    for p in range(P):
        obs, act, lp, v, adv, ret, mk = data[p]
        init_sd = {k: x.numpy() for k, x in nets[p].reference_state().items()}
        out = reference_learn(nets[p], None, obs, act, lp, adv, ret, v, perms_h[:, p], batch_size=128, epochs=4,
                              lr=1e-3, target_kl=target_kl, masks=mk)
        runs.append(out["epochs"])
        assert int(epochs[p]) == out["epochs"], (p, int(epochs[p]), out["epochs"])
        assert int(pop.opt.steps[p]) == out["step"]
        assert abs(float(loss[p]) - out["mean_loss"]) <= 1e-4 * abs(out["mean_loss"]) + 1e-7, p
        net64 = ActorCritic(8, 4, [64], 64, [64], [64])
        net64.load_reference(init_sd)
        o64 = reference_learn(net64.double(), None, obs, act, lp, adv, ret, v, perms_h[:, p], batch_size=128,
                              epochs=4, lr=1e-3, target_kl=target_kl, masks=mk, dtype=torch.float64)
        fl = lambda d: _flat_from_names(pop.spec, {k: t.numpy() for k, t in d.items()}, pop.spec.n_params)  # noqa
        _envelope(f"agent {p} params", got_p[p], fl(out["state"]), fl(o64["state"]))
        _envelope(f"agent {p} exp_avg", got_m[p], fl(out["exp_avg"]), fl(o64["exp_avg"]))
        _envelope(f"agent {p} exp_avg_sq", got_v[p], fl(out["exp_avg_sq"]), fl(o64["exp_avg_sq"]))
    if target_kl is not None:
        assert len(set(runs)) > 1, f"target_kl should stop agents at different epochs: {runs}"


def test_partner_stall_raises():
    """A partner workgroup that never arrives: the bounded wait sets the
    sticky error word and PPOPopulation.check_errors raises (no silently
    half-applied update reaches the caller)."""
    from agilerl_amd import _lib
    from agilerl_amd.population.learner import fused_learn

    pop, _, _ = _config2_population()
    lib = _lib.load()
    lib.agx_debug_learn_stall(1)
    try:
        fused_learn(pop)
        torch.cuda.synchronize()
    finally:
        lib.agx_debug_learn_stall(0)
    with pytest.raises(_lib.AgxError, match="partner"):
        pop.check_errors()
    pop.check_errors()  # the word was reset
    # and the next learn runs normally
    fused_learn(pop)
    torch.cuda.synchronize()
    pop.check_errors()


def test_target_kl_resyncs_global_numpy_stream():
    """With target_kl, agents stop after different numbers of epochs and the
    reference draws one np.random.shuffle per epoch run (ppo.py:836-842,
    917-918).  After learn() the global numpy state must be the state after
    exactly sum(epochs_run) shuffles from the state before the learn, so every
    later consumer of the stream (tournament, mutations, the next learn) sees
    the reference's state."""
    from agilerl_amd.rng import numpy_shuffle_perms

    pop, _, _ = _config2_population(0.0035, True)
    np.random.seed(77)
    pop.learn()
    torch.cuda.synchronize()
    pop.check_errors()
    ran = pop._fused.epochs_run.cpu().numpy()
    assert len(set(ran.tolist())) > 1 and ran.sum() < pop.P * 4, ran
    pop.sync_numpy_stream()
    got = np.random.randint(0, 2**31 - 1, 8)
    np.random.seed(77)
    numpy_shuffle_perms(1, int(ran.sum()), pop.S)
    assert np.array_equal(got, np.random.randint(0, 2**31 - 1, 8))


@pytest.mark.parametrize("bad", [2048 + 7, -3])
def test_bad_permutation_index_raises(bad):
    """A permutation index outside [0, S) (a host-side slip: the round-4
    fault was stale rows of the pinned shuffle buffer) is caught by the
    gather prologue on the device: the sticky error word gets
    AGX_LEARN_ERR_PERM, nothing is read out of bounds, and
    PPOPopulation.check_errors raises AgxError."""
    from agilerl_amd import _lib
    from agilerl_amd.population.learner import fused_learn

    pop, _, _ = _config2_population()
    E, P, S = pop.update_epochs, pop.P, pop.S
    block = np.stack([np.stack([np.random.default_rng(e * P + p).permutation(S) for p in range(P)])
                      for e in range(E)])[None].astype(np.int64)
    block[0, 1, 3, 17] = bad
    pop.set_generation_perms(block)
    fused_learn(pop)
    torch.cuda.synchronize()
    with pytest.raises(_lib.AgxError, match="permutation"):
        pop.check_errors()
    pop.check_errors()  # reset
    pop.set_generation_perms(None)
    fused_learn(pop)  # the next learn with valid shuffles runs clean
    torch.cuda.synchronize()
    pop.check_errors()
