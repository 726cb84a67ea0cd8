"""Population PPO engine on the GPU: the fused learner kernel (agx_ppo_learn)
against the plain-PyTorch fp32 learner on identical inputs and permutations,
and an end-to-end rollout -> GAE -> learn iteration."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _pop(P=3, N=16, learn_step=128, batch=64, epochs=1, seed=0, **kw):
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation

    spec = ActorCriticSpec(obs_dim=8, n_actions=4, **kw)
    pop = PPOPopulation(spec, P, N, learn_step=learn_step, batch_size=batch, lr=1e-3, update_epochs=epochs,
                        seeds=[seed + i for i in range(P)], device=DEV, fused=True)
    g = torch.Generator(device=DEV).manual_seed(seed + 99)
    pop.obs.copy_(torch.randn(pop.obs.shape, device=DEV, generator=g))
    pop.actions.copy_(torch.randint(0, 4, pop.actions.shape, device=DEV, generator=g))
    pop.rewards.copy_(torch.randn(pop.rewards.shape, device=DEV, generator=g))
    pop.dones.copy_((torch.rand(pop.dones.shape, device=DEV, generator=g) < 0.05).to(torch.uint8))
    with torch.no_grad():
        logits, value = spec.forward(pop.params.data, pop.obs.view(P, -1, 8))
        lp = torch.log_softmax(logits, -1).gather(-1, pop.actions.view(P, -1, 1)).squeeze(-1)
    pop.values.copy_(value.view_as(pop.values) + 0.1 * torch.randn(pop.values.shape, device=DEV, generator=g))
    pop.log_probs.copy_(lp.view_as(pop.log_probs) + 0.05 * torch.randn(pop.log_probs.shape, device=DEV, generator=g))
    last_obs = torch.randn(P, N, 8, device=DEV, generator=g)
    last_done = torch.zeros(P, N, dtype=torch.uint8, device=DEV)
    pop.finish_rollout(last_obs, last_done)
    return pop


def _clone_state(pop):
    return (pop.params.data.clone(), pop.opt.exp_avg.clone(), pop.opt.exp_avg_sq.clone(),
            pop.advantages.clone(), pop.opt.steps.clone())


def _restore(pop, st):
    pop.params.data.copy_(st[0])
    pop.opt.exp_avg.copy_(st[1])
    pop.opt.exp_avg_sq.copy_(st[2])
    pop.advantages.copy_(st[3])
    pop.opt.steps.copy_(st[4])


@pytest.mark.parametrize("N,learn_step,batch,epochs", [(16, 64, 64, 1), (16, 128, 64, 1), (8, 100, 32, 2),
                                                       (16, 128, 48, 1), (16, 512, 128, 2), (16, 400, 128, 1)])
def test_fused_learner_matches_torch_learner(N, learn_step, batch, epochs):
    from agilerl_amd.population.learner import fused_learn

    pop = _pop(N=N, learn_step=learn_step, batch=batch, epochs=epochs)
    st = _clone_state(pop)
    perms = pop.permutations()
    loss_t = pop._learn_torch(perms).clone()
    p_torch = pop.params.data.clone()
    m_torch = pop.opt.exp_avg.clone()
    _restore(pop, st)
    loss_f = fused_learn(pop, perms).clone()
    torch.cuda.synchronize()
    p0 = st[0]
    d_t = (p_torch - p0)
    d_f = (pop.params.data - p0)
    # Gradients are what the kernels compute: the Adam first moment carries
    # them.  The parameter update m/(sqrt(v)+eps) is ill-conditioned where
    # |g| ~ eps, so it is checked on 99.9% of the entries only.
    m_f, m_t = pop.opt.exp_avg.cpu().numpy(), m_torch.cpu().numpy()
    np.testing.assert_allclose(m_f, m_t, rtol=2e-3, atol=1e-5 * np.abs(m_t).max())
    scale = d_t.abs().max().item()
    assert scale > 0
    bad = ((d_f - d_t).abs() > 2e-3 * scale).float().mean().item()
    assert bad <= 1e-3, bad
    np.testing.assert_allclose(loss_f.cpu().numpy(), loss_t.cpu().numpy(), rtol=1e-4, atol=1e-7)


def test_fused_learner_single_update_tight():
    """One minibatch, one epoch: gradients and the single Adam step agree
    closely (only summation order differs)."""
    from agilerl_amd.population.learner import fused_learn

    pop = _pop(N=32, learn_step=64, batch=64, epochs=1, seed=5)
    st = _clone_state(pop)
    perms = pop.permutations()
    pop._learn_torch(perms)
    g_torch = pop.opt.grads.clone()  # clipped gradients of the single update
    m_t = pop.opt.exp_avg.clone()
    _restore(pop, st)
    fused_learn(pop, perms)
    torch.cuda.synchronize()
    # first Adam step: exp_avg = 0.1 * g_clipped exactly
    np.testing.assert_allclose(pop.opt.exp_avg.cpu().numpy(), m_t.cpu().numpy(), rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose((pop.opt.exp_avg / 0.1).cpu().numpy(), g_torch.cpu().numpy(), rtol=1e-3, atol=1e-8)


def test_runner_iteration_end_to_end():
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.hpo.population_sync import PopulationSync
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    spec = ActorCriticSpec(obs_dim=8, n_actions=4)
    pop = PPOPopulation(spec, 4, 32, learn_step=256, batch_size=64, update_epochs=2, device=DEV)
    runner = PopulationRunner(pop, SyntheticVecEnv(4 * 32, seed=3))
    p0 = pop.params.data.clone()
    for _ in range(2):
        loss = runner.iteration()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all()
    assert not torch.equal(p0, pop.params.data)
    assert runner.env_steps == 2 * 4 * 32 * 8
    # actions in range, stored dones match the env's
    assert int(pop.actions.min()) >= 0 and int(pop.actions.max()) < 4
    sync = PopulationSync(pop, runner, seed=1)
    parents = sync.generation()
    assert len(parents) == 4 and all(0 <= p < 4 for p in parents)


def test_generation_behind_queued_learner_matches_synchronous():
    """PopulationSync.generation straight after iteration() (the learner still
    queued): fitness read behind the rollout only, parent rows cloned in stream
    order after the learner.  Must equal the synchronous computation: the
    same parents from the same fitness, new row j = learned row parents[j]."""
    import numpy as np

    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.hpo.population_sync import PopulationSync
    from agilerl_amd.hpo.tournament import select_parents
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    def make():
        spec = ActorCriticSpec(obs_dim=8, n_actions=4)
        # two populations interleaved: each draws its minibatch orders from its
        # own (identically seeded) device generator, not the shared numpy stream
        pop = PPOPopulation(spec, 6, 32, learn_step=256, batch_size=64, update_epochs=2, device=DEV,
                            seeds=list(range(6)), perm_source="device")
        return pop, PopulationRunner(pop, SyntheticVecEnv(6 * 32, seed=7, p_done=0.2))

    a_pop, a_run = make()
    b_pop, b_run = make()
    sync = PopulationSync(a_pop, a_run, seed=3)
    for g in range(3):
        a_run.iteration()
        parents = sync.generation()  # no host sync before it
        b_run.iteration()
        torch.cuda.synchronize()
        r = b_run
        fit = torch.where(r.episodes > 0, r.episode_return_sum / r.episodes.clamp(min=1).double(),
                          torch.full_like(r.episode_return_sum, -1e9)).cpu().numpy()
        b_run.reset_episode_stats()
        if g == 0:
            rng = np.random.RandomState(3)
        _, exp = select_parents([np.asarray([f]) for f in fit], 2, True, 1, rng=rng)
        assert parents == exp
        idx = torch.as_tensor(exp, device=DEV)
        for buf in (b_pop.params.data, b_pop.opt.exp_avg, b_pop.opt.exp_avg_sq):
            buf.copy_(buf.index_select(0, idx))
        torch.cuda.synchronize()
        assert torch.equal(a_pop.params.data, b_pop.params.data)
        assert torch.equal(a_pop.opt.exp_avg_sq, b_pop.opt.exp_avg_sq)


@pytest.mark.parametrize("P,N", [(3, 16), (2, 45), (8, 1)])
def test_policy_step_matches_torch_forward(P, N):
    """agx_ppo_act vs the plain-PyTorch forward of the stacked networks:
    values, entropy, log-prob of the chosen action; greedy mode = argmax."""
    from agilerl_amd.population.learner import policy_step
    from agilerl_amd.population.nets import categorical

    pop = _pop(P=P, N=N, learn_step=4 * N, batch=4 * N)
    desc = pop.fused_descriptor()
    assert desc is not None
    obs = torch.randn(P, N, 8, device=DEV)
    logits, value = pop.spec.forward(pop.params.data, obs)
    logp_all, ent = categorical(logits)
    outs = dict(actions=torch.empty(P, N, dtype=torch.int64, device=DEV),
                log_probs=torch.empty(P, N, device=DEV), values=torch.empty(P, N, device=DEV),
                entropy=torch.empty(P, N, device=DEV), actions_flat=torch.empty(P * N, dtype=torch.int64, device=DEV))
    for sample in (False, True):
        policy_step(pop, desc, obs, N * 8, sample=sample, counter=7, out_agent_stride=N, **outs)
        torch.cuda.synchronize()
        a = outs["actions"]
        assert torch.equal(a.view(-1), outs["actions_flat"])
        if not sample:
            assert torch.equal(a, logits.argmax(-1))
        lp = logp_all.gather(-1, a.unsqueeze(-1)).squeeze(-1)
        torch.testing.assert_close(outs["log_probs"], lp, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(outs["values"], value, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(outs["entropy"], ent, rtol=1e-4, atol=1e-5)


def test_policy_step_sampling_distribution():
    """Gumbel-max draws follow softmax(logits): chi-square over many counters."""
    from agilerl_amd.population.learner import policy_step

    P, N = 2, 256
    pop = _pop(P=P, N=N, learn_step=N, batch=N)
    desc = pop.fused_descriptor()
    obs = torch.randn(P, 1, 8, device=DEV).expand(P, N, 8).contiguous()
    probs = torch.softmax(pop.spec.forward(pop.params.data, obs[:, :1])[0], -1)[:, 0]  # [P, A]
    counts = torch.zeros(P, 4, device=DEV)
    act = torch.empty(P, N, dtype=torch.int64, device=DEV)
    R = 64
    for c in range(R):
        policy_step(pop, desc, obs, N * 8, sample=True, counter=1000 + c, actions=act, out_agent_stride=N)
        counts += torch.nn.functional.one_hot(act, 4).sum(1).float()
    n = R * N
    exp = probs * n
    chi2 = (((counts - exp) ** 2) / exp).sum(-1).cpu().numpy()
    assert (chi2 < 25.0).all(), (chi2, probs)  # 3 dof: P(chi2 > 25) ~ 1.6e-5


def test_policy_step_rejects_unsupported_shape():
    from agilerl_amd import _lib
    from agilerl_amd.population.learner import AgxPPONet

    d = AgxPPONet()
    d.obs_dim, d.n_actions, d.n_enc = 7, 3, 2
    lib = _lib.load()
    rc = lib.agx_ppo_act(ctypes_byref(d), 1, 1, None, None, 0, None, 0, 0, 0, 0, None, None, None, None, 0, None,
                         None, None)
    assert rc != 0


def ctypes_byref(x):
    import ctypes

    return ctypes.byref(x)


@pytest.mark.parametrize("split", ["1", "2", "4", "8", "8wt", "4x16", "1x16"])
def test_fused_learner_partner_split_consistent(split, monkeypatch):
    """The learner spreads an agent's sub-batches (16 or 32 rows) over K
    partner workgroups that reduce-scatter partial gradients through HBM; K
    and the sub-batch rows only reorder the f32 gradient sums.
    One update: the first Adam moment (1 - b1) * clip * g agrees with the torch
    learner to f32 reordering noise.  Eight updates: Adam's sign-like first
    steps turn last-bit differences of near-zero gradients into full lr steps,
    so a few moments drift (the envelope tests in test_learner_parity_gpu.py
    bound that drift against fp64); the bulk and the loss still agree."""
    from agilerl_amd.population.learner import fused_learn

    if split.endswith("wt"):  # partners exchange through write-through stores (any XCD placement)
        split = split[:-2]
        monkeypatch.setenv("AGX_LEARN_WRITETHROUGH", "1")
    k, _, sb = split.partition("x")
    monkeypatch.setenv("AGX_LEARN_SPLIT", k)
    if sb:
        monkeypatch.setenv("AGX_LEARN_SB", sb)  # 16-row sub-batches, several per partner
    for learn_step, epochs in ((128, 1), (512, 2)):
        np.random.seed(learn_step)  # the minibatch shuffles: fixed, whatever ran before
        pop = _pop(P=4, N=16, learn_step=learn_step, batch=128, epochs=epochs, seed=11)
        st = _clone_state(pop)
        perms = pop.permutations()
        loss_t = pop._learn_torch(perms).clone()
        m_t = pop.opt.exp_avg.clone().cpu().numpy()
        _restore(pop, st)
        loss_f = fused_learn(pop, perms).clone()
        torch.cuda.synchronize()
        assert not pop._fused.timed_out(pop)
        m_f = pop.opt.exp_avg.cpu().numpy()
        scale = np.abs(m_t).max()
        np.testing.assert_allclose(loss_f.cpu().numpy(), loss_t.cpu().numpy(), rtol=1e-4, atol=1e-7)
        if epochs == 1:
            np.testing.assert_allclose(m_f, m_t, rtol=1e-4, atol=1e-6 * scale)
        else:
            bad = np.abs(m_f - m_t) > 2e-3 * np.abs(m_t) + 1e-5 * scale
            assert bad.mean() < 2e-3, f"{bad.sum()} of {bad.size} moments off"
            assert np.abs(m_f - m_t).max() < 1e-3 * scale


@pytest.mark.parametrize("fused", [True, False])
def test_collect_fills_rollout_like_the_reference_loop(fused):
    """One collect() against a replayed copy of the (action-independent)
    synthetic env: obs / reward / done land in the right slots (done of step
    t at slot t, on_policy.py:137-142; last_done = term), stored log-probs /
    values equal the torch forward of the stored obs and actions, and the
    episode accounting matches a recomputation from the stored rewards."""
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.population.nets import ActorCriticSpec, categorical
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    P, N = 3, 40
    spec = ActorCriticSpec(obs_dim=8, n_actions=4)
    pop = PPOPopulation(spec, P, N, learn_step=8 * N, batch_size=64, device=DEV, fused=fused)
    env = SyntheticVecEnv(P * N, seed=5, p_done=0.2)
    ref = SyntheticVecEnv(P * N, seed=5, p_done=0.2)
    runner = PopulationRunner(pop, env)
    T = pop.T
    for rep in range(2):
        runner.collect()
        torch.cuda.synchronize()
        if rep == 0:
            o, _ = ref.reset()
            exp_obs = [o.copy()]
        else:
            exp_obs = [exp_last]
        exp_r, exp_d = [], []
        for t in range(T):
            o, r, term, trunc, _ = ref.step(np.zeros(P * N, dtype=np.int64))
            exp_obs.append(o.copy())
            exp_r.append(r.copy())
            exp_d.append(term | trunc)
        exp_last = exp_obs[-1]
        got_obs = pop.obs.cpu().numpy()  # [P, T, N, D]
        for t in range(T):
            np.testing.assert_array_equal(got_obs[:, t].reshape(P * N, 8), exp_obs[t])
            np.testing.assert_array_equal(pop.rewards[:, t].cpu().numpy().reshape(-1), exp_r[t])
            np.testing.assert_array_equal(pop.dones[:, t].cpu().numpy().reshape(-1).astype(bool), exp_d[t])
        np.testing.assert_array_equal(runner.last_obs.cpu().numpy().reshape(P * N, 8), exp_obs[T])
        np.testing.assert_array_equal(runner.last_done.cpu().numpy().reshape(-1).astype(bool), term)
    # stored log-probs / values follow the stored (obs, action) pairs
    logits, value = spec.forward(pop.params.data, pop.obs.view(P, -1, 8))
    logp_all, _ = categorical(logits)
    lp = logp_all.gather(-1, pop.actions.view(P, -1, 1)).squeeze(-1)
    torch.testing.assert_close(pop.log_probs.view(P, -1), lp, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(pop.values.view(P, -1), value, rtol=1e-4, atol=1e-5)
    assert int(pop.actions.min()) >= 0 and int(pop.actions.max()) < 4
    if fused:  # bootstrap value computed by the final rollout-step launch
        _, lv = spec.forward(pop.params.data, runner.last_obs)
        torch.testing.assert_close(runner.last_value, lv, rtol=1e-4, atol=1e-5)


def test_collect_episode_accounting():
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    P, N = 2, 33
    spec = ActorCriticSpec(obs_dim=8, n_actions=4)
    pop = PPOPopulation(spec, P, N, learn_step=6 * N, batch_size=64, device=DEV)
    runner = PopulationRunner(pop, SyntheticVecEnv(P * N, seed=9, p_done=0.25))
    R, D = [], []
    for _ in range(3):
        runner.collect()
        torch.cuda.synchronize()
        R.append(pop.rewards.cpu().numpy())
        D.append(pop.dones.cpu().numpy().astype(bool))
    r = np.concatenate(R, axis=1).reshape(P, -1, N)  # [P, 3T, N]
    d = np.concatenate(D, axis=1).reshape(P, -1, N)
    score = np.zeros((P, N), np.float32)
    ret = np.zeros((P, N))
    eps = np.zeros((P, N), np.int64)
    for t in range(r.shape[1]):
        score = score + r[:, t]
        ret += np.where(d[:, t], score, 0.0)
        eps += d[:, t]
        score = np.where(d[:, t], 0.0, score).astype(np.float32)
    np.testing.assert_array_equal(runner.episodes.cpu().numpy(), eps.sum(1))
    np.testing.assert_allclose(runner.episode_return_sum.cpu().numpy(), ret.sum(1), rtol=1e-6)
    np.testing.assert_allclose(runner.scores.view(P, N).cpu().numpy(), score, rtol=1e-6, atol=1e-6)


def _runner_pair(monkeypatch, persistent, P=3, N=40, seed=5, perm_source="device"):
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    monkeypatch.setenv("AGX_PERSISTENT_ROLLOUT", "1" if persistent else "0")
    spec = ActorCriticSpec(obs_dim=8, n_actions=4)
    pop = PPOPopulation(spec, P, N, learn_step=8 * N, batch_size=64, update_epochs=2, device=DEV,
                        seeds=list(range(P)), fused=True, perm_source=perm_source)
    runner = PopulationRunner(pop, SyntheticVecEnv(P * N, seed=seed, p_done=0.2))
    assert runner.persistent == persistent
    return pop, runner


@pytest.mark.parametrize("perm_source", ["device", "numpy"])
def test_persistent_rollout_matches_per_step_launches(monkeypatch, perm_source):
    """ONE persistent launch per rollout (host-paced through the coherent
    control block) produces bit-identical rollouts, bootstrap values, episode
    statistics and — after learn() — parameters to one launch per step."""
    a_pop, a_run = _runner_pair(monkeypatch, True, perm_source=perm_source)
    b_pop, b_run = _runner_pair(monkeypatch, False, perm_source=perm_source)
    for _ in range(3):
        for run, seed in ((a_run, 77), (b_run, 77)):
            if perm_source == "numpy":  # each run's own copy of the global stream
                st = getattr(run, "_np_state", None)
                np.random.set_state(st) if st is not None else np.random.seed(seed)
            run.iteration()
            if perm_source == "numpy":
                run.pop.discard_prefetch()
                run._np_state = np.random.get_state()
        torch.cuda.synchronize()
        for name in ("obs", "actions", "log_probs", "values", "rewards", "dones", "advantages", "returns"):
            assert torch.equal(getattr(a_pop, name), getattr(b_pop, name)), name
        assert torch.equal(a_run.last_value, b_run.last_value)
        assert torch.equal(a_run.last_done, b_run.last_done)
        assert torch.equal(a_run.episodes, b_run.episodes)
        assert torch.equal(a_run.episode_return_sum, b_run.episode_return_sum)
        assert torch.equal(a_pop.params.data, b_pop.params.data)
    assert a_pop.act_counter == b_pop.act_counter
    assert int(a_run.ctl_h.view(torch.int32)[1]) == 0  # no workgroup timed out


def test_persistent_rollout_abort_releases_kernel(monkeypatch):
    """An env that raises mid-rollout: the runner releases the waiting
    workgroups (abort sequence), re-arms the control block, and the next
    collect() runs normally."""
    pop, run = _runner_pair(monkeypatch, True)
    run.collect()
    real = run._env_step
    calls = {"n": 0}

    def flaky():
        calls["n"] += 1
        if calls["n"] == 3:
            raise RuntimeError("env worker died")
        real()

    run._env_step = flaky
    with pytest.raises(RuntimeError, match="env worker died"):
        run.collect()
    run._env_step = real
    run.collect()
    torch.cuda.synchronize()
    assert run.seq_base == pop.T + 1
    assert int(pop.actions.min()) >= 0 and int(pop.actions.max()) < 4


def test_persistent_rollout_oversized_grid_falls_back():
    """A grid the GPU cannot hold at once (every persistent workgroup must be
    resident: the host paces them in lock step) is refused with
    AGX_EUNSUPPORTED, and PopulationRunner takes the per-step launches
    instead of deadlocking until the timeout."""
    import ctypes

    from agilerl_amd import _lib
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.population.runner import PopulationRunner

    pop0 = _pop(P=2, N=32)
    desc = pop0.fused_descriptor()
    lib = _lib.load()
    cap = int(lib.agx_rollout_max_workgroups(ctypes.byref(desc)))
    assert cap >= 256  # at least one workgroup per CU
    P = 2
    N = 32 * (cap // P + 1)
    assert lib.agx_rollout_workgroups(P, N) > cap
    pop = _pop(P=P, N=N, learn_step=2 * N, batch=N)
    run = PopulationRunner(pop, SyntheticVecEnv(P * N, seed=3))
    assert not run.persistent
    run.iteration()
    torch.cuda.synchronize()
    assert int(pop.actions.min()) >= 0 and int(pop.actions.max()) < 4
    assert torch.isfinite(pop.params.data).all()
    # and the ABI itself refuses the oversized persistent launch
    from agilerl_amd.population.runner import AgxRolloutIO

    ios = (AgxRolloutIO * 2)()
    for t in range(2):
        ios[t].stage_obs = pop.obs.data_ptr()
    ctl = torch.zeros(4096, dtype=torch.uint8)
    args = torch.zeros(4096, dtype=torch.uint8)
    rc = lib.agx_ppo_rollout_persistent(ctypes.byref(desc), P, N, pop.params.data.data_ptr(), ios, 2, 0, 1, 0,
                                        args.data_ptr(), ctl.data_ptr(), 1.0, _lib.stream())
    assert rc == -3, rc  # AGX_EUNSUPPORTED, nothing launched
    assert b"resident" in lib.agx_last_error()


class _FixedEpisodeEnv:
    """Env e pays c[e] per step and terminates every L[e] steps, whatever
    the actions: PPO.test's fitness (ppo.py:1113-1289) is then known exactly."""

    def __init__(self, P, N, seed=0):
        rng = np.random.default_rng(seed)
        self.num_envs = P * N
        self.L = rng.integers(1, 12, P * N)
        self.c = rng.normal(size=P * N)
        self.obs = rng.standard_normal((P * N, 8)).astype(np.float32)
        self.t = np.zeros(P * N, dtype=np.int64)
        self.seen = []

    def reset(self, **kw):
        self.t[:] = 0
        return self.obs.copy(), {}

    def step(self, actions):
        a = np.asarray(actions)
        assert a.shape == (self.num_envs,) and a.min() >= 0 and a.max() < 4
        self.seen.append(a.copy())
        self.t += 1
        term = self.t % self.L == 0
        return self.obs.copy(), self.c.astype(np.float32), term, np.zeros_like(term), {}


@pytest.mark.parametrize("max_steps", [None, 5])
def test_population_evaluate_matches_test_semantics(max_steps):
    """PopulationRunner.evaluate = agent.test for every agent at once: each
    env's first finished episode (or the max_steps cut) counts, mean over the
    agent's envs, then over the loop passes; the runner resumes from a reset."""
    from agilerl_amd.population.runner import PopulationRunner

    P, N = 3, 16
    pop = _pop(P=P, N=N)
    env = _FixedEpisodeEnv(P, N)
    runner = PopulationRunner(pop, env)
    fit = runner.evaluate(loop=2, max_steps=max_steps)
    steps = env.L if max_steps is None else np.minimum(env.L, max_steps)
    exp = (env.c.astype(np.float32).astype(np.float64) * steps).reshape(P, N).mean(1)
    np.testing.assert_allclose(fit, exp, rtol=1e-12)
    assert len(env.seen) == 2 * int(steps.max())
    # actions are the policy's: not constant across envs
    assert len(np.unique(np.concatenate(env.seen))) > 1


@pytest.mark.parametrize("source", ["numpy", "device"])
def test_permutation_prefetch_keeps_the_draw_sequence(monkeypatch, source):
    """The runner draws the next learn's permutations ahead (numpy: host
    shuffles after pacing the rollout; device: a side stream); the results
    are bit-identical to drawing them at the start of every learn(), and the
    global numpy stream ends where it would have."""
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.hpo.population_sync import PopulationSync
    from agilerl_amd.population.runner import PopulationRunner

    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("AGX_PREFETCH_PERMS", flag)
        np.random.seed(11)
        pop = _pop(P=3, N=32, learn_step=256, batch=64, epochs=2)
        pop.perm_source = source
        runner = PopulationRunner(pop, SyntheticVecEnv(3 * 32, seed=4, p_done=0.1))
        sync = PopulationSync(pop, runner, seed=None)  # tournament draws from the GLOBAL numpy stream
        for i in range(4):
            runner.iteration()
            if i == 1:
                sync.generation()  # discards a prefetched numpy draw first
        explicit = pop.permutations()  # an explicit draw takes the prefetched one
        torch.cuda.synchronize()
        out.append((pop.params.data.clone(), pop.opt.exp_avg.clone(), explicit.clone(),
                    torch.as_tensor(np.random.random(4))))
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


def test_env_exception_mid_rollout_leaves_learner_state_untouched(monkeypatch):
    """The pipelined iteration queues GAE and the learner behind the
    persistent rollout before the host paces it.  An env that raises mid
    rollout aborts the rollout; the queued learner reads the control block's
    timeout word when it starts and skips: parameters, both Adam moments and
    the step counts stay bit-identical, and the next iteration runs."""
    pop, run = _runner_pair(monkeypatch, True)
    run.iteration()
    torch.cuda.synchronize()
    before = [t.clone() for t in (pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq, pop.opt.steps)]
    real = run._env_step
    calls = {"n": 0}

    def flaky():
        calls["n"] += 1
        if calls["n"] == 4:
            raise RuntimeError("env worker died")
        real()

    run._env_step = flaky
    with pytest.raises(RuntimeError, match="env worker died"):
        run.iteration()
    torch.cuda.synchronize()
    pop.check_errors()
    after = (pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq, pop.opt.steps)
    for name, a, b in zip(("params", "exp_avg", "exp_avg_sq", "steps"), before, after):
        assert torch.equal(a, b), name
    run._env_step = real
    run.iteration()
    torch.cuda.synchronize()
    pop.check_errors()
    assert not torch.equal(before[0], pop.params.data)  # the next learn does update
    assert torch.equal(pop.opt.steps, before[3] + 2 * pop.n_minibatches())


def test_env_that_synchronizes_the_device_completes(monkeypatch):
    """An env whose step waits for the device (torch.cuda.synchronize()) would
    stall a persistent rollout until its timeout (the device waits for the
    host).  Under the default "auto" rule such an env — one that does not
    declare agx_device_free — gets one launch per vector step, and the
    iteration completes."""
    import time

    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    class SyncingEnv(SyntheticVecEnv):
        agx_device_free = False

        def step(self, actions, **kw):
            torch.cuda.synchronize()
            return super().step(actions, **kw)

    monkeypatch.delenv("AGX_PERSISTENT_ROLLOUT", raising=False)
    monkeypatch.setenv("AGX_ROLLOUT_TIMEOUT", "5")
    P, N = 2, 32
    pop = PPOPopulation(ActorCriticSpec(obs_dim=8, n_actions=4), P, N, learn_step=8 * N, batch_size=64,
                        update_epochs=2, device=DEV, fused=True)
    run = PopulationRunner(pop, SyncingEnv(P * N, seed=1))
    assert not run.persistent
    assert PopulationRunner(pop, SyntheticVecEnv(P * N, seed=1)).persistent  # device-free envs keep the fast path
    t0 = time.perf_counter()
    for _ in range(2):
        run.iteration()
    torch.cuda.synchronize()
    pop.check_errors()
    assert time.perf_counter() - t0 < 4.0
    assert torch.isfinite(pop.params.data).all()


@pytest.mark.parametrize("max_steps", [None, 13])
def test_persistent_evaluation_matches_per_step_launches(monkeypatch, max_steps):
    """The evaluation pass as ONE persistent launch (agx_ppo_eval_persistent,
    host-paced, ended by AGX_ROLLOUT_STOP once every env has finished) gives
    the fitness of one policy-step launch per vector step bit for bit — the
    same Philox counters, the same first-finished-episode tally — also when
    a pass needs several launches (chunk of 7 steps here); the rollout after
    it starts from a reset, as after the per-step pass."""
    from agilerl_amd.population import runner as R

    monkeypatch.setattr(R, "_EVAL_CHUNK", 7)
    out = []
    for persistent in (True, False):
        pop, run = _runner_pair(monkeypatch, persistent)
        run.env.max_episode_steps = 30
        run.iteration()
        fit = run.evaluate(loop=2, max_steps=max_steps)
        run.iteration()
        torch.cuda.synchronize()
        out.append((fit, pop.params.data.clone(), pop.obs.clone()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])
    assert np.all(np.isfinite(out[0][0]))


def test_engine_evaluates_groups_like_their_runners(monkeypatch):
    """A population split into groups (a learn_step mutation here): the
    engine's evaluation gives each group the fitness of its own runner's
    pass (the groups' samples depend only on their agents' counters)."""
    from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv
    from agilerl_amd.population.engine import PopulationEngine

    P, N = 4, 32
    pop, _ = _runner_pair(monkeypatch, True, P=P, N=N)
    envs = [SyntheticVecEnv(N, seed=10 + j, p_done=0.1, max_episode_steps=25) for j in range(P)]
    views = [type("V", (), {"learn_step": pop.T * pop.N})() for _ in range(P)]
    eng = PopulationEngine(pop, views, StackedVecEnv(envs))
    states = eng.local_states()
    states[1].learn_step = states[1].learn_step // 2
    states[3].learn_step = states[3].learn_step // 2
    eng.regroup(states)
    assert len(eng.groups) == 2
    eng.train(2 * pop.T * pop.N)
    fit = eng.evaluate(1, None)
    # the same evaluation round, group by group
    eng._eval_calls -= 1
    alone = [0.0] * P
    for g in eng.groups:
        g.pop.eval_rounds = eng._eval_calls  # runner.evaluate counts this round in
        f = g.runner.evaluate(loop=1, max_steps=None)
        for r, slot in enumerate(g.slots):
            alone[slot] = float(f[r])
    assert fit == alone


@pytest.mark.parametrize("mixed", [False, True])
def test_groups_paced_together_train_like_one_after_another(monkeypatch, mixed):
    """Groups of one population (a learn_step split; with ``mixed`` also an
    architecture-mutated network) trained with their rollouts paced together
    (PopulationEngine._train_paced_together) end with the parameters, Adam
    state and losses of the groups trained one iteration after another."""
    from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv
    from agilerl_amd.population.engine import PopulationEngine
    from agilerl_amd.population.nets import ActorCriticSpec

    out = []
    for together in ("1", "0"):
        monkeypatch.setenv("AGX_TRAIN_TOGETHER", together)
        P, N = 4, 32
        pop, _ = _runner_pair(monkeypatch, True, P=P, N=N)
        envs = [SyntheticVecEnv(N, seed=50 + j, p_done=0.05, max_episode_steps=30) for j in range(P)]
        views = [type("V", (), {"learn_step": pop.T * pop.N})() for _ in range(P)]
        eng = PopulationEngine(pop, views, StackedVecEnv(envs))
        states = eng.local_states()
        states[1].learn_step = states[1].learn_step // 2
        states[3].learn_step = states[3].learn_step // 2
        if mixed:
            mut = ActorCriticSpec(obs_dim=8, n_actions=4, encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64])
            g = torch.Generator(device=DEV).manual_seed(9)
            for j in (2, 3):
                st = states[j]
                st.spec = mut
                st.params = 0.1 * torch.randn(mut.n_params, device=DEV, generator=g)
                st.exp_avg = torch.zeros(mut.n_params, device=DEV)
                st.exp_avg_sq = torch.zeros(mut.n_params, device=DEV)
        eng.regroup(states)
        assert len(eng.groups) == (4 if mixed else 2)
        losses = []
        for _ in range(2):
            losses += eng.train(4 * pop.T * pop.N)
        torch.cuda.synchronize()
        st = eng.local_states()
        out.append(([s.params.cpu() for s in st], [s.exp_avg.cpu() for s in st], [s.step for s in st],
                    [np.asarray(x) for x in losses]))
    (pa, ma, sa, la), (pb, mb, sb, lb) = out
    assert sa == sb
    for x, y in zip(pa + ma, pb + mb):
        assert torch.equal(x, y)
    assert len(la) == len(lb) and all(np.array_equal(x, y) for x, y in zip(la, lb))


def test_engine_evaluates_mixed_shapes_in_one_launch(monkeypatch):
    """Groups of different networks (the compiled shape and an architecture-
    mutated one): the engine evaluates all agents in ONE persistent launch
    (agx_ppo_eval_multi_persistent, each agent on its own network) with the
    fitness of each group's own pass, and that pass equals one policy-step
    launch per vector step of the evaluation layer list."""
    from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv
    from agilerl_amd.population.engine import PopulationEngine
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.runner import population_eval_ok

    P, N = 4, 32
    pop, _ = _runner_pair(monkeypatch, True, P=P, N=N)
    envs = [SyntheticVecEnv(N, seed=30 + j, p_done=0.08, max_episode_steps=40) for j in range(P)]
    views = [type("V", (), {"learn_step": pop.T * pop.N})() for _ in range(P)]
    eng = PopulationEngine(pop, views, StackedVecEnv(envs))
    states = eng.local_states()
    mut = ActorCriticSpec(obs_dim=8, n_actions=4, encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64])
    g = torch.Generator(device=DEV).manual_seed(4)
    for j in (1, 3):
        st = states[j]
        st.spec = mut
        st.params = 0.1 * torch.randn(mut.n_params, device=DEV, generator=g)
        st.exp_avg = torch.zeros(mut.n_params, device=DEV)
        st.exp_avg_sq = torch.zeros(mut.n_params, device=DEV)
    eng.regroup(states)
    assert len(eng.groups) == 2
    runners = [gr.runner for gr in eng.groups]
    import os

    # AGX_GRAPH_FEW=0 (the general form only): each group's own pass instead
    assert population_eval_ok(runners) == (os.environ.get("AGX_GRAPH_FEW", "1") != "0")
    fit = eng.evaluate(1, None)
    assert all(np.isfinite(fit))
    eng._eval_calls -= 1
    alone = [0.0] * P
    for gr in eng.groups:
        gr.pop.eval_rounds = eng._eval_calls
        f = gr.runner.evaluate(loop=1, max_steps=None)
        for r, slot in enumerate(gr.slots):
            alone[slot] = float(f[r])
    assert fit == alone
    # one group's pass, persistent vs one launch per step
    gr = eng.groups[1]
    persistent = gr.runner.evaluate(loop=1, max_steps=None)
    monkeypatch.setattr(gr.runner, "persistent", False)
    monkeypatch.setattr(gr.runner, "graph_persistent", False)
    gr.pop.eval_rounds -= 1
    stepped = gr.runner.evaluate(loop=1, max_steps=None)
    np.testing.assert_array_equal(persistent, stepped)


@pytest.mark.parametrize("evaluate", [False, True])
def test_graph_persistent_rollout_matches_per_step_launches(monkeypatch, evaluate):
    """A mutated (runtime-shape) network: ONE persistent launch per rollout
    (agx_ppo_rollout_graph_persistent) gives the rollout, bootstrap values,
    episode statistics and — after the runtime-shape learn() — parameters of
    one agx_ppo_act_graph launch per step, bit for bit; so does the
    persistent evaluation (agx_ppo_eval_graph_persistent)."""
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    out = []
    for persistent in (True, False):
        monkeypatch.setenv("AGX_PERSISTENT_ROLLOUT", "1" if persistent else "0")
        spec = ActorCriticSpec(obs_dim=8, n_actions=4, encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64])
        P, N = 3, 40
        pop = PPOPopulation(spec, P, N, learn_step=8 * N, batch_size=64, update_epochs=2, device=DEV,
                            seeds=list(range(P)), fused=True, perm_source="device")
        assert pop.fused_descriptor() is None and pop.learn_descriptor() is not None
        run = PopulationRunner(pop, SyntheticVecEnv(P * N, seed=5, p_done=0.2, max_episode_steps=30))
        assert run.graph_persistent == persistent and not run.persistent
        fit = None
        for i in range(3):
            run.iteration()
            if evaluate and i == 1:
                fit = run.evaluate(loop=1, max_steps=None)
        torch.cuda.synchronize()
        out.append([pop.obs.clone(), pop.actions.clone(), pop.log_probs.clone(), pop.values.clone(),
                    pop.rewards.clone(), pop.dones.clone(), run.last_value.clone(), run.episodes.clone(),
                    pop.params.data.clone(), pop.opt.exp_avg.clone()])
        if evaluate:
            out[-1].append(torch.as_tensor(fit))
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


def _many_group_states(eng, pop):
    """Mutate a population of 8 slots into 7 groups: the compiled shape at
    two learn_steps and five runtime shapes (more groups than HIP's default 4
    hardware queues per process)."""
    from agilerl_amd.population.nets import ActorCriticSpec

    states = eng.local_states()
    shapes = [dict(encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64]),
              dict(encoder_hidden=[48], latent_dim=32),
              dict(encoder_hidden=[64, 32], latent_dim=40),
              dict(encoder_hidden=[96], latent_dim=24, critic_hidden=[48]),
              dict(encoder_hidden=[40], latent_dim=64, actor_hidden=[32])]
    g = torch.Generator(device=DEV).manual_seed(17)
    for j, kw in zip((2, 3, 4, 5, 6), shapes):
        spec = ActorCriticSpec(obs_dim=8, n_actions=4, **kw)
        st = states[j]
        st.spec = spec
        st.params = 0.1 * torch.randn(spec.n_params, device=DEV, generator=g)
        st.exp_avg = torch.zeros(spec.n_params, device=DEV)
        st.exp_avg_sq = torch.zeros(spec.n_params, device=DEV)
    states[1].learn_step = states[1].learn_step // 2
    states[7].learn_step = states[7].learn_step // 2
    return states


@pytest.mark.parametrize("budget", ["fits", "exceeded"])
def test_more_groups_than_hardware_queues_train_and_evaluate(monkeypatch, budget):
    """7 groups (5 runtime shapes + the compiled shape at two rollout lengths)
    > HIP's default 4 hardware queues (the package raises it to 8; either way
    groups share queues with the main and evaluation streams): one generation's training with the groups' persistent
    rollouts paced together (or, when the co-resident budget of rollouts +
    partnered learners exceeds the CUs, one group after another) and the
    population-wide evaluation complete (no agx_host_wait timeout: only
    launches whose workgroups are ALL resident are paced) and equal the
    one-group-after-another run bit for bit."""
    from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv
    from agilerl_amd.population.engine import PopulationEngine

    out = []
    for together in ("1", "0"):
        monkeypatch.setenv("AGX_TRAIN_TOGETHER", together)
        P, N = 8, 32
        pop, _ = _runner_pair(monkeypatch, True, P=P, N=N)
        envs = [SyntheticVecEnv(N, seed=70 + j, p_done=0.05, max_episode_steps=30) for j in range(P)]
        views = [type("V", (), {"learn_step": pop.T * pop.N})() for _ in range(P)]
        eng = PopulationEngine(pop, views, StackedVecEnv(envs))
        eng.regroup(_many_group_states(eng, pop))
        assert len(eng.groups) == 7
        if budget == "exceeded":
            monkeypatch.setattr(eng, "_cus", eng.co_resident_demand() - 1, raising=False)
        if together == "1":
            assert eng._paced_together() == (budget == "fits")
        losses = eng.train(2 * pop.T * pop.N)
        fit = eng.evaluate(1, None)
        torch.cuda.synchronize()
        for gr in eng.groups:
            gr.pop.check_errors()
        st = eng.local_states()
        out.append(([s.params.cpu() for s in st], [s.step for s in st], [np.asarray(x) for x in losses], fit))
    (pa, sa, la, fa), (pb, sb, lb, fb) = out
    assert sa == sb and fa == fb and all(np.isfinite(fa))
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
    assert len(la) == len(lb) and all(np.array_equal(x, y) for x, y in zip(la, lb))


def test_compiled_shape_evaluation_layer_list_matches_compiled_kernel(monkeypatch):
    """Where the population-wide launch can run, a compiled-shape group
    evaluates on its evaluation layer list (agx_ppo_act_graph); a full pass
    gives the fitness of the compiled policy step (agx_ppo_act) on the same
    counters — the samples agree (a tie within rounding between two logits
    would be the only way to differ)."""
    from agilerl_amd.population import runner as runner_mod

    pop, run = _runner_pair(monkeypatch, False, P=4, N=32)
    run.iteration()
    torch.cuda.synchronize()
    layer_list = run.evaluate(loop=2, max_steps=None)
    pop.eval_rounds -= 1
    monkeypatch.setattr(runner_mod, "population_eval_ok", lambda runners, paced=True: False)
    compiled = run.evaluate(loop=2, max_steps=None)
    assert np.all(np.isfinite(layer_list))
    np.testing.assert_array_equal(layer_list, compiled)
