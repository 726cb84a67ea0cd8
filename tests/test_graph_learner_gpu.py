"""agx_ppo_learn_graph (graph_learner.hip): the runtime-shape fused learner
for the network shapes architecture mutations produce, against the
plain-PyTorch fp32 learner on identical inputs and permutations (same bar as
test_population_gpu.py's fused-learner tests), and end to end: after
architecture mutations every agent still learns on a HIP learner."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")

# shapes the mutations of population/arch.py reach from ppo.yaml's network
# (encoder [64] -> latent 64 -> heads [64]), none of them a compiled plan
SHAPES = {
    "latent_56": dict(encoder_hidden=[64], latent_dim=56, actor_hidden=[64], critic_hidden=[64]),
    "enc_80_two_head_layers": dict(encoder_hidden=[80], latent_dim=64, actor_hidden=[64, 64], critic_hidden=[96]),
    "deep_encoder": dict(encoder_hidden=[64, 48, 32], latent_dim=72, actor_hidden=[32], critic_hidden=[16, 16]),
    "wide_500": dict(encoder_hidden=[500], latent_dim=128, actor_hidden=[500], critic_hidden=[64]),
    "no_layer_norm": dict(encoder_hidden=[64, 64], latent_dim=40, actor_hidden=[48], critic_hidden=[64],
                          layer_norm=False),
    "own_critic_encoder": dict(encoder_hidden=[64], latent_dim=48, actor_hidden=[64], critic_hidden=[32],
                               share_encoders=False),
}


def _pop(shape, P=3, N=16, learn_step=128, batch=64, epochs=1, seed=0, obs_dim=8, A=4, **kw):
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation

    spec = ActorCriticSpec(obs_dim=obs_dim, n_actions=A, **SHAPES[shape])
    pop = PPOPopulation(spec, P, N, learn_step=learn_step, batch_size=batch, lr=1e-3, update_epochs=epochs,
                        seeds=[seed + i for i in range(P)], device=DEV, fused=True, **kw)
    g = torch.Generator(device=DEV).manual_seed(seed + 99)
    pop.obs.copy_(torch.randn(pop.obs.shape, device=DEV, generator=g))
    pop.actions.copy_(torch.randint(0, A, pop.actions.shape, device=DEV, generator=g))
    pop.rewards.copy_(torch.randn(pop.rewards.shape, device=DEV, generator=g))
    pop.dones.copy_((torch.rand(pop.dones.shape, device=DEV, generator=g) < 0.05).to(torch.uint8))
    with torch.no_grad():
        logits, value = spec.forward(pop.params.data, pop.obs.view(P, -1, obs_dim))
        lp = torch.log_softmax(logits, -1).gather(-1, pop.actions.view(P, -1, 1)).squeeze(-1)
    pop.values.copy_(value.view_as(pop.values) + 0.1 * torch.randn(pop.values.shape, device=DEV, generator=g))
    pop.log_probs.copy_(lp.view_as(pop.log_probs) + 0.05 * torch.randn(pop.log_probs.shape, device=DEV, generator=g))
    last_obs = torch.randn(P, N, obs_dim, device=DEV, generator=g)
    last_done = torch.zeros(P, N, dtype=torch.uint8, device=DEV)
    pop.finish_rollout(last_obs, last_done)
    return pop


def _state(pop):
    return (pop.params.data.clone(), pop.opt.exp_avg.clone(), pop.opt.exp_avg_sq.clone(),
            pop.advantages.clone(), pop.opt.steps.clone())


def _restore(pop, st):
    pop.params.data.copy_(st[0])
    pop.opt.exp_avg.copy_(st[1])
    pop.opt.exp_avg_sq.copy_(st[2])
    pop.advantages.copy_(st[3])
    pop.opt.steps.copy_(st[4])


def _compare(pop, perms):
    """torch learner vs the graph learner from the same state -> (loss_t, loss_g)."""
    from agilerl_amd.population.learner import GraphLearner, fused_learn

    assert pop.fused_descriptor() is None and pop.learn_descriptor() is not None
    st = _state(pop)
    loss_t = pop._learn_torch(perms).clone()
    p_t, m_t, steps_t = pop.params.data.clone(), pop.opt.exp_avg.clone(), pop.opt.steps.clone()
    _restore(pop, st)
    loss_g = fused_learn(pop, perms).clone()
    torch.cuda.synchronize()
    assert isinstance(pop._fused, GraphLearner)
    # over many updates the two learners' summation orders drift apart; where a
    # moment is near zero the drift is large relative to it.  Bar: 99.5 % of the
    # moments within 2e-3 relative / 1e-5 of the largest, all within 1e-4 of it
    # (the single-update test above pins the gradients themselves)
    m_g, m_tn = pop.opt.exp_avg.cpu().numpy(), m_t.cpu().numpy()
    scale_m = np.abs(m_tn).max()
    off = np.abs(m_g - m_tn) > 2e-3 * np.abs(m_tn) + 1e-5 * scale_m
    assert off.mean() <= 5e-3, off.mean()
    assert np.abs(m_g - m_tn).max() <= 1e-4 * scale_m
    d_t, d_g = p_t - st[0], pop.params.data - st[0]
    scale = d_t.abs().max().item()
    assert scale > 0
    bad = ((d_g - d_t).abs() > 2e-3 * scale).float().mean().item()
    assert bad <= 1e-3, bad
    assert torch.equal(pop.opt.steps, steps_t)
    np.testing.assert_allclose(loss_g.cpu().numpy(), loss_t.cpu().numpy(), rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_graph_learner_single_update_tight(shape):
    """One minibatch, one epoch: the clipped gradient of the single update
    (exp_avg = 0.1 g after Adam's first step) matches the torch learner's."""
    from agilerl_amd.population.learner import fused_learn

    pop = _pop(shape, N=32, learn_step=64, batch=64, epochs=1, seed=5)
    st = _state(pop)
    perms = pop.permutations()
    pop._learn_torch(perms)
    g_t = pop.opt.grads.clone()
    m_t = pop.opt.exp_avg.clone()
    _restore(pop, st)
    fused_learn(pop, perms)
    torch.cuda.synchronize()
    # entries that are sums with cancellation get an absolute floor of 1e-6 of
    # the largest gradient
    m, mt = pop.opt.exp_avg.cpu().numpy(), m_t.cpu().numpy()
    np.testing.assert_allclose(m, mt, rtol=1e-4, atol=1e-6 * np.abs(mt).max())
    gt = g_t.cpu().numpy()
    np.testing.assert_allclose(m / 0.1, gt, rtol=1e-3, atol=1e-6 * np.abs(gt).max())


@pytest.mark.parametrize("shape,N,learn_step,batch,epochs", [
    ("latent_56", 16, 128, 64, 2), ("enc_80_two_head_layers", 8, 100, 32, 2), ("deep_encoder", 16, 400, 128, 1),
    ("wide_500", 16, 128, 48, 1), ("no_layer_norm", 16, 256, 64, 2), ("own_critic_encoder", 16, 128, 64, 2),
    ("latent_56", 16, 512, 256, 1), ("wide_500", 16, 256, 200, 1)])  # > 128 rows: several GEMM row blocks
def test_graph_learner_matches_torch_learner(shape, N, learn_step, batch, epochs):
    pop = _pop(shape, N=N, learn_step=learn_step, batch=batch, epochs=epochs)
    # the minibatch orders come from numpy's global shuffle stream (ppo.py:836-842):
    # seeded, so the drift bar below sees the same data whatever ran before
    np.random.seed(1234)
    _compare(pop, pop.permutations())


def test_graph_learner_heterogeneous_hparams_and_masks():
    """Per-agent minibatch size / epochs / entropy coefficient (RL-HP
    mutations) and legal-action masks through the graph learner."""
    pop = _pop("enc_80_two_head_layers", P=3, N=16, learn_step=128, batch=64, epochs=2, A=5, obs_dim=6,
               action_masks=True)
    pop.set_agent_hparam(1, "batch_size", 32)
    pop.set_agent_hparam(2, "update_epochs", 1)
    pop.set_agent_hparam(0, "ent_coef", 0.05)
    g = torch.Generator(device=DEV).manual_seed(3)
    masks = (torch.rand(pop.P, pop.T * pop.N, 5, device=DEV, generator=g) < 0.7).to(torch.uint8)
    masks[..., 0] = 1
    acts = pop.actions.view(pop.P, -1)
    masks.view(-1, 5).scatter_(1, acts.reshape(-1, 1), 1)  # the taken action was legal
    pop.action_masks.copy_(masks.view(pop.P, pop.T, pop.N, 5))
    _compare(pop, pop.permutations())


def test_graph_learner_is_independent_of_the_population():
    """An agent's update is the same alone and inside a population (fixed
    summation order; one workgroup per agent)."""
    from agilerl_amd.population.learner import fused_learn

    pop = _pop("deep_encoder", P=4, N=16, learn_step=128, batch=64, epochs=2, seed=11)
    perms = pop.permutations()
    st = _state(pop)
    fused_learn(pop, perms)
    all_p = pop.params.data.clone()
    _restore(pop, st)
    pop_1 = _pop("deep_encoder", P=1, N=16, learn_step=128, batch=64, epochs=2, seed=11)
    pop_1.params.data.copy_(st[0][2:3])
    pop_1.obs.copy_(pop.obs[2:3])
    pop_1.actions.copy_(pop.actions[2:3])
    pop_1.log_probs.copy_(pop.log_probs[2:3])
    pop_1.values.copy_(pop.values[2:3])
    pop_1.advantages.copy_(pop.advantages[2:3])
    pop_1.returns.copy_(pop.returns[2:3])
    pop_1.adv_stats.copy_(pop.adv_stats[2:3])
    fused_learn(pop_1, perms[:, 2:3].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(pop_1.params.data[0], all_p[2])


def test_graph_learner_target_kl_stops_like_torch():
    pop = _pop("latent_56", N=16, learn_step=128, batch=32, epochs=4, target_kl=1e-4)
    _compare(pop, pop.permutations())
    assert int(pop._fused.epochs_run.min()) < 4


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_graph_policy_step_matches_torch_forward(shape):
    """agx_ppo_act_graph (greedy) against the plain-PyTorch forward: actions,
    log-probs, entropy, values; 40 envs = two row blocks."""
    from agilerl_amd.population.learner import policy_step_graph

    P, N = 3, 40
    pop = _pop(shape, P=P, N=N)
    obs = torch.randn(P, N, 8, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    act = torch.empty(P, N, dtype=torch.int64, device=DEV)
    lp, v, ent = (torch.empty(P, N, device=DEV) for _ in range(3))
    policy_step_graph(pop, pop.learn_descriptor(), obs, N * 8, sample=False, counter=0, actions=act, log_probs=lp,
                      values=v, entropy=ent, out_agent_stride=N)
    logits, value = pop.spec.forward(pop.params.data, obs)
    logp_all = torch.log_softmax(logits, -1)
    assert torch.equal(act, logits.argmax(-1))
    torch.testing.assert_close(lp, logp_all.gather(-1, act.unsqueeze(-1)).squeeze(-1), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(v, value.view(P, N), rtol=1e-4, atol=1e-5)
    pa = logp_all.exp()
    torch.testing.assert_close(ent, -(pa * torch.log(pa + 1e-8)).sum(-1), rtol=1e-4, atol=1e-5)


def test_graph_policy_step_samples_the_fused_stream():
    """On a compiled shape both policy steps draw from the same Philox stream:
    the sampled actions agree (up to logits within rounding of a tie)."""
    from agilerl_amd.population.learner import graph_descriptor, policy_step, policy_step_graph
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation

    P, N = 4, 64
    spec = ActorCriticSpec(obs_dim=8, n_actions=4)
    pop = PPOPopulation(spec, P, N, learn_step=N, batch_size=N, device=DEV, fused=True, seeds=list(range(P)))
    assert pop.fused_descriptor() is not None
    obs = torch.randn(P, N, 8, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    a_f, a_g = (torch.empty(P, N, dtype=torch.int64, device=DEV) for _ in range(2))
    agree = []
    for counter in range(1, 6):
        policy_step(pop, pop.fused_descriptor(), obs, N * 8, sample=True, counter=counter, actions=a_f,
                    out_agent_stride=N)
        policy_step_graph(pop, graph_descriptor(spec), obs, N * 8, sample=True, counter=counter, actions=a_g,
                          out_agent_stride=N)
        agree.append((a_f == a_g).float().mean().item())
    assert min(agree) >= 0.99, agree
    assert len({tuple(a_g.view(-1).tolist())}) == 1
