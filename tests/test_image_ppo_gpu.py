"""Image-observation PPO (BASELINE config 5, Atari Breakout PPO): the
population engine with an EvolvableCNN shared encoder on the HIP conv
kernels, uint8 frames in the HBM rollout SoA.

* the population forward / backward against a plain-PyTorch twin
  (nn.Conv2d / nn.Linear with the reference's module names,
  oracle/ppo_learn.py ImageActorCritic) loaded from the same state dict;
* one learn() of every agent against oracle/ppo_learn.reference_learn
  (ppo.py:814-921 restated in PyTorch: torch.optim.Adam, clip_grad_norm_
  per network) fed the same numpy-stream permutations;
* the reference call site of ppo_image.yaml (channels 32-64-128, kernels
  8-4-3, strides 4-2-1, latent 256, heads [256]) through create_population +
  train_on_policy with a tournament and mutations on 84x84x4 frames.
Tolerances are fp32: the HIP implicit GEMM and the torch conv sum in
different orders.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

SMALL = dict(obs_shape=(4, 36, 36), channel_size=[8, 16], kernel_size=[8, 4], stride_size=[4, 2], latent_dim=32,
             actor_hidden=[32], critic_hidden=[16])


def _spec(**kw):
    from agilerl_amd.population.image_nets import ImageActorCriticSpec

    args = dict(SMALL, n_actions=4)
    args.update(kw)
    return ImageActorCriticSpec(**args)


def _twin(spec, flat_row: torch.Tensor):
    from oracle.ppo_learn import ImageActorCritic

    net = ImageActorCritic(spec.obs_shape, spec.n_actions, spec.channel_size, spec.kernel_size, spec.stride_size,
                           spec.latent_dim, spec.actor_hidden, spec.critic_hidden, spec.head_layer_norm,
                           spec.image_norm)
    sd = {k: flat_row[o:o + int(np.prod(sh))].view(sh).detach().cpu()
          for k, (o, sh) in spec.state_dict_keys().items() if not k.startswith("critic.encoder.")}
    net.load_reference(sd)
    return net, sd


@pytest.mark.parametrize("head_ln", [False, True])
def test_image_spec_forward_backward_matches_torch_twin(head_ln):
    spec = _spec(head_layer_norm=head_ln)
    P, B = 3, 40
    flat = torch.nn.Parameter(spec.init_params(P, [5, 6, 7], DEV))
    g = torch.Generator(device=DEV).manual_seed(1)
    obs = torch.randint(0, 256, (P, B, spec.obs_dim), dtype=torch.uint8, device=DEV, generator=g)
    r1 = torch.randn(P, B, spec.n_actions, device=DEV, generator=g)
    r2 = torch.randn(P, B, device=DEV, generator=g)
    logits, value = spec.forward(flat, obs)
    ((logits * r1).sum() + (value * r2).sum()).backward()
    keys = spec.state_dict_keys()
    for p in range(P):
        net, _ = _twin(spec, flat.data[p])
        net = net.to(DEV)
        x = spec.obs_shape
        xo = net.norm(obs[p].reshape(B, *x))
        lat = net.encoder(xo)
        lg, v = net.actor_head(lat), net.critic_head(lat).squeeze(-1)
        torch.testing.assert_close(logits[p].detach(), lg.detach(), rtol=2e-4, atol=2e-5)
        torch.testing.assert_close(value[p].detach(), v.detach(), rtol=2e-4, atol=2e-5)
        ((lg * r1[p]).sum() + (v * r2[p]).sum()).backward()
        for name, t in net.named_reference_params():
            off, sh = keys[name]
            got = flat.grad[p, off:off + t.numel()].view(sh)
            scale = t.grad.abs().max().item() + 1e-12
            err = (got - t.grad).abs().max().item()
            assert err <= 1e-4 * scale, (p, name, err, scale)


@pytest.mark.parametrize("target_kl", [None, 0.002])
def test_image_population_learn_matches_reference_learn(target_kl):
    """One learn() of P=2 image agents (uint8 frames) == the PyTorch
    restatement of ppo.py:814-921 per agent, same permutations."""
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from oracle.ppo_learn import reference_learn

    spec = _spec()
    P, N, T, batch, E, lr = 2, 16, 8, 64, 2, 1e-3
    pop = PPOPopulation(spec, P, N, learn_step=T * N, batch_size=batch, update_epochs=E, lr=lr,
                        target_kl=target_kl, seeds=[3, 4], device=DEV)
    assert pop.fused_descriptor() is None and pop.obs.dtype == torch.uint8
    g = torch.Generator(device=DEV).manual_seed(11)
    pop.obs.copy_(torch.randint(0, 256, pop.obs.shape, dtype=torch.uint8, device=DEV, generator=g))
    pop.actions.copy_(torch.randint(0, 4, pop.actions.shape, device=DEV, generator=g))
    pop.log_probs.copy_(-torch.rand(pop.log_probs.shape, device=DEV, generator=g) * 2 - 0.2)
    pop.values.copy_(torch.randn(pop.values.shape, device=DEV, generator=g))
    pop.advantages.copy_(torch.randn(pop.advantages.shape, device=DEV, generator=g))
    pop.returns.copy_(torch.randn(pop.returns.shape, device=DEV, generator=g))
    a = pop.advantages.view(P, -1).double()
    pop.adv_stats[:, 0], pop.adv_stats[:, 1] = a.mean(1), a.std(1)
    init = pop.params.data.clone()
    raw_adv = pop.advantages.clone()
    np.random.seed(21)
    perms = pop.permutations()
    loss = pop._learn_torch(perms)
    torch.cuda.synchronize()
    S = T * N
    keys = spec.state_dict_keys()
    for p in range(P):
        net, _ = _twin(spec, init[p])
        out = reference_learn(net, None, pop.obs[p].reshape(S, -1).cpu().numpy(),
                              pop.actions[p].reshape(-1).cpu().numpy(), pop.log_probs[p].reshape(-1).cpu().numpy(),
                              raw_adv[p].reshape(-1).cpu().numpy(), pop.returns[p].reshape(-1).cpu().numpy(),
                              pop.values[p].reshape(-1).cpu().numpy(), perms[:, p].cpu().numpy(), batch_size=batch,
                              epochs=E, lr=lr, target_kl=target_kl)
        assert abs(float(loss[p]) - out["mean_loss"]) <= 1e-4 * max(1.0, abs(out["mean_loss"])), p
        got = pop.params.data[p].cpu()
        for name, ref in out["state"].items():
            off, sh = keys[name]
            new = got[off:off + ref.numel()].view(sh)
            old = init[p, off:off + ref.numel()].cpu().view(sh)
            d_ref, d_got = ref - old, new - old
            # Adam moves every weight by ~lr per step: compare the moves
            bad = (d_got - d_ref).abs() > 2e-3 * lr * E * (S // batch) + 1e-6 * old.abs()
            assert bad.float().mean().item() <= 1e-3, (p, name, bad.sum().item(), ref.numel())
        assert int(pop.opt.steps[p]) == out["epochs"] * (S // batch), p


def test_image_population_single_update_matches_reference():
    """The single-update form of the image learner check: one minibatch
    update (E = 1, S = batch) from a continued Adam state (step 10, non-zero
    moments), every parameter entry within 1e-5 x (|ref| + rms(ref)) of the
    PyTorch restatement of ppo.py:814-921 (moments 1e-4), except at most
    0.01 % of entries."""
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from oracle.ppo_learn import reference_learn

    spec = _spec()
    P, N, T, lr = 2, 16, 4, 1e-3
    S = T * N
    pop = PPOPopulation(spec, P, N, learn_step=S, batch_size=S, update_epochs=1, lr=lr, seeds=[8, 9], device=DEV)
    g = torch.Generator(device=DEV).manual_seed(13)
    pop.obs.copy_(torch.randint(0, 256, pop.obs.shape, dtype=torch.uint8, device=DEV, generator=g))
    pop.actions.copy_(torch.randint(0, 4, pop.actions.shape, device=DEV, generator=g))
    pop.log_probs.copy_(-torch.rand(pop.log_probs.shape, device=DEV, generator=g) * 2 - 0.2)
    pop.values.copy_(torch.randn(pop.values.shape, device=DEV, generator=g))
    pop.advantages.copy_(torch.randn(pop.advantages.shape, device=DEV, generator=g))
    pop.returns.copy_(torch.randn(pop.returns.shape, device=DEV, generator=g))
    a = pop.advantages.view(P, -1).double()
    pop.adv_stats[:, 0], pop.adv_stats[:, 1] = a.mean(1), a.std(1)
    n = spec.n_params
    pop.opt.exp_avg.copy_(torch.randn(P, n, device=DEV, generator=g) * 1e-3)
    pop.opt.exp_avg_sq.copy_(torch.rand(P, n, device=DEV, generator=g) * 1e-5 + 1e-7)
    pop.opt.steps.fill_(10)
    init, m0, v0 = (x.clone() for x in (pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq))
    raw_adv = pop.advantages.clone()
    perms = torch.arange(S, device=DEV).repeat(1, P, 1).contiguous()
    pop._learn_torch(perms)
    torch.cuda.synchronize()
    keys = spec.state_dict_keys()

    def close(name, got, want, rtol):
        got, want = got.double().numpy().ravel(), want.double().numpy().ravel()
        bad = np.abs(got - want) > rtol * (np.abs(want) + np.sqrt(np.mean(want * want)))
        assert bad.mean() <= 1e-4, (name, int(bad.sum()), want.size)

    for p in range(P):
        net, _ = _twin(spec, init[p])
        adam = {k: (m0[p, o:o + int(np.prod(sh))].view(sh).cpu().numpy(),
                    v0[p, o:o + int(np.prod(sh))].view(sh).cpu().numpy())
                for k, (o, sh) in keys.items() if not k.startswith("critic.encoder.")}
        adam["step"] = 10
        out = reference_learn(net, adam, pop.obs[p].reshape(S, -1).cpu().numpy(),
                              pop.actions[p].reshape(-1).cpu().numpy(), pop.log_probs[p].reshape(-1).cpu().numpy(),
                              raw_adv[p].reshape(-1).cpu().numpy(), pop.returns[p].reshape(-1).cpu().numpy(),
                              pop.values[p].reshape(-1).cpu().numpy(), perms[:, p].cpu().numpy(), batch_size=S,
                              epochs=1, lr=lr)
        assert out["step"] == 11 and int(pop.opt.steps[p]) == 11
        for name, ref in out["state"].items():
            off, sh = keys[name]
            k = ref.numel()
            close(f"{p} {name}", pop.params.data[p, off:off + k].cpu(), ref.reshape(-1), 1e-5)
            close(f"{p} {name} exp_avg", pop.opt.exp_avg[p, off:off + k].cpu(), out["exp_avg"][name].reshape(-1),
                  1e-4)
            close(f"{p} {name} exp_avg_sq", pop.opt.exp_avg_sq[p, off:off + k].cpu(),
                  out["exp_avg_sq"][name].reshape(-1), 1e-4)


def test_config5_breakout_ppo_train_on_policy(tmp_path):
    """ppo_image.yaml on Breakout-shaped synthetic frames (uint8 4x84x84, 4
    actions): pop 4 per GPU x 64 envs (config 5's 32 agents / 2048 envs over 8
    GPUs), the reference call site with a shared N-env, tournament +
    mutations, two generations."""
    from agilerl_amd.envs import SyntheticAtariVecEnv
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.hpo.registry import HyperparameterConfig, RLParameter
    from agilerl_amd.hpo.tournament import TournamentSelection
    from agilerl_amd.training import train_on_policy
    from agilerl_amd.utils import create_population

    env = SyntheticAtariVecEnv(64, n_actions=4, p_done=1 / 50, seed=7)
    INIT_HP = {"BATCH_SIZE": 128, "LR": 1e-3, "LEARN_STEP": 256, "UPDATE_EPOCHS": 4, "GAMMA": 0.99,
               "GAE_LAMBDA": 0.95, "CLIP_COEF": 0.2, "ENT_COEF": 0.01, "VF_COEF": 0.5, "MAX_GRAD_NORM": 0.5}
    net_config = {"latent_dim": 256,
                  "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1],
                                     "activation": "ReLU", "layer_norm": False, "init_layers": True},
                  "head_config": {"hidden_size": [256], "activation": "ReLU", "layer_norm": False}}
    hp = HyperparameterConfig(lr=RLParameter(min=1e-4, max=1e-2), batch_size=RLParameter(min=64, max=256, dtype=int),
                              ent_coef=RLParameter(min=0.001, max=0.1))
    pop = create_population("PPO", net_config, INIT_HP, env.single_observation_space, env.single_action_space,
                            hp_config=hp, population_size=4, num_envs=64)
    population = pop[0].population
    assert population.obs.dtype == torch.uint8 and population.obs.shape == (4, 4, 64, 4 * 84 * 84)
    assert population.spec.feat_dim == 128 * 7 * 7
    tour = TournamentSelection(2, True, 4, 1)
    mut = Mutations(no_mutation=0.2, architecture=0, new_layer_prob=0.2, parameters=0.3, activation=0, rl_hp=0.5,
                    rand_seed=1)
    np.random.seed(0)
    pop, fits = train_on_policy(env, "BreakoutSynthetic", "PPO", pop, INIT_HP=INIT_HP, max_steps=1024, evo_steps=512,
                                eval_steps=20, tournament=tour, mutation=mut, verbose=False)
    assert len(fits) == 2 and all(len(f) == 4 and np.all(np.isfinite(f)) for f in fits)
    assert all(a.steps[-1] >= 1024 for a in pop)
    assert torch.isfinite(population.params.data).all()
    a, lp, ent, v = pop[0].get_action(np.random.randint(0, 256, (3, 4, 84, 84), dtype=np.uint8))
    assert a.shape == (3,) and np.all((a >= 0) & (a < 4)) and np.all(np.isfinite(v))


def test_config5_whole_population_on_one_gpu():
    """Config 5's WHOLE population — 32 agents x 64 envs (2048 envs, ~230 MB
    of uint8 rollout) — on one MI355X: one iteration (4-step rollout, GAE,
    4 epochs x 2 minibatches) with property checks: the rollout holds every
    agent's frames, every agent's loss is finite and every agent's parameters
    moved (and stayed finite)."""
    from agilerl_amd.envs import StackedVecEnv, SyntheticAtariVecEnv
    from agilerl_amd.population.runner import PopulationRunner
    from agilerl_amd.utils import create_population

    P, N = 32, 64
    hp = {"BATCH_SIZE": 128, "LR": 1e-3, "LEARN_STEP": 256, "UPDATE_EPOCHS": 4}
    net = {"latent_dim": 256,
           "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
           "head_config": {"hidden_size": [256], "layer_norm": False}}
    env = SyntheticAtariVecEnv(N, n_actions=4, seed=1)
    agents = create_population("PPO", net, hp, env.single_observation_space, env.single_action_space,
                               population_size=P, num_envs=N)
    pop = agents[0].population
    assert pop.P == P and pop.obs.dtype == torch.uint8
    assert pop.obs.numel() * pop.obs.element_size() == P * 4 * N * 4 * 84 * 84  # ~231 MB
    runner = PopulationRunner(pop, StackedVecEnv.from_shared(env, P))
    before = pop.params.data.clone()
    loss = runner.iteration()
    torch.cuda.synchronize()
    assert loss.shape == (P,) and torch.isfinite(loss).all()
    assert torch.isfinite(pop.params.data).all()
    assert bool(((pop.params.data - before).abs().amax(1) > 0).all())
    assert bool((pop.obs.view(P, -1)[:, ::97].float().std(1) > 0).all())
    assert int(pop.opt.steps.min()) == int(pop.opt.steps.max()) == 4 * 2
