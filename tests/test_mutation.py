"""HPO mutations (agilerl_amd.hpo.mutation) against the reference's own
Mutations run (tests/golden/mut*.npz): the per-agent mutation choices, the
RL-hyperparameter values (shared HyperparameterConfig, torch-drawn sample and
grow / shrink), the optimizer re-initialisations, and the parameter-mutated
policy weights — bit for bit."""

import types

import numpy as np
import pytest
import torch

from agilerl_amd.hpo.mutation import Mutations
from agilerl_amd.hpo.registry import HyperparameterConfig, MutationRegistry, RLParameter


class _Agent:
    def __init__(self, i, weights, hp):
        self.index, self.batch_size, self.ent_coef, self.update_epochs = i, 128, 0.01, 4
        self.lr = 1e-3
        self.registry = MutationRegistry(hp)
        self.w = {k: torch.tensor(v) for k, v in weights.items()}
        self.mut, self.reinits = None, 0

    def get_lr_names(self):
        return ["lr"]

    def reinit_optimizers(self, optimizer=None):
        self.reinits += 1

    def policy_weights(self):
        return self.w

    def mutation_hook(self):
        pass


@pytest.mark.parametrize("case", ["mut0", "mut1"])
def test_mutations_match_reference(golden, case):
    g = golden(case)
    P = int(g["P"])
    hp = HyperparameterConfig(lr=RLParameter(min=1e-4, max=1e-2), batch_size=RLParameter(min=8, max=1024, dtype=int),
                              ent_coef=RLParameter(min=0.001, max=0.1),
                              update_epochs=RLParameter(min=1, max=10, dtype=int))
    pop = []
    for i in range(P):
        pre = f"init.a{i}."
        pop.append(_Agent(i, {k[len(pre):]: g[k] for k in g if k.startswith(pre)}, hp))
    no, arch, par, act, rlhp = (float(x) for x in g["probs"])
    m = Mutations(no_mutation=no, architecture=arch, new_layer_prob=0.2, parameters=par, activation=act,
                  rl_hp=rlhp, mutation_sd=0.1, mutate_elite=bool(g["mutate_elite"]), rand_seed=int(g["seed"]))
    for gen in range(int(g["generations"])):
        pop = m.mutation(pop)
        assert [a.mut for a in pop] == list(g["muts"][gen]), gen
        got = np.array([[a.lr, a.batch_size, a.ent_coef, a.update_epochs, a.reinits] for a in pop], np.float64)
        np.testing.assert_array_equal(got, g["hps"][gen])
    for i, a in enumerate(pop):
        pre = f"final.a{i}."
        for k in (k for k in g if k.startswith(pre)):
            assert np.array_equal(a.w[k[len(pre):]].numpy(), g[k]), (i, k)


def test_rlparameter_bounds_and_dtype():
    torch.manual_seed(0)
    p = RLParameter(min=8, max=16, dtype=int)
    p.value = 15
    seen = {p.mutate() for _ in range(40)}
    assert all(isinstance(v, int) and 8 <= v <= 16 for v in seen)
    assert not HyperparameterConfig()
    with pytest.raises(TypeError):
        HyperparameterConfig(lr=1e-3)


def test_no_hp_config_is_no_mutation():
    a = types.SimpleNamespace(registry=MutationRegistry(None), mut=None)
    m = Mutations(0, 0, 0, 0, 0, 1, rand_seed=1)
    assert m.rl_hyperparam_mutation(a).mut == "None"


def _dqn_cpu(algo, hp=None):
    from agilerl_amd.algorithms.dqn import DQN, RainbowDQN
    from agilerl_amd.envs import Box, Discrete

    cls = DQN if algo == "DQN" else RainbowDQN
    torch.manual_seed(0)
    return cls(Box(-1, 1, (6,)), Discrete(3), hp_config=hp, device="cpu", batch_size=32, lr=1e-3)


@pytest.mark.parametrize("algo", ["DQN", "Rainbow DQN"])
def test_parameter_mutation_on_q_network_syncs_target(algo):
    """mutation.py:515-570 on DQN / Rainbow: only 2-D non-norm entries of the
    actor change (Rainbow: noisy mu / sigma / epsilon matrices included), the
    target (the policy group's shared network) loads the mutated actor, and a
    fresh optimizer is built."""
    from agilerl_amd.hpo.mutation import Mutations

    agent = _dqn_cpu(algo)
    before = {k: v.clone() for k, v in agent.actor.state_dict().items()}
    opt0 = agent.optimizer
    mut = Mutations(0, 0, 0.2, 1.0, 0, 0, rand_seed=5)
    mut.mutation([agent])
    assert agent.mut == "param" and agent.optimizer is not opt0
    after = agent.actor.state_dict()
    changed = [k for k in before if not torch.equal(before[k], after[k])]
    assert changed and all(after[k].dim() == 2 and "norm" not in k for k in changed)
    for k, v in agent.actor_target.state_dict().items():
        assert torch.equal(v, after[k]), k


def test_rl_hyperparameter_mutation_reinits_only_the_mutated_optimizer():
    """MADDPG (mutation.py:440-450): a mutated lr_actor re-creates the actor
    optimizers only; batch_size / learn_step land on the agent."""
    from agilerl_amd.algorithms.maddpg import MADDPG
    from agilerl_amd.envs import Box, Discrete
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.hpo.registry import HyperparameterConfig, RLParameter

    hp = HyperparameterConfig(lr_actor=RLParameter(min=1e-4, max=1e-2))
    ids = ["speaker_0", "listener_0"]
    agent = MADDPG({"speaker_0": Box(-1, 1, (3,)), "listener_0": Box(-1, 1, (11,))},
                   {"speaker_0": Discrete(3), "listener_0": Discrete(5)}, agent_ids=ids, hp_config=hp, device="cpu")
    a0, c0 = agent.actor_optimizers, agent.critic_optimizers
    lr0 = agent.lr_actor
    Mutations(0, 0, 0.2, 0, 0, 1.0, rand_seed=3).mutation([agent])
    assert agent.mut == "lr_actor" and agent.lr_actor != lr0
    assert agent.actor_optimizers is not a0 and agent.critic_optimizers is c0
    assert all(o.param_groups[0]["lr"] == agent.lr_actor for o in agent.actor_optimizers.values())
    # parameter mutation: each agent's actor in turn, targets synced
    before = {a: {k: v.clone() for k, v in agent.actors[a].state_dict().items()} for a in ids}
    Mutations(0, 0, 0.2, 1.0, 0, 0, rand_seed=4).mutation([agent])
    for a in ids:
        assert any(not torch.equal(before[a][k], v) for k, v in agent.actors[a].state_dict().items()), a
        for k, v in agent.actor_targets[a].state_dict().items():
            assert torch.equal(v, agent.actors[a].state_dict()[k])


@pytest.mark.parametrize("algo", ["DQN", "Rainbow DQN"])
def test_activation_mutation_dqn_family(algo):
    """mutation.py:457-513 on DQN / Rainbow: a new activation from
    activation_selection minus the current one (Mutations.rng), every module
    of the Q network recreated with it (encoder output activation too),
    parameters kept, the target re-made from the mutated network, fresh Adam."""
    from torch import nn

    from agilerl_amd.algorithms import DQN, RainbowDQN
    from agilerl_amd.envs import Box, Discrete
    from agilerl_amd.hpo.mutation import Mutations

    obs_space, act_space = Box(-np.inf, np.inf, (6,)), Discrete(3)
    cls = DQN if algo == "DQN" else RainbowDQN
    agent = cls(obs_space, act_space, device="cpu")
    before = {k: v.clone() for k, v in agent.actor.state_dict().items() if "epsilon" not in k}
    mut = Mutations(0, 0, 0, 0, 1.0, 0, rand_seed=3)
    (agent,) = mut.mutation([agent])
    assert agent.mut == "act"
    new = agent.actor.activation
    assert new in ("ELU", "GELU") and agent.actor.encoder.output_activation == new
    acts = {type(m).__name__ for m in agent.actor.modules()}
    assert {"ELU": "ELU", "GELU": "GELU"}[new] in acts and "ReLU" not in acts
    after = agent.actor.state_dict()
    assert all(torch.equal(after[k], v) for k, v in before.items())
    t = agent.actor_target.state_dict()
    assert all(torch.equal(t[k], v) for k, v in after.items())
    assert agent.actor_target is not agent.actor
    assert all(p is q for p, q in zip(agent.optimizer.param_groups[0]["params"], agent.actor.parameters()))
    x = torch.randn(4, 6)
    assert agent.actor(x).shape == (4, 3) and agent.actor_target(x).shape == (4, 3)
    assert not isinstance(agent.actor.encoder.model[1], nn.ReLU)


@pytest.mark.parametrize("algo", ["DQN", "Rainbow DQN"])
def test_architecture_mutation_dqn_family(algo):
    """mutation.py:373-411 / 829-885 on an MLP-encoder Q network: the method
    from the EvolvableNetwork table (population/arch.py) with Mutations.rng,
    applied with the modules' generators (fallbacks at the limits), the target
    re-made from the mutated network, fresh Adam; overlapping weights kept."""
    from agilerl_amd.algorithms import DQN, RainbowDQN
    from agilerl_amd.envs import Box, Discrete
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.population import arch

    obs_space, act_space = Box(-np.inf, np.inf, (6,)), Discrete(3)
    cls = DQN if algo == "DQN" else RainbowDQN
    seen, changed = set(), 0
    for seed in range(12):
        torch.manual_seed(seed)
        agent = cls(obs_space, act_space, device="cpu")
        assert agent.can_mutate_architecture
        before = {k: v.clone() for k, v in agent.actor.state_dict().items()}
        shape0 = {k: tuple(v.shape) for k, v in before.items()}
        mut = Mutations(0, 1.0, 0.5, 0, 0, 0, rand_seed=seed)
        want = np.random.default_rng(seed)  # the per-agent mutation draw, then the method draw
        want.choice(np.arange(len(mut.mut_options)), 1, p=mut.mut_proba)
        method = arch.sample_method(0.5, want)
        (agent,) = mut.mutation([agent])
        fallback = {"head_net.add_layer": "head_net.add_node", "head_net.remove_layer": "head_net.add_node"}
        assert agent.mut in (method, fallback.get(method)), (method, agent.mut)
        seen.add(agent.mut)
        after = agent.actor.state_dict()
        shapes = {k: tuple(v.shape) for k, v in after.items()}
        changed += shapes != shape0  # (a node / latent change at a limit keeps the shapes)
        for k, v in after.items():  # preserve_parameters: the overlap of every kept tensor is unchanged
            if k in before and "norm" not in k and "epsilon" not in k:
                sl = tuple(slice(0, min(a, b)) for a, b in zip(v.shape, before[k].shape))
                assert torch.equal(v[sl], before[k][sl]), (agent.mut, k)
        t = agent.actor_target.state_dict()
        assert all(torch.equal(t[k], v) for k, v in after.items())
        assert all(p is q for p, q in zip(agent.optimizer.param_groups[0]["params"], agent.actor.parameters()))
        assert agent.actor(torch.randn(2, 6)).shape == (2, 3)
    assert len(seen) >= 3 and changed >= 6, (seen, changed)


@pytest.mark.parametrize("algo", ["DQN", "Rainbow DQN"])
def test_architecture_mutation_cnn_q_networks(algo):
    """mutation.py:829-885 on a CNN-encoder Q network (configs 3 / 5 shape):
    the method from the CNN-encoder table (population/image_arch.py, the
    reference's order; the encoder's LAYER methods disabled) drawn with
    Mutations.rng, applied with the network's generator (fallbacks and the
    disabled add_layer as modules/cnn.py), the target re-made from the
    mutated network, fresh Adam; overlapping conv / linear weights kept
    (shrinking methods copy the leading [:c_out, :c_in] block).  CPU:
    construction and mutation only (the convolutions run on the GPU)."""
    from agilerl_amd.algorithms import DQN, RainbowDQN
    from agilerl_amd.envs import Box, Discrete
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.population import image_arch

    obs_space, act_space = Box(0, 255, (4, 52, 52), dtype=np.uint8), Discrete(6)
    net_config = {"encoder_config": {"channel_size": [8, 16, 16], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1],
                                     "min_channel_size": 8, "max_channel_size": 64},
                  "head_config": {"hidden_size": [32]}, "latent_dim": 32}
    cls = DQN if algo == "DQN" else RainbowDQN
    seen, changed = set(), 0
    for seed in range(16):
        torch.manual_seed(seed)
        agent = cls(obs_space, act_space, net_config=net_config, device="cpu")
        assert agent.can_mutate_architecture
        assert agent.actor.mutation_methods == image_arch.METHODS
        before = {k: v.clone() for k, v in agent.actor.state_dict().items()}
        shape0 = {k: tuple(v.shape) for k, v in before.items()}
        mut = Mutations(0, 1.0, 0.5, 0, 0, 0, rand_seed=seed)
        want = np.random.default_rng(seed)
        want.choice(np.arange(len(mut.mut_options)), 1, p=mut.mut_proba)
        method = image_arch.sample_method(0.5, want)
        (agent,) = mut.mutation([agent])
        fallback = {"head_net.add_layer": "head_net.add_node", "head_net.remove_layer": "head_net.add_node"}
        assert agent.mut in (method, fallback.get(method), "None"), (method, agent.mut)
        seen.add(agent.mut)
        after = agent.actor.state_dict()
        shapes = {k: tuple(v.shape) for k, v in after.items()}
        changed += shapes != shape0
        for k, v in after.items():
            if k in before and "norm" not in k and "epsilon" not in k and v.dim() != 4:
                sl = tuple(slice(0, min(a, b)) for a, b in zip(v.shape, before[k].shape))
                assert torch.equal(v[sl], before[k][sl]), (agent.mut, k)
            elif k in before and v.dim() == 4 and v.shape[2:] == before[k].shape[2:]:
                m0, m1 = min(v.shape[0], before[k].shape[0]), min(v.shape[1], before[k].shape[1])
                assert torch.equal(v[:m0, :m1], before[k][:m0, :m1]), (agent.mut, k)
        t = agent.actor_target.state_dict()
        assert all(torch.equal(t[k], v) for k, v in after.items())
        assert all(p is q for p, q in zip(agent.optimizer.param_groups[0]["params"], agent.actor.parameters()))
    assert any(m.startswith("encoder.") for m in seen) and changed >= 4, (seen, changed)


def test_heterogeneous_epoch_permutation_rows_stay_in_range():
    """An agent with fewer update_epochs than the population maximum draws
    fewer shuffles; its remaining rows of the (reused, uninitialised) host
    buffer must still be valid indices: the gather prologue and the PyTorch
    learner index with every row.  They get arange(S)."""
    import numpy as np

    from types import SimpleNamespace

    from agilerl_amd.population.ppo_pop import PPOPopulation

    # the host-side state _draw_numpy_perms reads (a population of 3, S = 32,
    # agent 1 mutated to 1 update epoch)
    pop = SimpleNamespace(P=3, global_P=3, S=32, update_epochs=3, agent_epochs=[3, 1, 3], heterogeneous=True)
    out = np.full((3, 3, pop.S), -7, dtype=np.int64)  # garbage a reused buffer may hold
    np.random.seed(0)
    PPOPopulation._draw_numpy_perms(pop, out)
    assert out.min() >= 0 and out.max() < pop.S
    assert np.array_equal(out[1:, 1], np.tile(np.arange(pop.S), (2, 1)))
    for e in range(3):
        for p in (0, 2):
            assert sorted(out[e, p]) == list(range(pop.S))
