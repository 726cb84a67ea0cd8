"""EvolvableMLP / QNetwork / RainbowQNetwork host logic (CPU, plain torch):
module names and state-dict keys of create_mlp (utils/evolvable_networks.py:
527-644), initialisation, output vanish / output LayerNorm, and the
architecture mutations of modules/mlp.py:214-336 with preserve_parameters
(modules/base.py:472-502)."""

import numpy as np
import pytest
import torch


def test_evolvable_mlp_layout_and_init():
    from agilerl_amd.modules import EvolvableMLP

    torch.manual_seed(0)
    net = EvolvableMLP(8, 4, [64, 32], output_layernorm=True, name="actor")
    keys = list(net.state_dict())
    assert keys == ["model.actor_linear_layer_1.weight", "model.actor_linear_layer_1.bias",
                    "model.actor_layer_norm_1.weight", "model.actor_layer_norm_1.bias",
                    "model.actor_linear_layer_2.weight", "model.actor_linear_layer_2.bias",
                    "model.actor_layer_norm_2.weight", "model.actor_layer_norm_2.bias",
                    "model.actor_linear_layer_output.weight", "model.actor_linear_layer_output.bias"]
    names = [n for n, _ in net.model.named_children()]
    assert names[-2:] == ["actor_layer_norm_output", "actor_activation_output"]
    w1 = net.model.actor_linear_layer_1.weight.detach()
    # orthogonal, gain sqrt(2): the 8 columns of the (64, 8) weight are orthogonal with norm^2 = 2
    assert torch.allclose(w1.T @ w1, 2 * torch.eye(8), atol=1e-5)
    assert torch.count_nonzero(net.model.actor_linear_layer_1.bias) == 0
    wo = net.get_output_dense().weight.detach()  # (4, 32) x 0.1 -> rows orthogonal with norm^2 = 0.02
    assert torch.allclose(wo @ wo.T, 0.02 * torch.eye(4), atol=1e-6)
    y = net(np.zeros(8, dtype=np.float32))
    assert y.shape == (1, 4)
    assert torch.allclose(y.mean(-1), torch.zeros(1), atol=1e-6)  # non-affine output LayerNorm
    assert net.net_config["hidden_size"] == [64, 32] and "num_inputs" not in net.net_config


def test_evolvable_mlp_mutations_preserve_parameters():
    from agilerl_amd.modules import EvolvableMLP

    torch.manual_seed(1)
    net = EvolvableMLP(6, 3, [32], max_hidden_layers=2, random_seed=7)
    w_old = net.model.mlp_linear_layer_1.weight.detach().clone()
    out_old = net.get_output_dense().weight.detach().clone()
    info = net.add_node(hidden_layer=0, numb_new_nodes=16)
    assert info == {"hidden_layer": 0, "numb_new_nodes": 16} and net.hidden_size == [48]
    assert torch.equal(net.model.mlp_linear_layer_1.weight[:32], w_old)
    assert torch.equal(net.get_output_dense().weight[:, :32], out_old)
    assert net.add_layer() is None and net.hidden_size == [48, 48]
    net.add_layer()  # at max_hidden_layers: falls back to add_node
    assert len(net.hidden_size) == 2 and sum(net.hidden_size) > 96
    net.remove_layer()
    assert len(net.hidden_size) == 1
    before = list(net.hidden_size)
    net.remove_node(hidden_layer=0, numb_new_nodes=64)  # would go below min_mlp_nodes unless large enough
    assert net.hidden_size[0] == (before[0] - 64 if before[0] - 64 > 32 else before[0])
    assert net(torch.zeros(2, 6)).shape == (2, 3)


def test_q_networks_reference_keys():
    from agilerl_amd.envs import Box, Discrete
    from agilerl_amd.networks import QNetwork, RainbowQNetwork

    obs, act = Box(-np.inf, np.inf, (8,)), Discrete(4)
    q = QNetwork(obs, act)
    sd = q.state_dict()
    assert sd["encoder.model.encoder_linear_layer_2.weight"].shape == (64, 64)  # default encoder [64, 64]
    assert sd["encoder.model.encoder_linear_layer_output.weight"].shape == (32, 64)  # latent 32
    assert "encoder.model.encoder_layer_norm_output.weight" not in sd  # output LN has no affine
    assert sd["head_net.model.value_linear_layer_1.weight"].shape == (32, 32)  # default head [32]
    assert q(torch.zeros(5, 8)).shape == (5, 4)
    support = torch.linspace(-10, 10, 11)
    r = RainbowQNetwork(obs, act, support=support, num_atoms=11, head_config={"hidden_size": [16]})
    sd = r.state_dict()
    assert sd["head_net.advantage_net.advantage_linear_layer_output.weight_mu"].shape == (44, 16)
    assert "head_net.support" not in sd
    p = r(torch.zeros(5, 8), q=False)
    assert p.shape == (5, 4, 11) and float(p.detach().min()) >= 1e-3
    lp = r(torch.zeros(5, 8), log=True)
    assert torch.allclose(lp.exp().sum(-1), torch.ones(5, 4), atol=1e-5)


@pytest.mark.parametrize("name,bad", [("num_inputs", 0), ("hidden_size", [])])
def test_evolvable_mlp_assertions(name, bad):
    from agilerl_amd.modules import EvolvableMLP

    kw = dict(num_inputs=4, num_outputs=2, hidden_size=[8])
    kw[name] = bad
    with pytest.raises(AssertionError):
        EvolvableMLP(**kw)


@pytest.mark.parametrize("algo", ["DQN", "RainbowDQN"])
def test_dqn_checkpoint_round_trip_cpu(algo, tmp_path):
    """save_checkpoint / load (core/base.py:939-1072 layout), read back with
    torch.load(weights_only=True): networks, optimizer and attributes."""
    from agilerl_amd.algorithms import dqn
    from agilerl_amd.envs import Box, Discrete

    cls = getattr(dqn, algo)
    agent = cls(Box(-np.inf, np.inf, (8,)), Discrete(4), device="cpu", lr=3e-4,
                net_config={"encoder_config": {"hidden_size": [32]}, "latent_dim": 16})
    agent.fitness, agent.steps, agent.scores = [1.5, 2.0], [0, 128], [3.0]
    path = str(tmp_path / "agent.pt")
    agent.save_checkpoint(path)
    ck = torch.load(path, weights_only=True)
    assert ck["network_info"]["network_names"] == ["actor", "actor_target"]
    assert "encoder.model.encoder_linear_layer_1.weight" in ck["network_info"]["modules"]["actor_state_dict"]
    other = cls.load(path, device="cpu")
    assert other.lr == 3e-4 and other.fitness == [1.5, 2.0] and other.steps == [0, 128]
    for k, v in agent.actor.state_dict().items():
        assert torch.equal(v, other.actor.state_dict()[k]), k
    wrong = (dqn.RainbowDQN if algo == "DQN" else dqn.DQN)(Box(-np.inf, np.inf, (8,)), Discrete(4), device="cpu")
    with pytest.raises(ValueError):  # registry mismatch (core/base.py:1046-1052)
        wrong.load_checkpoint(path)
