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


def test_evolvable_cnn_layout_and_seeded_init():
    """EvolvableCNN (modules/cnn.py:224-552): module names / state-dict keys of
    create_cnn (utils/evolvable_networks.py:460-525) + flatten / linear output,
    and the reference's draw order under one seed — each nn.Conv2d built then
    layer_init'd (orthogonal gain sqrt(2), bias 0), then the final Linear with
    torch's default init — so a seeded run starts from the reference's weights."""
    from torch import nn

    from agilerl_amd.modules import EvolvableCNN

    cfg = dict(channel_size=[32, 64, 128], kernel_size=[8, 4, 3], stride_size=[4, 2, 1])
    torch.manual_seed(3)
    net = EvolvableCNN([4, 84, 84], 256, name="encoder", output_activation="ReLU", **cfg)
    names = [n for n, _ in net.model.named_children()]
    assert names == ["encoder_conv_layer_1", "encoder_activation_1", "encoder_conv_layer_2", "encoder_activation_2",
                     "encoder_conv_layer_3", "encoder_activation_3", "encoder_flatten", "encoder_linear_output",
                     "encoder_output_activation"]
    assert tuple(net.cnn_output_size) == (1, 128, 7, 7)
    # restated reference construction order
    torch.manual_seed(3)
    want, c = [], 4
    for ch, k, s in zip(cfg["channel_size"], cfg["kernel_size"], cfg["stride_size"]):
        conv = nn.Conv2d(c, ch, k, s)
        nn.init.orthogonal_(conv.weight, np.sqrt(2))
        nn.init.constant_(conv.bias, 0.0)
        want += [conv.weight, conv.bias]
        c = ch
    lin = nn.Linear(128 * 7 * 7, 256)
    want += [lin.weight, lin.bias]
    got = list(net.state_dict().values())
    assert len(got) == len(want) and all(torch.equal(a, b) for a, b in zip(got, want))
    assert net.model.encoder_conv_layer_1.fuse_relu and net.model.encoder_conv_layer_1.image_norm is None
    net.set_image_norm(0.0, 255.0)
    assert net.model.encoder_conv_layer_1.image_norm == (0.0, 255.0)
    assert net.model.encoder_conv_layer_2.image_norm is None
    with pytest.raises(Exception):  # no CPU fallback for the convolutions
        net(torch.zeros(1, 4, 84, 84))


def test_image_space_networks_and_preprocessing():
    """Image Box spaces (is_image_space, evolvable_networks.py:74-84) get the
    default CNN encoder (32/32, 3/3, 1/1, evolvable_networks.py:190-196); the
    agents keep uint8 frames for the kernel's in-load normalisation and
    normalise f32 frames as apply_image_normalization (algo_utils.py:1134-1183)."""
    from agilerl_amd.algorithms import DQN, RainbowDQN
    from agilerl_amd.envs import Box, Discrete
    from agilerl_amd.modules import EvolvableCNN
    from agilerl_amd.networks.base import image_norm_bounds

    obs, act = Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6)
    d = DQN(obs, act, device="cpu")
    assert isinstance(d.actor.encoder, EvolvableCNN)
    assert d.actor.encoder.channel_size == [32, 32] and d.actor.encoder.kernel_size == [3, 3]
    assert d.actor.encoder.output_activation == "ReLU"
    r = RainbowDQN(obs, act, device="cpu", normalize_images=False)
    assert r._img_norm is None and r.actor.encoder.model.encoder_conv_layer_1.image_norm is None
    x = r._obs(np.full((2, 4, 84, 84), 255, np.uint8))
    assert x.dtype == torch.float32 and float(x.max()) == 255.0  # no normalisation requested
    u = d._obs(np.full((4, 84, 84), 51, np.uint8))
    assert u.dtype == torch.uint8 and u.shape == (1, 4, 84, 84)
    f = d._obs(np.full((1, 4, 84, 84), 51.0, np.float32))
    assert f.dtype == torch.float32 and float(f[0, 0, 0, 0]) == np.float32(51.0) / np.float32(255.0)
    assert image_norm_bounds(Box(0, 1, (3, 8, 8))) is None
    assert image_norm_bounds(Box(-np.inf, np.inf, (3, 8, 8))) is None
    assert image_norm_bounds(Box(-1, 7, (3, 8, 8))) == (-1.0, 7.0)


def test_image_actor_critic_spec_layout():
    """ppo_image.yaml's network as the population's flat layout: reference
    state-dict names (shared_encoder_conv_layer_i, linear_output, heads),
    the clip groups and the uint8 frame storage (CPU: no forward)."""
    import numpy as np

    from agilerl_amd.algorithms.ppo import spec_from_net_config
    from agilerl_amd.envs import Box, Discrete

    space = Box(0, 255, (4, 84, 84), dtype=np.uint8)
    net_config = {"latent_dim": 256,
                  "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
                  "head_config": {"hidden_size": [256], "layer_norm": False}}
    spec = spec_from_net_config(space, Discrete(4), net_config)
    keys = spec.state_dict_keys()
    assert keys["actor.encoder.model.shared_encoder_conv_layer_1.weight"][1] == (32, 4, 8, 8)
    assert keys["actor.encoder.model.shared_encoder_conv_layer_3.weight"][1] == (128, 64, 3, 3)
    assert keys["actor.encoder.model.shared_encoder_linear_output.weight"][1] == (256, 128 * 7 * 7)
    assert keys["actor.head_net._wrapped.model.actor_linear_layer_1.weight"][1] == (256, 256)
    assert keys["critic.head_net.model.value_linear_layer_output.weight"][1] == (1, 256)
    assert keys["critic.encoder.model.shared_encoder_conv_layer_2.bias"] == \
        keys["actor.encoder.model.shared_encoder_conv_layer_2.bias"]
    assert spec.group_offsets == [0, keys["critic.head_net.model.value_linear_layer_1.weight"][0], spec.n_params]
    assert spec.obs_dtype == torch.uint8 and spec.image_norm == (0.0, 255.0) and spec.obs_dim == 4 * 84 * 84
    # every parameter is covered exactly once by the state-dict map
    cover = np.zeros(spec.n_params, np.int32)
    for k, (o, sh) in keys.items():
        if not k.startswith("critic.encoder."):
            cover[o:o + int(np.prod(sh))] += 1
    assert (cover == 1).all()
    flat = spec.init_params(2, [0, 1])
    w1 = flat[0, :32 * 4 * 64].view(32, 256)
    torch.testing.assert_close(w1 @ w1.T, 2.0 * torch.eye(32), rtol=0, atol=1e-4)  # orthogonal, gain sqrt 2
    o, sh = keys["actor.head_net._wrapped.model.actor_linear_layer_output.weight"]
    assert flat[0, o:o + 4 * 256].abs().max() < 0.2  # output_vanish x0.1
