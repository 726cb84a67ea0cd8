"""Checkpoints the reference wrote (torch.save(pickle_module=dill) of
get_checkpoint_dict, agilerl/algorithms/core/base.py:168-224, 939-949) read
by algorithms/refckpt.py: torch's weights-only unpickler with inert
stand-ins for every class the file names.

* the reference's own DQN checkpoint (tutorials/pettingzoo/models/DQN/
  lesson1_trained_agent.pt, agilerl 2.2.0) loads into the agx DQN with every
  tensor, the Adam state and the hyper-parameters as stored (skipped where
  /root/reference is absent);
* the tutorial files written by agilerl < 2.0 (no ``network_info``) are
  refused with a clear error, not misread;
* a file in the reference's layout naming classes of a module that is not
  importable at load time, one of which would run a function when unpickled
  the reference's way, loads with nothing run;
* a MADDPG file in the multi-agent layout ({agent_id: state_dict} per network
  and per optimizer) restores every network and Adam state;
* (GPU) a PPO file in the reference's layout — one Adam over the actor's and
  the critic's parameter groups (ppo.py:329-333) — lands in the population
  rows: weights, both moments per parameter and the step."""

import os
import sys
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

REF_DQN = "/root/reference/tutorials/pettingzoo/models/DQN"
TRIPPED = []


def _fake_module():
    """A stand-in 'reference' package, importable only while the file is written."""
    mod = types.ModuleType("agxfake_ref")

    class Box:
        def __init__(self, shape):
            self._shape, self.low = tuple(shape), np.zeros(shape, np.float32)

    class Discrete:
        def __init__(self, n):
            self.n, self.start = np.int64(n), np.int64(0)

    def trip(*args):
        TRIPPED.append(args)
        return None

    class Registry:
        def __reduce__(self):  # unpickled the reference's way, this would call trip()
            return (trip, ("registry",))

    class QNetwork:
        pass

    for obj in (Box, Discrete, Registry, QNetwork, trip):
        obj.__module__, obj.__qualname__ = mod.__name__, obj.__name__  # pickled by reference
        setattr(mod, obj.__name__, obj)
    return mod


def _write_reference_file(path, algo, attrs, modules, optimizer_sd, networks):
    import dill

    mod = _fake_module()
    sys.modules[mod.__name__] = mod
    try:
        ck = dict(attrs)
        ck.update(algo=algo, agilerl_version="2.2.0", registry=mod.Registry(),
                  observation_space=mod.Box(attrs.pop("_obs_shape")), action_space=mod.Discrete(attrs.pop("_n")))
        ck.pop("_obs_shape"), ck.pop("_n")
        info_mods = {}
        for name, sd in modules.items():
            info_mods.update({f"{name}_cls": mod.QNetwork, f"{name}_init_dict": {"latent_dim": 32},
                              f"{name}_state_dict": OrderedDict(sd), f"{name}_module_dict_cls": None})
        ck["network_info"] = {"modules": info_mods, "network_names": list(modules),
                              "optimizers": {"optimizer_cls": "Adam", "optimizer_state_dict": optimizer_sd,
                                             "optimizer_networks": list(networks), "optimizer_lr": "lr",
                                             "optimizer_kwargs": {}},
                              "optimizer_names": ["optimizer"]}
        torch.save(ck, path, pickle_module=dill)
    finally:
        del sys.modules[mod.__name__]


@pytest.mark.skipif(not os.path.isdir(REF_DQN), reason="reference checkpoints not present")
def test_reference_dqn_checkpoint_loads():
    from agilerl_amd.algorithms import refckpt
    from agilerl_amd.algorithms.dqn import DQN

    path = f"{REF_DQN}/lesson1_trained_agent.pt"
    allow_before = list(torch.serialization.get_safe_globals())
    raw = refckpt.read_reference(path)
    assert set(torch.serialization.get_safe_globals()) == set(allow_before)  # nothing stays allow-listed
    assert isinstance(raw["registry"], refckpt.Inert) and isinstance(raw["observation_space"], refckpt.Inert)
    assert raw["observation_space"].attr("_shape") == (2, 6, 7)
    agent = DQN.load(path, device="cpu")
    assert agent.algo == "DQN" and agent.batch_size == 256 and agent.lr == 1e-4 and agent.double is True
    assert tuple(agent.observation_space.shape) == (2, 6, 7) and agent.action_space.n == 7
    sd = raw["network_info"]["modules"]["actor_state_dict"]
    mine = agent.actor.state_dict()
    assert list(mine) == list(sd)
    for k, t in sd.items():
        assert torch.equal(mine[k], t), k
    ref_opt = raw["network_info"]["optimizers"]["optimizer_state_dict"]
    opt = agent.optimizer.state_dict()
    assert len(opt["state"]) == len(ref_opt["state"]) == 14
    for i, s in ref_opt["state"].items():
        assert torch.equal(opt["state"][i]["exp_avg"], s["exp_avg"])
        assert torch.equal(opt["state"][i]["exp_avg_sq"], s["exp_avg_sq"])
        assert float(opt["state"][i]["step"]) == float(s["step"])


@pytest.mark.skipif(not os.path.isdir(REF_DQN), reason="reference checkpoints not present")
def test_pre_2_0_reference_checkpoint_refused():
    from agilerl_amd.algorithms.dqn import DQN

    with pytest.raises(ValueError, match="network_info"):
        DQN.load(f"{REF_DQN}/lesson2_trained_agent.pt", device="cpu")


def test_reference_layout_loads_with_nothing_run(tmp_path):
    from agilerl_amd.algorithms import refckpt
    from agilerl_amd.algorithms.dqn import DQN
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(0)
    net_config = {"encoder_config": {"hidden_size": [32]}, "head_config": {"hidden_size": [32]}}
    src = DQN(Box(-1, 1, (6,)), Discrete(3), net_config=net_config, device="cpu")
    for p in src.actor.parameters():
        p.data.normal_()
    opt = torch.optim.Adam(src.actor.parameters(), lr=3e-4)
    src.actor(torch.randn(5, 6)).sum().backward()
    opt.step()
    path = str(tmp_path / "ref_dqn.pt")
    TRIPPED.clear()
    _write_reference_file(path, "DQN", {"batch_size": 17, "lr": 3e-4, "gamma": 0.97, "net_config": net_config,
                                        "_obs_shape": (6,), "_n": 3},
                          {"actor": src.actor.state_dict(), "actor_target": {}}, opt.state_dict(), ["actor"])
    raw = refckpt.read_reference(path)
    assert not TRIPPED and isinstance(raw["registry"], refckpt.Inert)
    assert isinstance(raw["network_info"]["modules"]["actor_cls"], type)
    assert issubclass(raw["network_info"]["modules"]["actor_cls"], refckpt.Inert)
    agent = DQN.load(path, device="cpu")
    assert not TRIPPED
    mod = _fake_module()  # the same file unpickled the reference's way does run it (our own file)
    sys.modules[mod.__name__] = mod
    try:
        import dill

        torch.load(path, map_location="cpu", weights_only=False, pickle_module=dill)
    finally:
        del sys.modules[mod.__name__]
    assert TRIPPED == [("registry",)]
    assert agent.batch_size == 17 and agent.gamma == 0.97 and agent.action_space.n == 3
    for k, t in src.actor.state_dict().items():
        assert torch.equal(agent.actor.state_dict()[k], t)
    s0 = opt.state_dict()["state"][0]
    assert torch.equal(agent.optimizer.state_dict()["state"][0]["exp_avg"], s0["exp_avg"])


def test_reference_layout_maddpg_loads(tmp_path):
    """Multi-agent layout (algo_utils.py module_checkpoint_multiagent,
    OptimizerWrapper.state_dict per agent): {agent_id: state_dict} per
    network and per optimizer."""
    import dill

    from agilerl_amd.algorithms.maddpg import MADDPG
    from agilerl_amd.envs import Box, Discrete

    ids = ["speaker_0", "listener_0"]
    spaces = ({"speaker_0": Box(-1, 1, (3,)), "listener_0": Box(-1, 1, (11,))},
              {"speaker_0": Discrete(3), "listener_0": Discrete(5)})
    torch.manual_seed(0)
    src = MADDPG(*spaces, agent_ids=ids, device="cpu", batch_size=48)
    for net in ("actors", "critics"):
        for a in ids:
            for p in getattr(src, net)[a].parameters():
                p.data.normal_()
    opts = {}
    for a in ids:  # one step of each agent's Adams so the moments are non-trivial
        for net, opt in (("actors", src.actor_optimizers), ("critics", src.critic_optimizers)):
            for p in getattr(src, net)[a].parameters():
                p.grad = torch.randn_like(p)
            opt[a].step()
    for n in ("actor_optimizers", "critic_optimizers"):
        opts[n] = {a: o.state_dict() for a, o in getattr(src, n).items()}
    mod = _fake_module()
    sys.modules[mod.__name__] = mod
    try:
        info_mods = {}
        for n in ("actors", "actor_targets", "critics", "critic_targets"):
            info_mods.update({f"{n}_cls": {a: mod.QNetwork for a in ids}, f"{n}_init_dict": {a: {} for a in ids},
                              f"{n}_state_dict": {a: OrderedDict(getattr(src, n)[a].state_dict()) for a in ids},
                              f"{n}_module_dict_cls": mod.QNetwork})
        ck = {"algo": "MADDPG", "agilerl_version": "2.2.0", "registry": mod.Registry(), "agent_ids": ids,
              "batch_size": 48, "lr_actor": 0.001, "lr_critic": 0.01,
              "network_info": {"modules": info_mods, "network_names": ["actors", "actor_targets", "critics",
                                                                        "critic_targets"],
                               "optimizers": {f"{n}_state_dict": opts[n] for n in opts},
                               "optimizer_names": list(opts)}}
        path = str(tmp_path / "ref_maddpg.pt")
        torch.save(ck, path, pickle_module=dill)
    finally:
        del sys.modules[mod.__name__]
    dst = MADDPG(*spaces, agent_ids=ids, device="cpu")
    dst.load_checkpoint(path)
    assert dst.batch_size == 48
    for n in ("actors", "actor_targets", "critics", "critic_targets"):
        for a in ids:
            for k, t in getattr(src, n)[a].state_dict().items():
                assert torch.equal(getattr(dst, n)[a].state_dict()[k], t), (n, a, k)
    for n in ("actor_optimizers", "critic_optimizers"):
        for a in ids:
            s0, s1 = getattr(src, n)[a].state_dict()["state"], getattr(dst, n)[a].state_dict()["state"]
            assert set(s0) == set(s1)
            for i in s0:
                assert torch.equal(s0[i]["exp_avg"], s1[i]["exp_avg"])


def test_adam_rows_keys_by_network_order():
    """One Adam, one param group per network (optimizer_wrapper.py:45-53):
    state index i -> the i-th parameter of actor then critic."""
    from agilerl_amd.algorithms.refckpt import _adam_rows

    a = OrderedDict(w=torch.zeros(2, 2), b=torch.zeros(2))
    c = OrderedDict(w=torch.zeros(3), run=torch.zeros(1))
    params = [torch.nn.Parameter(torch.zeros(2, 2)), torch.nn.Parameter(torch.zeros(2)),
              torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(1))]
    opt = torch.optim.Adam([{"params": params[:2]}, {"params": params[2:]}])
    for i, p in enumerate(params):
        p.grad = torch.full_like(p, float(i + 1))
    opt.step()
    rows = _adam_rows(opt.state_dict(), [("actor", a), ("critic", c)])
    assert list(rows["exp_avg"]) == ["actor.w", "actor.b", "critic.w", "critic.run"] and rows["step"] == 1
    assert torch.allclose(rows["exp_avg"]["critic.w"], torch.full((3,), 0.3))
    with pytest.raises(ValueError):
        _adam_rows(opt.state_dict(), [("actor", a)])


@pytest.mark.gpu
def test_reference_layout_ppo_loads_into_population(tmp_path):
    from agilerl_amd.algorithms import PPO
    from agilerl_amd.envs import Box, Discrete, SyntheticVecEnv
    from agilerl_amd.rollouts import collect_rollouts

    src = PPO(Box(-np.inf, np.inf, (8,)), Discrete(4), num_envs=16, learn_step=64, batch_size=32, lr=2e-3)
    collect_rollouts(src, SyntheticVecEnv(16, seed=3))
    src.learn()
    sd = {k: t.detach().cpu().clone() for k, t in src.state_dict().items()}
    nets = {n: OrderedDict((k[len(n) + 1:], t) for k, t in sd.items() if k.startswith(n + "."))
            for n in ("actor", "critic")}
    # the reference's optimizer: Adam over [actor params], [critic params]
    groups = [[torch.nn.Parameter(t.clone()) for t in nets[n].values()] for n in ("actor", "critic")]
    opt = torch.optim.Adam([{"params": g, "lr": 2e-3} for g in groups])
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        for p in groups[0] + groups[1]:
            p.grad = torch.randn(p.shape, generator=g)
        opt.step()
    path = str(tmp_path / "ref_ppo.pt")
    _write_reference_file(path, "PPO", {"batch_size": 32, "lr": 2e-3, "learn_step": 64, "num_envs": 16,
                                        "fitness": [0.25], "_obs_shape": (8,), "_n": 4},
                          nets, opt.state_dict(), ["actor", "critic"])
    agent = PPO.load(path)
    assert agent.fitness == [0.25] and agent.batch_size == 32
    assert torch.equal(agent.population.params.data[0], src.population.params.data[0])
    keys = agent.spec.state_dict_keys()
    m, v = agent.population.opt.exp_avg[0].cpu(), agent.population.opt.exp_avg_sq[0].cpu()
    names = [f"{n}.{k}" for n in ("actor", "critic") for k in nets[n]]
    st = opt.state_dict()["state"]
    for i, name in enumerate(names):
        if name.startswith("critic.encoder."):
            continue
        o, sh = keys[name]
        n = int(np.prod(sh))
        assert torch.equal(m[o:o + n].view(sh), st[i]["exp_avg"]), name
        assert torch.equal(v[o:o + n].view(sh), st[i]["exp_avg_sq"]), name
    assert int(agent.population.opt.steps[0]) == 3
