"""Golden vectors for PPO architecture mutations, from the reference's OWN code.

Test infrastructure only (same rules as gen_golden.py: the reference's files
are executed in place, path-loaded, with minimal ``sys.modules`` stand-ins for
what is not installed here; only seeded inputs and the outputs the reference
produced are written).  Skips when /root/reference is absent.

Exercised (paths relative to /root/reference):
  * agilerl/modules/base.py            EvolvableModule: mutation-method registry,
                                       get_mutation_probs / sample_mutation_method
                                       (:661-711), preserve_parameters, the
                                       mutation wrapper that recreates the network
  * agilerl/modules/mlp.py:213-312     EvolvableMLP add_layer / remove_layer /
                                       add_node / remove_node
  * agilerl/networks/base.py:445-503   EvolvableNetwork add_latent_node /
                                       remove_latent_node, recreate_encoder
  * agilerl/networks/actors.py         StochasticActor (PPO's actor, ppo.py:302-310)
  * agilerl/networks/value_networks.py ValueNetwork (PPO's critic, ppo.py:312-320)
  * agilerl/hpo/mutation.py:829-885    the single-agent architecture mutation:
                                       the method sampled from the policy with
                                       Mutations.rng, applied to the policy, the
                                       same method + mutation dict applied to the
                                       critic (_apply_arch_mutation :1013-1070)
  * share_encoder_parameters (utils/algo_utils.py:164-187, the PPO mutation
    hook): the critic's encoder takes the actor's encoder parameters —
    restated here as a state-dict copy (tensordict is not installed).

The module random generator (``EvolvableModule.rng``, which draws the layer
and node counts) is seeded per case; the reference leaves it unseeded when the
algorithm builds its networks, so the fixture pins what the draws DO, for
given draws.  Fresh weights of a recreated network come from torch's global
CPU generator (seeded per case), as in the reference.

Hash seed.  The reference builds each module's mutation-method table with
``list(set(...))`` (agilerl/modules/base.py:570-571), so the table's ORDER —
and with it which method ``rng.choice`` samples — depends on Python's string
hash seed.  The reference's own test runner fixes it (pyproject.toml:91,
``PYTHONHASHSEED=0``), and so does this generator: it refuses to run under any
other seed and re-launches itself with ``PYTHONHASHSEED=0`` when the variable
is unset, before anything is imported.  META.json records the seed under
``arch_fixtures``; population/arch.py hard-codes the order that seed produces.

Usage:  python tests/golden/gen_arch_golden.py [--ref /root/reference]
"""

from __future__ import annotations

import os
import subprocess
import sys

HASH_SEED = "0"  # the reference's pytest setting, pyproject.toml:91
if __name__ == "__main__" and os.environ.get("PYTHONHASHSEED") is None:
    # the hash seed is fixed at interpreter start-up: re-launch before importing anything
    sys.exit(subprocess.call([sys.executable, *sys.argv], env={**os.environ, "PYTHONHASHSEED": HASH_SEED}))
if __name__ == "__main__" and os.environ.get("PYTHONHASHSEED") != HASH_SEED:
    sys.exit(f"gen_arch_golden.py: PYTHONHASHSEED={os.environ['PYTHONHASHSEED']!r}; the fixtures pin the "
             f"reference's method-table order under PYTHONHASHSEED={HASH_SEED} (agilerl/modules/base.py:570-571)")

import argparse  # noqa: E402
import copy  # noqa: E402
import importlib.util  # noqa: E402
import json  # noqa: E402
import types  # noqa: E402

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


# ---- gymnasium.spaces stand-ins (real classes: the reference checks isinstance) ----
class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = tuple(shape) if shape is not None else None
        self.dtype = np.dtype(dtype) if dtype is not None else None


class Box(Space):
    def __init__(self, low, high, shape, dtype=np.float32):
        super().__init__(shape, dtype)
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)


class Discrete(Space):
    def __init__(self, n):
        super().__init__((), np.int64)
        self.n = int(n)


class _Other(Space):
    pass


class Dict(Space):
    def __init__(self, spaces_=None):
        super().__init__(None, None)
        from collections import OrderedDict

        self.spaces = OrderedDict(spaces_ or {})

    def __getitem__(self, key):
        return self.spaces[key]

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def values(self):
        return self.spaces.values()

    def __len__(self):
        return len(self.spaces)


def _flatdim(space):
    if isinstance(space, Discrete):
        return space.n
    if isinstance(space, Dict):
        return sum(_flatdim(v) for v in space.spaces.values())
    return int(np.prod(space.shape))


def _package(name: str) -> types.ModuleType:
    mod = types.ModuleType(name)
    mod.__path__ = []
    sys.modules[name] = mod
    return mod


class _AnyModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        cls = type(name, (), {"__init__": lambda self, *a, **k: None})
        setattr(self, name, cls)
        return cls


def _any(name: str) -> types.ModuleType:
    mod = _AnyModule(name)
    mod.__path__ = []
    sys.modules[name] = mod
    return mod


def _load(ref: str, modname: str, relpath: str):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(ref, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def _setup(ref: str):
    gym = _package("gymnasium")
    sp = _package("gymnasium.spaces")
    for cls in (Space, Box, Discrete, Dict):
        setattr(sp, cls.__name__, cls)
    for name in ("Tuple", "MultiDiscrete", "MultiBinary", "Graph", "Text", "Sequence"):
        setattr(sp, name, type(name, (_Other,), {}))
    sp.flatdim = _flatdim
    gym.spaces = sp
    _any("tensordict")
    _any("tensordict.nn")
    agilerl = _package("agilerl")
    agilerl.__path__ = [os.path.join(ref, "agilerl")]
    _load(ref, "agilerl.protocols", "agilerl/protocols.py")
    _any("agilerl.typing")  # annotations only
    mods = _package("agilerl.modules")
    cc = _load(ref, "agilerl.modules.custom_components", "agilerl/modules/custom_components.py")
    base = _load(ref, "agilerl.modules.base", "agilerl/modules/base.py")
    for name in ("EvolvableModule", "EvolvableWrapper", "ModuleDict"):
        setattr(mods, name, getattr(base, name))
    for name in ("GumbelSoftmax", "NewGELU", "NoisyLinear"):
        setattr(mods, name, getattr(cc, name))
    cfg = _load(ref, "agilerl.modules.configs", "agilerl/modules/configs.py")
    utils = _package("agilerl.utils")
    au = types.ModuleType("agilerl.utils.algo_utils")
    au.get_output_size_from_space = lambda s: s.n if isinstance(s, Discrete) else int(np.prod(s.shape))
    sys.modules["agilerl.utils.algo_utils"] = au
    utils.algo_utils = au
    _load(ref, "agilerl.utils.torch_utils", "agilerl/utils/torch_utils.py")
    en = _load(ref, "agilerl.utils.evolvable_networks", "agilerl/utils/evolvable_networks.py")
    mlp = _load(ref, "agilerl.modules.mlp", "agilerl/modules/mlp.py")
    mods.EvolvableMLP = mlp.EvolvableMLP
    for name in ("EvolvableCNN", "EvolvableLSTM", "EvolvableMultiInput", "EvolvableSimBa", "EvolvableResNet",
                 "EvolvableBERT", "EvolvableGPT"):
        setattr(mods, name, type(name, (base.EvolvableModule,), {}))
    cnn = _load(ref, "agilerl.modules.cnn", "agilerl/modules/cnn.py")
    mods.EvolvableCNN = cnn.EvolvableCNN
    mods.ModuleDict = base.ModuleDict
    mi = _load(ref, "agilerl.modules.multi_input", "agilerl/modules/multi_input.py")
    mods.EvolvableMultiInput = mi.EvolvableMultiInput
    _package("agilerl.networks")
    _load(ref, "agilerl.networks.distributions", "agilerl/networks/distributions.py")
    nb = _load(ref, "agilerl.networks.base", "agilerl/networks/base.py")
    act = _load(ref, "agilerl.networks.actors", "agilerl/networks/actors.py")
    val = _load(ref, "agilerl.networks.value_networks", "agilerl/networks/value_networks.py")
    _load(ref, "agilerl.networks.custom_modules", "agilerl/networks/custom_modules.py")
    qn = _load(ref, "agilerl.networks.q_networks", "agilerl/networks/q_networks.py")
    return dict(base=base, cfg=cfg, en=en, mlp=mlp, cnn=cnn, nb=nb, actors=act, values=val, qnets=qn, mi=mi)


def _apply_arch_mutation(network, mut_method, applied_mut_dict=None):
    """agilerl/hpo/mutation.py:1013-1070 (_apply_arch_mutation), restated
    line by line on the loaded reference modules (the Mutations class itself
    would pull in the algorithm hierarchy)."""
    applied_mut_dict = applied_mut_dict or {}
    mut_dict = None
    if mut_method is None:
        mut_dict = {}
        network.last_mutation_attr = None
        network.last_mutation = None
    else:
        mut_return = getattr(network, mut_method)(**applied_mut_dict)
        mut_dict = mut_return if mut_return is not None else {}
    return network.last_mutation_attr, mut_dict


def _sd(prefix: str, net) -> dict:
    return {f"{prefix}.{k}": v.detach().numpy().copy() for k, v in net.state_dict().items()}


def _shape_info(net) -> dict:
    return {"latent": int(net.latent_dim), "enc_hidden": list(net.encoder.hidden_size),
            "head_hidden": list(net.head_net.net_config["hidden_size"]) if hasattr(net.head_net, "net_config")
            else None}


def gen_cases(m: dict, out: dict) -> None:
    """One architecture mutation of a freshly built PPO actor / critic pair per
    case — the situation of every mutation in training: tournament selection
    clones each agent (a new network object built from its init dict) right
    before the generation's mutation.  Starting shapes cover fresh and
    previously mutated architectures; the seeds cover every method."""
    actors, values = m["actors"], m["values"]
    obs, act = Box(-np.inf, np.inf, (8,)), Discrete(4)
    starts = [
        ([64], [64], 64), ([64], [64], 64), ([80], [64], 96), ([64], [64, 64], 64), ([128], [96, 64, 64], 72),
        ([64, 64], [64], 64), ([64], [64], 120), ([64], [64], 16), ([496], [496], 64), ([64], [64], 64),
    ]
    idx = 0
    for k in range(24):
        enc_h, head_h, latent = starts[k % len(starts)]
        nlp = (0.2, 0.5, 1.0, 0.0)[k % 4]
        enc = {"hidden_size": list(enc_h), "min_mlp_nodes": 64, "max_mlp_nodes": 500}
        head = {"hidden_size": list(head_h), "min_hidden_layers": 1, "max_hidden_layers": 3, "min_mlp_nodes": 64,
                "max_mlp_nodes": 500}
        torch.manual_seed(100 + k)
        # ppo.py:288-320: the critic gets a deep copy of the net config (and of the head config)
        import copy

        net_config = {"encoder_config": copy.deepcopy(enc), "head_config": copy.deepcopy(head), "latent_dim": latent}
        critic_config = copy.deepcopy(net_config)
        critic_config["head_config"]["output_activation"] = None
        actor = actors.StochasticActor(obs, act, device="cpu", encoder_name="shared_encoder", **net_config)
        critic = values.ValueNetwork(obs, device="cpu", encoder_name="shared_encoder", **critic_config)
        critic.encoder.load_state_dict(actor.encoder.state_dict())  # share_encoder_parameters
        actor.rng = np.random.default_rng(1000 + k)
        rng = np.random.default_rng(2000 + k)
        g = {"methods": np.array(actor.mutation_methods),
             "probs": np.array(actor.get_mutation_probs(nlp), dtype=np.float64),
             "new_layer_prob": np.array(nlp), "start": np.array(repr((enc_h, head_h, latent))),
             "module_rng_seed": np.array(1000 + k), "mutations_rng_seed": np.array(2000 + k)}
        before = {**_sd("actor", actor), **_sd("critic", critic)}
        torch.manual_seed(5000 + k)  # the fresh weights of the recreated networks
        g["torch_seed"] = np.array(5000 + k)
        mut_method = actor.sample_mutation_method(nlp, rng)  # queries the actor's method table
        applied, mut_dict = _apply_arch_mutation(actor, mut_method)
        if applied in critic.mutation_methods:
            _apply_arch_mutation(critic, applied, mut_dict)
        critic.encoder.load_state_dict(actor.encoder.state_dict())  # the PPO mutation hook
        g["sampled"] = np.array(str(mut_method))
        g["applied"] = np.array("None" if applied is None else str(applied))
        g["mut_dict"] = np.array(repr(sorted((kk, int(v)) for kk, v in (mut_dict or {}).items())))
        g["shapes"] = np.array(repr({"actor": _shape_info(actor), "critic": _shape_info(critic)}))
        for kk, v in before.items():
            g[f"before.{kk}"] = v
        for kk, v in {**_sd("actor", actor), **_sd("critic", critic)}.items():
            g[f"after.{kk}"] = v
        out[f"arch{idx}"] = g
        idx += 1


# ---------------------------------------------------------------------------
# EvolvableCNN (configs 3 and 5): module-level mutations, CNN-encoder network
# tables, and one architecture mutation of a PPO image actor / critic pair
# ---------------------------------------------------------------------------
CNN_STARTS = [  # (channels, kernels, strides, min / max channels)
    ([8, 16, 16], [8, 4, 3], [4, 2, 1], 8, 64),
    ([8], [8], [4], 8, 64),
    ([8, 16], [8, 4], [4, 2], 8, 24),
    ([16, 16, 16], [8, 4, 3], [4, 2, 1], 16, 32),
]
CNN_METHODS = ["add_layer", "remove_layer", "change_kernel", "add_channel", "remove_channel"]


def _cnn_state(net) -> dict:
    return {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}


def gen_cnn_cases(m: dict, out: dict) -> None:
    """EvolvableCNN (agilerl/modules/cnn.py:582-760, MutableKernelSizes
    :55-221): every mutation method from several starting architectures
    (limits included), the module's own generator seeded per case, fresh
    weights of the recreated network from torch's global CPU generator; the
    MutationContext fallbacks (add_layer -> add_channel, change_kernel ->
    add_layer, remove_layer -> add_channel) and the shrink / preserve
    parameter copies (cnn.py:418-456, base.py:472-502) as the reference
    applies them."""
    EvolvableCNN = m["cnn"].EvolvableCNN
    idx = 0
    for si, (ch, ks, ss, cmin, cmax) in enumerate(CNN_STARTS):
        for mi, meth in enumerate(CNN_METHODS):
            for rep in range(2):
                k = 100 * si + 10 * mi + rep
                torch.manual_seed(7000 + k)
                net = EvolvableCNN(input_shape=[4, 52, 52], num_outputs=8, channel_size=list(ch),
                                   kernel_size=list(ks), stride_size=list(ss), min_channel_size=cmin,
                                   max_channel_size=cmax, name="feature_net", output_activation="ReLU")
                net.rng = np.random.default_rng(8000 + k)
                net.mut_kernel_size.rng = net.rng
                before = _cnn_state(net)
                torch.manual_seed(9000 + k)
                ret = getattr(net, meth)()
                g = {"start": np.array(repr((ch, ks, ss, cmin, cmax))), "method": np.array(meth),
                     "module_rng_seed": np.array(8000 + k), "init_seed": np.array(7000 + k),
                     "torch_seed": np.array(9000 + k),
                     "applied": np.array("None" if net.last_mutation_attr is None else str(net.last_mutation_attr)),
                     "ret": np.array(repr(sorted((kk, int(v)) for kk, v in (ret or {}).items()))),
                     "after_cfg": np.array(repr((list(map(int, net.channel_size)), list(map(int, net.kernel_size)),
                                                 list(map(int, net.stride_size)))))}
                for kk, v in before.items():
                    g[f"before.{kk}"] = v
                for kk, v in _cnn_state(net).items():
                    g[f"after.{kk}"] = v
                out[f"cnnmut{idx}"] = g
                idx += 1


def gen_cnn_net_cases(m: dict, out: dict) -> None:
    """Mutation tables of CNN-encoder networks (the encoder's LAYER methods
    disabled, networks/base.py:266-268): QNetwork (DQN), RainbowQNetwork, and
    PPO's StochasticActor / ValueNetwork; then one architecture mutation of a
    PPO image actor / critic pair per case (mutation.py:829-885 restated as
    in gen_cases, share_encoder_parameters after), small CNNs on 4x52x52."""
    actors, values, qn = m["actors"], m["values"], m["qnets"]
    obs, act = Box(0, 255, (4, 52, 52), dtype=np.uint8), Discrete(6)
    enc = {"channel_size": [8, 16, 16], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1],
           "min_channel_size": 8, "max_channel_size": 64}
    head = {"hidden_size": [16], "min_hidden_layers": 1, "max_hidden_layers": 3, "min_mlp_nodes": 8,
            "max_mlp_nodes": 64}
    tables = {}
    torch.manual_seed(1)
    q = qn.QNetwork(obs, act, encoder_config=copy.deepcopy(enc), head_config=copy.deepcopy(head), latent_dim=16)
    tables["qnet"] = q
    rq = qn.RainbowQNetwork(obs, act, support=torch.linspace(-10, 10, 11), encoder_config=copy.deepcopy(enc),
                            head_config=copy.deepcopy(head), latent_dim=16)
    tables["rainbow"] = rq
    for name, net in tables.items():
        out[f"cnntab_{name}"] = {"methods": np.array(net.mutation_methods),
                                 "probs02": np.array(net.get_mutation_probs(0.2), dtype=np.float64),
                                 "probs05": np.array(net.get_mutation_probs(0.5), dtype=np.float64)}
    idx = 0
    for k in range(12):
        nlp = (0.2, 0.5, 1.0, 0.0)[k % 4]
        net_config = {"encoder_config": copy.deepcopy(enc), "head_config": copy.deepcopy(head), "latent_dim": 16,
                      "min_latent_dim": 8, "max_latent_dim": 64}
        torch.manual_seed(300 + k)
        critic_config = copy.deepcopy(net_config)
        critic_config["head_config"]["output_activation"] = None
        actor = actors.StochasticActor(obs, act, device="cpu", encoder_name="shared_encoder", **net_config)
        critic = values.ValueNetwork(obs, device="cpu", encoder_name="shared_encoder", **critic_config)
        critic.encoder.load_state_dict(actor.encoder.state_dict())
        # EvolvableModule.rng is shared by a network and its modules (ModuleMeta,
        # modules/base.py:253-255; the setter propagates); the CNN's kernel-size
        # helper keeps the generator the CNN was built with (MutableKernelSizes
        # is not a module), so it is seeded on its own
        actor.rng = np.random.default_rng(1300 + k)
        actor.encoder.mut_kernel_size.rng = np.random.default_rng(1400 + k)
        critic.rng = np.random.default_rng(1500 + k)
        critic.encoder.mut_kernel_size.rng = np.random.default_rng(1600 + k)
        rng = np.random.default_rng(2300 + k)
        g = {"methods": np.array(actor.mutation_methods), "critic_methods": np.array(critic.mutation_methods),
             "probs": np.array(actor.get_mutation_probs(nlp), dtype=np.float64), "new_layer_prob": np.array(nlp),
             "seeds": np.array([300 + k, 1300 + k, 1400 + k, 1500 + k, 1600 + k, 2300 + k, 5300 + k])}
        before = {**_sd("actor", actor), **_sd("critic", critic)}
        torch.manual_seed(5300 + k)
        mut_method = actor.sample_mutation_method(nlp, rng)
        applied, mut_dict = _apply_arch_mutation(actor, mut_method)
        if applied in critic.mutation_methods:
            _apply_arch_mutation(critic, applied, mut_dict)
        critic.encoder.load_state_dict(actor.encoder.state_dict())
        g["sampled"] = np.array(str(mut_method))
        g["applied"] = np.array("None" if applied is None else str(applied))
        g["mut_dict"] = np.array(repr(sorted((kk, int(v)) for kk, v in (mut_dict or {}).items())))
        g["shapes"] = np.array(repr({"actor_enc": (list(map(int, actor.encoder.channel_size)),
                                                   list(map(int, actor.encoder.kernel_size)),
                                                   list(map(int, actor.encoder.stride_size))),
                                     "latent": int(actor.latent_dim),
                                     "actor_head": list(actor.head_net.net_config["hidden_size"]),
                                     "critic_head": list(critic.head_net.net_config["hidden_size"])}))
        for kk, v in before.items():
            g[f"before.{kk}"] = v
        for kk, v in {**_sd("actor", actor), **_sd("critic", critic)}.items():
            g[f"after.{kk}"] = v
        out[f"cnnarch{idx}"] = g
        idx += 1


# ---------------------------------------------------------------------------
# MADDPG (config 4): the multi-agent architecture mutation
# ---------------------------------------------------------------------------
MA_AGENTS = ("speaker_0", "listener_0")


def _find_analogous_mutation(sampled_mutation, available_methods, policy_agent):
    """agilerl/hpo/mutation.py:1163-1203, restated line by line."""
    if not sampled_mutation:
        return None
    if sampled_mutation in available_methods:
        return sampled_mutation
    bottom = sampled_mutation.split(".")[-1]
    for method in available_methods:
        parts = method.split(".")
        if parts[-1] == bottom and (policy_agent in parts or "vector_mlp" in parts):
            return method
    return None


def _architecture_mutate_multi(actors, critics, new_layer_prob, rng):
    """agilerl/hpo/mutation.py:887-1011 (_architecture_mutate_multi), restated
    line by line on the reference's ModuleDicts (the algorithm object itself
    would pull in the whole algorithm hierarchy): the method sampled from the
    policy ModuleDict's table, applied to the sampled agent's actor, then to
    the other actors that have it, then an analogous method to every critic
    once per mutated agent (the repeat guard as written)."""
    mut_method = actors.sample_mutation_method(new_layer_prob, rng)
    applied_mutation, mut_dict = _apply_arch_mutation(actors, mut_method)
    applied_mutations = []
    if applied_mutation is not None:
        split = applied_mutation.split(".")
        sampled_agent_id, sampled_mutation = split[0], ".".join(split[1:])
        applied_mutations.append(sampled_agent_id)
    else:
        sampled_agent_id, sampled_mutation = mut_method.split(".")[0], None
    for agent_id, policy in actors.items():
        if agent_id == sampled_agent_id:
            continue
        applied_agent = None
        if sampled_mutation in policy.mutation_methods:
            applied_agent, _ = _apply_arch_mutation(policy, sampled_mutation, mut_dict)
        if applied_agent is not None:
            applied_mutations.append(agent_id)
    critic_applied = []
    for agent_id, agent_eval in critics.items():
        analogous = False
        for mutated_agent in applied_mutations:
            if analogous and agent_eval.last_mutation_attr == analogous:
                continue
            analogous = _find_analogous_mutation(sampled_mutation, agent_eval.mutation_methods, mutated_agent)
            if analogous is None:
                raise RuntimeError(f"no analogous method for {sampled_mutation}")
            _apply_arch_mutation(agent_eval, analogous, mut_dict)
            critic_applied.append((agent_id, analogous, str(agent_eval.last_mutation_attr)))
    return mut_method, applied_mutation, sampled_mutation, mut_dict, applied_mutations, critic_applied


def gen_maddpg_cases(m: dict, out: dict) -> None:
    """MADDPG on simple_speaker_listener's spaces (speaker obs 3, listener obs
    11; Discrete 3 / 5 actions) with maddpg.yaml's NET_CONFIG scaled down
    (latent 24, encoder [16], head [16, 16]): actors DeterministicActor with
    their encoders' mutations disabled (maddpg.py:338-348), critics
    ContinuousQNetwork on the Dict of all observations + all actions with
    the shared-critic encoder config (maddpg.py:306-335,
    utils/algo_utils.py:606-665).  One architecture mutation per case."""
    actors_mod, qn, base = m["actors"], m["qnets"], m["base"]
    obs = {"speaker_0": Box(-np.inf, np.inf, (3,)), "listener_0": Box(-np.inf, np.inf, (11,))}
    acts = {"speaker_0": Discrete(3), "listener_0": Discrete(5)}
    enc = {"hidden_size": [16], "min_mlp_nodes": 8, "max_mlp_nodes": 64}
    head = {"hidden_size": [16, 16], "activation": "ReLU", "min_hidden_layers": 1, "max_hidden_layers": 2,
            "min_mlp_nodes": 8, "max_mlp_nodes": 64}
    agent_cfg = {"latent_dim": 24, "min_latent_dim": 8, "max_latent_dim": 64, "encoder_config": enc,
                 "head_config": head}
    critic_cfg = {"encoder_config": {"mlp_config": copy.deepcopy(enc), "latent_dim": 16, "min_latent_dim": 8,
                                     "max_latent_dim": 64},
                  "head_config": copy.deepcopy(head), "latent_dim": 24, "min_latent_dim": 8, "max_latent_dim": 64}
    idx = 0
    for k in range(20):
        nlp = (0.2, 0.5, 1.0, 0.0)[k % 4]
        torch.manual_seed(600 + k)
        a_nets, c_nets = {}, {}
        for a in MA_AGENTS:
            net = actors_mod.DeterministicActor(obs[a], acts[a], device="cpu", **copy.deepcopy(agent_cfg))
            net.encoder.disable_mutations()
            a_nets[a] = net
        for a in MA_AGENTS:
            c_nets[a] = qn.ContinuousQNetwork(observation_space=Dict(obs), action_space=Discrete(8), device="cpu",
                                              **copy.deepcopy(critic_cfg))
        actors = base.ModuleDict(a_nets)
        critics = base.ModuleDict(c_nets)
        for i, a in enumerate(MA_AGENTS):
            a_nets[a].rng = np.random.default_rng(1700 + 10 * k + i)
            c_nets[a].rng = np.random.default_rng(1800 + 10 * k + i)
        g = {"actor_methods": np.array(actors.mutation_methods),
             "actor_probs": np.array(actors.get_mutation_probs(nlp), dtype=np.float64),
             "critic_methods": np.array(c_nets["speaker_0"].mutation_methods),
             "single_actor_methods": np.array(a_nets["speaker_0"].mutation_methods),
             "new_layer_prob": np.array(nlp),
             "seeds": np.array([600 + k, 1700 + 10 * k, 1800 + 10 * k, 2600 + k, 5600 + k])}
        before = {}
        for a in MA_AGENTS:
            before.update(_sd(f"actors.{a}", a_nets[a]))
            before.update(_sd(f"critics.{a}", c_nets[a]))
        torch.manual_seed(5600 + k)
        rng = np.random.default_rng(2600 + k)
        mut_method, applied, sampled, mut_dict, mutated, critic_applied = _architecture_mutate_multi(
            actors, critics, nlp, rng)
        g["sampled"] = np.array(str(mut_method))
        g["applied"] = np.array("None" if applied is None else str(applied))
        g["mut"] = np.array(sampled or "None")
        g["mut_dict"] = np.array(repr(sorted((kk, int(v)) for kk, v in (mut_dict or {}).items())))
        g["mutated_agents"] = np.array(repr(mutated))
        g["critic_applied"] = np.array(repr(critic_applied))
        g["shapes"] = np.array(repr({a: {"actor_latent": int(a_nets[a].latent_dim),
                                         "actor_head": list(a_nets[a].head_net.net_config["hidden_size"]),
                                         "critic_latent": int(c_nets[a].latent_dim),
                                         "critic_head": list(c_nets[a].head_net.net_config["hidden_size"])}
                                     for a in MA_AGENTS}))
        for kk, v in before.items():
            g[f"before.{kk}"] = v
        for a in MA_AGENTS:
            for kk, v in {**_sd(f"actors.{a}", a_nets[a]), **_sd(f"critics.{a}", c_nets[a])}.items():
                g[f"after.{kk}"] = v
        out[f"maddpgarch{idx}"] = g
        idx += 1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    if not os.path.isdir(os.path.join(args.ref, "agilerl")):
        print("reference checkout not found; skipping")
        return
    m = _setup(args.ref)
    out: dict = {}
    gen_cases(m, out)
    gen_cnn_cases(m, out)
    gen_cnn_net_cases(m, out)
    gen_maddpg_cases(m, out)
    for name, arrays in out.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    meta_path = os.path.join(HERE, "META.json")
    meta = json.load(open(meta_path)) if os.path.exists(meta_path) else {}
    meta["arch_fixtures"] = {
        "generator": "tests/golden/gen_arch_golden.py",
        "PYTHONHASHSEED": os.environ["PYTHONHASHSEED"],
        "hash_seed_reason": "method tables are list(set(...)) (agilerl/modules/base.py:570-571); "
                            "the reference's pytest runs under PYTHONHASHSEED=0 (pyproject.toml:91)",
        "torch": torch.__version__,
        "numpy": np.__version__,
        "groups": sorted(out),
    }
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)
    print(f"wrote {len(out)} fixture groups: {sorted(out)}")


if __name__ == "__main__":
    main()
