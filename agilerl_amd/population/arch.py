"""Architecture mutations of a PPO actor-critic held as a flat parameter row.

The reference mutates the policy network of an agent (hpo/mutation.py:
829-885, ``_architecture_mutate_single``): a method is sampled from the
actor's mutation-method table with ``Mutations.rng``
(modules/base.py:661-711), applied to the actor, and the method the actor
actually applied is applied to the critic with the same mutation dict
(``_apply_arch_mutation``, mutation.py:1013-1070); PPO's mutation hook then
gives the critic the actor's encoder (share_encoder_parameters,
utils/algo_utils.py:164-187).  For PPO's StochasticActor the table is, in
this order (layer methods, then node methods):

  head_net.remove_layer, head_net.add_layer          (LAYER; the encoder's
                                                      layer mutations are disabled,
                                                      networks/base.py:281-283)
  remove_latent_node, add_latent_node                (NODE, networks/base.py:457-491:
                                                      latent +- choice([8, 16, 32]))
  encoder.add_node, encoder.remove_node,             (NODE, modules/mlp.py:254-312:
  head_net.add_node, head_net.remove_node             layer integers(0, L), nodes
                                                      choice([16, 32, 64]))

with probabilities new_layer_prob / 2 for each layer method and
(1 - new_layer_prob) / 6 for each node method (uniform when one kind is
empty).  ``add_layer`` / ``remove_layer`` fall back to ``add_node`` at the
layer limits (mlp.py:227-252).  Every mutation recreates the mutated
network(s) (``create_mlp``, utils/evolvable_networks.py:527-644: fresh
nn.Linear + orthogonal initialisation, drawing from torch's global CPU
generator, actor before critic) and copies the old parameters over by name,
overlapping slices for resized weights, norms of a changed width left fresh
(``preserve_parameters``, modules/base.py:472-502).  Node / layer
mutations of the encoder or the head recreate that module; latent mutations
recreate the whole network (encoder and head).

Everything here runs on the host on one agent's row (a few hundred KB at
most); the population engine moves the result back into HBM.  Pinned
against the reference's own outputs: tests/golden/gen_arch_golden.py.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass

import numpy as np
import torch

from ..modules.mlp import create_mlp
from .nets import ActorCriticSpec

# The reference collects each class's methods into ``list(set(...))``
# (modules/base.py:570-571), so the table order is that of Python's string-hash
# seed.  The order below is the one PYTHONHASHSEED=0 produces — the seed the
# reference's own test runner sets (pyproject.toml:91) and the seed the
# fixtures of tests/golden/gen_arch_golden.py are made under (META.json
# ``arch_fixtures``).  A reference run under another seed samples from a
# permuted table and draws other methods from the same Mutations.rng stream.
METHOD_ORDER_HASH_SEED = "0"
LAYER_METHODS = ["head_net.remove_layer", "head_net.add_layer"]
NODE_METHODS = ["remove_latent_node", "add_latent_node", "encoder.add_node", "encoder.remove_node",
                "head_net.add_node", "head_net.remove_node"]
METHODS = LAYER_METHODS + NODE_METHODS


def method_probs(new_layer_prob: float) -> list[float]:
    """EvolvableModule.get_mutation_probs (modules/base.py:661-685)."""
    nl, nn_ = len(LAYER_METHODS), len(NODE_METHODS)
    return [new_layer_prob / nl] * nl + [(1 - new_layer_prob) / nn_] * nn_


def sample_method(new_layer_prob: float, rng: np.random.Generator) -> str:
    """sample_mutation_method (modules/base.py:687-711) with Mutations.rng."""
    return str(rng.choice(METHODS, p=method_probs(new_layer_prob), size=1)[0])


@dataclass
class _Mlp:
    """Mutable hyperparameters of one EvolvableMLP (hidden sizes + limits)."""
    hidden: list[int]
    min_layers: int
    max_layers: int
    min_nodes: int
    max_nodes: int

    def add_layer(self, rng):
        if len(self.hidden) < self.max_layers:
            self.hidden = self.hidden + [self.hidden[-1]]
            return "add_layer", {}
        return self.add_node(rng)

    def remove_layer(self, rng):
        if len(self.hidden) > self.min_layers:
            self.hidden = self.hidden[:-1]
            return "remove_layer", {}
        return self.add_node(rng)

    def _node(self, rng, hidden_layer, numb, sign):
        if hidden_layer is None:
            hidden_layer = rng.integers(0, len(self.hidden))
        else:
            hidden_layer = min(hidden_layer, len(self.hidden) - 1)
        if numb is None:
            numb = int(rng.choice([16, 32, 64]))
        h = list(self.hidden)
        if sign > 0 and h[hidden_layer] + numb <= self.max_nodes:
            h[hidden_layer] += numb
        if sign < 0 and h[hidden_layer] - numb > self.min_nodes:
            h[hidden_layer] -= numb
        self.hidden = h
        return ("add_node" if sign > 0 else "remove_node"), {"hidden_layer": int(hidden_layer),
                                                             "numb_new_nodes": int(numb)}

    def add_node(self, rng, hidden_layer=None, numb_new_nodes=None):
        return self._node(rng, hidden_layer, numb_new_nodes, +1)

    def remove_node(self, rng, hidden_layer=None, numb_new_nodes=None):
        return self._node(rng, hidden_layer, numb_new_nodes, -1)


@dataclass
class _Net:
    """One EvolvableNetwork (actor or critic) of the agent: encoder, latent, head."""
    encoder: _Mlp
    head: _Mlp
    latent: int
    min_latent: int
    max_latent: int

    def apply(self, method: str, rng, mut_dict: dict | None):
        """-> (applied method name, mutation dict, the modules to recreate)."""
        kw = dict(mut_dict or {})
        if method in ("add_latent_node", "remove_latent_node"):
            numb = kw.get("numb_new_nodes")
            if numb is None:
                numb = int(rng.choice([8, 16, 32]))
            if method == "add_latent_node" and self.latent + numb < self.max_latent:
                self.latent += numb
            if method == "remove_latent_node" and self.latent - numb > self.min_latent:
                self.latent -= numb
            return method, {"numb_new_nodes": int(numb)}, ("encoder", "head")
        owner, name = method.split(".")
        mod = self.encoder if owner == "encoder" else self.head
        applied, d = getattr(mod, name)(rng, **kw)
        return f"{owner}.{applied}", d, (owner if owner == "encoder" else "head",)


def _row_dict(spec: ActorCriticSpec, flat: torch.Tensor, net: str) -> dict[str, dict[str, torch.Tensor]]:
    """{"encoder": {param name: tensor}, "head": {...}} of the actor (net =
    "actor") or the critic, names as inside the module's nn.Sequential."""
    out = {"encoder": {}, "head": {}}
    for key, (off, shape) in spec.state_dict_keys().items():
        top, part = key.split(".")[:2]
        if top != net:
            continue
        out["encoder" if part == "encoder" else "head"][key.split(".model.", 1)[1]] = \
            flat[off:off + int(np.prod(shape))].view(shape)
    return out


def _new_module(spec: ActorCriticSpec, which: str, net: str, m: _Net) -> torch.nn.Module:
    """create_mlp exactly as the reference builds the module (draws from
    torch's global CPU generator)."""
    if which == "encoder":
        return create_mlp(input_size=spec.obs_dim, output_size=m.latent, hidden_size=list(m.encoder.hidden),
                          output_vanish=False, output_activation="ReLU", layer_norm=spec.layer_norm,
                          output_layernorm=spec.layer_norm, activation="ReLU", name=spec.encoder_name)
    return create_mlp(input_size=m.latent, output_size=spec.n_actions if net == "actor" else 1,
                      hidden_size=list(m.head.hidden), output_vanish=True, output_activation=None,
                      layer_norm=spec.layer_norm, output_layernorm=False, activation="ReLU",
                      name="actor" if net == "actor" else "value")


def _preserve(old: dict[str, torch.Tensor], new: torch.nn.Module) -> dict[str, torch.Tensor]:
    """preserve_parameters (modules/base.py:472-502) into a name -> tensor dict."""
    out = {}
    for key, param in new.named_parameters():
        data = param.detach().clone()
        if key in old:
            o = old[key]
            if tuple(o.shape) == tuple(data.shape):
                data = o.detach().clone()
            elif "norm" not in key:
                sl = tuple(slice(0, min(a, b)) for a, b in zip(o.shape, data.shape))
                data[sl] = o[sl]
        out[key] = data
    return out


def _nets(spec: ActorCriticSpec) -> dict[str, _Net]:
    def mlp(hidden, lim):
        return _Mlp(list(hidden), *lim)

    return {"actor": _Net(mlp(spec.encoder_hidden, spec.encoder_limits), mlp(spec.actor_hidden, spec.actor_limits),
                          spec.latent_dim, *spec.latent_limits),
            "critic": _Net(mlp(spec.encoder_hidden, spec.encoder_limits), mlp(spec.critic_hidden, spec.critic_limits),
                           spec.latent_dim, *spec.latent_limits)}


def mutate(spec: ActorCriticSpec, flat: torch.Tensor, method: str, rng: np.random.Generator,
           critic_rng: np.random.Generator | None = None):
    """Apply ``method`` (sampled from the actor's table) to the agent whose
    parameters are ``flat`` (1-D, CPU, ``spec`` layout): the actor first
    (its node / layer draws from ``rng``, the module's generator), then the
    method the actor applied to the critic with the same mutation dict
    (``critic_rng`` only where the critic falls back on its own draws), then
    the shared encoder.  -> (new spec, new flat row (CPU f32), applied
    method or None, mutation dict)."""
    flat = flat.detach().to("cpu", torch.float32)
    nets = _nets(spec)
    old = {net: _row_dict(spec, flat, net) for net in ("actor", "critic")}
    applied, mut_dict, rebuild = nets["actor"].apply(method, rng, None)
    new_mods = {}
    for which in rebuild:  # the actor's recreated modules (encoder first, then head)
        new_mods[("actor", which)] = _preserve(old["actor"][which], _new_module(spec, which, "actor", nets["actor"]))
    c_applied, _, c_rebuild = nets["critic"].apply(applied, critic_rng if critic_rng is not None else rng, mut_dict)
    for which in c_rebuild:
        new_mods[("critic", which)] = _preserve(old["critic"][which],
                                                _new_module(spec, which, "critic", nets["critic"]))
    a, c = nets["actor"], nets["critic"]
    new_spec = copy.deepcopy(spec)
    new_spec.encoder_hidden = list(a.encoder.hidden)
    new_spec.latent_dim = a.latent
    new_spec.actor_hidden = list(a.head.hidden)
    new_spec.critic_hidden = list(c.head.hidden)
    new_spec.__post_init__()
    out = torch.zeros(new_spec.n_params, dtype=torch.float32)
    for key, (off, shape) in new_spec.state_dict_keys().items():
        top, part = key.split(".")[:2]
        if top == "critic" and part == "encoder":
            continue  # one shared encoder region: the actor's (share_encoder_parameters)
        which = "encoder" if part == "encoder" else "head"
        name = key.split(".model.", 1)[1]
        src = new_mods.get((top, which))
        t = src[name] if src is not None else old[top][which][name]
        out[off:off + t.numel()] = t.reshape(-1)
    return new_spec, out, applied, mut_dict
