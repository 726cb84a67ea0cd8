"""Architecture mutations of an image PPO actor-critic (BASELINE config 5)
held as a flat parameter row (``ImageActorCriticSpec``).

The reference mutates the policy of a PPO agent (hpo/mutation.py:829-885):
a method sampled from the actor's table with ``Mutations.rng``, applied to
the actor, the method the actor applied then applied to the critic with the
same mutation dict (``_apply_arch_mutation``, :1013-1070), and the critic's
encoder given the actor's parameters (share_encoder_parameters,
utils/algo_utils.py:164-187).  With an EvolvableCNN encoder the actor's table
is, in the order the reference's ``list(set(...))`` gives under
PYTHONHASHSEED=0 (modules/base.py:570-571; the encoder's LAYER methods are
disabled, networks/base.py:266-268):

  head_net.remove_layer, head_net.add_layer, remove_latent_node,
  add_latent_node, encoder.remove_channel, encoder.change_kernel,
  encoder.add_channel, head_net.add_node, head_net.remove_node

The mutation runs on module copies of the row: the agx ``EvolvableCNN``
(modules/cnn.py, its mutation methods bit-exact against the reference) and
``EvolvableMLP`` heads, so every recreated module draws its fresh weights
from torch's global CPU generator in the reference's order (actor encoder,
actor head, then the critic's).  Draws: a network and its modules share one
generator (ModuleMeta, modules/base.py:253-255); the CNN's kernel-size helper
keeps its own (MutableKernelSizes is not a module).  Pinned against the
reference's own networks: tests/golden/gen_arch_golden.py (cnnarch*).
"""

from __future__ import annotations

import copy

import numpy as np
import torch

from ..modules.cnn import EvolvableCNN
from ..modules.mlp import EvolvableMLP
from .image_nets import ImageActorCriticSpec

LAYER_METHODS = ["head_net.remove_layer", "head_net.add_layer"]
NODE_METHODS = ["remove_latent_node", "add_latent_node", "encoder.remove_channel", "encoder.change_kernel",
                "encoder.add_channel", "head_net.add_node", "head_net.remove_node"]
METHODS = LAYER_METHODS + NODE_METHODS
METHOD_ORDER_HASH_SEED = "0"


def method_probs(new_layer_prob: float) -> list[float]:
    """EvolvableModule.get_mutation_probs (modules/base.py:661-685)."""
    nl, nn_ = len(LAYER_METHODS), len(NODE_METHODS)
    return [new_layer_prob / nl] * nl + [(1 - new_layer_prob) / nn_] * nn_


def sample_method(new_layer_prob: float, rng: np.random.Generator) -> str:
    """sample_mutation_method (modules/base.py:687-711) with Mutations.rng."""
    return str(rng.choice(METHODS, p=method_probs(new_layer_prob), size=1)[0])


class _Net:
    """One EvolvableNetwork of the agent (actor or critic) as modules."""

    def __init__(self, spec: ImageActorCriticSpec, flat: torch.Tensor, which: str, rng, kernel_rng):
        self.spec, self.which = spec, which
        cmin_l, cmax_l, cmin, cmax = spec.cnn_limits
        self.encoder = EvolvableCNN(input_shape=list(spec.obs_shape), num_outputs=spec.latent_dim,
                                    channel_size=list(spec.channel_size), kernel_size=list(spec.kernel_size),
                                    stride_size=list(spec.stride_size), min_hidden_layers=cmin_l,
                                    max_hidden_layers=cmax_l, min_channel_size=cmin, max_channel_size=cmax,
                                    output_activation="ReLU", name=spec.encoder_name)
        self.encoder.disable_mutations("layer")
        lim = spec.actor_limits if which == "actor" else spec.critic_limits
        self.head = EvolvableMLP(num_inputs=spec.latent_dim, num_outputs=spec.n_actions if which == "actor" else 1,
                                 hidden_size=list(spec.actor_hidden if which == "actor" else spec.critic_hidden),
                                 activation="ReLU", output_activation=None, min_hidden_layers=lim[0],
                                 max_hidden_layers=lim[1], min_mlp_nodes=lim[2], max_mlp_nodes=lim[3],
                                 layer_norm=spec.head_layer_norm, output_vanish=True,
                                 name="actor" if which == "actor" else "value")
        self.latent, (self.min_latent, self.max_latent) = spec.latent_dim, spec.latent_limits
        keys = spec.state_dict_keys()
        enc_prefix = f"{which}.encoder.model."
        head_prefix = "actor.head_net._wrapped.model." if which == "actor" else "critic.head_net.model."
        with torch.no_grad():
            for key, (off, shape) in keys.items():
                t = flat[off:off + int(np.prod(shape))].view(shape)
                if key.startswith(enc_prefix):
                    self.encoder.model.get_parameter(key[len(enc_prefix):]).copy_(t)
                elif key.startswith(head_prefix):
                    self.head.model.get_parameter(key[len(head_prefix):]).copy_(t)
        self.rng = self.encoder.rng = self.head.rng = rng
        self.encoder.kernel_rng = kernel_rng

    def apply(self, method: str, mut_dict: dict | None):
        """-> (applied method or None, mutation dict)."""
        kw = dict(mut_dict or {})
        if method in ("add_latent_node", "remove_latent_node"):
            numb = kw.get("numb_new_nodes")
            if numb is None:
                numb = int(self.rng.choice([8, 16, 32]))
            if method == "add_latent_node" and self.latent + numb < self.max_latent:
                self.latent += numb
            if method == "remove_latent_node" and self.latent - numb > self.min_latent:
                self.latent -= numb
            # EvolvableNetwork.recreate_network: the encoder (-> latent), then the head
            self.encoder.num_outputs = self.latent
            self.encoder.recreate_network()
            self.head.num_inputs = self.latent
            self.head.recreate_network()
            return method, {"numb_new_nodes": int(numb)}
        owner, name = method.split(".")
        mod = self.encoder if owner == "encoder" else self.head
        d = getattr(mod, name)(**kw)
        if mod.last_mutation_attr is None:
            return None, d or {}
        return f"{owner}.{mod.last_mutation_attr}", d or {}


def mutate(spec: ImageActorCriticSpec, flat: torch.Tensor, method: str, rng: np.random.Generator,
           kernel_rng: np.random.Generator, critic_rng: np.random.Generator | None = None,
           critic_kernel_rng: np.random.Generator | None = None):
    """Apply ``method`` (sampled from the actor's table) to the agent whose
    parameters are ``flat`` (1-D, ``spec`` layout): the actor first, then the
    method the actor applied to the critic with the same mutation dict, then
    the shared encoder.  -> (new spec, new flat row (CPU f32), applied method
    or None, mutation dict)."""
    flat = flat.detach().to("cpu", torch.float32)
    # the module copies' own construction must not advance torch's generator:
    # only the recreated modules draw, as in the reference
    with torch.random.fork_rng(devices=[]):
        actor = _Net(spec, flat, "actor", rng, kernel_rng)
        critic = _Net(spec, flat, "critic", critic_rng if critic_rng is not None else rng,
                      critic_kernel_rng if critic_kernel_rng is not None else kernel_rng)
    applied, mut_dict = actor.apply(method, None)
    if applied is not None:
        critic.apply(applied, mut_dict)
    enc, a_head, c_head = actor.encoder, actor.head, critic.head
    new_spec = copy.deepcopy(spec)
    new_spec.channel_size, new_spec.kernel_size = list(enc.channel_size), list(enc.kernel_size)
    new_spec.stride_size, new_spec.latent_dim = list(enc.stride_size), actor.latent
    new_spec.actor_hidden, new_spec.critic_hidden = list(a_head.hidden_size), list(c_head.hidden_size)
    new_spec.__post_init__()
    out = torch.zeros(new_spec.n_params, dtype=torch.float32)
    for key, (off, shape) in new_spec.state_dict_keys().items():
        if key.startswith("critic.encoder."):
            continue  # one shared encoder region: the actor's (share_encoder_parameters)
        if key.startswith("actor.encoder.model."):
            t = enc.model.get_parameter(key[len("actor.encoder.model."):])
        elif key.startswith("actor.head_net._wrapped.model."):
            t = a_head.model.get_parameter(key[len("actor.head_net._wrapped.model."):])
        else:
            t = c_head.model.get_parameter(key[len("critic.head_net.model."):])
        out[off:off + t.numel()] = t.detach().reshape(-1)
    return new_spec, out, applied, mut_dict
