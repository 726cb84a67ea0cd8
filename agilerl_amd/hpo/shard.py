"""The generation step of a population sharded over ranks, drawn once over
the GLOBAL population.

The reference mutates the whole population in one process, agent after
agent (utils/utils.py:1185-1211 -> hpo/mutation.py:311-362): one
``rng.choice`` over every agent, then each agent's own draws in population
order (RL-hyperparameter draws from the global torch generator, parameter
noise from ``Mutations.rng`` and torch.normal).  A rank that mutated only
its own shard would hand local agent j of every rank the same choice and the
same noise.  Here every rank runs the reference's loop over ALL G*P agents:

  * its own agents are the real objects, mutated in place;
  * the other ranks' agents are ``RemoteAgent`` stand-ins built from a
    gathered host record (hyperparameters, mutation registry, weight shapes):
    they take exactly the draws the real agent takes (the same calls run on
    zero tensors of the same shapes) and their results are discarded — the
    owning rank computes the same values for its real agent.

So the draws happen once, in the global order, identically on every rank,
and rank r keeps global slots r*P .. r*P + P - 1: the sharded population
equals the single-process one.  Before the draws the host generators
(numpy global, torch CPU, Python ``random``) are broadcast from rank 0, so a
rank whose local work consumed a stream differently (an off-policy rank's
own replay sampling) cannot desynchronise the selection or the mutations.

A mutation registry shared by construction (``create_population`` hands
every agent one ``hp_config`` object, whose ``RLParameter.value`` then
carries over from one agent's mutation to the next, registry.py) is shared
across ranks the same way: when every rank's agents share one object, the
stand-ins use the local shared object, which every rank advances through
the identical global sequence.
"""

from __future__ import annotations

import copy
import os
import pickle
import random
import time

import numpy as np
import torch
import torch.distributed as dist

#: per-agent RL hyperparameters a PPO view exposes as properties (not in vars)
_PPO_HP = ("lr", "batch_size", "update_epochs", "ent_coef", "learn_step")


#: per tag: [calls, seconds, pickled bytes this rank contributed] of the host-object
#: collectives of the generation step (diagnostic, enabled by AGX_SHARD_STATS=1;
#: the byte count pickles the payload once more)
EXCHANGE_STATS: dict[str, list] = {}


def _record(tag: str, t0: float, obj) -> None:
    if os.environ.get("AGX_SHARD_STATS"):
        st = EXCHANGE_STATS.setdefault(tag, [0, 0.0, 0])
        st[0] += 1
        st[1] += time.perf_counter() - t0
        st[2] += len(pickle.dumps(obj))


def all_gather_obj(box: list, obj, group=None, tag: str = "other") -> None:
    """dist.all_gather_object, timed per tag (EXCHANGE_STATS)."""
    t0 = time.perf_counter()
    dist.all_gather_object(box, obj, group=group)
    _record(tag, t0, obj)


def broadcast_obj(box: list, src: int, group=None, tag: str = "other") -> None:
    """dist.broadcast_object_list, timed per tag (EXCHANGE_STATS)."""
    t0 = time.perf_counter()
    dist.broadcast_object_list(box, src=src, group=group)
    _record(tag, t0, box)


def world_rank(group=None) -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def all_ranks(flag: bool, group=None) -> bool:
    """True on every rank iff ``flag`` holds on every rank (a decision that
    ends a rank's loop must be the same everywhere)."""
    world, _ = world_rank(group)
    if world == 1:
        return bool(flag)
    box: list = [None] * world
    all_gather_obj(box, bool(flag), group=group, tag="stop_flag")
    return all(box)


def sync_host_rngs(group=None) -> None:
    """Every rank takes rank 0's numpy global, torch CPU and Python random
    states (one object broadcast, a few KB)."""
    world, rank = world_rank(group)
    if world == 1:
        return
    box = [(np.random.get_state(legacy=True), torch.get_rng_state(), random.getstate())] if rank == 0 else [None]
    src = dist.get_global_rank(group, 0) if group is not None else 0
    broadcast_obj(box, src=src, group=group, tag="host_rngs")
    if rank != 0:
        np_state, t_state, py_state = box[0]
        np.random.set_state(np_state)
        torch.set_rng_state(t_state)
        random.setstate(py_state)


def _weight_groups(agent) -> list[dict[str, torch.Tensor]]:
    if hasattr(agent, "policy_weight_groups"):
        return agent.policy_weight_groups()
    if hasattr(agent, "policy_weights"):
        return [agent.policy_weights()]
    return []


def host_record(agent, adam_steps: dict | None = None) -> dict:
    """What another rank needs to replay this agent's mutation draws and to
    clone its host attributes: plain attributes, the hyperparameters the
    registry can mutate, the registry itself, the learning-rate names and the
    shapes of the policy's weights.  ``adam_steps``: id(population) -> its
    Adam step counts on the host (one device read per population, not one
    per agent)."""
    from .sharded import plain_attributes

    rec = plain_attributes(agent)
    hp = {}
    names = set(_PPO_HP) if hasattr(agent, "population") else set()
    registry = getattr(agent, "registry", None)
    cfg = getattr(registry, "hp_config", None)
    if cfg:
        names |= set(cfg.names())
    for name in sorted(names):
        try:
            hp[name] = getattr(agent, name)
        except (AttributeError, NotImplementedError):
            pass
    rec["_hp"] = hp
    rec["_registry"] = registry
    rec["_lr_names"] = list(agent.get_lr_names()) if hasattr(agent, "get_lr_names") else []
    rec["_weights"] = [[(k, tuple(t.shape), str(t.dtype).replace("torch.", "")) for k, t in g.items()]
                       for g in _weight_groups(agent)]
    rec["_groups_api"] = hasattr(agent, "policy_weight_groups")
    rec["algo"] = getattr(agent, "algo", None)
    if hasattr(agent, "population"):  # a PPO view: what a clone of it on another rank is made of
        rec["_spec"] = agent.spec
        steps = None if adam_steps is None else adam_steps.get(id(agent.population))
        rec["_adam_step"] = int(agent.population.opt.steps[agent.row] if steps is None else steps[agent.row])
        rngs = [agent.module_rng, agent.critic_rng]
        if hasattr(agent, "kernel_rng"):  # image actor-critics also draw kernel sizes (image_arch.mutate)
            rngs += [agent.kernel_rng, agent.critic_kernel_rng]
        rec["_arch_rngs"] = tuple(g.bit_generator.state for g in rngs)
    return rec


class RemoteAgent:
    """Stand-in for an agent another rank owns: takes the same mutation draws
    (hyperparameter reads and writes, zero tensors of the policy's weight
    shapes for parameter noise); nothing it computes is used."""

    def __init__(self, rec: dict, registry) -> None:
        d = self.__dict__
        for k, v in rec.items():
            if not k.startswith("_"):
                d[k] = copy.deepcopy(v)
        d["registry"] = registry
        d["_hp"] = dict(rec["_hp"])
        d["_lr_names"] = list(rec["_lr_names"])
        d["_weights"] = rec["_weights"]
        d["_groups_api"] = rec["_groups_api"]
        d["_spec"] = rec.get("_spec")
        d["_arch_rngs"] = rec.get("_arch_rngs")

    def __getattr__(self, name):
        hp = self.__dict__.get("_hp", {})
        if name in hp:
            return hp[name]
        raise AttributeError(name)

    def __setattr__(self, name, value) -> None:
        if name in self.__dict__.get("_hp", {}):
            self.__dict__["_hp"][name] = value
        else:
            self.__dict__[name] = value

    def _zeros(self) -> list[dict[str, torch.Tensor]]:
        return [{k: torch.zeros(shape, dtype=getattr(torch, dt)) for k, shape, dt in g} for g in self._weights]

    def policy_weight_groups(self):
        return self._zeros()

    def policy_weights(self):
        return self._zeros()[0]

    def get_lr_names(self) -> list[str]:
        return list(self._lr_names)

    def reinit_optimizers(self, *args, **kwargs) -> None:
        pass

    def sync_shared_networks(self) -> None:
        pass

    def mutation_hook(self) -> None:
        pass

    @property
    def can_mutate_architecture(self) -> bool:
        return self.__dict__.get("_spec") is not None

    def architecture_mutation(self, new_layer_prob: float, rng):
        """The draws of a PPO view's architecture mutation (population/arch.py
        for MLP actor-critics, population/image_arch.py for CNN ones): the
        method from ``rng`` (Mutations.rng), the module generators' node /
        layer / kernel draws, and torch's global CPU generator for the fresh
        weights (the same modules built on zeros)."""
        if self._spec is None:
            raise AttributeError("architecture_mutation")
        from ..population import arch, image_arch
        from ..population.image_nets import ImageActorCriticSpec

        gens = []
        for st in self._arch_rngs:
            g = np.random.default_rng()
            g.bit_generator.state = st
            gens.append(g)
        zeros = torch.zeros(self._spec.n_params)
        if isinstance(self._spec, ImageActorCriticSpec):
            if len(gens) != 4:
                raise ValueError("an image actor-critic record carries four architecture generators")
            method = image_arch.sample_method(new_layer_prob, rng)
            _, _, applied, _ = image_arch.mutate(self._spec, zeros, method, gens[0], gens[2], gens[1], gens[3])
        else:
            method = arch.sample_method(new_layer_prob, rng)
            _, _, applied, _ = arch.mutate(self._spec, zeros, method, gens[0], gens[1])
        return applied


def _local_records(pop) -> list[dict]:
    adam_steps = {}
    for a in pop:
        if hasattr(getattr(a, "population", None), "opt") and id(a.population) not in adam_steps:
            adam_steps[id(a.population)] = a.population.opt.steps.cpu().numpy()
    return [host_record(a, adam_steps) for a in pop]


def gather_fitness_records(pop, fitness: list, with_records: bool, group=None) -> tuple[list, list | None]:
    """The generation's fitness scalars of every rank (global order) and, when
    the generation step follows, every rank's agent records — one collective
    instead of two.  -> (global fitness, global records or None)."""
    world, _ = world_rank(group)
    local = (list(fitness), _local_records(pop) if with_records else None)
    if world == 1:
        return local
    box: list = [None] * world
    all_gather_obj(box, local, group=group, tag="fitness_records" if with_records else "fitness")
    if with_records and any(len(b[1]) != len(pop) for b in box):
        raise ValueError("every rank must hold the same number of agents")
    return [f for b in box for f in b[0]], ([r for b in box for r in b[1]] if with_records else None)


def gather_records(pop, group=None) -> list[dict]:
    """Every rank's agent records, in global agent order."""
    world, _ = world_rank(group)
    local = _local_records(pop)
    if world == 1:
        return local
    box: list = [None] * world
    all_gather_obj(box, local, group=group, tag="agent_records")
    if any(len(b) != len(pop) for b in box):
        raise ValueError("every rank must hold the same number of agents")
    return [r for b in box for r in b]


def mark_shared(hp_config) -> None:
    """Tag an hp_config that create_population hands to every agent; a deep
    copy (a clone's) no longer matches its tag, so it counts as private."""
    if hp_config is not None:
        try:
            hp_config._agx_share_id = id(hp_config)
        except AttributeError:
            pass


def _locally_shared_registry(pop):
    """A registry whose hp_config every local agent shares by construction
    (create_population's), or None."""
    regs = [getattr(a, "registry", None) for a in pop]
    cfgs = [getattr(r, "hp_config", None) for r in regs]
    c0 = cfgs[0] if cfgs else None
    if c0 is not None and all(c is c0 for c in cfgs) and getattr(c0, "_agx_share_id", None) == id(c0):
        return regs[0]
    return None


def global_view(pop, records: list[dict], group=None, all_shared: bool | None = None) -> list:
    """The global population as seen from this rank: its own agents in their
    global slots, RemoteAgent stand-ins elsewhere.  ``all_shared``: whether
    every rank's agents share one registry by construction (gathered here
    when not given)."""
    world, rank = world_rank(group)
    P = len(pop)
    shared = _locally_shared_registry(pop)
    if all_shared is None:
        flags = [shared is not None]
        if world > 1:
            box: list = [None] * world
            all_gather_obj(box, flags, group=group, tag="registry_flags")
            all_shared = all(b[0] for b in box)
        else:
            all_shared = flags[0]
    out = []
    for g, rec in enumerate(records):
        if g // P == rank:
            out.append(pop[g % P])
        else:
            out.append(RemoteAgent(rec, shared if all_shared else copy.deepcopy(rec["_registry"])))
    return out


def mark_sharded(pop) -> None:
    """Flag every local object-level agent as one shard of a global
    population.  The entry points treat any run with more than one rank as
    one population split over the ranks (the draws are replayed globally,
    selection is the sharded tournament), so an agent built outside
    ``create_population`` — directly, by ``load()``, or with
    ``shard=False`` — must take the sharded rules too: otherwise it would
    mutate its architecture on its own rank while the other ranks' stand-ins
    draw nothing, and the ranks' streams would diverge."""
    for a in pop:
        if hasattr(type(a), "sharded"):
            a.sharded = True


def mutate_population(mutation, pop, pre_training_mut: bool = False, group=None):
    """``mutation.mutation(pop)`` over the global population; returns this
    rank's slice (the real agents, mutated)."""
    world, rank = world_rank(group)
    if world == 1:
        return mutation.mutation(pop, pre_training_mut=pre_training_mut)
    mark_sharded(pop)
    # one collective for the three things the global draws need: rank 0's host
    # generator states (every rank takes them, as sync_host_rngs would), every
    # rank's agent records (gather_records) and its shared-registry flag
    # (global_view) — one exchange latency per generation instead of three
    rngs = (np.random.get_state(legacy=True), torch.get_rng_state(), random.getstate()) if rank == 0 else None
    local = (rngs, _local_records(pop), _locally_shared_registry(pop) is not None)
    box: list = [None] * world
    all_gather_obj(box, local, group=group, tag="mutation_state")
    if any(len(b[1]) != len(pop) for b in box):
        raise ValueError("every rank must hold the same number of agents")
    if rank != 0:
        np_state, t_state, py_state = box[0][0]
        np.random.set_state(np_state)
        torch.set_rng_state(t_state)
        random.setstate(py_state)
    records = [r for b in box for r in b[1]]
    glob = global_view(pop, records, group, all_shared=all(b[2] for b in box))
    out = mutation.mutation(glob, pre_training_mut=pre_training_mut)
    P = len(pop)
    mine = out[rank * P:(rank + 1) * P]
    if any(isinstance(a, RemoteAgent) for a in mine):
        raise RuntimeError("mutation returned a stand-in in this rank's slots")
    return mine
