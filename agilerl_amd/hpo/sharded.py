"""Tournament selection for an object-level population sharded over ranks.

The reference runs multi-process training through accelerate and selects on
rank 0 only, syncing every agent through checkpoint files on a shared
filesystem (agilerl/utils/utils.py:1185-1211).  Here each rank holds a shard
of ``P`` agents (global position ``rank * P + j``), and one generation is:

  1. one all-gather of every agent's plain attributes (fitness history,
     scores, steps, index, ...) — the only collective;
  2. identical selection on every rank: ``select_parents`` with the GLOBAL
     numpy RNG, exactly the draws of ``TournamentSelection.select``
     (tournament.py:41-119) over the concatenated population, so a common
     ``np.random.seed`` gives every rank the same parent list;
  3. each parent that lives on another rank crosses once, point to point: one
     packed byte message per (source, destination) pair holding every tensor
     of those parents (network state dicts, optimizer moments, exploration
     tensors), in a fixed walk order; local parents are cloned in place.

Indices follow the single-process rule: the elite keeps its index, the other
slots get ``max_id + 1, max_id + 2, ...`` in global slot order.  The returned
elite is the clone in global slot 0 (rank 0) and ``None`` on other ranks, as
the reference saves the elite on the main process only.

Used by DQN / RainbowDQN / MADDPG populations (configs 3 and 4 sharded); the
GPU-resident PPO population uses ``population_sync.PopulationSync``, which
moves parameter rows directly.  Architecture mutations are out of scope:
every agent must pack to the same byte layout (checked, ``ValueError``).
"""

from __future__ import annotations

import copy

import numpy as np
import torch
import torch.distributed as dist

from .shard import all_gather_obj
from .tournament import TournamentSelection, select_parents

_PLAIN = (bool, int, float, str, type(None), np.integer, np.floating)


def _is_plain(v) -> bool:
    if isinstance(v, _PLAIN):
        return True
    if isinstance(v, (list, tuple)):
        return all(_is_plain(x) for x in v)
    if isinstance(v, dict):
        return all(isinstance(k, str) and _is_plain(x) for k, x in v.items())
    return False


def plain_attributes(agent) -> dict:
    """The non-tensor, non-module attributes the reference's copy_attributes
    carries over (core/base.py:444-500), restricted to plain data."""
    return {k: copy.deepcopy(v) for k, v in vars(agent).items() if _is_plain(v)}


def _ensure_adam_state(opt: torch.optim.Optimizer) -> None:
    """Materialise lazily-created Adam state (zero moments, step 0): identical
    to an untouched optimizer on its next step, and gives every agent the same
    byte layout whether or not it has learned yet."""
    for group in opt.param_groups:
        for p in group["params"]:
            st = opt.state[p]
            if len(st) == 0 and isinstance(opt, torch.optim.Adam):
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if group.get("amsgrad", False):
                    st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)


def state_tensors(agent) -> list[torch.Tensor]:
    """Every tensor that defines the agent, in a fixed order: attributes by
    name; modules via state_dict; optimizers via their per-parameter state in
    param-group order; dicts by sorted key.  Shared storage is listed once."""
    out: list[torch.Tensor] = []
    seen: set[tuple] = set()

    def add(t: torch.Tensor) -> None:
        key = (t.device, t.data_ptr(), t.dtype, tuple(t.shape))
        if t.numel() == 0 or key in seen:
            return
        seen.add(key)
        out.append(t)

    def walk(v) -> None:
        if isinstance(v, torch.Tensor):
            add(v.data)
        elif isinstance(v, torch.nn.Module):
            for t in v.state_dict().values():
                if isinstance(t, torch.Tensor):
                    add(t)
        elif isinstance(v, torch.optim.Optimizer):
            _ensure_adam_state(v)
            for group in v.param_groups:
                for p in group["params"]:
                    st = v.state[p]
                    for k in sorted(st):
                        if isinstance(st[k], torch.Tensor):
                            add(st[k])
        elif isinstance(v, dict):
            for k in sorted(v, key=str):
                walk(v[k])
        elif isinstance(v, (list, tuple)) and not _is_plain(v):
            for x in v:
                walk(x)

    for name in sorted(vars(agent)):
        walk(getattr(agent, name))
    return out


def _bytes_of(t: torch.Tensor) -> torch.Tensor:
    return t.detach().contiguous().reshape(-1).view(torch.uint8)


def pack_agent(agent, device) -> torch.Tensor:
    return torch.cat([_bytes_of(t).to(device) for t in state_tensors(agent)])


@torch.no_grad()
def unpack_agent(agent, msg: torch.Tensor) -> None:
    off = 0
    for t in state_tensors(agent):
        n = t.numel() * t.element_size()
        t.reshape(-1).view(torch.uint8).copy_(msg[off:off + n].to(t.device))
        off += n
    if off != msg.numel():
        raise ValueError(f"agent state is {off} bytes, message {msg.numel()}")


class ShardedTournamentSelection:
    """``select(local_pop) -> (elite | None, new_local_pop)`` over the
    population formed by every rank's shard (equal shard sizes)."""

    def __init__(self, tournament: TournamentSelection, group=None):
        self.tournament = tournament
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.last_parents: list[int] = []

    def _device(self):
        if dist.is_initialized() and dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def select(self, population):
        t, world, me = self.tournament, self.world, self.rank
        P = len(population)
        nbytes = sum(x.numel() * x.element_size() for x in state_tensors(population[0]))
        info = [dict(plain_attributes(a), _nbytes=sum(x.numel() * x.element_size() for x in state_tensors(a)),
                     _registry=getattr(a, "registry", None))  # a clone deep-copies the parent's (values included)
                for a in population]
        if world > 1:
            gathered: list = [None] * world
            all_gather_obj(gathered, info, group=self.group, tag="tournament_attributes")
        else:
            gathered = [info]
        if any(len(g) != P for g in gathered):
            raise ValueError("ShardedTournamentSelection: every rank must hold the same number of agents")
        meta = [m for g in gathered for m in g]
        if any(m["_nbytes"] != nbytes for m in meta):
            raise ValueError("ShardedTournamentSelection: agents differ in state layout (architecture mutations "
                             "are outside the agx path)")
        fit = [m.get("fitness", []) for m in meta]
        elite_pos, parents = select_parents(fit, t.tournament_size, t.elitism, t.eval_loop)
        self.last_parents = parents
        max_id = max(m["index"] for m in meta)
        new_index = []
        for i in range(len(parents)):
            if t.elitism and i == 0:
                new_index.append(meta[parents[0]]["index"])
            else:
                max_id += 1
                new_index.append(max_id)

        # point-to-point plan, identical on every rank: need[dst][src] = sorted
        # unique local positions on src of the parents dst clones
        need = [[sorted({q % P for q in parents[d * P:(d + 1) * P] if q // P == s}) if s != d else []
                 for s in range(world)] for d in range(world)]
        dev = self._device()
        ops, recv, sends = [], {}, []
        for dst in range(world):
            rows = need[dst][me]
            if rows:
                msg = torch.cat([pack_agent(population[j], dev) for j in rows])
                sends.append(msg)
                ops.append(dist.P2POp(dist.isend, msg, dst, group=self.group))
        for src in range(world):
            rows = need[me][src]
            if rows:
                recv[src] = torch.empty(len(rows) * nbytes, dtype=torch.uint8, device=dev)
                ops.append(dist.P2POp(dist.irecv, recv[src], src, group=self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()

        new_pop = []
        for j in range(P):
            g = me * P + j
            q = parents[g]
            if q // P == me:
                child = population[q % P].clone(new_index[g], wrap=False)
            else:
                src = q // P
                k = need[me][src].index(q % P)
                child = population[0].clone(new_index[g], wrap=False)
                unpack_agent(child, recv[src][k * nbytes:(k + 1) * nbytes])
                for name, v in meta[q].items():
                    if name not in ("_nbytes", "_registry"):
                        setattr(child, name, copy.deepcopy(v))
                if meta[q]["_registry"] is not None:
                    child.registry = copy.deepcopy(meta[q]["_registry"])
                    if hasattr(child, "hp_config"):
                        child.hp_config = child.registry.hp_config
                child.index = new_index[g]
            new_pop.append(child)
        elite = new_pop[0].clone(wrap=False) if (t.elitism and me == 0) else None
        return elite, new_pop


def select_population(tournament: TournamentSelection, population):
    """The entry points' selection step: the per-process tournament, or the
    sharded one when a torch.distributed group of more than one rank is up."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        from .shard import mark_sharded

        mark_sharded(population)
        return ShardedTournamentSelection(tournament).select(population)
    return tournament.select(population)
