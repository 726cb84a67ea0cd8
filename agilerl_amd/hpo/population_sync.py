"""Generation step of a GPU-resident population, sharded over ranks.

Replaces tournament_selection_and_mutation's accelerate path
(agilerl/utils/utils.py:1185-1211: rank 0 selects, writes every agent's
checkpoint to a shared filesystem, the other ranks reload) with:
  1. fitness: mean return of the episodes finished since the last generation
     (per agent, on device);
  2. RCCL all-gather of the P fitness scalars of every rank over xGMI — the
     only collective;
  3. identical seeded tournament selection on every rank (select_parents), so
     every rank knows the whole transfer plan without exchanging it;
  4. each parent row that lives on another rank crosses once, point to point
     (one packed [rows, params | exp_avg | exp_avg_sq] message per (source,
     destination) pair that has any), local parents are copied on device.
Single rank: step 2 is the identity and step 4 a local gather.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .tournament import select_parents


class PopulationSync:
    def __init__(self, pop, runner, world: int = 1, rank: int = 0, seed: int = 42, tournament_size: int = 2,
                 elitism: bool = True, eval_loop: int = 1):
        self.pop, self.runner = pop, runner
        self.world, self.rank = world, rank
        # seed=None: draw from the GLOBAL numpy RNG, exactly as the reference's
        # TournamentSelection does (tournament.py:41-51); else a private stream
        self.rng_state = None if seed is None else np.random.RandomState(seed)
        self.fitness_override = None  # host fitness for the next generation (else from the episode stats)
        self.tournament_size, self.elitism, self.eval_loop = tournament_size, elitism, eval_loop
        self.history: list[np.ndarray] = []
        self.last_parents: list[int] = []

    def _fitness(self) -> torch.Tensor:
        if self.fitness_override is not None:
            f = torch.as_tensor(np.asarray(self.fitness_override, dtype=np.float64), device=self.pop.device)
            self.fitness_override = None
            self.runner.reset_episode_stats()
            return f
        r = self.runner
        f = torch.where(r.episodes > 0, r.episode_return_sum / r.episodes.clamp(min=1).double(),
                        torch.full_like(r.episode_return_sum, -1e9))
        r.reset_episode_stats()
        return f

    def _all_gather(self, x: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return x
        out = torch.empty((self.world * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous())
        return out

    @torch.no_grad()
    def _clone_rows(self, parents: list[int]) -> None:
        """Row j of this rank becomes global row parents[rank*P + j] (params and
        both Adam moments)."""
        pop, P, me = self.pop, self.pop.P, self.rank
        bufs = (pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq)
        n = bufs[0].shape[1]
        # rows each rank needs from each other rank (sorted, unique): the same
        # plan on every rank, derived from the shared parent list
        need = [[sorted({q % P for q in parents[r * P:(r + 1) * P] if q // P == src}) if src != r else []
                 for src in range(self.world)] for r in range(self.world)]
        ops, recv = [], {}
        sends = []
        for dst in range(self.world):
            rows = need[dst][me]
            if rows:
                idx = torch.as_tensor(rows, device=pop.device)
                msg = torch.cat([b.index_select(0, idx) for b in bufs], dim=1).contiguous()
                sends.append(msg)
                ops.append(dist.P2POp(dist.isend, msg, dst))
        for src in range(self.world):
            rows = need[me][src]
            if rows:
                recv[src] = torch.empty(len(rows), 3 * n, dtype=bufs[0].dtype, device=pop.device)
                ops.append(dist.P2POp(dist.irecv, recv[src], src))
        mine = parents[me * P:(me + 1) * P]
        local = [j for j in range(P) if mine[j] // P == me]
        snap = None
        if local:
            idx = torch.as_tensor([mine[j] % P for j in local], device=pop.device)
            snap = [b.index_select(0, idx) for b in bufs]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if local:
            dst_idx = torch.as_tensor(local, device=pop.device)
            for b, sv in zip(bufs, snap):
                b.index_copy_(0, dst_idx, sv)
        for src, msg in recv.items():
            pos = {row: k for k, row in enumerate(need[me][src])}
            js = [j for j in range(P) if mine[j] // P == src]
            sel = torch.as_tensor([pos[mine[j] % P] for j in js], device=pop.device)
            dst_idx = torch.as_tensor(js, device=pop.device)
            rows = msg.index_select(0, sel)
            for k, b in enumerate(bufs):
                b.index_copy_(0, dst_idx, rows[:, k * n:(k + 1) * n])

    @torch.no_grad()
    def generation(self) -> list[int]:
        pop = self.pop
        fit = self._all_gather(self._fitness()).cpu().numpy()  # the only host sync of the step
        self.history.append(fit)
        fits = [np.stack([h[i] for h in self.history[-self.eval_loop:]]) for i in range(len(fit))]
        if self.rng_state is None:
            _, parents = select_parents(fits, self.tournament_size, self.elitism, self.eval_loop)
        else:
            state = np.random.get_state()
            np.random.set_state(self.rng_state.get_state())
            _, parents = select_parents(fits, self.tournament_size, self.elitism, self.eval_loop)
            self.rng_state.set_state(np.random.get_state())
            np.random.set_state(state)
        self._clone_rows(parents)
        self.last_parents = parents
        return parents
