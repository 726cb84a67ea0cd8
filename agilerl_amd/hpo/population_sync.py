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

import os

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
        self._side = None      # stream for the fitness read (behind the rollout only)
        self._fit_h = None     # pinned landing buffer of the gathered fitness
        self._idx_h = None     # pinned parent indices -> device, non-blocking
        self._idx_d = None
        self._idx_ev = None
        # loopback (tests): a one-rank group runs the multi-rank exchange — every
        # parent row is packed, sent to this rank through the backend and
        # unpacked — so the device-tensor collective path (RCCL) executes on a
        # one-GPU box exactly as between ranks
        self.loopback = False
        # gloo moves host tensors only: device rows cross through host staging
        self.comm_device = pop.device
        if world > 1 and dist.get_backend() == "gloo":
            self.comm_device = torch.device("cpu")

    def _fitness_host(self) -> np.ndarray:
        """Every rank's fitness on the host.  The episode statistics are final
        once the rollout is (runner.stats_event); they are reduced, gathered
        (RCCL) and copied out on a side stream that waits only for that event,
        so the host does not wait for the learner queued behind the rollout."""
        if self.fitness_override is not None:
            f = np.asarray(self.fitness_override, dtype=np.float64)
            self.fitness_override = None
            self.runner.reset_episode_stats()
            if self.world == 1:
                return f
            t = torch.as_tensor(f, device=self.pop.device)
            return self._all_gather(t).cpu().numpy()
        r = self.runner
        ev = getattr(r, "stats_event", None)
        if self.pop.device.type != "cuda" or ev is None:
            f = torch.where(r.episodes > 0, r.episode_return_sum / r.episodes.clamp(min=1).double(),
                            torch.full_like(r.episode_return_sum, -1e9))
            r.reset_episode_stats()
            return self._all_gather(f).cpu().numpy()
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.pop.device)
            self._fit_h = torch.empty(self.world * self.pop.P, dtype=torch.float64, pin_memory=True)
        side = self._side
        side.wait_event(ev)
        with torch.cuda.stream(side):
            eps = r.episodes
            f = torch.where(eps > 0, r.episode_return_sum / eps.clamp(min=1).double(),
                            torch.full_like(r.episode_return_sum, -1e9))
            g = self._all_gather(f)
            self._fit_h.copy_(g, non_blocking=True)
            done = torch.cuda.Event()
            done.record(side)
        done.synchronize()
        r.reset_episode_stats()  # on the main stream: after the queued learner, before the next rollout
        return self._fit_h.numpy().copy()

    def _all_gather(self, x: torch.Tensor) -> torch.Tensor:
        if self.world == 1 and not self.loopback:
            return x
        src = x.contiguous().to(self.comm_device)
        out = torch.empty((self.world * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=self.comm_device)
        dist.all_gather_into_tensor(out, src)
        return out.to(x.device)

    def _dev_index(self, rows: list[int]) -> torch.Tensor:
        """A small index list on the device without a blocking copy: pinned
        staging (re-used only after its previous copy has landed)."""
        n = len(rows)
        if self._idx_h is None or self._idx_h.numel() < n:
            m = max(n, self.pop.P)
            self._idx_h = torch.empty(m, dtype=torch.int64, pin_memory=True)
            self._idx_d = torch.empty(m, dtype=torch.int64, device=self.pop.device)
            self._idx_ev = None
        if self._idx_ev is not None:
            self._idx_ev.synchronize()
        self._idx_h.numpy()[:n] = rows
        out = self._idx_d[:n]
        out.copy_(self._idx_h[:n], non_blocking=True)
        self._idx_ev = torch.cuda.Event()
        self._idx_ev.record()
        return out

    def _row_buffers(self) -> list[torch.Tensor]:
        """Every per-agent tensor a clone copies (agent.clone() deep-copies the
        networks, the optimizer state and the hyperparameters): params, both
        Adam moments, the learning rate and the Adam step count (int64 rows
        viewed as two f32 words: moved bit for bit, never computed on)."""
        pop, P = self.pop, self.pop.P
        bufs = [pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq]
        lr = getattr(pop.opt, "lr", None)
        if isinstance(lr, torch.Tensor) and lr.shape == (P,):
            bufs.append(lr.view(P, 1))
        steps = getattr(pop.opt, "steps", None)
        if isinstance(steps, torch.Tensor) and steps.shape == (P,) and steps.dtype == torch.int64:
            bufs.append(steps.view(torch.float32).view(P, 2))
        for name in ("hp_batch_d", "hp_epochs_d", "hp_ent_d"):  # per-agent RL hyperparameters
            t = getattr(pop, name, None)
            if isinstance(t, torch.Tensor) and t.shape == (P,):
                bufs.append(t.view(torch.float32).view(P, 1))
        return bufs

    def _rows_gather(self, bufs: list[torch.Tensor], idx: torch.Tensor) -> None:
        """agx_rows_gather: row j of every buffer := its old row idx[j]."""
        import ctypes

        from .. import _lib

        n, P = len(bufs), self.pop.P
        widths = (ctypes.c_int64 * n)(*[int(b.shape[1]) for b in bufs])
        ptrs = (ctypes.c_void_p * n)(*[b.data_ptr() for b in bufs])
        nbytes = int(_lib.load().agx_rows_gather_workspace_bytes(widths, n, P))
        if getattr(self, "_rows_ws", None) is None or self._rows_ws.numel() < nbytes:
            self._rows_ws = torch.empty(nbytes, dtype=torch.uint8, device=self.pop.device)
        _lib.call("agx_rows_gather", ptrs, widths, n, P, idx.data_ptr(), self._rows_ws.data_ptr(), _lib.stream())

    @torch.no_grad()
    def _clone_rows(self, parents: list[int]) -> None:
        """Row j of this rank becomes global row parents[rank*P + j] (params,
        both Adam moments, lr, Adam step).  Everything is enqueued on the
        current stream, in order after the learner; the host does not wait."""
        pop, P, me = self.pop, self.pop.P, self.rank
        bufs = self._row_buffers()
        widths = [b.shape[1] for b in bufs]
        offs = np.concatenate([[0], np.cumsum(widths)]).tolist()
        mine = parents[me * P:(me + 1) * P]
        if self.world == 1 and not self.loopback:  # a permutation-with-repeats of the rows: one gather per buffer
            if mine == list(range(P)):
                return
            if (pop.device.type == "cuda" and len(bufs) <= 8 and all(b.is_contiguous() for b in bufs)
                    and os.environ.get("AGX_ROWS_GATHER", "1") != "0"):
                self._rows_gather(bufs, self._dev_index(mine))  # every buffer in two launches
                return
            idx = self._dev_index(mine) if pop.device.type == "cuda" else torch.as_tensor(mine)
            for b in bufs:
                b.copy_(b.index_select(0, idx))
            return
        # rows each rank needs from each other rank (sorted, unique): the same
        # plan on every rank, derived from the shared parent list
        lb = self.loopback
        need = [[sorted({q % P for q in parents[r * P:(r + 1) * P] if q // P == src}) if (src != r or lb) else []
                 for src in range(self.world)] for r in range(self.world)]
        ops, recv = [], {}
        sends = []
        for dst in range(self.world):
            rows = need[dst][me]
            if rows:
                idx = torch.as_tensor(rows, device=pop.device)
                msg = torch.cat([b.index_select(0, idx) for b in bufs], dim=1).contiguous().to(self.comm_device)
                sends.append(msg)
                ops.append(dist.P2POp(dist.isend, msg, dst))
        for src in range(self.world):
            rows = need[me][src]
            if rows:
                recv[src] = torch.empty(len(rows), offs[-1], dtype=bufs[0].dtype, device=self.comm_device)
                ops.append(dist.P2POp(dist.irecv, recv[src], src))
        local = [] if lb else [j for j in range(P) if mine[j] // P == me]
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
            rows = msg.to(pop.device).index_select(0, sel)
            for k, b in enumerate(bufs):
                b.index_copy_(0, dst_idx, rows[:, offs[k]:offs[k + 1]])

    @torch.no_grad()
    def select(self) -> list[int]:
        """Fitness all-gather and the tournament over the global population
        (no row is moved): -> the parent of every global slot."""
        if self.rng_state is None and hasattr(self.pop, "discard_prefetch"):
            # the tournament draws from the global numpy stream: put back any
            # minibatch shuffles drawn ahead, so the draws keep the reference's order
            self.pop.discard_prefetch()
        fit = self._fitness_host()
        self.history.append(fit)
        fits = [np.stack([h[i] for h in self.history[-self.eval_loop:]]) for i in range(len(fit))]
        _, parents = select_parents(fits, self.tournament_size, self.elitism, self.eval_loop, rng=self.rng_state)
        # clones inherit their parent's fitness history (copy_attributes, core/base.py:444-503),
        # which the next generation's eval_loop window reads
        self.history = [np.asarray(h)[np.asarray(parents)] for h in self.history]
        self.last_parents = parents
        return parents

    @torch.no_grad()
    def generation(self) -> list[int]:
        parents = self.select()
        self._clone_rows(parents)
        if hasattr(self.pop, "after_clone"):
            P = self.pop.P
            mine = parents[self.rank * P:(self.rank + 1) * P]
            self.pop.after_clone([q % P for q in mine] if self.world == 1 else None)
        self.last_parents = parents
        return parents
