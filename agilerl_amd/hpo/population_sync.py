"""Generation step of a GPU-resident population, sharded over ranks.

Replaces tournament_selection_and_mutation's accelerate path
(agilerl/utils/utils.py:1185-1211: rank 0 selects, writes every agent's
checkpoint to a shared filesystem, the other ranks reload) with:
  1. fitness: mean return of the episodes finished since the last generation
     (per agent, on device);
  2. RCCL all-gather of the P fitness scalars of every rank over xGMI;
  3. identical seeded tournament selection on every rank (select_parents);
  4. one RCCL all-gather of the flat parameter + Adam-moment rows, from
     which each rank copies its new agents' parents (device-to-device).
Single rank: steps 2 and 4 are local gathers.
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
        P = pop.P
        mine = torch.as_tensor(parents[self.rank * P:(self.rank + 1) * P], device=pop.device)
        for buf in (pop.params.data, pop.opt.exp_avg, pop.opt.exp_avg_sq):
            allrows = self._all_gather(buf)
            buf.copy_(allrows.index_select(0, mine))
        self.last_parents = parents
        return parents
