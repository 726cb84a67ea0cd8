"""Tournament selection restatement (TEST INFRASTRUCTURE ONLY).

Follows ``agilerl/hpo/tournament.py``: ``_elitism`` (:53-69) ranks
``mean(fitness[-eval_loop:])`` with ``argsort(argsort(.))``, the elite is the
top rank; ``_tournament`` (:41-51) draws ``tournament_size`` indices with the
GLOBAL ``np.random.randint`` and keeps the max rank (first on ties);
``_select_standard_agents`` (:91-119) fills ``P - elitism`` slots.
Returns (elite position, parent positions in the new population order).
"""

from __future__ import annotations

import numpy as np


def select(fitnesses, tournament_size: int, elitism: bool, eval_loop: int):
    last = [np.mean(f[-eval_loop:]) for f in fitnesses]
    rank = np.argsort(last).argsort()
    elite = int(np.argsort(rank)[-1])
    parents = [elite] if elitism else []
    n = len(fitnesses) - (1 if elitism else 0)
    for _ in range(n):
        sel = np.random.randint(0, len(rank), size=tournament_size)
        vals = [rank[i] for i in sel]
        parents.append(int(sel[np.argmax(vals)]))
    return elite, parents
