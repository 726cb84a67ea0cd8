"""Tournament selection (drop-in for agilerl/hpo/tournament.py).

``select_parents`` is the index-level core shared by the per-object API and
the GPU population: elitism ranks ``mean(fitness[-eval_loop:])`` with
``argsort(argsort(.))`` (tournament.py:53-69), then ``P - elitism`` draws of
``tournament_size`` indices from the GLOBAL numpy RNG, each won by the highest
rank (first on ties, tournament.py:41-51) — the same stream and decisions as
the reference, so a fixed ``np.random.seed`` gives identical parents on every
rank without communicating them.
"""

from __future__ import annotations

import numpy as np


def select_parents(fitnesses, tournament_size: int, elitism: bool, eval_loop: int, rng=None):
    """-> (elite position, list of parent positions for the new population).
    rng: a numpy RandomState to draw from instead of the global one (the same
    legacy MT19937 randint stream)."""
    draw = np.random.randint if rng is None else rng.randint
    last = [np.mean(np.asarray(f)[-eval_loop:]) for f in fitnesses]
    rank = np.argsort(last).argsort()
    elite = int(np.argsort(rank)[-1])
    parents = [elite] if elitism else []
    for _ in range(len(fitnesses) - (1 if elitism else 0)):
        sel = draw(0, len(rank), size=tournament_size)
        parents.append(int(sel[np.argmax([rank[i] for i in sel])]))
    return elite, parents


class TournamentSelection:
    """Same constructor / ``select`` contract as the reference class."""

    def __init__(self, tournament_size: int, elitism: bool, population_size: int, eval_loop: int) -> None:
        assert tournament_size > 0, "Tournament size must be greater than zero."
        assert isinstance(elitism, bool), "Elitism must be boolean value True or False."
        assert population_size > 0, "Population size must be greater than zero."
        assert eval_loop > 0, "Evo step must be greater than zero."
        self.tournament_size = tournament_size
        self.elitism = elitism
        self.population_size = population_size
        self.eval_loop = eval_loop

    def _tournament(self, fitness_values):
        selection = np.random.randint(0, len(fitness_values), size=self.tournament_size)
        return selection[np.argmax([fitness_values[i] for i in selection])]

    def select(self, population):
        """-> (elite clone, new population of clones) like tournament.py:71-119."""
        fit = [agent.fitness for agent in population]
        elite_pos, parents = select_parents(fit, self.tournament_size, self.elitism, self.eval_loop)
        max_id = max(agent.index for agent in population)
        elite = population[elite_pos].clone()
        new_population = []
        start = 0
        if self.elitism:
            new_population.append(elite.clone(wrap=False))
            start = 1
        for pos in parents[start:]:
            max_id += 1
            new_population.append(population[pos].clone(max_id, wrap=False))
        return elite, new_population
