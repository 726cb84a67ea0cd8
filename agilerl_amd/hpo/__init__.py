from .tournament import TournamentSelection, select_parents

__all__ = ["TournamentSelection", "select_parents"]
