"""RL-hyperparameter mutation specs with the reference's semantics and RNG
draws (agilerl/algorithms/core/registry.py:110-242):

* ``RLParameter(min, max, shrink_factor=0.8, grow_factor=1.2, dtype=float)``;
  ``mutate()`` draws ``torch.rand(1)`` from the GLOBAL torch CPU generator:
  < 0.5 shrinks (value * shrink, floored at min), else grows (value * grow,
  capped at max), then clips and casts to ``dtype``; the new value is kept in
  the spec (``value``), which the reference shares between the agents that
  share the config object (create_population hands every agent the same
  one; clone() deep-copies it);
* ``HyperparameterConfig(**params).sample()`` picks
  ``torch.randperm(len(config))[0]``, again the global torch generator.

These are host-side decisions taken once per generation; drawing them from
the same generators as the reference keeps a seeded run's mutation sequence
identical to the reference's.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from numbers import Number

import numpy as np
import torch


@dataclass
class RLParameter:
    min: float
    max: float
    shrink_factor: float = 0.8
    grow_factor: float = 1.2
    dtype: type = float
    value: Number | np.ndarray | None = field(default=None, init=False)

    def mutate(self):
        """registry.py:136-187 (same draw, same arithmetic order)."""
        assert self.value is not None, "Hyperparameter value is not set"
        if torch.rand(1).item() < 0.5:
            if isinstance(self.value, np.ndarray):
                new = np.where(self.value * self.shrink_factor > self.min, self.value * self.shrink_factor,
                               self.min)
            elif self.value * self.shrink_factor > self.min:
                new = self.value * self.shrink_factor
            else:
                new = self.min
        elif isinstance(self.value, np.ndarray):
            new = np.where(self.value * self.grow_factor < self.max, self.value * self.grow_factor, self.max)
        elif self.value * self.grow_factor < self.max:
            new = self.value * self.grow_factor
        else:
            new = self.max
        if isinstance(new, np.ndarray):
            new = np.clip(new, self.min, self.max).astype(self.value.dtype)
        else:
            new = self.dtype(min(max(new, self.min), self.max))
        self.value = new
        return self.value


class HyperparameterConfig:
    def __init__(self, **kwargs: RLParameter) -> None:
        self.config = kwargs
        for k, v in kwargs.items():
            if not isinstance(v, RLParameter):
                raise TypeError("Expected RLParameter object for hyperparameter configuration.")
            setattr(self, k, v)

    def __bool__(self) -> bool:
        return bool(self.config)

    def __iter__(self):
        return iter(self.config)

    def __getitem__(self, key: str) -> RLParameter:
        return self.config[key]

    def __len__(self) -> int:
        return len(self.config)

    def items(self):
        return self.config.items()

    def names(self) -> list[str]:
        return list(self.config.keys())

    def sample(self) -> tuple[str, RLParameter]:
        """registry.py:235-242."""
        key = torch.randperm(len(self.config))[0]
        return list(self.config.keys())[key], list(self.config.values())[key]

    def __repr__(self) -> str:
        return "HyperparameterConfig(\n" + "\n".join(f"{k}: {v}" for k, v in self.config.items()) + "\n)"


class MutationRegistry:
    """The part of agilerl's MutationRegistry the HPO reads: ``hp_config``
    (None or an empty config: RL-hyperparameter mutations are no-ops)."""

    def __init__(self, hp_config: HyperparameterConfig | None = None) -> None:
        self.hp_config = hp_config
