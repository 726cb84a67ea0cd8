"""Drop-in ``MultiAgentReplayBuffer`` (agilerl/components/multi_agent_replay_buffer.py:16-300)
with the whole memory in HBM.

The reference keeps a deque of namedtuples of per-agent dicts and, on
``sample``, stacks B Python objects per (field, agent) on the host.  Here every
transition is ONE packed f32 row ``[field_0/agent_0 | field_0/agent_1 | ... ]``
of a ring ``storage[memory_size, W]`` in HBM: ``save_to_memory`` is one H2D
copy of the step's rows, ``sample`` one row gather (index_select) and
zero-copy column views per (field, agent).

Sample indices are the reference's: ``random.sample(memory, k)`` draws from
Python's global ``random`` using only ``len(memory)``, so
``random.sample(range(len), k)`` yields the same positions; deque position j
is ring slot ``(counter + j) % memory_size`` once the ring has wrapped.
Values follow ``_process_transition`` + ``obs_to_tensor``: everything comes
back f32 of shape (B, *item_shape) (scalars as (B, 1)); binary fields
(done / termination / truncation ...) are cast through uint8 unless the
sampled column holds a NaN.  Dict / tuple observations are outside the hot
path.
"""

from __future__ import annotations

import random
from typing import Any

import numpy as np
import torch

_BINARY = ("done", "termination", "terminated", "truncation", "truncated")


class MultiAgentReplayBuffer:
    def __init__(self, memory_size: int, field_names: list[str], agent_ids: list[str], device=None) -> None:
        assert memory_size > 0, "Memory size must be greater than zero."
        assert len(field_names) > 0, "Field names must contain at least one field name."
        assert len(agent_ids) > 0, "Agent ids must contain at least one agent id."
        self.memory_size = int(memory_size)
        self.field_names = list(field_names)
        self.agent_ids = list(agent_ids)
        self.device = torch.device(device if device is not None else "cuda")
        self.counter = 0
        self._size = 0
        self.storage: torch.Tensor | None = None
        self._layout: dict[tuple[str, str], tuple[int, int, tuple[int, ...]]] = {}

    def __len__(self) -> int:
        return self._size

    # ------------------------------------------------------------------ #
    def _init_layout(self, rows: list[dict[str, np.ndarray]]) -> None:
        col = 0
        for f, field in zip(self.field_names, rows):
            for a in self.agent_ids:
                shape = tuple(field[a].shape[1:])
                n = int(np.prod(shape)) if shape else 1
                self._layout[(f, a)] = (col, col + n, shape)
                col += n
        self.width = col
        self.storage = torch.zeros(self.memory_size, col, dtype=torch.float32, device=self.device)

    def _pack(self, args, vectorised: bool) -> np.ndarray:
        fields = []
        n = None
        for arg in args:
            per = {}
            for a in self.agent_ids:
                v = arg[a]
                if isinstance(v, (dict, tuple)):
                    raise NotImplementedError("dict / tuple observations are outside the agx hot path")
                v = np.asarray(v.cpu().numpy() if isinstance(v, torch.Tensor) else v)
                v = v if vectorised else v[None]
                per[a] = v
                n = v.shape[0] if n is None else n
                if v.shape[0] != n:
                    raise ValueError(f"agent {a!r}: {v.shape[0]} entries, expected {n}")
            fields.append(per)
        if self.storage is None:
            self._init_layout(fields)
        rows = np.empty((n, self.width), dtype=np.float32)
        for f, per in zip(self.field_names, fields):
            for a in self.agent_ids:
                c0, c1, _ = self._layout[(f, a)]
                rows[:, c0:c1] = per[a].reshape(n, c1 - c0)
        return rows

    def _write(self, rows: np.ndarray) -> None:
        n = rows.shape[0]
        src = torch.from_numpy(rows).to(self.device, non_blocking=False)
        start = self.counter % self.memory_size
        first = min(n, self.memory_size - start)
        self.storage[start:start + first] = src[:first]
        rest = n - first
        while rest > 0:  # more rows than the ring holds wrap again, like a deque(maxlen)
            k = min(rest, self.memory_size)
            self.storage[:k] = src[n - rest:n - rest + k]
            rest -= k
        self.counter += n
        self._size = min(self._size + n, self.memory_size)

    def save_to_memory_single_env(self, *args: dict[str, Any]) -> None:
        self._write(self._pack(args, vectorised=False))

    def save_to_memory_vect_envs(self, *args: dict[str, Any]) -> None:
        self._write(self._pack(args, vectorised=True))

    def save_to_memory(self, *args: dict[str, Any], is_vectorised: bool = False) -> None:
        if is_vectorised:
            self.save_to_memory_vect_envs(*args)
        else:
            self.save_to_memory_single_env(*args)

    # ------------------------------------------------------------------ #
    def sample_indices(self, batch_size: int) -> list[int]:
        """Deque positions of ``random.sample(self.memory, k=batch_size)``."""
        return random.sample(range(self._size), k=batch_size)

    def slots(self, positions) -> torch.Tensor:
        pos = torch.as_tensor(positions, dtype=torch.int64)
        if self.counter > self.memory_size:  # wrapped: oldest entry at the write cursor
            pos = (pos + self.counter) % self.memory_size
        return pos

    def sample(self, batch_size: int, *args: Any) -> tuple:
        idx = self.slots(self.sample_indices(batch_size)).to(self.device)
        batch = self.storage.index_select(0, idx)
        out = []
        for f in self.field_names:
            per = {}
            for a in self.agent_ids:
                c0, c1, shape = self._layout[(f, a)]
                t = batch[:, c0:c1]
                if shape:
                    t = t.reshape(batch_size, *shape)
                if f in _BINARY:  # astype(np.uint8) unless the sampled column holds a NaN
                    t = torch.where(torch.isnan(t).any(), t, t.to(torch.uint8).float())
                per[a] = t
            out.append(per)
        return tuple(out)
