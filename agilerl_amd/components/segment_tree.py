"""Drop-in SegmentTree / SumSegmentTree / MinSegmentTree with the tree in HBM.

Same constructor, ``__setitem__`` / ``__getitem__`` / ``operate`` / ``sum`` /
``min`` / ``retrieve`` contract and assertions as
agilerl/components/segment_tree.py (:5-196).  The heap (2 * capacity f64,
node k has children 2k, 2k+1, leaf i at capacity + i) lives on the GPU and
every operation is a libagx kernel (agx_segtree_*); results are bit-identical
to the reference's Python-float arithmetic.  Besides the scalar calls of the
reference, ``set_batch`` and ``retrieve_batch`` take whole index / upper-bound
tensors (one launch each) — what the replay buffer uses.
"""

from __future__ import annotations

import operator
from collections.abc import Callable

import torch

from .. import _lib


def _as_i64(x, device) -> torch.Tensor:
    return torch.as_tensor(x, dtype=torch.int64).reshape(-1).to(device).contiguous()


def _as_f64(x, device) -> torch.Tensor:
    return torch.as_tensor(x, dtype=torch.float64).reshape(-1).to(device).contiguous()


class SegmentTree:
    """Segment tree whose ``operation`` is ``operator.add`` or ``min``."""

    def __init__(self, capacity: int, operation: Callable, init_value: float, device="cuda") -> None:
        assert capacity > 0, "capacity must be positive and a power of 2."
        assert capacity & (capacity - 1) == 0, "capacity must be positive and a power of 2."
        if operation is operator.add and init_value == 0.0:
            self._op = 0
        elif operation is min and init_value == float("inf"):
            self._op = 1
        else:
            raise ValueError("agx segment trees implement (operator.add, 0.0) and (min, inf) only")
        self.capacity = capacity
        self.operation = operation
        self.device = torch.device(device)
        self._lib = _lib.load()
        self.tree = torch.empty(2 * capacity, dtype=torch.float64, device=self.device)
        self._out = torch.empty(1, dtype=torch.float64, device=self.device)
        self._ws = None
        _lib.check(self._lib.agx_segtree_init(self.tree.data_ptr(), capacity, self._op, _lib.stream()),
                   "agx_segtree_init")

    # ------------------------------------------------------------------ #
    def operate(self, start: int = 0, end: int = 0) -> float:
        """Reduce [start, end) (end <= 0 counts from capacity), segment_tree.py:61-79."""
        _lib.check(self._lib.agx_segtree_operate(self.tree.data_ptr(), self.capacity, self._op, int(start), int(end),
                                                 self._out.data_ptr(), _lib.stream()), "agx_segtree_operate")
        return float(self._out.item())

    def set_batch(self, indices, values) -> None:
        """``tree[i] = v`` for every pair, in order (last duplicate wins)."""
        idx = _as_i64(indices, self.device)
        val = _as_f64(values, self.device)
        assert idx.numel() == val.numel()
        n = idx.numel()
        ws = None
        if n > 1024:
            if self._ws is None:
                self._ws = torch.empty(self._lib.agx_segtree_workspace_bytes(self.capacity), dtype=torch.uint8,
                                       device=self.device)
            ws = self._ws.data_ptr()
        _lib.check(self._lib.agx_segtree_set(self.tree.data_ptr(), self.capacity, self._op, idx.data_ptr(),
                                             val.data_ptr(), n, ws, _lib.stream()), "agx_segtree_set")

    def __setitem__(self, idx: int, val: float) -> None:
        self.set_batch([int(idx)], [float(val)])

    def __getitem__(self, idx: int) -> float:
        assert 0 <= idx < self.capacity
        return float(self.tree[self.capacity + idx].item())


class SumSegmentTree(SegmentTree):
    def __init__(self, capacity: int, device="cuda") -> None:
        super().__init__(capacity=capacity, operation=operator.add, init_value=0.0, device=device)

    def sum(self, start: int = 0, end: int = 0) -> float:
        return super().operate(start, end)

    def retrieve_batch(self, upperbounds: torch.Tensor, check: bool = True) -> torch.Tensor:
        """Leaf index for each f64 upper bound (one launch); raises
        AssertionError like the reference if any bound is outside [0, sum + 1e-5]."""
        ub = _as_f64(upperbounds, self.device)
        out = torch.empty(ub.numel(), dtype=torch.int64, device=self.device)
        err = torch.zeros(1, dtype=torch.int32, device=self.device) if check else None
        _lib.check(self._lib.agx_segtree_retrieve(self.tree.data_ptr(), self.capacity, ub.data_ptr(), ub.numel(),
                                                  out.data_ptr(), _lib.ptr(err), _lib.stream()),
                   "agx_segtree_retrieve")
        if check and int(err.item()) != 0:
            raise AssertionError(f"upperbound outside [0, sum + 1e-5] for {int(err.item())} sample(s)")
        return out

    def retrieve(self, upperbound: float) -> int:
        return int(self.retrieve_batch([float(upperbound)])[0].item())


class MinSegmentTree(SegmentTree):
    def __init__(self, capacity: int, device="cuda") -> None:
        super().__init__(capacity=capacity, operation=min, init_value=float("inf"), device=device)

    def min(self, start: int = 0, end: int = 0) -> float:
        return super().operate(start, end)
