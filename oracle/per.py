"""Segment trees + prioritized replay restatement (TEST INFRASTRUCTURE ONLY).

Follows
* ``agilerl/components/segment_tree.py`` — 1-indexed heap of ``2*capacity``
  Python floats (f64); ``__setitem__`` (:81-95) writes the leaf and recomputes
  every ancestor as ``op(left, right)``; ``retrieve`` (:136-156) walks down with
  ``if tree[2k] > ub: k = 2k else: ub -= tree[2k]; k = 2k+1``; ``operate``
  (:42-79) is the recursive range query;
* ``agilerl/components/replay_buffer.py:261-428`` — ``PrioritizedReplayBuffer``:
  capacity = next pow2 >= max_size (:287-290), leaves ``priority ** alpha``
  (Python float ``pow`` = libm), ``max_priority = max(...)`` (:329), proportional
  sampling with one global-torch-CPU uniform per stratum (:357-381), IS weights
  (:383-409), ``update_priorities`` in order with a ``1e-5`` floor (:411-428).

The uniform stream is an INPUT here (the caller draws it with ``torch.rand``),
exactly as the HIP path takes it.
"""

from __future__ import annotations

import math
import operator

import numpy as np


class SegmentTree:
    def __init__(self, capacity: int, operation, init_value: float) -> None:
        assert capacity > 0 and capacity & (capacity - 1) == 0
        self.capacity = capacity
        self.tree = [init_value] * (2 * capacity)
        self.operation = operation

    def _helper(self, start, end, node, ns, ne):  # segment_tree.py:26-60
        if start == ns and end == ne:
            return self.tree[node]
        mid = (ns + ne) // 2
        if end <= mid:
            return self._helper(start, end, 2 * node, ns, mid)
        if mid + 1 <= start:
            return self._helper(start, end, 2 * node + 1, mid + 1, ne)
        return self.operation(
            self._helper(start, mid, 2 * node, ns, mid),
            self._helper(mid + 1, end, 2 * node + 1, mid + 1, ne),
        )

    def operate(self, start=0, end=0):  # segment_tree.py:62-79
        if end <= 0:
            end += self.capacity
        end -= 1
        return self._helper(start, end, 1, 0, self.capacity - 1)

    def __setitem__(self, idx, val):  # segment_tree.py:81-95
        idx += self.capacity
        self.tree[idx] = val
        idx //= 2
        while idx >= 1:
            self.tree[idx] = self.operation(self.tree[2 * idx], self.tree[2 * idx + 1])
            idx //= 2

    def __getitem__(self, idx):
        assert 0 <= idx < self.capacity
        return self.tree[self.capacity + idx]


class SumSegmentTree(SegmentTree):
    def __init__(self, capacity):
        super().__init__(capacity, operator.add, 0.0)

    def sum(self, start=0, end=0):
        return self.operate(start, end)

    def retrieve(self, upperbound: float) -> int:  # segment_tree.py:136-156
        assert 0 <= upperbound <= self.sum() + 1e-5
        idx = 1
        while idx < self.capacity:
            left = 2 * idx
            if self.tree[left] > upperbound:
                idx = left
            else:
                upperbound -= self.tree[left]
                idx = left + 1
        return idx - self.capacity


class MinSegmentTree(SegmentTree):
    def __init__(self, capacity):
        super().__init__(capacity, min, float("inf"))

    def min(self, start=0, end=0):
        return self.operate(start, end)


def tree_capacity(max_size: int) -> int:
    cap = 1
    while cap < max_size:
        cap *= 2
    return cap


class PER:
    """Priority bookkeeping of ``PrioritizedReplayBuffer`` (storage is separate)."""

    def __init__(self, max_size: int, alpha: float = 0.6) -> None:
        self.max_size = max_size
        self.alpha = alpha
        self.max_priority = 1.0
        self.tree_ptr = 0
        self.size = 0
        cap = tree_capacity(max_size)
        self.sum_tree = SumSegmentTree(cap)
        self.min_tree = MinSegmentTree(cap)

    def _update_priority(self, idx: int, priority: float) -> None:  # :311-329
        assert 0 <= idx < self.max_size
        pa = priority ** self.alpha
        self.sum_tree[idx] = pa
        self.min_tree[idx] = pa
        self.max_priority = max(self.max_priority, priority)

    def add(self, n: int) -> None:  # :296-309 (priority half)
        for _ in range(n):
            self._update_priority(self.tree_ptr, self.max_priority)
            self.tree_ptr = (self.tree_ptr + 1) % self.max_size
        self.size = min(self.size + n, self.max_size)

    def sample_indices(self, uniforms) -> np.ndarray:  # :357-381
        u = np.asarray(uniforms, dtype=np.float32)
        B = u.size
        total = self.sum_tree.sum()
        segment = total / B
        out = np.zeros(B, dtype=np.int64)
        for i in range(B):
            a = segment * i
            b = segment * (i + 1)
            ub = float(u[i]) * (b - a) + a
            out[i] = self.sum_tree.retrieve(ub)
        return out

    def weights(self, indices, beta: float) -> np.ndarray:  # :383-409
        p_min = self.min_tree.min() / self.sum_tree.sum()
        max_weight = (p_min * self.size) ** -beta
        w = np.zeros(len(indices), dtype=np.float32)
        for i, idx in enumerate(np.asarray(indices).reshape(-1)):
            p_sample = self.sum_tree[int(idx)] / self.sum_tree.sum()
            weight = (p_sample * self.size) ** -beta
            w[i] = weight / max_weight
        return w

    def update_priorities(self, indices, priorities) -> None:  # :411-428
        for idx, p in zip(np.asarray(indices).reshape(-1), np.asarray(priorities, dtype=np.float32)):
            self._update_priority(int(idx), max(float(p), 1e-5))


def build_tree_from_leaves(leaves: np.ndarray, cap: int, op: str) -> np.ndarray:
    """Bulk tree from leaf values (f64).  Every internal node of the reference
    tree equals ``op(left, right)`` of its current children (each update
    recomputes its whole root path), so the tree is a pure function of the
    leaves and this level-synchronous build is bit-identical."""
    tree = np.zeros(2 * cap, dtype=np.float64)
    tree[:cap] = 0.0 if op == "sum" else math.inf
    tree[cap:] = leaves
    lvl = cap
    while lvl > 1:
        lo = lvl // 2
        kids = tree[lvl: 2 * lvl]
        tree[lo:lvl] = kids[0::2] + kids[1::2] if op == "sum" else np.minimum(kids[0::2], kids[1::2])
        lvl = lo
    if op == "sum":
        tree[0] = 0.0
    else:
        tree[0] = math.inf
    return tree
