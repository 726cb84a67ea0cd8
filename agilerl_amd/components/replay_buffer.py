"""Drop-in ReplayBuffer / PrioritizedReplayBuffer with storage and trees in HBM.

Constructor arguments, ``add`` / ``sample`` / ``update_priorities`` /
``clear`` / ``size`` semantics follow agilerl/components/replay_buffer.py
(ReplayBuffer :12-138, PrioritizedReplayBuffer :261-428).  Differences of
form, not of results:

* transitions are ``dict[str, Tensor | ndarray]`` with a leading batch
  dimension (``tensordict`` is not a dependency); ``sample`` returns a dict;
* storage tensors live on ``device`` (default: the GPU) — HBM, sized once
  from the first ``add`` (uint8 frames stay uint8);
* the priority trees are one agx_per_* launch per ``add`` / ``sample`` /
  ``update_priorities`` call instead of a Python loop per transition.

Sample indices are bit-identical to the reference under the same global torch
seed: the B uniforms are ``torch.rand(B)`` from the global CPU generator — the
same stream as the reference's B calls of ``torch.rand(1)``
(replay_buffer.py:375).
"""

from __future__ import annotations

from collections import deque

import numpy as np
import torch

from .. import kernels as K
from .segment_tree import MinSegmentTree, SumSegmentTree

DataType = dict


def _to_tensor(v, device) -> torch.Tensor:
    t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
    return t.to(device)


class ReplayBuffer:
    """Circular uniform replay buffer (replay_buffer.py:12-138)."""

    def __init__(self, max_size: int, device="cuda", dtype: torch.dtype = torch.float32) -> None:
        self.max_size = int(max_size)
        self.device = torch.device(device)
        self.dtype = dtype
        self.counter = 0
        self.initialized = False
        self._cursor = 0
        self._size = 0
        self._storage: dict[str, torch.Tensor] | None = None

    @property
    def storage(self) -> dict[str, torch.Tensor] | None:
        return self._storage

    @property
    def size(self) -> int:
        return self._size

    @size.setter
    def size(self, value: int) -> None:
        self._size = value

    @property
    def is_full(self) -> bool:
        return len(self) == self.max_size

    def __len__(self) -> int:
        return self._size

    def _prepare(self, data: DataType) -> tuple[dict[str, torch.Tensor], int]:
        items = {k: _to_tensor(v, self.device) for k, v in data.items()}
        n = next(iter(items.values())).shape[0]
        for k, v in items.items():
            if v.shape[0] != n:
                raise ValueError(f"field {k!r} has batch {v.shape[0]}, expected {n}")
            if v.ndim == 1:  # (batch,) -> (batch, 1), replay_buffer.py:88-95
                items[k] = v.reshape(n, 1)
        return items, n

    def _init(self, items: dict[str, torch.Tensor]) -> None:
        self._storage = {k: torch.zeros((self.max_size, *v.shape[1:]), dtype=v.dtype, device=self.device)
                         for k, v in items.items()}
        self.initialized = True

    def add(self, data: DataType) -> None:
        items, n = self._prepare(data)
        if self._storage is None:
            self._init(items)
        start, end = self._cursor, self._cursor + n
        for k, v in items.items():
            dst = self._storage[k]
            if end > self.max_size:
                m = self.max_size - start
                dst[start:] = v[:m]
                dst[: n - m] = v[m:]
            else:
                dst[start:end] = v
        self._cursor = end % self.max_size
        self._size = min(self._size + n, self.max_size)
        self.counter += n

    def _gather(self, indices: torch.Tensor) -> dict[str, torch.Tensor]:
        idx = indices.to(self.device)
        return {k: v.index_select(0, idx) for k, v in self._storage.items()}

    def _gather_sampled(self, indices: torch.Tensor) -> dict[str, torch.Tensor]:
        """The sampler's own (in-range) indices: every field's rows in one
        agx_replay_gather launch on the GPU (one index op per field on the CPU)."""
        st = self._storage
        if (self.device.type != "cuda" or not st or len(st) > 8
                or any(not v.is_contiguous() or v.shape[0] != self.max_size for v in st.values())):
            return self._gather(indices)
        import ctypes

        from .. import _lib

        idx = indices.to(device=self.device, dtype=torch.int64).contiguous()
        B = idx.numel()
        outs = {k: torch.empty((B, *v.shape[1:]), dtype=v.dtype, device=self.device) for k, v in st.items()}
        vals = list(st.values())
        n = len(vals)
        srcs = (ctypes.c_void_p * n)(*[v.data_ptr() for v in vals])
        dsts = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs.values()])
        rbytes = (ctypes.c_int64 * n)(*[v[0].numel() * v.element_size() for v in vals])
        _lib.call("agx_replay_gather", ctypes.cast(srcs, ctypes.c_void_p), ctypes.cast(dsts, ctypes.c_void_p),
                  ctypes.cast(rbytes, ctypes.c_void_p), n, idx.data_ptr(), B, self.max_size, None, _lib.stream())
        return outs

    def sample(self, batch_size: int, return_idx: bool = False) -> dict[str, torch.Tensor]:
        indices = torch.randperm(self.size)[:batch_size]  # global CPU generator, as the reference
        samples = self._gather_sampled(indices)
        if return_idx:
            samples["idxs"] = indices.to(self.device)
        return samples

    def clear(self) -> None:
        self._size = 0
        self._cursor = 0
        self._storage = None
        self.initialized = False


class MultiStepReplayBuffer(ReplayBuffer):
    """n-step returns (replay_buffer.py:141-258): transitions pass through a
    deque of n batched steps held in HBM; once full, the folded transition
    r0 + sum_i r_{i+1} gamma**(i+1) (f32, the reference's weak-scalar
    multiply), with next_obs / done of the last folded step, is stored.  The
    fold stops after the first later step in which ANY env is done — the
    reference's ``done.bool().any()`` — and does not look at the first
    step's own done; both quirks are kept."""

    def __init__(self, max_size: int, n_step: int = 3, gamma: float = 0.99, device="cuda",
                 dtype: torch.dtype = torch.float32) -> None:
        super().__init__(max_size, device, dtype)
        self.n_step = int(n_step)
        self.gamma = float(gamma)
        self.n_step_buffer: deque = deque(maxlen=self.n_step)
        self.reward_key = "reward"
        self.done_key = None
        self.ns_key = "next_obs"

    def add(self, data: DataType):
        items = {k: _to_tensor(v, self.device) for k, v in data.items()}
        self.n_step_buffer.append(items)
        if len(self.n_step_buffer) < self.n_step:
            return None
        super().add(self._get_n_step_info())
        return self.n_step_buffer[0]

    def _get_n_step_info(self) -> dict[str, torch.Tensor]:
        first = {k: v.clone() for k, v in self.n_step_buffer[0].items()}
        if self.done_key is None:
            assert self.reward_key in first, f"Reward key not found in transition. Expected key: {self.reward_key}"
            assert self.ns_key in first, f"Next observation key not found in transition. Expected key: {self.ns_key}"
            for key in ("done", "termination", "terminated"):
                if key in first:
                    self.done_key = key
                    break
            assert self.done_key is not None, "No done/termination key found in transition."
        reward = first[self.reward_key].clone()
        for i, tr in enumerate(list(self.n_step_buffer)[1:]):
            reward += tr[self.reward_key] * (self.gamma ** (i + 1))
            first[self.ns_key] = tr[self.ns_key].clone()
            first[self.done_key] = tr[self.done_key].clone()
            if tr[self.done_key].bool().any():
                break
        first[self.reward_key] = reward
        return first

    def sample_from_indices(self, idxs) -> dict[str, torch.Tensor]:
        return self._gather(torch.as_tensor(idxs).reshape(-1).to(torch.int64))


class PrioritizedReplayBuffer(ReplayBuffer):
    """Proportional PER (replay_buffer.py:261-428) on agx_per_* kernels."""

    def __init__(self, max_size: int, alpha: float = 0.6, device="cuda", dtype: torch.dtype = torch.float32) -> None:
        super().__init__(max_size, device, dtype)
        self.alpha = float(alpha)
        self.tree_ptr = 0
        tree_capacity = 1
        while tree_capacity < self.max_size:
            tree_capacity *= 2
        self.tree_capacity = tree_capacity
        self.sum_tree = SumSegmentTree(tree_capacity, device=self.device)
        self.min_tree = MinSegmentTree(tree_capacity, device=self.device)
        self._max_priority = torch.ones(1, dtype=torch.float64, device=self.device)
        self._ws = K.per_workspace(tree_capacity, self.device)

    @property
    def max_priority(self) -> float:
        return float(self._max_priority.item())

    @max_priority.setter
    def max_priority(self, value: float) -> None:
        self._max_priority.fill_(float(value))

    def add(self, data: DataType) -> None:
        n = next(iter(data.values())).shape[0]
        super().add(data)
        # max_priority ** alpha at the n ring positions after tree_ptr (:296-309)
        K.per_add(self.sum_tree.tree, self.min_tree.tree, self.tree_capacity, self.max_size, self.tree_ptr, n,
                  self.alpha, self._max_priority, workspace=self._ws)
        self.tree_ptr = (self.tree_ptr + n) % self.max_size

    def _update_priority(self, idx: int, priority: float) -> None:
        assert 0 <= idx < self.max_size
        K.per_update(self.sum_tree.tree, self.min_tree.tree, self.tree_capacity, self.max_size,
                     torch.tensor([idx], dtype=torch.int64, device=self.device),
                     torch.tensor([priority], dtype=torch.float32, device=self.device), self.alpha,
                     self._max_priority, floor=float("-inf"), workspace=self._ws)

    def _sample_proportional(self, batch_size: int) -> torch.Tensor:
        u = torch.rand(batch_size).to(self.device)
        idx, _ = K.per_sample(self.sum_tree.tree, self.min_tree.tree, self.tree_capacity, u, weights=False)
        return idx

    def sample(self, batch_size: int, beta: float = 0.4) -> dict[str, torch.Tensor]:
        u = torch.rand(batch_size).to(self.device)
        err = torch.zeros(1, dtype=torch.int32, device=self.device)
        idx, w = K.per_sample(self.sum_tree.tree, self.min_tree.tree, self.tree_capacity, u, size=self.size,
                              beta=beta, weights=True, err=err)
        if int(err.item()) != 0:  # segment_tree.py:145
            raise AssertionError("upperbound outside [0, sum + 1e-5]")
        samples = self._gather_sampled(idx)
        samples["weights"] = w.unsqueeze(1)
        samples["idxs"] = idx.unsqueeze(1)
        self._sampled = (idx.data_ptr(), idx.numel(), idx._version)  # in range by construction (err checked)
        return samples

    def update_priorities(self, indices, priorities) -> None:
        """p = max(priority, 1e-5) ** alpha per index, in order (:411-428)."""
        idx = _to_tensor(indices, self.device).reshape(-1).to(torch.int64)
        pri = _to_tensor(priorities, self.device).reshape(-1).to(torch.float32)
        # the indices sample() itself handed out (same storage, unmodified) are
        # in range by construction: no device -> host read of their min / max
        trusted = (isinstance(indices, torch.Tensor) and getattr(self, "_sampled", None) is not None
                   and (idx.data_ptr(), idx.numel(), indices._version) == self._sampled)
        if idx.numel() and not trusted:
            lo, hi = torch.stack(torch.aminmax(idx)).tolist()  # one device->host read
            if lo < 0 or hi >= self.max_size:
                raise AssertionError("priority index out of range")
        K.per_update(self.sum_tree.tree, self.min_tree.tree, self.tree_capacity, self.max_size, idx.contiguous(),
                     pri.contiguous(), self.alpha, self._max_priority, floor=1e-5, workspace=self._ws)
