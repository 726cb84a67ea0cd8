"""Drop-in RolloutBuffer with the (capacity, num_envs) SoA resident in HBM.

Constructor, ``add`` / ``compute_returns_and_advantages`` /
``get_tensor_batch`` / ``get`` / ``reset`` / ``size`` follow
agilerl/components/rollout_buffer.py (:61-582) for flat (non-recurrent)
Box / Discrete spaces.  ``compute_returns_and_advantages`` is one agx_gae
launch, bit-identical to the reference's NumPy loop (f64 carry, NumPy-2
dtype flow) for f32 ``last_value``.  Fields are plain tensors in a dict
(``tensordict`` is not a dependency); ``get_tensor_batch`` returns a dict.

Recurrent / BPTT sequence storage (``recurrent=True``) is outside the hot
path and raises NotImplementedError.
"""

from __future__ import annotations

import warnings

import numpy as np
import torch

from .. import kernels as K


def _obs_shape(space) -> tuple[int, ...]:
    if hasattr(space, "n") and not getattr(space, "shape", None):
        return (1,)
    return tuple(space.shape)


def _num_actions(space) -> int:
    if hasattr(space, "n"):  # Discrete
        return 1
    return int(np.prod(space.shape))


class RolloutBuffer:
    def __init__(self, capacity: int, observation_space, action_space, num_envs: int = 1, device="cuda",
                 gae_lambda: float = 0.95, gamma: float = 0.99, recurrent: bool = False,
                 hidden_state_architecture=None, use_gae: bool = True, wrap_at_capacity: bool = False,
                 max_seq_len: int | None = None, bptt_sequence_type=None) -> None:
        if recurrent:
            raise NotImplementedError("recurrent (BPTT) rollout storage is not on the agx hot path")
        self.capacity = int(capacity)
        self.observation_space = observation_space
        self.action_space = action_space
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.gamma = float(gamma)
        self.gae_lambda = float(gae_lambda)
        self.recurrent = recurrent
        self.hidden_state_architecture = hidden_state_architecture
        self.use_gae = use_gae
        self.wrap_at_capacity = wrap_at_capacity
        self.max_seq_len = max_seq_len
        self.bptt_sequence_type = bptt_sequence_type
        self.pos = 0
        self.full = False
        self._initialize_buffers()

    def _initialize_buffers(self) -> None:
        C, N, dev = self.capacity, self.num_envs, self.device
        obs = _obs_shape(self.observation_space)
        f32 = dict(dtype=torch.float32, device=dev)
        self.buffer = {
            "observations": torch.zeros((C, N, *obs), **f32),
            "next_observations": torch.zeros((C, N, *obs), **f32),
            "actions": torch.zeros((C, N, _num_actions(self.action_space)), **f32),
            "rewards": torch.zeros((C, N), **f32),
            "dones": torch.zeros((C, N), dtype=torch.bool, device=dev),
            "values": torch.zeros((C, N), **f32),
            "log_probs": torch.zeros((C, N), **f32),
            "advantages": torch.zeros((C, N), **f32),
            "returns": torch.zeros((C, N), **f32),
            "episode_starts": torch.zeros((C, N), dtype=torch.bool, device=dev),
        }
        self._gae_ws = None

    # ------------------------------------------------------------------ #
    def size(self) -> int:
        return (self.capacity if self.full else self.pos) * self.num_envs

    def reset(self) -> None:
        self.pos = 0
        self.full = False

    def _put(self, key: str, value, shape, dtype=None) -> None:
        t = torch.as_tensor(value, dtype=dtype) if not isinstance(value, torch.Tensor) else value
        self.buffer[key][self.pos].copy_(t.reshape(shape), non_blocking=True)

    def add(self, obs, action, reward, done, value, log_prob, next_obs=None, hidden_state=None,
            next_hidden_state=None, episode_start=None, action_mask=None) -> None:
        if self.pos == self.capacity:
            if not self.wrap_at_capacity:
                raise ValueError(f"Buffer has reached capacity ({self.capacity} transitions) but received more "
                                 "transitions. Either increase capacity or set wrap_at_capacity=True.")
            self.pos = 0
        N = self.num_envs
        obs_shape = self.buffer["observations"].shape[2:]
        self._put("observations", obs, (N, *obs_shape), torch.float32)
        self._put("actions", action, (N, -1))
        self._put("rewards", reward, (N,), torch.float32)
        self._put("dones", done, (N,), torch.bool)
        self._put("values", value, (N,), torch.float32)
        self._put("log_probs", log_prob, (N,), torch.float32)
        if next_obs is not None:
            self._put("next_observations", next_obs, (N, *obs_shape), torch.float32)
        if episode_start is not None:
            self._put("episode_starts", episode_start, (N,), torch.bool)
        else:
            self.buffer["episode_starts"][self.pos].zero_()
        if action_mask is not None:
            m = torch.as_tensor(action_mask, dtype=torch.bool).reshape(N, -1)
            if "action_masks" not in self.buffer:
                self.buffer["action_masks"] = torch.ones((self.capacity, N, m.shape[-1]), dtype=torch.bool,
                                                         device=self.device)
            self.buffer["action_masks"][self.pos].copy_(m)
        self.pos += 1
        if self.pos == self.capacity:
            self.full = True

    # ------------------------------------------------------------------ #
    def compute_returns_and_advantages(self, last_value, last_done) -> None:
        """GAE (or Monte-Carlo returns) over the filled prefix, rollout_buffer.py:413-481."""
        T = self.capacity if self.full else self.pos
        if T == 0:
            return
        N, dev = self.num_envs, self.device
        lv = torch.as_tensor(last_value).to(dev, torch.float32).reshape(1, N).contiguous()
        ld = torch.as_tensor(last_done).to(dev).reshape(1, N).to(torch.uint8).contiguous()
        b = self.buffer
        rew = b["rewards"][:T].reshape(1, T, N)
        done = b["dones"][:T].view(torch.uint8).reshape(1, T, N)
        val = b["values"][:T].reshape(1, T, N)
        K.gae(rew, done, val, lv, ld, self.gamma, self.gae_lambda, self.use_gae,
              advantages=b["advantages"][:T].reshape(1, T, N), returns=b["returns"][:T].reshape(1, T, N))

    def get_tensor_batch(self, batch_size: int | None = None, device=None) -> dict[str, torch.Tensor]:
        target = torch.device(device) if device is not None else self.device
        T = self.capacity if self.full else self.pos
        total = T * self.num_envs
        if total == 0:
            return {}
        flat = {k: v[:T].reshape(total, *v.shape[2:]) for k, v in self.buffer.items()}
        if batch_size is not None:
            if batch_size > total:
                warnings.warn(f"Batch size {batch_size} is larger than buffer_size {total}. Returning all data.",
                              stacklevel=2)
            else:
                idx = torch.randperm(total, device="cpu")[:batch_size].to(self.device)
                flat = {k: v.index_select(0, idx) for k, v in flat.items()}
        return {k: v.to(target) for k, v in flat.items()}

    def get(self, batch_size: int | None = None) -> dict[str, np.ndarray]:
        T = self.capacity if self.full else self.pos
        total = T * self.num_envs
        if total == 0:
            return {}
        flat = {k: v[:T].reshape(total, *v.shape[2:]) for k, v in self.buffer.items()}
        if batch_size is not None and batch_size <= total:
            idx = torch.as_tensor(np.random.choice(total, size=batch_size, replace=False)).to(self.device)
            flat = {k: v.index_select(0, idx) for k, v in flat.items()}
        elif batch_size is not None:
            warnings.warn(f"Batch size {batch_size} is larger than buffer size {total}. Returning all data.",
                          stacklevel=2)
        return {k: v.cpu().numpy() for k, v in flat.items()}
