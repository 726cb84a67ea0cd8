"""MADDPG hot-path restatements (TEST INFRASTRUCTURE ONLY — never imported by
the product path).

Replay — ``agilerl/components/multi_agent_replay_buffer.py:16-300``: a
``deque(maxlen=memory_size)`` of per-transition tuples of per-agent dicts;
vectorised saves append one entry per env (``_reorganize_dicts``);
``sample`` = ``random.sample(memory, k)`` (Python's global ``random``) then,
per (field, agent), ``np.array`` of the B items (1-D results expanded to
(B, 1)); binary fields (done / termination / truncation ...) ``astype(uint8)``
unless they hold a NaN; everything returned as float32 (``obs_to_tensor``).

Critic target — ``agilerl/algorithms/maddpg.py:764-790``: rewards NaN -> 0,
dones NaN -> 1 then ``.to(uint8)``; ``y = r + ((1 - d) * gamma) * q'`` in f32
(``1 - d`` in uint8 arithmetic); ``loss = mean((q - y)^2)``;
``dloss/dq = 2 (q - y) / B``.
"""

from __future__ import annotations

import random
from collections import deque

import numpy as np

BINARY = ("done", "termination", "terminated", "truncation", "truncated")


class DequeReplay:
    def __init__(self, memory_size, field_names, agent_ids):
        self.memory = deque(maxlen=memory_size)
        self.field_names, self.agent_ids = list(field_names), list(agent_ids)

    def save(self, *args, is_vectorised=False):
        if not is_vectorised:
            self.memory.append(tuple(args))
            return
        n = len(np.asarray(next(iter(args[0].values()))))
        for i in range(n):
            self.memory.append(tuple({a: np.asarray(f[a])[i] for a in self.agent_ids} for f in args))

    def sample(self, batch_size):
        exps = random.sample(self.memory, k=batch_size)
        out = []
        for j, field in enumerate(self.field_names):
            per = {}
            for a in self.agent_ids:
                ts = np.array([e[j][a] for e in exps])
                if ts.ndim == 1:
                    ts = ts[:, None]
                if field in BINARY and not np.isnan(ts.astype(np.float64)).any():
                    ts = ts.astype(np.uint8)
                per[a] = ts.astype(np.float32)
            out.append(per)
        return tuple(out)


def critic_target(q, q_next, r, d, gamma):
    q = np.asarray(q, np.float32).reshape(-1)
    qn = np.asarray(q_next, np.float32).reshape(-1)
    r = np.asarray(r, np.float32).reshape(-1)
    d = np.asarray(d, np.float32).reshape(-1)
    r = np.where(np.isnan(r), np.float32(0), r)
    du = np.where(np.isnan(d), np.float32(1), d).astype(np.uint8)
    nd = (np.uint8(1) - du).astype(np.float32)
    y = r + (nd * np.float32(gamma)) * qn
    diff = (q - y).astype(np.float64)
    loss = np.float32(np.mean(diff * diff))
    g = ((q - y) * np.float32(2.0 / q.shape[0])).astype(np.float32)
    return y.astype(np.float32), g, loss
