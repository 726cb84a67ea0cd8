"""GAE / Monte-Carlo returns restatement (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Follows ``agilerl/components/rollout_buffer.py:413-481``
(``RolloutBuffer.compute_returns_and_advantages``) with the exact NumPy>=2
(NEP 50) dtype flow spelled out:

* ``t == T-1``: ``next_values = last_value.astype(float)`` (f64), so
  ``gamma * next_values`` is an f64 product;
* ``t <  T-1``: ``next_values = values[t+1]`` (f32 array) and ``gamma`` is a
  weak Python float, so ``gamma * next_values`` is an **f32** product that is
  then widened when multiplied by the f64 ``next_non_terminal``;
* ``delta = (r + gv*nnt) - v`` in f64 (left-to-right, no fused multiply-add);
* ``c = delta + ((gamma*lam) * nnt) * c`` in f64 — the carry stays f64 because
  the chained assignment binds ``last_gae_lambda`` to the f64 result;
* stores cast to f32; ``returns = adv_f32 + values_f32`` in f32.

Monte-Carlo branch (``:468-477``): ``carry = last_value*(1-last_done)`` f64;
``carry = r[t] + (gamma*carry)*(1-done[t])`` f64 (note ``done[t]``, not
``done[t+1]``); ``adv = ret_f32 - values_f32`` in f32.
"""

from __future__ import annotations

import numpy as np


def gae(rewards, values, dones, last_value, last_done, gamma=0.99, lam=0.95, use_gae=True):
    """Time-major ``(T, N)`` inputs -> ``(advantages, returns)`` f32 ``(T, N)``."""
    r = np.asarray(rewards, dtype=np.float32)
    v = np.asarray(values, dtype=np.float32)
    d = np.asarray(dones).astype(bool)
    lv = np.asarray(last_value, dtype=np.float32).reshape(-1)
    ld = np.asarray(last_done).astype(np.float64).reshape(-1)
    T, N = r.shape
    adv = np.zeros((T, N), dtype=np.float32)
    ret = np.zeros((T, N), dtype=np.float32)
    g64 = np.float64(gamma)
    if use_gae:
        g32 = np.float32(gamma)
        gl = np.float64(gamma) * np.float64(lam)
        c = np.zeros(N, dtype=np.float64)
        for t in range(T - 1, -1, -1):
            if t == T - 1:
                nnt = 1.0 - ld
                gv = g64 * lv.astype(np.float64)
            else:
                nnt = 1.0 - d[t + 1].astype(np.float64)
                gv = (g32 * v[t + 1]).astype(np.float64)  # f32 product, then widen
            delta = (r[t].astype(np.float64) + gv * nnt) - v[t].astype(np.float64)
            c = delta + (gl * nnt) * c
            adv[t] = c.astype(np.float32)
        ret = adv + v
    else:
        c = lv.astype(np.float64) * (1.0 - ld)
        for t in range(T - 1, -1, -1):
            c = r[t].astype(np.float64) + (g64 * c) * (1.0 - d[t].astype(np.float64))
            ret[t] = c.astype(np.float32)
        adv = ret - v
    return adv, ret


def adv_stats(adv):
    """Global mean / unbiased std of the f32 advantages (``ppo.py:829-834``),
    accumulated in f64.  Returns ``(mean, std)``."""
    a = np.asarray(adv, dtype=np.float64).reshape(-1)
    n = a.size
    mean = a.sum() / n
    var = ((a - mean) ** 2).sum() / max(n - 1, 1)
    return mean, np.sqrt(var)


def normalize_advantages(adv):
    """``(a - mean) / (std + 1e-8)`` as in ``ppo.py:829-834`` (f32 result)."""
    mean, std = adv_stats(adv)
    a = np.asarray(adv, dtype=np.float64)
    return ((a - mean) / (std + 1e-8)).astype(np.float32)
