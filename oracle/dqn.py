"""DQN TD target and Rainbow C51 projection restatements (TEST INFRASTRUCTURE ONLY).

TD target — ``agilerl/algorithms/dqn.py:296-314`` (``DQN.update``):
``q_t = max_a Q_tgt(s')`` or, double DQN, ``Q_tgt(s')[argmax_a Q(s')]``;
``y = r + (gamma*q_t)*(1-d)`` in f32 (two rounded products, one rounded sum);
``loss = mean((Q(s)[a] - y)^2)``.

C51 — ``agilerl/algorithms/dqn_rainbow.py:313-367`` (``RainbowDQN._dqn_loss``),
all f32 like the CPU reference:
``a* = argmax Q_online(s')`` (first maximum); ``p = P_tgt(s')[a*]``;
``t_z = clamp(r + ((1-d)*gamma)*z, vmin, vmax)``; ``b = (t_z - vmin) / f32(dz)``;
``L = floor(b)``, ``u = ceil(b)``; ``L[(u>0)&(u==L)] -= 1`` then
``u[(Z-1>L)&(u==L)] += 1``; two ``index_add_`` passes (all lower masses in atom
order, then all upper masses) — reproduced here as an ordered per-bin
accumulation, which is what a serial ``index_add_`` does;
``loss_i = -sum_z proj * log_p[a_i]``.
"""

from __future__ import annotations

import numpy as np


def td_target(q_next_online, q_next_target, r, d, gamma, double=False):
    qn = np.asarray(q_next_target, dtype=np.float32)
    if double:
        a = np.argmax(np.asarray(q_next_online, dtype=np.float32), axis=1)
        qt = qn[np.arange(qn.shape[0]), a][:, None]
    else:
        qt = qn.max(axis=1)[:, None]
    g = np.float32(gamma)
    r = np.asarray(r, dtype=np.float32).reshape(-1, 1)
    d = np.asarray(d, dtype=np.float32).reshape(-1, 1)
    return (r + (g * qt) * (np.float32(1.0) - d)).astype(np.float32)


def td_loss(q_cur, actions, y):
    q = np.asarray(q_cur, dtype=np.float64)
    a = np.asarray(actions).reshape(-1)
    qe = q[np.arange(q.shape[0]), a]
    diff = qe - np.asarray(y, dtype=np.float64).reshape(-1)
    loss = (diff ** 2).mean()
    g = np.zeros_like(q)
    g[np.arange(q.shape[0]), a] = 2.0 * diff / diff.size
    return loss, g


def c51_project(q_next, target_dist, r, d, support, vmin, vmax, gamma):
    """-> (a_star (B,), proj (B, Z) f32) exactly as the CPU reference computes it."""
    q_next = np.asarray(q_next, dtype=np.float32)
    td = np.asarray(target_dist, dtype=np.float32)
    z = np.asarray(support, dtype=np.float32)
    B, A, Z = td.shape
    a_star = np.argmax(q_next, axis=1)
    p = td[np.arange(B), a_star]  # (B, Z)
    r = np.asarray(r, dtype=np.float32).reshape(B, 1)
    d = np.asarray(d, dtype=np.float32).reshape(B, 1)
    with np.errstate(over="ignore", invalid="ignore"):
        t_z = r + ((np.float32(1.0) - d) * np.float32(gamma)) * z[None, :]
    t_z = np.clip(t_z, np.float32(vmin), np.float32(vmax)).astype(np.float32)
    dz = np.float32((vmax - vmin) / (Z - 1))
    b = ((t_z - np.float32(vmin)) / dz).astype(np.float32)
    L = np.floor(b).astype(np.int64)
    u = np.ceil(b).astype(np.int64)
    L[(u > 0) & (u == L)] -= 1
    u[((Z - 1) > L) & (u == L)] += 1
    ml = (p * (u.astype(np.float32) - b)).astype(np.float32)
    mu = (p * (b - L.astype(np.float32))).astype(np.float32)
    proj = np.zeros((B, Z), dtype=np.float32)
    for i in range(B):  # serial index_add_: first pass (lower), then second (upper)
        row = proj[i]
        for j in range(Z):
            row[L[i, j]] = np.float32(row[L[i, j]] + ml[i, j])
        for j in range(Z):
            row[u[i, j]] = np.float32(row[u[i, j]] + mu[i, j])
    return a_star, proj


def c51_loss(q_next, target_dist, logp_cur, actions, r, d, support, vmin, vmax, gamma):
    """-> (elementwise loss (B,) f64, proj (B,Z) f32)."""
    _, proj = c51_project(q_next, target_dist, r, d, support, vmin, vmax, gamma)
    lp = np.asarray(logp_cur, dtype=np.float32)
    B = lp.shape[0]
    a = np.asarray(actions).reshape(-1)
    log_p = lp[np.arange(B), a].astype(np.float64)
    return -(proj.astype(np.float64) * log_p).sum(1), proj


def nstep_fold(transitions, gamma: float):
    """MultiStepReplayBuffer._get_n_step_info (replay_buffer.py:196-258) on a
    list of n batched transitions (dicts of numpy arrays): reward folded as
    r0 + sum_i r_{i+1} * gamma**(i+1) in f32, next_obs / done taken from each
    later transition in turn, stopping after the first transition in which
    ANY env is done (the reference's ``done.bool().any()``)."""
    import numpy as _np

    first = {k: _np.array(v, copy=True) for k, v in transitions[0].items()}
    r = first["reward"].astype(_np.float32).copy()
    for i, tr in enumerate(transitions[1:]):
        r = (r + tr["reward"].astype(_np.float32) * _np.float32(gamma ** (i + 1))).astype(_np.float32)
        first["next_obs"] = _np.array(tr["next_obs"], copy=True)
        first["done"] = _np.array(tr["done"], copy=True)
        if _np.asarray(tr["done"]).astype(bool).any():
            break
    first["reward"] = r
    return first
