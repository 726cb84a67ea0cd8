"""PPO clipped-surrogate loss forward/backward restatement (TEST INFRASTRUCTURE ONLY).

Follows ``agilerl/algorithms/ppo.py:826-921`` (``_learn_from_rollout_buffer_flat``)
and the autograd rules torch applies to it:

* ``ratio = exp(logp - old_logp)``; ``pg = mean(max(-A*ratio, -A*clamp(ratio, 1-e, 1+e)))``
* ``v_clip = old_v + clamp(v - old_v, -e, e)``;
  ``vl = 0.5 * mean(max((v-R)^2, (v_clip-R)^2))``
* ``loss = pg + vf*vl - ent*mean(H)``;  ``approx_kl = mean((ratio-1) - log_ratio)``
* backward: ``torch.maximum`` splits the gradient 1/2 : 1/2 on ties,
  ``clamp`` passes it on the closed interval ``[lo, hi]``.

Computed in f64 (checked against the reference's f32 goldens with a relative
tolerance).  ``learn_flat`` reproduces the whole epoch / minibatch schedule
with the global numpy permutation stream (``ppo.py:838-845``).
"""

from __future__ import annotations

import numpy as np


def _max_grads(a, b):
    """d max(a,b)/da, d max(a,b)/db with torch's tie rule."""
    ga = np.where(a > b, 1.0, np.where(a == b, 0.5, 0.0))
    gb = np.where(b > a, 1.0, np.where(a == b, 0.5, 0.0))
    return ga, gb


def minibatch_loss(logp, old_logp, adv, ret, old_v, v, H, clip, vf_coef, ent_coef):
    """One minibatch -> (loss, parts dict, g_logp, g_v, g_H)  (all f64)."""
    logp, old_logp, adv, ret, old_v, v, H = (
        np.asarray(x, dtype=np.float64) for x in (logp, old_logp, adv, ret, old_v, v, H)
    )
    b = logp.size
    lr = logp - old_logp
    ratio = np.exp(lr)
    lo, hi = 1.0 - clip, 1.0 + clip
    rc = np.clip(ratio, lo, hi)
    pl1 = -adv * ratio
    pl2 = -adv * rc
    pg = np.maximum(pl1, pl2).mean()
    dv = v - old_v
    v_clip = old_v + np.clip(dv, -clip, clip)
    l_un = (v - ret) ** 2
    l_cl = (v_clip - ret) ** 2
    vl = 0.5 * np.maximum(l_un, l_cl).mean()
    ent = -H.mean()
    loss = pg + vf_coef * vl + ent_coef * ent
    kl = ((ratio - 1.0) - lr).mean()
    # backward
    g1, g2 = _max_grads(pl1, pl2)
    in_r = ((ratio >= lo) & (ratio <= hi)).astype(np.float64)
    d_ratio = (g1 * (-adv) + g2 * (-adv) * in_r) / b
    g_logp = d_ratio * ratio
    gu, gc = _max_grads(l_un, l_cl)
    in_v = ((dv >= -clip) & (dv <= clip)).astype(np.float64)
    g_v = vf_coef * 0.5 / b * (gu * 2.0 * (v - ret) + gc * 2.0 * (v_clip - ret) * in_v)
    g_H = np.full(b, -ent_coef / b)
    clipfrac = (np.abs(ratio - 1.0) > clip).mean()
    parts = dict(pg=pg, vl=vl, ent=ent, kl=kl, clipfrac=clipfrac)
    return loss, parts, g_logp, g_v, g_H


def learn_flat(old_logp, adv_norm, ret, old_v, new_logp, new_v, H, perms, batch, clip, vf, ent):
    """Replay the reference's epoch/minibatch loop with FIXED per-sample network
    outputs (the golden fixture's fake ``evaluate_actions``).  Returns the
    per-minibatch full-length gradient snapshots and ``mean_loss``."""
    S = len(old_logp)
    glp, gv, gh, total = [], [], [], 0.0
    for perm in perms:
        for s in range(0, S, batch):
            mb = perm[s: s + batch]
            loss, _, g1, g2, g3 = minibatch_loss(
                new_logp[mb], old_logp[mb], adv_norm[mb], ret[mb], old_v[mb], new_v[mb], H[mb],
                clip, vf, ent,
            )
            for acc, g in ((glp, g1), (gv, g2), (gh, g3)):
                full = np.zeros(S)
                np.add.at(full, mb, g)
                acc.append(full)
            total += loss
    return np.stack(glp), np.stack(gv), np.stack(gh), total / (S * len(perms))
