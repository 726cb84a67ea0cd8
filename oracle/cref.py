"""ctypes binding of oracle/c/oracle.c (TEST INFRASTRUCTURE ONLY, see oracle/__init__)."""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int64
_D = ctypes.c_double


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_gae.argtypes = [_P, _P, _P, _P, _P, _I, _I, _I, _D, _D, ctypes.c_int, _P, _P, ctypes.c_int]
        L.oracle_per_update.argtypes = [_P, _P, _I, _P, _P, _I, _D, _D]
        L.oracle_per_update.restype = _D
        L.oracle_per_add.argtypes = [_P, _P, _I, _I, _P, _I, _D, _D]
        L.oracle_per_sample.argtypes = [_P, _I, _P, _I, _P]
        L.oracle_per_sample.restype = _I
        L.oracle_per_weights.argtypes = [_P, _P, _I, _P, _I, _I, _D, _P]
        L.oracle_ppo_loss.argtypes = [_P] * 7 + [_I, _I, _D, _D, _D, _P, _P, _P, _P, ctypes.c_int]
        L.oracle_c51.argtypes = [_P] * 7 + [_I, _I, _I, _D, _D, _D, _P, _P]
        L.oracle_pow.argtypes = [_P, _P, _P, _I]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def gae(r, v, done, last_v, last_done, gamma, lam, use_gae=True, nthreads=1):
    """(P,T,N) or (T,N) arrays -> (adv, ret) of the same shape."""
    r = np.ascontiguousarray(r, np.float32)
    squeeze = r.ndim == 2
    if squeeze:
        r = r[None]
    P, T, N = r.shape
    v = np.ascontiguousarray(np.asarray(v, np.float32).reshape(P, T, N))
    d = np.ascontiguousarray(np.asarray(done).astype(np.uint8).reshape(P, T, N))
    lv = np.ascontiguousarray(np.asarray(last_v, np.float32).reshape(P, N))
    ld = np.ascontiguousarray(np.asarray(last_done).astype(np.uint8).reshape(P, N))
    adv = np.empty_like(r)
    ret = np.empty_like(r)
    lib().oracle_gae(_p(r), _p(d), _p(v), _p(lv), _p(ld), P, T, N, gamma, lam, int(use_gae),
                     _p(adv), _p(ret), int(nthreads))
    return (adv[0], ret[0]) if squeeze else (adv, ret)


class PERTree:
    """Segment-tree state + operations of the C restatement."""

    def __init__(self, max_size: int, alpha: float = 0.6):
        cap = 1
        while cap < max_size:
            cap *= 2
        self.cap, self.max_size, self.alpha = cap, max_size, alpha
        self.sum = np.zeros(2 * cap)
        self.min = np.full(2 * cap, np.inf)
        self.max_priority = 1.0
        self.tree_ptr = np.zeros(1, np.int64)
        self.size = 0

    def add(self, n: int):
        lib().oracle_per_add(_p(self.sum), _p(self.min), self.cap, self.max_size, _p(self.tree_ptr),
                             n, self.alpha, self.max_priority)
        self.size = min(self.size + n, self.max_size)

    def update(self, idx, pri):
        idx = np.ascontiguousarray(np.asarray(idx).reshape(-1), np.int64)
        pri = np.ascontiguousarray(np.asarray(pri).reshape(-1), np.float32)
        self.max_priority = lib().oracle_per_update(_p(self.sum), _p(self.min), self.cap, _p(idx),
                                                    _p(pri), idx.size, self.alpha, self.max_priority)

    def sample(self, u):
        u = np.ascontiguousarray(u, np.float32)
        out = np.empty(u.size, np.int64)
        bad = lib().oracle_per_sample(_p(self.sum), self.cap, _p(u), u.size, _p(out))
        return out, int(bad)

    def weights(self, idx, beta):
        idx = np.ascontiguousarray(idx, np.int64)
        w = np.empty(idx.size, np.float32)
        lib().oracle_per_weights(_p(self.sum), _p(self.min), self.cap, _p(idx), idx.size, self.size,
                                 beta, _p(w))
        return w


def ppo_loss(logp, old_logp, adv, ret, old_v, v, H, b, clip, vf, ent, nthreads=1):
    arrs = [np.ascontiguousarray(x, np.float32) for x in (logp, old_logp, adv, ret, old_v, v, H)]
    S = arrs[0].size
    nmb = S // b
    g = [np.empty(S, np.float32) for _ in range(3)]
    loss = np.empty(nmb)
    lib().oracle_ppo_loss(*[_p(a) for a in arrs], b, nmb, clip, vf, ent, _p(g[0]), _p(g[1]), _p(g[2]),
                          _p(loss), int(nthreads))
    return loss, g[0], g[1], g[2]


def c51(q_next, tdist, logp_cur, act, r, d, support, vmin, vmax, gamma):
    q_next = np.ascontiguousarray(q_next, np.float32)
    B, A = q_next.shape
    Z = np.asarray(support).size
    arrs = [q_next, np.ascontiguousarray(tdist, np.float32), np.ascontiguousarray(logp_cur, np.float32),
            np.ascontiguousarray(np.asarray(act).reshape(-1), np.int64),
            np.ascontiguousarray(np.asarray(r).reshape(-1), np.float32),
            np.ascontiguousarray(np.asarray(d).reshape(-1), np.float32),
            np.ascontiguousarray(support, np.float32)]
    proj = np.empty((B, Z), np.float32)
    loss = np.empty(B, np.float32)
    lib().oracle_c51(*[_p(a) for a in arrs], B, A, Z, vmin, vmax, gamma, _p(proj), _p(loss))
    return loss, proj


def libm_pow(x, y):
    """Element-wise libm pow (the reference's Python float ** float)."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(np.broadcast_to(np.asarray(y, np.float64), x.shape))
    out = np.empty_like(x)
    lib().oracle_pow(_p(x), _p(y), _p(out), x.size)
    return out
