"""The reference's host RNG streams, reproduced draw for draw.

* PPO minibatch order: ``np.random.shuffle`` on numpy's GLOBAL legacy
  RandomState (agilerl/algorithms/ppo.py:836-842), cumulative over the epochs
  of one learn(), agents learning one after another
  (train_on_policy.py:210).  ``numpy_shuffle_perms`` draws all of a
  population's permutations natively (agx_host_shuffle_perms) from the global
  generator's state and advances that state exactly as the reference's
  shuffles would, so a seeded run reproduces the reference's minibatches
  as long as every agent runs all its epochs.  With ``target_kl`` an agent
  that stops early draws fewer shuffles in the reference, which shifts every
  later agent's minibatch order; the population draws all agents' shuffles
  before its (parallel) learn, so those later agents' orders differ from the
  reference's, while the global state itself is re-synchronised to the
  reference's count afterwards (PPOPopulation.sync_numpy_stream).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def numpy_shuffle_perms(P: int, epochs: int, S: int, out: np.ndarray | None = None,
                        epochs_per_agent=None) -> np.ndarray:
    """[epochs, P, S] int64: for agent p = 0..P-1 in turn, arange(S) shuffled
    ``epochs`` times in place by the global ``np.random`` generator, row e =
    the order after the (e+1)-th shuffle.  Equivalent to (and as fast as a
    memcpy of) the Python loop::

        for p in range(P):
            idx = np.arange(S)
            for e in range(epochs):
                np.random.shuffle(idx); out[e, p] = idx

    ``epochs_per_agent``: agent p draws only its own number of shuffles
    (mutated update_epochs); rows beyond are left untouched.
    """
    if out is None:
        out = np.empty((epochs, P, S), dtype=np.int64)
    if out.shape != (epochs, P, S) or out.dtype != np.int64 or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous int64 array of shape (epochs, P, S)")
    name, key, pos, has_gauss, gauss = np.random.get_state(legacy=True)
    if name != "MT19937":
        raise RuntimeError(f"global numpy generator is {name}, expected MT19937")
    key = np.array(key, dtype=np.uint32)  # own, writable copy
    pos_c = ctypes.c_int32(int(pos))
    lib = _lib.load(require_gpu=False)  # host code: no device work
    ep = None
    if epochs_per_agent is not None:
        ep = np.ascontiguousarray(epochs_per_agent, dtype=np.int64)
        if ep.shape != (P,):
            raise ValueError("epochs_per_agent must have one entry per agent")
    _lib.check(lib.agx_host_shuffle_perms(key.ctypes.data, ctypes.byref(pos_c), int(P), int(epochs), int(S),
                                          None if ep is None else ep.ctypes.data, out.ctypes.data),
               "agx_host_shuffle_perms")
    np.random.set_state(("MT19937", key, int(pos_c.value), has_gauss, gauss))
    return out


def numpy_shuffle_perms_shard(out: np.ndarray, offset: int, global_P: int, epochs_global: list[int],
                              scratch: dict | None = None) -> np.ndarray:
    """The local slice of a population sharded over ranks: agents
    ``offset .. offset + P`` of the ``global_P`` agents that would learn one
    after another in the reference.  The shuffles of the agents before and
    after the slice are drawn too (into scratch, discarded), so the global
    generator ends where the unsharded population's draw leaves it and every
    rank's stream stays identical.  ``out``: [E, P, S] int64 (E >= the local
    agents' epochs); ``epochs_global``: every global agent's epochs."""
    E, P, S = out.shape
    eg = [int(e) for e in epochs_global]
    if len(eg) != global_P or offset < 0 or offset + P > global_P:
        raise ValueError("shard outside the global population")
    scratch = {} if scratch is None else scratch

    def _skip(lo: int, hi: int) -> None:
        if hi <= lo:
            return
        e = max(eg[lo:hi])
        key = (e, hi - lo, S)
        buf = scratch.get(key)
        if buf is None:
            buf = scratch[key] = np.empty(key, dtype=np.int64)
        numpy_shuffle_perms(hi - lo, e, S, out=buf, epochs_per_agent=eg[lo:hi])

    _skip(0, offset)
    local = eg[offset:offset + P]
    numpy_shuffle_perms(P, E, S, out=out, epochs_per_agent=None if all(x == E for x in local) else local)
    _skip(offset + P, global_P)
    return out
