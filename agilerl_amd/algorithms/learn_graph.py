"""One agent's off-policy update replayed from a captured hipGraph.

``train_off_policy`` (train_off_policy.py:249-345) calls each agent's own
``learn`` once per learn step.  At the config-3 shape (RainbowDQN, 84x84x4
frames, B = 64) that update is a few hundred small launches — the CNN
forward of s and s' through the online and target networks, the dueling
heads, the C51 rows loss, the backward pass, the flat clip + Adam, Polyak and
the noise resets of both networks — and the host's launch overhead, not the
GPU, sets its time.  Here the device work of the update is
captured once per (flat learner state, input shapes, hyperparameters) into a
graph (``torch.cuda.CUDAGraph``) and replayed on every later call:

* the first call with a key runs eagerly (it also makes every lazily created
  library handle and workspace); the second captures and replays;
* inputs are copied into the graph's static tensors (one launch); ``.grad`` of every
  parameter is re-pointed at the captured gradient tensors after a replay;
* the host bookkeeping of the flat tail (a mutated learning rate, a torch
  optimizer step taken outside ``learn``, the torch ``step`` tensors) runs
  around every replay (FlatLearnState.sync / advance), so everything the
  eager update reads from the host is current;
* the noise draws (torch.randn on the device generator) are captured with
  torch's graph-safe Philox offsets: a replay draws what the eager calls
  would have drawn from the generator's current seed and offset.

Anything the key does not cover falls back to the eager update: forward /
backward hooks on the networks (they only fire in Python), a flat state that
cannot take the update (a parameter without gradient), a capture that fails,
or ``AGX_LEARN_GRAPH=0``.  ``tests/test_flat_state_gpu.py`` and
``tests/test_cnn_gpu.py`` check the replayed update against the eager torch
update of a twin agent (noise buffers bit-equal)."""

from __future__ import annotations

import os
import warnings
import weakref

import torch

# FlatLearnState -> {key: _Entry}: dropped with the flat state (a mutation,
# clone or checkpoint load makes a new one); never deep-copied with the agent
_GRAPHS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
_CAPTURE_AFTER = 1  # eager calls of a key before it is captured


class _Entry:
    __slots__ = ("eager", "graph", "inputs", "outputs", "grads", "failed", "copy")

    def __init__(self):
        self.eager, self.graph, self.inputs, self.outputs, self.grads, self.failed = 0, None, None, None, None, False
        self.copy = None  # _copy_plan's result once the graph exists


def _copy_plan(statics: list):
    """The static inputs as one batched copy: when every one is contiguous
    with the same leading (batch) dimension B, agx_replay_gather over
    idx = arange(B) moves all of them in one launch (torch's _foreach_copy_
    is one blit per tensor here).  -> (idx, dst array, row-byte array) or
    False."""
    import ctypes

    if not statics or len(statics) > 8 or any(x.dim() == 0 for x in statics):
        return False
    B = statics[0].shape[0]
    if not 1 <= B < 65536 or any(x.shape[0] != B or not x.is_contiguous() or x[0].numel() == 0 for x in statics):
        return False
    n = len(statics)
    idx = torch.arange(B, dtype=torch.int64, device=statics[0].device)
    dsts = (ctypes.c_void_p * n)(*[x.data_ptr() for x in statics])
    rbytes = (ctypes.c_int64 * n)(*[x[0].numel() * x.element_size() for x in statics])
    return idx, dsts, rbytes


def _copy_inputs(ent, inputs: list) -> None:
    """The batch into the static inputs (same shapes and dtypes: the key)."""
    if ent.copy is None:
        ent.copy = _copy_plan(ent.inputs)
    if ent.copy is False or not all(x.is_contiguous() for x in inputs):
        torch._foreach_copy_(ent.inputs, inputs)
        return
    import ctypes

    from .. import _lib

    idx, dsts, rbytes = ent.copy
    n = len(inputs)
    srcs = (ctypes.c_void_p * n)(*[x.data_ptr() for x in inputs])
    B = idx.numel()
    _lib.call("agx_replay_gather", ctypes.cast(srcs, ctypes.c_void_p), ctypes.cast(dsts, ctypes.c_void_p),
              ctypes.cast(rbytes, ctypes.c_void_p), n, idx.data_ptr(), B, B, None, _lib.stream())


def enabled() -> bool:
    return os.environ.get("AGX_LEARN_GRAPH", "1") != "0"


def _hooked(*nets) -> bool:
    """Module hooks run Python during forward / backward: a replay would
    skip them."""
    from torch.nn.modules import module as M

    if (M._global_forward_hooks or M._global_forward_pre_hooks or M._global_backward_hooks or
            getattr(M, "_global_backward_pre_hooks", None)):
        return True
    for net in nets:
        for m in net.modules():
            if (m._forward_hooks or m._forward_pre_hooks or m._backward_hooks or
                    getattr(m, "_backward_pre_hooks", None)):
                return True
    return False


def _sig(t: torch.Tensor) -> tuple:
    return (tuple(t.shape), t.dtype, t.device)


def run(fs, key: tuple, inputs: list, body, nets: tuple, max_norm: float, tau: float):
    """One update: ``body(inputs) -> outputs`` computes the loss(es) and runs
    the backward pass; this function adds the flat tail (clip + Adam with
    ``max_norm``, Polyak with ``tau``; FlatLearnState.launch / polyak) and the
    noise resets of ``nets``.  Replayed from a graph when the key was seen
    before, else eager.  -> outputs (static tensors when replayed: read
    before the next update)."""
    if (fs is None or not enabled() or not all(isinstance(x, torch.Tensor) and x.is_cuda for x in inputs)
            or torch.cuda.is_current_stream_capturing() or _hooked(*nets)):
        return None
    key = key + tuple(_sig(x) for x in inputs) + tuple(n.training for n in nets)
    table = _GRAPHS.setdefault(fs, {})
    ent = table.get(key)
    if ent is None:
        ent = table[key] = _Entry()

    def device_work(xs):
        out = body(xs)
        fs.launch(max_norm)
        fs.polyak(tau)
        for n in nets:
            n.reset_noise()
        return out

    if ent.graph is None:
        if ent.failed or ent.eager < _CAPTURE_AFTER:
            return None  # the caller's eager update
        statics = [x.detach().clone() for x in inputs]
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        try:
            with torch.cuda.graph(g):
                outs = device_work(statics)
        except Exception as exc:  # noqa: BLE001 - any capture failure: stay eager for this key
            warnings.warn(f"agx learn graph: capture failed ({exc!r}); this update stays eager")
            ent.failed = True
            torch.cuda.synchronize()
            return None
        if any(p.grad is None for p in fs.params):
            ent.failed = True
            return None
        ent.graph, ent.inputs, ent.outputs = g, statics, outs
        ent.grads = [p.grad for p in fs.params]
    else:
        _copy_inputs(ent, inputs)
    fs.sync()
    ent.graph.replay()
    fs.advance()
    for p, gr in zip(fs.params, ent.grads):
        p.grad = gr
    return ent.outputs


def note_eager(fs, key: tuple, inputs: list, nets: tuple, flat_ok: bool) -> None:
    """Count an eager update of ``key`` (the next one captures); an update
    the flat tail could not take (``flat_ok`` False) is never captured."""
    if fs is None or not enabled():
        return
    key = key + tuple(_sig(x) for x in inputs if isinstance(x, torch.Tensor)) + tuple(n.training for n in nets)
    table = _GRAPHS.setdefault(fs, {})
    ent = table.get(key)
    if ent is None:
        ent = table[key] = _Entry()
    ent.eager += 1
    ent.failed = ent.failed or not flat_ok
