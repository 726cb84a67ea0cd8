"""Rainbow's dueling head streams on agx_noisy_streams_forward / _backward
(include/agx_noisy.h, csrc/noisy_mlp.hip).

DuelingDistributionalMLP.forward (agilerl/networks/custom_modules.py:127-162)
runs ``self.model(x)`` (the value stream) and ``self.advantage_net(x)``; each
is a create_mlp stack (agilerl/modules/mlp.py) NoisyLinear -> LayerNorm ->
ReLU ... -> NoisyLinear.  In torch that is, per stream and per layer, the
noisy weight and bias (mu + sigma * eps, custom_components.py:124-131), the
Linear, the LayerNorm and the ReLU, and autograd's backward of each — about
forty launches per forward + backward at B = 64 rows, every one of them
latency bound.  ``head_streams`` runs both streams as one launch per layer
depth forward and one per depth backward; the parameters stay the modules'
own tensors, gradients come back through autograd as usual (d mu = dW,
d sigma = dW * eps).

It applies to the stacks the reference builds for Rainbow's head (noisy or
plain Linear layers, every hidden layer followed by an affine LayerNorm and
ReLU, the output layer by Identity) on f32 CUDA tensors of at most 1024 rows;
any other stack (an activation mutation, a head without LayerNorm, module
hooks, more than four layers) keeps the torch modules.  AGX_NOISY_STREAMS=0
turns it off (the eager torch head, for A/B checks)."""

from __future__ import annotations

import ctypes
import os

import torch
from torch import nn

from .. import _lib
from .custom_components import NoisyLinear

_MAX_LAYERS = 4
_MAX_ROWS = 1024
_PTRS = ("w_mu", "w_sigma", "w_eps", "b_mu", "b_sigma", "b_eps", "ln_gamma", "ln_beta", "out", "ln_part",
         "grad_w_mu", "grad_w_sigma", "grad_b_mu", "grad_b_sigma", "grad_ln_gamma", "grad_ln_beta")


class AgxNoisyStreamLayer(ctypes.Structure):
    """Mirror of ``agx_noisy_stream_layer`` (include/agx_noisy.h)."""

    _fields_ = [(n, ctypes.c_void_p) for n in _PTRS] + [("fin", ctypes.c_int32), ("fout", ctypes.c_int32)]


def enabled() -> bool:
    return os.environ.get("AGX_NOISY_STREAMS", "1") != "0"


def _stream_plan(seq: nn.Module) -> list | None:
    """[(linear, layernorm | None)] of a create_mlp stack, or None."""
    mods = list(seq.children())
    plan, i = [], 0
    while i < len(mods):
        lin = mods[i]
        if type(lin) is nn.Linear:
            if lin.bias is None:
                return None
        elif type(lin) is not NoisyLinear:
            return None
        i += 1
        if i < len(mods) and type(mods[i]) is nn.LayerNorm:
            ln = mods[i]
            if (not ln.elementwise_affine or ln.weight is None or ln.bias is None or
                    tuple(ln.normalized_shape) != (lin.out_features,)):
                return None
            if i + 1 >= len(mods) or type(mods[i + 1]) is not nn.ReLU:
                return None
            plan.append((lin, ln))
            i += 2
        else:
            while i < len(mods) and type(mods[i]) is nn.Identity:
                i += 1
            if i != len(mods):
                return None
            plan.append((lin, None))
    if not plan or plan[-1][1] is not None or len(plan) > _MAX_LAYERS:
        return None
    return plan


class _Meta:
    """Per (stream, layer): indices of its tensors in the Function's inputs,
    its eps buffers (noisy train mode) and sizes."""

    __slots__ = ("S", "NL", "eps", "layers", "n_tensors")

    def __init__(self, S: int, NL: int, eps: float):
        self.S, self.NL, self.eps, self.layers, self.n_tensors = S, NL, eps, [], 0


def _params(plans: list) -> tuple[_Meta, list] | None:
    S, NL = len(plans), len(plans[0])
    eps = None
    ts: list[torch.Tensor] = []
    meta = _Meta(S, NL, 1e-5)

    def add(t):
        ts.append(t)
        return len(ts) - 1

    for plan in plans:
        for lin, ln in plan:
            d = {"fin": lin.in_features, "fout": lin.out_features}
            if type(lin) is NoisyLinear:
                d["w_mu"], d["b_mu"] = add(lin.weight_mu), add(lin.bias_mu)
                if lin.training:
                    d["w_sigma"], d["b_sigma"] = add(lin.weight_sigma), add(lin.bias_sigma)
                    d["w_eps"], d["b_eps"] = lin.weight_epsilon, lin.bias_epsilon
            else:
                d["w_mu"], d["b_mu"] = add(lin.weight), add(lin.bias)
            if ln is not None:
                if eps is not None and ln.eps != eps:
                    return None
                eps = ln.eps
                d["ln_gamma"], d["ln_beta"] = add(ln.weight), add(ln.bias)
            meta.layers.append(d)
    if eps is not None:
        meta.eps = float(eps)
    meta.n_tensors = len(ts)
    for t in ts + [d[k] for d in meta.layers for k in ("w_eps", "b_eps") if k in d]:
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            return None
    return meta, ts


def _layer_array(meta: _Meta, ts, outs, parts, grads=None) -> ctypes.Array:
    arr = (AgxNoisyStreamLayer * len(meta.layers))()
    for j, d in enumerate(meta.layers):
        e = arr[j]
        e.fin, e.fout = d["fin"], d["fout"]
        for k in ("w_mu", "w_sigma", "b_mu", "b_sigma", "ln_gamma", "ln_beta"):
            if k in d:
                setattr(e, k, ts[d[k]].data_ptr())
                if grads is not None:
                    setattr(e, "grad_" + k, grads[d[k]].data_ptr())
        for k in ("w_eps", "b_eps"):
            if k in d:
                setattr(e, k, d[k].data_ptr())
        e.out = outs[j].data_ptr()
        if parts[j] is not None:
            e.ln_part = parts[j].data_ptr()
    return arr


class NoisyStreamsFn(torch.autograd.Function):
    """(x [B, fin], stream parameters...) -> every stream's output [B, fout]."""

    @staticmethod
    def forward(ctx, meta: _Meta, x, *ts):
        x = x.contiguous()
        B = x.shape[0]
        outs = [torch.empty(B, d["fout"], dtype=torch.float32, device=x.device) for d in meta.layers]
        # hidden layers: per-tile LayerNorm statistics of out (read by the next depth and the backward)
        parts = [torch.empty(B, (d["fout"] + 15) // 16, 2, dtype=torch.float32, device=x.device)
                 if "ln_gamma" in d else None for d in meta.layers]
        arr = _layer_array(meta, ts, outs, parts)
        _lib.call("agx_noisy_streams_forward", ctypes.cast(arr, ctypes.c_void_p), meta.S, meta.NL, x.data_ptr(), B,
                  meta.eps, _lib.stream())
        ctx.meta = meta
        ctx.parts = [p is not None for p in parts]
        ctx.save_for_backward(x, *ts, *outs, *[p for p in parts if p is not None])
        return tuple(outs[s * meta.NL + meta.NL - 1] for s in range(meta.S))

    @staticmethod
    def backward(ctx, *gouts):
        return (None, *_streams_backward(ctx, ctx.meta, gouts, 1))


def _streams_backward(ctx, meta, gouts, first: int) -> list:
    """Gradients of x and of every stream tensor from the saved (x, ts, outs,
    parts); ``first``: index of x among the Function's inputs."""
    saved = ctx.saved_tensors
    nl = len(meta.layers)
    x, ts = saved[0], saved[1:1 + meta.n_tensors]
    outs = saved[1 + meta.n_tensors:1 + meta.n_tensors + nl]
    rest = iter(saved[1 + meta.n_tensors + nl:])
    parts = [next(rest) if has else None for has in ctx.parts]
    B = x.shape[0]
    grads = [torch.empty_like(t) for t in ts]
    gx = torch.empty_like(x) if ctx.needs_input_grad[first] else None
    gs = []
    for s, g in enumerate(gouts):
        fout = meta.layers[s * meta.NL + meta.NL - 1]["fout"]
        gs.append(torch.zeros(B, fout, dtype=torch.float32, device=x.device) if g is None else
                  g.to(torch.float32).contiguous())
    arr = _layer_array(meta, ts, outs, parts, grads)
    lib = _lib.load()
    nws = lib.agx_noisy_streams_workspace_bytes(ctypes.cast(arr, ctypes.c_void_p), meta.S, meta.NL, B)
    ws = torch.empty(max(16, nws), dtype=torch.uint8, device=x.device)
    gptr = (ctypes.c_void_p * meta.S)(*[g.data_ptr() for g in gs])
    _lib.call("agx_noisy_streams_backward", ctypes.cast(arr, ctypes.c_void_p), meta.S, meta.NL, x.data_ptr(), B,
              meta.eps, ctypes.cast(gptr, ctypes.c_void_p), _lib.ptr(gx), ws.data_ptr(), _lib.stream())
    return [gx, *[g if ctx.needs_input_grad[first + 1 + i] else None for i, g in enumerate(grads)]]


def head_streams(streams: list, x: torch.Tensor):
    """Outputs of ``streams`` (create_mlp stacks reading the same x) on the
    fused kernels, or None where they do not apply."""
    if (not enabled() or not isinstance(x, torch.Tensor) or not x.is_cuda or x.dtype != torch.float32 or
            x.dim() != 2 or x.shape[0] > _MAX_ROWS):
        return None
    from ..algorithms.learn_graph import _hooked

    plans = [_stream_plan(s) for s in streams]
    if any(p is None for p in plans) or len({len(p) for p in plans}) != 1 or _hooked(*streams):
        return None
    if any(p[0][0].in_features != x.shape[1] for p in plans):
        return None
    got = _params(plans)
    if got is None:
        return None
    meta, ts = got
    return NoisyStreamsFn.apply(meta, x, *ts)


@torch.no_grad()
def head_streams_each(streams: list, xs: list):
    """No-grad outputs of ``streams`` where stream s reads xs[s] (several
    networks' heads in one launch per depth, agx_noisy_streams_forward_each),
    or None where the fused kernels do not apply."""
    if not enabled() or len(streams) > 4 or len(xs) != len(streams):
        return None
    x0 = xs[0]
    if any(not isinstance(x, torch.Tensor) or not x.is_cuda or x.dtype != torch.float32 or x.dim() != 2 or
           x.shape != x0.shape or not x.is_contiguous() for x in xs) or x0.shape[0] > _MAX_ROWS:
        return None
    from ..algorithms.learn_graph import _hooked

    plans = [_stream_plan(s) for s in streams]
    if any(p is None for p in plans) or len({len(p) for p in plans}) != 1 or _hooked(*streams):
        return None
    if any(p[0][0].in_features != x0.shape[1] for p in plans):
        return None
    got = _params(plans)
    if got is None:
        return None
    meta, ts = got
    B = x0.shape[0]
    outs = [torch.empty(B, d["fout"], dtype=torch.float32, device=x0.device) for d in meta.layers]
    parts = [torch.empty(B, (d["fout"] + 15) // 16, 2, dtype=torch.float32, device=x0.device)
             if "ln_gamma" in d else None for d in meta.layers]
    arr = _layer_array(meta, ts, outs, parts)
    xp = (ctypes.c_void_p * len(xs))(*[x.data_ptr() for x in xs])
    _lib.call("agx_noisy_streams_forward_each", ctypes.cast(arr, ctypes.c_void_p), meta.S, meta.NL,
              ctypes.cast(xp, ctypes.c_void_p), B, meta.eps, _lib.stream())
    return tuple(outs[s * meta.NL + meta.NL - 1] for s in range(meta.S))


class MixedStreamsFn(torch.autograd.Function):
    """No-grad streams (each on its own input) and grad streams (on x) in one
    launch per depth (agx_noisy_streams_forward_each): -> the no-grad
    streams' outputs (without gradient), then the grad streams' outputs; the
    backward is the grad streams' alone (NoisyStreamsFn's)."""

    @staticmethod
    def forward(ctx, meta_g, meta_ng, ts_ng, xs_ng, x, *ts):
        x = x.contiguous()
        B = x.shape[0]
        S_ng, S_g = meta_ng.S, meta_g.S
        out_ng = [torch.empty(B, d["fout"], dtype=torch.float32, device=x.device) for d in meta_ng.layers]
        out_g = [torch.empty(B, d["fout"], dtype=torch.float32, device=x.device) for d in meta_g.layers]
        part = lambda d: (torch.empty(B, (d["fout"] + 15) // 16, 2, dtype=torch.float32, device=x.device)
                          if "ln_gamma" in d else None)
        part_ng = [part(d) for d in meta_ng.layers]
        part_g = [part(d) for d in meta_g.layers]
        a_ng = _layer_array(meta_ng, ts_ng, out_ng, part_ng)
        a_g = _layer_array(meta_g, ts, out_g, part_g)
        arr = (AgxNoisyStreamLayer * (len(a_ng) + len(a_g)))(*a_ng, *a_g)
        xp = (ctypes.c_void_p * (S_ng + S_g))(*[t.data_ptr() for t in xs_ng], *([x.data_ptr()] * S_g))
        _lib.call("agx_noisy_streams_forward_each", ctypes.cast(arr, ctypes.c_void_p), S_ng + S_g, meta_g.NL,
                  ctypes.cast(xp, ctypes.c_void_p), B, meta_g.eps, _lib.stream())
        ctx.meta = meta_g
        ctx.parts = [p is not None for p in part_g]
        ctx.save_for_backward(x, *ts, *out_g, *[p for p in part_g if p is not None])
        outs_ng = tuple(out_ng[s * meta_ng.NL + meta_ng.NL - 1] for s in range(S_ng))
        ctx.mark_non_differentiable(*outs_ng)
        return outs_ng + tuple(out_g[s * meta_g.NL + meta_g.NL - 1] for s in range(S_g))

    @staticmethod
    def backward(ctx, *gouts):
        meta = ctx.meta
        return (None, None, None, None, *_streams_backward(ctx, meta, gouts[len(gouts) - meta.S:], 4))


def mixed_streams(nograd_streams: list, nograd_xs: list, grad_streams: list, x: torch.Tensor):
    """(no-grad outputs..., grad outputs...) of RainbowDQN's update heads in
    one launch per depth (MixedStreamsFn), or None where the kernels do not
    apply (every stream a create_mlp stack of one depth, one LayerNorm eps,
    at most six streams)."""
    if not enabled() or len(nograd_streams) + len(grad_streams) > 6 or not grad_streams:
        return None
    if (not isinstance(x, torch.Tensor) or not x.is_cuda or x.dtype != torch.float32 or x.dim() != 2
            or x.shape[0] > _MAX_ROWS):
        return None
    if any(t.shape != x.shape or t.dtype != x.dtype or not t.is_cuda or not t.is_contiguous() for t in nograd_xs):
        return None
    from ..algorithms.learn_graph import _hooked

    plans_ng = [_stream_plan(s) for s in nograd_streams]
    plans_g = [_stream_plan(s) for s in grad_streams]
    plans = plans_ng + plans_g
    if any(p is None for p in plans) or len({len(p) for p in plans}) != 1 or _hooked(*nograd_streams, *grad_streams):
        return None
    if any(p[0][0].in_features != x.shape[1] for p in plans):
        return None
    got_ng, got_g = _params(plans_ng), _params(plans_g)
    if got_ng is None or got_g is None or got_ng[0].eps != got_g[0].eps:
        return None
    (meta_ng, ts_ng), (meta_g, ts_g) = got_ng, got_g
    return MixedStreamsFn.apply(meta_g, meta_ng, [t.detach() for t in ts_ng], list(nograd_xs), x, *ts_g)
