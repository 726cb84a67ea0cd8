"""Typed torch-tensor front end of the libagx.so C ABI (include/agx.h).

Every function takes device tensors, validates shapes/dtypes/devices on the
host (so a kernel never sees a mismatched grid), launches on the current HIP
stream and returns without synchronising.  No CPU fallback exists.
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib

_f32, _f64, _u8, _i64, _i32 = torch.float32, torch.float64, torch.uint8, torch.int64, torch.int32


def _need(t: torch.Tensor, name: str, dtype=None, shape=None, contiguous=True) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: must live on the GPU (got {t.device})")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# --------------------------------------------------------------------------- #
# GAE                                                                         #
# --------------------------------------------------------------------------- #
def gae(rewards, dones, values, last_value, last_done, gamma=0.99, gae_lambda=0.95, use_gae=True,
        advantages=None, returns=None, with_stats=False, workspace=None, stats_out=None):
    """rewards/values f32 [P,T,N] (or [T,N]), dones u8/bool, last_* [P,N].
    Returns (advantages, returns[, stats f64 [P,2] = mean, unbiased std])."""
    squeeze = rewards.dim() == 2
    r = rewards.unsqueeze(0) if squeeze else rewards
    P, T, N = r.shape
    v = values.reshape(P, T, N)
    d = dones.reshape(P, T, N)
    if d.dtype == torch.bool:
        d = d.view(torch.uint8)
    lv = last_value.reshape(P, N)
    ld = last_done.reshape(P, N)
    if ld.dtype == torch.bool:
        ld = ld.view(torch.uint8)
    _need(r, "rewards", _f32)
    _need(v, "values", _f32)
    _need(d, "dones", _u8)
    _need(lv, "last_value", _f32)
    _need(ld, "last_done", _u8)
    adv = torch.empty_like(r) if advantages is None else advantages.reshape(P, T, N)
    ret = torch.empty_like(r) if returns is None else returns.reshape(P, T, N)
    _need(adv, "advantages", _f32)
    _need(ret, "returns", _f32)
    stats = None
    if with_stats:
        stats = torch.empty(P, 2, dtype=_f64, device=r.device) if stats_out is None else stats_out
        _need(stats, "stats_out", _f64, (P, 2))
        if workspace is None:
            workspace = _ws(_lib.load().agx_gae_workspace_bytes(P, T, N), r.device)
    _lib.call("agx_gae", r.data_ptr(), d.data_ptr(), v.data_ptr(), lv.data_ptr(), ld.data_ptr(),
              P, T, N, float(gamma), float(gae_lambda), int(bool(use_gae)), adv.data_ptr(),
              ret.data_ptr(), _lib.ptr(stats), _lib.ptr(workspace), _lib.stream())
    if squeeze:
        adv, ret = adv[0], ret[0]
    return (adv, ret, stats) if with_stats else (adv, ret)


def gae_launcher(rewards, dones, values, last_value, last_done, gamma, gae_lambda, use_gae, advantages,
                 returns, stats_out, workspace):
    """Validate once, then return ``launch(stream)``: agx_gae on these fixed
    tensors (the population's persistent rollout buffers) with no per-call
    checks — the per-iteration call costs one ctypes call, not ~10 tensor
    validations (host time that sat between the rollout and the learner)."""
    adv, ret, _ = gae(rewards, dones, values, last_value, last_done, gamma, gae_lambda, use_gae,
                      advantages=advantages, returns=returns, with_stats=True, workspace=workspace,
                      stats_out=stats_out)  # validates (and runs once)
    P, T, N = adv.shape
    d = dones.view(torch.uint8) if dones.dtype == torch.bool else dones
    ld = last_done.view(torch.uint8) if last_done.dtype == torch.bool else last_done
    fn = _lib.load().agx_gae
    args = (rewards.data_ptr(), d.data_ptr(), values.data_ptr(), last_value.data_ptr(), ld.data_ptr(), P, T, N,
            float(gamma), float(gae_lambda), int(bool(use_gae)), adv.data_ptr(), ret.data_ptr(),
            stats_out.data_ptr(), workspace.data_ptr())

    def launch(stream: int) -> None:
        rc = fn(*args, stream)
        if rc != 0:
            _lib.check(rc, "agx_gae")

    return launch


def adv_normalize_(adv: torch.Tensor, stats: torch.Tensor) -> torch.Tensor:
    P = stats.shape[0]
    _need(adv, "adv", _f32)
    _need(stats, "stats", _f64, (P, 2))
    _lib.call("agx_adv_normalize", adv.data_ptr(), stats.data_ptr(), P, adv.numel() // P, _lib.stream())
    return adv


# --------------------------------------------------------------------------- #
# PPO loss                                                                    #
# --------------------------------------------------------------------------- #
def ppo_loss_fwd_bwd(logp, old_logp, adv, ret, old_value, value, entropy, batch, clip_coef=0.2,
                     vf_coef=0.5, ent_coef=0.01, index=None, out=None, stats=None):
    """Returns (g_logp, g_value, g_entropy, stats[nmb, 8])."""
    S = logp.numel()
    if S % batch:
        raise ValueError(f"samples ({S}) must be a multiple of batch ({batch}); call per minibatch")
    nmb = S // batch
    for t, n in ((logp, "logp"), (value, "value"), (entropy, "entropy")):
        _need(t, n, _f32)
        if t.numel() != S:
            raise ValueError(f"{n}: expected {S} elements")
    src = old_logp.numel()
    for t, n in ((old_logp, "old_logp"), (adv, "adv"), (ret, "ret"), (old_value, "old_value")):
        _need(t, n, _f32)
        if t.numel() != src:
            raise ValueError(f"{n}: expected {src} elements")
    if index is not None:
        _need(index, "index", _i64)
        if index.numel() != S:
            raise ValueError("index: one entry per sample")
    elif src != S:
        raise ValueError("without an index the old_* arrays must match logp")
    if out is None:
        out = tuple(torch.empty_like(logp) for _ in range(3))
    if stats is None:
        stats = torch.empty(nmb, 8, dtype=_f32, device=logp.device)
    _lib.call("agx_ppo_loss_fwd_bwd", logp.data_ptr(), old_logp.data_ptr(), adv.data_ptr(),
              ret.data_ptr(), old_value.data_ptr(), value.data_ptr(), entropy.data_ptr(),
              _lib.ptr(index), int(batch), int(nmb), float(clip_coef), float(vf_coef),
              float(ent_coef), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
              stats.data_ptr(), _lib.stream())
    return out[0], out[1], out[2], stats


# --------------------------------------------------------------------------- #
# PER                                                                         #
# --------------------------------------------------------------------------- #
def per_workspace(capacity: int, device) -> torch.Tensor:
    return _ws(_lib.load().agx_per_workspace_bytes(capacity, 0), device)


def per_init(sum_tree, min_tree, capacity):
    _need(sum_tree, "sum_tree", _f64, (2 * capacity,))
    _need(min_tree, "min_tree", _f64, (2 * capacity,))
    _lib.call("agx_per_init", sum_tree.data_ptr(), min_tree.data_ptr(), capacity, _lib.stream())


def per_add(sum_tree, min_tree, capacity, max_size, start, n, alpha, max_priority, workspace=None):
    _need(max_priority, "max_priority", _f64, (1,))
    _lib.call("agx_per_add", sum_tree.data_ptr(), min_tree.data_ptr(), capacity, max_size, int(start),
              int(n), float(alpha), max_priority.data_ptr(), _lib.ptr(workspace), _lib.stream())


def per_update(sum_tree, min_tree, capacity, max_size, indices, priorities, alpha, max_priority,
               floor=1e-5, workspace=None):
    idx = indices.reshape(-1)
    pri = priorities.reshape(-1)
    _need(idx, "indices", _i64)
    _need(pri, "priorities", _f32)
    if idx.numel() != pri.numel():
        raise ValueError("indices / priorities length mismatch")
    _need(max_priority, "max_priority", _f64, (1,))
    if workspace is None and idx.numel() > 1024:
        workspace = per_workspace(capacity, idx.device)
    _lib.call("agx_per_update", sum_tree.data_ptr(), min_tree.data_ptr(), capacity, max_size,
              idx.data_ptr(), pri.data_ptr(), idx.numel(), float(alpha), float(floor),
              max_priority.data_ptr(), _lib.ptr(workspace), _lib.stream())


def per_sample(sum_tree, min_tree, capacity, uniforms, size=0, beta=0.4, weights=True, err=None):
    u = uniforms.reshape(-1)
    _need(u, "uniforms", _f32)
    B = u.numel()
    idx = torch.empty(B, dtype=_i64, device=u.device)
    w = torch.empty(B, dtype=_f32, device=u.device) if weights else None
    if err is not None:
        _need(err, "err", _i32, (1,))
    _lib.call("agx_per_sample", sum_tree.data_ptr(), _lib.ptr(min_tree), capacity, u.data_ptr(), B,
              int(size), float(beta), idx.data_ptr(), _lib.ptr(w), _lib.ptr(err), _lib.stream())
    return idx, w


def per_gather(tree, nodes):
    _need(nodes, "nodes", _i64)
    out = torch.empty(nodes.numel(), dtype=_f64, device=tree.device)
    _lib.call("agx_per_gather", tree.data_ptr(), nodes.data_ptr(), nodes.numel(), out.data_ptr(),
              _lib.stream())
    return out


def debug_pow(x, y):
    _need(x, "x", _f64)
    _need(y, "y", _f64, tuple(x.shape))
    out = torch.empty_like(x)
    _lib.call("agx_debug_pow", x.data_ptr(), y.data_ptr(), out.data_ptr(), x.numel(), _lib.stream())
    return out


# --------------------------------------------------------------------------- #
# DQN / Rainbow                                                               #
# --------------------------------------------------------------------------- #
def td_target(q_next_target, rewards, dones, gamma, q_next_online=None, double=False, q_cur=None,
              actions=None, with_loss=True):
    B, A = q_next_target.shape
    _need(q_next_target, "q_next_target", _f32)
    r = rewards.reshape(-1)
    d = dones.reshape(-1)
    _need(r, "rewards", _f32, (B,))
    _need(d, "dones", _f32, (B,))
    if double:
        _need(q_next_online, "q_next_online", _f32, (B, A))
    y = torch.empty(B, 1, dtype=_f32, device=r.device)
    g_q = loss = None
    if with_loss:
        _need(q_cur, "q_cur", _f32, (B, A))
        a = actions.reshape(-1)
        _need(a, "actions", _i64, (B,))
        g_q = torch.empty(B, A, dtype=_f32, device=r.device)
        loss = torch.empty(1, dtype=_f32, device=r.device)
    else:
        a = None
    ws = _ws(_lib.load().agx_td_workspace_bytes(B), r.device) if with_loss else None
    _lib.call("agx_td_target", _lib.ptr(q_next_online), q_next_target.data_ptr(), _lib.ptr(q_cur),
              _lib.ptr(a), r.data_ptr(), d.data_ptr(), B, A, float(gamma), int(bool(double)),
              y.data_ptr(), _lib.ptr(g_q), _lib.ptr(loss), _lib.ptr(ws), _lib.stream())
    return y, g_q, loss


def maddpg_critic_target(q, q_next, rewards, dones, gamma):
    """-> (y (B,1), dloss/dq (B,1), loss (1,)) of MADDPG._learn_individual's
    critic step (maddpg.py:764-790) in one launch (+ the fixed-order loss sum)."""
    B = q.shape[0]
    qf, qn, r, d = (t.reshape(-1) for t in (q, q_next, rewards, dones))
    for t, name in ((qf, "q"), (qn, "q_next"), (r, "rewards"), (d, "dones")):
        _need(t, name, _f32, (B,))
    y = torch.empty(B, 1, dtype=_f32, device=r.device)
    g_q = torch.empty(B, 1, dtype=_f32, device=r.device)
    loss = torch.empty(1, dtype=_f32, device=r.device)
    ws = _ws(_lib.load().agx_td_workspace_bytes(B), r.device)
    _lib.call("agx_maddpg_critic_target", qf.data_ptr(), qn.data_ptr(), r.data_ptr(), d.data_ptr(), B,
              float(gamma), y.data_ptr(), g_q.data_ptr(), loss.data_ptr(), _lib.ptr(ws), _lib.stream())
    return y, g_q, loss


def c51_project_loss(q_next_online, target_dist, logp_cur, actions, rewards, dones, support, v_min,
                     v_max, gamma, with_proj=False):
    B, A, Z = target_dist.shape
    _need(q_next_online, "q_next_online", _f32, (B, A))
    _need(target_dist, "target_dist", _f32)
    _need(logp_cur, "logp_cur", _f32, (B, A, Z))
    a = actions.reshape(-1)
    _need(a, "actions", _i64, (B,))
    r = rewards.reshape(-1)
    d = dones.reshape(-1)
    _need(r, "rewards", _f32, (B,))
    _need(d, "dones", _f32, (B,))
    _need(support, "support", _f32, (Z,))
    loss = torch.empty(B, dtype=_f32, device=r.device)
    proj = torch.empty(B, Z, dtype=_f32, device=r.device) if with_proj else None
    _lib.call("agx_c51_project_loss", q_next_online.data_ptr(), target_dist.data_ptr(),
              logp_cur.data_ptr(), a.data_ptr(), r.data_ptr(), d.data_ptr(), support.data_ptr(), B, A,
              Z, float(v_min), float(v_max), float(gamma), loss.data_ptr(), _lib.ptr(proj),
              _lib.stream())
    return (loss, proj) if with_proj else loss


def c51_project_loss_rows(target_rows, logp_rows, rewards, dones, support, v_min, v_max, gamma, with_proj=False):
    """agx_c51_project_loss_rows: the projection + loss on the selected rows
    ([B][Z] target distribution of a*, [B][Z] log p of the taken action)."""
    B, Z = target_rows.shape
    _need(target_rows, "target_rows", _f32, (B, Z))
    _need(logp_rows, "logp_rows", _f32, (B, Z))
    r = rewards.reshape(-1)
    d = dones.reshape(-1)
    _need(r, "rewards", _f32, (B,))
    _need(d, "dones", _f32, (B,))
    _need(support, "support", _f32, (Z,))
    loss = torch.empty(B, dtype=_f32, device=r.device)
    proj = torch.empty(B, Z, dtype=_f32, device=r.device) if with_proj else None
    _lib.call("agx_c51_project_loss_rows", target_rows.data_ptr(), logp_rows.data_ptr(), r.data_ptr(), d.data_ptr(),
              support.data_ptr(), B, Z, float(v_min), float(v_max), float(gamma), loss.data_ptr(), _lib.ptr(proj),
              _lib.stream())
    return (loss, proj) if with_proj else loss


# --------------------------------------------------------------------------- #
# optimiser                                                                   #
# --------------------------------------------------------------------------- #
class ClipAdam:
    """Fused per-agent grad-norm clip + Adam over flat [P, n] buffers, with a
    per-agent Adam step count on the device (``steps``, int64 [P])."""

    def __init__(self, params: torch.Tensor, group_offsets, lr, betas=(0.9, 0.999), eps=1e-8,
                 max_norm=0.5, grads: torch.Tensor | None = None):
        _need(params, "params", _f32)
        if params.dim() != 2:
            raise ValueError("params must be [P, n]")
        self.params = params
        P, n = params.shape
        self.grads = torch.zeros_like(params) if grads is None else grads
        _need(self.grads, "grads", _f32, tuple(params.shape))
        self.exp_avg = torch.zeros_like(params)
        self.exp_avg_sq = torch.zeros_like(params)
        self.steps = torch.zeros(P, dtype=torch.int64, device=params.device)
        self.offsets = (torch.tensor(list(group_offsets), dtype=torch.int64)).contiguous()
        if int(self.offsets[0]) != 0 or int(self.offsets[-1]) != n:
            raise ValueError("group offsets must span [0, n)")
        lr_t = torch.as_tensor(lr, dtype=_f32).reshape(-1)
        self.lr = (lr_t.expand(P) if lr_t.numel() == 1 else lr_t).to(params.device).contiguous()
        self.betas, self.eps, self.max_norm = betas, eps, max_norm
        self.workspace = _ws(_lib.load().agx_adam_workspace_bytes(P, n), params.device)

    def step(self, active: torch.Tensor | None = None):
        """One clip + Adam update of every agent (or of the agents whose
        ``active`` u8 flag is set; the others are untouched)."""
        P, n = self.params.shape
        _lib.call("agx_clip_adam", self.params.data_ptr(), self.grads.data_ptr(),
                  self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), P, n,
                  self.offsets.data_ptr(), len(self.offsets) - 1, float(self.max_norm),
                  self.lr.data_ptr(), float(self.betas[0]), float(self.betas[1]), float(self.eps),
                  self.steps.data_ptr(), _lib.ptr(active), self.workspace.data_ptr(), _lib.stream())


class _NoisyLayer(ctypes.Structure):
    _fields_ = [("eps_in", ctypes.c_void_p), ("eps_out", ctypes.c_void_p), ("weight_epsilon", ctypes.c_void_p),
                ("bias_epsilon", ctypes.c_void_p), ("in_features", ctypes.c_int64), ("out_features", ctypes.c_int64)]


def noisy_reset_(layers: list) -> None:
    """agx_noisy_reset: ``layers`` = [(eps_in, eps_out, weight_epsilon,
    bias_epsilon)] — each layer's two N(0, 1) draws and its epsilon buffers
    (NoisyLinear.reset_noise, custom_components.py:116-131), one launch."""
    arr = (_NoisyLayer * max(1, len(layers)))()
    for k, (ei, eo, we, be) in enumerate(layers):
        n_in, n_out = ei.numel(), eo.numel()
        _need(ei, "eps_in", _f32)
        _need(eo, "eps_out", _f32)
        _need(we, "weight_epsilon", _f32, (n_out, n_in))
        _need(be, "bias_epsilon", _f32, (n_out,))
        arr[k] = _NoisyLayer(ei.data_ptr(), eo.data_ptr(), we.data_ptr(), be.data_ptr(), n_in, n_out)
    _lib.call("agx_noisy_reset", ctypes.cast(arr, ctypes.c_void_p), len(layers), _lib.stream())


def polyak_(target: torch.Tensor, online: torch.Tensor, tau: float) -> None:
    _need(target, "target", _f32)
    _need(online, "online", _f32, tuple(target.shape))
    _lib.call("agx_polyak", target.data_ptr(), online.data_ptr(), target.numel(), float(tau),
              _lib.stream())
