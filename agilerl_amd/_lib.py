"""ctypes binding of libagx.so (the C ABI declared in include/agx.h and
include/agx_graph.h).

This is the binding a maintainer of the reference would add (see
INTEGRATION.md).  The product path has NO CPU fallback: if the library is
missing or no GPU is visible, every op raises.
"""

from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must load torch's HIP runtime before libagx binds to it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AGX_LIB") or os.path.join(_HERE, "lib", "libagx.so")  # AGX_LIB: A/B builds

_P = ctypes.c_void_p
_I = ctypes.c_int64
_D = ctypes.c_double
_F = ctypes.c_float
_INT = ctypes.c_int
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/agx.h one-to-one
SIGNATURES = {
    "agx_last_error": (ctypes.c_char_p, []),
    "agx_version": (_INT, []),
    "agx_device_info": (_INT, [_P]),
    "agx_gae_workspace_bytes": (_SZ, [_I, _I, _I]),
    "agx_gae": (_INT, [_P, _P, _P, _P, _P, _I, _I, _I, _D, _D, _INT, _P, _P, _P, _P, _P]),
    "agx_adv_normalize": (_INT, [_P, _P, _I, _I, _P]),
    "agx_ppo_loss_fwd_bwd": (_INT, [_P] * 8 + [_I, _I, _F, _F, _F, _P, _P, _P, _P, _P]),
    "agx_ppo_learn_lds_bytes": (_SZ, [_P]),
    "agx_ppo_learn_workspace_bytes": (_SZ, [_P, _I, _I, _I]),
    "agx_ppo_learn_prepare": (_INT, [_P, _P, _P]),
    # include/agx_graph.h: the runtime-shape learner
    "agx_ppo_graph_check": (_INT, [_P]),
    "agx_ppo_learn_graph_workspace_bytes": (_SZ, [_P, _I, _I, _I, _I]),
    "agx_ppo_learn_graph": (_INT, [_P, _P, _P, _P]),
    "agx_ppo_act_graph_workspace_bytes": (_SZ, [_P, _I, _I]),
    "agx_debug_graph_stamps": (_INT, [_P]),
    "agx_ppo_rollout_graph_workgroups": (_I, [_I, _I]),
    "agx_ppo_rollout_graph_max_workgroups": (_I, []),
    "agx_ppo_rollout_graph_ctl_bytes": (_SZ, [_I, _I]),
    "agx_ppo_rollout_graph_persistent": (_INT, [_P, _I, _I, _P, _P, _I, ctypes.c_uint32, ctypes.c_uint64,
                                                ctypes.c_uint64, _P, _P, _D, _P, _P]),
    "agx_ppo_eval_graph_persistent": (_INT, [_P, _I, _I, _P, _P, _P, _P, _P, _I, ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.c_uint64, _P, _P, _D, _P, _P]),
    "agx_ppo_eval_multi_bytes": (_SZ, [_I]),
    "agx_debug_eval_stamps": (_INT, [_P]),
    "agx_ppo_eval_multi_supported": (_INT, [_P, _I, _I]),
    "agx_ppo_eval_multi_persistent": (_INT, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _I, ctypes.c_uint32, _P, _P, _P,
                                             _D, _P, _P]),
    "agx_ppo_act_graph": (_INT, [_P, _I, _I, _P, _P, _I, _P, _I, _INT, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P,
                                 _P, _I, _P, _P, _P, _P]),
    "agx_ppo_learn": (_INT, [_P, _P, _P, _P]),
    "agx_ppo_act": (_INT, [_P, _I, _I, _P, _P, _I, _P, _I, _INT, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P, _P,
                           _I, _P, _P, _P]),
    "agx_ppo_rollout_step": (_INT, [_P, _I, _I, _P, _P, _INT, _INT, ctypes.c_uint64, ctypes.c_uint64, _P]),
    "agx_rollout_workgroups": (_I, [_I, _I]),
    "agx_rollout_max_workgroups": (_I, [_P]),
    "agx_rollout_ctl_bytes": (_SZ, [_I, _I]),
    "agx_rollout_args_bytes": (_SZ, [_I]),
    "agx_ppo_rollout_persistent": (_INT, [_P, _I, _I, _P, _P, _I, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                          _P, _P, _D, _P]),
    "agx_ppo_eval_persistent": (_INT, [_P, _I, _I, _P, _P, _P, _P, _P, _I, ctypes.c_uint32, ctypes.c_uint64,
                                       ctypes.c_uint64, _P, _P, _D, _P]),
    "agx_host_alloc": (_P, [_SZ]),
    "agx_host_free": (_INT, [_P]),
    "agx_stream_create": (_P, []),
    "agx_host_signal": (_INT, [_P, ctypes.c_uint32]),
    "agx_host_wait": (_INT, [_P, _I, ctypes.c_uint32, _D]),
    "agx_host_signal_range": (_INT, [_P, _I, _I, ctypes.c_uint32]),
    "agx_host_wait_range": (_INT, [_P, _I, _I, ctypes.c_uint32, _D]),
    "agx_host_signal_wait_range": (_INT, [_P, _I, _I, ctypes.c_uint32, _I, _I, ctypes.c_uint32, _D]),
    "agx_per_workspace_bytes": (_SZ, [_I, _I]),
    "agx_per_init": (_INT, [_P, _P, _I, _P]),
    "agx_per_add": (_INT, [_P, _P, _I, _I, _I, _I, _D, _P, _P, _P]),
    "agx_per_update": (_INT, [_P, _P, _I, _I, _P, _P, _I, _D, _D, _P, _P, _P]),
    "agx_per_sample": (_INT, [_P, _P, _I, _P, _I, _I, _D, _P, _P, _P, _P]),
    "agx_per_gather": (_INT, [_P, _P, _I, _P, _P]),
    "agx_segtree_workspace_bytes": (_SZ, [_I]),
    "agx_segtree_init": (_INT, [_P, _I, _INT, _P]),
    "agx_segtree_set": (_INT, [_P, _I, _INT, _P, _P, _I, _P, _P]),
    "agx_segtree_operate": (_INT, [_P, _I, _INT, _I, _I, _P, _P]),
    "agx_segtree_retrieve": (_INT, [_P, _I, _P, _I, _P, _P, _P]),
    "agx_td_workspace_bytes": (_SZ, [_I]),
    "agx_td_target": (_INT, [_P] * 6 + [_I, _I, _D, _INT, _P, _P, _P, _P, _P]),
    "agx_maddpg_critic_target": (_INT, [_P] * 4 + [_I, _D, _P, _P, _P, _P, _P]),
    "agx_c51_project_loss": (_INT, [_P] * 7 + [_I, _I, _I, _D, _D, _D, _P, _P, _P]),
    "agx_c51_project_loss_rows": (_INT, [_P] * 5 + [_I, _I, _D, _D, _D, _P, _P, _P]),
    "agx_adam_workspace_bytes": (_SZ, [_I, _I]),
    "agx_clip_adam": (_INT, [_P, _P, _P, _P, _I, _I, _P, _INT, _F, _P, _F, _F, _F, _P, _P, _P, _P]),
    "agx_polyak": (_INT, [_P, _P, _I, _F, _P]),
    "agx_noisy_reset": (_INT, [_P, _INT, _P]),
    "agx_noisy_streams_forward": (_INT, [_P, _INT, _INT, _P, _I, _F, _P]),
    "agx_noisy_streams_forward_each": (_INT, [_P, _INT, _INT, _P, _I, _F, _P]),
    "agx_noisy_streams_workspace_bytes": (_SZ, [_P, _INT, _INT, _I]),
    "agx_noisy_streams_backward": (_INT, [_P, _INT, _INT, _P, _I, _F, _P, _P, _P, _P]),
    "agx_conv2d_forward": (_INT, [_P, _P, _INT, _F, _F, _P, _P, _INT, _P, _P]),
    "agx_conv2d_wgrad_workspace_bytes": (_SZ, [_P]),
    "agx_conv2d_backward": (_INT, [_P, _P, _INT, _F, _F, _P, _P, _P, _P, _P, _P, _INT, _P, _P]),
    "agx_rows_gather_workspace_bytes": (_SZ, [_P, _INT, _I]),
    "agx_rows_gather": (_INT, [_P, _P, _INT, _I, _P, _P, _P]),
    "agx_dueling_head_forward": (_INT, [_P, _P, _P, _I, _I, _I, _INT, _P, _P]),
    "agx_dueling_head_backward": (_INT, [_P, _P, _P, _P, _I, _I, _I, _INT, _P, _P, _P]),
    "agx_dueling_head_forward_rows": (_INT, [_P, _P, _P, _I, _I, _I, _INT, _P, _P]),
    "agx_dueling_head_backward_rows": (_INT, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "agx_conv2d_forward_grouped": (_INT, [_P, _I, _P, _I, _INT, _F, _F, _P, _I, _P, _I, _INT, _P, _I, _P]),
    "agx_conv2d_forward_grouped2": (_INT, [_P, _I, _I, _P, _I, _I, _INT, _F, _F, _P, _I, _I, _P, _I, _I, _INT, _P,
                                           _I, _I, _P]),
    "agx_replay_gather": (_INT, [_P, _P, _P, _INT, _P, _I, _I, _P, _P]),
    "agx_conv2d_wgrad_workspace_bytes_grouped": (_SZ, [_P, _I]),
    "agx_conv2d_backward_grouped": (_INT, [_P, _I, _P, _I, _INT, _F, _F, _P, _I, _P, _P, _I, _P, _P, _P,
                                           _INT, _P, _P]),
    "agx_debug_pow": (_INT, [_P, _P, _P, _I, _P]),
    "agx_debug_learn_stamps": (_INT, [_P]),
    "agx_debug_rollout_stamps": (_INT, [_P]),
    "agx_debug_learn_stall": (_INT, [_INT]),
    "agx_host_shuffle_perms": (_INT, [_P, _P, _I, _I, _I, _P, _P]),
    "agx_debug_stream": (_INT, [_P, _P, _I, _INT, _I, _P]),
}

_lib = None


class AgxError(RuntimeError):
    pass


def load(require_gpu: bool = True):
    """Load libagx.so (raises if absent).  With require_gpu, also insist on a
    visible ROCm device — the product path never runs on the CPU."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AgxError(
                f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("AGX_LIB") and not hasattr(lib, name):
                continue  # an A/B build of an older revision: only what it exports
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_gpu and not torch.cuda.is_available():
        raise AgxError("agilerl_amd needs an MI355X (ROCm device); no CPU fallback exists")
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib.agx_last_error().decode(errors="replace") if _lib is not None else ""
        raise AgxError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream(s=None) -> int:
    """hipStream_t of ``s`` (default: torch's current stream on the current
    device).  Read through torch's raw accessor: torch.cuda.current_stream()
    builds a Stream object per call (~2 us of host time on every launch)."""
    if s is not None:
        return s.cuda_stream
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def call(name: str, *args) -> None:
    lib = load()
    check(getattr(lib, name)(*args), name)
