"""Profile target: bench.config3_leg (config 3: the per-agent train_off_policy
update and the population-batched Rainbow learner).  Before and after each
timed loop a marker kernel (agx_debug_stream over 16 bytes) goes out, so
tools/trace_window.py can summarise the kernels of one timed loop alone,
without the agents' construction (orthogonal init) or the warm-up:

  rocprofv3 --kernel-trace --output-format csv -d DIR -o c3 -- python tools/prof_config3.py
  python tools/trace_window.py DIR/.../c3_kernel_trace.csv per_agent > r6_config3_kernel_stats.csv"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

from agilerl_amd import _lib  # noqa: E402

buf = None


def marker(name, start):
    global buf
    if buf is None:
        buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    # one marker launch per boundary; the loop order (batched, per_agent) is
    # fixed, so the window of loop k lies between markers 2k and 2k + 1
    _lib.call("agx_debug_stream", buf.data_ptr(), buf[32:].data_ptr(), 16, 1, 1, _lib.stream())
    torch.cuda.synchronize()


print(bench.config3_leg(iters=int(os.environ.get("ITERS", 5)), on_timed=marker))
