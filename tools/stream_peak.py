"""HBM bandwidth probes (agx_debug_stream): copy and read-only over 1 GiB
buffers for several grid sizes (diagnostic for bench.py's measured peak)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from agilerl_amd import _lib  # noqa: E402

lib = _lib.load()
nbytes = 1 << 30
a = torch.empty(nbytes // 4, device="cuda").uniform_()
b = torch.empty_like(a)
for mode in (0, 1):
    for grid in (0, 1024, 2048, 4096, 8192, 16384):
        run = lambda: _lib.check(lib.agx_debug_stream(a.data_ptr(), b.data_ptr(), nbytes, mode, grid, _lib.stream()), "s")
        for _ in range(3):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run()
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / 10
        moved = nbytes * (2 if mode == 0 else 1)
        print(f"mode {'copy' if mode == 0 else 'read'} grid {grid}: {moved / ms / 1e6:.1f} GB/s")
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    b.copy_(a)
e.record()
e.synchronize()
print(f"torch copy: {2 * nbytes / (s.elapsed_time(e) / 10) / 1e6:.1f} GB/s")
