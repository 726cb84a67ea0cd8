"""PER priority update of 2^16 indices on a 2^20 tree (bench.py kernels_leg
shape), 20 calls, for a per-kernel rocprofv3 breakdown."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agilerl_amd import kernels as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(2)
cap, max_size = 1 << 20, 1_000_000
st = torch.empty(2 * cap, dtype=torch.float64, device=dev)
mt = torch.empty_like(st)
K.per_init(st, mt, cap)
maxp = torch.ones(1, dtype=torch.float64, device=dev)
ws = K.per_workspace(cap, dev)
K.per_add(st, mt, cap, max_size, 0, max_size, 0.6, maxp, workspace=ws)
idx = torch.randint(0, max_size, (1 << 16,), device=dev, generator=g)
p2 = torch.rand(1 << 16, device=dev, generator=g)
torch.cuda.synchronize()
for _ in range(20):
    K.per_update(st, mt, cap, max_size, idx, p2, 0.6, maxp, workspace=ws)
torch.cuda.synchronize()
print("done")
