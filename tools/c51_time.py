"""A/B timing of agx_c51_project_loss at the SURVEY §8d shape (B=2^20, A=6,
Z=51): HIP events over 10 launches, with a loss checksum."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agilerl_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
B, A, Z = 1 << 20, 6, 51
g3 = torch.Generator(device=dev).manual_seed(3)
qn = torch.randn(B, A, device=dev, generator=g3)
td = torch.softmax(torch.randn(B, A, Z, device=dev, generator=g3), -1).clamp_(min=1e-3)
lp = torch.log_softmax(torch.randn(B, A, Z, device=dev, generator=g3), -1)
act = torch.randint(0, A, (B,), device=dev, generator=g3)
r = torch.randn(B, device=dev, generator=g3)
d = (torch.rand(B, device=dev, generator=g3) < 0.05).float()
sup = torch.linspace(-200, 200, Z, device=dev)
for _ in range(3):
    out = K.c51_project_loss(qn, td, lp, act, r, d, sup, -200.0, 200.0, 0.99 ** 4)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    K.c51_project_loss(qn, td, lp, act, r, d, sup, -200.0, 200.0, 0.99 ** 4)
e.record()
e.synchronize()
ms = s.elapsed_time(e) / 10
loss = out[0] if isinstance(out, tuple) else out
print(f"c51_project_loss: {ms * 1e3:.1f} us, "
      f"{444 * B / ms / 1e6:.0f} GB/s algorithmic, loss checksum {float(loss.double().sum()):.10e}")
