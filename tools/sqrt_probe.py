"""Which f32 square root torch's sqrt kernel computes on this build
(correctly rounded or the hardware approximation), against agx_noisy_reset."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from agilerl_amd import kernels as K  # noqa: E402

x = torch.randn(1 << 20, device="cuda")
t = x.abs().sqrt()
cr = torch.from_numpy(np.sqrt(x.abs().cpu().double().numpy()).astype(np.float32)).cuda()
print("torch sqrt vs correctly rounded: mismatches", int((t != cr).sum()))
one = torch.ones(1, device="cuda")
w = torch.empty(1, x.numel(), device="cuda")
b = torch.empty(1, device="cuda")
K.noisy_reset_([(x, one, w, b)])
ref = x.sign() * t
print("agx vs torch sign*sqrt: mismatches", int((w[0] != ref).sum()))
print("agx vs correctly rounded: mismatches", int((w[0] != x.sign() * cr).sum()))
