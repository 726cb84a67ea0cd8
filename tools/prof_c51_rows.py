"""PMC target: agx_c51_project_loss_rows at 2^20 rows (SURVEY 8d shape), 20 launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from agilerl_amd import kernels as K  # noqa: E402

B, A, Z = 1 << 20, 6, 51
g = torch.Generator(device="cuda").manual_seed(3)
tr = torch.softmax(torch.randn(B, Z, device="cuda", generator=g), -1).clamp_(min=1e-3)
lp = torch.log_softmax(torch.randn(B, Z, device="cuda", generator=g), -1)
r = torch.randn(B, device="cuda", generator=g)
d = (torch.rand(B, device="cuda", generator=g) < 0.05).float()
sup = torch.linspace(-200, 200, Z, device="cuda")
for _ in range(20):
    K.c51_project_loss_rows(tr, lp, r, d, sup, -200.0, 200.0, 0.99 ** 4)
torch.cuda.synchronize()
print("ok")
