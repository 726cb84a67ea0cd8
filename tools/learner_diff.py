"""Per-tensor gradient comparison: fused learner vs torch learner, one update
(diagnostic for the fused kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from test_population_gpu import _clone_state, _pop, _restore  # noqa: E402
from agilerl_amd.population.learner import fused_learn  # noqa: E402

N, LS, B = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (32, 64, 64)))
pop = _pop(N=N, learn_step=LS, batch=B, epochs=1, seed=5)
st = _clone_state(pop)
perms = pop.permutations()
lt = pop._learn_torch(perms).clone()
m_t = pop.opt.exp_avg.clone()
_restore(pop, st)
lf = fused_learn(pop, perms).clone()
torch.cuda.synchronize()
m_f = pop.opt.exp_avg
print("loss torch", lt.tolist(), "fused", lf.tolist())
for name, (off, shape) in pop.spec.state_dict_keys().items():
    n = 1
    for s in shape:
        n *= s
    a = m_f[:, off:off + n]
    b = m_t[:, off:off + n]
    err = (a - b).abs()
    rel = (err.max() / b.abs().max().clamp_min(1e-30)).item()
    print(f"{name:55s} {str(shape):12s} maxabs(t)={b.abs().max().item():.3e} max_err={err.max().item():.3e} rel={rel:.2e}")
    if rel > 1e-2 and len(shape) == 2:
        e = err[0].view(shape)
        r, c = divmod(int(e.argmax()), shape[1])
        print("     worst at row", r, "col", c, "fused", a[0].view(shape)[r, c].item(), "torch", b[0].view(shape)[r, c].item())
        bad_rows = (e.max(1).values > 1e-2 * b.abs().max()).nonzero().view(-1).tolist()
        bad_cols = (e.max(0).values > 1e-2 * b.abs().max()).nonzero().view(-1).tolist()
        print("     bad rows", bad_rows[:20], "bad cols", bad_cols[:20])
    elif rel > 1e-2:
        e = err[0]
        print("     fused", [round(x, 7) for x in a[0, :6].tolist()], "torch", [round(x, 7) for x in b[0, :6].tolist()])
        print("     bad idx", (e > 1e-2 * b.abs().max()).nonzero().view(-1).tolist()[:20])
