"""Localise a fused-learner mismatch against oracle/ppo_learn.py on a golden
case: runs (epochs, batch) variants and partner splits, prints per-layer max
|diff| of the parameters after the learn.  python tools/learner_diag.py learn0"""

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle.ppo_learn import ActorCritic, reference_learn  # noqa: E402
from test_learner_parity_gpu import DEV, _flat_from_names, _names, _pop, _set_stats  # noqa: E402


def run(g, E, B, split):
    from agilerl_amd.population.learner import fused_learn

    os.environ["AGX_LEARN_SPLIT"] = str(split)
    T, N = int(g["T"]), int(g["N"])
    S = T * N
    pop = _pop(1, N, T, int(g["obs_dim"]), int(g["n_actions"]), g["enc"], int(g["latent"]), g["actor_hidden"],
               g["critic_hidden"], B, E, float(g["lr"]))
    spec, n = pop.spec, pop.spec.n_params
    t = lambda x: torch.as_tensor(np.asarray(x)).to(DEV)  # noqa: E731
    init = _names(g, "init.")
    pop.params.data[0] = t(_flat_from_names(spec, init, n))
    pop.obs.view(-1)[:] = t(g["obs"]).view(-1)
    pop.actions.view(-1)[:] = t(g["actions"])
    pop.log_probs.view(-1)[:] = t(g["old_logp"])
    pop.values.view(-1)[:] = t(g["old_v"])
    pop.advantages.view(-1)[:] = t(g["adv"])
    pop.returns.view(-1)[:] = t(g["ret"])
    _set_stats(pop)
    perms = t(g["perms"][:E]).view(E, 1, S).contiguous()
    loss = fused_learn(pop, perms)
    torch.cuda.synchronize()
    got = pop.params.data[0].cpu().numpy()
    net = ActorCritic(int(g["obs_dim"]), int(g["n_actions"]), list(g["enc"]), int(g["latent"]),
                      list(g["actor_hidden"]), list(g["critic_hidden"]))
    net.load_reference(init)
    out = reference_learn(net, None, g["obs"], g["actions"], g["old_logp"], g["adv"], g["ret"], g["old_v"],
                          g["perms"][:E], batch_size=B, epochs=E, lr=float(g["lr"]))
    print(f"E={E} B={B} split={split}: loss gpu {float(loss[0]):.9g} oracle {out['mean_loss']:.9g}")
    for k, (off, shape) in spec.state_dict_keys().items():
        if k.startswith("critic.encoder."):
            continue
        m = int(np.prod(shape))
        a, b = got[off:off + m], out["state"][k].numpy().ravel()
        d = np.abs(a - b)
        print(f"   {k:55s} max|d| {d.max():.3e}  mean|d| {d.mean():.3e}  max|ref| {np.abs(b).max():.3e}")


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "learn0"
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", f"{name}.npz")))
    S = int(g["T"]) * int(g["N"])
    for E, B, split in [(1, S, 1), (1, S, 4), (1, 128, 1), (1, 128, 4), (4, 128, 4)]:
        run(g, E, B, split)
