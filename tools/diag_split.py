"""Diagnostic: fused learner partner splits vs each other and the torch learner (8 updates)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import torch
from test_population_gpu import _pop, _clone_state, _restore
from agilerl_amd.population.learner import fused_learn

res = {}
for lat in (64,):
    for split in ("1", "4", "1x16", "4x16", "4x16b", "8x16"):
        k, _, sb = split.rstrip("b").partition("x")
        os.environ["AGX_LEARN_SPLIT"] = k
        if sb:
            os.environ["AGX_LEARN_SB"] = sb
        else:
            os.environ.pop("AGX_LEARN_SB", None)
        np.random.seed(5)
        pop = _pop(P=4, N=16, learn_step=512, batch=128, epochs=2, seed=11, latent_dim=lat)
        st = _clone_state(pop)
        perms = pop.permutations()
        if "torch" not in res.get(lat, {}):
            pop._learn_torch(perms)
            res.setdefault(lat, {})["torch"] = pop.opt.exp_avg.cpu().numpy().copy()
            _restore(pop, st)
        fused_learn(pop, perms)
        torch.cuda.synchronize()
        res[lat][split] = pop.opt.exp_avg.cpu().numpy().copy()
        print(lat, split, "desc", pop.fused_descriptor(), flush=True)
    t = res[lat]["torch"]
    scale = np.abs(t).max()
    for name, m in res[lat].items():
        for ref in ("torch", "1"):
            r = res[lat][ref]
            bad = np.abs(m - r) > 2e-3 * np.abs(r) + 1e-5 * scale
            print(f"lat {lat} {name:6s} vs {ref:5s}: bad/agent {bad.mean(1).round(4)} max {np.abs(m - r).max() / scale:.2e}")
