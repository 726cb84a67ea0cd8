"""LDS-resident vs global-scratch partner activations: the same learn() (the
test_graph_learner_gpu no_layer_norm case) under AGX_GRAPH_LDS / AGX_GRAPH_ROWS
settings, compared bitwise with the global-scratch 16-row run."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_graph_learner_gpu import _pop, _restore, _state  # noqa: E402
from agilerl_amd.population.learner import fused_learn  # noqa: E402

pop = _pop("no_layer_norm", N=16, learn_step=256, batch=64, epochs=2)
perms = pop.permutations()
st = _state(pop)
res = {}
for name, env in [("g16", {"AGX_GRAPH_LDS": "0", "AGX_GRAPH_ROWS": "16"}),
                  ("l16", {"AGX_GRAPH_LDS": "1", "AGX_GRAPH_ROWS": "16"}),
                  ("g8", {"AGX_GRAPH_LDS": "0", "AGX_GRAPH_ROWS": "8"}),
                  ("l8", {"AGX_GRAPH_LDS": "1", "AGX_GRAPH_ROWS": "8"}),
                  ("auto", {})]:
    for k in ("AGX_GRAPH_LDS", "AGX_GRAPH_ROWS"):
        os.environ.pop(k, None)
    os.environ.update(env)
    _restore(pop, st)
    fused_learn(pop, perms)
    torch.cuda.synchronize()
    res[name] = (pop.params.data.clone(), pop.opt.exp_avg.clone())
for name in res:
    for ref in ("g16", "g8"):
        dp = (res[name][0] - res[ref][0]).abs().max().item()
        dm = (res[name][1] - res[ref][1]).abs().max().item()
        print(f"{name} vs {ref}: params max diff {dp:.3e}  exp_avg max diff {dm:.3e}")
