"""Attribute the runtime-shape learner's time to its phases: one learn() at
the config-2 shape with each phase skipped (AGX_GRAPH_DEBUG bits: 1 forward
GEMMs, 2 dW GEMMs, 4 dX GEMMs, 8 row passes, 16 column sums, 32 Adam).
Diagnostic only (results are wrong with a phase skipped)."""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from graph_bench import make  # noqa: E402

from agilerl_amd.population.learner import GraphLearner  # noqa: E402

pop = make(**json.loads(os.environ.get("SHAPE", "{}")))
perms = pop.permutations()
gl = GraphLearner(pop)
out = {}
for mask in (0, 1, 2, 4, 8, 16, 32, 63):
    os.environ["AGX_GRAPH_DEBUG"] = str(mask)
    gl.learn(pop, perms)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        gl.learn(pop, perms)
    torch.cuda.synchronize()
    out[mask] = round((time.perf_counter() - t0) / 3 * 1e3, 2)
print(json.dumps(out), flush=True)
