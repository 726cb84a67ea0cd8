"""Three learn() calls of the runtime-shape learner at the config-2 shape (a
short program for rocprofv3 counter passes)."""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from graph_bench import make  # noqa: E402

from agilerl_amd.population.learner import GraphLearner  # noqa: E402

pop = make()
perms = pop.permutations()
gl = GraphLearner(pop)
for _ in range(3):
    gl.learn(pop, perms)
torch.cuda.synchronize()
print("done", flush=True)
