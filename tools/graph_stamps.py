"""Phase timing of the partnered runtime-shape learner (agx_debug_graph_stamps):
agent 0, partner 0, update 1 of one learn() of graph_bench.py's mutated shape
(encoder [80] -> latent 56 -> actor [64, 64], 8 agents, S = 2048, batch 128,
4 epochs).  Prints the cycles of each phase."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

sys.argv = [sys.argv[0]]
from tools import graph_bench as gb  # noqa: E402
from agilerl_amd import _lib  # noqa: E402
from agilerl_amd.population.learner import GraphLearner  # noqa: E402

pop = gb.make(encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64])
perms = pop.permutations()
gl = GraphLearner(pop)
gl.learn(pop, perms)
torch.cuda.synchronize()
buf = torch.zeros(16 + 18 + 3 * 16, dtype=torch.int64, device="cuda")
lib = _lib.load()
lib.agx_debug_graph_stamps(buf.data_ptr())
t0 = time.perf_counter()
gl.learn(pop, perms)
torch.cuda.synchronize()
t1 = time.perf_counter()
lib.agx_debug_graph_stamps(None)
st = buf.cpu().tolist()
names = ["gradients (fwd + loss + bwd)", "loss words", "barrier 1", "reduce-scatter + norms", "barrier 2",
         "norm / loss read", "Adam", "barrier 3", "acquire"]
print(f"learn() wall {1e3 * (t1 - t0):.3f} ms; update cycles {st[9] - st[0]}")
for i, n in enumerate(names):
    print(f"  {n:32s} {st[i + 1] - st[i]}")

# inside the gradient pass (minibatch_grads' inner stamps)
inner = st[16:]
from agilerl_amd.population.learner import graph_descriptor  # noqa: E402
d = graph_descriptor(pop.spec)
print(f"  obs transpose                    {inner[0] - st[0]}")
prev = inner[0]
L = 0
while L < d.n_layers:
    print(f"  fwd layer {L:2d}                     {inner[1 + L] - prev}")
    prev = inner[1 + L]
    L += 1
print(f"  loss pass                        {inner[17] - prev}")
prev = inner[17]
for l in range(L - 1, -1, -1):
    rows, dx, dw = inner[18 + 3 * l], inner[19 + 3 * l], inner[20 + 3 * l]
    print(f"  bwd layer {l:2d}: rows {rows - prev:6d}  dW (+ column sums) {dx - rows:6d}  dX {dw - dx:6d}")
    prev = dw
for i in range(d.n_layers):
    x = d.layers[i]
    print(f"  layer {i:2d}: src {x.src:2d} {x.fin:3d} -> {x.fout:3d} ln {x.ln} relu {x.relu}")
