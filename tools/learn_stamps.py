"""Phase timing of the fused learner (diagnostic; uses agx_debug_learn_stamps).

Slots (learner.hip AGX_STAMP): sub-batch k of agent 0's first minibatch at
k*16 + {0 start, 4 sub-batch committed to LDS, 5 next prefetch issued,
1 barrier passed, 2 forward trunk, 3 head row pass (LN fwd + output layers +
loss + LN bwd), 6 output-layer + head dW / dX, 7 encoder bwd}; 64+9 gradients dumped, 64+10 Adam done;
partners: 64+11/12 first barrier ticket/passed, 64+13 reduce-scatter done,
64+8/15 second barrier ticket/passed, 64+14 norm done."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from agilerl_amd import _lib  # noqa: E402
from agilerl_amd.envs import SyntheticVecEnv  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402
from agilerl_amd.population.runner import PopulationRunner  # noqa: E402

P, N = int(os.environ.get("P", 8)), int(os.environ.get("N", 128))
spec = ActorCriticSpec(obs_dim=8, n_actions=4)
pop = PPOPopulation(spec, P, N, learn_step=2048, batch_size=128, update_epochs=4, device="cuda")
runner = PopulationRunner(pop, SyntheticVecEnv(P * N))
runner.iteration()
buf = torch.zeros(80, dtype=torch.int64, device="cuda")
lib = _lib.load()
lib.agx_debug_learn_stamps(buf.data_ptr())
runner.collect()
pop.finish_rollout(runner.last_obs, runner.last_done)
torch.cuda.synchronize()
t0 = time.perf_counter()
pop.learn()
torch.cuda.synchronize()
t1 = time.perf_counter()
lib.agx_debug_learn_stamps(None)
st = buf.cpu().tolist()
nmb = pop.update_epochs * pop.n_minibatches()
print(f"learn() wall {1e3 * (t1 - t0):.3f} ms  ({nmb} minibatch updates per agent, {P} agents)")
# slots in time order: 0 start, 4 committed, 5 next prefetch issued, 1 barrier,
# 2 trunk, 3 head row pass, 6 output/head dW + dX, 7 encoder bwd
order = [0, 4, 5, 1, 2, 3, 6, 7]
names = ["commit", "prefetch issue", "barrier", "trunk fwd", "head row pass", "out+head dW, dX", "enc bwd"]
for sb in range(4):
    row = [st[sb * 16 + k] for k in order]
    if not all(row):  # only workgroup 0 stamps: with K partners it runs 1 of every K sub-batches
        continue
    seg = [row[i + 1] - row[i] for i in range(7)]
    print(f"sb{sb}: " + "  ".join(f"{n}={c}" for n, c in zip(names, seg)) + f"  total={row[7] - row[0]}")
    # trunk sub-phases (slots 8..11: encoder layer L GEMM / LN passed, 2 = the head GEMM passed)
    sub = [st[sb * 16 + 1]] + [st[sb * 16 + k] for k in (8, 9, 10, 11)] + [st[sb * 16 + 2]]
    if all(sub):
        print("   trunk: " + "  ".join(f"{n}={sub[i + 1] - sub[i]}" for i, n in
                                     enumerate(["enc0 gemm", "enc0 LN", "enc1 gemm", "enc1 LN", "head gemm"])))
last = max(v for v in st[:64] if v)
if st[64 + 1]:  # partners: reduce-scatter + distributed Adam (three barriers)
    print("dump", st[64 + 9] - last, "| publish", st[64 + 11] - st[64 + 9], "wait", st[64 + 12] - st[64 + 11],
          "| RS loads+sum", st[64 + 3] - st[64 + 12], "norm partials", st[64 + 13] - st[64 + 3],
          "| B2 drain + ticket", st[64 + 8] - st[64 + 13], "wait", st[64 + 15] - st[64 + 8],
          "| norm read", st[64 + 14] - st[64 + 15], "adam + publish + B3 drain/ticket", st[64 + 0] - st[64 + 14],
          "B3 wait", st[64 + 1] - st[64 + 0], "param read", st[64 + 2] - st[64 + 1],
          "sync", st[64 + 10] - st[64 + 2], "| minibatch total cycles", st[64 + 10] - st[0])
elif st[64 + 15]:  # partners: reduce-scatter exchange (two barriers)
    print("dump", st[64 + 9] - last, "| publish", st[64 + 11] - st[64 + 9], "wait", st[64 + 12] - st[64 + 11],
          "reduce-scatter", st[64 + 13] - st[64 + 12], "| barrier 2 drain + ticket", st[64 + 8] - st[64 + 13],
          "wait", st[64 + 15] - st[64 + 8], "| sum read + norm", st[64 + 14] - st[64 + 15],
          "adam", st[64 + 10] - st[64 + 14], "| minibatch total cycles", st[64 + 10] - st[0])
else:
    print("dump", st[64 + 9] - last, "| norm", st[64 + 14] - st[64 + 9], "adam", st[64 + 10] - st[64 + 14],
          "| minibatch total cycles", st[64 + 10] - st[0])
