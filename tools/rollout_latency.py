"""Per-vector-step latency of the persistent rollout: host signal -> all
workgroups done (device step), and the host env step (diagnostic)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from agilerl_amd import _lib  # noqa: E402
from agilerl_amd.envs import SyntheticVecEnv  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402
from agilerl_amd.population.runner import PopulationRunner  # noqa: E402

P, N = 8, 128
pop = PPOPopulation(ActorCriticSpec(obs_dim=8, n_actions=4), P, N, learn_step=2048, batch_size=128,
                    update_epochs=4, device="cuda")
run = PopulationRunner(pop, SyntheticVecEnv(P * N))
assert run.persistent
for _ in range(3):
    run.iteration()
torch.cuda.synchronize()
lib = _lib.load()
T = pop.T
dev_t, env_t, launch_t = [], [], []
orig_env = run._env_step
orig_sig, orig_wait = lib.agx_host_signal, lib.agx_host_wait
marks = {}


class Sig:
    def __call__(self, ctl, seq):
        marks["s"] = time.perf_counter()
        return orig_sig(ctl, seq)


class Wait:
    def __call__(self, *a):
        rc = orig_wait(*a)
        dev_t.append(time.perf_counter() - marks["s"])
        return rc


def env_step():
    t0 = time.perf_counter()
    orig_env()
    env_t.append(time.perf_counter() - t0)


lib.agx_host_signal, lib.agx_host_wait = Sig(), Wait()
run._env_step = env_step
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.collect()
    launch_t.append(time.perf_counter() - t0)
    pop.finish_rollout(run.last_obs, run.last_done, run.last_value)
    pop.learn()
torch.cuda.synchronize()
lib.agx_host_signal, lib.agx_host_wait = orig_sig, orig_wait
dev_t = sorted(dev_t)
print(f"device step (signal -> all done): median {1e6 * dev_t[len(dev_t) // 2]:.1f} us, "
      f"p10 {1e6 * dev_t[len(dev_t) // 10]:.1f}, p90 {1e6 * dev_t[9 * len(dev_t) // 10]:.1f}; "
      f"first step incl. kernel start {1e6 * sum(dev_t[:1]):.1f}")
print(f"env step {1e6 * sum(env_t) / len(env_t):.1f} us; collect {1e3 * sum(launch_t) / len(launch_t):.3f} ms "
      f"({1e6 * sum(launch_t) / len(launch_t) / T:.1f} us/step)")

# in-kernel phases of workgroup 0 (s_memrealtime, 100 MHz)
buf = torch.zeros(384, dtype=torch.int64, device="cuda")
lib.agx_debug_rollout_stamps(ctypes.c_void_p(buf.data_ptr()))
run.collect()
lib.agx_debug_rollout_stamps(None)
pop.finish_rollout(run.last_obs, run.last_done, run.last_value)
torch.cuda.synchronize()
st = buf[:256].view(32, 8).cpu().numpy()[:T + 1].astype(float) * 10.0  # ns
names = ["wait for host", "host reads", "scatter+zero+forward", "sample+stores", "store acks"]
ph = [st[1:T, k + 1] - st[1:T, k] for k in range(5)]
print("in-kernel phases (us, median over steps 1..T-1): " +
      ", ".join(f"{n} {float(sorted(x)[len(x) // 2]) / 1e3:.2f}" for n, x in zip(names, ph)))
gap = st[2:T, 1] - st[1:T - 1, 5]
print(f"done -> next release seen: {float(sorted(gap)[len(gap) // 2]) / 1e3:.2f} us (host detect + env step + signal)")
nwg = run.n_wg
b = buf.cpu().numpy().astype(float) * 10.0
go, dn = b[256:256 + nwg], b[320:320 + nwg]
print(f"step 5 across {nwg} workgroups: release seen spread {(go.max() - go.min()) / 1e3:.2f} us, "
      f"done spread {(dn.max() - dn.min()) / 1e3:.2f} us, per-workgroup step median {np.median(dn - go) / 1e3:.2f} "
      f"max {(dn - go).max() / 1e3:.2f} us")
