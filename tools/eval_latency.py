"""Per-vector-step latency of the population-wide evaluation launch
(agx_ppo_eval_multi_persistent): the host's signal -> every workgroup done
(agx_host_wait), the host env step, and workgroup 0's device-side intervals
(agx_debug_eval_stamps: release seen -> observations staged -> forward done ->
done word written).  8 agents x 128 synthetic envs, the compiled shape
(diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from agilerl_amd import _lib  # noqa: E402
from agilerl_amd.envs import StackedVecEnv, SyntheticVecEnv  # noqa: E402
from agilerl_amd.population import runner as R  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402

P, N = 8, 128
kw = dict(encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64]) if os.environ.get("MUTATED") else {}
pop = PPOPopulation(ActorCriticSpec(obs_dim=8, n_actions=4, **kw), P, N, learn_step=2048, batch_size=128,
                    update_epochs=4, device="cuda")
env = StackedVecEnv.from_shared(SyntheticVecEnv(N, p_done=1 / 200, max_episode_steps=1000), P)
run = R.PopulationRunner(pop, env)
assert R.population_eval_ok([run])
run.evaluate(max_steps=50)
torch.cuda.synchronize()
lib = _lib.load()
KS = 6 + 16  # kEvalStamps
buf = torch.zeros(32 * KS, dtype=torch.int64, device="cuda")
lib.agx_debug_eval_stamps(buf.data_ptr())
waits, envs = [], []
orig_wait, orig_env = R._EvalDriver.wait, R._EvalDriver.env_step


def wait(self):
    t = time.perf_counter()
    orig_wait(self)
    waits.append(time.perf_counter() - t)


def env_step(self):
    t = time.perf_counter()
    r = orig_env(self)
    envs.append(time.perf_counter() - t)
    return r


R._EvalDriver.wait, R._EvalDriver.env_step = wait, env_step
t0 = time.perf_counter()
run.evaluate(max_steps=400)
dt = time.perf_counter() - t0
torch.cuda.synchronize()
lib.agx_debug_eval_stamps(None)
raw = buf.cpu().numpy().reshape(32, KS)
st = raw[:, :4].astype(np.float64) * 10e-3  # us
d = np.diff(st, axis=1)
cyc = raw[:, 4:].astype(np.float64)  # shader clock: forward start, then after each layer run
fwd_cyc = np.array([row[row > 0].max() - row[0] for row in cyc])
print(f"shader clock over the forward: {np.mean(fwd_cyc / (d[:, 1] * 1e-6)) / 1e9:.2f} GHz equivalent "
      f"({fwd_cyc.mean():.0f} cycles); per layer run (cycles):",
      [round(float(x)) for x in np.diff(np.concatenate([[cyc[0, 0]], cyc[0, 1:][cyc[0, 1:] > 0]]))])
for i in (1, 2, 3):
    print("   step", i, [round(float(x)) for x in np.diff(np.concatenate([[cyc[i, 0]], cyc[i, 1:][cyc[i, 1:] > 0]]))])
gap = st[1:, 0] - st[:-1, 3]  # done written -> next release seen (host env step + signal)
print(f"pass: {dt / 400 * 1e6:.1f} us per step; host wait {np.mean(waits) * 1e6:.1f} us, env step "
      f"{np.mean(envs) * 1e6:.1f} us")
print(f"device (workgroup 0): obs staged {d[:, 0].mean():.2f} us, forward {d[:, 1].mean():.2f} us, sample + "
      f"actions + done {d[:, 2].mean():.2f} us; done -> next release seen {gap.mean():.2f} us")

