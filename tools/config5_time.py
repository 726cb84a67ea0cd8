"""Config 5 (Atari Breakout PPO, ppo_image.yaml network) per-GPU shard:
4 agents x 64 envs of uint8 4x84x84 frames, learn_step 256 (T = 4),
batch 128, 4 epochs.  Times runner.iteration() and its parts:
  python tools/config5_time.py [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from agilerl_amd.envs import SyntheticAtariVecEnv, StackedVecEnv  # noqa: E402
from agilerl_amd.population.runner import PopulationRunner  # noqa: E402
from agilerl_amd.utils import create_population  # noqa: E402

P, N = int(os.environ.get("C5_P", "4")), int(os.environ.get("C5_N", "64"))
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
INIT_HP = {"BATCH_SIZE": 128, "LR": 1e-3, "LEARN_STEP": int(os.environ.get("C5_LEARN", "256")), "UPDATE_EPOCHS": 4}
net_config = {"latent_dim": 256,
              "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
              "head_config": {"hidden_size": [256], "layer_norm": False}}
env = SyntheticAtariVecEnv(N, n_actions=4, seed=1)
pop = create_population("PPO", net_config, INIT_HP, env.single_observation_space, env.single_action_space,
                        population_size=P, num_envs=N)
population = pop[0].population
runner = PopulationRunner(population, StackedVecEnv.from_shared(env, P))
np.random.seed(0)
for _ in range(2):
    runner.iteration()
torch.cuda.synchronize()
tc = tl = 0.0
t0 = time.perf_counter()
for _ in range(iters):
    a = time.perf_counter()
    runner.collect()
    population.finish_rollout(runner.last_obs, runner.last_done, None)
    torch.cuda.synchronize()
    b = time.perf_counter()
    population.learn()
    torch.cuda.synchronize()
    c = time.perf_counter()
    tc += b - a
    tl += c - b
dt = time.perf_counter() - t0
steps = P * N * population.T * iters
print(f"P={P} N={N} T={population.T}: {dt / iters * 1e3:.2f} ms/iter (collect+GAE {tc / iters * 1e3:.2f}, "
      f"learn {tl / iters * 1e3:.2f}), {steps / dt:.0f} env-steps/s, "
      f"{population.n_updates() * iters / dt:.0f} updates/s")
