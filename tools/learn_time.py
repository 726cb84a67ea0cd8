"""Mean wall time of PPOPopulation.learn() (gather prologue + fused learner)
over repeated calls on one collected rollout (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from agilerl_amd.envs import SyntheticVecEnv  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402
from agilerl_amd.population.runner import PopulationRunner  # noqa: E402

P = int(os.environ.get("P", 8))  # agents (P = 1: one agent per GPU, the 8-GPU strong-scaling shard)
spec = ActorCriticSpec(obs_dim=8, n_actions=4)
pop = PPOPopulation(spec, P, 128, learn_step=2048, batch_size=128, update_epochs=4, device="cuda")
runner = PopulationRunner(pop, SyntheticVecEnv(P * 128))
runner.collect()
pop.finish_rollout(runner.last_obs, runner.last_done, runner.last_value)
for _ in range(3):
    pop.learn()
torch.cuda.synchronize()
n = int(os.environ.get("REPS", 30))
t0 = time.perf_counter()
for _ in range(n):
    pop.learn()
torch.cuda.synchronize()
print(f"P={P}: learn() mean {1e3 * (time.perf_counter() - t0) / n:.3f} ms over {n} calls")
