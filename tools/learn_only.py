"""Runs the fused learner a few times on a collected rollout (for rocprofv3
--pmc passes on ppo_learn_kernel; diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from agilerl_amd.envs import SyntheticVecEnv  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402
from agilerl_amd.population.runner import PopulationRunner  # noqa: E402

spec = ActorCriticSpec(obs_dim=8, n_actions=4)
pop = PPOPopulation(spec, 8, 128, learn_step=2048, batch_size=128, update_epochs=4, device="cuda")
runner = PopulationRunner(pop, SyntheticVecEnv(8 * 128))
runner.collect()
pop.finish_rollout(runner.last_obs, runner.last_done, runner.last_value)
for _ in range(3):
    pop.learn()
torch.cuda.synchronize()
print("ok")
