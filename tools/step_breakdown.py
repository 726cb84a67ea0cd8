"""Wall-clock breakdown of one population iteration (collect / GAE / learn)
on the bench configuration (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from agilerl_amd.envs import SyntheticVecEnv  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402
from agilerl_amd.population.runner import PopulationRunner  # noqa: E402

P, N = 8, 128
spec = ActorCriticSpec(obs_dim=8, n_actions=4)
for mode in ("fused", "torch-collect"):
    pop = PPOPopulation(spec, P, N, learn_step=2048, batch_size=128, update_epochs=4, device="cuda")
    runner = PopulationRunner(pop, SyntheticVecEnv(P * N))
    coll = runner.collect if mode == "fused" else runner._collect_torch
    for _ in range(3):
        coll()
        pop.finish_rollout(runner.last_obs, runner.last_done)
        pop.learn()
    torch.cuda.synchronize()
    tc = tg = tl = 0.0
    K = 20
    for _ in range(K):
        t0 = time.perf_counter()
        coll()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        pop.finish_rollout(runner.last_obs, runner.last_done)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pop.learn()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        tc += t1 - t0
        tg += t2 - t1
        tl += t3 - t2
    from agilerl_amd.hpo.population_sync import PopulationSync
    sync = PopulationSync(pop, runner, seed=1)
    sync.generation()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        sync.generation()
    torch.cuda.synchronize()
    print(f"   generation {1e3 * (time.perf_counter() - t0) / 5:.3f} ms")
    print(f"{mode}: collect {1e3 * tc / K:.3f} ms ({1e6 * tc / K / pop.T:.1f} us/step)  "
          f"gae {1e3 * tg / K:.3f} ms  learn {1e3 * tl / K:.3f} ms")
    # per-step sub-phases of the env loop
    env = runner.env
    t_env = 0.0
    for _ in range(200):
        t0 = time.perf_counter()
        runner._env_step()
        t_env += time.perf_counter() - t0
    print(f"   host env step {1e6 * t_env / 200:.1f} us")
    ev = torch.cuda.Event()
    t0 = time.perf_counter()
    for _ in range(200):
        runner.act_h.copy_(runner.act_d, non_blocking=True)
        ev.record()
        ev.synchronize()
    print(f"   D2H + event sync {1e6 * (time.perf_counter() - t0) / 200:.1f} us")
    t0 = time.perf_counter()
    for _ in range(200):
        runner.stage_d.copy_(runner.stage_h, non_blocking=True)
    torch.cuda.synchronize()
    print(f"   H2D issue {1e6 * (time.perf_counter() - t0) / 200:.1f} us")
