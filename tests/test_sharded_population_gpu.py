"""A PPO population sharded over ranks trains exactly like the unsharded one.

train_on_policy with a 4-agent population, run in one process and as 2
ranks x 2 agents (gloo, both ranks on cuda:0 — the one-GPU box; on a
multi-GPU node the same test runs one rank per device).  With mutations
(parameters, RL hyperparameters incl. per-agent batch / epochs / entropy /
lr) and a tournament, every global agent must end with bit-identical
parameters and Adam moments, the same index, mutation label,
hyperparameters and fitness history: each agent samples its global env's
Philox stream, learns from its global shuffles of the numpy stream, and the
generation step is drawn once over the global population."""

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G_TOTAL = 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ActionRewardVecEnv:
    """LunarLander-shaped (obs 8, 4 actions); the reward depends on the
    action, episodes are truncated every 9 steps.  ``reseed`` gives a copy
    its own stream (StackedVecEnv.from_shared).  Host-only steps: the
    population paces persistent rollouts on it (both ranks' rollout kernels
    resident on the one card at once)."""

    agx_device_free = True

    def __init__(self, num_envs=16, seed=0):
        from agilerl_amd.envs import Box, Discrete

        self.num_envs = num_envs
        self.single_observation_space = self.observation_space = Box(-np.inf, np.inf, (8,))
        self.single_action_space = self.action_space = Discrete(4)
        self.seed = seed
        self.reseed(seed)

    def reseed(self, seed):
        self._obs = np.random.default_rng(seed).standard_normal((13, self.num_envs, 8)).astype(np.float32)
        self._k, self._t = 0, 0

    def reset(self, seed=None, options=None):
        self._k, self._t = 0, 0
        return self._obs[0].copy(), {}

    def step(self, actions):
        o = self._obs[self._k]
        target = (o[:, 0] > 0).astype(np.int64) * 2 + (o[:, 1] > 0).astype(np.int64)
        rew = (np.asarray(actions).reshape(-1) == target).astype(np.float32) - 0.25
        self._k = (self._k + 1) % 13
        self._t += 1
        trunc = np.full(self.num_envs, self._t % 9 == 0)
        return self._obs[self._k].copy(), rew, np.zeros(self.num_envs, bool), trunc, {}


def _run(world, rank, out_dir, port, arch=0.0):
    sys.path.insert(0, ROOT)
    torch.cuda.set_device(0)
    import random
    import warnings

    import torch.distributed as dist

    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.hpo.registry import HyperparameterConfig, RLParameter
    from agilerl_amd.hpo.tournament import TournamentSelection
    from agilerl_amd.training.train_on_policy import train_on_policy
    from agilerl_amd.utils import create_population

    np.random.seed(0)
    torch.manual_seed(0)
    random.seed(0)
    env = ActionRewardVecEnv()
    hp = HyperparameterConfig(lr=RLParameter(min=1e-5, max=1e-2), batch_size=RLParameter(min=8, max=64, dtype=int),
                              update_epochs=RLParameter(min=1, max=4, dtype=int),
                              ent_coef=RLParameter(min=1e-4, max=0.1),
                              **({"learn_step": RLParameter(min=32, max=256, dtype=int)} if arch else {}))
    net = {"encoder_config": {"hidden_size": [64], "min_mlp_nodes": 32, "max_mlp_nodes": 128},
           "head_config": {"hidden_size": [64], "min_mlp_nodes": 32, "max_mlp_nodes": 128}, "latent_dim": 64}
    init = {"BATCH_SIZE": 16, "LR": 1e-3, "LEARN_STEP": 64, "UPDATE_EPOCHS": 2}
    pop = create_population("PPO", net, init, env.observation_space, env.action_space, hp_config=hp,
                            population_size=G_TOTAL, num_envs=env.num_envs, device="cuda")
    mutation = Mutations(no_mutation=0.2, architecture=arch, new_layer_prob=0.2, parameters=0.4, activation=0.0,
                         rl_hp=0.4, mutation_sd=0.1, rand_seed=5)
    tournament = TournamentSelection(2, True, G_TOTAL, 1)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        pop, fits = train_on_policy(env, "ActionReward", "PPO", pop, max_steps=(4 if arch else 3) * 128, evo_steps=128,
                                    tournament=tournament, mutation=mutation, verbose=False)
    torch.cuda.synchronize()
    population = pop[0].population
    out = [dict(index=a.index, mut=a.mut, lr=float(a.lr), batch_size=int(a.batch_size),
                update_epochs=int(a.update_epochs), ent_coef=float(a.ent_coef), learn_step=int(a.learn_step),
                shape=repr(a.spec.shape_key()), fitness=[float(f) for f in a.fitness], steps=list(a.steps),
                params=a.population.params.data[a.row].cpu().clone(),
                exp_avg=a.population.opt.exp_avg[a.row].cpu().clone(),
                exp_avg_sq=a.population.opt.exp_avg_sq[a.row].cpu().clone()) for a in pop]
    torch.save({"agents": out, "fits": fits}, os.path.join(out_dir, f"w{world}_r{rank}.pt"))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _worker(rank, world, out_dir, port, arch):
    _run(world, rank, out_dir, port, arch)


def _launch(world, out_dir, arch=0.0):
    mp.start_processes(_worker, args=(world, out_dir, _free_port(), arch), nprocs=world, join=True,
                       start_method="spawn")
    got = [torch.load(os.path.join(out_dir, f"w{world}_r{r}.pt"), weights_only=True) for r in range(world)]
    return [a for g in got for a in g["agents"]], got[0]["fits"]


@pytest.mark.parametrize("arch", [0.0, 0.4])
def test_sharded_train_on_policy_equals_single_process(tmp_path, arch):
    """arch > 0: architecture and learn_step mutations too — agents with
    different networks and rollout lengths, in groups on each rank."""
    ref, ref_fits = _launch(1, str(tmp_path), arch)
    got, fits = _launch(2, str(tmp_path), arch)
    assert len(ref) == len(got) == G_TOTAL
    assert len({a["mut"] for a in ref}) > 1, [a["mut"] for a in ref]
    if arch:
        assert len({a["shape"] for a in ref}) > 1 or len({a["learn_step"] for a in ref}) > 1
    assert fits == ref_fits
    for g, (a, b) in enumerate(zip(got, ref)):
        for key in ("index", "mut", "lr", "batch_size", "update_epochs", "ent_coef", "learn_step", "shape", "fitness",
                    "steps"):
            assert a[key] == b[key], (g, key, a[key], b[key])
        for key in ("params", "exp_avg", "exp_avg_sq"):
            assert torch.equal(a[key], b[key]), (g, key, float((a[key] - b[key]).abs().max()))
