"""A population sharded over gloo ranks equals the single-process population.

train_off_policy with a DQN population of G*P = 4 agents, run in one
process and sharded over 2 and 4 ranks (CPU, gloo).  Every mutation
probability is non-zero; the generation step (tournament over every agent,
mutation draws taken once in the global order, hpo/shard.py) must leave
every global agent with the same index, mutation label, hyperparameters,
fitness history and byte-identical networks and optimizer state as the
single-process run.  Learning is off (``learning_delay`` above the run
length, greedy actions): each rank's own replay is a documented deviation
from the one shared memory, so learned weights are not comparable, while
everything the generation step does is.

Also: the mutation choices of the sharded run are not the per-shard ones
(local agent j of every rank would otherwise get the same choice)."""

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G_TOTAL = 4


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ActionRewardEnv:
    """Reward depends on the action (so agents differ in fitness): +1 when
    the action equals the sign pattern of the first observation entries;
    episodes are truncated every 6 steps."""

    def __init__(self, num_envs=3, obs_dim=6, n_actions=3, seed=0):
        from agilerl_amd.envs import Box, Discrete

        self.num_envs = num_envs
        self.single_observation_space = self.observation_space = Box(-np.inf, np.inf, (obs_dim,))
        self.single_action_space = self.action_space = Discrete(n_actions)
        rng = np.random.default_rng(seed)
        self._obs = rng.standard_normal((11, num_envs, obs_dim)).astype(np.float32)
        self._k = 0
        self._t = 0

    def reset(self, seed=None, options=None):
        self._k, self._t = 0, 0
        return self._obs[0].copy(), {}

    def step(self, actions):
        o = self._obs[self._k]
        target = (o[:, 0] > 0).astype(np.int64) + (o[:, 1] > 0).astype(np.int64)
        rew = (np.asarray(actions).reshape(-1) == target).astype(np.float32)
        self._k = (self._k + 1) % 11
        self._t += 1
        trunc = np.full(self.num_envs, self._t % 6 == 0)
        return self._obs[self._k].copy(), rew, np.zeros(self.num_envs, bool), trunc, {}


def _run(world: int, rank: int, out_dir: str, port: int) -> None:
    sys.path.insert(0, ROOT)
    torch.set_num_threads(1)
    import torch.distributed as dist

    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import random

    from agilerl_amd.components.replay_buffer import ReplayBuffer
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.hpo.registry import HyperparameterConfig, RLParameter
    from agilerl_amd.hpo.sharded import pack_agent
    from agilerl_amd.hpo.tournament import TournamentSelection
    from agilerl_amd.training.train_off_policy import train_off_policy
    from agilerl_amd.utils import create_population

    np.random.seed(0)
    torch.manual_seed(0)
    random.seed(0)
    env = ActionRewardEnv()
    hp = HyperparameterConfig(lr=RLParameter(min=1e-5, max=1e-2), batch_size=RLParameter(min=8, max=64, dtype=int),
                              learn_step=RLParameter(min=1, max=16, dtype=int))
    pop = create_population("DQN", {"head_config": {"hidden_size": [16]}}, {"BATCH_SIZE": 16, "LR": 1e-3},
                            env.observation_space, env.action_space, hp_config=hp, population_size=G_TOTAL,
                            device="cpu")
    # architecture / activation mutations of Q networks apply in single-process
    # runs only (hpo/mutation.py): the sharded run equals the single-process run
    # of the mutations both apply
    mutation = Mutations(no_mutation=0.2, architecture=0.0, new_layer_prob=0.2, parameters=0.4, activation=0.0,
                         rl_hp=0.4, mutation_sd=0.1, rand_seed=5)
    tournament = TournamentSelection(2, True, G_TOTAL, 1)
    memory = ReplayBuffer(500, device="cpu")
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        pop, fits = train_off_policy(env, "ActionReward", "DQN", pop, memory, max_steps=3 * 24, evo_steps=24,
                                     learning_delay=10**9, eps_start=0.0, eps_end=0.0, tournament=tournament,
                                     mutation=mutation, verbose=False)
    out = [dict(index=a.index, mut=a.mut, lr=float(a.lr), batch_size=int(a.batch_size),
                learn_step=int(a.learn_step), fitness=[float(f) for f in a.fitness],
                steps=list(a.steps), state=pack_agent(a, "cpu").clone()) for a in pop]
    torch.save({"agents": out, "fits": fits}, os.path.join(out_dir, f"w{world}_r{rank}.pt"))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _worker(rank, world, out_dir, port):
    _run(world, rank, out_dir, port)


def _launch(world: int, out_dir: str) -> list[dict]:
    mp.start_processes(_worker, args=(world, out_dir, _free_port()), nprocs=world, join=True, start_method="spawn")
    got = [torch.load(os.path.join(out_dir, f"w{world}_r{r}.pt"), weights_only=True) for r in range(world)]
    return [a for g in got for a in g["agents"]], got[0]["fits"]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_train_off_policy_equals_single_process(tmp_path, world):
    ref, ref_fits = _launch(1, str(tmp_path))
    got, fits = _launch(world, str(tmp_path))
    assert len(ref) == len(got) == G_TOTAL
    muts = [a["mut"] for a in ref]
    assert len(set(muts)) > 1, f"the run should mutate agents differently: {muts}"
    assert fits == ref_fits
    for g, (a, b) in enumerate(zip(got, ref)):
        for key in ("index", "mut", "lr", "batch_size", "learn_step", "fitness", "steps"):
            assert a[key] == b[key], (world, g, key, a[key], b[key])
        assert torch.equal(a["state"], b["state"]), (world, g, "network / optimizer bytes")
