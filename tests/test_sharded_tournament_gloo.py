"""Sharded generation step for object-level populations (DQN / Rainbow /
MADDPG at configs 3-4 across ranks), on CPU with two gloo ranks.

Each rank holds 3 agents; ShardedTournamentSelection.select must give every
rank exactly the agents the single-process TournamentSelection.select gives
over the concatenated population under the same np.random seed: same
parents, same indices, same fitness/score lists, byte-identical networks,
targets and Adam moments (including agents that never stepped)."""

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P, WORLD = 3, 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make_agent(kind: str, g: int):
    """Global agent g, deterministic in g alone (so both layouts build it)."""
    sys.path.insert(0, ROOT)
    from agilerl_amd.algorithms.dqn import DQN, RainbowDQN
    from agilerl_amd.envs import Box, Discrete

    torch.manual_seed(1000 + g)
    obs, act = Box(-np.inf, np.inf, (5,)), Discrete(3)
    if kind == "dqn":
        a = DQN(obs, act, index=g, batch_size=8, lr=1e-3, device="cpu")
        opt_params = a.actor.parameters()
        opt = a.optimizer
    elif kind == "maddpg":
        from agilerl_amd.algorithms.maddpg import MADDPG
        from agilerl_amd.envs import SyntheticMultiAgentVecEnv

        env = SyntheticMultiAgentVecEnv(4, seed=2)
        a = MADDPG([env.observation_spaces[i] for i in env.agents], [env.action_spaces[i] for i in env.agents],
                   agent_ids=env.agents, index=g, batch_size=8, vect_noise_dim=4, device="cpu")
        a.current_noise[env.agents[0]].normal_()  # exploration state crosses too
        opt_params = a.critics[env.agents[0]].parameters()
        opt = a.critic_optimizers[env.agents[0]]
    else:
        a = RainbowDQN(obs, act, index=g, batch_size=8, lr=1e-3, v_min=-5, v_max=5, num_atoms=11, device="cpu")
        opt_params = a.actor.parameters()
        opt = a.optimizer
    if g % 2 == 0:  # one plain torch step: Adam state exists only for even agents
        loss = sum((p * p).sum() for p in opt_params)
        opt.zero_grad()
        loss.backward()
        opt.step()
    rng = np.random.default_rng(g)
    a.fitness = [float(x) for x in rng.normal(size=3)]
    a.scores = [float(x) for x in rng.normal(size=g + 1)]
    a.steps = [100 * g, 100 * g + 7]
    return a


def _summary(agents):
    from agilerl_amd.hpo.sharded import pack_agent

    return [dict(index=a.index, fitness=list(a.fitness), scores=list(a.scores), steps=list(a.steps),
                 state=pack_agent(a, "cpu").clone()) for a in agents]


def _worker(rank, port, kind, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from agilerl_amd.hpo.sharded import ShardedTournamentSelection, select_population
    from agilerl_amd.hpo.tournament import TournamentSelection

    pop = [_make_agent(kind, rank * P + j) for j in range(P)]
    gen0 = _summary(pop)
    t = TournamentSelection(2, True, P * WORLD, 2)
    np.random.seed(11)
    sel = ShardedTournamentSelection(t)
    elite, new_pop = sel.select(pop)
    np.random.seed(12)
    _, newer = select_population(t, new_pop)  # second generation through the entry-point helper
    torch.save({"gen0": gen0, "gen1": _summary(new_pop), "gen2": _summary(newer), "parents": sel.last_parents,
                "elite": None if elite is None else _summary([elite])},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["dqn", "rainbow", "maddpg"])
def test_sharded_tournament_matches_single_process(tmp_path, kind):
    pytest.importorskip("torch.distributed")
    sys.path.insert(0, ROOT)
    from agilerl_amd.hpo.tournament import TournamentSelection

    port = _free_port()
    mp.start_processes(_worker, args=(port, kind, str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    got = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]

    from agilerl_amd.hpo.sharded import unpack_agent

    # the same agents in one process, carrying the ranks' exact initial bytes
    # (network init may differ in the last bits across processes' thread counts)
    full = [_make_agent(kind, g) for g in range(P * WORLD)]
    for g, a in enumerate(full):
        unpack_agent(a, got[g // P]["gen0"][g % P]["state"])
    t = TournamentSelection(2, True, P * WORLD, 2)
    np.random.seed(11)
    elite, gen1 = t.select(full)
    np.random.seed(12)
    _, gen2 = t.select(gen1)
    assert got[0]["parents"] == got[1]["parents"]
    assert any(q // P != g // P for g, q in enumerate(got[0]["parents"])), "no parent crossed ranks"
    assert got[1]["elite"] is None and got[0]["elite"][0]["index"] == elite.index
    for name, ref in (("gen1", gen1), ("gen2", gen2)):
        exp = _summary(ref)
        for g in range(P * WORLD):
            a, b = got[g // P][name][g % P], exp[g]
            assert a["index"] == b["index"], (name, g)
            assert a["fitness"] == b["fitness"] and a["scores"] == b["scores"] and a["steps"] == b["steps"]
            assert torch.equal(a["state"], b["state"]), (name, g)
