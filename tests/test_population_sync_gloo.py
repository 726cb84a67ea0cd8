"""N > 1 generation step on CPU: two gloo ranks, each holding a shard of the
population, run PopulationSync.generation (fitness all-gather, identical
seeded tournament on every rank, parent weights + Adam state sent point to
point to the ranks that clone them).  Checked against the oracle tournament on the gathered fitness."""

import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank: int, P: int, n: int):
    """Fake pop/runner exposing exactly what PopulationSync touches."""
    g = torch.Generator().manual_seed(100 + rank)
    params = torch.randn(P, n, generator=g)
    opt = types.SimpleNamespace(exp_avg=torch.randn(P, n, generator=g), exp_avg_sq=torch.rand(P, n, generator=g))
    pop = types.SimpleNamespace(P=P, device=torch.device("cpu"), params=torch.nn.Parameter(params), opt=opt)
    ret = torch.randn(P, generator=g).double() * 10
    eps = torch.randint(0, 4, (P,), generator=g)

    class Runner:
        def __init__(self):
            self.episode_return_sum = ret.clone()
            self.episodes = eps.clone()

        def reset_episode_stats(self):
            self.episode_return_sum.zero_()
            self.episodes.zero_()

    return pop, Runner()


def _worker(rank, world, port, P, n, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from agilerl_amd.hpo.population_sync import PopulationSync

    pop, runner = _shard(rank, P, n)
    sync = PopulationSync(pop, runner, world, rank, seed=7, tournament_size=2, elitism=True)
    parents = []
    for _ in range(2):
        parents.append(sync.generation())
    torch.save({"parents": parents, "params": pop.params.data.clone(), "m": pop.opt.exp_avg.clone(),
                "v": pop.opt.exp_avg_sq.clone(), "hist": [torch.as_tensor(h) for h in sync.history]},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 3), (2, 4), (4, 3)])
def test_generation_two_ranks(tmp_path, world, P):
    n = 37
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, P, n, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # every rank drew the same parents
    assert all(res[r]["parents"] == res[0]["parents"] for r in range(world))
    # oracle: same tournament on the gathered fitness with the same RNG stream
    sys.path.insert(0, ROOT)
    from oracle.tournament import select as oracle_select

    shards = [_shard(r, P, n) for r in range(world)]
    full_p = torch.cat([s[0].params.data for s in shards])
    full_m = torch.cat([s[0].opt.exp_avg for s in shards])
    fit = torch.cat([torch.where(s[1].episodes > 0, s[1].episode_return_sum / s[1].episodes.clamp(min=1).double(),
                                 torch.full_like(s[1].episode_return_sum, -1e9)) for s in shards]).numpy()
    rng = np.random.RandomState(7)
    state = np.random.get_state()
    np.random.set_state(rng.get_state())
    _, parents0 = oracle_select([[f] for f in fit], 2, True, 1)
    np.random.set_state(state)
    assert list(res[0]["parents"][0]) == list(parents0)
    # the fitness history follows the lineage: clones inherit their parent's record
    np.testing.assert_array_equal(res[0]["hist"][0].numpy(), fit[list(parents0)][list(res[0]["parents"][1])])
    # each rank's agents after two generations are the rows selected by
    # generation 1 (params and Adam state of the parents), re-selected by
    # generation 2 (fitness of the reset stats is -1e9 everywhere: ties)
    for r in range(world):
        par2 = res[r]["parents"][1]
        # rows after both generations = rows of the first generation's result, permuted by par2
        gen1_p = full_p[parents0]
        gen1_m = full_m[parents0]
        exp_p = gen1_p[par2][r * P:(r + 1) * P]
        exp_m = gen1_m[par2][r * P:(r + 1) * P]
        torch.testing.assert_close(res[r]["params"], exp_p, rtol=0, atol=0)
        torch.testing.assert_close(res[r]["m"], exp_m, rtol=0, atol=0)
