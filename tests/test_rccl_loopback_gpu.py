"""The device-tensor collective path of the generation step under RCCL.

Every multi-rank test runs gloo (host-staged rows); the one-GPU box cannot
host two RCCL ranks on one device.  PopulationSync's loopback mode runs the
MULTI-RANK exchange in a one-rank NCCL (= RCCL) group: the fitness
all-gather is an ``all_gather_into_tensor`` of device tensors and every
parent row is packed on the device, sent to this rank and received through
``batch_isend_irecv`` (RCCL send / recv to self), then unpacked — the same
pack / P2P / unpack code the ranks of an 8-GPU node run.  The result must
equal the plain row gather, bit for bit."""

import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, out_path):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    import torch.distributed as dist

    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from agilerl_amd.hpo.population_sync import PopulationSync
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation

    pop = PPOPopulation(ActorCriticSpec(obs_dim=8, n_actions=4), 4, 16, learn_step=64, batch_size=16,
                        update_epochs=1, device=torch.device("cuda"))
    g = torch.Generator(device="cuda").manual_seed(3)
    with torch.no_grad():
        pop.params.data.copy_(torch.randn(pop.params.shape, device="cuda", generator=g))
        pop.opt.exp_avg.copy_(torch.randn(pop.opt.exp_avg.shape, device="cuda", generator=g))
        pop.opt.exp_avg_sq.copy_(torch.rand(pop.opt.exp_avg_sq.shape, device="cuda", generator=g))
        pop.opt.steps.copy_(torch.tensor([5, 6, 7, 8], device=pop.opt.steps.device))
    sync = PopulationSync(pop, None, world=1, rank=0, seed=1)
    sync.loopback = True
    before = [b.clone() for b in sync._row_buffers()]
    parents = [2, 2, 0, 3]
    sync._clone_rows(parents)
    torch.cuda.synchronize()
    after = sync._row_buffers()
    ok = all(torch.equal(a, b[parents]) for a, b in zip(after, before))
    x = torch.arange(4, dtype=torch.float64, device="cuda") * 1.5
    gathered = sync._all_gather(x)
    torch.cuda.synchronize()
    torch.save({"rows_ok": ok, "gather_ok": bool(torch.equal(gathered, x)), "backend": dist.get_backend(),
                "n_buffers": len(after)}, out_path)
    dist.destroy_process_group()


def test_generation_exchange_over_rccl_loopback(tmp_path):
    out = str(tmp_path / "loopback.pt")
    mp.start_processes(_worker, args=(_free_port(), out), nprocs=1, join=True, start_method="spawn")
    r = torch.load(out, weights_only=True)
    assert r["backend"] == "nccl"
    assert r["n_buffers"] >= 4  # params, both Adam moments, the step count (+ lr / hyperparameters)
    assert r["rows_ok"] and r["gather_ok"], r
