"""Cost of the sharded generation step's host-object collectives
(hpo/shard.py all_gather_obj / broadcast_obj: agent records, host RNG states,
fitness, tournament attributes, ...) in tests/test_sharded_generation_gloo.py's
run: train_off_policy, a 4-agent DQN population on 2 gloo ranks, 3
generations.  Prints per tag: calls, ms per generation and pickled KB per
generation that rank 0 contributes (AGX_SHARD_STATS=1)."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

GENERATIONS = 3


def _worker(rank, world, out_dir, port):
    os.environ["AGX_SHARD_STATS"] = "1"
    import test_sharded_generation_gloo as t

    t._run(world, rank, out_dir, port)
    from agilerl_amd.hpo import shard

    with open(os.path.join(out_dir, f"stats_r{rank}.json"), "w") as f:
        json.dump(shard.EXCHANGE_STATS, f)


def main():
    import torch.multiprocessing as mp
    import test_sharded_generation_gloo as t

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, d, t._free_port()), nprocs=world, join=True, start_method="spawn")
        stats = json.load(open(os.path.join(d, "stats_r0.json")))
    out = {"world": world, "population": t.G_TOTAL, "generations": GENERATIONS, "per_generation": {
        k: {"calls": v[0] / GENERATIONS, "ms": round(v[1] / GENERATIONS * 1e3, 3), "kb": round(v[2] / GENERATIONS / 1024, 2)}
        for k, v in sorted(stats.items())}}
    out["total_ms_per_generation"] = round(sum(x["ms"] for x in out["per_generation"].values()), 3)
    out["total_kb_per_generation"] = round(sum(x["kb"] for x in out["per_generation"].values()), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
