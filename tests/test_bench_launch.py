"""bench.py --gpus N: the N-rank launch the driver's scaling run relies on.

``python bench.py --gpus 2`` with no launcher around it must start two ranks
itself (one child torch.distributed.run, before any GPU call), and the JSON
line must report the world size it actually ran at.  Exercised on CPU with
gloo through ``--dist-selftest`` (same launch, barrier and max-over-ranks
path as the GPU run)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dist-selftest", "--steps", "3",
                          "--warmup", "1", *extra], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    line = _run("--gpus", "2")
    assert line["n_gpus"] == 2 and line["steps"] == 3


def test_bench_single_rank_default():
    line = _run()
    assert line["n_gpus"] == 1


def test_bench_reads_the_roofline_pmc_summary():
    """bench.py's roofline.traffic comes from the newest profiles/rN_pmc_traffic.json
    (not another kernel's rN_*_pmc_traffic.json)."""
    import bench

    pmc = bench.load_pmc_traffic()
    assert pmc is not None and "gae_bytes" in pmc and "loss_bytes" in pmc, pmc
