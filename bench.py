"""Benchmark: population env-steps/s (+ learner updates/s) of an 8-agent PPO
population (config 2: LunarLander-shaped, 128 vec envs per agent, T=16,
B=128, E=4), plus the GAE + clipped-loss kernel roofline at the SURVEY §8d
synthetic shape, plus the reference-style CPU baseline.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: launched by torch.distributed.run, one rank per GPU over RCCL)

A "step" = one PPO iteration of the population: T vector steps of rollout
for every agent (host env + HBM rollout SoA), bootstrap + GAE, and E x M
minibatch learner updates per agent.  The headline is the north-star's
configuration, strong scaling: ONE 8-agent population (--pop, global) sharded
P = 8 / N agents per GPU; ranks exchange only fitness scalars (RCCL
all-gather) and the selected parents' parameters at generation boundaries
(--evo-every).  With N > 1 a weak-scaling leg (--pop-per-gpu agents on
every GPU, a shard of an N x 8 population) is reported as an extra key.
"""

from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import agilerl_amd  # noqa: E402,F401  (before the HIP runtime starts: hardware queues, agilerl_amd/__init__.py)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GAE_BYTES = 17          # per transition   
LOSS_BYTES = 40         # per sample·epoch
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md, chip-level parameters (spec)
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense peak (spec)


def log(msg: str) -> None:
    """Progress on stderr (stdout carries only the one JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pop", type=int, default=8, help="agents in the whole population (sharded over the GPUs)")
    ap.add_argument("--pop-per-gpu", type=int, default=8, help="agents per GPU of the extra weak-scaling leg (N > 1)")
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling leg")
    ap.add_argument("--num-envs", type=int, default=128)
    ap.add_argument("--learn-step", type=int, default=2048)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--evo-every", type=int, default=5, help="iterations per generation (0: never)")
    ap.add_argument("--learner", choices=["fused", "torch"], default="fused")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 (Atari PPO) side measurement")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 (Atari Rainbow) learner measurement")
    ap.add_argument("--no-train-on-policy", action="store_true",
                    help="skip the end-to-end train_on_policy (ppo.yaml generations) measurement")
    ap.add_argument("--roof-reps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--dist-selftest", action="store_true",
                    help="no GPU: gloo ranks run a trivial CPU step through the same launch, barrier and "
                         "max-over-ranks timing (tests/test_bench_launch.py)")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """``--gpus N`` (N > 1) without a torch.distributed launcher around us:
    start N ranks as ONE child ``torch.distributed.run`` before this process
    touches the GPU (no exec from a GPU-initialised process), relay its output
    (rank 0 prints the JSON line) and return its exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# --------------------------------------------------------------------------- #
def setup_dist(gpu: bool = True):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpu:
        torch.cuda.set_device(local)
    if world > 1:
        if gpu:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def dist_selftest(args, world, rank):
    """The launch / barrier / max-over-ranks skeleton of main() on CPU ranks."""
    x = torch.randn(256, 256)
    for _ in range(args.warmup):
        x = torch.tanh(x @ x.T * 1e-3)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = torch.tanh(x @ x.T * 1e-3)
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    if rank == 0:
        print(json.dumps({"metric": "dist selftest steps/s", "value": round(world * args.steps / dt, 1),
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(dt / args.steps * 1e3, 3), "selftest": True}))


# --------------------------------------------------------------------------- #
def population_leg(args, world, rank, P, steps=None):
    """P agents on this rank, global agents rank*P .. of a world*P population."""
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.hpo.population_sync import PopulationSync
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation
    from agilerl_amd.population.runner import PopulationRunner

    spec = ActorCriticSpec(obs_dim=8, n_actions=4, encoder_hidden=[64], latent_dim=64,
                           actor_hidden=[64], critic_hidden=[64])
    N = args.num_envs
    steps = args.steps if steps is None else steps
    seeds = [rank * P + i for i in range(P)]
    pop = PPOPopulation(spec, P, N, learn_step=args.learn_step, batch_size=args.batch_size, lr=1e-3,
                        update_epochs=args.epochs, seeds=seeds, device="cuda",
                        fused=args.learner == "fused", agent_offset=rank * P, global_pop_size=world * P,
                        seed_base=0)
    env = SyntheticVecEnv(P * N, seed=1000 + rank)
    runner = PopulationRunner(pop, env)
    sync = PopulationSync(pop, runner, world, rank, seed=42) if args.evo_every > 0 else None

    def step(i):
        runner.iteration()
        if sync is not None and (i + 1) % args.evo_every == 0:
            sync.generation()

    for i in range(args.warmup):
        runner.iteration()
    if sync is not None:  # first generation outside the timed region (loads its kernels)
        sync.generation()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0, world)
    pop.check_errors()  # a partner timeout in any timed learn() fails the run loudly
    env_steps = world * P * pop.S * steps
    updates = world * P * args.epochs * pop.n_minibatches() * steps
    # the dominant kernel alone: learn() (gather prologue + fused learner) on the
    # last rollout, HIP events on the launch stream
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pop.learn(prefetch=False)
    e1.record()
    torch.cuda.synchronize()
    pop.check_errors()
    learn_s = e0.elapsed_time(e1) * 1e-3 / reps
    flop = 79e3 * P * pop.S * args.epochs  # ~79 kFLOP per sample and update (fwd + bwd)
    learner = dict(kernel="agx_ppo_learn (gather prologue + ppo_learn_kernel)", ms_per_learn=round(learn_s * 1e3, 3),
                   updates_per_learn=P * args.epochs * pop.n_minibatches(),
                   us_per_update=round(learn_s * 1e6 / (args.epochs * pop.n_minibatches()), 2),
                   achieved_tflops=round(flop / learn_s / 1e12, 2), peak_tflops=F32_MFMA_PEAK_TFLOPS,
                   frac=round(flop / learn_s / 1e12 / F32_MFMA_PEAK_TFLOPS, 4),
                   bound="latency: 64 serial minibatch updates per agent, each a chain of barrier-separated "
                         "small GEMM / row phases and a 3-barrier partner hand-off (DESIGN §5)")
    out = dict(dt=dt, env_steps=env_steps, updates=updates, S=pop.S, T=pop.T, learner=learner,
               generations=(steps // args.evo_every) if args.evo_every else 0)
    del runner, pop, sync
    torch.cuda.empty_cache()
    return out


# --------------------------------------------------------------------------- #
def measure_hbm_peak():
    """STREAM-style probes (agx_debug_stream, 16 B/lane, one 16 KiB tile per
    block) over 1 GiB buffers — 4x the 256 MiB Infinity Cache — timed with HIP
    events on the launch stream: (copy GB/s counting read + write, read GB/s)."""
    from agilerl_amd import _lib

    nbytes = 1 << 30
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda").uniform_()
    b = torch.empty_like(a)
    lib = _lib.load()
    out = []
    for mode in (0, 1):
        def run():
            _lib.check(lib.agx_debug_stream(a.data_ptr(), b.data_ptr(), nbytes, mode, 0, _lib.stream()),
                       "agx_debug_stream")

        for _ in range(3):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        s.record()
        for _ in range(reps):
            run()
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / reps
        out.append((2 if mode == 0 else 1) * nbytes / (ms * 1e-3) / 1e9)
    del a, b
    torch.cuda.empty_cache()
    return out[0], out[1]


ROOF_P, ROOF_T, ROOF_N, ROOF_E, ROOF_B = 8, 1024, 8192, 4, 128


def roofline_workload():
    """Inputs of SURVEY §8d (GAE P=8 T=1024 N=8192; loss over the same 67.1 M
    samples, b = 128) -> (run_gae, run_loss, S).  Shared with
    tools/pmc_roofline.py (the rocprofv3 --pmc pass)."""
    from agilerl_amd import kernels as K

    P, T, N, b = ROOF_P, ROOF_T, ROOF_N, ROOF_B
    S = P * T * N
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    r = torch.randn(P, T, N, device=dev, generator=g)
    v = torch.randn(P, T, N, device=dev, generator=g)
    d = (torch.rand(P, T, N, device=dev, generator=g) < 0.01).to(torch.uint8)
    lv = torch.randn(P, N, device=dev, generator=g)
    ld = (torch.rand(P, N, device=dev, generator=g) < 0.01).to(torch.uint8)
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    stats = torch.empty(P, 2, dtype=torch.float64, device=dev)
    ws = torch.empty(max(16, K._lib.load().agx_gae_workspace_bytes(P, T, N)), dtype=torch.uint8, device=dev)
    g1 = torch.Generator(device=dev).manual_seed(1)
    old_logp = torch.rand(S, device=dev, generator=g1) * -2.95 - 0.05
    logp = old_logp + 0.05 * torch.randn(S, device=dev, generator=g1)
    newv = v.view(-1) + 0.1 * torch.randn(S, device=dev, generator=g1)
    H = torch.rand(S, device=dev, generator=g1) * float(np.log(4))
    out = tuple(torch.empty(S, device=dev) for _ in range(3))
    lstats = torch.empty(S // b, 8, device=dev)

    def run_gae():
        K.gae(r, d, v, lv, ld, 0.99, 0.95, True, advantages=adv, returns=ret, with_stats=True,
              workspace=ws, stats_out=stats)

    def run_loss():
        K.ppo_loss_fwd_bwd(logp, old_logp, adv.view(-1), ret.view(-1), v.view(-1), newv, H, b, 0.2, 0.5,
                           0.01, out=out, stats=lstats)

    return run_gae, run_loss, S


def load_pmc_traffic():
    """Per-launch HBM bytes of the roofline kernels from the committed
    rocprofv3 --pmc summary (tools/pmc_roofline.py), or None."""
    import glob

    import re

    paths = [q for q in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json"))
             if re.fullmatch(r"r\d+_pmc_traffic\.json", os.path.basename(q))]  # not r2_c51_pmc_traffic.json
    paths.sort(key=lambda q: int(os.path.basename(q)[1:].split("_")[0]))
    if not paths:
        return None
    with open(paths[-1]) as f:
        out = json.load(f)
    out["_source"] = "profiles/" + os.path.basename(paths[-1])
    return out


def roofline_leg(args):
    """GAE + E=4 passes of the loss fwd+bwd, timed per kernel with HIP events
    on the launch stream (torch's current stream: libagx launches there)."""
    E = ROOF_E
    run_gae, run_loss, S = roofline_workload()
    for _ in range(2):
        run_gae()
        run_loss()
    torch.cuda.synchronize()
    t_gae, t_loss = [], []
    for _ in range(args.roof_reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run_gae()
        e1.record()
        evs = []
        for _ in range(E):
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record()
            run_loss()
            a1.record()
            evs.append((a0, a1))
        torch.cuda.synchronize()
        t_gae.append(e0.elapsed_time(e1) * 1e-3)
        t_loss += [x.elapsed_time(y) * 1e-3 for x, y in evs]
    tg = float(np.mean(t_gae))
    tl = float(np.mean(t_loss))
    peak_copy, peak_read = measure_hbm_peak()
    peak_meas = max(peak_copy, peak_read)
    fused_bytes = (GAE_BYTES + E * LOSS_BYTES) * S
    fused_t = tg + E * tl
    ach = fused_bytes / fused_t / 1e9
    res = dict(
        bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
        frac=round(ach / HBM_PEAK_GBS, 4), traffic=None,
        kernel="agx_gae + 4 x agx_ppo_loss_fwd_bwd (GAE+loss, E=4)",
        units="transitions P=8 T=1024 N=8192 (67.1M), 177 B each (17 GAE + 4x40 loss)",
        gae_ms=round(tg * 1e3, 3), loss_ms=round(tl * 1e3, 3),
        gae_gbs=round(GAE_BYTES * S / tg / 1e9, 1), loss_gbs=round(LOSS_BYTES * S / tl / 1e9, 1),
        peak_measured_copy=round(peak_copy, 1), peak_measured_read=round(peak_read, 1),
        peak_measured=round(peak_meas, 1), frac_of_measured=round(ach / peak_meas, 4),
    )
    pmc = load_pmc_traffic()
    if pmc is not None:  # FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE, per launch set (1 GAE + E loss)
        res["traffic"] = pmc["gae_bytes"] + E * pmc["loss_bytes"]
        res["traffic_source"] = pmc["_source"] + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"
        res["algorithmic_bytes"] = fused_bytes
    del run_gae, run_loss
    torch.cuda.empty_cache()
    return res


# --------------------------------------------------------------------------- #
def _time(fn, reps=5):
    """Mean HIP-event time (s) of fn on the current (launch) stream."""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / reps


def _time_graph(fn, reps=20):
    """Mean time (s) of one fn call replayed from a HIP graph of ``reps``
    captured calls: the kernels back to back on the stream, without the
    Python / ctypes launch cost that dominates an eager loop of these
    microsecond-scale entry points (torch.cuda.CUDAGraph is hipGraph here)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    graph.replay()
    e.record()
    e.synchronize()
    del graph
    return s.elapsed_time(e) * 1e-3 / reps


def _both(fn):
    """(graph-replayed time, eager time) of fn."""
    return _time_graph(fn), _time(fn)


def kernels_leg(peak_meas):
    """Config-3 kernels at the SURVEY §8d synthetic shapes, algorithmic
    bytes / HIP-event time: PER retrieve (+ IS weights) over a 2^20-leaf tree
    with 2^20 uniforms, PER priority update of 2^16 indices (duplicates),
    C51 projection + loss over 2^20 rows (A=6, Z=51), DQN TD target + loss
    gradient over 2^20 rows (A=6).  The microsecond-scale entry points are
    timed replayed from a HIP graph (``ms``) and as an eager Python loop
    (``ms_eager``, launch-cost inclusive); rates use ``ms``."""
    from agilerl_amd import kernels as K

    dev = "cuda"
    out = {}
    g = torch.Generator(device=dev).manual_seed(2)
    cap, max_size = 1 << 20, 1_000_000
    st = torch.empty(2 * cap, dtype=torch.float64, device=dev)
    mt = torch.empty_like(st)
    K.per_init(st, mt, cap)
    maxp = torch.ones(1, dtype=torch.float64, device=dev)
    ws = K.per_workspace(cap, dev)
    K.per_add(st, mt, cap, max_size, 0, max_size, 0.6, maxp, workspace=ws)
    allidx = torch.arange(max_size, device=dev)
    pri = torch.randn(max_size, device=dev, generator=g).abs() + 1e-5
    K.per_update(st, mt, cap, max_size, allidx, pri, 0.6, maxp, workspace=ws)
    u = torch.rand(1 << 20, device=dev, generator=g)
    t, te = _both(lambda: K.per_sample(st, mt, cap, u, size=max_size, beta=0.4, weights=True))
    nb = (8 * 20 + 4 + 8 + 8 + 4) * u.numel()  # walk + uniform + index + leaf + weight
    # the 16 MiB sum tree is re-walked 2^20 times and stays cache resident (LDS
    # top levels, L2 / Infinity Cache): the walk's algorithmic bytes are not HBM
    # traffic, so no HBM fraction is claimed for it
    out["per_sample"] = dict(unit_bytes=nb // u.numel(), units=u.numel(), ms=round(t * 1e3, 4),
                             ms_eager=round(te * 1e3, 4),
                             samples_per_s=round(u.numel() / t, 1), walk_gbs=round(nb / t / 1e9, 1),
                             frac_of_measured=None,
                             bound="latency (dependent 20-level walk over a cache-resident 16 MiB tree)")
    idx = torch.randint(0, max_size, (1 << 16,), device=dev, generator=g)
    p2 = torch.rand(1 << 16, device=dev, generator=g)
    t, te = _both(lambda: K.per_update(st, mt, cap, max_size, idx, p2, 0.6, maxp, workspace=ws))
    nb = 976 * idx.numel()
    out["per_update"] = dict(unit_bytes=976, units=idx.numel(), ms=round(t * 1e3, 4), ms_eager=round(te * 1e3, 4),
                             gbs=round(nb / t / 1e9, 1),
                             frac_of_measured=round(nb / t / 1e9 / peak_meas, 4),
                             bound="launch latency (leaf claim + band rebuild)")
    del st, mt, ws, allidx, pri
    B, A, Z = 1 << 20, 6, 51
    g3 = torch.Generator(device=dev).manual_seed(3)
    qn = torch.randn(B, A, device=dev, generator=g3)
    td = torch.softmax(torch.randn(B, A, Z, device=dev, generator=g3), -1).clamp_(min=1e-3)
    lp = torch.log_softmax(torch.randn(B, A, Z, device=dev, generator=g3), -1)
    act = torch.randint(0, A, (B,), device=dev, generator=g3)
    r = torch.randn(B, device=dev, generator=g3)
    d = (torch.rand(B, device=dev, generator=g3) < 0.05).float()
    sup = torch.linspace(-200, 200, Z, device=dev)
    t, te = _both(lambda: K.c51_project_loss(qn, td, lp, act, r, d, sup, -200.0, 200.0, 0.99 ** 4))
    nb = 444 * B
    out["c51_project_loss"] = dict(unit_bytes=444, units=B, ms=round(t * 1e3, 4), ms_eager=round(te * 1e3, 4),
                                   gbs=round(nb / t / 1e9, 1),
                                   frac_of_measured=round(nb / t / 1e9 / peak_meas, 4), bound="hbm")
    # the selected-rows form (the heads emit target_dist[b, a*] and log p[b, a]
    # as two contiguous [B][Z] arrays): 204 + 204 + r, d in, loss out
    tr = td[torch.arange(B, device=dev), qn.argmax(1)].contiguous()
    lr_ = lp[torch.arange(B, device=dev), act].contiguous()
    del td, lp
    t, te = _both(lambda: K.c51_project_loss_rows(tr, lr_, r, d, sup, -200.0, 200.0, 0.99 ** 4))
    ub = 2 * 4 * Z + 4 + 4 + 4
    nb = ub * B
    out["c51_project_loss_rows"] = dict(unit_bytes=ub, units=B, ms=round(t * 1e3, 4), ms_eager=round(te * 1e3, 4),
                                        gbs=round(nb / t / 1e9, 1),
                                        frac_of_measured=round(nb / t / 1e9 / peak_meas, 4), bound="hbm")
    del tr, lr_
    qt = torch.randn(B, A, device=dev, generator=g3)
    qc = torch.randn(B, A, device=dev, generator=g3)
    t, te = _both(lambda: K.td_target(qt, r, d, 0.99, q_next_online=qn, double=True, q_cur=qc, actions=act))
    ub = 3 * 4 * A + 8 + 4 + 4 + 4 + 4 * A  # Q(s'), Qt(s'), Q(s) rows, a, r, d in; y, dL/dQ out
    nb = ub * B
    out["td_target"] = dict(unit_bytes=ub, units=B, ms=round(t * 1e3, 4), ms_eager=round(te * 1e3, 4),
                            gbs=round(nb / t / 1e9, 1),
                            frac_of_measured=round(nb / t / 1e9 / peak_meas, 4), bound="hbm")
    # MADDPG critic target (a22): q, q', r, d in; y, dL/dq out
    q1, qn1 = qc[:, 0].contiguous(), qt[:, 0].contiguous()
    t, te = _both(lambda: K.maddpg_critic_target(q1, qn1, r, d, 0.95))
    nb = 24 * B
    out["maddpg_critic_target"] = dict(unit_bytes=24, units=B, ms=round(t * 1e3, 4), ms_eager=round(te * 1e3, 4),
                                       gbs=round(nb / t / 1e9, 1),
                                       frac_of_measured=round(nb / t / 1e9 / peak_meas, 4), bound="hbm")
    del qn, qt, qc, q1, qn1
    # Polyak (a10) and clip + Adam (a8) over a population of flat parameter
    # rows: 8 agents x 2^22 parameters (large enough to leave the launch floor)
    # 4 rotating (target, online) pairs of 8 x 2^24 floats (1 GiB per pair): no
    # repetition finds its working set in the 256 MiB Infinity Cache
    n8 = 8 << 24
    pairs = [(torch.randn(n8, device=dev, generator=g3), torch.randn(n8, device=dev, generator=g3))
             for _ in range(4)]
    rot = {"i": 0}

    def polyak_rot():
        tg, on = pairs[rot["i"] % 4]
        rot["i"] += 1
        K.polyak_(tg, on, 0.005)

    t = _time(polyak_rot, reps=8)
    nb = 12 * n8  # read target, online; write target
    out["polyak"] = dict(unit_bytes=12, units=n8, ms=round(t * 1e3, 4), gbs=round(nb / t / 1e9, 1),
                         frac_of_measured=round(nb / t / 1e9 / peak_meas, 4), bound="hbm")
    del pairs
    prm = torch.randn(8, 1 << 22, device=dev, generator=g3)
    opt = K.ClipAdam(prm, [0, 1 << 21, 1 << 22], lr=1e-3, max_norm=0.5,
                     grads=torch.randn(8, 1 << 22, device=dev, generator=g3))
    t = _time(opt.step)
    nb = 32 * prm.numel()  # norm pass reads g; Adam reads p, g, m, v, writes p, m, v
    out["clip_adam"] = dict(unit_bytes=32, units=prm.numel(), ms=round(t * 1e3, 4), gbs=round(nb / t / 1e9, 1),
                            frac_of_measured=round(nb / t / 1e9 / peak_meas, 4), bound="hbm")
    del prm, opt
    torch.cuda.empty_cache()
    return out


# --------------------------------------------------------------------------- #
def cpu_baseline_leg(args, S_per_agent):
    """The reference-style CPU PPO iteration (oracle/ppo_cpu.py), one agent at a
    time like train_on_policy.py:210, on a bounded sample: whole agent
    iterations until --cpu-seconds elapse (at least one)."""
    from agilerl_amd.envs import SyntheticVecEnv
    from oracle.ppo_cpu import CpuPPOAgent

    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    agent = CpuPPOAgent(num_envs=args.num_envs, learn_step=args.learn_step, batch_size=args.batch_size,
                        update_epochs=args.epochs)
    env = SyntheticVecEnv(args.num_envs, seed=7)
    t0 = time.perf_counter()
    n = 0
    steps = 0
    while True:
        steps += agent.iteration(env)
        n += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    torch.set_num_threads(threads)
    return dict(value=round(steps / dt, 1), unit="env-steps/s", cores=1, kind="port",
                sample=f"{n} single-agent PPO iterations (T={agent.T}, N={args.num_envs}, "
                       f"E={args.epochs}, B={args.batch_size}) of oracle/ppo_cpu.py on 1 host thread "
                       f"({os.cpu_count()} CPUs visible), {dt:.1f}s; reference trains agents sequentially, "
                       f"so population env-steps/s = per-agent rate")


def _cpu_threads() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_agent_worker(cfg, seconds, seed, q):
    """One single-threaded CPU PPO agent (oracle/ppo_cpu.py) in its own
    process: (env-steps, seconds) of whole iterations until ``seconds``."""
    torch.set_num_threads(1)
    from agilerl_amd.envs import SyntheticVecEnv
    from oracle.ppo_cpu import CpuPPOAgent

    agent = CpuPPOAgent(**cfg)
    env = SyntheticVecEnv(cfg["num_envs"], seed=seed)
    agent.iteration(env)  # warm-up
    t0, steps = time.perf_counter(), 0
    while True:
        steps += agent.iteration(env)
        if time.perf_counter() - t0 >= seconds:
            break
    q.put((steps, time.perf_counter() - t0))


def cpu_population_all_cores(args, seconds, P: int = 8):
    """The population on every host core the box gives this job: P agents as
    P single-threaded processes of the CPU PPO port side by side (the
    reference's agents are independent between generations), summed
    env-steps/s.  (Torch intra-op threads on one agent's tiny ops were slower
    than one thread: round-3 VERDICT.)  Processes are started with
    ``spawn`` before nothing else — no GPU state is inherited."""
    import multiprocessing as mp

    n = max(1, min(P, _cpu_threads(), int(os.environ.get("OMP_NUM_THREADS", P))))
    cfg = dict(num_envs=args.num_envs, learn_step=args.learn_step, batch_size=args.batch_size,
               update_epochs=args.epochs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_agent_worker, args=(cfg, seconds, 7 + i, q)) for i in range(n)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=seconds + 300) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    value = sum(s / t for s, t in res)
    return dict(value=round(value, 1), unit="env-steps/s", cores=n, kind="port",
                sample=f"{n} agents of oracle/ppo_cpu.py as {n} single-threaded processes side by side, "
                       f"~{seconds:.0f}s of whole iterations each ({_cpu_threads()} CPUs allowed)")


def _ppo_loss_torch_batched(logp, old_logp, adv, ret, old_v, v, H, b, clip, vf, ent):
    """ppo.py:868-896 forward + its gradients (d/dlogp, d/dv, d/dH) as torch
    CPU ops over all minibatches at once ([S/b, b] views)."""
    t = [torch.from_numpy(np.ascontiguousarray(x)).view(-1, b) for x in (logp, old_logp, adv, ret, old_v, v, H)]
    logp, old_logp, adv, ret, old_v, v, H = t
    ratio = torch.exp(logp - old_logp)
    rc = ratio.clamp(1 - clip, 1 + clip)
    p1, p2 = -adv * ratio, -adv * rc
    pg = torch.maximum(p1, p2).mean(1)
    dv = v - old_v
    vcl = old_v + dv.clamp(-clip, clip)
    lu, lc = (v - ret) ** 2, (vcl - ret) ** 2
    vl = 0.5 * torch.maximum(lu, lc).mean(1)
    loss = pg + vf * vl - ent * H.mean(1)
    g1 = (p1 > p2).float() + 0.5 * (p1 == p2).float()
    g2 = (p2 > p1).float() + 0.5 * (p1 == p2).float()
    inr = ((ratio >= 1 - clip) & (ratio <= 1 + clip)).float()
    g_logp = (g1 * -adv + g2 * -adv * inr) / b * ratio
    gu = (lu > lc).float() + 0.5 * (lu == lc).float()
    gc = (lc > lu).float() + 0.5 * (lu == lc).float()
    inv = ((dv >= -clip) & (dv <= clip)).float()
    g_v = vf * 0.5 / b * (gu * 2 * (v - ret) + gc * 2 * (vcl - ret) * inv)
    g_H = torch.full_like(H, -ent / b)
    return loss, g_logp, g_v, g_H


def cpu_kernels_leg(seconds):
    """SURVEY §8d CPU lines for the roofline workload (GAE + 4 x loss, 177 B
    per transition): the numpy T-loop GAE + the torch-op loss on 1 thread, and
    the OpenMP C restatement (oracle/c/oracle.c) on every allowed core, each on
    a bounded slice of the §8d inputs (whole agents of T=1024 x N=8192)."""
    from oracle import cref
    from oracle import gae as ogae

    T, N, b = ROOF_T, ROOF_N, ROOF_B
    rng = np.random.default_rng(0)
    r = rng.standard_normal((T, N), dtype=np.float32)
    v = rng.standard_normal((T, N), dtype=np.float32)
    d = (rng.random((T, N)) < 0.01).astype(np.uint8)
    lv = rng.standard_normal(N, dtype=np.float32)
    ld = (rng.random(N) < 0.01).astype(np.uint8)
    S = T * N
    old_logp = (rng.random(S, dtype=np.float32) * -2.95 - 0.05).astype(np.float32)
    logp = (old_logp + 0.05 * rng.standard_normal(S, dtype=np.float32)).astype(np.float32)
    newv = (v.reshape(-1) + 0.1 * rng.standard_normal(S, dtype=np.float32)).astype(np.float32)
    H = (rng.random(S, dtype=np.float32) * np.float32(np.log(4))).astype(np.float32)
    out = {}
    # numpy / torch-op path, 1 thread: GAE once + loss x4 per agent slice
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    t0, n = time.perf_counter(), 0
    while True:
        adv, ret = ogae.gae(r, v, d.astype(bool), lv, ld.astype(bool))
        for _ in range(4):
            _ppo_loss_torch_batched(logp, old_logp, adv.reshape(-1), ret.reshape(-1), v.reshape(-1), newv, H,
                                    b, 0.2, 0.5, 0.01)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    torch.set_num_threads(threads)
    rate = n * S / dt
    out["numpy_torch_1t"] = dict(value=round(rate, 1), unit="transitions/s", gbs=round(rate * 177 / 1e9, 3),
                                 cores=1, kind="port",
                                 sample=f"{n} x (T={T}, N={N}) GAE numpy T-loop + 4 torch-op loss passes")
    n_thr = int(os.environ.get("OMP_NUM_THREADS", _cpu_threads()))
    t0, n = time.perf_counter(), 0
    while True:
        adv, ret = cref.gae(r, v, d, lv, ld, 0.99, 0.95, nthreads=n_thr)
        for _ in range(4):
            cref.ppo_loss(logp, old_logp, adv.reshape(-1), ret.reshape(-1), v.reshape(-1), newv, H, b, 0.2, 0.5,
                          0.01, nthreads=n_thr)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    rate = n * S / dt
    out["c_openmp"] = dict(value=round(rate, 1), unit="transitions/s", gbs=round(rate * 177 / 1e9, 3),
                           cores=n_thr, kind="port",
                           sample=f"{n} x (T={T}, N={N}) oracle_gae + 4 oracle_ppo_loss (gcc -O2 -fopenmp)")
    return out


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or platform.machine()


def _c51_torch_ops(q_next, target_dist, logp_cur, actions, r, d, support, v_min, v_max, gamma):
    """RainbowDQN._dqn_loss's projection + elementwise loss as the reference's
    torch ops (dqn_rainbow.py:313-367) on given network outputs."""
    B, Z = target_dist.shape[0], support.shape[0]
    delta_z = float(v_max - v_min) / (Z - 1)
    next_actions = q_next.argmax(1)
    tq = target_dist[torch.arange(B), next_actions]
    t_z = (r + (1 - d) * gamma * support).clamp(min=v_min, max=v_max)
    b = (t_z - v_min) / delta_z
    L, u = b.floor().long(), b.ceil().long()
    L[(u > 0) * (u == L)] -= 1
    u[((Z - 1) > L) * (u == L)] += 1
    offset = torch.linspace(0, (B - 1) * Z, B).long().unsqueeze(1).expand(B, Z)
    proj = torch.zeros(tq.size())
    proj.view(-1).index_add_(0, (L + offset).view(-1), (tq * (u.float() - b)).view(-1))
    proj.view(-1).index_add_(0, (u + offset).view(-1), (tq * (b - L.float())).view(-1))
    log_p = logp_cur[torch.arange(B), actions.squeeze(-1)]
    return -(proj * log_p).sum(1)


def cpu_offpolicy_leg(seconds):
    """BASELINE.md §3 / SURVEY §8d CPU lines beside the off-policy kernels, on
    1 host thread: the reference's Python-loop segment tree (oracle/per.py,
    segment_tree.py:81-156 + replay_buffer.py:357-428) timed on 2^14-sample
    slices of a 2^20-leaf tree and scaled per sample, and the torch-op C51
    projection + loss (dqn_rainbow.py:313-367) on bounded 2^15-row slices of
    the §8d C51 shape (A = 6, Z = 51, +-200)."""
    from oracle import per as oper

    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    out = {"cpu_model": _cpu_model(), "threads": 1}
    cap = 1 << 20
    rng = np.random.default_rng(2)
    leaves = (np.abs(rng.standard_normal(cap)) + 1e-5) ** 0.6
    buf = oper.PER(cap, alpha=0.6)
    buf.sum_tree.tree = oper.build_tree_from_leaves(leaves, cap, "sum").tolist()
    buf.min_tree.tree = oper.build_tree_from_leaves(leaves, cap, "min").tolist()
    buf.size, buf.tree_ptr = cap, 0
    n = 1 << 14
    u = torch.rand(n, generator=torch.Generator().manual_seed(2)).numpy()
    t0, reps = time.perf_counter(), 0
    while True:
        idx = buf.sample_indices(u)
        buf.weights(idx, 0.4)
        reps += 1
        if time.perf_counter() - t0 >= seconds / 3:
            break
    dt = time.perf_counter() - t0
    out["per_sample"] = dict(value=round(reps * n / dt, 1), unit="samples/s", cores=1, kind="port",
                             sample=f"{reps} x 2^14 proportional samples + IS weights (Python loop) on a 2^20-leaf "
                                    "tree, scaled per sample")
    idx = rng.integers(0, cap, n)
    pri = np.abs(rng.standard_normal(n)).astype(np.float32)
    t0, reps = time.perf_counter(), 0
    while True:
        buf.update_priorities(idx, pri)
        reps += 1
        if time.perf_counter() - t0 >= seconds / 3:
            break
    dt = time.perf_counter() - t0
    out["per_update"] = dict(value=round(reps * n / dt, 1), unit="updates/s", cores=1, kind="port",
                             sample=f"{reps} x 2^14 update_priorities (Python loop, two 20-level root paths each), "
                                    "scaled per update")
    B, A, Z = 1 << 15, 6, 51
    g = torch.Generator().manual_seed(3)
    q_next = torch.randn(B, A, generator=g)
    td = torch.softmax(torch.randn(B, A, Z, generator=g), -1).clamp(min=1e-3)
    logp = torch.log_softmax(torch.randn(B, A, Z, generator=g), -1)
    act = torch.randint(0, A, (B, 1), generator=g)
    r = torch.randn(B, 1, generator=g)
    d = (torch.rand(B, 1, generator=g) < 0.05).float()
    support = torch.linspace(-200.0, 200.0, Z)
    t0, reps = time.perf_counter(), 0
    while True:
        _c51_torch_ops(q_next, td, logp, act, r, d, support, -200.0, 200.0, 0.99 ** 4)
        reps += 1
        if time.perf_counter() - t0 >= seconds / 3:
            break
    dt = time.perf_counter() - t0
    out["c51_project_loss"] = dict(value=round(reps * B / dt, 1), unit="rows/s", gbs=round(reps * B * 444 / dt / 1e9, 3),
                                   cores=1, kind="port",
                                   sample=f"{reps} x 2^15 rows of the reference's torch-op projection + loss")
    torch.set_num_threads(threads)
    return out


# --------------------------------------------------------------------------- #
def config5_leg(iters: int = 5, P: int = 4):
    """Config 5's per-GPU shard (Atari Breakout PPO, ppo_image.yaml network:
    conv 32/64/128 k8/4/3 s4/2/1 -> latent 256 -> heads [256]): 4 agents x 64
    envs of uint8 4x84x84 frames (32 agents / 2048 envs over 8 GPUs), learn_step
    256 (T = 4), batch 128, 4 epochs; the population-grouped HIP convolutions
    and the autograd learner.  A side measurement, not the headline line."""
    from agilerl_amd.envs import StackedVecEnv, SyntheticAtariVecEnv
    from agilerl_amd.population.runner import PopulationRunner
    from agilerl_amd.utils import create_population

    N = 64
    hp = {"BATCH_SIZE": 128, "LR": 1e-3, "LEARN_STEP": 256, "UPDATE_EPOCHS": 4}
    net = {"latent_dim": 256,
           "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
           "head_config": {"hidden_size": [256], "layer_norm": False}}
    env = SyntheticAtariVecEnv(N, n_actions=4, seed=1)
    agents = create_population("PPO", net, hp, env.single_observation_space, env.single_action_space,
                               population_size=P, num_envs=N)
    pop = agents[0].population
    runner = PopulationRunner(pop, StackedVecEnv.from_shared(env, P))
    for _ in range(2):
        runner.iteration()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        runner.iteration()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"workload": f"config 5 {'shard' if P < 32 else 'whole population on one GPU'}: PPO pop={P} x 64 envs, "
                       "uint8 4x84x84 frames, T=4, batch 128, 4 epochs, CNN 32/64/128 -> 256, heads [256]",
           "rollout_bytes": int(pop.obs.numel() * pop.obs.element_size()),
           "iterations": iters, "ms_per_iteration": round(dt / iters * 1e3, 2),
           "env_steps_per_s": round(P * N * pop.T * iters / dt, 1),
           "learner_updates_per_s": round(pop.n_updates() * iters / dt, 1)}
    del runner, agents, pop
    torch.cuda.empty_cache()
    return out


CONFIG3_NET = {"latent_dim": 256, "min_latent_dim": 128, "max_latent_dim": 512,
               "encoder_config": {"channel_size": [32, 64, 128], "kernel_size": [8, 4, 3], "stride_size": [4, 2, 1]},
               "head_config": {"hidden_size": [256]}}


def mutated_learner_leg(P: int = 8):
    """One learn() of an architecture-mutated agent population (config-2 sizes:
    S = 2048 samples per agent, batch 128, 4 epochs) on the
    runtime-shape HIP learner (agx_ppo_learn_graph) against the plain-PyTorch
    learner it replaces, beside the compiled fused learner on the unmutated
    shape.  Shape: encoder [80] -> latent 56 -> actor head [64, 64] / critic
    [64] (three mutations from ppo.yaml's network)."""
    from agilerl_amd.population.learner import FusedLearner, GraphLearner
    from agilerl_amd.population.nets import ActorCriticSpec
    from agilerl_amd.population.ppo_pop import PPOPopulation

    dev = torch.device("cuda:0")

    def make(**kw):
        spec = ActorCriticSpec(obs_dim=8, n_actions=4, **kw)
        pop = PPOPopulation(spec, P, 16, learn_step=2048, batch_size=128, update_epochs=4, device=dev, fused=True,
                            seeds=list(range(P)), perm_source="device")
        g = torch.Generator(device=dev).manual_seed(0)
        pop.obs.copy_(torch.randn(pop.obs.shape, device=dev, generator=g))
        pop.actions.copy_(torch.randint(0, 4, pop.actions.shape, device=dev, generator=g))
        pop.rewards.copy_(torch.randn(pop.rewards.shape, device=dev, generator=g))
        pop.values.copy_(torch.randn(pop.values.shape, device=dev, generator=g))
        pop.log_probs.copy_(-torch.rand(pop.log_probs.shape, device=dev, generator=g) - 0.5)
        pop.finish_rollout(torch.randn(P, 16, 8, device=dev, generator=g),
                           torch.zeros(P, 16, dtype=torch.uint8, device=dev))
        return pop, pop.permutations()

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / reps * 1e3, 3)

    pop, perms = make()
    fl = FusedLearner(pop)
    out = {"workload": f"{P} agents x S 2048, batch 128, 4 epochs (64 updates per agent per learn)",
           "compiled_shape_fused_ms": timed(lambda: fl.learn(pop, perms), 5)}
    del fl, pop
    pop, perms = make(encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64])
    gl = GraphLearner(pop)
    out["mutated_shape"] = "encoder [80] -> latent 56 -> actor [64, 64] / critic [64]"
    out["mutated_graph_ms"] = timed(lambda: gl.learn(pop, perms), 5)
    out["mutated_torch_ms"] = timed(lambda: pop._learn_torch(perms), 1)
    del gl, pop
    torch.cuda.empty_cache()
    return out


def train_on_policy_leg(generations: int = 3, P: int = 8, N: int = 128):
    """The end-to-end entry point: ``train_on_policy`` (training/train_on_policy.py)
    on an 8-agent population with ppo.yaml's INIT_HP / NET_CONFIG /
    MUTATION_PARAMS (LEARN_STEP 2048, BATCH 128, 4 epochs, EVO_STEPS 10240,
    EVAL_STEPS empty = each evaluation episode runs to its end, tournament 2 with
    elitism), N synthetic LunarLander-shaped envs per agent (the reference's
    N-env cloned per agent).  Per generation: 5 collect + learn iterations per
    agent, agent.test evaluation, tournament, mutations (RL hyperparameters,
    parameters, architecture, learn_step) and the regroup.  Timed over
    ``generations`` generations after one warm-up generation; env-steps are
    the training steps the reference counts (agent.steps), evaluation steps
    not included.  Reported with ppo.yaml's MUTATION_PARAMS as they are
    (ARCH_MUT 0.2) and with ARCH_MUT = 0 (every agent stays on the compiled
    kernels; the other mutation kinds as ppo.yaml); each also over
    AGX_BENCH_E2E_LONG (default 10) generations, with the milliseconds per
    generation split by phase (train / evaluate / select / mutate / regroup)
    and the count of agents on each kernel family at the end."""
    from agilerl_amd.envs import SyntheticVecEnv
    from agilerl_amd.hpo.mutation import Mutations
    from agilerl_amd.hpo.registry import HyperparameterConfig, RLParameter
    from agilerl_amd.hpo.tournament import TournamentSelection
    from agilerl_amd.training import train_on_policy
    from agilerl_amd.utils import create_population

    INIT_HP = {"BATCH_SIZE": 128, "LR": 0.001, "LEARN_STEP": 2048, "GAMMA": 0.99, "GAE_LAMBDA": 0.95,
               "CLIP_COEF": 0.2, "ENT_COEF": 0.01, "VF_COEF": 0.5, "MAX_GRAD_NORM": 0.5, "TARGET_KL": None,
               "UPDATE_EPOCHS": 4}
    NET_CONFIG = {"latent_dim": 64,
                  "encoder_config": {"hidden_size": [64], "activation": "ReLU", "min_mlp_nodes": 64,
                                     "max_mlp_nodes": 500, "layer_norm": True},
                  "head_config": {"hidden_size": [64], "activation": "ReLU", "min_hidden_layers": 1,
                                  "max_hidden_layers": 3, "min_mlp_nodes": 64, "max_mlp_nodes": 500,
                                  "output_vanish": True, "layer_norm": True}}
    evo_steps = 10_240
    out = {"workload": f"train_on_policy, {P}-agent PPO population, ppo.yaml (evo_steps {evo_steps}, eval to "
                       f"episode end, tournament 2 + elitism, MUT_P of ppo.yaml), {N} synthetic envs per agent",
           "generations_timed": generations}

    def run(arch: float, gens: int, seed: int):
        np.random.seed(seed)
        torch.manual_seed(seed)
        # LunarLander-v3 episodes end at its TimeLimit (1000 steps) at the latest: the
        # evaluation (EVAL_STEPS empty) runs every env to the end of its episode
        env = SyntheticVecEnv(N, seed=seed, p_done=1 / 200, max_episode_steps=1000)
        hp = HyperparameterConfig(lr=RLParameter(min=0.0001, max=0.01),
                                  batch_size=RLParameter(min=8, max=1024, dtype=int),
                                  learn_step=RLParameter(min=256, max=8192, dtype=int, grow_factor=1.5,
                                                         shrink_factor=0.75),
                                  ent_coef=RLParameter(min=0.001, max=0.1),
                                  update_epochs=RLParameter(min=1, max=10, dtype=int))
        pop = create_population("PPO", NET_CONFIG, INIT_HP, env.single_observation_space,
                                env.single_action_space, hp_config=hp, population_size=P, num_envs=N)
        mut = Mutations(no_mutation=0.4, architecture=arch, new_layer_prob=0.2, parameters=0.2, activation=0.2,
                        rl_hp=0.2, mutation_sd=0.1, rand_seed=42)
        tour = TournamentSelection(2, True, P, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        import contextlib

        with contextlib.redirect_stdout(sys.stderr):  # stdout carries the one JSON line only
            pop, _ = train_on_policy(env, "LunarLanderSynthetic", "PPO", pop, INIT_HP=INIT_HP,
                                     max_steps=gens * evo_steps, evo_steps=evo_steps, eval_steps=None, eval_loop=1,
                                     tournament=tour, mutation=mut, verbose=True)  # per-generation progress
        torch.cuda.synchronize()
        return time.perf_counter() - t0, pop

    import warnings

    # ppo.yaml's MUTATION_PARAMS as they are (ARCH_MUT 0.2: mutated agents run the
    # runtime-shape kernels, agx_ppo_learn_graph / agx_ppo_act_graph), and with
    # architecture mutations off (every agent stays on the compiled kernels)
    variants = [("ppo_yaml", 0.2), ("no_arch_mutation", 0.0)]
    if os.environ.get("AGX_BENCH_E2E_NO_ARCH_ONLY"):
        variants = variants[1:]
    import importlib

    top_mod = importlib.import_module("agilerl_amd.training.train_on_policy")  # the module (PHASE_TIMES)

    def one(arch: float, gens: int, seed: int) -> dict:
        top_mod.PHASE_TIMES.clear()
        dt, pop = run(arch, gens, seed)
        steps = sum(a.steps[-1] for a in pop)
        fused = sum(a.population.fused_descriptor() is not None for a in pop)
        hip = sum(a.population.learn_descriptor() is not None for a in pop)
        phases = {k: round(v / gens * 1e3, 2) for k, v in sorted(top_mod.PHASE_TIMES.items())}
        phases["other"] = round(dt / gens * 1e3 - sum(phases.values()), 2)
        return {"env_steps_per_s": round(steps / dt, 1), "ms_per_generation": round(dt / gens * 1e3, 2),
                "ms_per_generation_by_phase": phases, "env_steps": int(steps),
                "agents_on_compiled_kernels_at_end": int(fused),
                "agents_on_runtime_shape_kernels_at_end": int(hip - fused),
                "agents_on_pytorch_learner_at_end": int(len(pop) - hip),
                "groups_at_end": len({id(a.population) for a in pop}),
                "final_shapes": sorted({str(a.spec.shape_key()[2:6]) for a in pop})}

    long_gens = int(os.environ.get("AGX_BENCH_E2E_LONG", 10))
    for name, arch in variants:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            run(arch, 1, 5)  # warm-up (first-use allocations, library start-up)
            log(f"train_on_policy {name}: warm-up done")
            out[name] = one(arch, generations, 6)
            log(f"train_on_policy {name}: {generations} generations: {out[name]['ms_per_generation']} ms each, "
                f"by phase {out[name]['ms_per_generation_by_phase']}, {out[name]['groups_at_end']} groups")
            if long_gens > generations:
                # the decay as mutations move agents to other groups / kernels
                out[name][f"{long_gens}_generations"] = one(arch, long_gens, 7)
                lg = out[name][f'{long_gens}_generations']
                log(f"train_on_policy {name}: {long_gens} generations: {lg['ms_per_generation']} ms each, "
                    f"by phase {lg['ms_per_generation_by_phase']}, {lg['groups_at_end']} groups")
    return out


def config3_leg(iters: int = 10, P: int = 8, B: int = 64, fill: int = 1 << 15, on_timed=None):
    """Config 3 (Atari Pong Rainbow DQN, pop 8): learner updates/s of the
    population-batched learner (algorithms/rainbow_pop.py) on uint8 4x84x84
    frames, CNN 32/64/128 -> 256, dueling noisy heads [256], A = 6, Z = 51 on
    +-200, B = 64, PER (alpha 0.6, beta 0.4) over a 1M-transition buffer
    (2^20-leaf trees) holding `fill` synthetic transitions.  One iteration =
    the P agents' samples in one draw (the same torch.rand stream as P
    draws), one batched learn, the P priority updates in agent order.  The
    per-agent loop of the reference (sample, agent.learn, update per agent)
    is timed on copies of the same agents beside it.  ``on_timed(name,
    start)``: called right before / after each timed loop (profiling markers,
    tools/prof_config3.py)."""
    from agilerl_amd.algorithms import RainbowDQN
    from agilerl_amd.algorithms.rainbow_pop import RainbowPopulationLearner
    from agilerl_amd.components import PrioritizedReplayBuffer
    from agilerl_amd.envs import Box, Discrete

    dev = torch.device("cuda")
    obs_space, act_space = Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6)
    torch.manual_seed(0)
    agents = [RainbowDQN(obs_space, act_space, net_config=CONFIG3_NET, batch_size=B, lr=1e-4, gamma=0.99, tau=1e-3,
                         v_min=-200.0, v_max=200.0, num_atoms=51) for _ in range(P)]
    memory = PrioritizedReplayBuffer(1_000_000, alpha=0.6)
    g = torch.Generator(device=dev).manual_seed(1)
    for c in range(0, fill, 4096):
        n = min(4096, fill - c)
        memory.add({"obs": torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g),
                    "action": torch.randint(0, 6, (n,), device=dev, generator=g),
                    "reward": torch.randn(n, device=dev, generator=g),
                    "next_obs": torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g),
                    "done": (torch.rand(n, device=dev, generator=g) < 0.02).float()})
    # the per-agent leg runs on its own copies: the population learner takes the
    # agents' tensors over as rows of its flat buffers, which the entry point's
    # agents never are (their own learn keeps its flat state, flat_state.py)
    solo = [copy.deepcopy(a) for a in agents]
    learner = RainbowPopulationLearner(agents)

    def batched():
        s = memory.sample(P * B, beta=0.4)
        exps = [{k: v[p * B:(p + 1) * B] for k, v in s.items()} for p in range(P)]
        outs = learner.learn(exps, per=True)
        memory.update_priorities(torch.cat([o[1].reshape(-1) for o in outs]),
                                 np.concatenate([o[2].reshape(-1) for o in outs]))

    def per_agent():
        for a in solo:
            s = memory.sample(B, beta=0.4)
            _, idxs, pri = a.learn(s, per=True)
            memory.update_priorities(idxs, pri)

    out = {"workload": f"config 3: Rainbow DQN pop={P}, B={B}, uint8 4x84x84 frames, CNN 32/64/128 -> 256, dueling "
                       "noisy heads [256], A=6, Z=51 (+-200), PER alpha 0.6 / beta 0.4 on a 1M-transition buffer "
                       f"(2^20-leaf trees, {fill} transitions stored)", "iterations": iters}
    for name, fn in (("batched", batched), ("per_agent", per_agent)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        if on_timed is not None:
            on_timed(name, True)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if on_timed is not None:
            on_timed(name, False)
        out[name] = {"learner_updates_per_s": round(P * iters / dt, 1), "ms_per_iteration": round(dt / iters * 1e3, 3)}
    # the headline is what the drop-in entry point runs: train_off_policy learns
    # agent after agent (the reference's train_off_policy.py:355-429); the
    # population-batched learner (one launch chain for all P agents, lock-step
    # sampling) is reported beside it as an extra, not as the config-3 number
    out["learner_updates_per_s"] = out["per_agent"]["learner_updates_per_s"]
    out["entry_point"] = "per_agent (train_off_policy); batched = algorithms/rainbow_pop.py, not on the entry point"
    del learner, agents, solo, memory
    torch.cuda.empty_cache()
    return out


def cpu_config3_learn(seconds: float, B: int = 64):
    """The reference's Rainbow update (dqn_rainbow.py:284-490: three forwards,
    the torch-op C51 projection + loss, backward, clip_grad_norm_(10), Adam,
    soft update, noise reset) restated in plain torch ops on the host cores,
    for ONE agent of the config-3 network; bounded to ~`seconds`."""
    from torch import nn
    from torch.nn import functional as F

    threads = torch.get_num_threads()
    A, Z = 6, 51

    class Noisy(nn.Module):
        def __init__(self, i, o):
            super().__init__()
            self.mu_w = nn.Parameter(torch.randn(o, i) / i ** 0.5)
            self.sg_w = nn.Parameter(torch.full((o, i), 0.5 / i ** 0.5))
            self.mu_b = nn.Parameter(torch.zeros(o))
            self.sg_b = nn.Parameter(torch.full((o,), 0.5 / o ** 0.5))
            self.reset()

        def reset(self):
            f = lambda n: (lambda x: x.sign() * x.abs().sqrt())(torch.randn(n))  # noqa: E731
            ei, eo = f(self.mu_w.shape[1]), f(self.mu_w.shape[0])
            self.eps_w, self.eps_b = torch.outer(eo, ei), eo

        def forward(self, x):
            return F.linear(x, self.mu_w + self.sg_w * self.eps_w, self.mu_b + self.sg_b * self.eps_b)

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.enc = nn.Sequential(nn.Conv2d(4, 32, 8, 4), nn.ReLU(), nn.Conv2d(32, 64, 4, 2), nn.ReLU(),
                                     nn.Conv2d(64, 128, 3, 1), nn.ReLU(), nn.Flatten(), nn.Linear(128 * 7 * 7, 256),
                                     nn.ReLU())
            self.v1, self.v2, self.vn = Noisy(256, 256), Noisy(256, Z), nn.LayerNorm(256)
            self.a1, self.a2, self.an = Noisy(256, 256), Noisy(256, A * Z), nn.LayerNorm(256)

        def forward(self, x, log=False):
            h = self.enc(x.float() / 255.0)
            v = self.v2(F.relu(self.vn(self.v1(h)))).view(-1, 1, Z)
            a = self.a2(F.relu(self.an(self.a1(h)))).view(-1, A, Z)
            x = v + a - a.mean(1, keepdim=True)
            return F.log_softmax(x, -1) if log else F.softmax(x, -1).clamp(min=1e-3)

        def noise(self):
            for m in (self.v1, self.v2, self.a1, self.a2):
                m.reset()

    torch.manual_seed(0)
    net, tgt = Net(), Net()
    tgt.load_state_dict(net.state_dict())
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    support = torch.linspace(-200.0, 200.0, Z)
    g = torch.Generator().manual_seed(2)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g)
    nobs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g)
    act = torch.randint(0, A, (B, 1), generator=g)
    r, d = torch.randn(B, 1, generator=g), (torch.rand(B, 1, generator=g) < 0.02).float()
    w = torch.rand(B, 1, generator=g)
    t0, reps = time.perf_counter(), 0
    while True:
        with torch.no_grad():
            q_next = (net(nobs) * support).sum(2)
            td = tgt(nobs)
        logp = net(obs, log=True)
        el = _c51_torch_ops(q_next, td, logp, act, r, d, support, -200.0, 200.0, 0.99)
        loss = torch.mean(el * w)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 10.0)
        opt.step()
        with torch.no_grad():
            for pt, po in zip(tgt.parameters(), net.parameters()):
                pt.copy_(1e-3 * po + (1 - 1e-3) * pt)
        net.noise()
        tgt.noise()
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return dict(value=round(reps / dt, 2), unit="learner updates/s", cores=threads, kind="port",
                sample=f"{reps} Rainbow updates of one config-3 agent (B={B}) in torch CPU ops on {threads} threads")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world, rank, local = setup_dist(gpu=not args.dist_selftest)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dist_selftest:
        dist_selftest(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    from agilerl_amd import _lib

    _lib.load()
    if args.pop % world:
        raise SystemExit(f"bench.py: --pop {args.pop} agents cannot be sharded over {world} GPUs")
    log("population leg")
    res = population_leg(args, world, rank, args.pop // world)
    weak = None
    if world > 1 and not args.no_weak:
        w = population_leg(args, world, rank, args.pop_per_gpu)
        weak = {"value": round(w["env_steps"] / w["dt"], 1), "unit": "env-steps/s",
                "ms_per_step": round(w["dt"] / args.steps * 1e3, 3),
                "learner_updates_per_s": round(w["updates"] / w["dt"], 1),
                "workload": f"{args.pop_per_gpu} agents per GPU ({args.pop_per_gpu * world}-agent population)"}
    roof = kern = None
    if not args.no_roofline:
        log("roofline leg")
        roof = roofline_leg(args)
        kern = kernels_leg(roof["peak_measured"])
    log("config-5 leg")
    c5 = config5_leg() if (world == 1 and not args.no_config5) else None
    if c5 is not None:
        log("config-5 whole-population leg")
        # config 5's whole 32-agent population on one GPU (2048 envs, ~230 MB of
        # uint8 rollout): what one MI355X holds that the 8-GPU shard does not need
        c5["pop32_one_gpu"] = config5_leg(iters=2, P=32)
    log("config-3 leg")
    c3 = config3_leg() if (world == 1 and not args.no_config3) else None
    log("train_on_policy leg")
    tp = train_on_policy_leg() if (world == 1 and not args.no_train_on_policy) else None
    log("mutated-shape learner leg")
    ml = mutated_learner_leg() if world == 1 else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log("CPU baseline legs")
        cpu = cpu_baseline_leg(args, res["S"])
        cpu["all_cores"] = cpu_population_all_cores(args, min(args.cpu_seconds, 10.0))
        cpu["roofline_workload"] = cpu_kernels_leg(min(args.cpu_seconds, 8.0))
        cpu["off_policy"] = cpu_offpolicy_leg(min(args.cpu_seconds, 9.0))
        cpu["cpu_model"] = cpu["off_policy"]["cpu_model"]
        if c3 is not None:
            cpu["config3_learn"] = cpu_config3_learn(min(args.cpu_seconds, 10.0))
    if rank == 0:
        value = res["env_steps"] / res["dt"]
        line = {
            "metric": "population env-steps/sec + learner updates/sec, 8-agent PPO at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(res["dt"] / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32 (GAE carry f64)",
            "data": "synthetic (host SyntheticVecEnv: obs 8 f32, 4 actions, r~N(0,1), done~Bern(1/200))",
            "config": {
                "workload": f"config 2: one {args.pop}-agent PPO population sharded {args.pop // world} agents per "
                            "GPU, 128 vec envs per agent, T=16, batch 128, 4 epochs, MLP enc[64]->64 + heads[64] "
                            f"(shared encoder), tournament every {args.evo_every} iterations",
                "population": args.pop, "pop_per_gpu": args.pop // world, "num_envs": args.num_envs,
                "learn_step": args.learn_step,
                "batch_size": args.batch_size, "update_epochs": args.epochs, "learner": args.learner,
                "parallelism": f"population-sharded x{world}",
            },
            "learner_updates_per_s": round(res["updates"] / res["dt"], 1),
            "weak_scaling": weak,
            "learner": res["learner"],
            "generations": res["generations"],
            "generation_fitness": "mean return of the training episodes finished since the previous generation "
                                  "(fitness all-gather + tournament + parent clone are timed; a separate "
                                  "agent.test() evaluation pass is not run in the timed loop)",
            "minibatch_order": "numpy global MT19937 np.random.shuffle stream (reference-reproducible), drawn "
                               "natively on the host while the GPU learns",
            "roofline": roof,
            "kernels": kern,
            "config5": c5,
            "config3": c3,
            "train_on_policy": tp,
            "mutated_shape_learner": ml,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
