"""Per-launch device time of agx_noisy_streams_forward / _backward
(csrc/noisy_mlp.hip) at the config-3 head (latent 256, head [256], A = 6,
Z = 51, B = 64) and at one-layer stacks (no LayerNorm input), each replayed
200 times from a captured graph and timed with HIP events.

    python tools/noisy_streams_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=200):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from agilerl_amd.modules.mlp import create_mlp
    from agilerl_amd.modules.noisy_streams import head_streams

    dev = torch.device("cuda")
    B = int(os.environ.get("B", 64))
    cases = {"1": ([256],), "0": ([],)}.get(os.environ.get("HIDDEN", ""), ([256], []))
    for hidden in cases:
        torch.manual_seed(0)
        kw = dict(output_vanish=True, noisy=True, init_layers=False, layer_norm=True, noise_std=0.5, device=dev)
        v = create_mlp(256, 51, hidden, name="value", **kw)
        a = create_mlp(256, 306, hidden, name="advantage", **kw)
        x = torch.randn(B, 256, device=dev)
        xg = x.clone().requires_grad_(True)
        gv, ga = torch.randn(B, 51, device=dev), torch.randn(B, 306, device=dev)

        def fwd():
            with torch.no_grad():
                head_streams([v, a], x)

        def fwd_bwd():
            vo, ao = head_streams([v, a], xg)
            torch.autograd.backward([vo, ao], [gv, ga])

        f = timed(fwd)
        fb = timed(fwd_bwd)
        print(f"hidden {hidden}: forward {f:.1f} us per call ({len(hidden) + 1} launches), "
              f"forward + backward {fb:.1f} us (backward ~{fb - f:.1f} us incl. grad allocation)", flush=True)


if __name__ == "__main__":
    main()
