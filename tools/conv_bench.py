"""Device time of the HIP implicit-GEMM convolutions (csrc/conv.hip) at the
Atari encoder's layers (8x8/4, 4x4/2, 3x3/1 over 4x84x84 uint8 frames; 32 /
64 / 128 channels): forward, and forward + backward (wgrad + dgrad), each
replayed from a captured graph and timed with HIP events.  B = 64 is the
config-3 per-agent update; G = 4 groups of B = 128 the config-5 grouped
update.

    python tools/conv_bench.py            # B=64 single and G=4 x 128 grouped
    LAYER=2 python tools/conv_bench.py    # one layer (under rocprofv3 --pmc)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = [(4, 84, 32, 8, 4), (32, 20, 64, 4, 2), (64, 9, 128, 3, 1)]  # Cin, H, Cout, k, stride


def timed(fn, reps=100):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from agilerl_amd.modules.cnn import Conv2dFn, Conv2dGroupedFn

    dev = torch.device("cuda")
    only = os.environ.get("LAYER")
    for G, B in ((1, 64), (4, 128)):
        for li, (cin, h, cout, k, st) in enumerate(LAYERS):
            if only is not None and int(only) != li:
                continue
            torch.manual_seed(li)
            if li == 0:
                x = torch.randint(0, 256, (G, B, cin, h, h), dtype=torch.uint8, device=dev)
            else:
                x = torch.randn(G, B, cin, h, h, device=dev).relu()
            w = (torch.randn(G, cout, cin, k, k, device=dev) * 0.05).requires_grad_(True)
            b = torch.zeros(G, cout, device=dev, requires_grad=True)
            xg = x if li == 0 else x.clone().requires_grad_(True)
            norm = (0.0, 255.0) if li == 0 else None

            if G == 1:
                def fwd():
                    with torch.no_grad():
                        Conv2dFn.apply(x[0], w[0], b[0], st, True, norm)

                def fb():
                    y = Conv2dFn.apply(xg[0], w[0], b[0], st, True, norm)
                    y.backward(torch.ones_like(y))
            else:
                def fwd():
                    with torch.no_grad():
                        Conv2dGroupedFn.apply(x, w, b, st, True, norm)

                def fb():
                    y = Conv2dGroupedFn.apply(xg, w, b, st, True, norm)
                    y.backward(torch.ones_like(y))
            f = timed(fwd)
            t = timed(fb)
            oh = (h - k) // st + 1
            flops = 2.0 * G * B * oh * oh * cout * cin * k * k
            print(f"G={G} B={B} layer {li + 1} ({cin}x{h}x{h} -> {cout}, k{k}/s{st}): forward {f:.1f} us "
                  f"({flops / f / 1e6:.1f} TFLOP/s), forward+backward {t:.1f} us", flush=True)


if __name__ == "__main__":
    main()
