"""Time the weight-gradient launch (kernel + ordered sums) of every C4 layer (dev A/B tool).

    python tools/wgrad_bench.py [--batch 128] [--reps 30] [--dtype bf16]

One line per layer of the reference model (VAE/manual_scan_3layers.py:186-199) at the C4
shape (128 x 128 x 1 input): the forward geometry, its dOut shape and the microseconds of
torch.ops.specenh.conv2d_wgrad_out (workspace preallocated)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spectrogram-enhancement_amd"))
import specenh  # noqa: E402,F401
from specenh import ae, ops  # noqa: E402

# (name, kind, cin, cout, input H)
LAYERS = [("conv1", "conv", 1, 16, 128), ("conv2", "conv", 16, 32, 64),
          ("conv3", "conv", 32, 64, 32), ("convT1", "convT", 64, 64, 16),
          ("convT2", "convT", 64, 32, 32), ("convT3", "convT", 32, 16, 64),
          ("conv_out", "conv", 16, 1, 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    dev, N = "cuda:0", a.batch
    total = 0.0
    for name, kind, cin, cout, H in LAYERS:
        op = ae.ConvOp(kind, cin, cout, 5, "relu", stride=2 if kind == "convT" else 1)
        OH, OW = op.out_hw(H, H)
        s, pt, pl, dil = op.fwd_geom()
        x = torch.randn(N, H, H, cin, device=dev, dtype=dt)
        dz = torch.randn(N, OH, OW, cout, device=dev, dtype=dt)
        kh = kw = 5
        wcin, wcout = (cin, cout)
        dw = torch.zeros((wcout, kh, kw, wcin), dtype=torch.float32, device=dev)
        db = torch.zeros((wcout,), dtype=torch.float32, device=dev)
        ws = ops.wgrad_workspace(x, dz, kh, kw)

        def run():
            torch.ops.specenh.conv2d_wgrad_out(x, dz, kh, kw, s, pt, pl, dil, dw, db, ws)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        total += us
        print(f"{name:9s} x {tuple(x.shape)} dOut {tuple(dz.shape)}: {us:7.1f} us")
    print(f"total {total:.1f} us")


if __name__ == "__main__":
    main()
