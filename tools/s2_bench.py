"""Time single conv launches of the C4 backward shapes (dev A/B tool).

    python tools/s2_bench.py [--batch 128] [--reps 50]

Rows: the Conv2DTranspose input gradients (stride-2 convs over dOut) with and without the
ReLU mask, on the stride-2 patch kernel and on the generic gather kernel
(SPECENH_CONV_NO_S2=1), plus the stride-1 conv of the same GEMM size for comparison."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spectrogram-enhancement_amd"))
import specenh  # noqa: E402,F401
from specenh import _lib  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev, dt, N = "cuda:0", torch.bfloat16, a.batch
    # (name, C, CO, H (input), stride)
    shapes = [("ct3_dgrad", 16, 32, 128, 2), ("ct2_dgrad", 32, 64, 64, 2),
              ("ct1_dgrad", 64, 64, 32, 2), ("s1_same_gemm_as_ct3", 16, 32, 64, 1)]
    for name, C, CO, H, s in shapes:
        OH = (H + s - 1) // s
        x = torch.randn(N, H, H, C, device=dev, dtype=dt)
        w = torch.randn(CO, 5, 5, C, device=dev, dtype=dt) * 0.1
        mask = torch.randn(N, OH, OH, CO, device=dev, dtype=dt)
        out = torch.empty(N, OH, OH, CO, device=dev, dtype=dt)
        for masked in (False, True):
            for generic in ((False, True) if s == 2 else (False,)):
                # the variant switches are read from the environment once per process:
                # select through the library, not os.environ
                _lib.set_variant("CONV_NO_S2", 1 if generic else 0)

                def run():
                    torch.ops.specenh.conv2d_out(x, w, None, 5, 5, CO, s, 2 if s == 2 else 2, 2, 1,
                                                 OH, OH, 0, mask if masked else None, None, out,
                                                 False, None)
                us = timeit(run, a.reps)
                gb = (x.numel() + out.numel() * (2 if masked else 1)) * 2 / 1e9
                print(f"{name:22s} mask={int(masked)} generic={int(generic)} {us:8.1f} us "
                      f"({gb / us * 1e3:6.0f} GB/s)")
    _lib.set_variant("CONV_NO_S2", 0)


if __name__ == "__main__":
    main()
