"""C4 step time with the pool routing on a subset of the pooled Conv2Ds (dev probe):
    python tools/c4_routed_probe.py [--steps 40]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng, X, Y = bench.c4_engine_and_batch(dev, 128)
full = set(eng.pool_routed)
for rnd in range(3):
    for sub in (full, {4}, {2}, set()):
        eng.pool_routed = set(sub)
        for _ in range(3):
            eng.train_step(X, Y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            eng.train_step(X, Y)
        e1.record()
        e1.synchronize()
        print(f"round {rnd} routed {sorted(sub)}: {e0.elapsed_time(e1) / a.steps:.4f} ms")
