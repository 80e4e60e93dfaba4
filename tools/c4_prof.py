"""C4 train steps only (bf16, batch 128), for rocprofv3 kernel stats of the step:
    rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/c4_prof.py [--steps 30]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng, X, Y = bench.c4_engine_and_batch(dev, 128)
for _ in range(3):
    eng.train_step(X, Y)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.steps):
    eng.train_step(X, Y)
e1.record()
e1.synchronize()
print(f"c4 train step {e0.elapsed_time(e1) / a.steps:.4f} ms")
