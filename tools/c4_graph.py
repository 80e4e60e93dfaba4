"""Is the C4 train step launch-bound? (dev probe)

    python tools/c4_graph.py [--steps 100] [--batch 128]

Times the eager step (wall and host enqueue time per step) and the same step with forward +
BCE + backward replayed from one captured HIP graph (Adam eager: its bias correction is a
host scalar)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--batch", type=int, default=128)
a = ap.parse_args()
dev = torch.device("cuda", 0)
eng, X, Y = bench.c4_engine_and_batch(dev, a.batch)
for _ in range(3):
    eng.train_step(X, Y)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    eng.train_step(X, Y)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"eager: {(t2 - t0) / a.steps * 1e3:.4f} ms/step wall, "
      f"{(t1 - t0) / a.steps * 1e3:.4f} ms/step host enqueue")

xs, ys = X.clone(), Y.clone()
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    for _ in range(3):
        eng.forward(xs, train=True)
        eng.loss_and_grad(ys)
        eng.backward()
torch.cuda.current_stream(dev).wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    eng.forward(xs, train=True)
    eng.loss_and_grad(ys)
    eng.backward()
torch.cuda.synchronize()
for _ in range(3):
    g.replay()
    eng.adam()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    g.replay()
    eng.adam()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"graph: {(t2 - t0) / a.steps * 1e3:.4f} ms/step wall, "
      f"{(t1 - t0) / a.steps * 1e3:.4f} ms/step host enqueue")
