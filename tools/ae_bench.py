"""Time the conv-AE train step and inference forward (C4 shape: 128x128x1, 3-layer
16/32/64 k5) on one GPU. Usage: python tools/ae_bench.py [--batch 128] [--dtype bf16]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spectrogram-enhancement_amd"))
from specenh import ae  # noqa: E402

FLOP_FWD = 2 * 248.9e6  # per sample, SURVEY.md §8 A7 (sum of per-layer MACs x 2)


def ops():
    C, P = ae.ConvOp, ae.PoolOp
    return [C("conv", 1, 16, 5, "relu"), P(), C("conv", 16, 32, 5, "relu"), P(),
            C("conv", 32, 64, 5, "relu"), P(), C("convT", 64, 64, 5, "relu", stride=2),
            C("convT", 64, 32, 5, "relu", stride=2), C("convT", 32, 16, 5, "relu", stride=2),
            C("conv", 16, 1, 5, "sigmoid")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--infer-batch", type=int, default=1024)
    a = ap.parse_args()
    eng = ae.AutoencoderEngine(ops(), (128, 128, 1), compute_dtype=a.dtype, device="cuda:0")
    rng = np.random.default_rng(0)
    ws = []
    for op in eng.ops:
        if isinstance(op, ae.ConvOp):
            shape = (op.k, op.k, op.cin, op.cout) if op.kind == "conv" else (op.k, op.k, op.cout, op.cin)
            lim = np.sqrt(6.0 / (op.k * op.k * (op.cin + op.cout)))
            ws += [rng.uniform(-lim, lim, shape).astype(np.float32), np.zeros(op.cout, np.float32)]
    eng.set_keras_weights(ws)
    x = eng.to_compute(torch.rand(a.batch, 128, 128, 1, device="cuda:0"))
    y = eng.to_compute(torch.rand(a.batch, 128, 128, 1, device="cuda:0"))
    for _ in range(3):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    train_ms = (time.perf_counter() - t0) / a.steps * 1e3
    xi = eng.to_compute(torch.rand(a.infer_batch, 128, 128, 1, device="cuda:0"))
    for _ in range(2):
        eng.forward(xi)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.forward(xi)
    torch.cuda.synchronize()
    inf_ms = (time.perf_counter() - t0) / a.steps * 1e3
    res = {"dtype": a.dtype, "train_batch": a.batch, "train_ms": train_ms,
           "train_samples_per_s": a.batch / train_ms * 1e3,
           "train_tflops": 3 * FLOP_FWD * a.batch / train_ms / 1e9,
           "infer_batch": a.infer_batch, "infer_ms": inf_ms,
           "infer_samples_per_s": a.infer_batch / inf_ms * 1e3,
           "infer_tflops": FLOP_FWD * a.infer_batch / inf_ms / 1e9}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
