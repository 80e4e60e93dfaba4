"""Run one autoencoder layer's forward launch repeatedly (for rocprofv3 PMC passes).

    python tools/conv_one.py LAYER [--batch 4096] [--reps 20] [--dtype float16]
LAYER: l1 l2 l3 ct1 ct2 ct3 last (the C5 model at 128x128), tail (convT3 + conv_out, the
fused decoder tail) or all
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spectrogram-enhancement_amd"))
from specenh import ae  # noqa: E402

# (kind, cin, cout, input H, pool_after)
LAYERS = {"l1": ("conv", 1, 16, 128, True), "l2": ("conv", 16, 32, 64, True),
          "l3": ("conv", 32, 64, 32, True), "ct1": ("convT", 64, 64, 16, False),
          "ct2": ("convT", 64, 32, 32, False), "ct3": ("convT", 32, 16, 64, False),
          "last": ("conv", 16, 1, 128, False), "tail": ("convT", 32, 16, 64, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("layer")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="float16")
    a = ap.parse_args()
    names = list(LAYERS) if a.layer == "all" else [a.layer]
    for name in names:
        kind, cin, cout, H, pool = LAYERS[name]
        ops = [ae.ConvOp(kind, cin, cout, 5, "sigmoid" if name == "last" else "relu",
                         stride=2 if kind == "convT" else 1)]
        if pool:  # pool + a 1x1 tail so the pool is fused as in the model
            ops += [ae.PoolOp(), ae.ConvOp("conv", cout, 16, 1, "relu")]
        elif name == "tail":  # the model's last two layers: fused into one launch
            ops += [ae.ConvOp("conv", cout, 1, 5, "sigmoid")]
        elif kind == "convT":  # a 1x1 tail: the layer writes T activations as in the model
            ops += [ae.ConvOp("conv", cout, 16, 1, "relu")]
        eng = ae.AutoencoderEngine(ops, (H, H, cin), compute_dtype=a.dtype, device="cuda:0")
        rng = np.random.default_rng(0)
        ws = []
        for op in ops:
            if isinstance(op, ae.ConvOp):
                shape = ((op.k, op.k, op.cin, op.cout) if op.kind == "conv"
                         else (op.k, op.k, op.cout, op.cin))
                ws += [rng.uniform(-0.1, 0.1, shape).astype(np.float32),
                       np.zeros(op.cout, np.float32)]
        eng.set_keras_weights(ws)
        x = eng.to_compute(torch.rand(a.batch, H, H, cin, device="cuda:0"))
        for _ in range(3):
            eng.forward(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            eng.forward(x)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        print(f"{name}: {ms:.3f} ms/launch-group (batch {a.batch}, {a.dtype}, fused pool {pool})")


if __name__ == "__main__":
    main()
