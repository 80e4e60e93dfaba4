"""Time the conv-AE train step and inference forward on one GPU.

    python tools/ae_bench.py [--model 3layer] [--batch 128] [--dtype bf16]

Models (the reference's graphs, Keras layer order):
  3layer        VAE/manual_scan_3layers.py:186-199, 128x128x1 (C4): conv 16/32/64 k5, pools,
                convT 64/32/16 k5 s2, conv 1 k5 (the bench's model)
  manual_scan   VAE/manual_scan.py:190-199 at (conv1, conv2, k) = (64, 32, 5), 256x128x1:
                conv 64, pool, conv 32, pool, convT 32, convT 64, conv 1 (all k5)
  hyper_k3/k5/k7  VAE/hyperparam_scan.py:153-161 (32/32 at kernel 3/5/7), 256x128x1
  graphs        VAE/graphs.ipynb (the notebook's model = hyper_k3), 256x128x1
FLOPs are counted from the layer list (2 x MACs, x3 for a training step)."""
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

def ops(model="3layer"):
    C, P = ae.ConvOp, ae.PoolOp
    if model == "3layer":
        return [C("conv", 1, 16, 5, "relu"), P(), C("conv", 16, 32, 5, "relu"), P(),
                C("conv", 32, 64, 5, "relu"), P(), C("convT", 64, 64, 5, "relu", stride=2),
                C("convT", 64, 32, 5, "relu", stride=2), C("convT", 32, 16, 5, "relu", stride=2),
                C("conv", 16, 1, 5, "sigmoid")], (128, 128, 1)
    if model == "manual_scan":
        c1, c2, k = 64, 32, 5
    elif model in ("hyper_k3", "hyper_k5", "hyper_k7", "graphs"):
        c1 = c2 = 32
        k = 3 if model == "graphs" else int(model[-1])
    else:
        raise SystemExit(f"unknown model {model}")
    return [C("conv", 1, c1, k, "relu"), P(), C("conv", c1, c2, k, "relu"), P(),
            C("convT", c2, c2, k, "relu", stride=2), C("convT", c2, c1, k, "relu", stride=2),
            C("conv", c1, 1, k, "sigmoid")], (256, 128, 1)


def fwd_flops(layer_ops, shape):
    h, w, _ = shape
    f = 0
    for op in layer_ops:
        if isinstance(op, ae.PoolOp):
            h, w = h // 2, w // 2
            continue
        if op.kind == "convT":  # MACs at the input resolution x stride^2 = output pixels x k^2 ci co / s^2
            f += 2 * h * w * op.k * op.k * op.cin * op.cout
            h, w = h * op.stride, w * op.stride
        else:
            f += 2 * h * w * op.k * op.k * op.cin * op.cout
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="3layer")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--infer-batch", type=int, default=None,
                    help="default 1024 at 128 x 128, 512 at 256 x 128")
    a = ap.parse_args()
    layer_ops, shape = ops(a.model)
    if a.infer_batch is None:
        a.infer_batch = 1024 if shape[0] == 128 else 512
    FLOP_FWD = fwd_flops(layer_ops, shape)
    eng = ae.AutoencoderEngine(layer_ops, shape, compute_dtype=a.dtype, device="cuda:0")
    rng = np.random.default_rng(0)
    ws = []
    for op in eng.ops:
        if isinstance(op, ae.ConvOp):
            kshape = (op.k, op.k, op.cin, op.cout) if op.kind == "conv" else (op.k, op.k, op.cout, op.cin)
            lim = np.sqrt(6.0 / (op.k * op.k * (op.cin + op.cout)))
            ws += [rng.uniform(-lim, lim, kshape).astype(np.float32), np.zeros(op.cout, np.float32)]
    eng.set_keras_weights(ws)
    x = eng.to_compute(torch.rand(a.batch, *shape, device="cuda:0"))
    y = eng.to_compute(torch.rand(a.batch, *shape, device="cuda:0"))
    for _ in range(3):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    train_ms = (time.perf_counter() - t0) / a.steps * 1e3
    xi = eng.to_compute(torch.rand(a.infer_batch, *shape, device="cuda:0"))
    for _ in range(2):
        eng.forward(xi)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.forward(xi)
    torch.cuda.synchronize()
    inf_ms = (time.perf_counter() - t0) / a.steps * 1e3
    res = {"model": a.model, "input": shape, "fwd_gflop_per_sample": FLOP_FWD / 1e9,
           "fused": {"enc2": eng.enc2, "dec3": eng.dec3, "tail": eng.tail,
                     "conv_pool": sorted(eng.fused)},
           "dtype": a.dtype, "train_batch": a.batch, "train_ms": train_ms,
           "train_samples_per_s": a.batch / train_ms * 1e3,
           "train_tflops": 3 * FLOP_FWD * a.batch / train_ms / 1e9,
           "infer_batch": a.infer_batch, "infer_ms": inf_ms,
           "infer_samples_per_s": a.infer_batch / inf_ms * 1e3,
           "infer_tflops": FLOP_FWD * a.infer_batch / inf_ms / 1e9,
           "infer_frac_of_16bit_mfma_peak": FLOP_FWD * a.infer_batch / inf_ms / 1e9 / 2500.0}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
