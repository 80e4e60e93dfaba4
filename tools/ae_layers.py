"""Per-launch inference time of a reference AE variant (tools/ae_bench.py models) on one GPU:
    python tools/ae_layers.py --model hyper_k3 [--batch 512] [--dtype fp16]
prints each convolution launch's kernel symbol, ms (median of --reps), and its share."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd"), os.path.join(REPO, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ae_bench  # noqa: E402
from specenh import ae  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="hyper_k3")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--dtype", default="fp16")
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
layer_ops, shape = ae_bench.ops(a.model)
eng = ae.AutoencoderEngine(layer_ops, shape, compute_dtype=a.dtype, device="cuda:0")
rng = np.random.default_rng(0)
ws = []
for op in eng.ops:
    if isinstance(op, ae.ConvOp):
        ks = (op.k, op.k, op.cin, op.cout) if op.kind == "conv" else (op.k, op.k, op.cout, op.cin)
        lim = np.sqrt(6.0 / (op.k * op.k * (op.cin + op.cout)))
        ws += [rng.uniform(-lim, lim, ks).astype(np.float32), np.zeros(op.cout, np.float32)]
eng.set_keras_weights(ws)
x = eng.to_compute(torch.rand(a.batch, *shape, device="cuda:0"))
eng.forward(x)
torch.cuda.synchronize()
runs, names = [], []
for rep in range(a.reps):
    timing, kern = [], []
    eng.forward(x, timing=timing, kernels=kern)
    torch.cuda.synchronize()
    runs.append([s.elapsed_time(e) for s, e in timing])
    names = kern
med = np.median(np.array(runs), axis=0)
tot = float(med.sum())
print(json.dumps({"model": a.model, "batch": a.batch, "dtype": a.dtype, "total_ms": round(tot, 4),
                  "launches": [{"kernel": n[:90], "ms": round(float(t), 4),
                                "share": round(float(t) / tot, 3)} for n, t in zip(names, med)]}))
