"""Per-layer A/B of the C5 autoencoder forward (GPU): HIP-event times of every launch at
the bench's launch shape, for each environment variant given on the command line.

    python tools/layer_ab.py [--batch 2048] [--reps 20] "" "SPECENH_PATCH_WSPLIT=0" ...

Each variant is a space-separated list of NAME=VALUE kernel switches (SPECENH_CONV_NO_ROWS=1,
...), applied through specenh_set_variant (the library reads the environment only once) and
reset to their defaults between variants. Variants are interleaved per repetition so clock
drift hits them alike; medians are printed."""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import bench  # noqa: E402
from specenh import _lib, ae  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    variants = a.variants or [""]
    dev = torch.device("cuda", 0)
    ops = []
    for lay in bench.ae_layers():
        ops.append(ae.PoolOp() if lay[0] == "pool" else
                   ae.ConvOp(lay[0], lay[1], lay[2], lay[3], lay[4],
                             stride=2 if lay[0] == "convT" else 1))
    names_used = {kv.split("=", 1)[0] for v in variants for kv in v.split()}
    defaults = {k: _lib.get_variant(k) for k in names_used}

    def apply(v):
        for k, val in defaults.items():
            _lib.set_variant(k, val)
        for kv in v.split():
            k, val = kv.split("=", 1)
            _lib.set_variant(k, int(val))

    # one engine per variant, built under its switches (the engine picks its fusions, e.g.
    # SPECENH_ENCODER_UNFUSED / DECODER_UNFUSED, at construction)
    engs = {}
    for v in variants:
        apply(v)
        e = ae.AutoencoderEngine(ops, (128, 128, 1), compute_dtype="float16", device=dev)
        e.set_keras_weights(bench.ae_weights())
        engs[v] = e
    eng = engs[variants[0]]
    x = eng.to_compute(torch.rand(a.batch, 128, 128, 1, device=dev))
    res = {v: [] for v in variants}
    for rep in range(a.reps + 2):
        for v in variants:
            apply(v)
            timing = []
            engs[v].forward(x, timing=timing)
            torch.cuda.synchronize()
            if rep >= 2:
                res[v].append([s.elapsed_time(e) for s, e in timing])
    names = bench.layer_names(eng)
    if len({len(r[0]) for r in res.values()}) > 1:  # variants with different launch lists
        for v in variants:
            med = np.median(np.array(res[v]), axis=0)
            print((v or "default").ljust(40) + " ".join(f"{m:.4f}" for m in med) +
                  f"  total {med.sum():.4f}")
        return
    print("variant".ljust(40) + "".join(n.rjust(17) for n in names) + "total".rjust(10))
    for v in variants:
        med = np.median(np.array(res[v]), axis=0)
        print((v or "default").ljust(40) + "".join(f"{m:17.4f}" for m in med) +
              f"{med.sum():10.4f}")


if __name__ == "__main__":
    main()
