"""Autoencoder weights with non-degenerate outputs for the parity tests and the bench.

Glorot weights with zero biases (the reference's untrained init) put the 3-layer AE's
outputs at 0.5 +- 4e-4 (logits |z| < 0.01): a kernel that wrote a constant would pass a
PSNR-at-peak-1 check. These weights are the oracle's own fp32 Keras-Adam training
(oracle/autoencoder.py train_step: BCE from logits, lr 1e-3) of the reference model
(VAE/manual_scan_3layers.py:186-212) on C4-style data: inputs are the C1 spectrograms
(256 hann / hop 128 -> 128 x 128) of seeded noisy chirps after denoiseSignal's default,
targets the spectrograms of the same chirps without noise (SURVEY.md §8 d, C4). After
training the logits span O(1), so output errors are measured against a real signal.

Test infrastructure (uses the oracle); the result is committed as ae_c4_trained.npz.
Usage:  python tests/golden/make_ae_weights.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]

from oracle import autoencoder as ora  # noqa: E402
from oracle import svd as osvd  # noqa: E402
from oracle.spectrogram import specgr_arrays  # noqa: E402
from specenh.synthetic import plasma_chirps  # noqa: E402

SPEC1 = {"nperseg": 256, "noverlap": 128, "fs": 500000, "window": "hann",
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
L1 = 16512


def c4_pairs(n, seed0):
    """(noisy input after denoiseSignal default, clean target), NHWC float32."""
    noisy = plasma_chirps(n, L1, seed0=seed0, dtype=np.float64)
    clean = plasma_chirps(n, L1, seed0=seed0, sigma=0.0, dtype=np.float64)
    x = np.empty((n, 128, 128, 1), np.float32)
    y = np.empty((n, 128, 128, 1), np.float32)
    for i in range(n):
        S, _, _ = specgr_arrays(noisy[i], SPEC1)
        x[i, :, :, 0] = osvd.denoiseSignal(S)
        y[i, :, :, 0] = specgr_arrays(clean[i], SPEC1)[0]
    return x, y


def main(n=256, steps=400, batch=16, seed=0):
    torch.manual_seed(seed)
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    spec = ora.ae_spec()
    params = ora.glorot_params(spec, seed=seed)
    tp = [None if p is None else {"W": torch.tensor(p["W"], requires_grad=True),
                                  "b": torch.tensor(p["b"], requires_grad=True)}
          for p in params]
    x, y = c4_pairs(n, seed0=5000)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    opt = ora.KerasAdam()
    rng = np.random.default_rng(seed)
    t0 = time.time()
    for s in range(steps):
        idx = rng.choice(n, batch, replace=False)
        loss = ora.train_step(spec, tp, xt[idx], yt[idx], opt)
        if s % 20 == 0 or s == steps - 1:
            print(f"step {s}: loss {loss:.5f} ({time.time() - t0:.0f} s)")
    ws = []
    for p in tp:
        if p is not None:
            ws += [p["W"].detach().numpy().astype(np.float32),
                   p["b"].detach().numpy().astype(np.float32)]
    with torch.no_grad():
        out, z = ora.forward(spec, tp, xt[:16], return_logits=True)
    print(f"logits mean {float(z.mean()):.3f} std {float(z.std()):.3f}; "
          f"outputs mean {float(out.mean()):.3f} std {float(out.std()):.3f}")
    np.savez_compressed(os.path.join(HERE, "ae_c4_trained.npz"),
                        **{f"w{i:02d}": w for i, w in enumerate(ws)})


def load(path=os.path.join(HERE, "ae_c4_trained.npz")):
    """[kernel0, bias0, ...] in Keras shapes (the committed fixture)."""
    with np.load(path, allow_pickle=False) as d:
        return [d[k] for k in sorted(d.files)]


if __name__ == "__main__":
    main()
