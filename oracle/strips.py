"""ORACLE (test infrastructure only): the strip layout glue between STFT and the AE.

Restates ``VAE/manual_scan_3layers.py:28-54`` (identical copies in manual_scan.py,
hyperparam_scan.py, graphs.ipynb, denoising_by_svd.ipynb):
  * patch:   ``patchify(S, (256, 128), step=128)[0][x]`` for x < 30 is
             ``S[:, 128x : 128x+128]`` (patchify is absent here; its documented
             non-overlapping-window semantics are restated), stacked to (30n, 256, 128).
  * unpatch: concatenates each run of 30 strips back to (256, 3840).
  * reshape: (N, 256, 128) -> (N, 256, 128, 1) NHWC.
patchify is not installed, so these are parity-unpinned restatements of its
documented behaviour (window views with step == window width).
"""
from __future__ import annotations

import numpy as np


def patch(arr, rows=256, width=128, n_strips=30):
    out = np.empty((len(arr) * n_strips, rows, width))
    for i, s in enumerate(arr):
        s = np.asarray(s)
        for x in range(n_strips):
            out[x + n_strips * i] = s[:rows, width * x: width * x + width]
    return out


def unpatch(arr, n_strips=30):
    arr = np.asarray(arr)
    return np.stack([np.concatenate(list(arr[n_strips * i: n_strips * (i + 1)]), axis=1)
                     for i in range(len(arr) // n_strips)])


def reshape(arr, rows=256, width=128):
    return np.reshape(arr, (len(arr), rows, width, 1))
