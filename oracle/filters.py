"""ORACLE (test infrastructure only): the image-filter helpers of pipeline_data.py.

Restates ``spec_denoising/pipeline_data.py``:
  * ``norm``      (:38-41)  (x - mean) / std over the whole array
  * ``rescale``   (:43-44)  min-max to [0, 1] over the whole array
  * ``quantfilt`` (:46-49)  zero every entry below its column's thr-quantile
                            (np.quantile, 'linear' interpolation, axis=0)
  * ``meansub``   (:58-61)  |x - row mean| then rescale
``gaussblr``/``morph`` (:52-55, :64-72) need cv2, which is absent: parity unpinned.
"""
from __future__ import annotations

import numpy as np


def norm(data):
    return (data - data.mean()) / data.std()


def rescale(data):
    return (data - data.min()) / (data.max() - data.min())


def quantile_linear(col_sorted: np.ndarray, q: float) -> np.ndarray:
    """numpy 'linear' quantile on pre-sorted columns (axis 0): h=(n-1)q, lerp."""
    n = col_sorted.shape[0]
    h = (n - 1) * q
    lo = int(np.floor(h))
    hi = min(lo + 1, n - 1)
    frac = h - lo
    a, b = col_sorted[lo], col_sorted[hi]
    return a + (b - a) * frac


def quantfilt(src, thr=0.9):
    filt = np.quantile(src, thr, axis=0)
    return np.where(src < filt, 0, src)


def meansub(src):
    mn = np.mean(src, axis=1)[:, np.newaxis]
    return rescale(np.absolute(src - mn))
