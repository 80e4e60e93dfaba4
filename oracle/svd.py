"""ORACLE (test infrastructure only): the SVD spectrogram denoiser.

Restates ``spec_denoising/denoising_by_svd.ipynb`` code cell 1:
  * ``omega``          (:155-159)  Gavish-Donoho polynomial 0.56b^3-0.95b^2+1.82b+1.43
  * ``computeSignal``  (:161-186)  sum of s_i u_i v_i^T for i in [1, 2*num_sing)
  * ``denoiseSignal``  (:188-229)  thin SVD, keep components [start, stop):
      defaults start=1, stop=r (i.e. A minus its top component);
      use_optimal: start=0, stop=num_sing-1 with num_sing = #(s > omega(beta)*median(s));
      clamps start<0 -> 0 and stop>r -> r (:224-227), then slices u[:, start:stop] with
      Python semantics (:228): a negative stop counts from the end (stop + r, floored at 0),
      so use_optimal with num_sing == 0 (stop = -1) keeps [0, r-1); an empty slice gives
      zeros.
The arithmetic is numpy -> LAPACK gesdd; here it is evaluated in float64.
Pinned by tests/test_oracle_golden.py against the notebook's own outputs.
"""
from __future__ import annotations

import numpy as np


def omega(beta: float) -> float:
    coef = [0.56, -0.95, 1.82, 1.43]
    poly = [beta ** (3 - n) for n in range(4)]
    return sum(c * p for c, p in zip(coef, poly))


def optimal_rank(s: np.ndarray, shape) -> int:
    beta = np.min(shape) / np.max(shape)
    t_star = omega(beta) * np.median(s)
    return int((s > t_star).sum())


def slice_bounds(r: int, start: int, stop: int):
    """Python's slice s[start:stop] on a length-r axis as [lo, hi) (start already >= 0)."""
    sl = range(r)[start:stop]
    return sl.start, max(sl.stop, sl.start)


def resolve_range(r: int, start=None, stop=None, use_optimal=False, s=None, shape=None):
    """The start/stop logic of denoiseSignal (:210-228), returned as the kept [lo, hi)."""
    if use_optimal:
        num_sing = optimal_rank(s, shape)
        start, stop = 0, num_sing - 1
    else:
        if start is None:
            start = 1
        if stop is None:
            stop = r
    if start < 0:
        start = 0
    if stop > r:
        stop = r
    return slice_bounds(r, int(start), int(stop))


def denoiseSignal(matrix, start=None, stop=None, use_optimal=False):
    a = np.asarray(matrix, dtype=np.float64)
    u, s, vh = np.linalg.svd(a, full_matrices=False)
    lo, hi = resolve_range(len(s), start, stop, use_optimal, s, a.shape)
    if hi <= lo:
        return np.zeros_like(a)
    return (u[:, lo:hi] * s[lo:hi]) @ vh[lo:hi, :]


def computeSignal(matrix):
    a = np.asarray(matrix, dtype=np.float64)
    u, s, vh = np.linalg.svd(a, full_matrices=False)
    num_sing = optimal_rank(s, a.shape)
    out = np.zeros_like(a)
    for idx in range(1, 2 * num_sing):
        out += s[idx] * np.outer(u[:, idx], vh[idx, :])
    return out
