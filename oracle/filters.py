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


# ---------------------------------------------------------------- cv2 steps (unpinned)
# gaussblr (:52-55) and morph (:64-72) run OpenCV on uint8 images. OpenCV is absent here,
# so these restate its documented 8-bit algorithms (parity unpinned):
#   * ``(rescale(src)*255).astype('uint8')``: float -> uint8 truncation (numpy astype).
#   * ``cv2.GaussianBlur(u8, (kw, kh), 0)``: separable, sigma from ksize when 0
#     (0.3*((n-1)/2 - 1) + 0.8; n <= 7 odd uses the fixed small tables), taps normalised to
#     sum 1 and quantised to 8 fractional bits by error diffusion (centre tap takes the
#     remainder so the taps sum to exactly 256); rows then columns in integer arithmetic,
#     final (v + 2^15) >> 16; BORDER_REFLECT_101.
#   * ``cv2.morphologyEx`` CLOSE with a 4x4 rect then OPEN with a 3x1 (w x h) rect:
#     dilate = max, erode = min over src(y + i - ay, x + j - ax) with the anchor at the
#     kernel centre (k // 2) for both; pixels outside the image are ignored (OpenCV's
#     default morphology border value).

_SMALL_GAUSS = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
                7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}


def gaussian_taps_q8(n: int, sigma: float = 0.0) -> np.ndarray:
    """Integer taps (sum 256) of an n-tap OpenCV Gaussian for 8-bit images."""
    if n % 2 != 1 or n < 1:
        raise ValueError("Gaussian kernel size must be odd and positive")
    if n <= 7 and sigma <= 0:
        k = np.asarray(_SMALL_GAUSS[n], dtype=np.float64)
    else:
        s = sigma if sigma > 0 else ((n - 1) * 0.5 - 1) * 0.3 + 0.8
        scale2 = -0.5 / (s * s)
        x = np.arange(n, dtype=np.float64) - (n - 1) * 0.5
        v = np.exp(scale2 * x * x)
        half = n // 2
        tot = 2.0 * float(np.sum(v[:half])) + 1.0
        k = v / tot
        k[half] = 1.0 / tot
    half = n // 2
    out = np.zeros(n, dtype=np.int64)
    err, tot = 0.0, 0
    for i in range(half):  # error diffusion from the outside in
        adj = k[i] * 256.0 + err
        q = int(np.rint(adj))
        err = adj - q
        out[i] = out[n - 1 - i] = q
        tot += q
    out[half] = 256 - 2 * tot
    return out


def _reflect101(idx: np.ndarray, n: int) -> np.ndarray:
    if n == 1:
        return np.zeros_like(idx)
    idx = idx.copy()
    for _ in range(64):
        idx = np.where(idx < 0, -idx, idx)
        idx = np.where(idx >= n, 2 * n - 2 - idx, idx)
        if ((idx >= 0) & (idx < n)).all():
            break
    return idx


def to_u8(src):
    """(rescale(src) * 255).astype('uint8') (:53, :65)."""
    return (rescale(src) * 255).astype(np.uint8)


def gaussian_blur_u8(u8: np.ndarray, ksize=(31, 3), sigma: float = 0.0) -> np.ndarray:
    kw, kh = ksize
    kx, ky = gaussian_taps_q8(kw, sigma), gaussian_taps_q8(kh, sigma)
    rows, cols = u8.shape
    a = u8.astype(np.int64)
    ci = _reflect101(np.arange(cols)[:, None] + np.arange(kw)[None, :] - kw // 2, cols)
    h = (a[:, ci] * kx[None, None, :]).sum(axis=2)            # Q8 row sums
    ri = _reflect101(np.arange(rows)[:, None] + np.arange(kh)[None, :] - kh // 2, rows)
    v = (h[ri, :] * ky[None, :, None]).sum(axis=1)            # Q16
    return np.minimum((v + (1 << 15)) >> 16, 255).astype(np.uint8)


def _morph_u8(a: np.ndarray, kh: int, kw: int, is_max: bool) -> np.ndarray:
    rows, cols = a.shape
    ay, ax = kh // 2, kw // 2
    fill = 0 if is_max else 255
    pad = np.full((rows + kh, cols + kw), fill, dtype=np.uint8)
    pad[ay:ay + rows, ax:ax + cols] = a
    out = None
    for i in range(kh):
        for j in range(kw):
            w = pad[i:i + rows, j:j + cols]
            out = w.copy() if out is None else (np.maximum(out, w) if is_max else np.minimum(out, w))
    return out


def morph_u8(u8: np.ndarray) -> np.ndarray:
    """CLOSE 4x4 then OPEN 3x1 (w x h) on uint8 (:66-70)."""
    c = _morph_u8(_morph_u8(u8, 4, 4, True), 4, 4, False)
    return _morph_u8(_morph_u8(c, 1, 3, False), 1, 3, True)


def rescale_u8(u8: np.ndarray) -> np.ndarray:
    """rescale() of a uint8 image as numpy evaluates it: uint8 differences, true divide."""
    mn, mx = u8.min(), u8.max()
    with np.errstate(invalid="ignore", divide="ignore"):
        return (u8 - mn) / (mx - mn)


def gaussblr(src, filt=(31, 3)):
    return rescale_u8(gaussian_blur_u8(to_u8(src), filt))


def morph(src):
    return rescale_u8(morph_u8(to_u8(src)))


def label_pipeline(s, thr=0.9):
    """pipeline_data.py:101-110: quantfilt -> gaussblr -> meansub -> morph -> meansub."""
    return meansub(morph(meansub(gaussblr(quantfilt(s, thr), (31, 3)))))
