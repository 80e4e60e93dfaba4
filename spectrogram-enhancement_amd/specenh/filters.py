"""GPU label filters: norm / rescale / meansub / quantfilt / gaussblr / morph of
spec_denoising/pipeline_data.py (:38-72) through ``torch.ops.specenh`` (csrc/filters.hip), and the
whole label chain of its main loop (:101-110) as ``label_pipeline``. The reference-named functions live in
``specenh.pipeline_data``; this module holds the device paths.

  * numpy input (the reference's float64 spectrograms): uploaded unchanged, computed in
    fp64 on the GPU, returned as float64 numpy (numpy's formulas; fp64 sums reordered).
  * torch input on the GPU (float32 / float64): device-resident; 2-D = one spectrogram,
    3-D ``[B, rows, cols]`` = a batch, every spectrogram filtered independently.
N-D numpy inputs keep the reference's whole-array semantics: norm / rescale over all
elements, quantfilt per column of axis 0, meansub over axis 1 with one global rescale.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

_DT = {torch.float32: 0, torch.float64: 3}


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("specenh requires a ROCm GPU (HIP); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _run(kind, t: torch.Tensor, arg):
    """t: device tensor [B, rows, cols] float32/float64 -> torch.ops.specenh.<filter>."""
    from .ops import ops
    if t.device.type != "cuda":
        raise RuntimeError("specenh.filters runs on the GPU only (no CPU fallback)")
    if t.dtype not in _DT:
        t = t.double()
    t = t.contiguous()
    if kind == "gaussblr":
        kw, kh = arg
        return ops.gaussblr(t, int(kw), int(kh), 0.0)
    if kind == "morph":
        return ops.morph(t)
    if kind == "quantfilt":
        return ops.quantfilt(t, float(arg))
    return ops.label_filter(t, int(arg))


def _apply(kind, src, arg, to2d, back):
    if isinstance(src, torch.Tensor):
        if src.dim() == 2:
            return _run(kind, src.unsqueeze(0), arg)[0]
        if src.dim() == 3:
            return _run(kind, src, arg)
        raise ValueError("device tensors must be [rows, cols] or [batch, rows, cols]")
    a = np.asarray(src)
    if a.dtype != np.float32:
        a = a.astype(np.float64)
    a2 = to2d(a)
    t = torch.as_tensor(np.ascontiguousarray(a2), device=_device()).unsqueeze(0)
    return back(_run(kind, t, arg)[0].cpu().numpy(), a)


def norm(data):
    return _apply("norm", data, _lib.FILTER_NORM, lambda a: a.reshape(1, -1),
                  lambda r, a: r.reshape(a.shape))


def rescale(data):
    return _apply("rescale", data, _lib.FILTER_RESCALE, lambda a: a.reshape(1, -1),
                  lambda r, a: r.reshape(a.shape))


def quantfilt(src, thr=0.9):
    return _apply("quantfilt", src, thr, lambda a: a.reshape(a.shape[0], -1),
                  lambda r, a: r.reshape(a.shape))


def meansub(src):
    def to2d(a):  # rows = every index but axis 1, cols = axis 1
        m = np.moveaxis(a, 1, -1)
        return m.reshape(-1, a.shape[1])

    def back(r, a):
        m = np.moveaxis(a, 1, -1)
        return np.moveaxis(r.reshape(m.shape), -1, 1)

    return _apply("meansub", src, _lib.FILTER_MEANSUB, to2d, back)


def _image2d(a):
    if a.ndim != 2:
        raise ValueError("cv2 filters take one 2-D image (or a [batch, rows, cols] device tensor)")
    return a


def gaussblr(src, filt=(31, 3)):
    """pipeline_data.py:52-55: uint8 quantisation, cv2.GaussianBlur(u8, filt, 0), rescale.
    ``filt`` is OpenCV's (width, height): width taps along columns (time), height along rows."""
    kw, kh = (int(filt[0]), int(filt[1]))
    return _apply("gaussblr", src, (kw, kh), _image2d, lambda r, a: r)


def morph(src):
    """pipeline_data.py:64-72: uint8 quantisation, MORPH_CLOSE 4x4 then MORPH_OPEN 3x1, rescale."""
    return _apply("morph", src, None, _image2d, lambda r, a: r)


def label_pipeline(s, thr=0.9):
    """The label chain of pipeline_data.py:101-110 on the GPU:
    quantfilt(thr) -> gaussblr((31, 3)) -> meansub -> morph -> meansub.
    numpy in -> float64 numpy out; a device tensor (2-D or [B, rows, cols]) stays on device."""
    if isinstance(s, torch.Tensor):
        t = s
    else:
        a = np.asarray(s)
        if a.ndim != 2:
            raise ValueError("label_pipeline takes one 2-D spectrogram (or a device batch)")
        t = torch.as_tensor(np.ascontiguousarray(a.astype(np.float64)), device=_device())
    out = meansub(morph(meansub(gaussblr(quantfilt(t, thr), (31, 3)))))
    return out if isinstance(s, torch.Tensor) else out.cpu().numpy()
