"""Drop-in for spec_denoising/pipeline_data.py (the reference's STFT front-end API).

Same names, arguments, return types and exceptions as the reference, so the
reference's scripts and notebooks call it unchanged:

    from specenh.pipeline_data import specgr, norm, rescale, quantfilt, meansub
    s, f, t = specgr(fname, chn + 1, spec_params, 2)        # pipeline_data.py:97

``specgr`` runs the whole spectrogram -> log -> min-max -> drop-Nyquist chain as
one HIP launch pair on the GPU (csrc/stft_psd.hip) and returns float64 numpy
arrays like the reference (computed in fp32 on the device; tolerance in
DESIGN.md). ``specgr_batch`` is the tensor-in/tensor-out fast path that keeps
data on the device.

The image-filter helpers ``norm/rescale/quantfilt/meansub/gaussblr/morph`` (:38-72), the
label-generator chain, run as HIP kernels too (csrc/filters.hip):
numpy inputs come back as float64 numpy, device tensors stay on the device.
``gaussblr``/``morph`` restate OpenCV's GaussianBlur / MORPH_CLOSE+OPEN on the uint8
quantisation (cv2 itself is absent here: their parity rests on that restatement and the
filter goldens).
"""
from __future__ import annotations

import pickle

import numpy as np
import torch

from . import filters as _filters
from . import stft as _stft


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("specenh requires a ROCm GPU (HIP); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _params(spec_params):
    return dict(nperseg=int(spec_params["nperseg"]), noverlap=int(spec_params["noverlap"]),
                fs=spec_params["fs"], window=spec_params["window"],
                scaling=spec_params.get("scaling", "density"),
                detrend=spec_params.get("detrend", "linear"),
                eps=float(spec_params.get("eps", 1e-11)))


def specgr_batch(x: torch.Tensor, spec_params: dict, cut_shot: float | None = None,
                 out: torch.Tensor | None = None, exact: bool = False) -> torch.Tensor:
    """Batched specgr on device tensors: ``x[B, L]`` -> ``Sxx[B, nperseg//2, T]`` fp32.

    Normalisation is per spectrogram (pipeline_data.py:34 applied to each row of x).
    ``exact=True`` runs one frame per FFT (the numpy entries below use it): the default
    two-for-one FFT hands a bin at a spectral null the partner frame's fp32 rounding, which
    on the reference's 1M-sample production shots reaches 1.02e-5.
    """
    p = _params(spec_params)
    if cut_shot is not None:
        x = x[..., : np.int_(cut_shot * p["fs"])]
    return _stft.stft_psd(x, p["nperseg"], p["noverlap"], p["window"], p["fs"], p["scaling"],
                          p["detrend"], p["eps"], log=True, normalize=True, drop_nyquist=True,
                          out=out, exact=exact)


def specgr_array(sig_in, spec_params: dict):
    """specgr on an in-memory 1-D signal: returns (Sxx float64, f, t) like the reference."""
    p = _params(spec_params)
    x = torch.as_tensor(np.ascontiguousarray(sig_in), dtype=torch.float32, device=_device())
    S = specgr_batch(x.unsqueeze(0), spec_params, exact=True)[0]
    f = _stft.frequencies(p["nperseg"], p["fs"])[:-1]
    t = _stft.times(x.shape[-1], p["nperseg"], p["noverlap"], p["fs"])
    return S.double().cpu().numpy(), f, t


def specgr(fname, ecen, spec_params, cut_shot=2, key_format="\\tecef%.2i", field=None):
    """pipeline_data.py:28-36. ``key_format``/``field`` select the BES variant of
    denoising_by_svd.ipynb cell 1 (``'besfu%02d'``, ``'data.BES'``)."""
    with open(fname, "rb") as fh:
        ece_data = pickle.load(fh)  # pickle.UnpicklingError propagates (caller catches it)
    rec = ece_data[key_format % (ecen)]  # KeyError for a missing channel
    if field is not None:
        rec = rec[field]
    sig_in = np.asarray(rec)[: np.int_(cut_shot * spec_params["fs"])]
    return specgr_array(sig_in, spec_params)


# ------------------------------------------------------------- filter helpers
# The label-generator chain (:38-61) on the GPU (csrc/filters.hip via specenh.filters):
# numpy in -> numpy out (float64, like the reference), device tensors stay on the device.
def norm(data):
    """pipeline_data.py:38-41: (data - mean) / std over the whole array."""
    return _filters.norm(data)


def rescale(data):
    """pipeline_data.py:43-44: min-max to [0, 1] over the whole array."""
    return _filters.rescale(data)


def quantfilt(src, thr=0.9):
    """pipeline_data.py:46-49: zero entries below their column's thr-quantile (axis 0)."""
    return _filters.quantfilt(src, thr)


def meansub(src):
    """pipeline_data.py:58-61: |src - mean over axis 1|, then rescale."""
    return _filters.meansub(src)


def gaussblr(src, filt=(31, 3)):
    """pipeline_data.py:52-55: (rescale(src)*255).astype('uint8') -> cv2.GaussianBlur(., filt, 0)
    -> rescale, on the GPU (OpenCV's 8-bit algorithm restated; cv2 absent: parity unpinned)."""
    return _filters.gaussblr(src, filt)


def morph(src):
    """pipeline_data.py:64-72: uint8 quantisation -> MORPH_CLOSE 4x4 -> MORPH_OPEN 3x1 ->
    rescale, on the GPU (OpenCV's 8-bit algorithm restated; cv2 absent: parity unpinned)."""
    return _filters.morph(src)


def label_pipeline(s, thr=0.9):
    """The label chain of pipeline_data.py:101-110 (quantfilt -> gaussblr -> meansub -> morph
    -> meansub) on the GPU."""
    return _filters.label_pipeline(s, thr)
