"""Cross-power spectrograms of signal pairs on the GPU.

interferometer/crosspowerspec.py:39 calls ``ampsp, freq, time = ae_co2(signal1[i],
signal2[i], t)`` from ``co2_deps`` — a module absent from the reference — and plots
``np.log(ampsp).T`` with frequency in kHz and time in ms (:46-50), so ``ampsp`` is
``(time, freq)``. What it stands for is scipy's two-signal spectral helper
(``scipy/signal/_spectral_py.py`` ``_spectral_helper(x, y, mode='psd')``): per frame
``Pxy = conj(X) * Y * scale`` with one-sided doubling, the un-averaged form of
``scipy.signal.csd``. That arithmetic is what runs here (csrc/cross_spectrum.hip through
``torch.ops.specenh.csd`` -> ``specenh_csd``), pinned against scipy; ae_co2's own normalisation is unknown
("parity unpinned"), so :func:`crosspower_amplitude` documents the choice it makes.
"""
from __future__ import annotations

import ctypes
import hashlib
import threading

import numpy as np
import torch

from . import _lib
from .stft import _norm_detrend, _norm_scaling, frame_count, frequencies, get_window, times

CSD_COMPLEX, CSD_AMPLITUDE = 0, 1


class CsdPlan:
    """Owns a ``specenh_csd_plan`` (device-resident window and twiddle tables)."""

    def __init__(self, key, window: np.ndarray):
        self.key = key
        dev, nperseg, noverlap, _, fs, scaling, detrend = key
        h = ctypes.c_void_p()
        w = np.ascontiguousarray(window, dtype=np.float64)
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().specenh_csd_plan_create(
                ctypes.byref(h), nperseg, noverlap,
                w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), fs, scaling, detrend),
                "csd_plan_create")
        self.handle = h

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.lib().specenh_csd_plan_destroy(self.handle)
        except Exception:
            pass


_plans: dict = {}
_lock = threading.Lock()


def get_plan_key(device, nperseg, noverlap, window: str, fs, scaling: int, detrend: int) -> CsdPlan:
    """Plan lookup from the csd operator's arguments (window by name / registered key)."""
    from .ops import window_coefs
    nperseg, noverlap = int(nperseg), int(noverlap)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    w = window_coefs(window, nperseg)
    dev = device.index if device.index is not None else torch.cuda.current_device()
    key = (dev, nperseg, noverlap, hashlib.sha1(w.tobytes()).hexdigest(), float(fs),
           int(scaling), int(detrend))
    with _lock:
        p = _plans.get(key)
        if p is None:
            p = _plans[key] = CsdPlan(key, w)
    return p


def _as_pairs(x: torch.Tensor, y: torch.Tensor):
    for name, v in (("x", x), ("y", y)):
        if not isinstance(v, torch.Tensor):
            raise TypeError(f"{name} must be a torch.Tensor")
        if v.device.type != "cuda":
            raise RuntimeError("specenh.cross runs on the GPU only (no CPU fallback)")
    if x.shape != y.shape or x.device != y.device:
        raise ValueError("x and y must have the same shape and device")
    squeeze = x.dim() == 1
    if squeeze:
        x, y = x.unsqueeze(0), y.unsqueeze(0)
    if x.dim() != 2:
        raise ValueError("x and y must be [batch, length]")
    x = x.float() if x.dtype != torch.float32 else x
    y = y.float() if y.dtype != torch.float32 else y
    x = x if x.stride(1) == 1 else x.contiguous()
    y = y if y.stride(1) == 1 else y.contiguous()
    return x, y, squeeze


def cross_spectrogram_batch(x: torch.Tensor, y: torch.Tensor, fs: float = 1.0, window="hann",
                            nperseg: int = 256, noverlap: int | None = None,
                            detrend="constant", scaling="density", amplitude: bool = False):
    """``Pxy[B, F, T]`` (complex64, or ``|Pxy|`` float32 with ``amplitude``) of device signal
    pairs ``x, y[B, L]``, with scipy's ``_spectral_helper(x, y, mode='psd')`` semantics
    (scipy.signal.csd's defaults: hann, 50 % overlap, constant detrend, density).
    Returns ``(f, t, Pxy)``; ``f``/``t`` are float64 numpy arrays bit-equal to scipy's."""
    from .ops import ops, window_key
    x, y, squeeze = _as_pairs(x, y)
    if noverlap is None:
        noverlap = int(nperseg) // 2
    nperseg, noverlap = int(nperseg), int(noverlap)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    L = x.shape[1]
    frame_count(L, nperseg, noverlap)  # ValueError for a signal shorter than nperseg
    out = ops.csd(x, y, nperseg, noverlap, window_key(window, nperseg), float(fs),
                  _norm_scaling(scaling), _norm_detrend(detrend),
                  CSD_AMPLITUDE if amplitude else CSD_COMPLEX)
    f = frequencies(int(nperseg), fs)
    t = times(L, int(nperseg), int(noverlap), fs)
    return f, t, (out[0] if squeeze else out)


def cross_spectrogram(x, y, fs: float = 1.0, window="hann", nperseg: int = 256,
                      noverlap: int | None = None, detrend="constant", scaling="density"):
    """numpy in / numpy out (complex128, like scipy on float64 input): the two-signal
    spectral helper for 1-D or ``[B, L]`` arrays, computed on the current GPU."""
    xt = torch.as_tensor(np.asarray(x, dtype=np.float32), device="cuda")
    yt = torch.as_tensor(np.asarray(y, dtype=np.float32), device="cuda")
    f, t, P = cross_spectrogram_batch(xt, yt, fs, window, nperseg, noverlap, detrend, scaling)
    return f, t, P.cpu().numpy().astype(np.complex128)


def csd(x, y, fs: float = 1.0, window="hann", nperseg: int = 256, noverlap: int | None = None,
        detrend="constant", scaling="density"):
    """``scipy.signal.csd`` (average='mean', one-sided): ``(f, mean_t Pxy)``."""
    f, _, P = cross_spectrogram(x, y, fs, window, nperseg, noverlap, detrend, scaling)
    return f, P.mean(axis=-1)


def crosspower_amplitude(signal1, signal2, t, spec_params: dict | None = None):
    """The call shape of ``ae_co2(signal1, signal2, t)`` (crosspowerspec.py:39):
    returns ``(ampsp[T, F], freq_kHz[F], time_ms[T])`` with ``ampsp = |Pxy|`` per frame,
    ``fs`` from the time base ``t`` (seconds, uniform), frame times offset by ``t[0]``.
    ae_co2's window/normalisation is unknown (co2_deps absent): parity unpinned; the
    defaults below are the reference's own spectrogram parameters (pipeline_data.py:77-84)."""
    p = {"nperseg": 512, "noverlap": 256, "window": "hamm", "scaling": "density",
         "detrend": "linear"}
    p.update(spec_params or {})
    t = np.asarray(t, dtype=np.float64)
    fs = 1.0 / float(t[1] - t[0])
    xt = torch.as_tensor(np.asarray(signal1, dtype=np.float32), device="cuda")
    yt = torch.as_tensor(np.asarray(signal2, dtype=np.float32), device="cuda")
    f, tt, A = cross_spectrogram_batch(xt, yt, fs, p["window"], p["nperseg"], p["noverlap"],
                                       p["detrend"], p["scaling"], amplitude=True)
    return A.T.cpu().numpy().astype(np.float64), f / 1e3, (tt + t[0]) * 1e3
