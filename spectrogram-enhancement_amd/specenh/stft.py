"""Batched STFT-PSD on the GPU: plan cache + the tensor API over ``torch.ops.specenh.stft_psd``.

Tensor-in / tensor-out fast path behind ``pipeline_data.specgr`` (SURVEY.md §8(b)
B1/B2). The arithmetic is the HIP kernel in csrc/stft_psd.hip, reached through the
operator ``torch.ops.specenh.stft_psd[_out]`` (specenh/ops.py) and the C-ABI
``specenh_stft_psd`` (include/specenh.h); this module validates arguments and
builds/caches plans (window + twiddle tables resident on the device).

Semantics follow scipy.signal.spectrogram as called by
spec_denoising/pipeline_data.py:32 (mode='psd', one-sided, no boundary padding),
plus the optional log / min-max / drop-Nyquist post-processing of :33-35.
"""
from __future__ import annotations

import ctypes
import functools
import hashlib
import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib


@functools.lru_cache(maxsize=64)
def _named_window(window, nperseg: int) -> np.ndarray:
    import scipy.signal

    w = np.asarray(scipy.signal.get_window(window, nperseg), dtype=np.float64)
    w.setflags(write=False)
    return w


def get_window(window, nperseg: int) -> np.ndarray:
    """Periodic window as scipy.signal.spectrogram builds it (get_window(..., fftbins=True)).

    Host-side coefficient generation (nperseg numbers); the reference's
    ``spec_params['window']`` strings ('hamm', 'hann', ...) are resolved by scipy,
    which is the reference's own definition of those names.
    """
    if isinstance(window, (str, tuple)):
        return _named_window(window, int(nperseg))
    w = np.asarray(window, dtype=np.float64)
    if w.ndim != 1 or w.shape[0] != nperseg:
        raise ValueError("window must be 1-D with length nperseg")
    return w


def frame_count(length: int, nperseg: int, noverlap: int) -> int:
    return int(_lib.check(_lib.lib().specenh_stft_frames(int(length), int(nperseg), int(noverlap)),
                          "stft_frames"))


def frequencies(nperseg: int, fs: float) -> np.ndarray:
    """scipy's ``rfftfreq(nfft, 1/fs)`` (_spectral_py.py:2115), bit-identical."""
    val = 1.0 / (nperseg * (1.0 / fs))
    return np.arange(0, nperseg // 2 + 1, dtype=np.int64) * val


def times(length: int, nperseg: int, noverlap: int, fs: float) -> np.ndarray:
    """scipy's ``arange(nperseg/2, L-nperseg/2+1, step)/fs`` (_spectral_py.py:2136)."""
    return np.arange(nperseg / 2, length - nperseg / 2 + 1, nperseg - noverlap) / float(fs)


@dataclass(frozen=True)
class PlanKey:
    device: int
    nperseg: int
    noverlap: int
    window_digest: str
    fs: float
    scaling: int
    detrend: int
    eps: float


class StftPlan:
    """Owns a ``specenh_stft_plan`` (device-resident window and twiddle tables)."""

    def __init__(self, key: PlanKey, window: np.ndarray):
        self.key = key
        L = _lib.lib()
        h = ctypes.c_void_p()
        w = np.ascontiguousarray(window, dtype=np.float64)
        with torch.cuda.device(key.device):
            _lib.check(L.specenh_stft_plan_create(
                ctypes.byref(h), key.nperseg, key.noverlap,
                w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), key.fs, key.scaling,
                key.detrend, key.eps), "stft_plan_create")
        self.handle = h

    def workspace(self, batch: int, device) -> torch.Tensor:
        """A fresh workspace per call from torch's caching allocator on the current stream
        (the team schedule's timeout word, granules and tile flags live here): two streams
        sharing one plan never share a workspace, and a buffer returns to the pool only
        when the stream that used it is done with it."""
        nbytes = int(_lib.lib().specenh_stft_workspace_bytes(self.handle, batch))
        return torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.lib().specenh_stft_plan_destroy(self.handle)
        except Exception:
            pass


_plans: dict = {}
_plans_lock = threading.Lock()


def _norm_detrend(detrend) -> int:
    if callable(detrend):
        raise NotImplementedError("callable detrend is not supported on the GPU path")
    if detrend is True:
        raise ValueError("Trend type must be 'linear' or 'constant'.")
    try:
        return _lib.DETREND[detrend]
    except (KeyError, TypeError):
        raise ValueError("Trend type must be 'linear' or 'constant'.") from None


def _norm_scaling(scaling) -> int:
    try:
        return _lib.SCALING[scaling]
    except (KeyError, TypeError):
        raise ValueError(f"Unknown scaling: {scaling!r}") from None


def get_plan(device: torch.device, nperseg: int, noverlap: int, window="hann", fs: float = 1.0,
             scaling="density", detrend="linear", eps: float = 1e-11) -> StftPlan:
    from .ops import window_key
    return get_plan_key(device, nperseg, noverlap, window_key(window, nperseg), fs,
                        _norm_scaling(scaling), _norm_detrend(detrend), eps)


_fast: dict = {}


def get_plan_key(device: torch.device, nperseg: int, noverlap: int, window: str, fs: float,
                 scaling: int, detrend: int, eps: float) -> StftPlan:
    """Plan lookup from the operator's arguments (window by name / registered key)."""
    dev = device.index if device.index is not None else torch.cuda.current_device()
    fk = (dev, nperseg, noverlap, window, fs, scaling, detrend, eps)
    p = _fast.get(fk)
    if p is not None:
        return p
    from .ops import window_coefs
    nperseg = int(nperseg)
    noverlap = int(noverlap)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    w = window_coefs(window, nperseg)
    key = PlanKey(dev, nperseg, noverlap, hashlib.sha1(w.tobytes()).hexdigest(), float(fs),
                  int(scaling), int(detrend), float(eps))
    with _plans_lock:
        p = _plans.get(key)
        if p is None:
            p = _plans[key] = StftPlan(key, w)
        _fast[fk] = p
    return p


def _launch(plan: StftPlan, x: torch.Tensor, out: torch.Tensor, flags: int, workspace=None):
    """Direct C-ABI launch on a plan (tests use it for the development flags and an explicit
    workspace); the API below goes through torch.ops.specenh.stft_psd_out."""
    L = _lib.lib()
    st = ctypes.c_void_p(_lib.current_stream_handle(x.device))
    if x.dtype == torch.float16:
        _lib.check(L.specenh_stft_psd_f16(plan.handle, ctypes.c_void_p(x.data_ptr()), x.shape[0],
                                          x.shape[1], x.stride(0),
                                          ctypes.c_void_p(out.data_ptr()), flags, st),
                   "stft_psd_f16")
        return
    ws = plan.workspace(x.shape[0], x.device) if workspace is None else workspace
    _lib.check(L.specenh_stft_psd(plan.handle, ctypes.c_void_p(x.data_ptr()), x.shape[0],
                                  x.shape[1], x.stride(0), ctypes.c_void_p(out.data_ptr()), flags,
                                  ctypes.c_void_p(ws.data_ptr()), st), "stft_psd")


def _check_input(x: torch.Tensor) -> torch.Tensor:
    if not isinstance(x, torch.Tensor):
        raise TypeError("x must be a torch.Tensor")
    if x.device.type != "cuda":
        raise RuntimeError("specenh.stft_psd runs on the GPU only (no CPU fallback); "
                           "move the signal to a ROCm device first")
    if x.dim() == 1:
        x = x.unsqueeze(0)
    if x.dim() != 2:
        raise ValueError("x must be [batch, length]")
    if x.dtype not in (torch.float32, torch.float16):
        x = x.float()
    if x.stride(1) != 1:
        x = x.contiguous()
    return x


def stft_psd(x: torch.Tensor, nperseg: int, noverlap: int, window="hann", fs: float = 1.0,
             scaling="density", detrend="linear", eps: float = 1e-11, log: bool = False,
             normalize: bool = False, drop_nyquist: bool = False,
             out: torch.Tensor | None = None, exact: bool = False) -> torch.Tensor:
    """Batched spectrogram of ``x[B, L]`` (fp32 or fp16 samples, on a ROCm device) ->
    ``[B, F, T]`` fp32 (fp16 samples are widened on load; the arithmetic is fp32).

    ``F = nperseg//2 + 1`` (``nperseg//2`` with ``drop_nyquist``),
    ``T = (L - nperseg)//(nperseg - noverlap) + 1``.
    ``normalize`` implies ``log`` (the specgr chain of pipeline_data.py:33-35).
    ``exact``: one real frame per complex FFT instead of two (SPECENH_STFT_EXACT; twice the
    FFT work): keeps bins at spectral nulls free of the partner frame's rounding.
    """
    from .ops import ops, window_key
    squeeze = x.dim() == 1
    x = _check_input(x)
    nperseg, noverlap = int(nperseg), int(noverlap)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    T = frame_count(x.shape[1], nperseg, noverlap)
    F = nperseg // 2 + (0 if drop_nyquist else 1)
    flags = ((_lib.STFT_LOG if log else 0) | (_lib.STFT_NORMALIZE if normalize else 0)
             | (_lib.STFT_DROP_NYQUIST if drop_nyquist else 0)
             | (_lib.STFT_EXACT if exact else 0))
    if out is None:
        out = torch.empty((x.shape[0], F, T), dtype=torch.float32, device=x.device)
    elif out.shape != (x.shape[0], F, T) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be contiguous float32 of shape {(x.shape[0], F, T)}")
    ops.stft_psd_out(x, nperseg, noverlap, window_key(window, nperseg), float(fs),
                     _norm_scaling(scaling), _norm_detrend(detrend), float(eps), flags, out)
    return out[0] if squeeze else out
