"""ORACLE (test infrastructure only): spectrogram PSD + specgr post-processing.

Restates, in numpy, the arithmetic the reference reaches through
``scipy.signal.spectrogram`` (a third-party dependency the reference does not
vendor or pin; the container has scipy 1.15.3) and the post-processing of
``specgr`` itself:

* ``spec_denoising/pipeline_data.py:28-36``  specgr: cut, spectrogram, log(S+eps),
  whole-spectrogram min-max, drop the last (Nyquist) row of S and f.
* ``scipy/signal/_spectral_py.py:1863-2155`` (_spectral_helper) and ``:2158-2204``
  (_fft_helper): frames ``x[k*step : k*step+N]`` (no padding/boundary for
  ``spectrogram``), per-frame detrend, window multiply, ``rfft``, ``conj(X)*X``,
  ``scale = 1/(fs*sum(w^2))`` ('density') or ``1/sum(w)^2`` ('spectrum'),
  one-sided doubling of bins ``1..N/2-1`` (even N), ``f = rfftfreq(N, 1/fs)``,
  ``t = arange(N/2, L-N/2+1, step)/fs``.
* ``scipy/signal/_signaltools.py:3905-3960`` detrend: 'linear' is the least-squares
  line fit ``A=[(1..N)/N, 1]`` per frame (restated in closed form), 'constant'
  subtracts the mean.

Pinned by tests/test_oracle_golden.py against fixtures produced by the
reference's own specgr (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np


def get_window(window, nperseg: int) -> np.ndarray:
    """Periodic ('DFT-even') window exactly as scipy.signal.spectrogram builds it.

    ``_spectral_py.py:_triage_segments`` -> ``get_window(window, nperseg)`` with
    the default ``fftbins=True``. Window *coefficient generation* is delegated to
    scipy (it is the reference's own specification of e.g. 'hamm'); an explicit
    array is passed through.
    """
    if isinstance(window, (str, tuple)):
        import scipy.signal

        return scipy.signal.get_window(window, nperseg)
    w = np.asarray(window, dtype=np.float64)
    if w.shape != (nperseg,):
        raise ValueError("window must be 1-D of length nperseg")
    return w


def frequencies(nperseg: int, fs: float) -> np.ndarray:
    """``f = rfftfreq(nfft, 1/fs)`` (``_spectral_py.py:2115``): arange(n//2+1) * (1/(n*d))."""
    val = 1.0 / (nperseg * (1.0 / fs))
    return np.arange(0, nperseg // 2 + 1, dtype=np.int64) * val


def times(length: int, nperseg: int, noverlap: int, fs: float) -> np.ndarray:
    """``arange(nperseg/2, L - nperseg/2 + 1, step)/fs`` (``_spectral_py.py:2136``)."""
    return np.arange(nperseg / 2, length - nperseg / 2 + 1, nperseg - noverlap) / float(fs)


def _detrend(frames: np.ndarray, kind) -> np.ndarray:
    """Per-frame detrend along the last axis (``_signaltools.py:3922-3960``)."""
    if not kind:
        return frames
    if kind in ("constant", "c"):
        return frames - frames.mean(axis=-1, keepdims=True)
    if kind in ("linear", "l"):
        n = frames.shape[-1]
        # Least squares of y on [n, 1]; closed form with a centred abscissa.
        k = np.arange(n, dtype=np.float64) - (n - 1) / 2.0
        mean = frames.mean(axis=-1, keepdims=True)
        slope = (frames * k).sum(axis=-1, keepdims=True) / (k * k).sum()
        return frames - mean - slope * k
    raise ValueError("Trend type must be 'linear' or 'constant'.")


def spectrogram_psd(x, fs: float = 1.0, window="hann", nperseg: int = 256,
                    noverlap: int | None = None, detrend="linear", scaling="density",
                    compute_dtype=np.float64):
    """(f, t, Sxx[..., F, T]) with ``scipy.signal.spectrogram(mode='psd')`` semantics."""
    x = np.asarray(x)
    if noverlap is None:
        noverlap = nperseg // 8  # spectrogram's own default (_spectral_py.py:972)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    step = nperseg - noverlap
    length = x.shape[-1]
    if length < nperseg:
        raise ValueError("nperseg must not exceed the signal length")
    win = get_window(window, nperseg)
    if scaling == "density":
        scale = 1.0 / (fs * (win * win).sum())
    elif scaling == "spectrum":
        scale = 1.0 / win.sum() ** 2
    else:
        raise ValueError(f"Unknown scaling: {scaling!r}")
    frames = np.lib.stride_tricks.sliding_window_view(x, nperseg, axis=-1)[..., ::step, :]
    frames = frames.astype(compute_dtype)
    y = _detrend(frames, detrend) * win.astype(compute_dtype)
    X = np.fft.rfft(y, n=nperseg, axis=-1)
    P = (X.real * X.real + X.imag * X.imag) * scale
    if nperseg % 2:
        P[..., 1:] *= 2
    else:
        P[..., 1:-1] *= 2
    P = np.moveaxis(P, -1, -2)  # (..., F, T): frequency-major like scipy
    return frequencies(nperseg, fs), times(length, nperseg, noverlap, fs), P


def log_minmax(P: np.ndarray, eps: float, drop_nyquist: bool = True) -> np.ndarray:
    """``pipeline_data.py:33-35``: log(S+eps), per-spectrogram min-max over ALL rows,
    then drop the last row. Reductions are over the last two axes (one spectrogram)."""
    L = np.log(P + eps)
    mn = L.min(axis=(-2, -1), keepdims=True)
    mx = L.max(axis=(-2, -1), keepdims=True)
    with np.errstate(invalid="ignore", divide="ignore"):
        S = (L - mn) / (mx - mn)
    return S[..., :-1, :] if drop_nyquist else S


def specgr_arrays(x, spec_params: dict, cut_shot: float = 2):
    """The array part of ``specgr`` (``pipeline_data.py:28-36``) for 1-D or batched x."""
    x = np.asarray(x)
    x = x[..., : np.int_(cut_shot * spec_params["fs"])]
    f, t, P = spectrogram_psd(x, fs=spec_params["fs"], window=spec_params["window"],
                              nperseg=spec_params["nperseg"],
                              noverlap=spec_params["noverlap"],
                              detrend=spec_params["detrend"],
                              scaling=spec_params["scaling"])
    S = log_minmax(P, spec_params["eps"])
    return S, f[:-1], t


def specgr_scipy(x, spec_params: dict):
    """The reference's exact call chain (``pipeline_data.py:32-35``) on an array, via scipy.

    This is the CPU baseline timed by bench.py (the reference path minus pickle I/O).
    """
    import scipy.signal

    f, t, S = scipy.signal.spectrogram(x, nperseg=spec_params["nperseg"],
                                       noverlap=spec_params["noverlap"], fs=spec_params["fs"],
                                       window=spec_params["window"],
                                       scaling=spec_params["scaling"],
                                       detrend=spec_params["detrend"])
    S = np.log(S + spec_params["eps"])
    S = (S - np.min(S)) / (np.max(S) - np.min(S))
    return S[:-1, :], f[:-1], t


def cross_spectrogram(x, y, fs: float = 1.0, window="hann", nperseg: int = 256,
                      noverlap: int | None = None, detrend="constant", scaling="density",
                      compute_dtype=np.float64):
    """(f, t, Pxy[..., F, T]): scipy's two-signal ``_spectral_helper(x, y, mode='psd')``
    (``_spectral_py.py`` ``if not same_data: result = np.conjugate(result) * result_y``,
    then ``result *= scale`` and the one-sided doubling), the un-averaged
    ``scipy.signal.csd`` — what ``ae_co2`` (interferometer/crosspowerspec.py:39, source
    absent) stands for. Same framing / detrend / window / scale as :func:`spectrogram_psd`;
    ``noverlap`` defaults to ``nperseg // 2`` as in csd."""
    x = np.asarray(x)
    y = np.asarray(y)
    if noverlap is None:
        noverlap = nperseg // 2
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    step = nperseg - noverlap
    win = get_window(window, nperseg)
    scale = 1.0 / (fs * (win * win).sum()) if scaling == "density" else 1.0 / win.sum() ** 2

    def spec(sig):
        fr = np.lib.stride_tricks.sliding_window_view(sig, nperseg, axis=-1)[..., ::step, :]
        return np.fft.rfft(_detrend(fr.astype(compute_dtype), detrend) * win, axis=-1)

    P = np.conjugate(spec(x)) * spec(y) * scale
    if nperseg % 2:
        P[..., 1:] *= 2
    else:
        P[..., 1:-1] *= 2
    P = np.moveaxis(P, -1, -2)
    return frequencies(nperseg, fs), times(x.shape[-1], nperseg, noverlap, fs), P
