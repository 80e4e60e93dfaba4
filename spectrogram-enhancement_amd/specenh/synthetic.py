"""Synthetic plasma time-series ("Synthetic plasma time-series").

The reference reads ECE/BES shots from pickles on a cluster filesystem
(``spec_denoising/pipeline_data.py:29-31``); none of that data ships, so every
test, fixture and benchmark in this repo drives the hot path with seeded chirps:

    x[n] = sum_{m=1..3} A_m sin(2*pi*(f0_m t + k_m t^2 / 2) + phi_m)
           + sigma * N(0, 1) + d * n / L,          t = n / fs

with f0 ~ U[10, 200] kHz, k ~ U[-5e5, 5e5] Hz/s, A ~ U[0.2, 1], phi ~ U[0, 2pi),
sigma = 0.5 and a linear drift d ~ U[-1, 1] (so that the linear detrend of
``pipeline_data.py:32`` has something to remove).

``plasma_chirps`` is the byte-exact generator (numpy PCG64, one stream per shot:
``default_rng(seed0 + shot)``); golden fixtures store only its seed and a digest.
``plasma_chirps_torch`` is a device-side generator of the same *shape* of signal
used by the benchmark, where bit-exactness with numpy is not needed.
"""
from __future__ import annotations

import hashlib

import numpy as np

FS_DEFAULT = 500_000.0


def _one_shot(rng: np.random.Generator, length: int, fs: float, n_tones: int,
              sigma: float) -> np.ndarray:
    n = np.arange(length, dtype=np.float64)
    t = n / fs
    x = np.zeros(length, dtype=np.float64)
    for _ in range(n_tones):
        f0 = rng.uniform(10e3, 200e3)
        k = rng.uniform(-5e5, 5e5)
        amp = rng.uniform(0.2, 1.0)
        phi = rng.uniform(0.0, 2.0 * np.pi)
        x += amp * np.sin(2.0 * np.pi * (f0 * t + 0.5 * k * t * t) + phi)
    if sigma:
        x += sigma * rng.standard_normal(length)
    else:
        rng.standard_normal(length)  # keep the stream aligned with sigma > 0
    x += rng.uniform(-1.0, 1.0) * n / length
    return x


def plasma_chirps(n_shots: int, length: int, seed0: int = 0, fs: float = FS_DEFAULT,
                  n_tones: int = 3, sigma: float = 0.5,
                  dtype=np.float32) -> np.ndarray:
    """Return ``(n_shots, length)`` seeded synthetic shots (byte-exact, numpy PCG64)."""
    out = np.empty((n_shots, length), dtype=dtype)
    for s in range(n_shots):
        rng = np.random.default_rng(seed0 + s)
        out[s] = _one_shot(rng, length, fs, n_tones, sigma)
    return out


def digest(a: np.ndarray) -> str:
    """sha256 of the array bytes (C order) — pins fixtures to the generator."""
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def plasma_chirps_torch(n_shots: int, length: int, seed: int = 0, fs: float = FS_DEFAULT,
                        n_tones: int = 3, sigma: float = 0.5, device="cuda",
                        dtype=None, chunk: int = 256):
    """Device-side generator with the same statistics (not bit-identical to numpy).

    Used for benchmark-sized batches (4096 x 65536) that would take minutes to
    synthesise on the host. Generated in chunks of shots to bound temporaries.
    """
    import torch

    dtype = dtype or torch.float32
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((n_shots, length), device=device, dtype=dtype)
    n = torch.arange(length, device=device, dtype=torch.float64)
    t = n / fs
    for s0 in range(0, n_shots, chunk):
        b = min(chunk, n_shots - s0)
        x = torch.zeros((b, length), device=device, dtype=torch.float64)
        for _ in range(n_tones):
            u = torch.rand((b, 4), generator=g, device=device, dtype=torch.float64)
            f0 = 10e3 + 190e3 * u[:, 0:1]
            k = -5e5 + 1e6 * u[:, 1:2]
            amp = 0.2 + 0.8 * u[:, 2:3]
            phi = 2.0 * np.pi * u[:, 3:4]
            x += amp * torch.sin(2.0 * np.pi * (f0 * t + 0.5 * k * t * t) + phi)
        x += sigma * torch.randn((b, length), generator=g, device=device, dtype=torch.float64)
        d = -1.0 + 2.0 * torch.rand((b, 1), generator=g, device=device, dtype=torch.float64)
        x += d * n / length
        out[s0:s0 + b] = x.to(dtype)
    return out


# BASELINE config 4 / SURVEY.md §8(d) C4: C1-style spectrograms (16,512 samples, hann 256 /
# hop 128 -> 128 x 128, specgr's log + min-max) of seeded noisy chirps as inputs, the
# spectrograms of the same chirps without noise (sigma = 0), normalised identically, as
# targets: a synthetic stand-in for the cv2 label pipeline (pipeline_data.py:101-110).
C4_LENGTH = 16512
C4_SPEC = {"nperseg": 256, "noverlap": 128, "fs": 500000, "window": "hann",
           "scaling": "density", "detrend": "linear", "eps": 1e-11}


def c4_pairs_torch(n: int, seed: int = 0, device="cuda", dtype=None, chunk: int = 2048):
    """Device C4 pairs ``(x, y)`` [n, 128, 128, 1] (``dtype``, default fp32) generated and
    transformed on the GPU (plasma_chirps_torch -> specgr_batch): the bench's training set.
    The noisy and clean shots of one seed share every chirp parameter (the noise draw is
    made either way)."""
    import torch

    from .pipeline_data import specgr_batch

    dtype = dtype or torch.float32
    x = torch.empty((n, 128, 128, 1), dtype=dtype, device=device)
    y = torch.empty_like(x)
    S = torch.empty((min(n, chunk), 128, 128), dtype=torch.float32, device=device)
    for s0 in range(0, n, chunk):
        b = min(chunk, n - s0)
        for dst, sigma in ((x, 0.5), (y, 0.0)):
            sh = plasma_chirps_torch(b, C4_LENGTH, seed=seed + s0, sigma=sigma, device=device)
            specgr_batch(sh, C4_SPEC, out=S[:b])
            dst[s0:s0 + b, :, :, 0] = S[:b].to(dtype)
            del sh
    return x, y
