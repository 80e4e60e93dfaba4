"""Can the STFT's DFT stages run on the matrix cores at the §8(d) 1e-5 bound? An fp32/fp16
emulation of a two-stage matrix DFT (N = R1 x R2: an R1-point DFT over n1 as one real matrix
product per frame, the W_N^{n2 k1} twiddle on the vector unit, an R2-point complex DFT over n2
as a second product) with every operand split into fp16 hi + lo and the products
hi*hi + hi*lo + lo*hi (optionally + lo*lo) accumulated in fp32, as v_mfma_f32_32x32x16_f16
would run them. Operands are scaled per frame by a power of two into fp16's range first.
The normalised log spectrogram (pipeline_data.py:32-35; DC bin from the fp64 path as in the
kernel) is compared with the fp64 truth of the same fp32 samples.

CPU only:  python tools/stft_mfma_emul.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
from oracle import spectrogram as ref  # noqa: E402
from specenh.synthetic import plasma_chirps  # noqa: E402

f16, f32 = np.float16, np.float32


def split(a, terms):
    """fp32 -> fp16 hi (+ lo) after a per-row power-of-two scale into [2^13, 2^14)."""
    m = np.abs(a).max(axis=-1, keepdims=True)
    e = np.where(m > 0, 13 - np.floor(np.log2(np.where(m > 0, m, 1))), 0)
    s = np.exp2(e).astype(f32)
    a = (a * s).astype(f32)
    hi = a.astype(f16)
    lo = (a - hi.astype(f32)).astype(f16)
    return hi, lo, s


def mm(a, b, terms):
    """a [..., M, K] (data, scaled per frame) @ b [K, N] (constant matrix) in split fp16."""
    a2 = a.reshape(-1, a.shape[-1])
    ah, al, s = split(a2, terms)
    bh = b.astype(f16)
    bl = (b - bh.astype(f32)).astype(f16)
    h = lambda x: x.astype(f32)  # noqa: E731  (fp16 * fp16 is exact in fp32)
    r = h(ah) @ h(bh) + h(ah) @ h(bl) + h(al) @ h(bh)
    if terms == 4:
        r = r + h(al) @ h(bl)
    return (r / s).astype(f32).reshape(a.shape[:-1] + (b.shape[1],))


def matrix_dft(y, R1, terms):
    """X[k] of real frames y [F, N] (fp32) via the two-stage split-fp16 matrix DFT."""
    F, N = y.shape
    R2 = N // R1
    n1 = np.arange(R1)
    W1 = np.exp(-2j * np.pi * np.outer(n1, n1) / R1)  # [n1, k1]
    X = y.reshape(F, R1, R2).transpose(0, 2, 1)  # [F, n2, n1]
    Yr = mm(X, W1.real.astype(f32), terms)  # [F, n2, k1]
    Yi = mm(X, W1.imag.astype(f32), terms)
    n2 = np.arange(R2)
    tw = np.exp(-2j * np.pi * np.outer(n2, n1) / N)  # [n2, k1]
    twr, twi = tw.real.astype(f32), tw.imag.astype(f32)
    Tr = (Yr * twr - Yi * twi).astype(f32)
    Ti = (Yr * twi + Yi * twr).astype(f32)
    # stage B over n2: rows (frame, k1), [Tr Ti] @ [[Cr, Ci], [-Ci, Cr]]
    W2 = np.exp(-2j * np.pi * np.outer(n2, n2) / R2)  # [n2, k2]
    B = np.block([[W2.real, W2.imag], [-W2.imag, W2.real]]).astype(f32)
    A = np.concatenate([Tr.transpose(0, 2, 1), Ti.transpose(0, 2, 1)], axis=-1)  # [F, k1, 2 R2]
    Z = mm(A, B, terms)  # [F, k1, 2 R2]
    Xc = Z[..., :R2].astype(np.float64) + 1j * Z[..., R2:]
    return Xc.transpose(0, 2, 1).reshape(F, N)  # k = k1 + R1 k2


def spectrogram_emul(x, p, R1, terms):
    N, hop = p["nperseg"], p["nperseg"] - p["noverlap"]
    w = ref.get_window(p["window"], N)
    T = (len(x) - N) // hop + 1
    fr = x[np.arange(T)[:, None] * hop + np.arange(N)[None, :]].astype(np.float64)
    n = np.arange(N) - 0.5 * (N - 1)
    yv = fr - fr.mean(1, keepdims=True) - (fr * n).sum(1, keepdims=True) / (n * n).sum() * n
    y = (yv * w).astype(f32)
    X = matrix_dft(y, R1, terms)[:, : N // 2 + 1]
    scale = 1.0 / (p["fs"] * (w * w).sum())
    P = np.abs(X) ** 2 * scale
    P[:, 1:-1] *= 2
    P[:, 0] = np.abs((yv * w).sum(1)) ** 2 * scale  # DC from the fp64 path
    return ref.log_minmax(P.T, p["eps"])


def main():
    cases = [("C2 hamm1024", 1024, 768, "hamm", 65536, 32, 0),
             ("prod hamm512", 512, 256, "hamm", 1_000_000, 16, 1)]
    for name, N, nov, win, L, R1, ch in cases:
        p = {"nperseg": N, "noverlap": nov, "fs": 500000, "window": win, "scaling": "density",
             "detrend": "linear", "eps": 1e-11}
        if name.startswith("prod"):
            xs = plasma_chirps(3, 1_200_000, seed0=11, dtype=np.float32)[:, :L]
        else:
            xs = plasma_chirps(3, L, seed0=7, dtype=np.float32)
        for terms in (3, 4):
            errs = []
            for x in xs:
                truth, _, _ = ref.specgr_arrays(x.astype(np.float64), p)
                S = spectrogram_emul(x, p, R1, terms)
                errs.append(np.abs(S - truth).max())
            print(f"{name:14s} R1={R1:2d} terms={terms}: max |err| per shot "
                  + " ".join(f"{e:.2e}" for e in errs))


if __name__ == "__main__":
    main()
