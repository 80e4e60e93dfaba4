"""Why the production-shot STFT misses 1e-5 by 2% at one bin: an fp32 emulation of the
kernel's FFT arithmetic (stft_psd.hip: radix-32 DIF in registers, fp32 twiddle multiply,
radix-16 DIF; fp32 twiddles, FMA complex products) on frames 2440-2459 of channel 1 of the
production shot (tests/test_reference_shapes_gpu.py), run ONE frame per complex FFT and TWO
frames per FFT (z = a + i b, the kernel's two-for-one), against an fp64 FFT of the same
fp32-rounded windowed frames, next to scipy.fft.rfft of the same fp32 frames (what
scipy.signal.spectrogram runs on fp32 input; numpy's rfft computes fp32 input in fp64).
CPU only:  python tools/stft_pair_error.py

Result (max |ln PSD error| over bins >= 3 of the 20 frames; the worst bin is a spectral null
1e-6 below its neighbours): kernel arithmetic with one frame per FFT 8.3e-5 (3.4e-5 at frame
2450 bin 116), two-for-one 3.2e-4 (1.5e-4 at frame 2450 bin 116; the GPU's 1.0165e-5
normalised error there is 1.78e-4 in ln PSD). The separation A_k = (Z_k + conj Z_{N-k}) / 2
inherits the partner frame's rounding at bin k, which at a null of frame a is relatively
large. scipy's fp32 rfft: 3.8e-4 max (its absolute error at the frame-2448 null is 1.07e-6,
the kernel's one-frame FFT 2.9e-7): the paired kernel sits at scipy's own fp32 level.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
from specenh.synthetic import plasma_chirps  # noqa: E402

f32 = np.float32


def r32(a):
    return a.astype(np.float32)


def cmul(d, wr, wi):  # fft_common.hpp pk::cmul: (fma(d.x, w.x, -d.y w.y), fma(d.x, w.y, d.y w.x))
    dr, di = d
    t1 = r32(-(di.astype(np.float64) * wi))
    t2 = r32(di.astype(np.float64) * wr)
    return r32(dr.astype(np.float64) * wr + t1), r32(dr.astype(np.float64) * wi + t2)


def tw(k, m):
    a = -2 * np.pi * k / m
    return f32(np.cos(a)), f32(np.sin(a))


def dif(v):  # fft_dif<R>: radix-2 DIF, trivial twiddles free; v[r] ends at bin bitrev(r)
    R = len(v)
    H = R // 2
    while H >= 1:
        for S in range(0, R, 2 * H):
            for K in range(H):
                a, b = v[S + K], v[S + K + H]
                v[S + K] = (r32(a[0] + b[0]), r32(a[1] + b[1]))
                d = (r32(a[0] - b[0]), r32(a[1] - b[1]))
                if K == 0:
                    v[S + K + H] = d
                elif 4 * K == 2 * H:
                    v[S + K + H] = (d[1], r32(-d[0]))
                else:
                    v[S + K + H] = cmul(d, *tw(K, 2 * H))
        H //= 2
    return v


def bitrev(v, bits):
    return int(format(v, "0%db" % bits)[::-1], 2)


def fft_kernel(zr, zi, N, R1):
    """Cfg<512>: R1-point DIF over r (stride N/R1), twiddle W_N^{b k1}, N/R1-point DIF."""
    NB1 = N // R1
    lb1, lb2 = int(np.log2(R1)), int(np.log2(NB1))
    vals = dif([(zr[:, r * NB1:(r + 1) * NB1], zi[:, r * NB1:(r + 1) * NB1]) for r in range(R1)])
    A = [None] * R1
    for r in range(R1):
        A[bitrev(r, lb1)] = vals[r]
    b = np.arange(NB1)
    out_r, out_i = np.empty_like(zr), np.empty_like(zi)
    for k1 in range(R1):
        ang = -2 * np.pi * ((b * k1) % N) / N
        A[k1] = cmul(A[k1], f32(np.cos(ang)), f32(np.sin(ang)))
        v2 = dif([(A[k1][0][:, j], A[k1][1][:, j]) for j in range(NB1)])
        for r in range(NB1):
            k2 = bitrev(r, lb2)
            out_r[:, k1 + R1 * k2], out_i[:, k1 + R1 * k2] = v2[r]
    return out_r, out_i


def main():
    from scipy.signal import get_window

    x = plasma_chirps(3, 1_200_000, seed0=11, dtype=np.float32)[1][:1_000_000]
    N, hop = 512, 256
    w = get_window("hamming", N)
    fr = np.arange(2440, 2460)
    F = x[fr[:, None] * hop + np.arange(N)[None, :]].astype(np.float64)
    n = np.arange(N) - 0.5 * (N - 1)
    y = F - F.mean(1, keepdims=True) - (F * n).sum(1, keepdims=True) / (n * n).sum() * n
    yw = r32(y * w)  # the FFT's input rounded to fp32: only FFT rounding is compared
    P64 = np.abs(np.fft.rfft(yw.astype(np.float64), axis=1)) ** 2
    zr, zi = fft_kernel(yw, np.zeros_like(yw), N, 32)
    P1 = (zr.astype(np.float64) ** 2 + zi.astype(np.float64) ** 2)[:, :257]
    zr, zi = fft_kernel(yw[0::2], yw[1::2], N, 32)
    Z = zr.astype(np.float64) + 1j * zi
    k = np.arange(257)
    m = (-k) % N
    P2 = np.empty((len(fr), 257))
    P2[0::2] = np.abs((Z[:, k] + np.conj(Z[:, m])) / 2) ** 2
    P2[1::2] = np.abs((Z[:, k] - np.conj(Z[:, m])) / 2j) ** 2
    import scipy.fft
    Pn = np.abs(scipy.fft.rfft(yw, axis=1).astype(np.complex128)) ** 2
    for name, P in [("scipy.fft fp32", Pn), ("kernel, one frame per FFT", P1),
                    ("kernel, two-for-one", P2)]:
        d = np.abs(np.log(P[:, :256]) - np.log(P64[:, :256]))
        d[:, :3] = 0
        i = np.unravel_index(d.argmax(), d.shape)
        print(f"{name:28s} max ln err {d.max():.2e} at frame {fr[i[0]]} bin {i[1]}; "
              f"frame 2450 bin 116: {d[10, 116]:.2e}")


if __name__ == "__main__":
    main()
