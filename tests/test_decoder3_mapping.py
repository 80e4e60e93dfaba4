"""CPU check of decoder3's map-free Conv2D(1) (csrc/decoder_tail.hip, decoder3_kernel<T, false>).

The consumer waves never store the 16-channel map: each tail step packs its Conv2DTranspose
accumulators (map rows 2tl, 2tl + 1; 16 positions x 16 channels x 4 phases per wave) into the
B operand of v_mfma_f32_16x16x32 and multiplies them by six weight fragments wd[d][py] into
three rolling output-row-pair accumulators; a completed pair is finished with two DPP row
shifts (columns from positions m - 1 / m + 1) and, at the 16-position block edges, one word
exchanged between waves. Here every lane's fragment is built by the kernel's formulas and the
MFMA is evaluated by its lane layout (A[i][k] in lane i + 16 (k / 8), B[k][n] in lane
n + 16 (k / 8), D[i][n] in lane n + 16 (i / 4), register i % 4), then compared with the plain
5 x 5 'same' convolution (VAE/manual_scan_3layers.py:199, Conv2D(1, 5, sigmoid)).
"""
import numpy as np
import pytest

KO, CO, MW = 5, 16, 128


def wd_fragments(w):
    """wd[d][py][lane][8]: the kernel's A fragments (w: [5][5][16] Conv2D(1) weights)."""
    wd = np.zeros((3, 2, 64, 8))
    for lane in range(64):
        i, kA = lane & 15, lane >> 4
        gO, j = i >> 2, i & 3
        r, o = gO >> 1, gO & 1
        ox = o + {0: 0, 1: 2, 2: -2, 3: 0}[j]
        for d in range(3):
            for py in range(2):
                ky = py + 2 - 2 * (d - 1) - r
                for el in range(8):
                    px, c = el >> 2, el & 3
                    kx = px + 2 - ox
                    if j < 3 and 0 <= ky < KO and 0 <= kx < KO:
                        wd[d, py, lane, el] = w[ky, kx, 4 * kA + c]
    return wd


def mfma(a, b, acc):
    """v_mfma_f32_16x16x32 by lane layout: a, b [64][8] fragments, acc [64][4]."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for lane in range(64):
        A[lane & 15, 8 * (lane >> 4):8 * (lane >> 4) + 8] = a[lane]
        B[8 * (lane >> 4):8 * (lane >> 4) + 8, lane & 15] = b[lane]
    D = A @ B
    out = acc.copy()
    for lane in range(64):
        for j in range(4):
            out[lane, j] += D[4 * (lane >> 4) + j, lane & 15]
    return out


def decoder3_conv_out(M, w, bo):
    """The consumer's schedule on a map M [H3][128][16] (rows >= H3 zero) -> pre-sigmoid out."""
    H3 = M.shape[0]
    H2 = H3 // 2
    TPI = H2 + 2
    wd = wd_fragments(w)
    Mp = np.zeros((2 * TPI, MW, CO))
    Mp[:H3] = M
    out = np.full((H3, MW), np.nan)
    P = [np.zeros((4, 64, 4)) for _ in range(3)]  # per wave: P0, P1, P2
    for tl in range(TPI):
        E = np.zeros((4, 64, 4))
        for wv in range(4):
            bv = np.zeros((2, 64, 8))
            if tl < H2:
                for lane in range(64):
                    m, kg = lane & 15, lane >> 4
                    for py in range(2):
                        for px in range(2):
                            bv[py, lane, 4 * px:4 * px + 4] = \
                                Mp[2 * tl + py, 32 * wv + 2 * m + px, 4 * kg:4 * kg + 4]
            for py in range(2):
                for d in range(3):
                    P[d][wv] = mfma(wd[d, py], bv[py], P[d][wv])
            E[wv] = P[0][wv]
        P = [P[1], P[2], np.zeros((4, 64, 4))]
        if not 1 <= tl <= H2:
            continue
        for wv in range(4):
            for lane in range(64):
                m, g = lane & 15, lane >> 4
                s = bo + E[wv, lane, 0]
                # DPP row_shr:1 / row_shl:1 inside the 16-lane row, else the neighbour wave
                if m > 0:
                    s += E[wv, lane - 1, 1]
                elif wv > 0:
                    s += E[wv - 1, 15 + 16 * g, 1]
                if m < 15:
                    s += E[wv, lane + 1, 2]
                elif wv < 3:
                    s += E[wv + 1, 16 * g, 2]
                out[2 * (tl - 1) + (g >> 1), 32 * wv + 2 * m + (g & 1)] = s
    return out


def conv_same(M, w, bo):
    H3 = M.shape[0]
    pad = np.zeros((H3 + 4, MW + 4, CO))
    pad[2:-2, 2:-2] = M
    out = np.full((H3, MW), bo)
    for ky in range(KO):
        for kx in range(KO):
            out += pad[ky:ky + H3, kx:kx + MW] @ w[ky, kx]
    return out


@pytest.mark.parametrize("H1", [1, 2, 3])
def test_mapfree_conv_out_matches_conv(H1):
    rng = np.random.default_rng(7 + H1)
    M = np.maximum(rng.standard_normal((4 * H1, MW, CO)), 0)
    w = rng.standard_normal((KO, KO, CO))
    got = decoder3_conv_out(M, w, 0.3)
    ref = conv_same(M, w, 0.3)
    assert not np.isnan(got).any()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-10)
