"""Cross-power spectrograms (interferometer/crosspowerspec.py:39).

The oracle (oracle.spectrogram.cross_spectrogram) is pinned against scipy's own
two-signal spectral helper (tests/golden/csd.npz, tests/golden/make_golden_csd.py);
the GPU path (csrc/cross_spectrum.hip via specenh_csd) is checked against both.
Tolerances: f/t bit-exact; Pxy normwise ||d||_inf / ||P||_inf <= 1e-5 for the fp32 GPU
path (and for the fp64 oracle vs scipy's fp32 arithmetic on fp32 inputs), 1e-10 for the
fp64 oracle vs scipy on fp64 inputs. ae_co2 itself is absent: parity unpinned."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import spectrogram as ref

G = load_golden("csd")
CASES = sorted({k.split("/")[0] for k in G})
PARAMS = {  # mirrors tests/golden/make_golden_csd.py
    "hann256_const_density_f64": (256, 128, "hann", "constant", "density"),
    "hamm512_lin_density_f32": (512, 256, "hamm", "linear", "density"),
    "blackman1024_none_spectrum_f64": (1024, 768, "blackman", False, "spectrum"),
    "hann64_lin_density_f32": (64, 48, "hann", "linear", "density"),
}


def _nrel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_scipy_cross_helper(case):
    n, ov, win, det, sc = PARAMS[case]
    x, y = G[f"{case}/x"], G[f"{case}/y"]
    f, t, P = ref.cross_spectrogram(x, y, 5e5, win, n, ov, det, sc)
    assert np.array_equal(f, G[f"{case}/f"]) and np.array_equal(t, G[f"{case}/t"])
    assert P.shape == G[f"{case}/P"].shape
    tol = 1e-10 if x.dtype == np.float64 else 1e-5
    assert _nrel(P, G[f"{case}/P"]) <= tol


def test_oracle_same_signal_is_the_psd():
    x = G["hann256_const_density_f64/x"]
    _, _, P = ref.cross_spectrogram(x, x, 5e5, "hann", 256, 128, "linear", "density")
    _, _, S = ref.spectrogram_psd(x, 5e5, "hann", 256, 128, "linear", "density")
    assert np.abs(P.imag).max() <= 1e-12 * np.abs(S).max()
    assert _nrel(P.real, S) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_matches_scipy_golden(case, gpu_device):
    from specenh import cross

    n, ov, win, det, sc = PARAMS[case]
    x, y = G[f"{case}/x"], G[f"{case}/y"]
    f, t, P = cross.cross_spectrogram(x, y, 5e5, win, n, ov, det, sc)
    assert np.array_equal(f, G[f"{case}/f"]) and np.array_equal(t, G[f"{case}/t"])
    assert P.shape == G[f"{case}/P"].shape
    assert _nrel(P, G[f"{case}/P"]) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("n,ov", [(128, 64), (2048, 1536), (4096, 0)])
def test_gpu_batched_pairs_and_amplitude(gpu_device, n, ov):
    import torch

    from specenh import cross
    from specenh.synthetic import plasma_chirps

    L = 3 * n + 77
    xy = plasma_chirps(10, L, seed0=90 + n, dtype=np.float32)
    x, y = torch.as_tensor(xy[:5], device=gpu_device), torch.as_tensor(xy[5:], device=gpu_device)
    f, t, P = cross.cross_spectrogram_batch(x, y, 5e5, "hann", n, ov, "linear", "density")
    _, _, A = cross.cross_spectrogram_batch(x, y, 5e5, "hann", n, ov, "linear", "density",
                                            amplitude=True)
    torch.cuda.synchronize()
    P = P.cpu().numpy()
    A = A.cpu().numpy()
    for b in range(5):
        _, _, R = ref.cross_spectrogram(xy[b].astype(np.float64), xy[5 + b].astype(np.float64),
                                        5e5, "hann", n, ov, "linear", "density")
        assert _nrel(P[b], R) <= 1e-5
        # amplitude: the STFT team schedule (nperseg <= 1024) or csd_kernel (larger)
        assert _nrel(A[b], np.abs(R)) <= 1e-5
    assert _nrel(A, np.abs(P)) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("n,ov,win,det,sc", [(1024, 768, "hamm", "linear", "density"),
                                             (512, 256, "hann", "constant", "spectrum"),
                                             (256, 128, "blackman", False, "density"),
                                             (64, 32, "hann", "linear", "density")])
def test_gpu_amplitude_team_schedule(gpu_device, n, ov, win, det, sc):
    """|Pxy| on the STFT team kernel (MODE 3) at many frames per pair, strided rows,
    against the fp64 oracle: every tile, the ragged last tile and the DC/Nyquist rows."""
    import torch

    from specenh import cross
    from specenh.synthetic import plasma_chirps

    hop = n - ov
    L = 61 * hop + n + 13  # 62 frames: several tiles plus a ragged one
    xy = plasma_chirps(6, L, seed0=300 + n, dtype=np.float32)
    big = torch.as_tensor(np.pad(xy, ((0, 0), (0, 40))), device=gpu_device)
    x, y = big[:3, :L], big[3:, :L]  # row stride L + 40
    _, _, A = cross.cross_spectrogram_batch(x, y, 5e5, win, n, ov, det, sc, amplitude=True)
    torch.cuda.synchronize()
    A = A.cpu().numpy()
    for b in range(3):
        _, _, R = ref.cross_spectrogram(xy[b].astype(np.float64), xy[3 + b].astype(np.float64),
                                        5e5, win, n, ov, det, sc)
        assert A[b].shape == R.shape
        assert _nrel(A[b], np.abs(R)) <= 1e-5, (b, _nrel(A[b], np.abs(R)))


@pytest.mark.gpu
def test_gpu_csd_and_ae_co2_call_shape(gpu_device):
    from specenh import cross

    x, y = G["hann256_const_density_f64/x"], G["hann256_const_density_f64/y"]
    f, Pm = cross.csd(x, y, fs=5e5)  # scipy.signal.csd defaults
    _, _, R = ref.cross_spectrogram(x, y, 5e5)
    assert _nrel(Pm, R.mean(axis=-1)) <= 1e-5
    t = np.arange(x.size) / 5e5 + 1.25
    amp, fk, tm = cross.crosspower_amplitude(x, y, t)
    _, tt, R2 = ref.cross_spectrogram(x, y, 5e5, "hamm", 512, 256, "linear", "density")
    assert amp.shape == R2.shape[::-1] and fk.shape == (257,) and tm.shape == tt.shape
    assert _nrel(amp, np.abs(R2).T) <= 1e-5
    assert np.allclose(tm, (tt + 1.25) * 1e3) and fk[-1] == pytest.approx(250.0, rel=1e-9)


@pytest.mark.gpu
def test_gpu_errors(gpu_device):
    import torch

    from specenh import cross

    x = torch.zeros(2, 4000, device=gpu_device)
    with pytest.raises(ValueError):
        cross.cross_spectrogram_batch(x, x, nperseg=256, noverlap=256)
    with pytest.raises(NotImplementedError):
        cross.cross_spectrogram_batch(x, x, nperseg=300, noverlap=100)
    with pytest.raises(ValueError):
        cross.cross_spectrogram_batch(x, x[:1], nperseg=256)
    with pytest.raises(RuntimeError):
        cross.cross_spectrogram_batch(x.cpu(), x.cpu(), nperseg=256)
