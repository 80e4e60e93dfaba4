"""GPU parity of the SVD denoiser (denoising_by_svd.ipynb:188-229) through the C-ABI.

Tolerance: ||GPU - ref||_F / ||ref||_F <= 1e-5 on inputs with a
spectral gap at the cut (fp32 GPU vs the notebook's own float64 output). Reconstructions
are compared, never U/V (sign/rotation ambiguity)."""
import numpy as np
import pytest

from conftest import load_golden, svd_cases
from oracle import svd as ref

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.mark.parametrize("case", svd_cases())
def test_denoise_matches_notebook(case, gpu_device):
    from specenh import svd

    g = load_golden(f"svd_{case}")
    A = g["A"]
    r = min(A.shape)
    for key, args in [("default", ()), ("r16", (0, 16)), ("s2_10", (2, 10)),
                      ("clamp", (-3, 10_000))]:
        out = svd.denoiseSignal(A, *args)
        assert out.dtype == np.float64 and out.shape == A.shape
        # fp32 input path: compare to the notebook's output on the same (fp32-cast) matrix
        assert _rel(out, g[key]) <= (TOL if key != "clamp" else 1e-6), (key, _rel(out, g[key]))
    assert not np.any(svd.denoiseSignal(A, 7, 3))
    assert svd.omega(r / max(A.shape)) == pytest.approx(float(g["omega_beta"]), abs=0)


def test_batched_gapped_c3_shape(gpu_device):
    """BASELINE config 3 geometry (513 x 256) on a batch of gapped matrices, rank-16."""
    import torch

    from specenh import svd
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    A = np.stack([gapped_matrix(900 + i, 513, 256, dtype=np.float32) for i in range(8)])
    out = svd.denoise_batch(torch.as_tensor(A, device=gpu_device), 0, 16).double().cpu().numpy()
    default = svd.denoise_batch(torch.as_tensor(A, device=gpu_device)).double().cpu().numpy()
    for b in range(8):
        assert _rel(out[b], ref.denoiseSignal(A[b].astype(np.float64), 0, 16)) <= TOL
        assert _rel(default[b], ref.denoiseSignal(A[b].astype(np.float64))) <= TOL


def test_wide_matrix_reference_usage(gpu_device):
    """The notebook's real call: denoiseSignal(s) on a (256, T) spectrogram, m < n."""
    from specenh import pipeline_data, svd
    from specenh.synthetic import plasma_chirps

    x = plasma_chirps(1, 65792, seed0=31, dtype=np.float64)[0]
    p = {"nperseg": 512, "noverlap": 256, "fs": 500000, "window": "hamm",
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
    S, _, _ = pipeline_data.specgr_array(x, p)            # (256, 256) spectrogram
    Sw = np.concatenate([S, S[:, ::-1]], axis=1)          # (256, 512): m < n
    out = svd.denoiseSignal(Sw)
    assert _rel(out, ref.denoiseSignal(Sw.astype(np.float32).astype(np.float64))) <= 1e-4


def test_unsupported_modes_raise(gpu_device):
    from specenh import svd

    A = np.random.default_rng(0).standard_normal((64, 48))
    with pytest.raises(NotImplementedError):
        svd.denoiseSignal(A, use_optimal=True)
    with pytest.raises(NotImplementedError):
        svd.computeSignal(A)
    big = np.random.default_rng(1).standard_normal((128, 96))
    with pytest.raises(NotImplementedError):
        svd.denoiseSignal(big, 0, 80)   # needs a top-80 subspace (> 40)
