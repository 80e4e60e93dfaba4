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


@pytest.mark.parametrize("case", svd_cases())
def test_optimal_threshold_matches_notebook(case, gpu_device):
    """use_optimal (:210-217): components [0, num_sing - 1) of the Gavish-Donoho threshold;
    num_sing and the median come from the fp64 Gram's eigenvalues on the GPU."""
    import torch

    from specenh import svd

    g = load_golden(f"svd_{case}")
    A = g["A"]
    out = svd.denoiseSignal(A, use_optimal=True)
    assert out.dtype == np.float64 and out.shape == A.shape
    assert _rel(out, g["optimal"]) <= TOL, _rel(out, g["optimal"])
    _, ns, med = svd.optimal_batch(torch.as_tensor(A.astype(np.float32), device=gpu_device),
                                   return_rank=True)
    assert int(ns[0]) == ref.optimal_rank(g["s"], A.shape)
    assert float(med[0]) == pytest.approx(float(np.median(g["s"])), rel=1e-5)


@pytest.mark.parametrize("case", svd_cases())
def test_compute_signal_matches_notebook(case, gpu_device):
    """computeSignal (:161-186): components [1, 2*num_sing). The band ends inside the noise
    bulk (indices 16..31 of ~uniform noise singular values), where the individual noise
    components are not determined to fp32 (no spectral gap): the signal part is pinned to
    1e-5 of the output norm and the rest is bounded by the noise band's own norm."""
    from specenh import svd

    g = load_golden(f"svd_{case}")
    A = g["A"]
    out = svd.computeSignal(A)
    ref_out = g["compute"]
    s = g["s"]
    noise = np.sqrt(np.sum(s[16:] ** 2))
    assert np.linalg.norm(out - ref_out) <= 2 * noise
    # the signal components 1..15 exactly: project out everything past the gap
    u, _, vh = np.linalg.svd(A.astype(np.float64), full_matrices=False)
    P = lambda X: u[:, :16].T @ X @ vh[:16].T  # noqa: E731
    assert _rel(P(out), P(ref_out)) <= TOL


def test_optimal_batched_c3_shape(gpu_device):
    """513 x 256 gapped matrices (BASELINE config 3 geometry), use_optimal in one batch."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    A = np.stack([gapped_matrix(950 + i, 513, 256, dtype=np.float32) for i in range(6)])
    out, ns, _ = svd.optimal_batch(torch.as_tensor(A, device=gpu_device), return_rank=True)
    out = out.double().cpu().numpy()
    for b in range(6):
        r64 = A[b].astype(np.float64)
        assert int(ns[b]) == ref.optimal_rank(np.linalg.svd(r64, compute_uv=False), r64.shape)
        assert _rel(out[b], ref.denoiseSignal(r64, use_optimal=True)) <= TOL


def test_unsupported_modes_raise(gpu_device):
    from specenh import svd

    big = np.random.default_rng(1).standard_normal((128, 96))
    with pytest.raises(NotImplementedError):
        svd.denoiseSignal(big, 0, 80)   # needs a top-80 subspace (> 40)
    with pytest.raises(NotImplementedError):
        svd.denoiseSignal(np.random.default_rng(2).standard_normal((300, 280)),
                          use_optimal=True)  # min(m, n) > 256 on the optimal path


@pytest.mark.parametrize("shape", [(128, 128), (96, 128), (128, 40), (52, 100)])
def test_gram_paths_agree(gpu_device, shape, monkeypatch):
    """The LDS-chunked Gram (r <= 128: row-major and transposed X, ragged chunks and tiles)
    and the one-wave-per-tile Gram give the same reconstruction to fp32 rounding, and both
    match the oracle on a gapped matrix."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    m, n = shape
    A = np.stack([gapped_matrix(700 + i, m, n, dtype=np.float32) for i in range(3)])
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("SPECENH_SVD_GRAM_TILES", flag)
        outs.append(svd.denoise_batch(torch.as_tensor(A, device=gpu_device), 0, 16).double().cpu().numpy())
    for b in range(3):
        truth = ref.denoiseSignal(A[b].astype(np.float64), 0, 16)
        assert _rel(outs[0][b], truth) <= TOL
        assert _rel(outs[1][b], truth) <= TOL
        assert _rel(outs[0][b], outs[1][b]) <= 1e-6


@pytest.mark.parametrize("args", [(), (0, 16), (0, 10_000), (5, 2)])
def test_half_precision_output_is_rounded_fp32(gpu_device, args):
    """specenh_svd_denoise_ex writes fp16/bf16 straight from the fp32 reconstruction: the
    same bits as the fp32 output rounded once (the C5 stream's autoencoder input)."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    A = torch.as_tensor(np.stack([gapped_matrix(40 + i, 128, 128, dtype=np.float32)
                                  for i in range(4)]), device=gpu_device)
    ref32 = svd.denoise_batch(A, *args)
    for dt in (torch.float16, torch.bfloat16):
        out = torch.empty(A.shape, dtype=dt, device=gpu_device)
        svd.denoise_batch(A, *args, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref32.to(dt)), dt
