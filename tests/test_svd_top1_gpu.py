"""GPU parity of the one-pass top-1 complement (top1_kernel, svd_denoise.hip): the default
denoiseSignal kept range [1, r) (denoising_by_svd.ipynb:188-229) for matrices up to
128 x 128, vs the float64 oracle and vs the Gram + subspace + reconstruction pipeline it
replaces (kernel variant SVD_NO_TOP1). Tolerance as test_svd_gpu.py: 1e-5 relative
(Frobenius) on inputs with a gap at the cut; rank-deficient inputs relative to ||A||."""
import os
import sys

import numpy as np
import pytest

from oracle import svd as ref

pytestmark = pytest.mark.gpu
TOL = 1e-5
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))


def _err(got, want, A):
    nw, na = np.linalg.norm(want), np.linalg.norm(A)
    return np.linalg.norm(got - want) / max(nw, 0.01 * na, 1e-300)


def _run(A, dev, **kw):
    """denoise_batch default range; returns (out, kernel symbols launched)."""
    import torch

    from specenh import _lib, svd

    t = torch.as_tensor(A, device=dev)
    n0 = _lib.launch_count()
    out = svd.denoise_batch(t, **kw)
    torch.cuda.synchronize()
    names = _lib.kernel_names(n0, _lib.launch_count())
    return out.double().cpu().numpy(), names


def _used_top1(names):
    return any("top1_kernel" in s for s in names)


@pytest.mark.parametrize("shape", [(128, 128), (96, 128), (128, 40), (52, 100), (8, 4),
                                   (128, 4), (4, 128)])
def test_top1_matches_oracle_and_pipeline(gpu_device, shape, kernel_variant):
    from make_golden import gapped_matrix

    m, n = shape
    A = np.stack([gapped_matrix(300 + i, m, n, k=min(16, min(m, n)), dtype=np.float32)
                  for i in range(5)])
    got, names = _run(A, gpu_device)
    assert _used_top1(names), names
    kernel_variant("SVD_NO_TOP1", 1)
    old, names_old = _run(A, gpu_device)
    assert not _used_top1(names_old)
    for b in range(len(A)):
        want = ref.denoiseSignal(A[b].astype(np.float64))
        assert _err(got[b], want, A[b]) <= TOL, (b, _err(got[b], want, A[b]))
        assert _err(old[b], want, A[b]) <= TOL


def test_top1_rank_deficient_and_zero(gpu_device):
    """Rank 1 (the complement is exactly zero), rank 2 and 3, the zero matrix: dead basis
    columns in the CholeskyQR and the Rayleigh-Ritz Gram."""
    rng = np.random.default_rng(11)
    mats = []
    for k in (1, 2, 3):
        mats.append((rng.standard_normal((128, k)) * np.array([5.0, 1.0, 0.3][:k]))
                    @ rng.standard_normal((k, 128)))
    mats.append(np.zeros((128, 128)))
    A = np.stack(mats).astype(np.float32)
    got, names = _run(A, gpu_device)
    assert _used_top1(names)
    assert np.all(np.isfinite(got))
    for b in range(len(A)):
        want = ref.denoiseSignal(A[b].astype(np.float64))
        assert _err(got[b], want, A[b]) <= TOL, (b, _err(got[b], want, A[b]))
    assert not np.any(got[3])


def test_top1_c5_spectrograms(gpu_device, kernel_variant):
    """The C5 stream's matrices (128 x 128 log spectrograms of the synthetic plasma
    chirps): oracle parity and agreement with the pipeline path."""
    import torch

    import bench
    from specenh import pipeline_data
    from specenh.synthetic import plasma_chirps_torch

    x = plasma_chirps_torch(6, bench.L5, seed=1000, device=gpu_device).to(torch.float16)
    S = torch.empty((6, 128, 128), dtype=torch.float32, device=gpu_device)
    pipeline_data.specgr_batch(x, bench.SPEC5, out=S)
    A = S.cpu().numpy()
    got, names = _run(A, gpu_device)
    assert _used_top1(names)
    kernel_variant("SVD_NO_TOP1", 1)
    old, _ = _run(A, gpu_device)
    for b in range(len(A)):
        want = ref.denoiseSignal(A[b].astype(np.float64))
        assert _err(got[b], want, A[b]) <= TOL
        assert _err(got[b], old[b], A[b]) <= 2 * TOL


def test_top1_ties_at_the_cut(gpu_device):
    """A near-tie of the top pair (theta gap 2e-3 relative: Rayleigh-Ritz in the 4-vector
    block separates it) must match the oracle; an exact tie (no gap: the kernel flags it and
    the fp64 eigen path writes the output; any rotation of the top pair is a valid SVD)
    must match it up to that rotation, i.e. in its singular values."""
    rng = np.random.default_rng(3)
    u, _ = np.linalg.qr(rng.standard_normal((128, 128)))
    v, _ = np.linalg.qr(rng.standard_normal((128, 128)))
    s = 0.01 * rng.uniform(0.5, 1.0, 128)
    mats = []
    for second in (10.0 * (1 - 1e-3), 10.0):
        s2 = s.copy()
        s2[0], s2[1] = 10.0, second
        mats.append(((u * s2) @ v.T).astype(np.float32))
    A = np.stack(mats)
    got, names = _run(A, gpu_device)
    assert _used_top1(names)
    want = ref.denoiseSignal(A[0].astype(np.float64))
    assert _err(got[0], want, A[0]) <= TOL, _err(got[0], want, A[0])
    sv_got = np.linalg.svd(got[1], compute_uv=False)
    sv_want = np.linalg.svd(ref.denoiseSignal(A[1].astype(np.float64)), compute_uv=False)
    assert np.max(np.abs(sv_got - sv_want)) <= TOL * sv_want[0]


@pytest.mark.parametrize("shape", [(132, 128), (128, 130), (126, 64)])
def test_shapes_outside_top1_use_pipeline(gpu_device, shape):
    from make_golden import gapped_matrix

    m, n = shape
    A = gapped_matrix(77, m, n, dtype=np.float32)[None]
    got, names = _run(A, gpu_device)
    assert not _used_top1(names)
    assert _err(got[0], ref.denoiseSignal(A[0].astype(np.float64)), A[0]) <= TOL
