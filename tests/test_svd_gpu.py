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

    wide = np.random.default_rng(2).standard_normal((300, 280))
    with pytest.raises(NotImplementedError):
        svd.denoiseSignal(wide, 0, 80)        # eigen path needs min(m, n) <= 256
    with pytest.raises(NotImplementedError):
        svd.denoiseSignal(wide, use_optimal=True)


def _ranges():
    from test_oracle_golden import _ranges_fixture
    return _ranges_fixture()


def _range_err(got, want, A):
    """||got - want||_F / ||want||_F, or relative to ||A||_F when the kept part carries
    less than 1% of the matrix norm (fp32 reconstruction error scales with ||A||)."""
    nw, na = np.linalg.norm(want), np.linalg.norm(A)
    return np.linalg.norm(got - want) / max(nw, 0.01 * na, 1e-300)


@pytest.mark.parametrize("tag", ["noise64x48", "noise40x72", "gap96x80", "gap72x100"])
def test_slice_semantics_match_notebook(tag, gpu_device):
    """denoising_by_svd.ipynb:216-228 with Python slicing: negative stop, empty slices,
    wide kept ranges (K > 40, through the fp64 eigen path), use_optimal with
    num_sing == 0 (keeps [0, r-1)) and computeSignal, vs the notebook's own outputs."""
    import torch

    from test_oracle_golden import range_args
    from specenh import svd

    e = _ranges()[tag]
    A = e["A"]
    A64 = A.astype(np.float64)
    errs = {}
    for key, want in e.items():
        if key.startswith("r_"):
            got = svd.denoiseSignal(A, *range_args(key))
        elif key == "optimal":
            got = svd.denoiseSignal(A, use_optimal=True)
        elif key == "compute":
            got = svd.computeSignal(A)
        else:
            continue
        assert got.shape == A.shape and got.dtype == np.float64
        errs[key] = _range_err(got, want.astype(np.float64), A64)
        if not np.any(want):
            assert not np.any(got), key
    print(tag, {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, bad
    _, ns, _ = svd.optimal_batch(torch.as_tensor(A, device=gpu_device), return_rank=True)
    assert int(ns[0]) == int(e["num_sing"])


def test_noise_optimal_keeps_all_but_last(gpu_device):
    """Pure noise: num_sing == 0, stop = -1: the output is A minus its smallest component
    (not zeros), batched with a gapped matrix whose range differs."""
    import torch

    from specenh import svd

    fx = _ranges()
    A = fx["noise64x48"]["A"]
    B = fx["gap96x80"]["A"][:64, :48].copy()
    X = torch.as_tensor(np.stack([A, B]), device=gpu_device)
    out, ns, _ = svd.optimal_batch(X, return_rank=True)
    out = out.double().cpu().numpy()
    for b, M in enumerate((A, B)):
        M64 = M.astype(np.float64)
        assert _range_err(out[b], ref.denoiseSignal(M64, use_optimal=True), M64) <= TOL
    assert int(ns[0]) == 0 and int(ns[1]) > 0


def test_c3_geometry_wide_range(gpu_device):
    """513 x 256 (BASELINE config 3) with a K = 100 kept range: golden from the notebook."""
    import torch

    from specenh import svd

    e = _ranges()["c3_513x256"]
    A = np.stack([e["A"], e["A"][::-1].copy()])
    out = svd.denoise_batch(torch.as_tensor(A, device=gpu_device), 0, 100).double().cpu().numpy()
    assert _range_err(out[0], e["r_0_100"].astype(np.float64), A[0].astype(np.float64)) <= TOL
    flipped = e["r_0_100"][::-1].astype(np.float64)  # row permutation commutes with the SVD
    assert _range_err(out[1], flipped, A[1].astype(np.float64)) <= TOL


@pytest.mark.parametrize("args", [(0, 100), (1, -1), (0, -3), (3, 45)])
def test_eigen_path_half_precision_output(gpu_device, args):
    """The eigen path's fp16/bf16 store is the fp32 result rounded once."""
    import torch

    from specenh import svd

    A = torch.as_tensor(np.stack([_ranges()["gap96x80"]["A"]] * 3), device=gpu_device)
    ref32 = svd.denoise_batch(A, *args)
    for dt in (torch.float16, torch.bfloat16):
        out = torch.empty(A.shape, dtype=dt, device=gpu_device)
        svd.denoise_batch(A, *args, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref32.to(dt)), dt


def test_rank_deficient_complement(gpu_device):
    """Exactly degenerate eigenvalues (a rank-3 matrix: 45 zero singular values) at the
    bottom of the spectrum: [0, r-2) through the complement of the bottom 2 (one cluster
    iterated in sequence) and [0, 40) directly, vs float64 numpy."""
    from specenh import svd

    rng = np.random.default_rng(5)
    A = (rng.standard_normal((64, 3)) @ rng.standard_normal((3, 48))).astype(np.float32)
    A64 = A.astype(np.float64)
    for args in [(0, -2), (0, 46), (1, -1), (0, 45)]:
        got = svd.denoiseSignal(A, *args)
        assert _range_err(got, ref.denoiseSignal(A64, *args), A64) <= TOL, args


@pytest.mark.parametrize("shape", [(128, 128), (96, 128), (128, 40), (52, 100),
                                   (513, 256), (256, 513), (300, 200), (201, 132), (140, 301)])
def test_gram_paths_agree(gpu_device, shape, kernel_variant):
    """The LDS-chunked Grams (gram_lds_kernel for r <= 128; for 128 < r <= 256 the fp16
    hi/lo split gram256s_kernel and the fp32 gram256_kernel: row-major and transposed X,
    ragged chunks, odd K, r not a multiple of 32) and the one-wave-per-tile Gram give the
    same reconstruction to fp32 rounding, and all match the oracle on a gapped matrix.
    (513, 256) is BASELINE config 3's geometry."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    m, n = shape
    A = np.stack([gapped_matrix(700 + i, m, n, dtype=np.float32) for i in range(3)])
    outs = []
    for tiles, f32 in ((0, 0), (1, 0), (0, 1)):
        kernel_variant("SVD_GRAM_TILES", tiles)
        kernel_variant("SVD_GRAM_F32", f32)
        outs.append(svd.denoise_batch(torch.as_tensor(A, device=gpu_device), 0, 16).double().cpu().numpy())
    for b in range(3):
        truth = ref.denoiseSignal(A[b].astype(np.float64), 0, 16)
        for o in outs:
            assert _rel(o[b], truth) <= TOL
        assert _rel(outs[1][b], outs[2][b]) <= 1e-6  # fp32 Grams: same products, other order
        # the split Gram (default; other arithmetic) no further from the truth than fp32's
        assert _rel(outs[0][b], truth) <= _rel(outs[2][b], truth) + 1e-6


@pytest.mark.parametrize("shape,args", [((513, 256), (0, 16)), ((513, 256), ()),
                                        ((300, 132), (0, 16)), ((201, 130), (0, 16)),
                                        ((140, 301), ()), ((64, 48), (2, 30))])
def test_subspace_gz_paths_agree(gpu_device, shape, args, kernel_variant):
    """subspace_kernel's G Z with four rows per thread (default; r % 4 == 0, j range split
    over the four waves and summed in wave order) and one row per thread (SVD_GZ_ROWS=1):
    the same reconstruction to fp32 rounding, both on the oracle, and each bitwise
    independent of the matrix's position in the batch. r = 130 takes the one-row path
    either way; (64, 48) at (2, 30) runs the 40-wide subspace (one row per thread only)."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    m, n = shape
    A = np.stack([gapped_matrix(1200 + i, m, n, dtype=np.float32) for i in range(3)])
    At = torch.as_tensor(np.concatenate([A, A[::-1]]), device=gpu_device)
    outs = []
    for rows in (0, 1):
        kernel_variant("SVD_GZ_ROWS", rows)
        o = svd.denoise_batch(At, *args)
        assert torch.equal(o[:3], o[3:].flip(0)), rows  # position-independent
        outs.append(o[:3].double().cpu().numpy())
    for b in range(3):
        truth = ref.denoiseSignal(A[b].astype(np.float64), *args)
        for o in outs:
            assert _rel(o[b], truth) <= TOL
        assert _rel(outs[0][b], outs[1][b]) <= 1e-6


@pytest.mark.parametrize("case", ["tiny", "huge", "late_rows", "zero_head", "col_range",
                                  "transposed_rows"])
def test_split_gram_scale(gpu_device, case, kernel_variant):
    """gram256s_kernel's running power-of-two scale (fp16 hi/lo split, 128 < r <= 256): the
    reconstruction matches float64 numpy and the fp32 Gram path for magnitudes far outside
    fp16's range (1e-15, 1e15), rows that grow 1e6-fold after the first chunks (accumulators
    rescaled mid-matrix), leading all-zero chunks, and columns 1e-4 / 1e4 apart."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix

    m, n = (256, 300) if case == "transposed_rows" else (300, 200)
    A = np.stack([gapped_matrix(900 + i, m, n) for i in range(2)])
    if case == "tiny":
        A = A * 1e-15
    elif case == "huge":
        A = A * 1e15
    elif case == "late_rows":  # the first 40 rows 1e-6 of the rest: rescale in chunk 3
        A[:, :40] *= 1e-6
    elif case == "zero_head":
        A[:, :37] = 0.0
    elif case == "col_range":  # (row scalings keep the rank-16 + noise gap; so do these)
        A[:, :, ::2] *= 1e4
        A[:, :, 1::2] *= 1e-4
    elif case == "transposed_rows":  # m < n: X = A^T, K = 300 rows of X are A's columns
        A[:, :, 100:] *= 1e5
    A = A.astype(np.float32)
    outs = []
    for f32 in (0, 1):
        kernel_variant("SVD_GRAM_F32", f32)
        outs.append(svd.denoise_batch(torch.as_tensor(A, device=gpu_device), 0, 16).double().cpu().numpy())
    for b in range(2):
        truth = ref.denoiseSignal(A[b].astype(np.float64), 0, 16)
        assert _rel(outs[0][b], truth) <= TOL, (case, b, _rel(outs[0][b], truth))
        assert _rel(outs[0][b], truth) <= max(2 * _rel(outs[1][b], truth), 1e-6), case


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


@pytest.mark.parametrize("m,n", [(513, 256), (100, 72), (48, 64), (130, 200), (256, 100)])
@pytest.mark.parametrize("rng_k", [(None, None), (0, 16), (2, 30), (0, 40)])
def test_recon_mfma_matches_scalar_recon(gpu_device, kernel_variant, m, n, rng_k):
    """The matrix-core reconstructions — recon_stream_kernel (default: runs of row blocks per
    workgroup) and recon_mfma_kernel (SVD_RECON_BLOCKS=1: one block per workgroup) — vs
    recon_kernel (scalar FMAs, SVD_RECON_VALU=1): the same subspace, products summed in another
    order — equal to fp32 rounding (1e-6 relative Frobenius), across both orientations, r not
    a multiple of 16 and kept ranges that need 8 .. 48 padded columns."""
    import os
    import sys

    import torch

    from specenh import _lib, svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix
    start, stop = rng_k
    r = min(m, n)
    if stop is not None and stop > r:
        pytest.skip("range beyond the rank")
    A = np.stack([gapped_matrix(900 + i, m, n, k=min(48, r - 2)) for i in range(5)]).astype(np.float32)
    At = torch.as_tensor(A, device=gpu_device)
    outs, names = [], []
    for var in (None, "SVD_RECON_BLOCKS", "SVD_RECON_VALU"):
        if var:
            kernel_variant(var, 1)
        n0 = _lib.launch_count()
        outs.append(svd.denoise_batch(At, start, stop).double().cpu().numpy())
        names.append(" ".join(_lib.kernel_names(n0, _lib.launch_count())))
    if "12recon_kernel" in names[2]:  # (top-1 / eigen paths have no subspace reconstruction)
        assert "recon_stream_kernel" in names[0] and "recon_mfma_kernel" in names[1]
    for a in outs[:2]:
        for i in range(len(A)):
            e = np.linalg.norm(a[i] - outs[2][i]) / max(np.linalg.norm(outs[2][i]), 1e-30)
            assert e <= 1e-6, (i, e)


@pytest.mark.parametrize("m,n", [(513, 256), (256, 300), (300, 132)])
@pytest.mark.parametrize("rng_k", [(None, None), (0, 16)])
def test_recon_stream_runs(gpu_device, kernel_variant, m, n, rng_k):
    """A batch that fills the chip (1100 matrices: 5 distinct ones tiled) puts every row block
    of a matrix in one recon_stream_kernel workgroup (V staged once, the next block's loads in
    flight): equal to recon_mfma_kernel's one-block workgroups to fp32 rounding (1e-6; the
    products are summed in another order), and every copy of a matrix gets the same output."""
    import os
    import sys

    import torch

    from specenh import _lib, svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix
    A = np.stack([gapped_matrix(950 + i, m, n) for i in range(5)]).astype(np.float32)
    At = torch.as_tensor(np.tile(A, (220, 1, 1)), device=gpu_device)
    n0 = _lib.launch_count()
    a = svd.denoise_batch(At, *rng_k)
    assert "recon_stream_kernel" in " ".join(_lib.kernel_names(n0, _lib.launch_count()))
    kernel_variant("SVD_RECON_BLOCKS", 1)
    b = svd.denoise_batch(At, *rng_k)
    assert float((a - b).norm() / b.norm()) <= 1e-6
    a5 = a.view(220, 5, m, n)
    assert torch.equal(a5, a5[:1].expand_as(a5))
    for i in range(5):
        truth = ref.denoiseSignal(A[i].astype(np.float64), *[v for v in rng_k if v is not None])
        assert _rel(a[i].double().cpu().numpy(), truth) <= TOL


@pytest.mark.parametrize("shape,args", [((64, 48), ()), ((300, 200), (0, 16))])
def test_fallback_loops_over_many_flagged(gpu_device, shape, args):
    """Ungapped (pure noise) matrices at a batch larger than the fp64 fallback's grid (two
    workgroups per CU): most are flagged by top1 / the subspace check and redone by the eigen
    path, whose kernels then loop over several matrices per workgroup."""
    import torch

    from specenh import svd
    rng = np.random.default_rng(11)
    A = rng.standard_normal((600,) + shape).astype(np.float32)
    out = svd.denoise_batch(torch.as_tensor(A, device=gpu_device), *args).double().cpu().numpy()
    for b in (0, 1, 299, 511, 512, 599):
        truth = ref.denoiseSignal(A[b].astype(np.float64), *args)
        assert _range_err(out[b], truth, A[b].astype(np.float64)) <= TOL, b


@pytest.mark.parametrize("shape,args", [((64, 48), ()), ((128, 128), ()), ((300, 200), (0, 16)),
                                        ((128, 128), (0, 16))])
def test_merged_fallback_equals_four_launches(gpu_device, shape, args, kernel_variant):
    """The flagged-matrix fp64 fallback as one launch (eig_fallback_kernel: Gram tiles,
    tridiagonalisation, eigenvectors and reconstruction blocks per workgroup, default) and as
    the four separate launches (EIG_SPLIT=1): the same kernels' arithmetic in the same order,
    so bitwise equal outputs, on a batch where noise matrices are flagged between gapped ones
    that are not."""
    import os
    import sys

    import torch

    from specenh import svd
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import gapped_matrix
    rng = np.random.default_rng(23)
    mats = [gapped_matrix(1500 + i, *shape, dtype=np.float32) if i % 3 else
            rng.standard_normal(shape).astype(np.float32) for i in range(40)]
    At = torch.as_tensor(np.stack(mats), device=gpu_device)
    outs = []
    for split in (0, 1):
        kernel_variant("EIG_SPLIT", split)
        outs.append(svd.denoise_batch(At, *args))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    for b in (0, 1, 3, 39):
        truth = ref.denoiseSignal(mats[b].astype(np.float64), *args)
        assert _range_err(outs[0][b].double().cpu().numpy(), truth,
                          mats[b].astype(np.float64)) <= TOL, b
