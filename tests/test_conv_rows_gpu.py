"""The encoder's pooled 5 x 5 convolutions as a row sweep (csrc/conv_rows.hip
conv_rows_pool_kernel; VAE/manual_scan_3layers.py:188-193: Conv2D(32, 5, relu, same) +
MaxPooling2D(2) on 64-wide 16-channel maps, Conv2D(64, 5, ...) on 32-wide 32-channel maps).

Against a float64 torch conv + bias + ReLU + max-pool of the same 16-bit operands, element by
element: products of 16-bit values are exact in fp32, so the kernel differs from float64 by
the fp32 summation (bounded by 1e-5 of the sum of |products| of the pooled window) and one
rounding to the 16-bit type. Batches that give the persistent workgroups unequal image
counts, heights from 2 (one pooled row) up, and the tile kernel (SPECENH_CONV_NO_ROWS) on
the same inputs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import specenh  # noqa: F401  (registers torch.ops.specenh.*)
from specenh import _lib

pytestmark = pytest.mark.gpu

# (C, CO, W, K): the 3-layer model's conv2 and conv3 (manual_scan_3layers.py:189-191), and the
# 32 -> 32 conv2 of hyperparam_scan.py:157 at its 256 x 128 input, k = 5 and 3 (round 6)
SHAPES = [(16, 32, 64, 5), (32, 64, 32, 5), (32, 32, 64, 5), (32, 32, 64, 3)]


def _run(x, w, bias, CO, pool_out, K=5):
    N, H, W, C = x.shape
    torch.ops.specenh.conv2d_out(x, w, bias, K, K, CO, 1, K // 2, K // 2, 1, H, W, 1, None, None,
                                 pool_out, True, None)


def _ref(x, w, bias, K=5):
    xd = x.double().cpu().permute(0, 3, 1, 2)
    wd = w.double().cpu().permute(0, 3, 1, 2)
    b = bias.double().cpu().view(1, -1, 1, 1)
    ref = F.max_pool2d(torch.relu(F.conv2d(xd, wd, padding=K // 2) + b), 2)
    mag = F.max_pool2d(F.conv2d(xd.abs(), wd.abs(), padding=K // 2) + b.abs(), 2)
    return ref.permute(0, 2, 3, 1), mag.permute(0, 2, 3, 1)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("C,CO,W,K", SHAPES)
@pytest.mark.parametrize("N,H", [(1, 64), (3, 32), (7, 2), (5, 18), (513, 8)])
def test_rows_vs_float64(gpu_device, dtype, C, CO, W, K, N, H):
    rng = np.random.default_rng(C + CO + N + H + K)
    x = torch.tensor(rng.standard_normal((N, H, W, C)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, K, K, C)) * 0.1, dtype=dtype, device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO) * 0.5, dtype=torch.float32, device=gpu_device)
    out = torch.full((N, H // 2, W // 2, CO), float("nan"), dtype=dtype, device=gpu_device)
    _run(x, w, bias, CO, out, K)
    torch.cuda.synchronize()
    assert "conv_rows_pool_kernel" in _lib.last_kernel_name()
    ref, mag = _ref(x, w, bias, K)
    got = out.double().cpu()
    assert bool(torch.isfinite(got).all())
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)


@pytest.mark.parametrize("C,CO,W,K", SHAPES)
def test_rows_matches_tile_kernel(gpu_device, kernel_variant, C, CO, W, K):
    """The same layer through conv_patch_kernel (16 x 16 tiles): equal up to fp32 summation
    order and one 16-bit rounding (the row sweep starts its sums at the bias)."""
    N, H = 300, 64 if C == 16 else 32
    rng = np.random.default_rng(5 + C + K)
    x = torch.tensor(rng.uniform(0, 1, (N, H, W, C)), dtype=torch.float16, device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, K, K, C)) * 0.05, dtype=torch.float16,
                     device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO) * 0.1, dtype=torch.float32, device=gpu_device)
    a = torch.empty((N, H // 2, W // 2, CO), dtype=torch.float16, device=gpu_device)
    b = torch.empty_like(a)
    _run(x, w, bias, CO, a, K)
    kernel_variant("CONV_NO_ROWS", 1)
    _run(x, w, bias, CO, b, K)
    torch.cuda.synchronize()
    assert "conv_patch_kernel" in _lib.last_kernel_name()
    d = (a.float() - b.float()).abs()
    assert float(d.max()) <= 2.0 ** -10 * float(b.float().abs().max())


# ---------------------------------------------------------------- Conv2DTranspose row sweep
# (csrc/conv_rows.hip convt_rows_kernel; VAE/manual_scan_3layers.py:196-197). The engine's
# forward GEMM form: a stride-1 conv of the zero-interleaved input (pad 3 top/left, 2
# bottom/right) with the [CO][5][5][64] GEMM weights.
def _convt_ref(x, w, bias):
    N, H, W, C = x.shape
    xd = torch.zeros((N, C, 2 * H - 1, 2 * W - 1), dtype=torch.float64)
    xd[:, :, ::2, ::2] = x.double().cpu().permute(0, 3, 1, 2)
    xd = F.pad(xd, (3, 2, 3, 2))
    wd = w.double().cpu().permute(0, 3, 1, 2)
    b = bias.double().cpu().view(1, -1, 1, 1)
    ref = torch.relu(F.conv2d(xd, wd) + b)
    mag = F.conv2d(xd.abs(), wd.abs()) + b.abs()
    return ref.permute(0, 2, 3, 1), mag.permute(0, 2, 3, 1)


def _convt_run(x, w, bias, CO, out):
    N, H, W, C = x.shape
    torch.ops.specenh.conv2d_out(x, w, bias, 5, 5, CO, 1, 3, 3, 2, 2 * H, 2 * W, 1, None, None,
                                 out, False, None)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("CO,W", [(64, 16), (32, 32)])
@pytest.mark.parametrize("N,H", [(1, 16), (3, 1), (5, 7), (300, 4), (1100, 3)])
def test_convt_rows_vs_float64(gpu_device, dtype, CO, W, N, H):
    rng = np.random.default_rng(CO + W + N + H)
    x = torch.tensor(np.maximum(rng.standard_normal((N, H, W, 64)), 0), dtype=dtype,
                     device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, 5, 5, 64)) * 0.05, dtype=dtype, device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO) * 0.3, dtype=torch.float32, device=gpu_device)
    out = torch.full((N, 2 * H, 2 * W, CO), float("nan"), dtype=dtype, device=gpu_device)
    _convt_run(x, w, bias, CO, out)
    torch.cuda.synchronize()
    assert "convt_rows" in _lib.last_kernel_name()
    ref, mag = _convt_ref(x, w, bias)
    got = out.double().cpu()
    assert bool(torch.isfinite(got).all())
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)


def _convt32_ref(x, w, bias, K):
    """Conv2DTranspose(K, s2, same) as the stride-1 conv of the dilated input, pad
    PT = K - 1 - (K - 2) // 2 before and K - PT after (Keras SAME)."""
    N, H, W, C = x.shape
    PT = K - 1 - (K - 2) // 2
    xd = torch.zeros((N, C, 2 * H - 1, 2 * W - 1), dtype=torch.float64)
    xd[:, :, ::2, ::2] = x.double().cpu().permute(0, 3, 1, 2)
    xd = F.pad(xd, (PT, K - PT, PT, K - PT))
    wd = w.double().cpu().permute(0, 3, 1, 2)
    b = bias.double().cpu().view(1, -1, 1, 1)
    ref = torch.relu(F.conv2d(xd, wd) + b)
    mag = F.conv2d(xd.abs(), wd.abs()) + b.abs()
    return ref.permute(0, 2, 3, 1), mag.permute(0, 2, 3, 1)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("K", [3, 5, 7])
@pytest.mark.parametrize("N,H", [(1, 16), (3, 1), (5, 7), (300, 4), (2, 64)])
def test_convt_rows32_vs_float64(gpu_device, dtype, K, N, H):
    """convt_rows32_kernel (round 6): the scan models' Conv2DTranspose(32, K, s2) on 32-wide
    32-channel maps (hyperparam_scan.py:160, manual_scan.py:197), NaN-poisoned output."""
    rng = np.random.default_rng(K + N + H)
    x = torch.tensor(np.maximum(rng.standard_normal((N, H, 32, 32)), 0), dtype=dtype,
                     device=gpu_device)
    w = torch.tensor(rng.standard_normal((32, K, K, 32)) * 0.08, dtype=dtype, device=gpu_device)
    bias = torch.tensor(rng.standard_normal(32) * 0.3, dtype=torch.float32, device=gpu_device)
    out = torch.full((N, 2 * H, 64, 32), float("nan"), dtype=dtype, device=gpu_device)
    PT = K - 1 - (K - 2) // 2
    torch.ops.specenh.conv2d_out(x, w, bias, K, K, 32, 1, PT, PT, 2, 2 * H, 64, 1, None, None,
                                 out, False, None)
    torch.cuda.synchronize()
    assert "convt_rows32" in _lib.last_kernel_name()
    ref, mag = _convt32_ref(x, w, bias, K)
    got = out.double().cpu()
    assert bool(torch.isfinite(got).all())
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)


@pytest.mark.parametrize("CO,W", [(64, 16), (32, 32)])
def test_convt_rows_matches_tile_kernel(gpu_device, kernel_variant, CO, W):
    N, H = 257, W
    rng = np.random.default_rng(11 + CO)
    x = torch.tensor(rng.uniform(0, 1, (N, H, W, 64)), dtype=torch.float16, device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, 5, 5, 64)) * 0.03, dtype=torch.float16,
                     device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO) * 0.1, dtype=torch.float32, device=gpu_device)
    a = torch.empty((N, 2 * H, 2 * W, CO), dtype=torch.float16, device=gpu_device)
    b = torch.empty_like(a)
    _convt_run(x, w, bias, CO, a)
    kernel_variant("CONVT_NO_ROWS", 1)
    _convt_run(x, w, bias, CO, b)
    torch.cuda.synchronize()
    assert "conv_patch_kernel" in _lib.last_kernel_name()
    d = (a.float() - b.float()).abs()
    assert float(d.max()) <= 2.0 ** -10 * float(b.float().abs().max())


@pytest.mark.parametrize("N,H", [(1, 5), (3, 1), (700, 16), (1100, 3)])
def test_convt_rows_per_wave_ring_bitwise(gpu_device, kernel_variant, N, H):
    """convT1 (CO 64 on 16-wide rows): the per-wave-ring kernel (default), the phase-split
    trial (CONVT_PG: 8 waves, two phases each, B fragments read ahead) and the shared ring
    (CONVT_SHARED_RING): the same per-phase MFMA order, bitwise equal; several images per
    persistent workgroup at N = 700 / 1100."""
    rng = np.random.default_rng(17 + N + H)
    x = torch.tensor(rng.uniform(0, 1, (N, H, 16, 64)), dtype=torch.float16, device=gpu_device)
    w = torch.tensor(rng.standard_normal((64, 5, 5, 64)) * 0.03, dtype=torch.float16,
                     device=gpu_device)
    bias = torch.tensor(rng.standard_normal(64) * 0.1, dtype=torch.float32, device=gpu_device)
    a = torch.full((N, 2 * H, 32, 64), float("nan"), dtype=torch.float16, device=gpu_device)
    b = torch.full_like(a, float("nan"))
    c = torch.full_like(a, float("nan"))
    _convt_run(x, w, bias, 64, a)
    assert "convt_rows_pw_kernel" in _lib.last_kernel_name()
    kernel_variant("CONVT_PG", 1)
    _convt_run(x, w, bias, 64, c)
    assert "convt_rows_pg_kernel" in _lib.last_kernel_name()
    kernel_variant("CONVT_SHARED_RING", 1)
    _convt_run(x, w, bias, 64, b)
    torch.cuda.synchronize()
    assert "convt_rows_kernel" in _lib.last_kernel_name()
    assert bool(torch.isfinite(a).all())
    assert torch.equal(a, c)
    assert torch.equal(a, b)


@pytest.mark.parametrize("CO,W", [(64, 16), (32, 32)])
@pytest.mark.parametrize("N,H", [(1, 5), (700, 16)])
def test_convt_rows_lead_bitwise(gpu_device, kernel_variant, CO, W, N, H):
    """Three ring refills in flight (default) vs the round-3 one-step lead: the waits differ,
    the arithmetic does not (several images per persistent workgroup at N = 700)."""
    rng = np.random.default_rng(5 + CO + N)
    x = torch.tensor(rng.uniform(0, 1, (N, H, W, 64)), dtype=torch.float16, device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, 5, 5, 64)) * 0.03, dtype=torch.float16,
                     device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO) * 0.1, dtype=torch.float32, device=gpu_device)
    a = torch.full((N, 2 * H, 2 * W, CO), float("nan"), dtype=torch.float16, device=gpu_device)
    b = torch.full_like(a, float("nan"))
    kernel_variant("CONVT_SHARED_RING", 1)  # (the LEAD variants are the shared-ring kernel's)
    _convt_run(x, w, bias, CO, a)
    kernel_variant("ROWS_SHORT_LEAD", 1)
    _convt_run(x, w, bias, CO, b)
    torch.cuda.synchronize()
    assert "convt_rows" in _lib.last_kernel_name()
    assert bool(torch.isfinite(a).all())
    assert torch.equal(a, b)


# ---------------------------------------------------------------- C = 1 row sweep
# (csrc/conv_rows.hip conv1_rows_pool_kernel; VAE/manual_scan_3layers.py:187-188)
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H", [(1, 128), (3, 2), (5, 10), (300, 64), (2, 130), (4200, 4)])
def test_conv1_rows_vs_float64(gpu_device, dtype, N, H):
    rng = np.random.default_rng(N + H)
    x = torch.tensor(rng.uniform(0, 1, (N, H, 128, 1)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((16, 5, 5, 1)) * 0.3, dtype=dtype, device=gpu_device)
    bias = torch.tensor(rng.standard_normal(16) * 0.2, dtype=torch.float32, device=gpu_device)
    out = torch.full((N, H // 2, 64, 16), float("nan"), dtype=dtype, device=gpu_device)
    _run(x, w, bias, 16, out)
    torch.cuda.synchronize()
    assert "conv1_rows_pool_kernel" in _lib.last_kernel_name()
    ref, mag = _ref(x, w, bias)
    got = out.double().cpu()
    assert bool(torch.isfinite(got).all())
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)


def test_conv1_rows_matches_tile_kernel(gpu_device, kernel_variant):
    N, H = 2048, 128
    rng = np.random.default_rng(77)
    x = torch.tensor(rng.uniform(0, 1, (N, H, 128, 1)), dtype=torch.float16, device=gpu_device)
    w = torch.tensor(rng.standard_normal((16, 5, 5, 1)) * 0.3, dtype=torch.float16,
                     device=gpu_device)
    bias = torch.tensor(rng.standard_normal(16) * 0.2, dtype=torch.float32, device=gpu_device)
    a = torch.full((N, 64, 64, 16), float("nan"), dtype=torch.float16, device=gpu_device)
    b = torch.empty_like(a)
    _run(x, w, bias, 16, a)
    kernel_variant("CONV1_NO_ROWS", 1)
    _run(x, w, bias, 16, b)
    torch.cuda.synchronize()
    assert "conv_c1_mfma_kernel" in _lib.last_kernel_name()
    d = (a.float() - b.float()).abs()
    assert float(d.max()) <= 2.0 ** -10 * float(b.float().abs().max())


# ---------------------------------------------------------------- encoder 1 + 2 fused
# (csrc/conv_rows.hip enc2_rows_kernel, specenh_encoder2; VAE/manual_scan_3layers.py:187-191)
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H", [(1, 128), (7, 4), (5, 12), (300, 128), (3, 132), (1300, 128),
                                 (1100, 8)])
@pytest.mark.parametrize("wpe2", [0, 1])
def test_encoder2_equals_two_launches(gpu_device, dtype, N, H, wpe2, kernel_variant):
    """The fused launch runs the two row sweeps' arithmetic step for step: bitwise equal to
    conv1_rows_pool_kernel + conv_rows_pool_kernel, and within the 16-bit rounding of a
    float64 composite (the intermediate map rounded to the 16-bit type as stored). N > 512:
    several images per persistent workgroup (the image-to-image hand-over of the row
    streams; a bubble-step F term once leaked into the next image's row 1). wpe2: the
    one-workgroup-per-CU build (256 VGPRs)."""
    kernel_variant("ENC2_WPE2", wpe2)
    rng = np.random.default_rng(N + 3 * H)
    x = torch.tensor(rng.uniform(0, 1, (N, H, 128, 1)), dtype=dtype, device=gpu_device)
    w1 = torch.tensor(rng.standard_normal((16, 5, 5, 1)) * 0.3, dtype=dtype, device=gpu_device)
    b1 = torch.tensor(rng.standard_normal(16) * 0.2, dtype=torch.float32, device=gpu_device)
    w2 = torch.tensor(rng.standard_normal((32, 5, 5, 16)) * 0.08, dtype=dtype, device=gpu_device)
    b2 = torch.tensor(rng.standard_normal(32) * 0.2, dtype=torch.float32, device=gpu_device)
    out = torch.full((N, H // 4, 32, 32), float("nan"), dtype=dtype, device=gpu_device)
    torch.ops.specenh.encoder2_out(x, w1, b1, 16, w2, b2, 32, 5, out)
    torch.cuda.synchronize()
    assert "enc2_rows_kernel" in _lib.last_kernel_name()
    h1 = torch.empty((N, H // 2, 64, 16), dtype=dtype, device=gpu_device)
    _run(x, w1, b1, 16, h1)
    two = torch.empty_like(out)
    _run(h1, w2, b2, 32, two)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(out).all())
    assert torch.equal(out, two)
    ref, mag = _ref(h1, w2, b2)  # second layer in float64 on the stored intermediate
    got = out.double().cpu()
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)


def test_encoder2_engine_path(gpu_device, kernel_variant):
    """AutoencoderEngine.forward at the C5 shape takes the fused launch (enc2) and matches
    the unfused engine (SPECENH_ENCODER_UNFUSED) bitwise."""
    import bench

    x = torch.rand(64, 128, 128, 1, device=gpu_device).to(torch.float16)
    eng = bench.make_c5_engine(gpu_device)
    assert eng.enc2
    a = eng.forward(x).clone()
    kernel_variant("ENCODER_UNFUSED", 1)
    eng2 = bench.make_c5_engine(gpu_device)
    assert not eng2.enc2
    b = eng2.forward(x)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("CO,W,ring", [(64, 16, "pw"), (64, 16, "shared"), (32, 32, "shared")])
@pytest.mark.parametrize("N,H", [(1, 16), (3, 32), (128, 16), (200, 8), (5, 12)])
def test_convt_rows_bands_bitwise(gpu_device, kernel_variant, CO, W, ring, N, H):
    """Row bands (round 6): a small batch's images cut into 2 / 4 / 8 bands of rows (halo rows
    read from the neighbouring band, two bubble steps between bands) give the whole-image
    sweep's outputs bit for bit; N = 128 is the C4 training batch the automatic choice bands."""
    rng = np.random.default_rng(23 + CO + N + H)
    x = torch.tensor(rng.uniform(0, 1, (N, H, W, 64)), dtype=torch.float16, device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, 5, 5, 64)) * 0.03, dtype=torch.float16,
                     device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO) * 0.1, dtype=torch.float32, device=gpu_device)
    if ring == "shared":
        kernel_variant("CONVT_SHARED_RING", 1)
    kernel_variant("ROWS_BANDS", 0)
    ref = torch.full((N, 2 * H, 2 * W, CO), float("nan"), dtype=torch.float16, device=gpu_device)
    _convt_run(x, w, bias, CO, ref)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(ref).all())
    for lg in (1, 2, 3, -1):
        kernel_variant("ROWS_BANDS", lg)
        got = torch.full_like(ref, float("nan"))
        _convt_run(x, w, bias, CO, got)
        torch.cuda.synchronize()
        name = _lib.last_kernel_name()
        assert ("convt_rows_pw_kernel" if ring == "pw" else "convt_rows_kernel") in name
        assert torch.equal(got, ref), (lg, float((got.float() - ref.float()).abs().max()))
