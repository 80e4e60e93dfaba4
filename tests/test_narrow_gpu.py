"""Narrow-channel convolutions on the GPU against a float64 torch convolution of the same
16-bit operands.

One input channel: conv_c1_mfma_kernel (csrc/conv_c1_mfma.hip, window rows as MFMA K runs),
conv_c1_kernel (csrc/conv_narrow.hip, VALU dot2) and the generic MFMA kernels, forward with
and without the fused 2x2 max-pool, and with the ReLU mask of the backward pass (the input
gradient of the 16 -> 1 output conv, VAE/manual_scan_3layers.py:199). One output channel:
conv_co1_kernel split into row bands at batch sizes and heights that leave ragged bands.
Products of two 16-bit values are exact in fp32, so the fp32 accumulation differs from
float64 by rounding only: |err| <= 1e-5 * sum|products| (fp32 out), or one rounding to the
16-bit type on top of that (16-bit out)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import specenh  # noqa: F401  (registers torch.ops.specenh.*)

pytestmark = pytest.mark.gpu


def _ref(x, w, bias, k):
    """float64 'same' convolution: x [N,H,W,C], w [CO][K][K][C] -> [N,H,W,CO], and the
    sum of |products| per output (the error scale)."""
    xd = x.double().permute(0, 3, 1, 2).cpu()
    wd = w.double().permute(0, 3, 1, 2).cpu()
    out = F.conv2d(xd, wd, padding=k // 2) + bias.double().cpu().view(1, -1, 1, 1)
    mag = F.conv2d(xd.abs(), wd.abs(), padding=k // 2)
    return out.permute(0, 2, 3, 1), mag.permute(0, 2, 3, 1)


def _path(kernel_variant, path):
    """c1mfma: conv_c1_mfma.hip (the default for C == 1); narrow: the VALU dot2 kernel;
    generic: the MFMA patch/gather kernels."""
    if path in ("narrow", "generic"):
        kernel_variant("CONV_NO_C1MFMA", 1)
    if path == "generic":
        kernel_variant("CONV_NO_NARROW", 1)


def _conv(x, w, bias, k, co, act, out_dtype, mask=None):
    N, H, W, _ = x.shape
    out = torch.empty((N, H, W, co), dtype=out_dtype, device=x.device)
    torch.ops.specenh.conv2d_out(x, w, bias, k, k, co, 1, k // 2, k // 2, 1, H, W, act, mask,
                                 None, out, False, None)
    return out


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W", [(3, 64, 64), (2, 37, 70), (1, 128, 128)])
@pytest.mark.parametrize("path", ["c1mfma", "narrow", "generic"])
def test_c1_masked_dgrad(gpu_device, kernel_variant, dtype, N, H, W, path):
    _path(kernel_variant, path)
    rng = np.random.default_rng(N * 1000 + H + W)
    k, co = 5, 16
    x = torch.tensor(rng.standard_normal((N, H, W, 1)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((co, k, k, 1)) * 0.2, dtype=dtype, device=gpu_device)
    bias = torch.zeros(co, dtype=torch.float32, device=gpu_device)
    mask = torch.tensor(rng.standard_normal((N, H, W, co)), dtype=dtype, device=gpu_device)
    mask[0, 0, :4] = 0.0  # exact zeros: masked like negatives
    got = _conv(x, w, bias, k, co, 0, dtype, mask).double().cpu()
    from specenh import _lib
    name = _lib.last_kernel_name()
    assert {"c1mfma": "conv_c1_mfma_kernel", "narrow": "conv_c1_kernel",
            "generic": "conv_patch_kernel"}[path] in name, name
    ref, mag = _ref(x, w, bias, k)
    keep = (mask.double().cpu() > 0)
    ref = torch.where(keep, ref, torch.zeros_like(ref))
    assert torch.all(got[~keep] == 0)
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [16, 32])
@pytest.mark.parametrize("N,H,W", [(128, 128, 128), (3, 40, 200), (5, 17, 130), (2, 1, 9)])
def test_co1_bands(gpu_device, dtype, C, N, H, W):
    rng = np.random.default_rng(C + N + H + W)
    k = 5
    x = torch.tensor(rng.standard_normal((N, H, W, C)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((1, k, k, C)) * 0.1, dtype=dtype, device=gpu_device)
    bias = torch.tensor([0.25], dtype=torch.float32, device=gpu_device)
    got = _conv(x, w, bias, k, 1, 0, torch.float32).double().cpu()
    ref, mag = _ref(x, w, bias, k)
    assert torch.all((got - ref).abs() <= 1e-5 * (mag + 0.25) + 1e-30)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,k", [(64, 5), (64, 3), (64, 7), (32, 5), (32, 7)])
@pytest.mark.parametrize("N,H,W", [(4, 256, 128), (3, 37, 70), (2, 9, 17), (1, 1, 5)])
@pytest.mark.parametrize("out", ["f32", "lowp_sigmoid", "logits"])
def test_co1_mfma(gpu_device, kernel_variant, dtype, C, k, N, H, W, out):
    """conv_co1m_kernel (one output channel from 32 / 64 channels on the MFMA, the last
    Conv2D of manual_scan.py / hyperparam_scan.py): against float64 at ragged widths and
    heights (partial 16-column strips, partial 8-row bands), fp32 or 16-bit sigmoid output,
    and the fp32 logits of a training forward; for C = 32 also against the VALU kernel
    (CO1_VALU=1)."""
    rng = np.random.default_rng(C * 7 + k + N + H + W)
    x = torch.tensor(rng.standard_normal((N, H, W, C)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((1, k, k, C)) * 0.1, dtype=dtype, device=gpu_device)
    bias = torch.tensor([0.25], dtype=torch.float32, device=gpu_device)
    ref, mag = _ref(x, w, bias, k)
    tol = 1e-5 * (mag + 0.25) + 1e-30
    act = 2 if out == "lowp_sigmoid" else 0  # SPECENH_ACT_SIGMOID
    odt = dtype if out == "lowp_sigmoid" else torch.float32

    def run():
        y = torch.empty((N, H, W, 1), dtype=odt, device=gpu_device)
        z = torch.full((N, H, W, 1), float("nan"), dtype=torch.float32, device=gpu_device) \
            if out == "logits" else None
        torch.ops.specenh.conv2d_out(x, w, bias, k, k, 1, 1, k // 2, k // 2, 1, H, W, act, None,
                                     z, y, False, None)
        return y, z

    y, z = run()
    if out == "lowp_sigmoid":
        want = torch.sigmoid(ref)
        assert torch.all((y.double().cpu() - want).abs() <= 2 ** -8 * want.abs() + tol)
    else:
        assert torch.all((y.double().cpu() - ref).abs() <= tol)
    if out == "logits":
        assert torch.all((z.double().cpu() - ref).abs() <= tol)
    if C == 32:
        kernel_variant("CO1_VALU", 1)
        y2, _ = run()
        assert torch.all((y2.double().cpu() - y.double().cpu()).abs() <= 2 * tol + (2 ** -8 if out == "lowp_sigmoid" else 0))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [16, 8, 3])
@pytest.mark.parametrize("masked", [False, True])
def test_maxpool2_bwd_routes_to_argmax(gpu_device, dtype, C, masked):
    """MaxPooling2D backward (the 16-byte vector kernel for C % 8 == 0, the scalar one
    otherwise): the gradient goes to the argmax position, zero where the pooled value is not
    positive (the ReLU mask), exactly."""
    rng = np.random.default_rng(C + 2 * masked)
    N, H, W = 3, 18, 22
    x = torch.tensor(rng.standard_normal((N, H, W, C)), dtype=dtype, device=gpu_device)
    pooled, am = torch.ops.specenh.maxpool2(x)
    dy = torch.tensor(rng.standard_normal((N, H // 2, W // 2, C)), dtype=dtype, device=gpu_device)
    dx = torch.ops.specenh.maxpool2_bwd(dy, am, pooled if masked else None).cpu()
    g = dy.cpu().clone()
    if masked:
        g[pooled.cpu().float() <= 0] = 0
    ref = torch.zeros((N, H, W, C), dtype=dtype)
    a = am.cpu().long()
    for q in range(4):
        sel = (a == q)
        ref[:, (q >> 1)::2, (q & 1)::2, :] = torch.where(sel, g, torch.zeros_like(g))
    assert torch.equal(dx, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k,co,N,H,W", [(5, 16, 3, 64, 64), (5, 16, 2, 50, 70), (3, 32, 2, 36, 34),
                                        (7, 16, 1, 40, 24), (4, 16, 2, 32, 32)])
@pytest.mark.parametrize("path", ["c1mfma", "narrow", "generic"])
@pytest.mark.parametrize("pool", [False, True])
def test_c1_forward(gpu_device, kernel_variant, dtype, k, co, N, H, W, path, pool):
    """Conv2D(1 -> co, relu) [+ MaxPooling2D]: values within one 16-bit rounding of the
    float64 result; the pooled output is the max of the stored values with its argmax."""
    if path == "narrow" and k % 2 == 0:
        pytest.skip("the VALU kernel takes odd kernels")
    if path == "generic" and pool and k > 5:
        pytest.skip("the fused pool needs the LDS-patch kernel (k <= 5)")
    _path(kernel_variant, path)
    rng = np.random.default_rng(k * 100 + co + H)
    x = torch.tensor(rng.uniform(0, 1, (N, H, W, 1)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((co, k, k, 1)) * 0.3, dtype=dtype, device=gpu_device)
    bias = torch.tensor(rng.standard_normal(co) * 0.1, dtype=torch.float32, device=gpu_device)
    pt, pl = (k - 1) // 2, (k - 1) // 2
    xd = F.pad(x.double().cpu().permute(0, 3, 1, 2), (pl, k - 1 - pl, pt, k - 1 - pt))
    wd = w.double().cpu().permute(0, 3, 1, 2)
    ref = (F.conv2d(xd, wd) + bias.double().cpu().view(1, -1, 1, 1)).clamp_min(0)
    mag = F.conv2d(xd.abs(), wd.abs()) + bias.double().cpu().abs().view(1, -1, 1, 1)
    ref, mag = ref.permute(0, 2, 3, 1), mag.permute(0, 2, 3, 1)
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    if not pool:
        out = torch.empty((N, H, W, co), dtype=dtype, device=gpu_device)
        torch.ops.specenh.conv2d_out(x, w, bias, k, k, co, 1, pt, pl, 1, H, W, 1, None, None,
                                     out, False, None)
        got = out.double().cpu()
        assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)
        return
    out = torch.empty((N, H // 2, W // 2, co), dtype=dtype, device=gpu_device)
    am = torch.empty((N, H // 2, W // 2, co), dtype=torch.uint8, device=gpu_device)
    torch.ops.specenh.conv2d_out(x, w, bias, k, k, co, 1, pt, pl, 1, H, W, 1, None, None, out,
                                 True, am)
    got = out.double().cpu()
    win = ref[:, :H // 2 * 2, :W // 2 * 2].reshape(N, H // 2, 2, W // 2, 2, co)
    pref = win.amax(dim=(2, 4))
    pmag = mag[:, :H // 2 * 2, :W // 2 * 2].reshape(N, H // 2, 2, W // 2, 2, co).amax(dim=(2, 4))
    assert torch.all((got - pref).abs() <= eps * pref.abs() + 1e-5 * pmag + 1e-30)
    # the argmax points at a window element whose value rounds to the pooled value
    a = am.cpu().long()
    sel = win.permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, co, 4)
    picked = torch.gather(sel, 4, a.unsqueeze(-1)).squeeze(-1)
    assert torch.all((picked - got).abs() <= 2 * eps * got.abs() + 2e-5 * pmag + 1e-30)
