"""Narrow-channel direct convolutions (csrc/conv_narrow.hip) on the GPU against a float64
torch convolution of the same 16-bit operands.

conv_c1_kernel (1 input channel) with the ReLU mask of the backward pass (the input gradient
of the 16 -> 1 output conv, VAE/manual_scan_3layers.py:199), and conv_co1_kernel (1 output
channel) split into row bands at batch sizes and heights that leave ragged last bands.
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


def _conv(x, w, bias, k, co, act, out_dtype, mask=None):
    N, H, W, _ = x.shape
    out = torch.empty((N, H, W, co), dtype=out_dtype, device=x.device)
    torch.ops.specenh.conv2d_out(x, w, bias, k, k, co, 1, k // 2, k // 2, 1, H, W, act, mask,
                                 None, out, False, None)
    return out


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W", [(3, 64, 64), (2, 37, 70), (1, 128, 128)])
@pytest.mark.parametrize("path", ["narrow", "mfma"])
def test_c1_masked_dgrad(gpu_device, monkeypatch, dtype, N, H, W, path):
    if path == "mfma":
        monkeypatch.setenv("SPECENH_CONV_NO_NARROW", "1")
    rng = np.random.default_rng(N * 1000 + H + W)
    k, co = 5, 16
    x = torch.tensor(rng.standard_normal((N, H, W, 1)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((co, k, k, 1)) * 0.2, dtype=dtype, device=gpu_device)
    bias = torch.zeros(co, dtype=torch.float32, device=gpu_device)
    mask = torch.tensor(rng.standard_normal((N, H, W, co)), dtype=dtype, device=gpu_device)
    mask[0, 0, :4] = 0.0  # exact zeros: masked like negatives
    got = _conv(x, w, bias, k, co, 0, dtype, mask).double().cpu()
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
