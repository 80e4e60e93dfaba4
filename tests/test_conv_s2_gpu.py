"""Stride-2 convolutions (the input gradient of a Conv2DTranspose) on the GPU: the
de-interleaved 16-channel patch kernel (csrc/conv_ae.hip conv_patch_kernel<..., S2>) and the
generic gather kernel (SPECENH_CONV_NO_S2=1) against a float64 torch convolution of the same
16-bit operands, with the optional ReLU mask of the backward pass. Products of 16-bit values
are exact in fp32: the results differ from float64 by the fp32 summation and one rounding
to the 16-bit type."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import specenh  # noqa: F401  (registers torch.ops.specenh.*)

pytestmark = pytest.mark.gpu

# (C, CO, K, H, W, N, pad): the reference model's Conv2DTranspose input gradients
# (C = channels of dOut) at reduced size, plus ragged tiles and other kernel sizes
CASES = [(16, 32, 5, 40, 36, 2, 2), (32, 64, 5, 32, 32, 2, 2), (64, 64, 5, 18, 34, 1, 2),
         (16, 16, 3, 33, 17, 3, 1), (32, 48, 4, 20, 20, 2, 1), (64, 16, 5, 64, 64, 1, 2)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,CO,K,H,W,N,pad", CASES)
@pytest.mark.parametrize("path", ["patch", "generic"])
@pytest.mark.parametrize("masked", [False, True])
def test_stride2_conv(gpu_device, kernel_variant, dtype, C, CO, K, H, W, N, pad, path, masked):
    if path == "generic":
        kernel_variant("CONV_NO_S2", 1)
    rng = np.random.default_rng(C * 7 + CO + K + H)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    x = torch.tensor(rng.standard_normal((N, H, W, C)), dtype=dtype, device=gpu_device)
    w = torch.tensor(rng.standard_normal((CO, K, K, C)) * 0.1, dtype=dtype, device=gpu_device)
    bias = torch.tensor(rng.standard_normal(CO), dtype=torch.float32, device=gpu_device)
    mask = None
    if masked:
        mask = torch.tensor(rng.standard_normal((N, OH, OW, CO)), dtype=dtype, device=gpu_device)
    out = torch.empty((N, OH, OW, CO), dtype=dtype, device=gpu_device)
    torch.ops.specenh.conv2d_out(x, w, bias, K, K, CO, 2, pad, pad, 1, OH, OW, 0, mask, None,
                                 out, False, None)
    xd = F.pad(x.double().cpu().permute(0, 3, 1, 2), (pad, 2 * K, pad, 2 * K))
    wd = w.double().cpu().permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, stride=2)[:, :, :OH, :OW] + bias.double().cpu().view(1, -1, 1, 1)
    mag = F.conv2d(xd.abs(), wd.abs(), stride=2)[:, :, :OH, :OW] + bias.double().cpu().abs().view(1, -1, 1, 1)
    ref, mag = ref.permute(0, 2, 3, 1), mag.permute(0, 2, 3, 1)
    if masked:
        ref = torch.where(mask.double().cpu() > 0, ref, torch.zeros_like(ref))
    got = out.double().cpu()
    eps = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    assert torch.all((got - ref).abs() <= eps * ref.abs() + 1e-5 * mag + 1e-30)
