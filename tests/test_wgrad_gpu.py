"""Weight / bias gradients of the 16-bit conv layers (specenh_conv2d_wgrad) on the GPU.

The MFMA paths (csrc/conv_ae.hip wgrad_tr_kernel: C % 16 == 0 or C == 1 via an LDS im2col
block, transposed LDS fragment reads; wgrad_trp_kernel: the four Conv2DTranspose phases per
workgroup, SPECENH_WGRAD_PERPHASE=1 forces one phase per workgroup; wgrad_co1_kernel: one
output channel as shifted-input x shifted-dOut MFMAs, SPECENH_WGRAD_NO_CO1=1 turns it off)
and the generic gather kernel (SPECENH_WGRAD_GENERIC=1) are both checked against the
float64 im2col product dW = dZ^T A of the header's gather formula (test_ae_mapping.igemm)
on the same bf16 / f16-rounded operands: products are exact in the fp32 accumulators, so
only the summation order differs (normwise relative error <= 2e-5). Every geometry of the
reference autoencoder's layers is covered (stride-1 'same' convs and the stride-2
Conv2DTranspose phases), plus partial tiles, a 1-channel output and odd batch sizes."""
import numpy as np
import pytest
import torch

from specenh import ae
from test_ae_mapping import igemm

pytestmark = pytest.mark.gpu

# (kind, cin, cout, k, H, W, N): the C4/C5 model layers at reduced size, ragged tiles
CASES = [("conv", 16, 32, 5, 20, 18, 3), ("conv", 32, 64, 5, 16, 16, 2),
         ("conv", 16, 1, 5, 24, 20, 2), ("conv", 32, 16, 3, 9, 13, 3),
         ("convT", 64, 64, 5, 8, 8, 2), ("convT", 64, 32, 5, 10, 6, 3),
         ("convT", 32, 16, 5, 12, 12, 2), ("conv", 64, 48, 5, 17, 17, 1),
         ("conv", 1, 16, 5, 33, 18, 2), ("conv", 1, 32, 3, 16, 16, 1),
         ("conv", 16, 1, 5, 37, 29, 3), ("conv", 16, 1, 3, 16, 40, 1),
         # 7 x 7 (hyperparam_scan.py:153-161; round 5: two 28-tap groups per workgroup row)
         ("conv", 32, 32, 7, 23, 19, 2), ("conv", 32, 1, 7, 21, 30, 2),
         ("convT", 32, 32, 7, 9, 7, 2), ("conv", 16, 24, 7, 16, 16, 1), ("conv", 1, 32, 7, 20, 14, 2)]


def _reference(x, dz, op):
    k = op.k
    OH, OW = dz.shape[1:3]
    A, _ = igemm(x, np.zeros((1, k * k * x.shape[3])), k, OH, OW, op.fwd_geom())
    cout = dz.shape[3]
    dbt = dz.reshape(-1, cout).T @ A          # [co][(ky, kx, ci)]
    return dbt.reshape(cout, k, k, x.shape[3]), dz.reshape(-1, cout).sum(0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("kind,cin,cout,k,H,W,N", CASES)
@pytest.mark.parametrize("path", ["mfma", "mfma_alt", "generic"])
def test_wgrad_matches_im2col(gpu_device, kernel_variant, dtype, kind, cin, cout, k, H, W, N, path):
    if path == "generic":
        kernel_variant("WGRAD_GENERIC", 1)
    elif path == "mfma_alt":  # the general MFMA kernel where a specialised one exists
        if kind != "convT" and cout != 1:
            pytest.skip("no specialised launch for this geometry")
        kernel_variant("WGRAD_PERPHASE", 1)
        kernel_variant("WGRAD_NO_CO1", 1)
    op = ae.ConvOp(kind, cin, cout, k, "relu", stride=2 if kind == "convT" else 1)
    OH, OW = op.out_hw(H, W)
    rng = np.random.default_rng(cin * 131 + cout * 7 + k + H)
    x = torch.tensor(rng.standard_normal((N, H, W, cin)), dtype=dtype)
    dz = torch.tensor(rng.standard_normal((N, OH, OW, cout)), dtype=dtype)
    s, pt, pl, dil = op.fwd_geom()
    dw, db = torch.ops.specenh.conv2d_wgrad(x.to(gpu_device), dz.to(gpu_device), k, k, s, pt, pl,
                                            dil)
    ref_w, ref_b = _reference(x.double().numpy(), dz.double().numpy(), op)
    got_w, got_b = dw.double().cpu().numpy(), db.double().cpu().numpy()
    assert np.linalg.norm(got_w - ref_w) <= 2e-5 * np.linalg.norm(ref_w)
    assert np.linalg.norm(got_b - ref_b) <= 2e-5 * np.linalg.norm(ref_b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("perphase", [False, True])
def test_wgrad_mfma_is_bitwise_deterministic(gpu_device, kernel_variant, dtype, perphase):
    if perphase:
        kernel_variant("WGRAD_PERPHASE", 1)
    op = ae.ConvOp("convT", 32, 16, 5, "relu", stride=2)
    rng = np.random.default_rng(5)
    x = torch.tensor(rng.standard_normal((4, 32, 32, 32)), dtype=dtype, device=gpu_device)
    dz = torch.tensor(rng.standard_normal((4, 64, 64, 16)), dtype=dtype, device=gpu_device)
    s, pt, pl, dil = op.fwd_geom()
    a = torch.ops.specenh.conv2d_wgrad(x, dz, 5, 5, s, pt, pl, dil)
    b = torch.ops.specenh.conv2d_wgrad(x, dz, 5, 5, s, pt, pl, dil)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_wgrad_co1_is_bitwise_deterministic(gpu_device, dtype):
    op = ae.ConvOp("conv", 16, 1, 5, "sigmoid")
    rng = np.random.default_rng(6)
    x = torch.tensor(rng.standard_normal((8, 64, 64, 16)), dtype=dtype, device=gpu_device)
    dz = torch.tensor(rng.standard_normal((8, 64, 64, 1)), dtype=dtype, device=gpu_device)
    s, pt, pl, dil = op.fwd_geom()
    a = torch.ops.specenh.conv2d_wgrad(x, dz, 5, 5, s, pt, pl, dil)
    b = torch.ops.specenh.conv2d_wgrad(x, dz, 5, 5, s, pt, pl, dil)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
