"""GPU checks of the torch-op boundary (specenh/ops.py):
``torch.library.opcheck`` (schema / mutation annotations, autograd registration, fake
kernels vs the real outputs, AOT dispatch with dynamic shapes) on every operator, and the
differentiable API (specenh/autograd.py) against the autograd of the fp64 oracle."""
import numpy as np
import pytest
import torch

from oracle import autoencoder as ora

pytestmark = pytest.mark.gpu


def _cases(dev):
    g = torch.Generator(device="cpu").manual_seed(0)

    def r(*shape, dtype=torch.float32, lo=0.0, hi=1.0):
        return (lo + (hi - lo) * torch.rand(shape, generator=g)).to(dtype).to(dev)

    x = r(2, 4096, lo=-1)
    S = torch.empty(2, 128, 31, device=dev)
    A = r(3, 48, 40, lo=-1)
    xc, wc, bc = r(2, 8, 8, 4), r(8 * 9 * 4, lo=-0.3, hi=0.3), r(8, lo=-0.1, hi=0.1)
    xb = r(2, 16, 16, 16, dtype=torch.bfloat16)
    wb = r(32 * 25 * 16, dtype=torch.bfloat16, lo=-0.1, hi=0.1)
    dout = r(2, 8, 8, 8, lo=-1)
    pin = r(2, 8, 6, 4, lo=-1)
    pooled, am = torch.ops.specenh.maxpool2(pin)
    z, t = r(300, lo=-3, hi=3), r(300)
    w, gr, m, v = r(1000, lo=-1), r(1000, lo=-1), r(1000, lo=-1), r(1000)
    F64 = r(2, 32, 40, dtype=torch.float64)
    xt = r(2, 20, 12, 32, dtype=torch.float16)
    xb1 = r(2, 8, 8, 1, dtype=torch.bfloat16)
    pooled_b, am_b = r(2, 4, 4, 8, dtype=torch.bfloat16), torch.zeros(2, 4, 4, 8, dtype=torch.uint8,
                                                                     device=dev)
    pq_b = r(2, 4, 4, 32, dtype=torch.bfloat16, lo=-1)
    am_q = torch.randint(0, 4, (2, 4, 4, 32), dtype=torch.uint8, device=dev)
    wq_b = r(16 * 9 * 32, dtype=torch.bfloat16, lo=-0.1, hi=0.1)
    wt, bc16 = r(16 * 25 * 32, dtype=torch.float16, lo=-0.1, hi=0.1), r(16, lo=-0.1, hi=0.1)
    wo, bo = r(25 * 16, dtype=torch.float16, lo=-0.2, hi=0.2), r(1)
    Sp = r(1, 256, 3845)
    x3 = r(2, 3, 32, 64, dtype=torch.float16)
    xe = torch.rand(2, 12, 128, 1, device=dev, dtype=torch.float16)
    we1 = (torch.randn(16 * 25, device=dev) * 0.1).to(torch.float16)
    be1 = torch.randn(16, device=dev)
    we2 = (torch.randn(32 * 25 * 16, device=dev) * 0.05).to(torch.float16)
    be2 = torch.randn(32, device=dev)
    w3a, b3a = r(32 * 25 * 64, dtype=torch.float16, lo=-0.05, hi=0.05), r(32, lo=-0.1, hi=0.1)
    ops = torch.ops.specenh
    return [
        (ops.stft_psd, (x, 256, 128, "hann", 5e5, 0, 2, 1e-11, 7)),
        (ops.stft_psd_out, (x, 256, 128, "hann", 5e5, 0, 2, 1e-11, 7, S)),
        (ops.csd, (x, x.flip(1).contiguous(), 256, 128, "hamm", 5e5, 0, 2, 0)),
        (ops.csd, (x, x.flip(1).contiguous(), 256, 128, "hamm", 5e5, 0, 2, 1)),
        (ops.svd_denoise, (A, 0, 5, torch.float32)),
        (ops.svd_denoise, (A, 1, -1, torch.float16)),
        (ops.svd_denoise_out, (A, 2, 9, torch.empty_like(A))),
        (ops.svd_denoise_optimal, (A, 0)),
        (ops.svd_denoise_optimal_out, (A, 1, torch.empty_like(A),
                                       torch.empty(A.shape[0], dtype=torch.int32, device=dev),
                                       torch.empty(A.shape[0], dtype=torch.float64, device=dev))),
        (ops.conv2d, (xc, wc, bc, 3, 3, 8, 1, 1, 1, 1, 8, 8, 1)),
        (ops.conv2d, (xc, wc, None, 3, 3, 8, 1, 1, 1, 2, 16, 16, 0)),
        (ops.conv2d_out, (xc, wc, bc, 3, 3, 8, 1, 1, 1, 1, 8, 8, 2, None,
                          torch.empty(2, 8, 8, 8, device=dev), torch.empty(2, 8, 8, 8, device=dev),
                          False, None)),
        (ops.conv2d_out, (xb, wb, r(32), 5, 5, 32, 1, 2, 2, 1, 16, 16, 1, None, None,
                          torch.empty(2, 8, 8, 32, device=dev, dtype=torch.bfloat16), True,
                          torch.empty(2, 8, 8, 32, device=dev, dtype=torch.uint8))),
        (ops.conv2d_wgrad, (xc, dout, 3, 3, 1, 1, 1, 1)),
        (ops.conv2d_wgrad_out, (xc, dout, 3, 3, 1, 1, 1, 1, torch.zeros(8, 3, 3, 4, device=dev),
                                torch.zeros(8, device=dev),
                                torch.empty(1 << 20, dtype=torch.uint8, device=dev))),
        (ops.conv2d_wgrad_pooled_out, (xb1, pooled_b, am_b, pooled_b, 3, 3, 1, 1, 1, 1,
                                       torch.zeros(8, 3, 3, 1, device=dev),
                                       torch.zeros(8, device=dev),
                                       torch.empty(1 << 20, dtype=torch.uint8, device=dev))),
        (ops.conv2d_pooled_in_out, (pq_b, am_q, pq_b, wq_b, None, 3, 3, 16, 1, 1, 8, 8, 0,
                                    r(2, 8, 8, 16, dtype=torch.bfloat16, lo=-1),
                                    torch.empty(2, 8, 8, 16, device=dev, dtype=torch.bfloat16))),
        (ops.conv2d_wgrad_out, (xc, dout, 3, 3, 1, 1, 1, 1, torch.zeros(8, 3, 3, 4, device=dev),
                                torch.zeros(8, device=dev),
                                torch.empty(1 << 20, dtype=torch.uint8, device=dev), True)),
        (ops.convt_conv_out, (xt, wt, bc16, 16, 5, wo, bo, 5)),
        (ops.convt_conv_out_out, (xt, wt, bc16, 16, 5, wo, bo, 5,
                                  torch.empty(2, 40, 24, 1, device=dev))),
        (ops.convt_conv_out_train_out, (r(2, 4, 64, 32, dtype=torch.float16), wt, bc16, 16, 5, wo,
                                        bo, 5, torch.empty(2, 8, 128, 16, device=dev,
                                                           dtype=torch.float16),
                                        torch.empty(2, 8, 128, 1, device=dev),
                                        torch.empty(2, 8, 128, 1, device=dev,
                                                    dtype=torch.float16))),
        (ops.decoder3, (x3, w3a, b3a, 32, wt, bc16, 16, wo, bo, 5)),
        (ops.decoder3_out, (x3, w3a, b3a, 32, wt, bc16, 16, wo, bo, 5,
                            torch.empty(2, 12, 128, 1, device=dev))),
        (ops.encoder2, (xe, we1, be1, 16, we2, be2, 32, 5)),
        (ops.encoder2_out, (xe, we1, be1, 16, we2, be2, 32, 5,
                            torch.empty(2, 3, 32, 32, device=dev, dtype=torch.float16))),
        (ops.maxpool2, (pin,)),
        (ops.maxpool2_out, (pin, torch.empty_like(pooled), torch.empty_like(am))),
        (ops.maxpool2_bwd, (pooled.clone(), am, pooled)),
        (ops.maxpool2_bwd_out, (pooled.clone(), am, None, torch.empty_like(pin))),
        (ops.bce_logits, (z, t, torch.float32)),
        (ops.bce_logits_out, (z, t, torch.empty_like(z),
                              torch.zeros(1, dtype=torch.float64, device=dev))),
        (ops.adam_step_, (w, gr, m, v, 1e-3, 0.9, 0.999, 1e-7, 0.5,
                          torch.empty(1000, dtype=torch.bfloat16, device=dev))),
        (ops.adam_step_flip_, (w, gr, m, v, 1e-3, 0.9, 0.999, 1e-7, 0.5,
                               torch.empty(1000, dtype=torch.bfloat16, device=dev), [8, 300],
                               [3, 4, 8, 5, 2, 3],
                               [torch.empty(288, dtype=torch.bfloat16, device=dev),
                                torch.empty(150, dtype=torch.bfloat16, device=dev)])),
        (ops.weight_flip_transpose, (wc, 3, 4, 8)),
        (ops.weight_flip_transpose_out, (wc, 3, 4, 8, torch.empty_like(wc))),
        (ops.cast, (xc, torch.float16)),
        (ops.cast_out, (xc, torch.empty_like(xc, dtype=torch.bfloat16))),
        (ops.label_filter, (F64, 0)),
        (ops.label_filter, (F64, 2)),
        (ops.quantfilt, (F64, 0.9)),
        (ops.gaussblr, (F64, 31, 3, 0.0)),
        (ops.morph, (F64,)),
        (ops.strips_pack, (Sp, 256, 128, 30, torch.float32)),
        (ops.strips_unpack, (r(60, 256, 128, 1), 256, 128, 30)),
        (ops.strips_pack_out, (Sp, 256, 128, 30,
                               torch.empty(30, 256, 128, 1, device=dev, dtype=torch.bfloat16))),
        (ops.strips_unpack_out, (r(60, 256, 128, 1, dtype=torch.bfloat16), 256, 128, 30,
                                 torch.empty(2, 256, 3840, device=dev))),
    ]


def test_opcheck_every_operator(gpu_device):
    cases = _cases(gpu_device)
    seen = set()
    for op, args in cases:
        torch.library.opcheck(op, args)
        seen.add(op._qualified_op_name)
    from test_ops_registry import OPS
    assert seen == {f"specenh::{n}" for n in OPS}


def _oracle_grads(spec, params, x, y):
    tp = [None if p is None else {"W": torch.tensor(p["W"], dtype=torch.float64, requires_grad=True),
                                  "b": torch.tensor(p["b"], dtype=torch.float64, requires_grad=True)}
          for p in params]
    _, z = ora.forward(spec, tp, torch.tensor(x, dtype=torch.float64), return_logits=True)
    loss = ora.bce_from_logits(z, torch.tensor(y, dtype=torch.float64))
    loss.backward()
    g = []
    for p in tp:
        if p is not None:
            g += [p["W"].grad.numpy(), p["b"].grad.numpy()]
    return float(loss), z.detach().numpy(), g


def test_autograd_model_matches_oracle(gpu_device):
    """The reference's 3-layer autoencoder shape (reduced widths) written with
    specenh.autograd: logits, BCE loss and every parameter gradient vs fp64 autograd."""
    from specenh import autograd as F

    spec = ora.ae_spec(8, 16, 16, k=5)
    params = ora.glorot_params(spec, seed=3)
    rng = np.random.default_rng(4)
    for p in params:
        if p is not None:
            p["b"] = (0.05 * rng.standard_normal(p["b"].shape)).astype(np.float32)
    x = rng.uniform(0, 1, (3, 32, 32, 1)).astype(np.float32)
    y = rng.uniform(0, 1, (3, 32, 32, 1)).astype(np.float32)
    ref_loss, ref_z, ref_g = _oracle_grads(spec, params, x, y)

    dev = gpu_device
    tp = [None if p is None else
          {"W": torch.tensor(p["W"], device=dev, requires_grad=True),
           "b": torch.tensor(p["b"], device=dev, requires_grad=True)} for p in params]
    h = torch.tensor(x, device=dev)
    for lay, p in zip(spec, tp):
        if lay[0] == "pool":
            h = F.max_pool2(h)
            continue
        act = None if lay[4] == "sigmoid" else lay[4]  # the last layer yields logits
        fn = F.conv2d_same if lay[0] == "conv" else F.conv2d_transpose_same
        h = fn(h, p["W"], p["b"], act)
    loss = F.binary_crossentropy_with_logits(h, torch.tensor(y, device=dev))
    loss.backward()
    assert abs(float(loss) - ref_loss) <= 1e-5 * ref_loss
    z = h.detach().cpu().numpy()
    assert np.linalg.norm(z - ref_z) <= 1e-5 * np.linalg.norm(ref_z)
    got = []
    for p in tp:
        if p is not None:
            got += [p["W"].grad.cpu().numpy(), p["b"].grad.cpu().numpy()]
    for a, b in zip(got, ref_g):
        assert np.linalg.norm(a - b) <= 1e-5 * np.linalg.norm(b)


def test_autograd_model_bf16_end_to_end(gpu_device):
    """The docstring example in bfloat16: a bf16 last layer's logits go
    straight into binary_crossentropy_with_logits (widened to fp32 inside, the gradient
    flowing back through the cast). Against fp64 autograd on the same bf16-rounded inputs
    and weights: loss within 1e-2, logits within 5e-2 normwise, gradients within 0.2 normwise
    (bf16 activations, output gradients and backward maps: 8-bit mantissas; the small
    gradients of this 3-image batch measured up to ~0.1 — a missing or mis-signed term
    gives ~1)."""
    from specenh import autograd as F

    spec = ora.ae_spec(8, 16, 16, k=5)
    params = ora.glorot_params(spec, seed=5)
    rng = np.random.default_rng(6)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).float().numpy()  # noqa: E731
    for p in params:
        if p is not None:
            p["W"] = bf(p["W"])
            p["b"] = (0.05 * rng.standard_normal(p["b"].shape)).astype(np.float32)
    x = bf(rng.uniform(0, 1, (3, 32, 32, 1)).astype(np.float32))
    y = rng.uniform(0, 1, (3, 32, 32, 1)).astype(np.float32)
    ref_loss, ref_z, ref_g = _oracle_grads(spec, params, x, y)

    dev = gpu_device
    tp = [None if p is None else
          {"W": torch.tensor(p["W"], device=dev).to(torch.bfloat16).requires_grad_(),
           "b": torch.tensor(p["b"], device=dev, requires_grad=True)} for p in params]
    h = torch.tensor(x, device=dev).to(torch.bfloat16)
    for lay, p in zip(spec, tp):
        if lay[0] == "pool":
            h = F.max_pool2(h)
            continue
        act = None if lay[4] == "sigmoid" else lay[4]
        fn = F.conv2d_same if lay[0] == "conv" else F.conv2d_transpose_same
        h = fn(h, p["W"], p["b"], act)
    assert h.dtype == torch.bfloat16
    loss = F.binary_crossentropy_with_logits(h, torch.tensor(y, device=dev))
    loss.backward()
    assert abs(float(loss) - ref_loss) <= 1e-2 * ref_loss
    z = h.detach().float().cpu().numpy()
    assert np.linalg.norm(z - ref_z) <= 5e-2 * np.linalg.norm(ref_z)
    got = []
    for p in tp:
        if p is not None:
            got += [p["W"].grad.float().cpu().numpy(), p["b"].grad.cpu().numpy()]
    for a, b in zip(got, ref_g):
        assert np.linalg.norm(a - b) <= 0.2 * np.linalg.norm(b)


def test_autograd_sigmoid_output_grad(gpu_device):
    """Conv2D with a fused sigmoid: the gradient through the activation."""
    from specenh import autograd as F

    rng = np.random.default_rng(6)
    x = rng.uniform(0, 1, (2, 12, 10, 3)).astype(np.float32)
    W = (0.3 * rng.standard_normal((3, 3, 3, 4))).astype(np.float32)
    b = (0.1 * rng.standard_normal(4)).astype(np.float32)
    xt = torch.tensor(x, device=gpu_device, requires_grad=True)
    Wt = torch.tensor(W, device=gpu_device, requires_grad=True)
    bt = torch.tensor(b, device=gpu_device, requires_grad=True)
    out = F.conv2d_same(xt, Wt, bt, "sigmoid")
    (out * out).sum().backward()
    xr = torch.tensor(x, dtype=torch.float64, requires_grad=True)
    Wr = torch.tensor(W, dtype=torch.float64, requires_grad=True)
    br = torch.tensor(b, dtype=torch.float64, requires_grad=True)
    o = torch.sigmoid(ora.conv2d_same(xr, Wr, br))
    (o * o).sum().backward()
    for a, r in ((xt, xr), (Wt, Wr), (bt, br)):
        ga, gr = a.grad.cpu().double().numpy(), r.grad.numpy()
        assert np.linalg.norm(ga - gr) <= 1e-5 * np.linalg.norm(gr)
