"""GPU parity of the conv autoencoder (csrc/conv_ae.hip via the C-ABI) against the
oracle (oracle/autoencoder.py, a PyTorch-CPU restatement of the Keras model — parity
vs Keras itself is unpinned: TensorFlow is absent, SURVEY.md §8 c).

Tolerances (SURVEY.md §8 d, oracle/checks.py):
  * fp32 compute: outputs ||d||_inf / ||ref||_inf <= 1e-5; gradients per tensor
    ||d||_2 / ||ref||_2 <= 1e-5 (fp32 accumulation over up to 10^6 terms).
  * fp16 / bf16 compute: on weights whose outputs carry a real signal (the trained fixture
    tests/golden/ae_c4_trained.npz, or gain-scaled glorot for the reference's other
    variants), out_rel = ||y - y_ref|| / ||y_ref - mean(y_ref)|| and
    logit_rel = ||z - z_ref|| / ||z_ref|| within checks.TOL (fp16 2e-3, bf16 1e-2; a dropped
    MFMA k-step moves them by >= 1.3e-2, tests/test_ae_sensitivity.py); bf16 gradient
    cosine similarity >= 0.99.
"""
import math

import numpy as np
import pytest
import torch

from oracle import autoencoder as ora
from oracle import checks

pytestmark = pytest.mark.gpu

TOL_OUT = 1e-5
TOL_GRAD = 1e-5


def _ae():
    from specenh import ae
    return ae


def oracle_spec(ops):
    spec = []
    for op in ops:
        if op.kind == "pool":
            spec.append(("pool",))
        else:
            spec.append((op.kind, op.cin, op.cout, op.k, op.act))
    return spec


def make(ops, hwc, dtype="float32", seed=0, device="cuda:0"):
    ae = _ae()
    eng = ae.AutoencoderEngine(ops, hwc, compute_dtype=dtype, device=device)
    params = ora.glorot_params(oracle_spec(ops), seed=seed)
    rng = np.random.default_rng(seed + 100)
    for p in params:  # non-zero biases exercise the bias path
        if p is not None:
            p["b"] = (0.05 * rng.standard_normal(p["b"].shape)).astype(np.float32)
    ws = []
    for p in params:
        if p is not None:
            ws += [p["W"], p["b"]]
    eng.set_keras_weights(ws)
    return eng, params


def ref_forward(ops, params, x, grads=False, y=None):
    tp = [None if p is None else {"W": torch.tensor(p["W"], dtype=torch.float64,
                                                    requires_grad=grads),
                                  "b": torch.tensor(p["b"], dtype=torch.float64,
                                                    requires_grad=grads)} for p in params]
    xt = torch.tensor(x, dtype=torch.float64)
    out, z = ora.forward(oracle_spec(ops), tp, xt, return_logits=True)
    if not grads:
        return out.numpy(), z.numpy()
    loss = ora.bce_from_logits(z, torch.tensor(y, dtype=torch.float64))
    loss.backward()
    g = []
    for p in tp:
        if p is not None:
            g += [p["W"].grad.numpy(), p["b"].grad.numpy()]
    return out.detach().numpy(), float(loss), g


def engine_grads(eng):
    ae = _ae()
    host = eng.g.cpu().numpy()
    out = []
    for op in eng.ops:
        if isinstance(op, ae.ConvOp):
            out.append(ae.gemm_to_keras(op, host[op.off_w:op.off_w + op.n_w]))
            out.append(host[op.off_b:op.off_b + op.cout])
    return out


def normwise(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def trained_c4(n=6, seed0=9100):
    """The trained reference-model weights and C4-style (input, target) pairs."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_ae_weights import c4_pairs, load
    x, y = c4_pairs(n, seed0)
    return load(), x, y


def set_params(eng, ws):
    """Keras weight list -> engine + the oracle's per-layer params list."""
    eng.set_keras_weights(ws)
    it, params = iter(ws), []
    for op in eng.ops:
        params.append(None if op.kind == "pool" else {"W": next(it), "b": next(it)})
    return params


def lowp_errors(eng, params, x):
    """(out_rel, logit_rel) of the engine's inference output and training-mode logits vs
    the fp64 oracle."""
    ref, zref = ref_forward(eng.ops, params, x)
    got = eng.forward(upload(eng, x), train=False).cpu().numpy()
    eng.forward(upload(eng, x), train=True)
    z = eng.last_logits().cpu().numpy()
    return checks.out_rel(got, ref), checks.logit_rel(z, zref), float(np.std(zref))


def ref_model_ops(c1=16, c2=32, c3=64, k=5):
    ae = _ae()
    C = ae.ConvOp
    P = ae.PoolOp
    return [C("conv", 1, c1, k, "relu"), P(), C("conv", c1, c2, k, "relu"), P(),
            C("conv", c2, c3, k, "relu"), P(), C("convT", c3, c3, k, "relu", stride=2),
            C("convT", c3, c2, k, "relu", stride=2), C("convT", c2, c1, k, "relu", stride=2),
            C("conv", c1, 1, k, "sigmoid")]


def upload(eng, a):
    return eng.to_compute(torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)))


# ----------------------------------------------------------------------------- single ops
SINGLE = [("conv", 1, 16, 5, 20, 12), ("conv", 16, 32, 5, 16, 16), ("conv", 24, 1, 3, 9, 7),
          ("conv", 8, 40, 5, 8, 8), ("convT", 64, 64, 5, 8, 8), ("convT", 32, 16, 5, 10, 6),
          ("convT", 3, 5, 3, 5, 7), ("convT", 4, 8, 4, 6, 6)]


@pytest.mark.parametrize("kind,cin,cout,k,H,W", SINGLE)
def test_single_layer_forward_and_wgrad_fp32(gpu_device, kind, cin, cout, k, H, W):
    ae = _ae()
    ops = [ae.ConvOp(kind, cin, cout, k, "sigmoid", stride=2 if kind == "convT" else 1)]
    eng, params = make(ops, (H, W, cin), seed=cin * 7 + cout)
    rng = np.random.default_rng(1)
    x = rng.uniform(0, 1, (3, H, W, cin)).astype(np.float32)
    out_shape = (3,) + eng.output_shape
    y = rng.uniform(0, 1, out_shape).astype(np.float32)
    ref, ref_loss, ref_g = ref_forward(ops, params, x, grads=True, y=y)
    got = eng.forward(upload(eng, x), train=False).cpu().numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() / np.abs(ref).max() <= TOL_OUT
    eng.forward(upload(eng, x), train=True)
    loss = eng.loss_and_grad(upload(eng, y))
    eng.backward()
    assert abs(float(loss.item()) / y.size - ref_loss) <= 1e-6 * abs(ref_loss)
    for a, b in zip(engine_grads(eng), ref_g):
        assert normwise(a, b) <= TOL_GRAD


@pytest.mark.parametrize("first,second", [("conv", "conv"), ("conv", "convT"),
                                          ("convT", "conv"), ("convT", "convT")])
def test_two_layer_dgrad_through_relu_fp32(gpu_device, first, second):
    """Input gradients (dgrad conv + fused ReLU mask) of both layer kinds."""
    ae = _ae()
    ops = [ae.ConvOp(first, 8, 16, 5, "relu", stride=2),
           ae.ConvOp(second, 16, 1, 5, "sigmoid", stride=2)]
    eng, params = make(ops, (8, 6, 8), seed=5)
    rng = np.random.default_rng(2)
    x = rng.uniform(0, 1, (2, 8, 6, 8)).astype(np.float32)
    y = rng.uniform(0, 1, (2,) + eng.output_shape).astype(np.float32)
    _, ref_loss, ref_g = ref_forward(ops, params, x, grads=True, y=y)
    eng.forward(upload(eng, x), train=True)
    eng.loss_and_grad(upload(eng, y))
    eng.backward()
    for a, b in zip(engine_grads(eng), ref_g):
        assert normwise(a, b) <= TOL_GRAD


def test_pool_backward_routes_to_argmax_with_relu_mask(gpu_device):
    ae = _ae()
    ops = [ae.ConvOp("conv", 1, 8, 3, "relu"), ae.PoolOp(), ae.ConvOp("conv", 8, 1, 3, "sigmoid")]
    eng, params = make(ops, (16, 12, 1), seed=9)
    rng = np.random.default_rng(3)
    x = rng.uniform(0, 1, (4, 16, 12, 1)).astype(np.float32)
    y = rng.uniform(0, 1, (4, 8, 6, 1)).astype(np.float32)
    _, _, ref_g = ref_forward(ops, params, x, grads=True, y=y)
    eng.forward(upload(eng, x), train=True)
    eng.loss_and_grad(upload(eng, y))
    eng.backward()
    for a, b in zip(engine_grads(eng), ref_g):
        assert normwise(a, b) <= TOL_GRAD


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hw,co,k,relu", [((128, 128), 16, 5, True), ((20, 36), 8, 3, True),
                                          ((34, 18), 24, 5, False)])
def test_wgrad_pooled_equals_pool_backward_then_wgrad(gpu_device, dtype, hw, co, k, relu):
    """specenh_conv2d_wgrad_pooled (the first Conv2D's weight gradient formed from its pool's
    gradient, argmax and ReLU mask while the tiles are staged; it overwrites dw / dbias) is
    bitwise specenh_maxpool2_bwd + specenh_conv2d_wgrad into zeroed buffers, incl. ragged
    tiles and no ReLU mask."""
    from specenh.ops import ops, wgrad_workspace
    dev = torch.device(gpu_device)
    g = torch.Generator(device=dev).manual_seed(5)
    N, (H, W) = 3, hw
    x = torch.rand(N, H, W, 1, device=dev, generator=g).to(dtype)
    conv = (torch.randn(N, H, W, co, device=dev, generator=g)).to(dtype)
    pooled, am = ops.maxpool2(conv)
    dpool = torch.randn(N, H // 2, W // 2, co, device=dev, generator=g).to(dtype)
    ws = wgrad_workspace(x, conv, k, k)
    p = (k - 1) // 2
    res = []
    for fused in (True, False):
        # the pooled form OVERWRITES dw / dbias (no zeroing launch before it)
        dw = torch.full((co, k, k, 1), 7.0 if fused else 0.0, device=dev)
        db = torch.full((co,), -3.0 if fused else 0.0, device=dev)
        if fused:
            ops.conv2d_wgrad_pooled_out(x, dpool, am, pooled if relu else None, k, k, 1, p, p, 1,
                                        dw, db, ws)
        else:
            d = torch.empty_like(conv)
            ops.maxpool2_bwd_out(dpool, am, pooled if relu else None, d)
            ops.conv2d_wgrad_out(x, d, k, k, 1, p, p, 1, dw, db, ws)
        res.append((dw, db))
    assert float(res[1][0].abs().max()) > 0
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_engine_wgrad_pooled_is_bitwise(gpu_device):
    """The engine's first-layer weight gradient through conv2d_wgrad_pooled (default) and
    through the pool backward + wgrad (wgrad_pooled = False): bitwise equal gradients."""
    ops_ = ref_model_ops()
    rng = np.random.default_rng(21)
    x = rng.uniform(0, 1, (8, 64, 64, 1))
    y = rng.uniform(0, 1, (8, 64, 64, 1))
    grads = []
    for pooled in (True, False):
        eng, _ = make(ops_, (64, 64, 1), dtype="mixed_bfloat16", seed=23)
        assert eng.wgrad_pooled
        eng.wgrad_pooled = pooled
        eng.forward(upload(eng, x), train=True)
        eng.loss_and_grad(upload(eng, y))
        eng.backward()
        grads.append(eng.g.clone())
    assert float(grads[0].abs().max()) > 0
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hw,c,co,k", [((32, 32), 64, 32, 5), ((64, 64), 32, 16, 5),
                                        ((18, 22), 16, 32, 3), ((10, 6), 32, 48, 7)])
@pytest.mark.parametrize("relu", [True, False])
def test_pool_routed_equals_pool_backward(gpu_device, dtype, hw, c, co, k, relu):
    """Round 6: the pooled Conv2Ds after the first (C = 16 / 32 / 64 in, the C4 model's conv2
    and conv3 at (64, 64) / (32, 32)) take their input gradient (specenh_conv2d_pooled_in) and
    weight gradient (specenh_conv2d_wgrad_pooled, now any C % 16 == 0) straight from the
    pool's gradient: bitwise specenh_maxpool2_bwd followed by specenh_conv2d / _wgrad, incl.
    the ReLU mask of the layer below, ragged tiles and no pooled-output mask."""
    from specenh import _lib
    from specenh.ops import ops, wgrad_workspace
    dev = torch.device(gpu_device)
    g = torch.Generator(device=dev).manual_seed(7 + c + k)
    N, (H, W) = 3, hw
    p = (k - 1) // 2
    # the conv's input (its own gradient's ReLU mask) and its pre-pool output's pool
    x = torch.randn(N, H, W, co, device=dev, generator=g).to(dtype)
    pre = torch.randn(N, H, W, c, device=dev, generator=g).to(dtype)
    pooled, am = ops.maxpool2(pre)
    dpool = torch.randn(N, H // 2, W // 2, c, device=dev, generator=g).to(dtype)
    wd = (torch.randn(co, k, k, c, device=dev, generator=g) * 0.1).to(dtype)
    mask = x if relu else None
    pm = pooled if relu else None
    # input gradient
    d = torch.empty_like(pre)
    ops.maxpool2_bwd_out(dpool, am, pm, d)
    ref = torch.full((N, H, W, co), float("nan"), device=dev, dtype=dtype)
    ops.conv2d_out(d, wd, None, k, k, co, 1, p, p, 1, H, W, 0, mask, None, ref, False, None)
    got = torch.full_like(ref, float("nan"))
    ops.conv2d_pooled_in_out(dpool, am, pm, wd, None, k, k, co, p, p, H, W, 0, mask, got)
    torch.cuda.synchronize()
    assert "conv_patch_kernel" in _lib.last_kernel_name()
    assert bool(torch.isfinite(ref).all()) and float(ref.float().abs().max()) > 0
    assert torch.equal(got, ref)
    # weight gradient of the conv whose input is x (C = co) and output the pre-pool map
    ws = wgrad_workspace(x, pre, k, k)
    res = []
    for fused in (True, False):
        dw = torch.full((c, k, k, co), 7.0 if fused else 0.0, device=dev)
        db = torch.full((c,), -3.0 if fused else 0.0, device=dev)
        if fused:
            ops.conv2d_wgrad_pooled_out(x, dpool, am, pm, k, k, 1, p, p, 1, dw, db, ws)
        else:
            ops.conv2d_wgrad_out(x, d, k, k, 1, p, p, 1, dw, db, ws)
        res.append((dw, db))
    torch.cuda.synchronize()
    assert float(res[1][0].abs().max()) > 0
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("dtype", ["mixed_bfloat16", "mixed_float16"])
def test_engine_pool_routed_is_bitwise(gpu_device, monkeypatch, dtype):
    """The engine's pool-routed backward (round 6 default: no pool backward launches for
    conv2 / conv3) and the pool backward + plain launches (SPECENH_NO_POOL_ROUTED=1):
    bitwise equal gradients, with the weight gradients on the second stream and serial."""
    ops_ = ref_model_ops()
    rng = np.random.default_rng(29)
    x = rng.uniform(0, 1, (8, 64, 64, 1))
    y = rng.uniform(0, 1, (8, 64, 64, 1))
    for serial in ("0", "1"):
        monkeypatch.setenv("SPECENH_WGRAD_SERIAL", serial)
        grads = []
        for off in ("0", "1"):
            monkeypatch.setenv("SPECENH_NO_POOL_ROUTED", off)
            eng, _ = make(ops_, (64, 64, 1), dtype=dtype, seed=31)
            assert eng.pool_routed == ({2, 4} if off == "0" else set())
            eng.forward(upload(eng, x), train=True)
            eng.loss_and_grad(upload(eng, y))
            eng.backward()
            grads.append(eng.g.clone())
        assert float(grads[0].abs().max()) > 0
        assert torch.equal(grads[0], grads[1])


# ----------------------------------------------------------------------------- full model
def test_reference_model_forward_fp32(gpu_device):
    ops = ref_model_ops()
    eng, params = make(ops, (128, 128, 1), seed=11)
    x = np.random.default_rng(4).uniform(0, 1, (4, 128, 128, 1)).astype(np.float32)
    ref, _ = ref_forward(ops, params, x)
    got = eng.forward(upload(eng, x), train=False).cpu().numpy()
    assert np.abs(got - ref).max() / np.abs(ref).max() <= TOL_OUT


def test_reference_model_gradients_fp32(gpu_device):
    ops = ref_model_ops()
    eng, params = make(ops, (128, 128, 1), seed=12)
    rng = np.random.default_rng(5)
    x = rng.uniform(0, 1, (4, 128, 128, 1)).astype(np.float32)
    y = rng.uniform(0, 1, (4, 128, 128, 1)).astype(np.float32)
    _, ref_loss, ref_g = ref_forward(ops, params, x, grads=True, y=y)
    eng.forward(upload(eng, x), train=True)
    loss = eng.loss_and_grad(upload(eng, y))
    eng.backward()
    assert abs(float(loss.item()) / y.size - ref_loss) <= 1e-6 * ref_loss
    errs = [normwise(a, b) for a, b in zip(engine_grads(eng), ref_g)]
    assert max(errs) <= TOL_GRAD, errs


def test_reference_model_bf16_relative_and_gradients(gpu_device):
    """mixed_bfloat16 on the trained weights and C4-style data: output and logits within
    checks.TOL of the fp64 oracle, loss within 1e-3 (the trained loss is ~0.18, not the
    0.69 of an untrained model), gradient cosine >= 0.99 per tensor."""
    ops = ref_model_ops()
    eng, _ = make(ops, (128, 128, 1), dtype="mixed_bfloat16")
    ws, x, y = trained_c4(4)
    params = set_params(eng, ws)
    o, zr, zstd = lowp_errors(eng, params, x)
    assert zstd > 1.0
    tol = checks.TOL["mixed_bfloat16"]
    assert o <= tol["out_rel"] and zr <= tol["logit_rel"], (o, zr)
    _, ref_loss, ref_g = ref_forward(ops, params, x, grads=True, y=y)
    assert ref_loss < 0.4
    eng.forward(upload(eng, x), train=True)
    loss = eng.loss_and_grad(upload(eng, y))
    eng.backward()
    assert abs(float(loss.item()) / y.size - ref_loss) <= 1e-3 * ref_loss
    for a, b in zip(engine_grads(eng), ref_g):
        cos = float(np.dot(a.ravel(), b.ravel()) /
                    (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))
        if np.linalg.norm(b) > 0:
            assert cos >= 0.99


def test_adam_trajectory_fp32_matches_keras_adam(gpu_device):
    """10 fit() steps (forward, BCE, backward, Keras Adam) vs oracle.train_step."""
    ops = ref_model_ops(4, 8, 8, 5)
    eng, params = make(ops, (32, 32, 1), seed=21)
    rng = np.random.default_rng(7)
    x = rng.uniform(0, 1, (8, 32, 32, 1)).astype(np.float32)
    y = (x > 0.5).astype(np.float32)
    spec = oracle_spec(ops)
    tp = [None if p is None else {"W": torch.tensor(p["W"], dtype=torch.float64,
                                                    requires_grad=True),
                                  "b": torch.tensor(p["b"], dtype=torch.float64,
                                                    requires_grad=True)} for p in params]
    opt = ora.KerasAdam()
    xt, yt = torch.tensor(x, dtype=torch.float64), torch.tensor(y, dtype=torch.float64)
    xd, yd = upload(eng, x), upload(eng, y)
    w0 = [w.copy() for w in eng.get_keras_weights()]
    for step in range(10):
        ref_loss = ora.train_step(spec, tp, xt, yt, opt)
        loss = float(eng.train_step(xd, yd).item()) / y.size
        assert abs(loss - ref_loss) <= 1e-4 * ref_loss, (step, loss, ref_loss)
    ref_w = []
    for p in tp:
        if p is not None:
            ref_w += [p["W"].detach().numpy(), p["b"].detach().numpy()]
    got_w = eng.get_keras_weights()
    moved = np.sqrt(sum(np.sum((r - a) ** 2) for r, a in zip(ref_w, w0)))
    diff = np.sqrt(sum(np.sum((r - g) ** 2) for r, g in zip(ref_w, got_w)))
    assert diff <= 1e-2 * moved


def test_adam_kernel_formula(gpu_device):
    from specenh import _lib
    L = _lib.lib()
    rng = np.random.default_rng(8)
    n = 10_000
    w, g, m, v = (rng.standard_normal(n).astype(np.float32) for _ in range(4))
    v = np.abs(v)
    d = [torch.from_numpy(a.copy()).to(gpu_device) for a in (w, g, m, v)]
    wb = torch.empty(n, dtype=torch.bfloat16, device=gpu_device)
    lr_t, b1, b2, eps, sc = 1e-3 * math.sqrt(1 - 0.999 ** 3) / (1 - 0.9 ** 3), 0.9, 0.999, 1e-7, 0.5
    import ctypes
    _lib.check(L.specenh_adam_step(*(ctypes.c_void_p(t.data_ptr()) for t in d), n, lr_t, b1, b2,
                                   eps, sc, ctypes.c_void_p(wb.data_ptr()), 1, None))
    torch.cuda.synchronize()
    g2 = g.astype(np.float64) * sc
    m2 = b1 * m + (1 - b1) * g2
    v2 = b2 * v + (1 - b2) * g2 * g2
    w2 = w - lr_t * m2 / (np.sqrt(v2) + eps)
    np.testing.assert_allclose(d[0].cpu().numpy(), w2, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(d[2].cpu().numpy(), m2, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(d[3].cpu().numpy(), v2, rtol=1e-6, atol=1e-7)
    assert torch.equal(wb, d[0].to(torch.bfloat16))


@pytest.mark.parametrize("lowp", [None, torch.bfloat16, torch.float16])
def test_adam_flip_equals_adam_then_flips(gpu_device, lowp):
    """specenh_adam_step_flip (one launch) == specenh_adam_step + one
    specenh_weight_flip_transpose per layer, bitwise, on the C4 model's weight layout."""
    import bench
    from specenh import ae
    from specenh.ops import ops  # the torch.ops.specenh namespace, as specenh.ae uses it
    dt = {None: "float32", torch.bfloat16: "mixed_bfloat16", torch.float16: "float16"}[lowp]
    engs = []
    for _ in range(2):
        e = ae.AutoencoderEngine(bench.ae_ops(), (128, 128, 1), compute_dtype=dt, device=gpu_device)
        e.set_keras_weights(bench.ae_weights())
        gen = torch.Generator(device=gpu_device).manual_seed(3)
        e.g.copy_(torch.randn(e.g.shape, device=gpu_device, generator=gen))
        e.m.copy_(torch.randn(e.m.shape, device=gpu_device, generator=gen))
        e.v.copy_(torch.rand(e.v.shape, device=gpu_device, generator=gen))
        engs.append(e)
    assert len(engs[0].w_d) == 6
    engs[0].adam(1e-3, grad_scale=0.5)                   # fused
    e = engs[1]                                           # reference: the two-step path
    e.t += 1
    lr_t = 1e-3 * math.sqrt(1.0 - 0.999 ** e.t) / (1.0 - 0.9 ** e.t)
    ops.adam_step_(e.w, e.g, e.m, e.v, lr_t, 0.9, 0.999, 1e-7, 0.5, e.w_lp)
    for i, wd in e.w_d.items():
        op = e.ops[i]
        ops.weight_flip_transpose_out(e._wv[i], op.k, op.cin, op.cout, wd)
    torch.cuda.synchronize()
    for a, b in ((engs[0].w, e.w), (engs[0].m, e.m), (engs[0].v, e.v)):
        assert torch.equal(a, b)
    if lowp is not None:
        assert torch.equal(engs[0].w_lp, e.w_lp)
    for i in e.w_d:
        assert torch.equal(engs[0].w_d[i], e.w_d[i]), i


# ----------------------------------------------------------------------------- facade
def _small_model(policy="float32"):
    from specenh.keras import layers, mixed_precision
    from specenh.keras.models import Model
    mixed_precision.set_global_policy(policy)
    try:
        inp = layers.Input(shape=(32, 32, 1))
        x = layers.Conv2D(8, 5, activation="relu", padding="same")(inp)
        x = layers.MaxPooling2D((2, 2), padding="same")(x)
        x = layers.Conv2D(16, 5, activation="relu", padding="same")(x)
        x = layers.MaxPooling2D((2, 2), padding="same")(x)
        x = layers.Conv2DTranspose(16, 5, strides=2, activation="relu", padding="same")(x)
        x = layers.Conv2DTranspose(8, 5, strides=2, activation="relu", padding="same")(x)
        x = layers.Conv2D(1, 5, activation="sigmoid", padding="same")(x)
        m = Model(inp, x)
    finally:
        mixed_precision.set_global_policy("float32")
    m.compile(optimizer="adam", loss="binary_crossentropy")
    return m


def _toy_data(n, seed=0):
    rng = np.random.default_rng(seed)
    clean = np.zeros((n, 32, 32, 1), np.float32)
    for i in range(n):
        r = rng.integers(4, 28)
        clean[i, r - 2:r + 2, :, 0] = 1.0
    noisy = np.clip(clean + 0.3 * rng.standard_normal(clean.shape), 0, 1).astype(np.float32)
    return noisy, clean


@pytest.mark.parametrize("policy", ["float32", "mixed_bfloat16"])
def test_fit_predict_evaluate_history(gpu_device, policy):
    from specenh.keras import callbacks, utils
    utils.set_random_seed(0)
    m = _small_model(policy)
    x, y = _toy_data(96)
    xv, yv = _toy_data(32, seed=1)
    es = callbacks.EarlyStopping(monitor="val_loss", mode="min", patience=50)
    hist = m.fit(x=x, y=y, epochs=6, batch_size=16, shuffle=True, validation_data=(xv, yv),
                 verbose=0, callbacks=[es])
    assert set(hist.history) == {"loss", "val_loss"}
    assert len(hist.history["val_loss"]) == 6
    assert hist.history["loss"][-1] < hist.history["loss"][0]
    assert all(np.isfinite(hist.history["val_loss"]))
    p = m.predict(xv)
    assert p.shape == (32, 32, 32, 1) and p.dtype == np.float32
    assert np.all((p >= 0) & (p <= 1))
    # predict is independent of batch composition (per-sample computation)
    np.testing.assert_array_equal(m.predict(xv[:5]), p[:5])
    ev = m.evaluate(xv, yv, batch_size=8)
    assert abs(ev - hist.history["val_loss"][-1]) <= 1e-6 * ev


def test_fit_loss_matches_oracle_fp32(gpu_device):
    """One epoch without shuffling: history['loss'] is the batch-weighted mean of the
    per-step losses of oracle.train_step on the same batches (last batch partial)."""
    from specenh.keras import utils
    utils.set_random_seed(0)
    m = _small_model()
    x, y = _toy_data(40)
    spec = oracle_spec(m._ops)
    ws = m.get_weights()
    tp, j = [], 0
    for s in spec:
        if s[0] == "pool":
            tp.append(None)
        else:
            tp.append({"W": torch.tensor(ws[j], dtype=torch.float64, requires_grad=True),
                       "b": torch.tensor(ws[j + 1], dtype=torch.float64, requires_grad=True)})
            j += 2
    opt = ora.KerasAdam()
    tot = 0.0
    for s in range(0, 40, 16):
        xb = torch.tensor(x[s:s + 16], dtype=torch.float64)
        yb = torch.tensor(y[s:s + 16], dtype=torch.float64)
        tot += ora.train_step(spec, tp, xb, yb, opt) * xb.shape[0]
    hist = m.fit(x, y, epochs=1, batch_size=16, shuffle=False, verbose=0)
    assert abs(hist.history["loss"][0] - tot / 40) <= 1e-5 * (tot / 40)


def test_save_load_predict_identical(gpu_device, tmp_path):
    from specenh.keras.models import load_model
    m = _small_model()
    x, y = _toy_data(32)
    m.fit(x, y, epochs=1, batch_size=16, verbose=0)
    m.save(str(tmp_path / "m"))
    m2 = load_model(str(tmp_path / "m"))
    np.testing.assert_array_equal(m2.predict(x), m.predict(x))
    # optimizer state travels: one more identical step on both
    m.fit(x, y, epochs=1, batch_size=32, shuffle=False, verbose=0)
    m2.fit(x, y, epochs=1, batch_size=32, shuffle=False, verbose=0)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)


def test_errors(gpu_device):
    m = _small_model()
    with pytest.raises(ValueError):
        m.predict(np.zeros((2, 32, 16, 1), np.float32))
    with pytest.raises(ValueError):
        m.fit(np.zeros((2, 32, 32, 1)), np.zeros((3, 32, 32, 1)))
    ae = _ae()
    with pytest.raises(RuntimeError, match="GPU only"):
        ae.AutoencoderEngine(m._ops, (32, 32, 1), device="cpu")
    from specenh import _lib
    L = _lib.lib()
    with pytest.raises(ValueError):
        _lib.check(L.specenh_maxpool2_fwd(0, None, 1, 3, 4, 1, None, None, None))
    with pytest.raises(ValueError):
        _lib.check(L.specenh_conv2d(0, None, 1, 4, 4, 1, None, 3, 3, 1, None, 1, 1, 1, 1, 4, 4,
                                    0, None, None, None, 1, 0, None, None))


def test_backward_is_bitwise_deterministic(gpu_device):
    ops = ref_model_ops()
    eng, _ = make(ops, (64, 64, 1), dtype="mixed_bfloat16", seed=31)
    rng = np.random.default_rng(9)
    x = upload(eng, rng.uniform(0, 1, (16, 64, 64, 1)))
    y = upload(eng, rng.uniform(0, 1, (16, 64, 64, 1)))
    grads = []
    for _ in range(2):
        eng.forward(x, train=True)
        eng.loss_and_grad(y)
        eng.backward()
        grads.append(eng.g.clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("dtype,hw,n", [("mixed_bfloat16", (128, 128), 128),
                                        ("float16", (64, 64), 16), ("float32", (32, 32), 4)])
def test_wgrad_side_stream_is_bitwise_serial(gpu_device, dtype, hw, n):
    """backward() enqueues every weight gradient on a second stream beside the input-
    gradient chain (default) or on the current stream (wgrad_overlap = False): after three
    train steps (forward, BCE, backward, Adam) the gradients, weights and Adam moments of
    both engines are bitwise equal, and the on_layer_done hook sees each layer once."""
    ops = ref_model_ops()
    rng = np.random.default_rng(17)
    xs = [rng.uniform(0, 1, (n, *hw, 1)) for _ in range(3)]
    ys = [rng.uniform(0, 1, (n, *hw, 1)) for _ in range(3)]
    state = []
    # (overlap, side streams, overwrite): the round-6 default (two side streams, overwriting
    # weight gradients), round 5's one accumulating side stream, and the serial orders
    for overlap, streams, ow in ((True, 2, True), (True, 3, True), (True, 1, False),
                                 (False, 1, True), (False, 1, False)):
        eng, _ = make(ops, (*hw, 1), dtype=dtype, seed=41)
        eng.wgrad_overlap = overlap
        eng.wgrad_streams = streams
        eng.wgrad_overwrite = ow
        seen = []
        for x, y in zip(xs, ys):
            eng.forward(upload(eng, x), train=True)
            eng.loss_and_grad(upload(eng, y))
            eng.backward(on_layer_done=seen.append)
            eng.adam()
        torch.cuda.synchronize()
        assert seen == [i for i in range(len(ops) - 1, -1, -1) if ops[i].__class__.__name__ == "ConvOp"] * 3
        state.append([t.clone() for t in (eng.g, eng.w, eng.m, eng.v)])
    for other in state[1:]:
        for a, b in zip(state[0], other):
            assert torch.equal(a, b)


def test_reference_model_fp16_relative(gpu_device):
    """C5 runs the autoencoder forward in fp16 (MFMA f16, fp32 accumulation): trained
    weights, C4-style inputs, out_rel / logit_rel within checks.TOL['float16']."""
    ops = ref_model_ops()
    eng, _ = make(ops, (128, 128, 1), dtype="float16")
    ws, x, _ = trained_c4(6)
    params = set_params(eng, ws)
    o, zr, zstd = lowp_errors(eng, params, x)
    print(f"fp16 out_rel {o:.2e} logit_rel {zr:.2e}")
    assert zstd > 1.0
    tol = checks.TOL["float16"]
    assert o <= tol["out_rel"] and zr <= tol["logit_rel"], (o, zr)


def _gain_scaled(ops, seed):
    """Glorot kernels with a relu gain (He-like variance) and random biases: outputs of an
    untrained variant that still span the sigmoid (logit std > 0.5)."""
    params = ora.glorot_params(oracle_spec(ops), seed=seed)
    rng = np.random.default_rng(seed + 1)
    ws = []
    for op, p in zip(ops, params):
        if p is None:
            continue
        k = op.k
        fan_in = k * k * (op.cin if op.kind == "conv" else op.cin)
        fan_out = k * k * op.cout
        g = math.sqrt(2.0 * (fan_in + fan_out) / (2.0 * fan_in)) * (1.6 if op.kind == "convT" else 1.0)
        if op.act == "sigmoid":
            g *= 6.0
        ws += [(p["W"] * g).astype(np.float32),
               (0.1 * rng.standard_normal(op.cout)).astype(np.float32)]
    return ws


def variant_ops(name):
    """The reference's other autoencoders (all layers padding='same', MaxPool 2x2)."""
    ae = _ae()
    C, P = ae.ConvOp, ae.PoolOp
    if name == "3layer_256x128":     # manual_scan_3layers.py:186-199, its real input shape
        return ref_model_ops(), (256, 128, 1)
    if name == "2layer_64_32_k5":    # manual_scan.py:120-124, 190-199
        return [C("conv", 1, 64, 5, "relu"), P(), C("conv", 64, 32, 5, "relu"), P(),
                C("convT", 32, 32, 5, "relu", stride=2), C("convT", 32, 64, 5, "relu", stride=2),
                C("conv", 64, 1, 5, "sigmoid")], (256, 128, 1)
    k = {"2layer_32_k7": 7, "2layer_32_k3": 3}[name]  # hyperparam_scan.py:123,153-162;
    return [C("conv", 1, 32, k, "relu"), P(), C("conv", 32, 32, k, "relu"), P(),  # graphs.ipynb
            C("convT", 32, 32, k, "relu", stride=2), C("convT", 32, 32, k, "relu", stride=2),
            C("conv", 32, 1, k, "sigmoid")], (256, 128, 1)


@pytest.mark.parametrize("dtype", ["float32", "float16", "mixed_bfloat16"])
@pytest.mark.parametrize("name", ["3layer_256x128", "2layer_64_32_k5", "2layer_32_k7",
                                  "2layer_32_k3"])
def test_reference_variants(gpu_device, name, dtype):
    """Every autoencoder the reference builds, at its (256, 128, 1) input: fp32 within
    1e-5 (max-norm), fp16/bf16 within checks.TOL, vs the fp64 oracle."""
    ops, hwc = variant_ops(name)
    eng, _ = make(ops, hwc, dtype=dtype)
    params = set_params(eng, _gain_scaled(ops, seed=len(name)))
    x = np.random.default_rng(14).uniform(0, 1, (3,) + hwc).astype(np.float32)
    if dtype == "float32":
        ref, _ = ref_forward(ops, params, x)
        got = eng.forward(upload(eng, x), train=False).cpu().numpy()
        assert np.abs(got - ref).max() / np.abs(ref).max() <= TOL_OUT
        return
    o, zr, zstd = lowp_errors(eng, params, x)
    print(f"{name} {dtype}: out_rel {o:.2e} logit_rel {zr:.2e} (logit std {zstd:.2f})")
    assert zstd > 0.5
    tol = checks.TOL[dtype]
    assert o <= tol["out_rel"] and zr <= tol["logit_rel"], (o, zr)


@pytest.mark.parametrize("dtype", ["mixed_bfloat16", "float16"])
@pytest.mark.parametrize("model", ["3layer", "2layer_32_k7"])
def test_fused_conv_pool_is_bitwise_identical_to_unfused(gpu_device, dtype, model):
    """Conv2D + MaxPooling2D in one launch (pool taken in the conv's registers) gives the
    same forward output and the same gradients as the two launches; 2layer_32_k7: the 7 x 7
    convolutions (C = 1 on conv_c1_mfma, 32 channels on the patch kernel; round 5, k <= 5
    before) fused with their pools."""
    if model == "3layer":
        ops, hwc, want = ref_model_ops(), (64, 64, 1), {0, 2, 4}
    else:
        ops, _ = variant_ops(model)
        hwc, want = (64, 48, 1), {0, 2}
    fused, _ = make(ops, hwc, dtype=dtype, seed=41)
    plain, _ = make(ops, hwc, dtype=dtype, seed=41)
    assert fused.fused == want
    plain.fused = set()
    rng = np.random.default_rng(11)
    x = rng.uniform(0, 1, (6,) + hwc).astype(np.float32)
    y = rng.uniform(0, 1, (6,) + hwc).astype(np.float32)
    outs, grads = [], []
    for eng in (fused, plain):
        outs.append(eng.forward(upload(eng, x)).clone())
        eng.forward(upload(eng, x), train=True)
        eng.loss_and_grad(upload(eng, y))
        eng.backward()
        grads.append(eng.g.clone())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("dtype", ["mixed_bfloat16", "float16"])
@pytest.mark.parametrize("hwc,n", [((128, 128, 1), 6), ((256, 128, 1), 3), ((128, 128, 1), 130)])
def test_training_tail_matches_two_launches(gpu_device, dtype, hwc, n):
    """forward(train=True) runs Conv2DTranspose(16) + Conv2D(1) as ONE row-sweep launch that
    also stores the 16-channel map, the fp32 logits and the sigmoid output (round 5,
    decoder_tail.hip tail_rows_kernel<T, true>). Against the two launches (conv_patch +
    conv_co1): the same products in another fp32 order, so the map is equal up to one
    rounding step of T in a few elements, the logits agree to 1e-3 of their spread, the output
    is the sigmoid of the logits rounded to T, and the gradients agree to 1e-2 (cosine 0.9999).
    n = 130: bands of one image on several workgroups AND a partial last wave."""
    ops = ref_model_ops()
    fused, _ = make(ops, hwc, dtype=dtype, seed=43)
    plain, _ = make(ops, hwc, dtype=dtype, seed=43)
    assert fused.tail_train
    plain.tail_train = False
    ws, _, _ = trained_c4(1)
    set_params(fused, ws)
    set_params(plain, ws)
    rng = np.random.default_rng(12)
    x = rng.uniform(0, 1, (n,) + hwc).astype(np.float32)
    y = rng.uniform(0, 1, (n,) + hwc).astype(np.float32)
    res = []
    for eng in (fused, plain):
        out = eng.forward(upload(eng, x), train=True)
        b = eng._buffers(n, True)
        mp = b["h"][len(ops) - 1].float()
        z = eng.last_logits().clone()
        eng.loss_and_grad(upload(eng, y))
        eng.backward()
        res.append((mp, z, out.float().clone(), eng.g.clone()))
    (m0, z0, o0, g0), (m1, z1, o1, g1) = res
    ulp = 2.0 ** (-7 if dtype == "mixed_bfloat16" else -10)
    dm = (m0 - m1).abs()
    assert float((dm > 0).float().mean()) < 0.01
    # one rounding step of T, or (sums that cancel to near zero, where the fp32 order
    # matters more than T's step) 1e-4 of the map's range
    bound = ulp * m1.abs() * 1.01 + 1e-4 * float(m1.abs().max())
    j = int(torch.argmax(dm - bound))
    print(f"map max diff {float(dm.max()):.3e} at worst {float(m0.flatten()[j]):.5e} vs "
          f"{float(m1.flatten()[j]):.5e} (range {float(m1.abs().max()):.3e})")
    assert bool((dm <= bound).all())
    spread = float(z1.max() - z1.min())
    assert spread > 1.0
    print(f"map diff frac {float((dm > 0).float().mean()):.2e}, logit diff / spread "
          f"{float((z0 - z1).abs().max()) / spread:.2e}")
    assert float((z0 - z1).abs().max()) <= 1e-3 * spread
    sig = torch.sigmoid(z0.double())
    assert float((o0.double().reshape(sig.shape) - sig).abs().max()) <= 2 * ulp
    cos = float(torch.dot(g0, g1) / (g0.norm() * g1.norm()))
    assert cos >= 0.9999
    assert float((g0 - g1).norm() / g1.norm()) <= 1e-2


@pytest.mark.parametrize("dtype", ["mixed_bfloat16", "float16"])
@pytest.mark.parametrize("hw", [(128, 128), (40, 56), (24, 8)])
def test_convt_row_phase_pairs_bitwise_identical(gpu_device, dtype, hw, kernel_variant):
    """Conv2DTranspose forward in (tile, row-phase) workgroups with LDS-staged whole-row
    stores (opt-in: SPECENH_CONVT_PAIR=1, measured slower) gives the same
    bits as the four-phase workgroups with per-phase stores, at
    tile-aligned and ragged sizes, in inference and in training (which keeps the
    per-phase path only where it needs the pre-activation)."""
    ops = ref_model_ops()
    H, W = hw
    eng, _ = make(ops, (H, W, 1), dtype=dtype, seed=43)
    rng = np.random.default_rng(12)
    x = rng.uniform(0, 1, (5, H, W, 1)).astype(np.float32)
    y = rng.uniform(0, 1, (5, H, W, 1)).astype(np.float32)
    outs, grads = [], []
    for flag in ("1", "0"):
        kernel_variant("CONVT_PAIR", int(flag))
        outs.append(eng.forward(upload(eng, x), train=False).clone())
        eng.forward(upload(eng, x), train=True)
        eng.loss_and_grad(upload(eng, y))
        eng.backward()
        grads.append(eng.g.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("switch", [("SPECENH_PATCH_WSPLIT", "1", "0"),
                                    ("SPECENH_PATCH_NO_WL", "0", "1")])
@pytest.mark.parametrize("dtype", ["mixed_bfloat16", "float16"])
def test_wave_split_patch_kernel_is_bitwise_identical(gpu_device, dtype, switch, kernel_variant):
    """conv_patch_kernel's variants run the same k-step order per output: the 2 x 2 wave
    split (8 rows x half the channels per wave, the default for 32/64-channel chunks) vs the
    4 x 1 split, and the 16-channel kernel's LDS-resident weights vs the register ring fed
    from L2. Forward outputs and gradients are bitwise equal, each variant forced on and off."""
    env, on, off = switch
    ops = ref_model_ops()
    rng = np.random.default_rng(13)
    x = rng.uniform(0, 1, (4, 64, 64, 1)).astype(np.float32)
    y = rng.uniform(0, 1, (4, 64, 64, 1)).astype(np.float32)
    outs, grads = [], []
    for flag in (on, off):
        # a fresh engine whose every activation buffer starts as NaN: an output element a
        # variant fails to write cannot inherit the other variant's value
        eng, _ = make(ops, (64, 64, 1), dtype=dtype, seed=47)
        kernel_variant(env, int(flag))
        poison(eng, 4, False)
        outs.append(eng.forward(upload(eng, x), train=False).clone())
        poison(eng, 4, True)
        eng.forward(upload(eng, x), train=True)
        eng.loss_and_grad(upload(eng, y))
        eng.backward()
        grads.append(eng.g.clone())
    torch.cuda.synchronize()
    assert bool(torch.isfinite(outs[0]).all())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(grads[0], grads[1])


def poison(eng, N, train):
    """Fill every cached activation / gradient buffer of the engine for batch N with NaN
    (0xFF for argmax bytes), so unwritten output elements show up in comparisons."""
    b = eng._buffers(N, train)
    for key in ("h", "d"):
        for i, t in enumerate(b[key]):
            if t is not None and i > 0:
                t.fill_(float("nan"))
    for t in b["am"]:
        if t is not None:
            t.fill_(255)


@pytest.mark.parametrize("dtype", ["mixed_bfloat16", "float16"])
def test_c5_shape_layers_at_large_batch(gpu_device, dtype):
    """Near the launch shapes of the C5 bench (256 shots, 128 x 128): at this batch every layer
    takes its large-grid variant (wave split, persistent C = 1 and tail kernels), which small
    parity cases never select. Every intermediate (poisoned with NaN beforehand) vs a torch
    fp32 layer applied to the same low-precision input: relative error within the
    compute dtype's rounding."""
    ops = ref_model_ops()
    N = 256
    eng, params = make(ops, (128, 128, 1), dtype=dtype, seed=53)
    rng = np.random.default_rng(14)
    x = upload(eng, rng.uniform(0, 1, (N, 128, 128, 1)).astype(np.float32))
    poison(eng, N, False)
    out = eng.forward(x, train=False)
    torch.cuda.synchronize()
    b = eng._buffers(N, False)
    ws = [p for p in params if p is not None]
    tol = 4e-3 if eng.tdt == torch.bfloat16 else 1e-3
    torch.backends.cudnn.allow_tf32 = False
    h, j, i = x, 0, 0
    while i < len(ops):
        op = ops[i]
        # the engine's low-precision weights, fp32 biases
        w = torch.as_tensor(ws[j]["W"], device=gpu_device).to(eng.tdt).float()
        bias = torch.as_tensor(ws[j]["b"], device=gpu_device).float()
        with torch.no_grad():
            r = (ora.conv2d_same if op.kind == "conv" else ora.conv2d_transpose_same)(
                h.float(), w, bias)
            r = torch.sigmoid(r) if op.act == "sigmoid" else torch.relu(r)
            pool = i + 1 < len(ops) and isinstance(ops[i + 1], type(ops[1]))
            if pool:
                r = ora.maxpool2(r)
        got = b["h"][i + (2 if pool else 1)]
        if got is None:  # a fused map (encoder2 / the decoder tail) never reaches memory:
            h = r.to(eng.tdt).contiguous()  # compare at the fused launch's output
            i += 2 if pool else 1
            j += 1
            continue
        got = got.float()
        assert bool(torch.isfinite(got).all()), f"layer {i}: unwritten / non-finite elements"
        err = float((got - r).norm() / r.norm())
        assert err <= tol, f"layer {i} ({op.kind} {op.cin}->{op.cout}): rel {err:.2e}"
        h = got.to(eng.tdt) if got.dtype != eng.tdt else b["h"][i + (2 if pool else 1)]
        i += 2 if pool else 1
        j += 1
    assert out is b["h"][len(ops)]
