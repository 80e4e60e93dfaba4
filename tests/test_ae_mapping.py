"""CPU checks of the conv-autoencoder lowering (no GPU).

The HIP kernel computes out[m][co] = sum_k A[m][k] Bf[k][co] with A gathered by the
index formula documented in include/specenh.h (specenh_conv2d). Here that formula is
evaluated in numpy (an im2col written from the header, not from the kernel) and, with
the engine's weight mappings (specenh.ae.keras_to_gemm, the flip/transpose of
specenh_weight_flip_transpose, ConvOp.fwd_geom / dgrad_geom), compared with the
oracle's Keras-semantics conv / conv-transpose and their autograd gradients. It pins
every geometry the GPU path uses before any kernel runs.
"""
import numpy as np
import pytest
import torch

from oracle import autoencoder as ora
from specenh import ae
from specenh.keras import layers, mixed_precision
from specenh.keras.models import Model, load_model


def igemm(x, bt, k, OH, OW, geom):
    """numpy restatement of the specenh_conv2d gather (include/specenh.h)."""
    stride, pt, pl, dil = geom
    N, IH, IW, C = x.shape
    A = np.zeros((N, OH, OW, k, k, C), dtype=np.float64)
    oy = np.arange(OH)[:, None]
    ox = np.arange(OW)[None, :]
    for ky in range(k):
        vy = oy * stride - pt + ky
        okx = (vy >= 0) & (vy % dil == 0) & (vy // dil < IH)
        iy = np.clip(vy // dil, 0, IH - 1)
        for kx in range(k):
            vx = ox * stride - pl + kx
            oky = (vx >= 0) & (vx % dil == 0) & (vx // dil < IW)
            ix = np.clip(vx // dil, 0, IW - 1)
            ok = (okx & oky)[None, :, :, None]
            A[:, :, :, ky, kx, :] = np.where(ok, x[:, iy, ix, :], 0.0)
    A = A.reshape(N * OH * OW, -1)
    return A, (A @ bt.T).reshape(N, OH, OW, -1)


def flip_transpose(bt_flat, k, ci, co):
    """specenh_weight_flip_transpose: bd[ci][a][b][co] = bt[co][k-1-a][k-1-b][ci]."""
    bt = bt_flat.reshape(co, k, k, ci)
    return np.ascontiguousarray(bt[:, ::-1, ::-1, :].transpose(3, 1, 2, 0)).reshape(ci, k * k * co)


CASES = [("conv", 1, 16, 5, 12, 10), ("conv", 16, 8, 3, 9, 7), ("conv", 8, 1, 5, 8, 8),
         ("convT", 64, 32, 5, 6, 4), ("convT", 3, 5, 3, 5, 7), ("convT", 4, 4, 4, 3, 3)]


@pytest.mark.parametrize("kind,cin,cout,k,H,W", CASES)
def test_forward_dgrad_wgrad_lowering(kind, cin, cout, k, H, W):
    rng = np.random.default_rng(hash((kind, cin, cout, k)) % 2**32)
    op = ae.ConvOp(kind, cin, cout, k, "relu", stride=2 if kind == "convT" else 1)
    shape = (k, k, cin, cout) if kind == "conv" else (k, k, cout, cin)
    Wk = rng.standard_normal(shape)
    x = rng.standard_normal((2, H, W, cin))
    xt = torch.tensor(x, requires_grad=True)
    Wt = torch.tensor(Wk, requires_grad=True)
    b = torch.zeros(cout, dtype=torch.float64)
    f = ora.conv2d_same if kind == "conv" else ora.conv2d_transpose_same
    ref = f(xt, Wt, b)
    OH, OW = op.out_hw(H, W)
    assert ref.shape == (2, OH, OW, cout)

    bt = ae.keras_to_gemm(op, Wk.astype(np.float32)).astype(np.float64)
    # keras_to_gemm casts to fp32: compare against the fp32-rounded kernel
    Wt32 = torch.tensor(Wk.astype(np.float32).astype(np.float64), requires_grad=True)
    ref = f(xt, Wt32, b)
    A, out = igemm(x, bt.reshape(cout, -1), k, OH, OW, op.fwd_geom())
    np.testing.assert_allclose(out, ref.detach().numpy(), rtol=1e-12, atol=1e-12)

    # backward: dX via the dgrad conv, dW via A^T dZ
    dz = rng.standard_normal(ref.shape)
    ref.backward(torch.tensor(dz))
    bd = flip_transpose(bt, k, cin, cout)
    _, dx = igemm(dz, bd, k, H, W, op.dgrad_geom())
    np.testing.assert_allclose(dx, xt.grad.numpy(), rtol=1e-11, atol=1e-11)
    dbt = dz.reshape(-1, cout).T @ A  # [co][k], the specenh_conv2d_wgrad layout
    bt4 = dbt.reshape(cout, k, k, cin)
    dW = bt4.transpose(1, 2, 3, 0) if kind == "conv" else bt4[:, ::-1, ::-1, :].transpose(1, 2, 0, 3)
    np.testing.assert_allclose(dW, Wt32.grad.numpy(), rtol=1e-11, atol=1e-11)


def test_gemm_layout_round_trip():
    rng = np.random.default_rng(3)
    for kind in ("conv", "convT"):
        op = ae.ConvOp(kind, 6, 10, 5, "relu", stride=2)
        shape = (5, 5, 6, 10) if kind == "conv" else (5, 5, 10, 6)
        Wk = rng.standard_normal(shape).astype(np.float32)
        np.testing.assert_array_equal(ae.gemm_to_keras(op, ae.keras_to_gemm(op, Wk)), Wk)


def build_reference_model(h=256, w=128, c1=16, c2=32, c3=64, k=5):
    """manual_scan_3layers.py:186-199 through the facade."""
    inp = layers.Input(shape=(h, w, 1))
    x = layers.Conv2D(c1, k, activation="relu", padding="same")(inp)
    x = layers.MaxPooling2D((2, 2), padding="same")(x)
    x = layers.Conv2D(c2, k, activation="relu", padding="same")(x)
    x = layers.MaxPooling2D((2, 2), padding="same")(x)
    x = layers.Conv2D(c3, k, activation="relu", padding="same")(x)
    x = layers.MaxPooling2D((2, 2), padding="same")(x)
    x = layers.Conv2DTranspose(c3, k, strides=2, activation="relu", padding="same")(x)
    x = layers.Conv2DTranspose(c2, k, strides=2, activation="relu", padding="same")(x)
    x = layers.Conv2DTranspose(c1, k, strides=2, activation="relu", padding="same")(x)
    x = layers.Conv2D(1, k, activation="sigmoid", padding="same")(x)
    return Model(inp, x)


def test_facade_matches_reference_architecture(capsys):
    m = build_reference_model()
    m.compile(optimizer="adam", loss="binary_crossentropy")
    assert m.count_params() == 231_425
    assert m.output_shape == (None, 256, 128, 1)
    m.summary()
    out = capsys.readouterr().out
    assert "Total params: 231,425" in out
    # the layer chain lowers to the oracle's spec
    spec = ora.ae_spec()
    ops = m._ops
    assert len(ops) == len(spec)
    for op, s in zip(ops, spec):
        if s[0] == "pool":
            assert isinstance(op, ae.PoolOp)
        else:
            assert (op.kind, op.cin, op.cout, op.k, op.act) == s
    # Keras-shaped weights with glorot limits
    ws = m.get_weights()
    assert ws[0].shape == (5, 5, 1, 16) and ws[6].shape == (5, 5, 64, 64)
    lim = np.sqrt(6.0 / (25 * 1 + 25 * 16))
    assert np.abs(ws[0]).max() <= lim and np.all(ws[1] == 0)


def test_facade_errors():
    inp = layers.Input(shape=(32, 32, 1))
    with pytest.raises(NotImplementedError):
        layers.Conv2D(4, 3, activation="tanh", padding="same")
    with pytest.raises(NotImplementedError):
        layers.MaxPooling2D((3, 3))
    x = layers.Conv2D(4, 3, activation="relu", padding="same")(inp)
    m = Model(inp, x)
    with pytest.raises(NotImplementedError, match="sigmoid"):
        m.compile(optimizer="adam", loss="binary_crossentropy")
    y = layers.Conv2D(1, 3, activation="sigmoid", padding="same")(x)
    m = Model(inp, y)
    with pytest.raises(NotImplementedError):
        m.compile(optimizer="adam", loss="mse")
    with pytest.raises(NotImplementedError):
        m.compile(optimizer="sgd", loss="binary_crossentropy")
    with pytest.raises(RuntimeError, match="compile"):
        m.fit(np.zeros((2, 32, 32, 1)), np.zeros((2, 32, 32, 1)))
    with pytest.raises(ValueError):
        mixed_precision.set_global_policy("float64")


def test_save_load_round_trip_on_host(tmp_path):
    m = build_reference_model(64, 32, 4, 8, 8, 3)
    m.compile(optimizer="adam", loss="binary_crossentropy")
    m.save(str(tmp_path / "model"))
    m2 = load_model(str(tmp_path / "model"))
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    assert [type(l).__name__ for l in m2.layers] == [type(l).__name__ for l in m.layers]
    assert m2.count_params() == m.count_params()
