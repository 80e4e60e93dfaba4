"""The fused decoder tail (csrc/decoder_tail.hip: Conv2DTranspose(16, 5, strides=2, relu) +
Conv2D(1, 5, sigmoid) in one launch, the 16-channel map kept in LDS) against the two-launch
path and the fp64 oracle: same map rounding, so the outputs agree to fp32 accumulation-order
differences (the map may differ by one fp16 ulp where the two MFMA orders round apart)."""
import numpy as np
import pytest
import torch

from oracle import autoencoder as ora
from oracle import checks

pytestmark = pytest.mark.gpu


def _tail_model(dtype, hw, seed):
    from specenh import ae
    C = ae.ConvOp
    ops_ = [C("conv", 1, 32, 3, "relu"), C("convT", 32, 16, 5, "relu", stride=2),
            C("conv", 16, 1, 5, "sigmoid")]
    eng = ae.AutoencoderEngine(ops_, hw + (1,), compute_dtype=dtype, device="cuda")
    rng = np.random.default_rng(seed)
    ws = [(0.5 * rng.standard_normal((3, 3, 1, 32))).astype(np.float32),
          (0.1 * rng.standard_normal(32)).astype(np.float32),
          (0.08 * rng.standard_normal((5, 5, 16, 32))).astype(np.float32),
          (0.1 * rng.standard_normal(16)).astype(np.float32),
          (0.25 * rng.standard_normal((5, 5, 16, 1))).astype(np.float32),
          (0.1 * rng.standard_normal(1)).astype(np.float32)]
    eng.set_keras_weights(ws)
    return eng, ops_, ws


@pytest.mark.parametrize("dtype", ["float16", "mixed_bfloat16"])
@pytest.mark.parametrize("hw", [(64, 64), (20, 28), (9, 33), (1, 1)])
def test_fused_tail_matches_two_launches_and_oracle(gpu_device, dtype, hw, monkeypatch):
    eng, ops_, ws = _tail_model(dtype, hw, seed=hw[0] * 7 + hw[1])
    assert eng.tail
    x = np.random.default_rng(1).uniform(0, 1, (5,) + hw + (1,)).astype(np.float32)
    xd = eng.to_compute(torch.from_numpy(x))
    fused = eng.forward(xd).clone()
    monkeypatch.setenv("SPECENH_NO_TAIL_FUSION", "1")
    from specenh import ae
    plain_eng = ae.AutoencoderEngine(ops_, hw + (1,), compute_dtype=dtype, device="cuda")
    assert not plain_eng.tail
    plain_eng.set_keras_weights(ws)
    plain = plain_eng.forward(xd).clone()
    torch.cuda.synchronize()
    assert fused.shape == plain.shape == (5, 2 * hw[0], 2 * hw[1], 1)
    d = (fused - plain).abs().max().item()
    assert d <= 2e-3, d
    spec = [("conv", 1, 32, 3, "relu"), ("convT", 32, 16, 5, "relu"),
            ("conv", 16, 1, 5, "sigmoid")]
    it = iter(ws)
    params = [{"W": torch.tensor(next(it), dtype=torch.float64),
               "b": torch.tensor(next(it), dtype=torch.float64)} for _ in spec]
    with torch.no_grad():
        ref = ora.forward(spec, params, torch.tensor(x, dtype=torch.float64)).numpy()
    err = checks.out_rel(fused.cpu().numpy(), ref)
    assert err <= checks.TOL[dtype]["out_rel"], err


@pytest.mark.parametrize("dtype", ["float16", "mixed_bfloat16"])
@pytest.mark.parametrize("hw,n", [((64, 64), 5), ((64, 64), 600), ((8, 64), 3), ((13, 64), 4),
                                  ((128, 64), 2)])
def test_row_sweep_tail_matches_tile_kernel(gpu_device, dtype, hw, n, kernel_variant):
    """tail_rows_kernel (64-position-wide inputs: the model's 128-wide outputs) vs the 2-D
    tile kernel (TAIL_TILES=1) and the fp64 oracle, with the output buffer NaN-poisoned
    before each launch (an unwritten pixel fails). Batches of 5 / 3 / 4 / 2 images run in
    8 / 2 / ... bands per image (recomputed halo position rows at band edges), 600 images
    in one band; 8 and 13 position rows exercise short and odd heights, 128 rows the
    reference's 256 x 128 input."""
    eng, ops_, ws = _tail_model(dtype, hw, seed=hw[0] * 11 + n)
    x = np.random.default_rng(n).uniform(0, 1, (n,) + hw + (1,)).astype(np.float32)
    xd = eng.to_compute(torch.from_numpy(x))
    outs = []
    for tiles in (0, 1):
        kernel_variant("TAIL_TILES", tiles)
        eng.forward(xd)  # allocate, then poison the output and run again
        eng._buffers(n, False)["h"][len(ops_)].fill_(float("nan"))
        outs.append(eng.forward(xd).clone())
    torch.cuda.synchronize()
    rows_out, tile_out = outs
    assert not torch.isnan(rows_out).any()
    d = (rows_out - tile_out).abs().max().item()
    assert d <= 2e-3, d
    if n <= 5:
        spec = [("conv", 1, 32, 3, "relu"), ("convT", 32, 16, 5, "relu"),
                ("conv", 16, 1, 5, "sigmoid")]
        it = iter(ws)
        params = [{"W": torch.tensor(next(it), dtype=torch.float64),
                   "b": torch.tensor(next(it), dtype=torch.float64)} for _ in spec]
        with torch.no_grad():
            ref = ora.forward(spec, params, torch.tensor(x, dtype=torch.float64)).numpy()
        err = checks.out_rel(rows_out.cpu().numpy(), ref)
        assert err <= checks.TOL[dtype]["out_rel"], err


def _dec3_model(dtype, hw, seed):
    from specenh import ae
    C = ae.ConvOp
    ops_ = [C("conv", 1, 64, 3, "relu"), C("convT", 64, 32, 5, "relu", stride=2),
            C("convT", 32, 16, 5, "relu", stride=2), C("conv", 16, 1, 5, "sigmoid")]
    rng = np.random.default_rng(seed)
    ws = [(0.5 * rng.standard_normal((3, 3, 1, 64))).astype(np.float32),
          (0.1 * rng.standard_normal(64)).astype(np.float32),
          (0.05 * rng.standard_normal((5, 5, 32, 64))).astype(np.float32),
          (0.1 * rng.standard_normal(32)).astype(np.float32),
          (0.08 * rng.standard_normal((5, 5, 16, 32))).astype(np.float32),
          (0.1 * rng.standard_normal(16)).astype(np.float32),
          (0.25 * rng.standard_normal((5, 5, 16, 1))).astype(np.float32),
          (0.1 * rng.standard_normal(1)).astype(np.float32)]
    eng = ae.AutoencoderEngine(ops_, hw + (1,), compute_dtype=dtype, device="cuda")
    eng.set_keras_weights(ws)
    return eng, ops_, ws


@pytest.mark.parametrize("dtype", ["float16", "mixed_bfloat16"])
@pytest.mark.parametrize("hw,n", [((32, 32), 3), ((8, 32), 2), ((5, 32), 1), ((64, 32), 2),
                                  ((1, 32), 2), ((32, 32), 600), ((3, 32), 1000)])
@pytest.mark.parametrize("d3map", [0, 1])
def test_decoder3_matches_unfused_and_oracle(gpu_device, dtype, hw, n, d3map, kernel_variant):
    """decoder3_kernel (Conv2DTranspose(32) + Conv2DTranspose(16) + Conv2D(1), both maps in
    LDS) vs the same engine with the decoder unfused (DECODER_UNFUSED=1: convT2 through
    conv_patch + the row-sweep tail) and the fp64 oracle; output NaN-poisoned first. The
    32-channel map is rounded to T in both paths after its ReLU, so they differ only by
    accumulation order (and the fp16 roundings that follow from it). n > 256: several images
    per persistent workgroup (the row stream's image-to-image hand-over). d3map = 1: the
    round-3 consumer (16-channel map ring in LDS) instead of the map-free Conv2D(1)."""
    kernel_variant("D3_MAP", d3map)
    eng, ops_, ws = _dec3_model(dtype, hw, seed=hw[0] * 13 + n)
    assert eng.dec3
    x = np.random.default_rng(n + 5).uniform(0, 1, (n,) + hw + (1,)).astype(np.float32)
    xd = eng.to_compute(torch.from_numpy(x))
    eng.forward(xd)
    eng._buffers(n, False)["h"][len(ops_)].fill_(float("nan"))
    fused = eng.forward(xd).clone()
    kernel_variant("DECODER_UNFUSED", 1)
    from specenh import ae
    plain_eng = ae.AutoencoderEngine(ops_, hw + (1,), compute_dtype=dtype, device="cuda")
    assert not plain_eng.dec3 and plain_eng.tail
    plain_eng.set_keras_weights(ws)
    plain = plain_eng.forward(xd).clone()
    torch.cuda.synchronize()
    assert fused.shape == plain.shape == (n, 4 * hw[0], 4 * hw[1], 1)
    assert not torch.isnan(fused).any()
    d = (fused - plain).abs().max().item()
    assert d <= 4e-3, d
    spec = [(o.kind, o.cin, o.cout, o.k, o.act) for o in ops_]
    it = iter(ws)
    params = [{"W": torch.tensor(next(it), dtype=torch.float64),
               "b": torch.tensor(next(it), dtype=torch.float64)} for _ in spec]
    # the fp64 oracle on images that fall into different workgroups and stream positions
    idx = sorted({i for i in (0, 1, 255, 256, 257, 511, 512, n - 1) if i < n})
    with torch.no_grad():
        ref = ora.forward(spec, params, torch.tensor(x[idx], dtype=torch.float64)).numpy()
    err = checks.out_rel(fused.cpu().numpy()[idx], ref)
    assert err <= checks.TOL[dtype]["out_rel"], err


@pytest.mark.parametrize("hw,n", [((32, 32), 3), ((32, 32), 600), ((3, 32), 1000)])
def test_decoder3_lead_bitwise(gpu_device, hw, n, kernel_variant):
    """decoder3's producer with three input-ring refills in flight (default) vs the round-3
    wait for the refill issued in the same macro step: only the waits differ."""
    from specenh import _lib
    eng, ops_, ws = _dec3_model("float16", hw, seed=n + 3)
    x = np.random.default_rng(n + 9).uniform(0, 1, (n,) + hw + (1,)).astype(np.float32)
    xd = eng.to_compute(torch.from_numpy(x))
    a = eng.forward(xd).clone()
    kernel_variant("ROWS_SHORT_LEAD", 1)
    eng._buffers(n, False)["h"][len(ops_)].fill_(float("nan"))
    b = eng.forward(xd).clone()
    torch.cuda.synchronize()
    assert "decoder3_kernel" in _lib.last_kernel_name()
    assert not torch.isnan(a).any()
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", ["float16", "mixed_bfloat16"])
@pytest.mark.parametrize("hw,n", [((32, 32), 3), ((32, 32), 600), ((3, 32), 1000)])
def test_decoder3_fp16_output(gpu_device, dtype, hw, n):
    """set_inference_output_dtype(float16) (BASELINE config 5's fp16 reconstructions): the same
    launch stores each sigmoid output rounded once to fp16, i.e. exactly the fp32 output cast
    to fp16 (round to nearest even); the fp16 buffer is NaN-poisoned first."""
    from specenh import _lib
    eng, ops_, ws = _dec3_model(dtype, hw, seed=n + 21)
    x = np.random.default_rng(n + 2).uniform(0, 1, (n,) + hw + (1,)).astype(np.float32)
    xd = eng.to_compute(torch.from_numpy(x))
    y32 = eng.forward(xd).clone()
    eng.set_inference_output_dtype(torch.float16)
    eng.forward(xd)
    out = eng._buffers(n, False)["h"][len(ops_)]
    assert out.dtype == torch.float16
    out.fill_(float("nan"))
    y16 = eng.forward(xd).clone()
    torch.cuda.synchronize()
    assert "decoder3_kernel" in _lib.last_kernel_name()
    assert y16.dtype == torch.float16 and y16.shape == y32.shape
    assert torch.equal(y16, y32.to(torch.float16))
    eng.set_inference_output_dtype(torch.float32)
    assert torch.equal(eng.forward(xd), y32)


def test_fp16_output_needs_the_fused_decoder(gpu_device, kernel_variant):
    kernel_variant("DECODER_UNFUSED", 1)
    eng, _, _ = _dec3_model("float16", (8, 32), seed=1)
    assert not eng.dec3
    with pytest.raises(NotImplementedError, match="fused three-layer decoder"):
        eng.set_inference_output_dtype(torch.float16)
