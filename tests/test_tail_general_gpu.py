"""The general row-sweep decoder tail (csrc/tail_rows_g.hip): Conv2DTranspose(32, k, s2, relu) +
Conv2D(1, k, sigmoid) in one launch on 64-position-wide 32-channel inputs, k = 3 / 5 / 7 —
the last two layers of the 32/32 models of VAE/hyperparam_scan.py:153-162 at their 256 x 128
input. Against the two-launch path (SPECENH_NO_TAIL_FUSION) with the output NaN-poisoned
before the fused launch, and against the fp64 oracle. The map is rounded to the compute dtype
after the ReLU as the two-launch path stores it; only the fp32 summation order differs, so the
outputs agree to 2e-3 (the sigmoid's output scale) and the oracle bound is checks.TOL."""
import numpy as np
import pytest
import torch

from oracle import autoencoder as ora
from oracle import checks

pytestmark = pytest.mark.gpu


def _model(dtype, hw, k, seed, co=32):
    from specenh import ae
    C = ae.ConvOp
    ops_ = [C("conv", 1, 32, 3, "relu"), C("convT", 32, co, k, "relu", stride=2),
            C("conv", co, 1, k, "sigmoid")]
    rng = np.random.default_rng(seed)
    g = 5.0 / k
    ws = [(0.5 * rng.standard_normal((3, 3, 1, 32))).astype(np.float32),
          (0.1 * rng.standard_normal(32)).astype(np.float32),
          (0.06 * g * rng.standard_normal((k, k, co, 32))).astype(np.float32),
          (0.1 * rng.standard_normal(co)).astype(np.float32),
          (0.18 * g * (32 / co) ** 0.5 * rng.standard_normal((k, k, co, 1))).astype(np.float32),
          (0.1 * rng.standard_normal(1)).astype(np.float32)]
    eng = ae.AutoencoderEngine(ops_, hw + (1,), compute_dtype=dtype, device="cuda")
    eng.set_keras_weights(ws)
    return eng, ops_, ws


@pytest.mark.parametrize("dtype", ["float16", "mixed_bfloat16"])
@pytest.mark.parametrize("co,k", [(32, 3), (32, 5), (32, 7), (64, 3), (64, 5)])
@pytest.mark.parametrize("hw,n", [((16, 64), 3), ((7, 64), 2), ((1, 64), 2), ((128, 64), 2),
                                  ((24, 64), 300)])
def test_general_tail_matches_two_launches_and_oracle(gpu_device, dtype, co, k, hw, n,
                                                      monkeypatch):
    eng, ops_, ws = _model(dtype, hw, k, seed=31 * k + hw[0] + n, co=co)
    assert eng.tail and not eng.tail_train
    x = np.random.default_rng(k + n).uniform(0, 1, (n,) + hw + (1,)).astype(np.float32)
    xd = eng.to_compute(torch.from_numpy(x))
    eng.forward(xd)  # allocate, then poison the output and run again
    eng._buffers(n, False)["h"][len(ops_)].fill_(float("nan"))
    fused = eng.forward(xd).clone()
    monkeypatch.setenv("SPECENH_NO_TAIL_FUSION", "1")
    from specenh import ae
    plain_eng = ae.AutoencoderEngine(ops_, hw + (1,), compute_dtype=dtype, device="cuda")
    assert not plain_eng.tail
    plain_eng.set_keras_weights(ws)
    plain = plain_eng.forward(xd).clone()
    torch.cuda.synchronize()
    assert fused.shape == plain.shape == (n, 2 * hw[0], 2 * hw[1], 1)
    assert not torch.isnan(fused).any()
    d = (fused - plain).abs().max().item()
    print(f"co {co} k {k} {dtype} {hw} x {n}: fused vs two launches {d:.2e}")
    assert d <= 2e-3, d
    if n <= 3:
        spec = [("conv", 1, 32, 3, "relu"), ("convT", 32, co, k, "relu"),
                ("conv", co, 1, k, "sigmoid")]
        it = iter(ws)
        params = [{"W": torch.tensor(next(it), dtype=torch.float64),
                   "b": torch.tensor(next(it), dtype=torch.float64)} for _ in spec]
        with torch.no_grad():
            ref = ora.forward(spec, params, torch.tensor(x, dtype=torch.float64)).numpy()
        err = checks.out_rel(fused.cpu().numpy(), ref)
        print(f"  vs fp64 oracle out_rel {err:.2e}")
        assert err <= checks.TOL[dtype]["out_rel"], err


def test_general_tail_c_abi_shapes(gpu_device):
    """The C-ABI entry takes the new configurations on 64-wide inputs only; other widths and
    channel counts stay SPECENH_EUNSUPPORTED (the engine then runs two launches)."""
    from specenh import ops
    assert ops.tail_supported(torch.float16, 32, 32, 3, 3, 64)
    assert ops.tail_supported(torch.bfloat16, 32, 32, 7, 7, 64)
    assert not ops.tail_supported(torch.float16, 32, 32, 5, 5, 32)
    assert ops.tail_supported(torch.float16, 32, 64, 5, 5, 64)
    assert not ops.tail_supported(torch.float16, 32, 64, 7, 7, 64)
    assert not ops.tail_supported(torch.float32, 32, 32, 5, 5, 64)
    x = torch.zeros((1, 4, 32, 32), dtype=torch.float16, device=gpu_device)
    wt = torch.zeros(32 * 9 * 32, dtype=torch.float16, device=gpu_device)
    wo = torch.zeros(9 * 32, dtype=torch.float16, device=gpu_device)
    bt = torch.zeros(32, dtype=torch.float32, device=gpu_device)
    bo = torch.zeros(1, dtype=torch.float32, device=gpu_device)
    with pytest.raises(NotImplementedError):
        ops.ops.convt_conv_out(x, wt, bt, 32, 3, wo, bo, 3)
