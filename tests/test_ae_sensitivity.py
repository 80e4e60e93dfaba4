"""The low-precision autoencoder checks can fail: a kernel that dropped one MFMA k-step
(one 5x5 tap of one layer's reduction, 16-32 products of each output's sum) moves the
metrics of oracle/checks.py by far more than the fp16/bf16 tolerances, and a constant
output fails outright. CPU only (fp64 oracle on the trained weights)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))

from oracle import autoencoder as ora  # noqa: E402
from oracle import checks  # noqa: E402


@pytest.fixture(scope="module")
def trained():
    from make_ae_weights import c4_pairs, load

    x, _ = c4_pairs(3, seed0=9000)
    return load(), torch.tensor(x, dtype=torch.float64)


def _params(spec, ws):
    it, out = iter(ws), []
    for lay in spec:
        out.append(None if lay[0] == "pool" else
                   {"W": torch.tensor(next(it), dtype=torch.float64),
                    "b": torch.tensor(next(it), dtype=torch.float64)})
    return out


def test_trained_weights_are_not_degenerate(trained):
    ws, x = trained
    spec = ora.ae_spec()
    with torch.no_grad():
        out, z = ora.forward(spec, _params(spec, ws), x, return_logits=True)
    assert float(out.std()) > 0.1 and float(z.std()) > 1.0
    # a constant output at the mean fails every tolerance
    const = np.full(out.shape, float(out.mean()))
    assert checks.out_rel(const, out.numpy()) >= 0.99


@pytest.mark.parametrize("layer,tap", [(2, (2, 2)), (4, (0, 0)), (6, (4, 4)), (7, (1, 3)),
                                       (8, (2, 2)), (9, (2, 2))])
def test_dropped_kstep_fails_the_checks(trained, layer, tap):
    ws, x = trained
    spec = ora.ae_spec()
    with torch.no_grad():
        out0, z0 = ora.forward(spec, _params(spec, ws), x, return_logits=True)
    convs = [i for i, lay in enumerate(spec) if lay[0] != "pool"]
    w2 = [w.copy() for w in ws]
    W = w2[2 * convs.index(layer)]
    ky, kx = tap
    if spec[layer][0] == "conv":
        W[ky, kx, :32, :] = 0.0   # reduction index (ky, kx, ci < 32): one 16x16x32 k-step
    else:
        W[ky, kx, :, :32] = 0.0
    with torch.no_grad():
        out1, z1 = ora.forward(spec, _params(spec, w2), x, return_logits=True)
    o, zz = checks.out_rel(out1.numpy(), out0.numpy()), checks.logit_rel(z1.numpy(), z0.numpy())
    assert max(o, zz) >= checks.KSTEP_MIN, (o, zz)
    for dt in ("float16", "mixed_bfloat16"):
        tol = checks.TOL[dt]
        assert o > tol["out_rel"] or zz > tol["logit_rel"], dt
