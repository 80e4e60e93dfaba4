"""Strip glue (csrc/strips.hip) vs the restated oracle (oracle/strips.py; patchify is
absent, so parity with patchify itself is unpinned — see the oracle's header).
Copies are exact: inputs are fp32-representable, bf16 packing equals a bf16 cast."""
import numpy as np
import pytest
import torch

from oracle import strips as ora

pytestmark = pytest.mark.gpu


def test_patch_unpatch_reshape_match_oracle(gpu_device):
    from specenh import strips
    rng = np.random.default_rng(0)
    specs = [rng.standard_normal((256, 3905)).astype(np.float32).astype(np.float64) for _ in range(3)]
    got = strips.patch(specs)
    ref = ora.patch(specs)
    assert got.dtype == np.float64 and got.shape == (90, 256, 128)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(strips.unpatch(got), ora.unpatch(ref))
    assert strips.reshape(got).shape == (90, 256, 128, 1)
    # len not a multiple of 30: the reference keeps int(len/30) spectrograms
    np.testing.assert_array_equal(strips.unpatch(got[:65]), ora.unpatch(ref[:65]))


def test_patch_batch_bf16_and_rows_from_taller_spectrogram(gpu_device):
    from specenh import strips
    S = torch.randn(2, 513, 4000, device=gpu_device)
    out = strips.patch_batch(S, dtype=torch.bfloat16)
    ref = torch.stack([S[b, :256, 128 * x:128 * x + 128] for b in range(2) for x in range(30)])
    assert torch.equal(out[..., 0], ref.to(torch.bfloat16))
    back = strips.unpatch_batch(out)
    assert torch.equal(back, ref.to(torch.bfloat16).float().reshape(2, 30, 256, 128)
                       .permute(0, 2, 1, 3).reshape(2, 256, 3840))


def test_patch_errors(gpu_device):
    from specenh import strips
    with pytest.raises(ValueError):
        strips.patch_batch(torch.zeros(1, 128, 4000, device=gpu_device))
    with pytest.raises(ValueError):
        strips.patch_batch(torch.zeros(1, 256, 3000, device=gpu_device))
    with pytest.raises(RuntimeError, match="GPU only"):
        strips.patch_batch(torch.zeros(1, 256, 4000))
