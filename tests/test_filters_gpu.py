"""GPU parity of the label filters (csrc/filters.hip) — pipeline_data.py:38-61, SURVEY §8 f1 —
against the reference's own outputs (tests/golden/filters.npz, made by the reference's
functions) and the numpy restatement (oracle/filters.py).

Tolerances: quantfilt is exact (same order statistics, numpy's lerp reproduced in fp64,
then a comparison: bit-identical output); rescale is exact (min/max are exact);
norm / meansub reorder fp64 sums: max |delta| <= 1e-12 of the output range."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import filters as ref

pytestmark = pytest.mark.gpu


def test_filters_match_reference_fixture(gpu_device):
    from specenh import pipeline_data as pd

    g = load_golden("filters")
    src = g["src"]
    np.testing.assert_array_equal(pd.quantfilt(src), g["quantfilt"])
    np.testing.assert_array_equal(pd.quantfilt(src, 0.5), g["quantfilt_05"])
    np.testing.assert_array_equal(pd.rescale(src), g["rescale"])
    for name in ("norm", "meansub"):
        got = getattr(pd, name)(src)
        assert got.dtype == np.float64 and got.shape == src.shape
        assert np.abs(got - g[name]).max() <= 1e-12 * np.ptp(g[name]), name


@pytest.mark.parametrize("shape", [(256, 3905), (128, 128), (7, 5), (513, 3)])
def test_numpy_api_vs_oracle_shapes(shape, gpu_device):
    from specenh import pipeline_data as pd

    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    src = rng.random(shape)
    for thr in (0.9, 0.0, 1.0, 0.37):
        np.testing.assert_array_equal(pd.quantfilt(src, thr), ref.quantfilt(src, thr))
    np.testing.assert_array_equal(pd.rescale(src), ref.rescale(src))
    assert np.abs(pd.norm(src) - ref.norm(src)).max() <= 1e-12 * np.ptp(ref.norm(src))
    assert np.abs(pd.meansub(src) - ref.meansub(src)).max() <= 1e-12


def test_ties_and_nd_stacks(gpu_device):
    """Repeated values (stable ranks) and the notebooks' np.dstack'd (F, T, C) stacks."""
    from specenh import pipeline_data as pd

    rng = np.random.default_rng(3)
    src = rng.integers(0, 4, (40, 30)).astype(np.float64)
    np.testing.assert_array_equal(pd.quantfilt(src), ref.quantfilt(src))
    stack = rng.random((32, 50, 4))
    np.testing.assert_array_equal(pd.quantfilt(stack), ref.quantfilt(stack))
    np.testing.assert_array_equal(pd.rescale(stack), ref.rescale(stack))
    assert np.abs(pd.meansub(stack) - ref.meansub(stack)).max() <= 1e-12
    assert np.abs(pd.norm(stack) - ref.norm(stack)).max() <= 1e-11


def test_device_batch_fp32(gpu_device):
    """[B, F, T] float32 spectrograms on the device, each filtered independently."""
    import torch

    from specenh import filters

    rng = np.random.default_rng(4)
    S = rng.random((6, 128, 96)).astype(np.float32)
    t = torch.as_tensor(S, device=gpu_device)
    q = filters.quantfilt(t).cpu().numpy()
    m = filters.meansub(t).cpu().numpy()
    r = filters.rescale(t).cpu().numpy()
    for b in range(6):
        np.testing.assert_array_equal(q[b], ref.quantfilt(S[b]))
        np.testing.assert_allclose(r[b], ref.rescale(S[b]), rtol=0, atol=2e-7)
        np.testing.assert_allclose(m[b], ref.meansub(S[b].astype(np.float64)), rtol=0, atol=1e-6)


def test_errors(gpu_device):
    from specenh import pipeline_data as pd

    with pytest.raises(ValueError):
        pd.quantfilt(np.ones((4, 4)), 1.5)
    with pytest.raises(ValueError):  # cv2: ksize must be odd
        pd.gaussblr(np.random.default_rng(0).random((8, 8)), (4, 3))


# ---------------------------------------------------------------- cv2 steps (f1)
# gaussblr / morph: OpenCV is absent, so the oracle restates its 8-bit algorithms (integer
# arithmetic) and parity with cv2 itself is unpinned. GPU vs the restatement is exact on the
# uint8 image (integer taps and sums; the uint8 quantisation repeats numpy's expression in
# the same precision), so the rescaled outputs agree to the last fp64 bit.
_CV_SHAPES = [(256, 128), (129, 97), (5, 40), (64, 7), (1, 33), (3, 1)]


@pytest.mark.parametrize("shape", _CV_SHAPES)
def test_gaussblr_morph_match_restatement(gpu_device, shape):
    from specenh import pipeline_data as pd

    rng = np.random.default_rng(sum(shape))
    s = rng.random(shape) ** 3  # skewed, like a log spectrogram after quantfilt
    np.testing.assert_array_equal(pd.gaussblr(s), ref.gaussblr(s))
    np.testing.assert_array_equal(pd.gaussblr(s, (5, 5)), ref.gaussblr(s, (5, 5)))
    np.testing.assert_array_equal(pd.morph(s), ref.morph(s))


def test_label_pipeline_matches_restatement(gpu_device):
    """pipeline_data.py:101-110 (quantfilt -> gaussblr -> meansub -> morph -> meansub) on a
    real specgr output (fixture input regenerated from its seed)."""
    from specenh import pipeline_data as pd

    g = load_golden("filters")
    src = g["src"]
    out = pd.label_pipeline(src)
    exp = ref.label_pipeline(src)
    # the two meansub stages reorder fp64 row sums; the uint8 stages between them are exact
    # unless a value sits within ~1e-15 of a quantisation step
    assert out.shape == exp.shape and out.dtype == np.float64
    assert np.abs(out - exp).max() <= 1e-12


def test_label_pipeline_device_batch(gpu_device):
    """[B, rows, cols] float32 device batch: every spectrogram through the chain independently."""
    import torch

    from specenh import filters

    rng = np.random.default_rng(9)
    S = rng.random((4, 128, 128)).astype(np.float32)
    out = filters.label_pipeline(torch.as_tensor(S, device=gpu_device)).cpu().numpy()
    for b in range(4):
        g = filters.label_pipeline(torch.as_tensor(S[b], device=gpu_device)).cpu().numpy()
        np.testing.assert_array_equal(out[b], g)
        u = filters.gaussblr(torch.as_tensor(S[b], device=gpu_device)).cpu().numpy()
        np.testing.assert_allclose(u, ref.gaussblr(S[b]).astype(np.float32), rtol=0, atol=0)


def test_gaussblr_morph_constant_and_fp32(gpu_device):
    """Edge cases the reference hits: a constant image (rescale's 0/0 -> NaN, as numpy),
    and float32 device input quantised in float32 (numpy would do the same for an fp32
    array)."""
    import torch

    from specenh import filters

    c = np.full((16, 40), 0.25)
    with np.errstate(invalid="ignore"):
        np.testing.assert_array_equal(filters.gaussblr(c), ref.gaussblr(c))
        np.testing.assert_array_equal(filters.morph(c), ref.morph(c))
    assert np.isnan(filters.morph(c)).all()
    s = (np.random.default_rng(11).random((40, 70)) ** 2).astype(np.float32)
    m = filters.morph(torch.as_tensor(s, device=gpu_device)).cpu().numpy()
    np.testing.assert_array_equal(m, ref.morph(s).astype(np.float32))
