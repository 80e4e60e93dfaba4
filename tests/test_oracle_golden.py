"""Pin the oracle to the reference: every oracle function vs the golden fixtures
captured from the reference's own code (tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest

from conftest import golden_params, golden_signal, load_golden, stft_cases, svd_cases
from oracle import filters, spectrogram, strips, svd


@pytest.mark.parametrize("case", stft_cases())
def test_specgr_matches_reference(case):
    g = load_golden(f"stft_{case}")
    x = golden_signal(g)
    p = golden_params(g)
    S, f, t = spectrogram.specgr_arrays(x, p)
    # bin/time indexing is bit-exact (same float64 formulas as scipy)
    assert np.array_equal(f, g["f"])
    assert np.array_equal(t, g["t"])
    assert S.shape == g["Sxx"].shape
    if g["Sxx"].dtype == np.float64:
        np.testing.assert_allclose(S, g["Sxx"], rtol=0, atol=1e-10)
    else:
        # fp32 fixture: scipy ran in fp32 and its fp32 lstsq detrend leaves up to
        # ~1e-3 relative error in the (tiny, post-detrend) DC row; the oracle is
        # fp64 truth on the same fp32 samples. Rows >= 1 agree to fp32 rounding.
        np.testing.assert_allclose(S[1:], g["Sxx"][1:], rtol=0, atol=1e-5)
        np.testing.assert_allclose(S[0], g["Sxx"][0], rtol=0, atol=1e-4)


@pytest.mark.parametrize("case", [c for c in stft_cases() if c != "bes_variant"])
def test_raw_psd_matches_scipy(case):
    g = load_golden(f"stft_{case}")
    x = golden_signal(g)
    p = golden_params(g)
    f, t, P = spectrogram.spectrogram_psd(x, fs=p["fs"], window=p["window"],
                                          nperseg=p["nperseg"], noverlap=p["noverlap"],
                                          detrend=p["detrend"], scaling=p["scaling"])
    assert np.array_equal(f, g["f_raw"]) and np.array_equal(t, g["t_raw"])
    ref = g["psd"].astype(np.float64)
    err = np.abs(P - ref).max() / np.abs(ref).max()
    assert err <= (1e-12 if g["psd"].dtype == np.float64 else 1e-5), err


def test_specgr_scipy_path_is_the_reference_chain():
    g = load_golden("stft_ref_hamm512")
    x = golden_signal(g)
    S, f, t = spectrogram.specgr_scipy(x, golden_params(g))
    np.testing.assert_array_equal(S, g["Sxx"])
    np.testing.assert_array_equal(f, g["f"])


@pytest.mark.parametrize("case", svd_cases())
def test_svd_denoiser_matches_reference(case):
    g = load_golden(f"svd_{case}")
    A = g["A"]
    tol = 1e-9 if A.dtype == np.float64 else 1e-4
    ref_norm = np.linalg.norm(A)

    def close(out, key):
        err = np.linalg.norm(out - g[key]) / ref_norm
        assert err <= tol, (key, err)

    close(svd.denoiseSignal(A), "default")
    close(svd.denoiseSignal(A, 0, 16), "r16")
    close(svd.denoiseSignal(A, 2, 10), "s2_10")
    close(svd.denoiseSignal(A, -3, 10_000), "clamp")
    assert not np.any(svd.denoiseSignal(A, 7, 3)) and not np.any(g["empty"])
    close(svd.denoiseSignal(A, use_optimal=True), "optimal")
    if "compute" in g:
        close(svd.computeSignal(A), "compute")
    m, n = A.shape
    assert svd.omega(min(m, n) / max(m, n)) == pytest.approx(float(g["omega_beta"]), abs=0)


def test_filters_match_reference():
    g = load_golden("filters")
    src = g["src"]
    np.testing.assert_allclose(filters.norm(src), g["norm"], atol=1e-13)
    np.testing.assert_allclose(filters.rescale(src), g["rescale"], atol=1e-13)
    np.testing.assert_array_equal(filters.quantfilt(src), g["quantfilt"])
    np.testing.assert_array_equal(filters.quantfilt(src, 0.5), g["quantfilt_05"])
    np.testing.assert_allclose(filters.meansub(src), g["meansub"], atol=1e-13)
    # the explicit linear-interpolation restatement equals np.quantile
    q = filters.quantile_linear(np.sort(src, axis=0), 0.9)
    np.testing.assert_allclose(q, np.quantile(src, 0.9, axis=0), atol=1e-15)


def test_strip_glue_index_map():
    S = np.arange(256 * 3905, dtype=np.float64).reshape(256, 3905)
    p = strips.patch([S, S + 1])
    assert p.shape == (60, 256, 128)
    assert np.array_equal(p[3], S[:, 384:512])
    assert np.array_equal(p[30 + 29], S[:, 3712:3840] + 1)
    u = strips.unpatch(p)
    assert u.shape == (2, 256, 3840)
    assert np.array_equal(u[0], S[:, :3840])
    assert strips.reshape(p).shape == (60, 256, 128, 1)


def test_cv2_restatement_properties():
    """gaussblr / morph restatement (cv2 absent: unpinned) — properties OpenCV documents:
    taps sum to 256 and are symmetric, sigma from ksize, the 3-tap small table, a constant
    image is a fixed point of the blur, OPEN with the centred 3x1 rect is anti-extensive."""
    t = filters.gaussian_taps_q8(31)
    assert t.sum() == 256 and (t == t[::-1]).all() and t[15] == t.max()
    assert filters.gaussian_taps_q8(3).tolist() == [64, 128, 64]
    c = np.full((9, 40), 77, np.uint8)
    np.testing.assert_array_equal(filters.gaussian_blur_u8(c), c)
    u = (np.random.default_rng(3).random((32, 48)) * 255).astype(np.uint8)
    opened = filters._morph_u8(filters._morph_u8(u, 1, 3, False), 1, 3, True)
    assert (opened <= u).all()
    out = filters.label_pipeline(np.random.default_rng(4).random((64, 96)))
    assert out.min() == 0.0 and out.max() == 1.0


def _ranges_fixture():
    d = load_golden("ranges_svd")
    out = {}
    for k, v in d.items():
        tag, key = k.split("__")
        out.setdefault(tag, {})[key] = v
    return out


def range_args(key):
    """'r_m4_m2' -> (-4, -2) (make_golden_svd_ranges.py's key format)."""
    a, b = key[2:].split("_")
    return tuple(-int(v[1:]) if v.startswith("m") else int(v) for v in (a, b))


def test_svd_slice_semantics_match_notebook():
    """Negative stop, num_sing == 0 under use_optimal, wide kept ranges: the oracle
    reproduces the notebook's Python slicing (denoising_by_svd.ipynb:216-228)."""
    for tag, e in _ranges_fixture().items():
        A = e["A"].astype(np.float64)
        scale = np.linalg.norm(A)
        for key, want in e.items():
            if key.startswith("r_"):
                got = svd.denoiseSignal(A, *range_args(key))
            elif key == "optimal":
                got = svd.denoiseSignal(A, use_optimal=True)
            elif key == "compute":
                got = svd.computeSignal(A)
            else:
                continue
            assert np.linalg.norm(got - want) <= 1e-6 * scale, (tag, key)
        if "num_sing" in e:
            assert svd.optimal_rank(e["s"], A.shape) == int(e["num_sing"])
    noise = _ranges_fixture()["noise64x48"]
    assert int(noise["num_sing"]) == 0 and np.any(noise["optimal"])  # keeps [0, r-1), not zeros
