"""Dataset builder of pipeline_data.py's main loop (:86-123): group layout
``ece_<shot>/chn_<n>/{spec,f,t,pipeline_out}``, skip-on-error behaviour, and GPU parity of
the batched per-shot path with the per-channel reference chain (oracle restatement)."""
import os
import pickle

import numpy as np
import pytest

from oracle import filters as ref_filters
from oracle import spectrogram as ref_spec


def _store_mod():
    from specenh import dataset

    return dataset


def test_store_layout_and_errors(tmp_path):
    ds = _store_mod()
    assert ds.shot_number("/data/ECE_data/ece_178631.pkl") == "178631"
    with ds.SpectrogramStore(str(tmp_path / "out")) as st:
        g = st.create_group("ece_1/chn_3")
        g.create_dataset("spec", data=np.arange(6.0).reshape(2, 3))
        with pytest.raises(ValueError):
            st.create_group("ece_1/chn_3")
        with pytest.raises(ValueError):
            g.create_dataset("spec", data=np.zeros(1))
        assert st.groups() == ["ece_1/chn_3"]
        np.testing.assert_array_equal(st["ece_1/chn_3"]["spec"], np.arange(6.0).reshape(2, 3))
        with pytest.raises(KeyError):
            st["ece_2/chn_1"]


def _chirp(seed, n):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 5e5
    f0, k = rng.uniform(1e4, 2e5), rng.uniform(-5e5, 5e5)
    return (np.sin(2 * np.pi * (f0 * t + 0.5 * k * t * t)) + 0.5 * rng.standard_normal(n)
            + rng.uniform(-1, 1) * np.arange(n) / n)


@pytest.mark.gpu
def test_build_dataset_matches_per_channel_chain(gpu_device, tmp_path):
    ds = _store_mod()
    params = dict(ds.REFERENCE_SPEC_PARAMS)
    n = 33_024  # 128 frames of 512 / hop 256 (cut_shot = 1 s keeps every sample)
    good = str(tmp_path / "ece_4242.pkl")
    with open(good, "wb") as fh:  # channels 1, 2 and 4 (3 missing -> reported, skipped)
        pickle.dump({"\\tecef%.2i" % c: _chirp(c, n) for c in (1, 2, 4)}, fh)
    bad = str(tmp_path / "ece_999.pkl")
    with open(bad, "wb") as fh:
        fh.write(b"not a pickle")
    msgs = []
    out = str(tmp_path / "store")
    total = ds.build_dataset([good, bad], out, params, n_channels=4, cut_shot=1,
                             log=msgs.append)
    assert total == 3 and len(msgs) == 1 and "KeyError" in msgs[0]
    st = ds.SpectrogramStore(out)
    assert st.groups() == ["ece_4242/chn_1", "ece_4242/chn_2", "ece_4242/chn_4"]
    for c in (1, 2, 4):
        g = st["ece_4242/chn_%d" % c]
        x = _chirp(c, n).astype(np.float32).astype(np.float64)  # what the GPU receives
        S, f, t = ref_spec.specgr_arrays(x, params, cut_shot=1)
        assert g["spec"].shape == S.shape == (256, 128)
        np.testing.assert_array_equal(g["f"], f)
        np.testing.assert_array_equal(g["t"], t)
        assert np.abs(g["spec"] - S).max() <= 1e-5  # §8(d) STFT fp32 tolerance
        lab = ref_filters.label_pipeline(g["spec"])  # label chain on the stored spectrogram
        assert np.abs(g["pipeline_out"] - lab).max() <= 1e-12
