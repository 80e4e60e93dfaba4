"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Runs only in the build container (it needs /root/reference). The reference
cannot travel to the GPU box, so what it computes here is frozen as small npz
fixtures (inputs are regenerated from seeds by ``specenh.synthetic``; a sha256
digest of each regenerated input is stored so tests can prove the generator is
byte-identical).

How the reference is loaded (verified recipes):
  * ``spec_denoising/pipeline_data.py`` is imported normally after inserting stub
    modules for its unused heavy imports (patchify, cv2, skimage, h5py). Only
    ``specgr, norm, rescale, quantfilt, meansub`` are exercised; ``gaussblr`` and
    ``morph`` need the real cv2, which is absent (parity unpinned for those).
  * ``spec_denoising/denoising_by_svd.ipynb`` code cell 1 (which defines the BES
    ``specgr`` variant, ``omega``, ``computeSignal``, ``denoiseSignal``) is exec'd
    from its JSON source.
The reference reads shots from pickles; we write the seeded synthetic shots to
temporary pickles under the keys the reference expects.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import pickle
import sys
import tempfile
import types

import numpy as np

sys.dont_write_bytecode = True  # never write into the read-only reference tree

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "spectrogram-enhancement_amd"))

from specenh.synthetic import digest, plasma_chirps  # noqa: E402


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m


def load_reference():
    _stub("patchify", patchify=None, unpatchify=None)
    _stub("cv2")
    _stub("h5py")
    _stub("skimage", color=None, data=None, restoration=None)
    _stub("skimage.exposure", rescale_intensity=None)
    sys.path.insert(0, os.path.join(REF, "spec_denoising"))
    import pipeline_data as ref  # noqa: E402

    import scipy  # noqa: F401
    import scipy.signal  # noqa: F401
    nb = json.load(open(os.path.join(REF, "spec_denoising", "denoising_by_svd.ipynb")))
    g = {"np": np, "scipy": scipy, "pickle": pickle}
    exec("".join(nb["cells"][1]["source"]), g)
    return ref, g


FS = 500000

STFT_CASES = [
    # name, seed, length, spec_params overrides, input dtype
    ("c1_hann256", 101, 16512, dict(nperseg=256, noverlap=128, window="hann"), "float64"),
    ("ref_hamm512", 202, 65792, dict(nperseg=512, noverlap=256, window="hamm"), "float64"),
    ("c2_hamm1024_f64", 303, 32768, dict(nperseg=1024, noverlap=768, window="hamm"), "float64"),
    ("c2_hamm1024_f32", 303, 32768, dict(nperseg=1024, noverlap=768, window="hamm"), "float32"),
    # spec_params variants the reference's dict documents (pipeline_data.py:77-84)
    ("v_const_spectrum", 404, 4096, dict(nperseg=256, noverlap=192, window="hann",
                                         detrend="constant", scaling="spectrum"), "float64"),
    ("v_nodetrend_blackman", 405, 4096, dict(nperseg=256, noverlap=192, window="blackman",
                                             detrend=False), "float64"),
    ("v_boxcar_hop_odd", 406, 5000, dict(nperseg=128, noverlap=61, window="boxcar"), "float64"),
    # edge cases: a single frame; leftover samples that do not fill a frame; odd T
    ("e_single_frame", 407, 512, dict(nperseg=512, noverlap=256, window="hamm"), "float64"),
    ("e_leftover", 408, 1024 + 3 * 256 + 255, dict(nperseg=1024, noverlap=768, window="hamm"),
     "float64"),
    ("e_n64", 409, 640, dict(nperseg=64, noverlap=32, window="hann"), "float64"),
    ("e_n2048", 410, 2048 * 4, dict(nperseg=2048, noverlap=1024, window="hamm"), "float64"),
    ("e_n4096", 411, 4096 * 3, dict(nperseg=4096, noverlap=2048, window="hann"), "float32"),
]


def base_params(**over):
    p = {"nperseg": 512, "noverlap": 256, "fs": FS, "window": "hamm",
         "scaling": "density", "detrend": "linear", "eps": 1e-11}
    p.update(over)
    return p


def gapped_matrix(seed, m, n, k=16, dtype=np.float64):
    """U diag(s) V^T with s_i = 10*0.8^i (i<k) then a gap to 0.01*U[0.5,1]."""
    rng = np.random.default_rng(seed)
    r = min(m, n)
    u, _ = np.linalg.qr(rng.standard_normal((m, r)))
    v, _ = np.linalg.qr(rng.standard_normal((n, r)))
    s = np.empty(r)
    s[:k] = 10.0 * 0.8 ** np.arange(k)
    s[k:] = 0.01 * rng.uniform(0.5, 1.0, r - k)
    return ((u * s) @ v.T).astype(dtype)


def main():
    import scipy.signal

    ref, nb = load_reference()
    tmp = tempfile.mkdtemp()
    fixtures = {}

    # ---------------- (g1)/(g2) specgr + raw scipy PSD ----------------
    for name, seed, length, over, dt in STFT_CASES:
        x = plasma_chirps(1, length, seed0=seed, dtype=np.dtype(dt))[0]
        p = base_params(**over)
        fname = os.path.join(tmp, f"{name}.pkl")
        with open(fname, "wb") as fh:
            pickle.dump({"\\tecef01": x}, fh)
        S, f, t = ref.specgr(fname, 1, p, 2)
        f_raw, t_raw, P = scipy.signal.spectrogram(
            x, nperseg=p["nperseg"], noverlap=p["noverlap"], fs=p["fs"], window=p["window"],
            scaling=p["scaling"], detrend=p["detrend"])
        entry = {
            "seed": np.int64(seed), "length": np.int64(length), "dtype": np.str_(dt),
            "params": np.str_(json.dumps(p)), "x_digest": np.str_(digest(x)),
            "Sxx": S, "f": f, "t": t, "psd": P, "f_raw": f_raw, "t_raw": t_raw,
        }
        fixtures[f"stft_{name}"] = entry
        print(f"stft {name}: Sxx {S.shape} {S.dtype}, psd {P.shape} {P.dtype}")

    # BES variant of specgr (denoising_by_svd.ipynb cell 1): key 'besfu%02d'/'data.BES'
    x = plasma_chirps(1, 16640, seed0=501, dtype=np.float64)[0]
    fname = os.path.join(tmp, "bes.pkl")
    with open(fname, "wb") as fh:
        pickle.dump({"besfu03": {"data.BES": x}}, fh)
    S, f, t = nb["specgr"](fname, 3, nb["spec_params"], 2)
    fixtures["stft_bes_variant"] = {
        "seed": np.int64(501), "length": np.int64(16640), "dtype": np.str_("float64"),
        "params": np.str_(json.dumps(nb["spec_params"])), "x_digest": np.str_(digest(x)),
        "Sxx": S, "f": f, "t": t}
    print("stft bes_variant:", S.shape)

    # ---------------- (g3) SVD denoiser ----------------
    svd = {}
    for tag, seed, m, n, dt in [("s64x48_f64", 601, 64, 48, np.float64),
                                ("s64x48_f32", 601, 64, 48, np.float32),
                                ("s48x64_f64", 602, 48, 64, np.float64),
                                ("s128x96_f64", 603, 128, 96, np.float64),
                                ("s160x128_f32", 604, 160, 128, np.float32)]:
        A = gapped_matrix(seed, m, n, dtype=dt)
        e = {"A": A}
        e["default"] = nb["denoiseSignal"](A)
        e["r16"] = nb["denoiseSignal"](A, 0, 16)
        e["s2_10"] = nb["denoiseSignal"](A, 2, 10)
        e["clamp"] = nb["denoiseSignal"](A, -3, 10_000)
        e["empty"] = nb["denoiseSignal"](A, 7, 3)
        e["optimal"] = nb["denoiseSignal"](A, use_optimal=True)
        try:
            e["compute"] = nb["computeSignal"](A)
        except IndexError:
            e["compute_raises"] = np.bool_(True)
        e["omega_beta"] = np.float64(nb["omega"](min(m, n) / max(m, n)))
        _, s, _ = np.linalg.svd(A.astype(np.float64), full_matrices=False)
        e["s"] = s
        svd[tag] = e
        print("svd", tag, {k: getattr(v, "shape", v) for k, v in e.items() if k != "A"})
    for tag, e in svd.items():
        fixtures[f"svd_{tag}"] = e
    # ---------------- (g4) filter helpers ----------------
    rng = np.random.default_rng(701)
    src = rng.random((64, 80))
    fixtures["filters"] = {
        "src": src,
        "norm": ref.norm(src), "rescale": ref.rescale(src),
        "quantfilt": ref.quantfilt(src), "quantfilt_05": ref.quantfilt(src, 0.5),
        "meansub": ref.meansub(src),
    }

    for name, entry in fixtures.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **entry)
    total = sum(os.path.getsize(os.path.join(HERE, f"{n}.npz")) for n in fixtures)
    print(f"wrote {len(fixtures)} fixtures, {total/1e6:.2f} MB")


if __name__ == "__main__":
    main()
