import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "spectrogram-enhancement_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def stft_cases():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, "stft_*.npz")))


def svd_cases():
    return sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, "svd_*.npz")))


def golden_signal(entry):
    """Regenerate the fixture's input from its seed and prove it is byte-identical."""
    from specenh.synthetic import digest, plasma_chirps

    x = plasma_chirps(1, int(entry["length"]), seed0=int(entry["seed"]),
                      dtype=np.dtype(str(entry["dtype"])))[0]
    assert digest(x) == str(entry["x_digest"]), "synthetic generator drifted from the fixture"
    return x


def golden_params(entry):
    return json.loads(str(entry["params"]))


@pytest.fixture(scope="session")
def gpu_device():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def kernel_variant():
    """kernel_variant("CONV_NO_S2", 1): select a kernel variant through the C-ABI switch
    (specenh_set_variant; the library reads the environment once), restored afterwards."""
    from specenh import _lib

    saved = {}

    def setv(name, value):
        name = name[8:] if name.startswith("SPECENH_") else name
        if name not in saved:
            saved[name] = _lib.get_variant(name)
        _lib.set_variant(name, int(value))

    yield setv
    for name, value in saved.items():
        _lib.set_variant(name, value)
