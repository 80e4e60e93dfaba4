"""Golden fixtures for denoiseSignal's full slice semantics, from the REFERENCE's notebook.

``denoising_by_svd.ipynb:216-228`` ends with ``u[:, start:stop] @ np.diag(s[start:stop]) @
vh[start:stop, :]`` after clamping only ``start < 0`` and ``stop > r``: a negative ``stop``
is a Python slice bound (``stop + r``), and ``use_optimal`` with ``num_sing == 0`` sets
``stop = -1``, i.e. keeps components ``[0, r - 1)``. These fixtures pin that branch and the
wide kept ranges (K > 40) that need more than a top-K subspace.

Every matrix is rounded to float32 first and stored that way, so the GPU (which computes
from fp32 inputs) and the notebook (float64 LAPACK on the same values) see identical data.
Runs only in the build container (needs /root/reference), like make_golden.py.

Usage:  python tests/golden/make_golden_svd_ranges.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import gapped_matrix, load_reference  # noqa: E402

# (tag, builder, list of (key, args, kwargs))
RANGES = [(1, -1), (0, -3), (2, -5), (0, -100), (-4, -2), (5, 3), (0, 100), (0, 40),
          (0, 41), (3, 45), (10, 30)]


def _key(a, b):
    return f"r_{a}_{b}".replace("-", "m")


def main():
    _, nb = load_reference()
    den, comp = nb["denoiseSignal"], nb["computeSignal"]
    out = {}
    cases = {
        # pure Gaussian noise: num_sing == 0, so use_optimal keeps [0, r-1)
        "noise64x48": np.random.default_rng(811).standard_normal((64, 48)),
        "noise40x72": np.random.default_rng(812).standard_normal((40, 72)),
        # designed gap after 16 components (SURVEY §8(d) C3 construction)
        "gap96x80": gapped_matrix(813, 96, 80),
        "gap72x100": gapped_matrix(814, 72, 100),
    }
    for tag, A in cases.items():
        A32 = A.astype(np.float32)
        A64 = A32.astype(np.float64)
        e = {"A": A32}
        s = np.linalg.svd(A64, compute_uv=False)
        e["s"] = s
        # outputs stored as float32: 6e-8 relative, far inside the 1e-5 parity tolerance
        e["optimal"] = den(A64, use_optimal=True).astype(np.float32)
        e["compute"] = comp(A64).astype(np.float32)
        for a, b in RANGES:
            e[_key(a, b)] = den(A64, a, b).astype(np.float32)
        beta = min(A.shape) / max(A.shape)
        e["num_sing"] = np.int64((s > nb["omega"](beta) * np.median(s)).sum())
        out[tag] = e
        print(tag, A.shape, "num_sing", int(e["num_sing"]))
    # BASELINE config-3 geometry (513 x 256) with a K = 100 range (cut inside the noise)
    A32 = gapped_matrix(815, 513, 256).astype(np.float32)
    A64 = A32.astype(np.float64)
    out["c3_513x256"] = {"A": A32, "r_0_100": den(A64, 0, 100).astype(np.float32)}
    np.savez_compressed(os.path.join(HERE, "ranges_svd.npz"),
                        **{f"{t}__{k}": v for t, e in out.items() for k, v in e.items()})
    print("wrote ranges_svd.npz", os.path.getsize(os.path.join(HERE, "ranges_svd.npz")) / 1e6, "MB")


if __name__ == "__main__":
    main()
