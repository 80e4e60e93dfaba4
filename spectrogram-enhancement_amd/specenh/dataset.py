"""The dataset builder of spec_denoising/pipeline_data.py's main loop (:86-123).

The reference walks ``*.pkl`` shot files; for each of 20 ECE channels it runs ``specgr``
and the label chain (quantfilt -> gaussblr -> meansub -> morph -> meansub, :101-110) one
channel at a time on the CPU and writes an HDF5 group ``ece_<shot>/chn_<n>`` holding the
datasets ``spec``, ``f``, ``t`` and ``pipeline_out`` (:112-116). Here every channel of a
shot goes through the GPU in ONE batch: the signals are uploaded together, one
``specgr_batch`` launch gives all spectrograms and one ``label_pipeline`` pass gives all
labels; only the finished arrays come back to the host.

Storage: the same group/dataset paths. h5py (the reference's writer) is not installed in
this image, so :class:`SpectrogramStore` keeps them as ``<root>/ece_<shot>/chn_<n>/<name>.npy``
(loaded with ``allow_pickle=False``); with h5py importable ``backend="hdf5"`` writes the
reference's HDF5 file itself. Error behaviour follows the loop: a file that fails to
unpickle is skipped (``pickle.UnpicklingError``, :118-119); a missing channel or any other
per-channel failure is reported and skipped (:120-122); an existing group is an error, as
``h5py.Group.create_group`` makes it.
"""
from __future__ import annotations

import os
import pickle
import traceback

import numpy as np
import torch

from . import filters as _filters
from . import pipeline_data as _pd
from . import stft as _stft

REFERENCE_SPEC_PARAMS = {  # pipeline_data.py:77-84
    "nperseg": 512, "noverlap": 256, "fs": 500000, "window": "hamm",
    "scaling": "density", "detrend": "linear", "eps": 1e-11,
}


class _NpyGroup:
    def __init__(self, path):
        self.path = path

    def create_dataset(self, name, data):
        p = os.path.join(self.path, name + ".npy")
        if os.path.exists(p):
            raise ValueError(f"Unable to create dataset (name already exists): {name}")
        np.save(p, np.asarray(data), allow_pickle=False)

    def __getitem__(self, name):
        return np.load(os.path.join(self.path, name + ".npy"), allow_pickle=False)

    def keys(self):
        return sorted(f[:-4] for f in os.listdir(self.path) if f.endswith(".npy"))


class SpectrogramStore:
    """``ece_<shot>/chn_<n>/{spec,f,t,pipeline_out}`` groups (pipeline_data.py:90,112-116)."""

    def __init__(self, root, mode="a", backend="npy"):
        self.backend = backend
        if backend == "hdf5":
            import h5py  # the reference's writer; absent in this image

            self._h5 = h5py.File(root, mode)
        elif backend == "npy":
            self._h5 = None
            self.root = root
            os.makedirs(root, exist_ok=True)
        else:
            raise ValueError(f"unknown backend {backend!r}")

    def create_group(self, name):
        if self._h5 is not None:
            return self._h5.create_group(name)
        p = os.path.join(self.root, *name.split("/"))
        if os.path.isdir(p):
            raise ValueError(f"Unable to create group (name already exists): {name}")
        os.makedirs(p)
        return _NpyGroup(p)

    def __getitem__(self, name):
        if self._h5 is not None:
            return self._h5[name]
        p = os.path.join(self.root, *name.split("/"))
        if not os.path.isdir(p):
            raise KeyError(name)
        return _NpyGroup(p)

    def groups(self):
        """Every ``ece_<shot>/chn_<n>`` path in the store, sorted."""
        if self._h5 is not None:
            return sorted(f"{s}/{c}" for s in self._h5 for c in self._h5[s])
        out = []
        for s in sorted(os.listdir(self.root)):
            sp = os.path.join(self.root, s)
            if os.path.isdir(sp):
                out += [f"{s}/{c}" for c in sorted(os.listdir(sp))]
        return out

    def close(self):
        if self._h5 is not None:
            self._h5.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def shot_number(fname):
    """pipeline_data.py:91: the text between the last '_' and the last '.'."""
    return fname[fname.rfind("_") + 1:fname.rfind(".")]


def process_shot(fname, spec_params, store, n_channels=20, cut_shot=2, thr=0.9,
                 key_format="\\tecef%.2i", log=print):
    """All channels of one shot file -> the store. Returns the number of groups written."""
    shotn = shot_number(fname)
    try:
        with open(fname, "rb") as fh:
            data = pickle.load(fh)  # the reference's own data format (its shot files)
    except pickle.UnpicklingError:
        return 0
    n_samp = int(np.int_(cut_shot * spec_params["fs"]))
    sigs, chans = [], []
    for chn in range(1, n_channels + 1):
        try:
            sig = np.asarray(data[key_format % chn], dtype=np.float32)[:n_samp]
            sigs.append(sig)
            chans.append(chn)
        except Exception:  # noqa: BLE001 — the reference prints and continues (:120-122)
            log(traceback.format_exc())
    written = 0
    # channels of one shot normally share a length: one launch per distinct length
    for L in sorted({s.shape[0] for s in sigs}):
        idx = [i for i, s in enumerate(sigs) if s.shape[0] == L]
        try:
            x = torch.as_tensor(np.stack([sigs[i] for i in idx]), device=_pd._device())
            S = _pd.specgr_batch(x, spec_params)
            lab = _filters.label_pipeline(S.double(), thr)
            S_h, lab_h = S.double().cpu().numpy(), lab.cpu().numpy()
        except Exception:  # noqa: BLE001
            log(traceback.format_exc())
            continue
        p = _pd._params(spec_params)
        f = _stft.frequencies(p["nperseg"], p["fs"])[:-1]
        t = _stft.times(L, p["nperseg"], p["noverlap"], p["fs"])
        for j, i in enumerate(idx):
            grp = store.create_group("ece_" + shotn + "/chn_" + str(chans[i]))
            grp.create_dataset("spec", data=S_h[j])
            grp.create_dataset("f", data=f)
            grp.create_dataset("t", data=t)
            grp.create_dataset("pipeline_out", data=lab_h[j])
            written += 1
    return written


def build_dataset(flist, out_path, spec_params=None, n_channels=20, cut_shot=2, thr=0.9,
                  backend="npy", log=print):
    """pipeline_data.py:86-123 over a list of shot files. Returns groups written."""
    spec_params = REFERENCE_SPEC_PARAMS if spec_params is None else spec_params
    total = 0
    with SpectrogramStore(out_path, "a", backend) as store:
        for fname in flist:
            total += process_shot(fname, spec_params, store, n_channels, cut_shot, thr, log=log)
    return total
