"""Workloads for rocprofv3 PMC passes, at the bench's launch shapes, with a manifest that
maps every library dispatch to its stage (tools/pmc_fold.py keys the counters by it).

    python tools/pmc_workload.py TARGET OUTDIR [--reps 3]

TARGET  c5    the bench's timed chain on one 2048-shot slice (one stream): specgr (fp16 in)
              -> denoiseSignal default (fp16 out) -> fp16 autoencoder forward (bench.py)
        c2    STFT C2: 4096 x 65,536 fp32, nperseg 1024 / hop 256, specgr normalisation
        csd   cross-power amplitude, 2048 pairs at the C2 geometry
        c3    SVD C3: 4096 x 513 x 256 gapped, rank 16 and default
        c4    one bf16 fit step, batch 128 (forward, BCE, backward, Adam)

Every kernel the library launches is counted on the host (specenh_launch_count); the i-th
one is the i-th specenh dispatch of the process in the rocprofv3 CSV. The manifest lists,
per profiled repetition, the dispatch index range of each stage and, for each autoencoder
layer, the symbol the engine recorded for it (specenh_last_kernel_name); other stages list
the symbols of their launches (specenh_kernel_name_at).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib, ae, pipeline_data, svd  # noqa: E402
from specenh.synthetic import plasma_chirps_torch  # noqa: E402

WARMUP = 2


def stages_c5(dev):
    Hs = 2048
    x16 = plasma_chirps_torch(Hs, bench.L5, seed=1000, device=dev).to(torch.float16)
    S = torch.empty((Hs, bench.HW5, bench.HW5), dtype=torch.float32, device=dev)
    A = torch.empty((Hs, bench.HW5, bench.HW5, 1), dtype=torch.float16, device=dev)
    eng = bench.make_c5_engine(dev)
    names = bench.layer_names(eng)

    def stft():
        pipeline_data.specgr_batch(x16, bench.SPEC5, out=S)

    def svd_():
        svd.denoise_batch(S, out=A.view(Hs, bench.HW5, bench.HW5))

    def forward(kernels):
        eng.forward(A, timing=[], kernels=kernels)

    return {"batch": Hs, "stages": [("stft_c5", stft), ("svd_c5", svd_)],
            "layers": (forward, names)}


def stages_c2(dev):
    B = 4096
    x = plasma_chirps_torch(B, bench.L2, seed=7, device=dev)
    o = torch.empty((B, bench.F2, bench.T2), dtype=torch.float32, device=dev)
    return {"batch": B, "stages": [("stft_c2", lambda: pipeline_data.specgr_batch(
        x, bench.SPEC2, out=o))]}


def stages_csd(dev):
    from specenh import cross
    B = 2048
    x = plasma_chirps_torch(2 * B, bench.L2, seed=7, device=dev)
    xa, xb = x[:B], x[B:]
    return {"batch": B, "stages": [("csd_c2", lambda: cross.cross_spectrogram_batch(
        xa, xb, 5e5, "hamm", 1024, 768, "linear", "density", amplitude=True))]}


def stages_c3(dev):
    A = bench.c3_matrices(dev)
    out = torch.empty_like(A)
    return {"batch": A.shape[0], "stages": [
        ("svd_c3_rank16", lambda: svd.denoise_batch(A, 0, 16, out=out)),
        ("svd_c3_default", lambda: svd.denoise_batch(A, None, None, out=out))]}


def stages_c4(dev):
    eng, x, y = bench.c4_engine_and_batch(dev, 128)
    return {"batch": 128, "stages": [("c4_train_step", lambda: eng.train_step(x, y))]}


TARGETS = {"c5": stages_c5, "c2": stages_c2, "csd": stages_csd, "c3": stages_c3,
           "c4": stages_c4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("target", choices=sorted(TARGETS))
    ap.add_argument("outdir")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = TARGETS[a.target](dev)
    reps = []
    for r in range(WARMUP + a.reps):
        rec = []
        for name, fn in w["stages"]:
            c0 = _lib.launch_count()
            fn()
            c1 = _lib.launch_count()
            rec.append({"stage": name, "first": c0, "end": c1,
                        "symbols": _lib.kernel_names(c0, c1)})
        if "layers" in w:
            forward, names = w["layers"]
            c0 = _lib.launch_count()
            kernels = []
            forward(kernels)
            c1 = _lib.launch_count()
            if c1 - c0 != len(kernels):
                raise RuntimeError(f"forward launched {c1 - c0} kernels, recorded {len(kernels)}")
            for i, (nm, sym) in enumerate(zip(names, kernels)):
                rec.append({"stage": nm, "first": c0 + i, "end": c0 + i + 1, "symbols": [sym]})
        if r >= WARMUP:
            reps.append(rec)
    torch.cuda.synchronize()
    os.makedirs(a.outdir, exist_ok=True)
    with open(os.path.join(a.outdir, "manifest.json"), "w") as fh:
        json.dump({"target": a.target, "batch": w["batch"], "reps": reps,
                   "total_launches": _lib.launch_count()}, fh, indent=1)
    print(f"[pmc_workload] {a.target}: {len(reps)} reps, {_lib.launch_count()} launches")


if __name__ == "__main__":
    main()
