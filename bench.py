"""Benchmark of the spectrogram hot path (BASELINE.json config 2) on 1..N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one pass of the hot path over one batch resident in HBM:
4096 synthetic plasma shots x 65,536 fp32 samples -> specgr chain (spectrogram PSD
with nperseg 1024 / hop 256 'hamm' window, linear detrend, density scaling,
log(S+eps), per-spectrogram min-max, drop Nyquist) -> 4096 x 512 x 253 fp32.
Each rank owns its own 4096 shots (shot-sharded, no collective in the data path;
weak scaling); value = all ranks' spectrograms / max-over-ranks wall time.

Rank 0 prints ONE JSON line (contract in the task statement) with:
  roofline      the dominant (and only) kernel of a step, stft_psd_kernel<1024>, timed
                with HIP events on the stream it runs on; achieved = 780,288
                algorithmic bytes per spectrogram x 4096 / its average launch time
                (SURVEY.md §8(d) C2).
  cpu_baseline  the reference's CPU chain (scipy.signal.spectrogram -> log -> min-max
                -> drop row, oracle.spectrogram.specgr_scipy) on a bounded sample of
                the same workload, timed on this host's cores before the GPU is
                touched (a reported baseline, not the target).
  psnr_db       PSNR of GPU spectrograms vs the fp64 CPU oracle on sample shots.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]

B_SHOTS = 4096
LENGTH = 65536
SPEC = {"nperseg": 1024, "noverlap": 768, "fs": 500000, "window": "hamm",
        "scaling": "density", "detrend": "linear", "eps": 1e-11}
F_OUT = SPEC["nperseg"] // 2
T_FRAMES = (LENGTH - SPEC["nperseg"]) // (SPEC["nperseg"] - SPEC["noverlap"]) + 1
ALG_BYTES = 4 * LENGTH + 4 * F_OUT * T_FRAMES  # 780,288 B per spectrogram
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "spectrograms/s (STFT+VAE-denoise fwd) at 1/2/4/8 GPUs; PSNR vs CPU ref"


# ------------------------------------------------------------------ CPU baseline
def _cpu_worker(args):
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    shots = args
    from oracle.spectrogram import specgr_scipy

    for x in shots:
        specgr_scipy(x, SPEC)
    return len(shots)


def cpu_baseline(n_shots: int) -> dict:
    """Reference CPU chain on n_shots of the same workload, one shot per task, all cores."""
    from specenh.synthetic import plasma_chirps

    cores = min(16, len(os.sched_getaffinity(0)))
    x = plasma_chirps(n_shots, LENGTH, seed0=0, dtype=np.float32)
    chunks = [x[i::cores] for i in range(cores)]
    ctx = mp.get_context("fork")  # before any GPU initialisation in this process
    with ctx.Pool(cores) as pool:
        pool.map(_cpu_worker, [c[:1] for c in chunks])  # warm imports
        t0 = time.perf_counter()
        done = sum(pool.map(_cpu_worker, chunks))
        dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "spectrograms/s", "cores": cores, "kind": "port",
            "sample": f"{done} shots x {LENGTH} fp32 samples through scipy.signal.spectrogram "
                      f"(nperseg 1024/hop 256 hamm, linear detrend) + log + min-max + drop row, "
                      f"{cores} worker processes x 1 thread, {dt:.2f} s wall"}


# ------------------------------------------------------------------ GPU
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=B_SHOTS)
    ap.add_argument("--cpu-shots", type=int, default=768)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_shots)

    import torch
    import torch.distributed as dist

    from specenh import pipeline_data
    from specenh.synthetic import plasma_chirps_torch

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    B = args.batch
    x = plasma_chirps_torch(B, LENGTH, seed=1000 + rank, device=dev)
    out = torch.empty((B, F_OUT, T_FRAMES), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()

    def step():
        pipeline_data.specgr_batch(x, SPEC, out=out)

    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- dominant kernel: the step IS one launch of stft_psd_kernel<1024> (log, min-max
    # and drop-Nyquist fused); time that launch with HIP events on the stream it runs on ----
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kreps = max(5, args.steps)
    ev0.record(stream)
    for _ in range(kreps):
        step()
    ev1.record(stream)
    ev1.synchronize()
    kernel_ms = ev0.elapsed_time(ev1) / kreps
    achieved = ALG_BYTES * B / (kernel_ms * 1e-3) / 1e9

    # ---- PSNR vs the fp64 CPU oracle on sample shots ----
    psnr = None
    if rank == 0:
        from oracle.spectrogram import specgr_arrays

        step()
        torch.cuda.synchronize()
        mses = []
        for b in (0, B // 2, B - 1):
            truth, _, _ = specgr_arrays(x[b].double().cpu().numpy(), SPEC)
            mses.append(float(np.mean((out[b].double().cpu().numpy() - truth) ** 2)))
        mse = max(np.mean(mses), 1e-300)
        psnr = 10.0 * np.log10(1.0 / mse)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return

    total = world * B * args.steps
    res = {
        "metric": METRIC,
        "value": total / elapsed,
        "unit": "spectrograms/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded plasma chirps + noise + drift, generated on device)",
        "config": {"workload": "BASELINE config 2: batched specgr, 4096 shots x 65536 fp32 "
                               "samples/GPU, nperseg 1024 hop 256 hamm, linear detrend, "
                               "density, log + per-spectrogram min-max + drop Nyquist -> "
                               "4096 x 512 x 253 fp32 (STFT stage; AE stage not in this line)",
                   "shots_per_gpu": B, "samples": LENGTH, "nperseg": 1024, "hop": 256,
                   "parallelism": f"shot-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "kernel": "stft_psd_kernel<1024>", "kernel_ms": kernel_ms,
                     "alg_bytes_per_launch": ALG_BYTES * B},
        "cpu_baseline": cpu,
        "psnr_db": psnr,
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
