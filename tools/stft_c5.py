"""C5 STFT stage timing (HIP events): 2048 fp16 shots x 16,512 samples -> specgr 128 x 128
(hann 256 / hop 128, linear, density, log, min-max, drop Nyquist), held tiles vs the raw-rows +
re-read sweep (SPECENH_STFT_NO_HOLD), interleaved.

    python tools/stft_c5.py [shots]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib, pipeline_data  # noqa: E402
from specenh.synthetic import plasma_chirps_torch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    dev = torch.device("cuda", 0)
    x = plasma_chirps_torch(B, bench.L5, seed=3, device=dev).to(torch.float16)
    out = torch.empty((B, bench.HW5, bench.HW5), dtype=torch.float32, device=dev)
    res = {0: [], 1: []}
    for rep in range(12):
        for v in (0, 1):
            _lib.set_variant("STFT_NO_HOLD", v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                pipeline_data.specgr_batch(x, bench.SPEC5, out=out)
            e1.record()
            e1.synchronize()
            if rep >= 2:
                res[v].append(e0.elapsed_time(e1) / 5)
    alg = (bench.L5 * 2 + bench.HW5 * bench.HW5 * 4) * B
    for v, name in ((0, "held tiles"), (1, "rows + sweep")):
        ms = float(np.median(res[v]))
        print(f"{name:14s} {ms:.4f} ms  {alg / ms / 1e6:.0f} GB/s ({alg / ms / 1e6 / 8000:.3f} of HBM)")


if __name__ == "__main__":
    main()
