"""C5 host-stream stage (bench.c5_host_stream_stage) at several (chunk, slots) settings on one
box, interleaved, to pick the default:  python tools/host_stream_ab.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for rnd in range(2):
    for chunk, slots in [(2048, 4), (1024, 8), (2048, 6), (4096, 3)]:
        r = bench.c5_host_stream_stage(dev, lambda: bench.make_c5_engine(dev), chunk=chunk,
                                       slots=slots)
        print(json.dumps({"round": rnd, "chunk": chunk, "slots": slots,
                          "spectrograms_per_s": round(r["spectrograms_per_s"]),
                          "frac_of_copy_ceiling": round(r["frac_of_copy_ceiling"], 3),
                          "copy_only_GBps": {k: round(v, 1) for k, v in r["copy_only_GBps"].items()}}),
              flush=True)
