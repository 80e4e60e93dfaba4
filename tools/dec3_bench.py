"""The C5 decoder's last three layers at the bench's launch shape (2048 x 32 x 32 x 64 fp16):
decoder3_kernel (one launch) vs the unfused engine path (convT2 conv_patch launch + the
row-sweep tail), interleaved rounds in one process, HIP events.  python tools/dec3_bench.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]


def main():
    import numpy as np
    import torch

    import bench
    from specenh import _lib, ae
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    dev = torch.device("cuda")
    ops_ = bench.ae_ops()[-3:]
    w = bench.ae_weights()[-6:]
    engs = {}
    for v in (0, 1):
        _lib.set_variant("DECODER_UNFUSED", v)
        e = ae.AutoencoderEngine(ops_, (32, 32, 64), compute_dtype="float16", device=dev)
        e.set_keras_weights(w)
        engs[v] = e
    _lib.set_variant("DECODER_UNFUSED", 0)
    x = (torch.rand(N, 32, 32, 64, device=dev) * 0.5).half()
    res = {0: [], 1: []}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(6):
        for v in (0, 1):
            engs[v].forward(x)
            e0.record()
            for _ in range(10):
                engs[v].forward(x)
            e1.record()
            e1.synchronize()
            if rnd:
                res[v].append(e0.elapsed_time(e1) / 10)
    d = (engs[0].forward(x) - engs[1].forward(x)).abs().max().item()
    for v, name in ((0, "decoder3"), (1, "unfused")):
        print(f"{name:9s} N={N}: median {np.median(res[v]):.4f} ms  min {min(res[v]):.4f}", flush=True)
    print(f"max |fused - unfused| = {d:.2e}")


if __name__ == "__main__":
    main()
