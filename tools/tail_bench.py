"""Time the fused decoder tail (torch.ops.specenh.convt_conv_out) at the C5 launch shape:
the row-sweep kernel vs the 2-D tile kernel (kernel variant TAIL_TILES), interleaved
rounds in one process (HIP events, median of rounds).   python tools/tail_bench.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]


def main():
    import numpy as np
    import torch

    from specenh import _lib
    ops = torch.ops.specenh
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    dev = torch.device("cuda")
    x = torch.rand(N, 64, 64, 32, device=dev).half()
    wt = (0.05 * torch.randn(16 * 25 * 32, device=dev)).half()
    bt = 0.1 * torch.randn(16, device=dev)
    wo = (0.1 * torch.randn(25 * 16, device=dev)).half()
    bo = torch.zeros(1, device=dev)
    out = torch.empty(N, 128, 128, 1, device=dev)
    res = {0: [], 1: []}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(6):
        for v in (0, 1):
            _lib.set_variant("TAIL_TILES", v)
            ops.convt_conv_out_out(x, wt, bt, 16, 5, wo, bo, 5, out)
            e0.record()
            for _ in range(10):
                ops.convt_conv_out_out(x, wt, bt, 16, 5, wo, bo, 5, out)
            e1.record()
            e1.synchronize()
            if rnd:
                res[v].append(e0.elapsed_time(e1) / 10)
    for v, name in ((0, "rows"), (1, "tiles")):
        _lib.set_variant("TAIL_TILES", v)
        ops.convt_conv_out_out(x, wt, bt, 16, 5, wo, bo, 5, out)
        print(f"{name:6s} N={N}: median {np.median(res[v]):.4f} ms  min {min(res[v]):.4f}  "
              f"{_lib.last_kernel_name()}", flush=True)


if __name__ == "__main__":
    main()
