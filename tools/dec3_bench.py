"""The C5 decoder's last three layers at the bench's launch shape (2048 x 32 x 32 x 64 fp16):
decoder3_kernel map-free (default) vs its round-3 map-ring consumer (D3_MAP=1) vs the unfused
engine path (convT2 conv_patch launch + the row-sweep tail), interleaved rounds in one
process, HIP events.  python tools/dec3_bench.py [N] [arm,arm...]  (D3_OUT16=1: fp16 output)"""
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
        if v == 0 and os.environ.get("D3_OUT16"):  # the bench's fp16 reconstructions
            e.set_inference_output_dtype(torch.float16)
        engs[v] = e
    _lib.set_variant("DECODER_UNFUSED", 0)
    arms = {"mapfree": (engs[0], 0), "map": (engs[0], 1), "unfused": (engs[1], 0)}
    if len(sys.argv) > 2:
        arms = {k: v for k, v in arms.items() if k in sys.argv[2].split(",")}
    x = (torch.rand(N, 32, 32, 64, device=dev) * 0.5).half()
    res = {k: [] for k in arms}
    outs = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(6):
        for name, (eng, mp) in arms.items():
            _lib.set_variant("D3_MAP", mp)
            outs[name] = eng.forward(x).clone()
            e0.record()
            for _ in range(10):
                eng.forward(x)
            e1.record()
            e1.synchronize()
            if rnd:
                res[name].append(e0.elapsed_time(e1) / 10)
    _lib.set_variant("D3_MAP", 0)
    flop = 2.0 * N * (32 * 32 * 25 * 64 * 32 + 64 * 64 * 25 * 32 * 16 + 128 * 128 * 25 * 16)
    for name in arms:
        med = float(np.median(res[name]))
        print(f"{name:8s} N={N}: median {med:.4f} ms  min {min(res[name]):.4f}  "
              f"({flop / med / 1e9:.0f} TF/s = {flop / med / 1e9 / 2500:.3f} of 2.5 PF)", flush=True)
    for name in ("map", "unfused"):
        if name not in outs or "mapfree" not in outs:
            continue
        d = (outs["mapfree"] - outs[name]).abs().max().item()
        print(f"max |mapfree - {name}| = {d:.2e}")


if __name__ == "__main__":
    main()
