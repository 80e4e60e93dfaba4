"""Time the fused decoder tail (torch.ops.specenh.convt_conv_out) at the C5 shape, with
development variants (SPECENH_TAIL_DEV bits: 1 no MFMA items, 2 no Conv2D(1), 4 no staging)
and the two-launch path, to see where the kernel's time goes.  python tools/tail_bench.py"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]


def run():
    import torch
    import specenh  # noqa: F401
    ops = torch.ops.specenh
    N = int(os.environ.get("TAIL_N", "2048"))
    dev = torch.device("cuda")
    x = torch.rand(N, 64, 64, 32, device=dev).half()
    wt = (0.05 * torch.randn(16 * 25 * 32, device=dev)).half()
    bt = 0.1 * torch.randn(16, device=dev)
    wo = (0.1 * torch.randn(25 * 16, device=dev)).half()
    bo = torch.zeros(1, device=dev)
    out = torch.empty(N, 128, 128, 1, device=dev)
    for _ in range(3):
        ops.convt_conv_out_out(x, wt, bt, 16, 5, wo, bo, 5, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.convt_conv_out_out(x, wt, bt, 16, 5, wo, bo, 5, out)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / 10


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        print(f"{run():.4f}")
        sys.exit(0)
    for d in ["0", "1", "2", "3", "4", "7"]:
        env = dict(os.environ, SPECENH_TAIL_DEV=d)
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True,
                           text=True, timeout=300)
        print(f"dev={d}: {r.stdout.strip()} ms  {r.stderr.strip()[-200:] if r.returncode else ''}",
              flush=True)
