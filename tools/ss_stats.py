"""Per-phase shader clocks of subspace_kernel on BASELINE C3's matrices (development build):
    tools/build_variant.sh ssstats svd_denoise.hip -DSPECENH_SS_STATS
    SPECENH_LIB=$PWD/tools/variants/libspecenh_ssstats.so python tools/ss_stats.py
Thread 0's clocks per phase, written over each matrix's (dead) Gram by that build."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 4096))
m, n = 513, 256
A = bench.c3_matrices(dev, B, m, n, 16)
out = torch.empty_like(A)
L = _lib.lib()
names = ["G Z (first)", "CholeskyQR", "G Z", "Rayleigh-Ritz", "Jacobi+sort", "check", "V out"]
for lo, hi in [(0, 16), (1, 256)]:
    nb = int(L.specenh_svd_denoise_workspace_bytes(B, m, n, lo, hi))
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    for _ in range(2):
        _lib.check(L.specenh_svd_denoise_ex(ctypes.c_void_p(A.data_ptr()), B, m, n, m * n, lo, hi,
                                            ctypes.c_void_p(out.data_ptr()), 0,
                                            ctypes.c_void_p(ws.data_ptr()), None))
    torch.cuda.synchronize()
    clk = ws[:B * n * n * 4].view(torch.int64).view(B, n * n // 2)[:, :11].double().cpu()
    tot = clk[:, :7].sum(1)
    print(f"[{lo}, {hi}): shader clocks per matrix (thread 0, mean over {B}): total "
          f"{tot.mean():.0f}, Jacobi sweeps mean {clk[:, 7].mean():.2f} max {clk[:, 7].max():.0f}")
    for q, nm in enumerate(names):
        print(f"  {nm:14s} {clk[:, q].mean():10.0f}  ({100 * clk[:, q].mean() / tot.mean():4.1f}%)")
    for q, nm in zip(range(8, 11), ["  Gram Y^T Y", "  Cholesky", "  Z = Y R^-1"]):
        print(f"  {nm:14s} {clk[:, q].mean():10.0f}  (of CholeskyQR, thread 0)")
