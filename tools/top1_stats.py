"""Rounds top1_kernel needs on the C5 stream's matrices (development build with the round
count in the flag word):
    tools/build_variant.sh t1stats svd_denoise.hip -DSPECENH_TOP1_STATS
    SPECENH_LIB=$PWD/tools/variants/libspecenh_t1stats.so python tools/top1_stats.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib, pipeline_data  # noqa: E402
from specenh.synthetic import plasma_chirps_torch  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 2048))
x = plasma_chirps_torch(B, bench.L5, seed=1000, device=dev).to(torch.float16)
S = torch.empty((B, 128, 128), dtype=torch.float32, device=dev)
pipeline_data.specgr_batch(x, bench.SPEC5, out=S)
A = torch.empty((B, 128, 128), dtype=torch.float16, device=dev)
L = _lib.lib()
m = n = r = 128
nb = int(L.specenh_svd_denoise_workspace_bytes(B, m, n, 1, 128))
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
_lib.check(L.specenh_svd_denoise_ex(ctypes.c_void_p(S.data_ptr()), B, m, n, m * n, 1, 128,
                                    ctypes.c_void_p(A.data_ptr()), 2,
                                    ctypes.c_void_p(ws.data_ptr()), None))
torch.cuda.synchronize()
off = (B * r * r + B * r + B) * 4
off = (off + 255) // 256 * 256
f = ws[off:off + 4 * B].view(torch.int32).cpu().numpy()
rounds, bad = f >> 1, f & 1
vals, cnt = np.unique(rounds, return_counts=True)
print("rounds histogram:", dict(zip(vals.tolist(), cnt.tolist())), "flagged", int(bad.sum()))
clk = ws[:64 * B].view(torch.int64).view(B, 8).double().cpu().numpy()
names = ["stage X", "U = X Z", "Y = X^T U", "reduce+cholqr", "check", "fp64 step", "output"]
tot = clk[:, :7].sum(1)
print(f"shader clocks per matrix (thread 0, mean over {B}): total {tot.mean():.0f}")
for q, nm in enumerate(names):
    print(f"  {nm:14s} {clk[:, q].mean():9.0f}  ({100 * clk[:, q].mean() / tot.mean():4.1f}%)")
