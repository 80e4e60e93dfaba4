"""How many C3 matrices the subspace path's convergence check sends to the fp64 eigen path
(debug: reads the per-matrix flags out of the workspace; layout of specenh_svd_denoise_ex)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib  # noqa: E402

dev = torch.device("cuda")
B = int(os.environ.get("B", 512))
A = bench.c3_matrices(dev, B)
L = _lib.lib()
m, n = 513, 256
r = 256
for name, (lo, hi, K) in {"rank16": (0, 16, 16), "default": (1, 256, 1)}.items():
    nb = int(L.specenh_svd_denoise_workspace_bytes(B, m, n, lo, hi))
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    out = torch.empty_like(A)
    _lib.check(L.specenh_svd_denoise_ex(ctypes.c_void_p(A.data_ptr()), B, m, n, m * n, lo, hi,
                                        ctypes.c_void_p(out.data_ptr()), 0,
                                        ctypes.c_void_p(ws.data_ptr()), None))
    torch.cuda.synchronize()
    off = (B * r * r + B * r * K + B * K) * 4
    off = (off + 255) // 256 * 256
    flags = ws[off:off + 8 * B].view(torch.int32)
    print(name, "flagged", int(flags[:B].sum()), "then", int(flags[B:].sum()), "of", B)
