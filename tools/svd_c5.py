"""The C5 stream's SVD stage alone (GPU): denoiseSignal default on B spectrograms of the C5
chain (128 x 128), fp16 output; prints the convergence-flag counts of the two subspace
passes and the HIP-event time per call. Run under rocprofv3 --kernel-trace --stats for the
per-kernel split."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib, pipeline_data, svd  # noqa: E402
from specenh.synthetic import plasma_chirps_torch  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 2048))
x = plasma_chirps_torch(B, bench.L5, seed=1000, device=dev).to(torch.float16)
S = torch.empty((B, 128, 128), dtype=torch.float32, device=dev)
pipeline_data.specgr_batch(x, bench.SPEC5, out=S)
A = torch.empty((B, 128, 128), dtype=torch.float16, device=dev)
L = _lib.lib()
m = n = r = 128
lo, hi, K = 1, 128, 1
nb = int(L.specenh_svd_denoise_workspace_bytes(B, m, n, lo, hi))
ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
_lib.check(L.specenh_svd_denoise_ex(ctypes.c_void_p(S.data_ptr()), B, m, n, m * n, lo, hi,
                                    ctypes.c_void_p(A.data_ptr()), 2,
                                    ctypes.c_void_p(ws.data_ptr()), None))
torch.cuda.synchronize()
off = (B * r * r + B * r * K + B * K) * 4
off = (off + 255) // 256 * 256
flags = ws[off:off + 8 * B].view(torch.int32)
print("flagged (top1_kernel, or the first subspace pass)", int(flags[:B].sum()), "of", B)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {}
for rnd in range(4):
    for v in (0, 1):  # SVD_NO_TOP1: one-pass top1_kernel vs Gram + subspace + recon
        _lib.set_variant("SVD_NO_TOP1", v)
        svd.denoise_batch(S, out=A)
        e0.record()
        for _ in range(10):
            svd.denoise_batch(S, out=A)
        e1.record()
        e1.synchronize()
        if rnd:
            res.setdefault(v, []).append(e0.elapsed_time(e1) / 10)
for v, name in ((0, "top1"), (1, "pipeline")):
    print(f"denoise_batch {B} x 128 x 128 -> fp16 [{name}]: {min(res[v]):.4f} ms "
          f"(rounds {', '.join(f'{t:.4f}' for t in res[v])})")
_lib.set_variant("SVD_NO_TOP1", 0)
