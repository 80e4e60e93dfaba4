"""Per-wave barrier clocks of decoder3_kernel at the C5 launch shape (development build):
    tools/build_variant.sh d3stats decoder_tail.hip -DSPECENH_D3_STATS
    SPECENH_LIB=$PWD/tools/variants/libspecenh_d3stats.so python tools/d3_stats.py [N]
busy = shader clocks from leaving one macro-step barrier to arriving at the next (the wave's
own work and waits), wait = clocks parked in s_barrier. Waves 0-3 produce, 4-7 consume."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from specenh import _lib, ae  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda", 0)
e = ae.AutoencoderEngine(bench.ae_ops()[-3:], (32, 32, 64), compute_dtype="float16", device=dev)
e.set_keras_weights(bench.ae_weights()[-6:])
x = (torch.rand(N, 32, 32, 64, device=dev) * 0.5).half()
for _ in range(3):
    e.forward(x)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(10):
    e.forward(x)
ev[1].record()
ev[1].synchronize()
print(f"decoder3 N={N}: {ev[0].elapsed_time(ev[1]) / 10:.4f} ms per launch (stats build)")
L = _lib.lib()
buf = (ctypes.c_ulonglong * (1024 * 8 * 4))()
assert L.specenh_d3_stats(buf, ctypes.sizeof(buf)) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8, 4).astype(np.float64)
G = min(N, 256)
st = st[:G]
n = st[:, :, 2]
busy = st[:, :, 0] / np.maximum(n - 1, 1)
wait = st[:, :, 1] / np.maximum(n, 1)
for w in range(8):
    role = "producer" if w < 4 else "consumer"
    print(f"wave {w} ({role}): steps {n[:, w].mean():.0f}  busy/step {busy[:, w].mean():7.0f}  "
          f"wait/step {wait[:, w].mean():7.0f}  (min busy {busy[:, w].min():.0f}, "
          f"max {busy[:, w].max():.0f})")
tot = busy + wait
print(f"step period (clocks): {tot.mean():.0f}; producer busy share {busy[:, :4].mean() / tot.mean():.2f}, "
      f"consumer busy share {busy[:, 4:].mean() / tot.mean():.2f}")
