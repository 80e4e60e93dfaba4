"""Dev timing experiments for the STFT kernel (variants via env knobs / dev flags)."""
import os, sys, json, subprocess
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch
from specenh import stft, _lib
from specenh.synthetic import plasma_chirps_torch

B, L = int(os.environ.get("B", 4096)), 65536
x = plasma_chirps_torch(B, L, seed=1, device="cuda")
T = (L - 1024) // 256 + 1
out = torch.empty((B, 513, T), device="cuda")
plan = stft.get_plan(x.device, 1024, 768, "hamm", 500000.0, "density", "linear", 1e-11)
def run(flags):
    stft._launch(plan, x, out[:, :, :] if not flags & 4 else out[:, :512, :].contiguous(), flags)
def timeit(flags, reps=10):
    for _ in range(2): stft._launch(plan, x, out, flags)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): stft._launch(plan, x, out, flags)
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / reps
res = {}
for name, flags in [("log", 1), ("log_nostore", 1 | (1 << 16)), ("norm", 2 | 0), ("psd", 0)]:
    res[name] = timeit(flags)
print(os.environ.get("SPECENH_DEV_TPW", "auto"), json.dumps(res))
