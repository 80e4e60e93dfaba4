"""Run the C2 STFT kernel a few times (workload for rocprofv3 PMC passes).
FLAGS env: C-ABI flags (default 7 = log|normalize|drop); 65537 = log + dev no-store."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch
from specenh import stft
from specenh.synthetic import plasma_chirps_torch
B = int(os.environ.get("B", 4096))
flags = int(os.environ.get("FLAGS", 7))
x = plasma_chirps_torch(B, 65536, seed=1, device="cuda")
out = torch.empty((B, 513, 253), device="cuda")
plan = stft.get_plan(x.device, 1024, 768, "hamm", 500000.0, "density", "linear", 1e-11)
for _ in range(int(os.environ.get("REPS", 3))):
    stft._launch(plan, x, out, flags)
torch.cuda.synchronize()
