"""Run the C2 STFT kernel a few times (workload for rocprofv3 PMC passes)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch
from specenh import stft
from specenh.synthetic import plasma_chirps_torch
B = int(os.environ.get("B", 4096))
x = plasma_chirps_torch(B, 65536, seed=1, device="cuda")
out = torch.empty((B, 512, 253), device="cuda")
for _ in range(int(os.environ.get("REPS", 3))):
    stft.stft_psd(x, 1024, 768, "hamm", 500000.0, log=True, drop_nyquist=True, out=out)
torch.cuda.synchronize()
