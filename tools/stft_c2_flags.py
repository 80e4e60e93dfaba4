"""Time the C2 team STFT kernel under development flags (attribution of its time).
    python tools/stft_c2_flags.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch  # noqa: E402
from specenh import stft  # noqa: E402
from specenh.synthetic import plasma_chirps_torch  # noqa: E402

B = 4096
x = plasma_chirps_torch(B, 65536, seed=1, device="cuda")
plan = stft.get_plan(x.device, 1024, 768, "hamm", 500000.0, "density", "linear", 1e-11)
out = torch.empty((B, 512, 253), device="cuda")
NOSTORE, NOTEAM, NOWAIT, NOLOAD = 1 << 16, 1 << 17, 1 << 20, 1 << 21


def timed(flags, reps=10):
    for _ in range(2):
        stft._launch(plan, x, out, flags)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        stft._launch(plan, x, out, flags)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for name, fl in (("team", 7), ("team_nostore", 7 | NOSTORE), ("team_nowait", 7 | NOWAIT),
                 ("team_nostore_nowait", 7 | NOSTORE | NOWAIT), ("sweep", 7 | NOTEAM),
                 ("psd_nonorm_nostore", 5 | NOSTORE | NOTEAM), ("psd_nonorm", 5 | NOTEAM),
                 ("team_nonorm", 5), ("team_noload", 7 | NOLOAD),
                 ("team_noload_nostore_nowait", 7 | NOLOAD | NOSTORE | NOWAIT)):
    print(f"{name:22s} {timed(fl):.4f} ms", flush=True)
