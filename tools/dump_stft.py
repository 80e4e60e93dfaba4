"""Debug helper: dump GPU STFT outputs for golden cases to gpurun_out/ for offline analysis."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd"), os.path.join(REPO, "tests")]
import torch
from conftest import golden_params, golden_signal, load_golden
from specenh import stft, pipeline_data

out = {}
for case in sys.argv[1:]:
    g = load_golden(f"stft_{case}")
    x = golden_signal(g).astype(np.float32)
    p = golden_params(g)
    xt = torch.as_tensor(x, device="cuda").unsqueeze(0)
    kw = dict(nperseg=p["nperseg"], noverlap=p["noverlap"], window=p["window"], fs=p["fs"],
              scaling=p["scaling"], detrend=p["detrend"], eps=p["eps"])
    out[case + "_psd"] = stft.stft_psd(xt, **kw)[0].cpu().numpy()
    out[case + "_log"] = stft.stft_psd(xt, log=True, **kw)[0].cpu().numpy()
    out[case + "_S"] = pipeline_data.specgr_batch(xt, p)[0].cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dump_stft.npz", **out)
print("dumped", list(out))
