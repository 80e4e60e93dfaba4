"""Where the fp32 STFT's largest errors sit on the reference production shot (1,000,000
samples, hamm 512 / hop 256 -> 256 x 3905): the error map of specgr_batch vs the fp64
oracle, its argmax, and the contribution of the min/max normalisation (the truth's argmin /
argmax bins).  python tools/diag_prodshot.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import spectrogram as ref  # noqa: E402
from specenh import pipeline_data, stft  # noqa: E402
from specenh.synthetic import plasma_chirps  # noqa: E402

SPEC = {"nperseg": 512, "noverlap": 256, "fs": 500000, "window": "hamm", "scaling": "density",
        "detrend": "linear", "eps": 1e-11}
shots = plasma_chirps(3, 1_200_000, seed0=11, dtype=np.float32)
x = torch.as_tensor(shots, device="cuda")
S = pipeline_data.specgr_batch(x, SPEC, cut_shot=2).double().cpu().numpy()
P = stft.stft_psd(x[:, :1_000_000].contiguous(), 512, 256, "hamm", 500000, "density", "linear",
                  1e-11).double().cpu().numpy()
for c in range(3):
    xc = shots[c][:1_000_000].astype(np.float64)
    St, _, _ = ref.specgr_arrays(xc, SPEC)
    _, _, Pt = ref.spectrogram_psd(xc, fs=500000, window="hamm", nperseg=512, noverlap=256,
                                   detrend="linear", scaling="density")
    e = np.abs(S[c] - St)
    i = np.unravel_index(np.argmax(e), e.shape)
    Lt = np.log(Pt + 1e-11)[:-1]
    Lg = np.log(P[c] + 1e-11)[:-1]
    imn = np.unravel_index(np.argmin(Lt), Lt.shape)
    imx = np.unravel_index(np.argmax(Lt), Lt.shape)
    dl = Lg - Lt
    print(f"ch {c}: max err {e.max():.3e} at {i} (S {St[i]:.4f}); p99.99 {np.quantile(e, 0.9999):.2e}; "
          f"DC-row max {e[0].max():.2e}, other rows {e[1:].max():.2e}", flush=True)
    print(f"   ln-PSD err at truth argmin {imn}: {dl[imn]:+.3e} (min {Lt[imn]:.3f}), at argmax {imx}: "
          f"{dl[imx]:+.3e}; range {Lt.max() - Lt.min():.3f}; max |ln err| {np.abs(dl).max():.3e} at "
          f"{np.unravel_index(np.argmax(np.abs(dl)), dl.shape)}", flush=True)
