import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "spectrogram-enhancement_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np, torch
from specenh import _lib, ae
from test_decoder_tail_gpu import _dec3_model
for dmap in (0, 1):
    for lead in (0, 1):
        _lib.set_variant("D3_MAP", dmap); _lib.set_variant("ROWS_SHORT_LEAD", lead)
        eng, ops_, ws = _dec3_model("float16", (32, 32), seed=7)
        x = np.random.default_rng(5).uniform(0, 1, (3, 32, 32, 1)).astype(np.float32)
        xd = eng.to_compute(torch.from_numpy(x))
        f = eng.forward(xd).clone()
        _lib.set_variant("DECODER_UNFUSED", 1)
        pe = ae.AutoencoderEngine(ops_, (32, 32, 1), compute_dtype="float16", device="cuda")
        pe.set_keras_weights(ws)
        p = pe.forward(xd).clone()
        _lib.set_variant("DECODER_UNFUSED", 0)
        torch.cuda.synchronize()
        d = (f - p).abs()[..., 0]
        print(f"map={dmap} short_lead={lead}: max {d.max().item():.3e}", flush=True)
        if d.max() > 4e-3:
            bad = (d > 4e-3)
            rows = bad.any(2)[0].nonzero().flatten().tolist()
            cols = bad.any(1)[0].nonzero().flatten().tolist()
            print("  image0 bad rows", rows[:40], "n", len(rows))
            print("  image0 bad cols", cols[:40], "n", len(cols))
            print("  per-image max", d.amax((1, 2)).tolist())
            print("  fused row 0 cols 0..8", f[0, 0, :8, 0].tolist())
            print("  plain row 0 cols 0..8", p[0, 0, :8, 0].tolist())
            print("  fused row 10 cols 30..36", f[0, 10, 30:36, 0].tolist())
            print("  plain row 10 cols 30..36", p[0, 10, 30:36, 0].tolist())
