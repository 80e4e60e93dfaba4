"""Time BASELINE config 3 (4096 x 513 x 256 fp32, rank-16 / default) on the GPU."""
import os, sys, time, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import torch
from specenh import svd
B = int(os.environ.get("B", 4096))
g = torch.Generator(device="cuda"); g.manual_seed(0)
A = torch.randn((B, 513, 256), device="cuda", generator=g)
out = torch.empty_like(A)
res = {}
for name, (s0, s1) in {"rank16": (0, 16), "default": (None, None)}.items():
    for _ in range(2): svd.denoise_batch(A, s0, s1, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(5): svd.denoise_batch(A, s0, s1, out=out)
    e1.record(); e1.synchronize()
    res[name] = e0.elapsed_time(e1) / 5
print(json.dumps(res))
