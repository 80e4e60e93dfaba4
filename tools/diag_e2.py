import sys, os
sys.path[:0] = [os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "spectrogram-enhancement_amd")]
import numpy as np, torch
import specenh
from specenh import _lib
dev = torch.device("cuda", 0)
N, H = 1300, 128
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.rand(N, H, 128, 1, generator=g).to(dev).to(torch.float16)
w1 = (torch.randn(16*25, generator=g)*0.3).to(dev).to(torch.float16)
b1 = (torch.randn(16, generator=g)*0.2).to(dev)
w2 = (torch.randn(32*25*16, generator=g)*0.08).to(dev).to(torch.float16)
b2 = (torch.randn(32, generator=g)*0.2).to(dev)
out = torch.full((N, H//4, 32, 32), float("nan"), dtype=torch.float16, device=dev)
torch.ops.specenh.encoder2_out(x, w1, b1, 16, w2, b2, 32, 5, out)
h1 = torch.full((N, H//2, 64, 16), float("nan"), dtype=torch.float16, device=dev)
torch.ops.specenh.conv2d_out(x, w1, b1, 5, 5, 16, 1, 2, 2, 1, H, 128, 1, None, None, h1, True, None)
print("conv1 kernel", _lib.last_kernel_name())
_lib.set_variant("CONV1_NO_ROWS", 1)
h1b = torch.empty_like(h1)
torch.ops.specenh.conv2d_out(x, w1, b1, 5, 5, 16, 1, 2, 2, 1, H, 128, 1, None, None, h1b, True, None)
print("conv1 ref kernel", _lib.last_kernel_name())
d1 = (h1.float()-h1b.float()).abs().amax(dim=(1,2,3))
print("conv1 rows vs tiles: bad images", torch.nonzero(d1 > 1e-2).flatten()[:20].tolist(), float(d1.max()))
two = torch.empty_like(out)
torch.ops.specenh.conv2d_out(h1b, w2, b2, 5, 5, 32, 1, 2, 2, 1, H//2, 64, 1, None, None, two, True, None)
torch.cuda.synchronize()
d = (out.float()-two.float()).abs().amax(dim=(1,2,3))
bad = torch.nonzero(d > 1e-2).flatten()
print("enc2 vs two launches: bad images", bad[:20].tolist(), len(bad), float(d.max()))
if len(bad):
    i = int(bad[0]); dd = (out[i].float()-two[i].float()).abs()
    print("rows with error in image", i, torch.nonzero(dd.amax(dim=(1,2)) > 1e-2).flatten().tolist())
