"""Batch-size diagnostic (GPU): the C5 chain over B shots in one launch vs the same shots in
small launches. Shots are independent, so every intermediate must agree; prints the
per-stage max relative difference (the first stage that disagrees is the culprit)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "spectrogram-enhancement_amd")]
import bench  # noqa: E402
from specenh import ae, pipeline_data, svd  # noqa: E402
from specenh.synthetic import plasma_chirps_torch  # noqa: E402


def engine(dev, tail=True):
    ops = []
    for lay in bench.ae_layers():
        ops.append(ae.PoolOp() if lay[0] == "pool" else
                   ae.ConvOp(lay[0], lay[1], lay[2], lay[3], lay[4],
                             stride=2 if lay[0] == "convT" else 1))
    e = ae.AutoencoderEngine(ops, (128, 128, 1), compute_dtype="float16", device=dev)
    e.set_keras_weights(bench.ae_weights())
    if not tail:
        e.tail = False
    return e


def inter(e, N):
    b = e._buffers(N, False)
    return [h.clone() if h is not None else None for h in b["h"][1:]]


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    small = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    x = plasma_chirps_torch(B, bench.L5, seed=1000, device=dev).to(torch.float16)
    S = torch.empty((B, 128, 128), dtype=torch.float32, device=dev)
    A = torch.empty((B, 128, 128, 1), dtype=torch.float16, device=dev)
    pipeline_data.specgr_batch(x, bench.SPEC5, out=S)
    svd.denoise_batch(S, out=A.view(B, 128, 128))
    S2, A2 = torch.empty_like(S), torch.empty_like(A)
    for i in range(0, B, small):
        sl = slice(i, i + small)
        pipeline_data.specgr_batch(x[sl], bench.SPEC5, out=S2[sl])
        svd.denoise_batch(S2[sl], out=A2[sl].view(-1, 128, 128))
    torch.cuda.synchronize()
    print(f"stft  rel {rel(S, S2):.3e}   svd rel {rel(A, A2):.3e}")
    for tail in (True, False):
        eb, es = engine(dev, tail), engine(dev, tail)
        yb = eb.forward(A).clone()
        hb = inter(eb, B)
        hs = [None if h is None else torch.empty_like(h) for h in hb]
        ys = torch.empty_like(yb)
        for i in range(0, B, small):
            sl = slice(i, i + small)
            ys[sl] = es.forward(A[sl].contiguous())
            for j, h in enumerate(inter(es, A[sl].shape[0])):
                if h is not None and hs[j] is not None:
                    hs[j][sl] = h
        torch.cuda.synchronize()
        # conv2 + relu + pool in fp32 torch from the (agreeing) conv1+pool output
        w = bench.ae_weights()
        k2 = torch.as_tensor(w[2], device=dev).permute(3, 2, 0, 1).float()
        b2 = torch.as_tensor(w[3], device=dev).float()
        for tag, hh in (("big", hb), ("small", hs)):
            xin = hh[1][:4].float().permute(0, 3, 1, 2)
            r = torch.nn.functional.max_pool2d(torch.relu(
                torch.nn.functional.conv2d(xin, k2, b2, padding=2)), 2).permute(0, 2, 3, 1)
            got = hh[3][:4].float()
            print(f"   {tag}: conv2+pool vs torch rel {rel(got, r):.3e}; finite "
                  f"{bool(torch.isfinite(got).all())}; max|got| {float(got.abs().max()):.3e} "
                  f"max|ref| {float(r.abs().max()):.3e}")
        names = []
        for j, (a, b) in enumerate(zip(hb, hs)):
            if a is not None and b is not None:
                d = (a.double() - b.double()).flatten(1).norm(dim=1) / \
                    b.double().flatten(1).norm(dim=1).clamp_min(1e-30)
                bad = int((d > 1e-3).sum())
                names.append(f"h{j + 1} max {float(d.max()):.2e} bad {bad} first "
                             f"{int(torch.nonzero(d > 1e-3)[0]) if bad else -1}")
        d = (yb.double() - ys.double()).flatten(1).norm(dim=1) / ys.double().flatten(1).norm(dim=1)
        print(f"tail={tail}: out max rel {float(d.max()):.3e}, bad shots {int((d > 1e-3).sum())}")
        for n in names:
            print("   ", n)


if __name__ == "__main__":
    main()
