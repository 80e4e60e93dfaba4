"""Drop-in for the strip glue of VAE/manual_scan_3layers.py:28-54 (same copies in
manual_scan.py, hyperparam_scan.py, graphs.ipynb):

    patch(arr)    list of spectrograms (256, T >= 3840) -> (30 * len, 256, 128) float64
    unpatch(arr)  (30 * n, 256, 128) -> (n, 256, 3840) float64
    reshape(arr)  (N, 256, 128) -> (N, 256, 128, 1)

numpy in -> numpy float64 out like the reference (patchify views, ``np.empty`` float64);
the copies run on the GPU (csrc/strips.hip via ``torch.ops.specenh.strips_pack/unpack``). ``patch_batch`` / ``unpatch_batch`` are the
device fast path: fp32 spectrograms [B, F, T] -> AE input [B*30, 256, 128, 1] already in
the AE's compute dtype (bf16 or fp32), and back.
"""
from __future__ import annotations

import numpy as np
import torch


ROWS, WIDTH, N_STRIPS = 256, 128, 30
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def patch_batch(S: torch.Tensor, dtype=torch.float32, rows=ROWS, width=WIDTH,
                n_strips=N_STRIPS, out=None) -> torch.Tensor:
    """S: device fp32 [B, F, T] (row-major, each spectrogram contiguous) ->
    [B * n_strips, rows, width, 1] in ``dtype``."""
    if not isinstance(S, torch.Tensor) or S.device.type != "cuda":
        raise RuntimeError("specenh.strips runs on the GPU only (no CPU fallback)")
    if S.dim() == 2:
        S = S.unsqueeze(0)
    if S.dtype != torch.float32:
        raise TypeError("spectrograms must be float32")
    if not (S.stride(2) == 1 and S.stride(1) == S.shape[2]):
        S = S.contiguous()
    from .ops import ops
    if out is None:
        return ops.strips_pack(S, rows, width, n_strips, dtype)
    B = S.shape[0]
    if (out.dtype in (torch.float32, torch.bfloat16, torch.float16) and out.is_contiguous()
            and out.numel() == B * n_strips * rows * width and out.device == S.device):
        ops.strips_pack_out(S, rows, width, n_strips, out)  # straight into the caller's buffer
    else:  # strided / other dtype: pack, then copy_ (casts and strides as torch does)
        res = ops.strips_pack(S, rows, width, n_strips, dtype)
        out.copy_(res.view(out.shape) if out.numel() == res.numel() else res)
    return out


def unpatch_batch(strips: torch.Tensor, rows=ROWS, width=WIDTH, n_strips=N_STRIPS,
                  out=None) -> torch.Tensor:
    """strips: device [B * n_strips, rows, width(, 1)] fp32/bf16 -> fp32 [B, rows, n*width]."""
    if not isinstance(strips, torch.Tensor) or strips.device.type != "cuda":
        raise RuntimeError("specenh.strips runs on the GPU only (no CPU fallback)")
    strips = strips.contiguous()
    if strips.shape[0] % n_strips or tuple(strips.shape[1:3]) != (rows, width):
        raise ValueError(f"strips must be [k*{n_strips}, {rows}, {width}(, 1)]")
    from .ops import ops
    if out is None:
        return ops.strips_unpack(strips, rows, width, n_strips)
    ops.strips_unpack_out(strips, rows, width, n_strips, out)
    return out


def _gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("specenh requires a ROCm GPU (HIP); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def patch(arr):
    """manual_scan_3layers.py:28-36."""
    dev = _gpu()
    S = torch.stack([torch.as_tensor(np.asarray(a), dtype=torch.float32) for a in arr]).to(dev)
    return patch_batch(S)[..., 0].double().cpu().numpy()


def unpatch(arr):
    """manual_scan_3layers.py:39-50 (len(arr) // 30 spectrograms of (256, 3840))."""
    a = np.asarray(arr)
    n = (len(a) // N_STRIPS) * N_STRIPS
    t = torch.as_tensor(a[:n], dtype=torch.float32).to(_gpu())
    return unpatch_batch(t).double().cpu().numpy()


def reshape(arr):
    """manual_scan_3layers.py:53-55."""
    return np.reshape(arr, (len(arr), ROWS, WIDTH, 1))
