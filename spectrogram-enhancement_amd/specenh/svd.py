"""Drop-in for the SVD denoiser of spec_denoising/denoising_by_svd.ipynb (cell 1).

    from specenh.svd import omega, denoiseSignal, computeSignal
    svd = denoiseSignal(s)                       # denoising_by_svd.ipynb:263

Same names, arguments and semantics as the notebook (:155-229):
  * ``omega(beta)``          Gavish-Donoho polynomial (host scalar, as in the notebook)
  * ``denoiseSignal(matrix, start=None, stop=None, use_optimal=False)``
        keep singular components u[:, start:stop] — defaults start=1, stop=r; clamps
        start<0 -> 0 and stop>r -> r, then Python slicing (a negative stop counts from
        the end; an empty slice gives zeros).
  * ``denoise_batch(A[B, m, n], start, stop)`` — device tensors in/out (fast path).

  * ``computeSignal(matrix)``  components [1, 2*num_sing) (:161-186), IndexError when
        2*num_sing > min(m, n) like the notebook
  * ``optimal_batch(A[B, m, n], mode)`` — use_optimal / computeSignal on device tensors.

The arithmetic runs on the GPU (csrc/svd_denoise.hip, reached through
``torch.ops.specenh.svd_denoise_out`` / ``svd_denoise_optimal`` and the C-ABI): fp32-MFMA
Gram matrix, top-K subspace iteration with fp64 CholeskyQR2 + Rayleigh-Ritz,
reconstruction ``A V V^T``; wide or bottom-of-spectrum ranges and the optimal threshold use
fp64 eigenvectors of the Gram matrix (Householder tridiagonalisation, Sturm bisection,
inverse iteration). numpy inputs come back as float64 numpy arrays like the reference.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def omega(beta):
    """denoising_by_svd.ipynb:155-159 (http://www.pyrunner.com/weblog/2016/08/01/optimal-svht/)."""
    coef = [0.56, -0.95, 1.82, 1.43]
    poly = [beta ** (3 - n) for n in range(4)]
    return sum(c * p for c, p in zip(coef, poly))


def _resolve(r: int, start, stop):
    """denoising_by_svd.ipynb:219-227 (non-optimal branch): defaults and clamping. The
    slice itself (negative stop, empty ranges) is resolved by the C-ABI like Python does."""
    if start is None:
        start = 1
    if stop is None:
        stop = r
    start = int(start)
    stop = int(stop)
    if start < 0:
        start = 0
    if stop > r:
        stop = r
    return start, stop


_OUT_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}  # SPECENH_DTYPE_*


def denoise_batch(A: torch.Tensor, start=None, stop=None,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Batched denoiseSignal on device tensors: ``A[B, m, n]`` (or ``[m, n]``) fp32."""
    if not isinstance(A, torch.Tensor) or A.device.type != "cuda":
        raise RuntimeError("specenh.svd.denoise_batch runs on the GPU only (no CPU fallback)")
    squeeze = A.dim() == 2
    if squeeze:
        A = A.unsqueeze(0)
    if A.dim() != 3:
        raise ValueError("A must be [batch, m, n]")
    if A.dtype != torch.float32:
        A = A.float()
    if not (A.stride(2) == 1 and A.stride(1) == A.shape[2]):
        A = A.contiguous()
    B, m, n = A.shape
    r = min(m, n)
    start, stop = _resolve(r, start, stop)
    if out is None:
        out = torch.empty((B, m, n), dtype=torch.float32, device=A.device)
    # out may be fp16/bf16 (e.g. the autoencoder's input): the reconstruction stores in that
    # type directly (specenh_svd_denoise_ex), no separate cast pass
    odt = _OUT_DTYPES.get(out.dtype)
    if odt is None or out.numel() != B * m * n or not out.is_contiguous() or out.device != A.device:
        raise ValueError("out must be a contiguous [B, m, n] float32/bfloat16/float16 tensor "
                         "on A's device")
    from .ops import ops
    ops.svd_denoise_out(A, start, stop, out.view(B, m, n))
    return out[0] if squeeze else out


def optimal_batch(A: torch.Tensor, mode: int = _lib.SVD_OPTIMAL, out: torch.Tensor | None = None,
                  return_rank: bool = False):
    """Optimal hard-threshold modes on device tensors ``A[B, m, n]`` (or ``[m, n]``) fp32:
    ``mode`` SVD_OPTIMAL = denoiseSignal(use_optimal=True), SVD_COMPUTE = computeSignal.
    With ``return_rank`` also returns (num_sing int32[B], median singular value f64[B])."""
    if not isinstance(A, torch.Tensor) or A.device.type != "cuda":
        raise RuntimeError("specenh.svd.optimal_batch runs on the GPU only (no CPU fallback)")
    squeeze = A.dim() == 2
    if squeeze:
        A = A.unsqueeze(0)
    if A.dim() != 3:
        raise ValueError("A must be [batch, m, n]")
    if A.dtype != torch.float32:
        A = A.float()
    if not (A.stride(2) == 1 and A.stride(1) == A.shape[2]):
        A = A.contiguous()
    B, m, n = A.shape
    from .ops import ops
    if out is None:
        out, ns, med = ops.svd_denoise_optimal(A, int(mode))
    elif (out.dtype == torch.float32 and out.is_contiguous() and out.numel() == B * m * n
          and out.device == A.device):  # straight into the caller's buffer
        ns = torch.empty(B, dtype=torch.int32, device=A.device)
        med = torch.empty(B, dtype=torch.float64, device=A.device)
        ops.svd_denoise_optimal_out(A, int(mode), out.view(B, m, n), ns, med)
    else:  # strided / other dtype: compute, then copy_ (casts and strides as torch does)
        res, ns, med = ops.svd_denoise_optimal(A, int(mode))
        out.copy_(res.view(out.shape) if out.shape != res.shape and out.numel() == res.numel()
                  else res)
    res = out[0] if squeeze else out
    return (res, ns, med) if return_rank else res


def _host(matrix, fn):
    if isinstance(matrix, torch.Tensor):
        return fn(matrix)
    a = np.asarray(matrix)
    if not torch.cuda.is_available():
        raise RuntimeError("specenh requires a ROCm GPU (HIP); there is no CPU fallback")
    t = torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda")
    return fn(t).double().cpu().numpy()


def denoiseSignal(matrix, start=None, stop=None, use_optimal=False):
    """denoising_by_svd.ipynb:188-229."""
    if use_optimal:  # :210-217 (start/stop are overridden, as in the notebook)
        return _host(matrix, lambda t: optimal_batch(t, _lib.SVD_OPTIMAL))
    return _host(matrix, lambda t: denoise_batch(t, start, stop))


def computeSignal(matrix):
    """denoising_by_svd.ipynb:161-186: components [1, 2*num_sing) of the optimal threshold
    (IndexError when 2*num_sing > min(m, n), as the notebook's s[idx])."""
    return _host(matrix, lambda t: optimal_batch(t, _lib.SVD_COMPUTE))
