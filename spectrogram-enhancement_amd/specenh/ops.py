"""``torch.ops.specenh.*``: every entry point of the C-ABI (include/specenh.h) as a PyTorch
operator.

The Python API that keeps the reference's names (``pipeline_data``, ``svd``, ``keras``,
``strips``, ``cross``, ``filters``) reaches the HIP kernels only through these operators:

    reference call site -> specenh.<module> -> torch.ops.specenh.<op> -> C-ABI -> HIP

Each operator is defined with an explicit schema on a ``torch.library.Library`` (its
dispatch costs ~2.5 us a call, a sixth of ``torch.library.custom_op``'s), implemented for
the CUDA (= HIP on ROCm) dispatch key only — a CPU tensor raises NotImplementedError, there
is no fallback — and has a fake (meta) kernel, so shapes propagate through FakeTensor /
``torch.compile`` tracing. Operators ending in ``_out`` write caller-owned buffers (the
autoencoder engine reuses its activations across calls); the others allocate.
``tests/test_ops_gpu.py`` runs ``torch.library.opcheck`` on each.

Every launch goes on the current HIP stream of the tensors' device.
"""
from __future__ import annotations

import ctypes
import hashlib
import threading

import numpy as np
import torch

from . import _lib

F32, BF16, F16, F64 = 0, 1, 2, 3
_CODE = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16, torch.float64: F64}


def _vp(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _st(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _code(t: torch.Tensor, allowed=(F32, BF16, F16)) -> int:
    c = _CODE.get(t.dtype)
    if c is None or c not in allowed:
        raise TypeError(f"unsupported dtype {t.dtype}")
    return c


def _need(t: torch.Tensor, name: str):
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_LIB = torch.library.Library("specenh", "DEF")


def _op(schema: str, impl, fake):
    name = schema.split("(", 1)[0]
    _LIB.define(schema)
    _LIB.impl(name, impl, "CUDA")
    torch.library.register_fake(f"specenh::{name}", fake, lib=_LIB)


# ---------------------------------------------------------------- windows / plans
_windows: dict = {}
_wlock = threading.Lock()


def window_key(window, nperseg: int) -> str:
    """A string naming a window for the STFT / CSD operators: scipy window names pass
    through; tuples and coefficient arrays are registered under their sha1 digest."""
    if isinstance(window, str):
        return window
    from .stft import get_window
    w = np.ascontiguousarray(get_window(window, int(nperseg)), dtype=np.float64)
    key = "sha1:" + hashlib.sha1(w.tobytes()).hexdigest()
    with _wlock:
        _windows.setdefault(key, w)
    return key


def window_coefs(key: str, nperseg: int) -> np.ndarray:
    if key.startswith("sha1:"):
        w = _windows.get(key)
        if w is None or w.shape[0] != nperseg:
            raise ValueError(f"unknown window {key!r} (register it with ops.window_key)")
        return w
    from .stft import get_window
    return get_window(key, int(nperseg))


# ---------------------------------------------------------------- STFT-PSD
def _stft_shape(x, nperseg, noverlap, flags):
    T = (x.shape[-1] - nperseg) // (nperseg - noverlap) + 1
    F = nperseg // 2 + (0 if flags & _lib.STFT_DROP_NYQUIST else 1)
    return x.shape[0], F, T


def _stft_out(x, nperseg, noverlap, window, fs, scaling, detrend, eps, flags, out):
    from . import stft
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be [batch, length] with unit stride along length")
    if x.dtype not in (torch.float32, torch.float16):
        raise TypeError("x must be float32 or float16")
    if tuple(out.shape) != _stft_shape(x, nperseg, noverlap, flags) or \
            out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be contiguous float32 [batch, F, T]")
    plan = stft.get_plan_key(x.device, nperseg, noverlap, window, fs, scaling, detrend, eps)
    L = _lib.lib()
    if x.dtype == torch.float16 and nperseg > 1024:
        x = x.float()  # the fp16-sample kernel covers nperseg <= 1024
    if x.dtype == torch.float16:  # fp16 samples widened on load: no conversion pass
        _lib.check(L.specenh_stft_psd_f16(plan.handle, _vp(x), x.shape[0], x.shape[1],
                                          x.stride(0), _vp(out), flags, _st(x)), "stft_psd_f16")
        return
    ws = plan.workspace(x.shape[0], x.device)
    _lib.check(L.specenh_stft_psd(plan.handle, _vp(x), x.shape[0], x.shape[1], x.stride(0),
                                  _vp(out), flags, _vp(ws), _st(x)), "stft_psd")


def _stft(x, nperseg, noverlap, window, fs, scaling, detrend, eps, flags):
    out = torch.empty(_stft_shape(x, nperseg, noverlap, flags), dtype=torch.float32,
                      device=x.device)
    _stft_out(x, nperseg, noverlap, window, fs, scaling, detrend, eps, flags, out)
    return out


_STFT_ARGS = "int nperseg, int noverlap, str window, float fs, int scaling, int detrend, " \
             "float eps, int flags"
_op(f"stft_psd(Tensor x, {_STFT_ARGS}) -> Tensor", _stft,
    lambda x, nperseg, noverlap, window, fs, scaling, detrend, eps, flags:
    x.new_empty(_stft_shape(x, nperseg, noverlap, flags), dtype=torch.float32))
_op(f"stft_psd_out(Tensor x, {_STFT_ARGS}, Tensor(a!) out) -> ()", _stft_out,
    lambda *a: None)


# ---------------------------------------------------------------- cross spectrum
def _csd(x, y, nperseg, noverlap, window, fs, scaling, detrend, mode):
    from . import cross
    if x.shape != y.shape or x.dim() != 2 or x.dtype != torch.float32 or y.dtype != torch.float32:
        raise ValueError("x and y must be float32 [batch, length] of the same shape")
    if x.stride(1) != 1 or y.stride(1) != 1:
        raise ValueError("x and y need unit stride along length")
    plan = cross.get_plan_key(x.device, nperseg, noverlap, window, fs, scaling, detrend)
    B, L = x.shape
    T = (L - nperseg) // (nperseg - noverlap) + 1
    F = nperseg // 2 + 1
    out = torch.empty((B, F, T), dtype=torch.float32 if mode == 1 else torch.complex64,
                      device=x.device)
    for b0 in range(0, B, 65535):
        b1 = min(B, b0 + 65535)
        _lib.check(_lib.lib().specenh_csd(
            plan.handle, _vp(x[b0:b1]), _vp(y[b0:b1]), b1 - b0, L, x.stride(0), y.stride(0),
            _vp(out[b0:b1]), int(mode), _st(x)), "csd")
    return out


def _csd_fake(x, y, nperseg, noverlap, window, fs, scaling, detrend, mode):
    T = (x.shape[1] - nperseg) // (nperseg - noverlap) + 1
    return x.new_empty((x.shape[0], nperseg // 2 + 1, T),
                       dtype=torch.float32 if mode == 1 else torch.complex64)


_op("csd(Tensor x, Tensor y, int nperseg, int noverlap, str window, float fs, int scaling, "
    "int detrend, int mode) -> Tensor", _csd, _csd_fake)


# ---------------------------------------------------------------- SVD denoiser
def _bstride(A):
    """Batch stride for the C-ABI: a batch of one may carry any stride (e.g. 0 from a numpy
    [None] view); the kernels only need it to reach matrix b for b >= 1."""
    return A.stride(0) if A.shape[0] > 1 else A.shape[1] * A.shape[2]


def _svd_check(A):
    if A.dim() != 3 or A.dtype != torch.float32 or A.stride(2) != 1 or A.stride(1) != A.shape[2]:
        raise ValueError("A must be float32 [batch, m, n] with row-major matrices")


def _svd_out(A, start, stop, out):
    _svd_check(A)
    B, m, n = A.shape
    if out.shape != A.shape or not out.is_contiguous() or out.device != A.device:
        raise ValueError("out must be a contiguous [B, m, n] tensor on A's device")
    L = _lib.lib()
    ws = torch.empty(max(16, int(L.specenh_svd_denoise_workspace_bytes(B, m, n, start, stop))),
                     dtype=torch.uint8, device=A.device)
    _lib.check(L.specenh_svd_denoise_ex(_vp(A), B, m, n, _bstride(A), start, stop, _vp(out),
                                        _code(out), _vp(ws), _st(A)), "svd_denoise")


def _svd(A, start, stop, out_dtype):
    out = torch.empty(A.shape, dtype=out_dtype, device=A.device)
    _svd_out(A, start, stop, out)
    return out


def _svd_opt_out(A, kind, out, num_sing, median):
    _svd_check(A)
    B, m, n = A.shape
    if (out.shape != A.shape or out.dtype != torch.float32 or not out.is_contiguous()
            or out.device != A.device):
        raise ValueError("out must be a contiguous float32 [B, m, n] tensor on A's device")
    if (num_sing.numel() != B or num_sing.dtype != torch.int32 or median.numel() != B
            or median.dtype != torch.float64 or num_sing.device != A.device
            or median.device != A.device):
        raise ValueError("num_sing / median must be int32 / float64 [B] tensors on A's device")
    L = _lib.lib()
    ws = torch.empty(max(16, int(L.specenh_svd_optimal_workspace_bytes(B, m, n))),
                     dtype=torch.uint8, device=A.device)
    _lib.check(L.specenh_svd_denoise_optimal(_vp(A), B, m, n, _bstride(A), int(kind), _vp(out),
                                             _vp(num_sing), _vp(median), _vp(ws), _st(A)),
               "svd_denoise_optimal")


def _svd_opt(A, mode):
    out = torch.empty(A.shape, dtype=torch.float32, device=A.device)
    ns = torch.empty(A.shape[0], dtype=torch.int32, device=A.device)
    med = torch.empty(A.shape[0], dtype=torch.float64, device=A.device)
    _svd_opt_out(A, mode, out, ns, med)
    return out, ns, med


_op("svd_denoise(Tensor A, int start, int stop, ScalarType out_dtype) -> Tensor", _svd,
    lambda A, start, stop, out_dtype: A.new_empty(A.shape, dtype=out_dtype))
_op("svd_denoise_out(Tensor A, int start, int stop, Tensor(a!) out) -> ()", _svd_out,
    lambda *a: None)
_op("svd_denoise_optimal(Tensor A, int mode) -> (Tensor, Tensor, Tensor)", _svd_opt,
    lambda A, mode: (A.new_empty(A.shape), A.new_empty((A.shape[0],), dtype=torch.int32),
                     A.new_empty((A.shape[0],), dtype=torch.float64)))
# (the mode argument is "kind" here: auto_functionalized reserves the name "mode")
_op("svd_denoise_optimal_out(Tensor A, int kind, Tensor(a!) out, Tensor(b!) num_sing, "
    "Tensor(c!) median) -> ()", _svd_opt_out, lambda *a: None)


# ---------------------------------------------------------------- convolutions
def _conv_out(x, w, bias, kh, kw, cout, stride, pad_t, pad_l, in_dil, oh, ow, act, mask,
              logits, out, pool, argmax):
    if x.dim() != 4:
        raise ValueError("x must be NHWC [N, H, W, C]")
    _need(x, "x")
    _need(out, "out")
    N, IH, IW, C = x.shape
    dt = _code(x)
    if w.dtype != x.dtype or w.numel() != cout * kh * kw * C:
        raise ValueError("w must be the [CO][KH][KW][C] GEMM weights in x's dtype")
    _need(w, "w")
    oshape = (N, oh // 2, ow // 2, cout) if pool else (N, oh, ow, cout)
    if tuple(out.shape) != oshape or out.dtype not in (x.dtype, torch.float32):
        raise ValueError(f"out must be {oshape} in x's dtype or float32")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != cout):
        raise ValueError("bias must be float32 [CO]")
    if mask is not None and (mask.dtype != x.dtype or mask.numel() != N * oh * ow * cout):
        raise ValueError("mask must match the output (compute dtype)")
    if logits is not None and (logits.dtype != torch.float32 or
                               logits.numel() != N * oh * ow * cout):
        raise ValueError("logits must be float32 [N, OH, OW, CO]")
    if argmax is not None and (argmax.dtype != torch.uint8 or tuple(argmax.shape) != oshape):
        raise ValueError("argmax must be uint8 like the pooled output")
    out_f32 = int(out.dtype == torch.float32)
    _lib.check(_lib.lib().specenh_conv2d(
        dt, _vp(x), N, IH, IW, C, _vp(w), kh, kw, cout, _vp(bias), stride, pad_t, pad_l, in_dil,
        oh, ow, act, _vp(mask), _vp(logits), _vp(out), out_f32, int(pool), _vp(argmax), _st(x)),
        "conv2d")


def _conv(x, w, bias, kh, kw, cout, stride, pad_t, pad_l, in_dil, oh, ow, act):
    out = torch.empty((x.shape[0], oh, ow, cout), dtype=x.dtype, device=x.device)
    _conv_out(x, w, bias, kh, kw, cout, stride, pad_t, pad_l, in_dil, oh, ow, act, None, None,
              out, False, None)
    return out


_CONV_ARGS = "int kh, int kw, int cout, int stride, int pad_t, int pad_l, int in_dil, int oh, " \
             "int ow, int act"
_op(f"conv2d(Tensor x, Tensor w, Tensor? bias, {_CONV_ARGS}) -> Tensor", _conv,
    lambda x, w, bias, kh, kw, cout, stride, pad_t, pad_l, in_dil, oh, ow, act:
    x.new_empty((x.shape[0], oh, ow, cout)))
_op(f"conv2d_out(Tensor x, Tensor w, Tensor? bias, {_CONV_ARGS}, Tensor? mask, "
    "Tensor(a!)? logits, Tensor(b!) out, bool pool, Tensor(c!)? argmax) -> ()", _conv_out,
    lambda *a: None)


def wgrad_workspace(x, dout, kh, kw):
    N, _, _, C = x.shape
    _, OH, OW, CO = dout.shape
    n = int(_lib.lib().specenh_conv2d_wgrad_workspace_bytes(N, OH, OW, kh, kw, C, CO))
    return torch.empty(max(16, n), dtype=torch.uint8, device=x.device)


def _wgrad_out(x, dout, kh, kw, stride, pad_t, pad_l, in_dil, dw, dbias, workspace,
               overwrite=False):
    _need(x, "x")
    _need(dout, "dout")
    N, IH, IW, C = x.shape
    _, OH, OW, CO = dout.shape
    if dout.dtype != x.dtype or dout.shape[0] != N:
        raise ValueError("dout must be [N, OH, OW, CO] in x's dtype")
    if dw.dtype != torch.float32 or dw.numel() != CO * kh * kw * C or not dw.is_contiguous():
        raise ValueError("dw must be contiguous float32 [CO][KH][KW][C]")
    if dbias is not None and (dbias.dtype != torch.float32 or dbias.numel() != CO):
        raise ValueError("dbias must be float32 [CO]")
    need = int(_lib.lib().specenh_conv2d_wgrad_workspace_bytes(N, OH, OW, kh, kw, C, CO))
    if workspace.numel() < need:
        raise ValueError(f"workspace needs {need} bytes")
    if overwrite:  # dw / dbias = the gradient (no zeroing beforehand)
        _lib.check(_lib.lib().specenh_conv2d_wgrad_ex(
            _code(x), _vp(x), N, IH, IW, C, _vp(dout), kh, kw, CO, stride, pad_t, pad_l, in_dil,
            OH, OW, _vp(dw), _vp(dbias), 1, _vp(workspace), _st(x)), "conv2d_wgrad")
        return
    _lib.check(_lib.lib().specenh_conv2d_wgrad(
        _code(x), _vp(x), N, IH, IW, C, _vp(dout), kh, kw, CO, stride, pad_t, pad_l, in_dil, OH,
        OW, _vp(dw), _vp(dbias), _vp(workspace), _st(x)), "conv2d_wgrad")


def _wgrad(x, dout, kh, kw, stride, pad_t, pad_l, in_dil):
    C, CO = x.shape[3], dout.shape[3]
    dw = torch.zeros((CO, kh, kw, C), dtype=torch.float32, device=x.device)
    db = torch.zeros((CO,), dtype=torch.float32, device=x.device)
    _wgrad_out(x, dout, kh, kw, stride, pad_t, pad_l, in_dil, dw, db,
               wgrad_workspace(x, dout, kh, kw))
    return dw, db


_WG_ARGS = "int kh, int kw, int stride, int pad_t, int pad_l, int in_dil"
_op(f"conv2d_wgrad(Tensor x, Tensor dout, {_WG_ARGS}) -> (Tensor, Tensor)", _wgrad,
    lambda x, dout, kh, kw, stride, pad_t, pad_l, in_dil:
    (x.new_empty((dout.shape[3], kh, kw, x.shape[3]), dtype=torch.float32),
     x.new_empty((dout.shape[3],), dtype=torch.float32)))
_op(f"conv2d_wgrad_out(Tensor x, Tensor dout, {_WG_ARGS}, Tensor(a!) dw, Tensor(b!)? dbias, "
    "Tensor(c!) workspace, bool overwrite=False) -> ()", _wgrad_out, lambda *a, **k: None)


def _wgrad_pooled_out(x, dpool, argmax, pooled, kh, kw, stride, pad_t, pad_l, in_dil, dw, dbias,
                      workspace):
    _need(x, "x")
    _need(dpool, "dpool")
    N, IH, IW, C = x.shape
    _, PH, PW, CO = dpool.shape
    OH, OW = 2 * PH, 2 * PW
    if dpool.dtype != x.dtype or dpool.shape[0] != N:
        raise ValueError("dpool must be [N, OH/2, OW/2, CO] in x's dtype")
    if argmax.dtype != torch.uint8 or argmax.shape != dpool.shape:
        raise ValueError("argmax must be uint8 like dpool")
    if pooled is not None and (pooled.dtype != x.dtype or pooled.shape != dpool.shape):
        raise ValueError("pooled must be like dpool")
    if dw.dtype != torch.float32 or dw.numel() != CO * kh * kw * C or not dw.is_contiguous():
        raise ValueError("dw must be contiguous float32 [CO][KH][KW][C]")
    if dbias is not None and (dbias.dtype != torch.float32 or dbias.numel() != CO):
        raise ValueError("dbias must be float32 [CO]")
    need = int(_lib.lib().specenh_conv2d_wgrad_workspace_bytes(N, OH, OW, kh, kw, C, CO))
    if workspace.numel() < need:
        raise ValueError(f"workspace needs {need} bytes")
    _lib.check(_lib.lib().specenh_conv2d_wgrad_pooled(
        _code(x), _vp(x), N, IH, IW, C, _vp(dpool), _vp(argmax), _vp(pooled), kh, kw, CO, stride,
        pad_t, pad_l, in_dil, OH, OW, _vp(dw), _vp(dbias), _vp(workspace), _st(x)),
        "conv2d_wgrad_pooled")


_op(f"conv2d_wgrad_pooled_out(Tensor x, Tensor dpool, Tensor argmax, Tensor? pooled, {_WG_ARGS}, "
    "Tensor(a!) dw, Tensor(b!)? dbias, Tensor(c!) workspace) -> ()", _wgrad_pooled_out,
    lambda *a: None)


def _conv_pooled_in_out(dpool, argmax, pooled, w, bias, kh, kw, cout, pad_t, pad_l, oh, ow, act,
                        mask, out):
    """specenh_conv2d_pooled_in: a stride-1 conv of the full-resolution gradient of a ReLU +
    MaxPooling2D((2,2)) given as the pool's gradient dpool [N, IH/2, IW/2, C] (+ argmax, pooled
    output): bitwise maxpool2_bwd followed by conv2d_out, without the full-resolution tensor."""
    _need(dpool, "dpool")
    _need(out, "out")
    N, PH, PW, C = dpool.shape
    IH, IW = 2 * PH, 2 * PW
    if argmax.dtype != torch.uint8 or argmax.shape != dpool.shape:
        raise ValueError("argmax must be uint8 like dpool")
    if pooled is not None and (pooled.dtype != dpool.dtype or pooled.shape != dpool.shape):
        raise ValueError("pooled must be like dpool")
    if w.dtype != dpool.dtype or w.numel() != cout * kh * kw * C:
        raise ValueError("w must be the [CO][KH][KW][C] GEMM weights in dpool's dtype")
    _need(w, "w")
    if tuple(out.shape) != (N, oh, ow, cout) or out.dtype != dpool.dtype:
        raise ValueError(f"out must be {(N, oh, ow, cout)} in dpool's dtype")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != cout):
        raise ValueError("bias must be float32 [CO]")
    if mask is not None and (mask.dtype != dpool.dtype or mask.numel() != N * oh * ow * cout):
        raise ValueError("mask must match the output (compute dtype)")
    _lib.check(_lib.lib().specenh_conv2d_pooled_in(
        _code(dpool), _vp(dpool), _vp(argmax), _vp(pooled), N, IH, IW, C, _vp(w), kh, kw, cout,
        _vp(bias), pad_t, pad_l, oh, ow, act, _vp(mask), _vp(out), _st(dpool)),
        "conv2d_pooled_in")


_op("conv2d_pooled_in_out(Tensor dpool, Tensor argmax, Tensor? pooled, Tensor w, Tensor? bias, "
    "int kh, int kw, int cout, int pad_t, int pad_l, int oh, int ow, int act, Tensor? mask, "
    "Tensor(a!) out) -> ()", _conv_pooled_in_out, lambda *a: None)


def _tail_out(x, wt, bt, cout, kt, wo, bo, ko, out):
    _need(x, "x")
    _need(out, "out")
    N, H, W, C = x.shape
    if wt.dtype != x.dtype or wo.dtype != x.dtype or wt.numel() != cout * kt * kt * C or \
            wo.numel() != ko * ko * cout:
        raise ValueError("wt / wo must be the two layers' GEMM weights in x's dtype")
    if bt.dtype != torch.float32 or bt.numel() != cout or bo.dtype != torch.float32 or \
            bo.numel() != 1:
        raise ValueError("biases must be float32 [CO] and [1]")
    if out.dtype != torch.float32 or out.numel() != N * 4 * H * W:
        raise ValueError("out must be float32 [N, 2H, 2W(, 1)]")
    _lib.check(_lib.lib().specenh_convt_conv_out(
        _code(x), _vp(x), N, H, W, C, _vp(wt), _vp(bt), cout, kt, _vp(wo), _vp(bo), ko, _vp(out),
        _st(x)), "convt_conv_out")


def _tail(x, wt, bt, cout, kt, wo, bo, ko):
    N, H, W, _ = x.shape
    out = torch.empty((N, 2 * H, 2 * W, 1), dtype=torch.float32, device=x.device)
    _tail_out(x, wt, bt, cout, kt, wo, bo, ko, out)
    return out


_op("convt_conv_out(Tensor x, Tensor wt, Tensor bt, int cout, int kt, Tensor wo, Tensor bo, "
    "int ko) -> Tensor", _tail,
    lambda x, wt, bt, cout, kt, wo, bo, ko:
    x.new_empty((x.shape[0], 2 * x.shape[1], 2 * x.shape[2], 1), dtype=torch.float32))
_op("convt_conv_out_out(Tensor x, Tensor wt, Tensor bt, int cout, int kt, Tensor wo, Tensor bo, "
    "int ko, Tensor(a!) out) -> ()", _tail_out, lambda *a: None)


def _tail_train_out(x, wt, bt, cout, kt, wo, bo, ko, map_out, logits, out):
    _need(x, "x")
    for t, n in ((map_out, "map_out"), (logits, "logits"), (out, "out")):
        _need(t, n)
    N, H, W, C = x.shape
    if wt.dtype != x.dtype or wo.dtype != x.dtype or wt.numel() != cout * kt * kt * C or \
            wo.numel() != ko * ko * cout:
        raise ValueError("wt / wo must be the two layers' GEMM weights in x's dtype")
    if bt.dtype != torch.float32 or bt.numel() != cout or bo.dtype != torch.float32 or \
            bo.numel() != 1:
        raise ValueError("biases must be float32 [CO] and [1]")
    if tuple(map_out.shape) != (N, 2 * H, 2 * W, cout) or map_out.dtype != x.dtype:
        raise ValueError("map_out must be [N, 2H, 2W, cout] in x's dtype")
    if logits.dtype != torch.float32 or logits.numel() != N * 4 * H * W:
        raise ValueError("logits must be float32 [N, 2H, 2W(, 1)]")
    if out.dtype != x.dtype or out.numel() != N * 4 * H * W:
        raise ValueError("out must be [N, 2H, 2W(, 1)] in x's dtype")
    _lib.check(_lib.lib().specenh_convt_conv_out_train(
        _code(x), _vp(x), N, H, W, C, _vp(wt), _vp(bt), cout, kt, _vp(wo), _vp(bo), ko,
        _vp(map_out), _vp(logits), _vp(out), _st(x)), "convt_conv_out_train")


_op("convt_conv_out_train_out(Tensor x, Tensor wt, Tensor bt, int cout, int kt, Tensor wo, "
    "Tensor bo, int ko, Tensor(a!) map_out, Tensor(b!) logits, Tensor(c!) out) -> ()",
    _tail_train_out, lambda *a: None)


def _dec3_out(x, w1, b1, cout1, wt, bt, cout2, wo, bo, k, out):
    _need(x, "x")
    _need(out, "out")
    N, H, W, C = x.shape
    if any(t.dtype != x.dtype for t in (w1, wt, wo)) or w1.numel() != cout1 * k * k * C or \
            wt.numel() != cout2 * k * k * cout1 or wo.numel() != k * k * cout2:
        raise ValueError("w1 / wt / wo must be the three layers' GEMM weights in x's dtype")
    if any(t.dtype != torch.float32 for t in (b1, bt, bo)) or b1.numel() != cout1 or \
            bt.numel() != cout2 or bo.numel() != 1:
        raise ValueError("biases must be float32 [CO1], [CO2] and [1]")
    if out.dtype not in (torch.float32, torch.float16) or out.numel() != N * 16 * H * W:
        raise ValueError("out must be float32 or float16 [N, 4H, 4W(, 1)]")
    _lib.check(_lib.lib().specenh_decoder3_ex(
        _code(x), _vp(x), N, H, W, C, _vp(w1), _vp(b1), cout1, _vp(wt), _vp(bt), cout2, _vp(wo),
        _vp(bo), k, _vp(out), _code(out), _st(x)), "decoder3")


def _dec3(x, w1, b1, cout1, wt, bt, cout2, wo, bo, k):
    N, H, W, _ = x.shape
    out = torch.empty((N, 4 * H, 4 * W, 1), dtype=torch.float32, device=x.device)
    _dec3_out(x, w1, b1, cout1, wt, bt, cout2, wo, bo, k, out)
    return out


_D3 = ("Tensor x, Tensor w1, Tensor b1, int cout1, Tensor wt, Tensor bt, int cout2, Tensor wo, "
       "Tensor bo, int k")
_op(f"decoder3({_D3}) -> Tensor", _dec3,
    lambda x, w1, b1, cout1, wt, bt, cout2, wo, bo, k:
    x.new_empty((x.shape[0], 4 * x.shape[1], 4 * x.shape[2], 1), dtype=torch.float32))
_op(f"decoder3_out({_D3}, Tensor(a!) out) -> ()", _dec3_out, lambda *a: None)


def _enc2_out(x, w1, b1, cout1, w2, b2, cout2, k, out):
    _need(x, "x")
    _need(out, "out")
    N, H, W, C = x.shape
    if C != 1:
        raise ValueError("x must be [N, H, W, 1]")
    if any(t.dtype != x.dtype for t in (w1, w2)) or w1.numel() != cout1 * k * k or \
            w2.numel() != cout2 * k * k * cout1:
        raise ValueError("w1 / w2 must be the two layers' GEMM weights in x's dtype")
    if any(t.dtype != torch.float32 for t in (b1, b2)) or b1.numel() != cout1 or \
            b2.numel() != cout2:
        raise ValueError("biases must be float32 [CO1] and [CO2]")
    if out.dtype != x.dtype or tuple(out.shape) != (N, H // 4, W // 4, cout2):
        raise ValueError("out must be [N, H/4, W/4, CO2] in x's dtype")
    _lib.check(_lib.lib().specenh_encoder2(
        _code(x), _vp(x), N, H, W, _vp(w1), _vp(b1), cout1, _vp(w2), _vp(b2), cout2, k, _vp(out),
        _st(x)), "encoder2")


def _enc2(x, w1, b1, cout1, w2, b2, cout2, k):
    N, H, W, _ = x.shape
    out = torch.empty((N, H // 4, W // 4, cout2), dtype=x.dtype, device=x.device)
    _enc2_out(x, w1, b1, cout1, w2, b2, cout2, k, out)
    return out


_E2 = "Tensor x, Tensor w1, Tensor b1, int cout1, Tensor w2, Tensor b2, int cout2, int k"
_op(f"encoder2({_E2}) -> Tensor", _enc2,
    lambda x, w1, b1, cout1, w2, b2, cout2, k:
    x.new_empty((x.shape[0], x.shape[1] // 4, x.shape[2] // 4, cout2)))
_op(f"encoder2_out({_E2}, Tensor(a!) out) -> ()", _enc2_out, lambda *a: None)


def encoder2_supported(dtype: torch.dtype, cin: int, cout1: int, cout2: int, k: int,
                       height: int, width: int) -> bool:
    """specenh_encoder2's configuration: the reference model's first two layers on 128-wide
    one-channel images."""
    return dtype in (torch.float16, torch.bfloat16) and (cin, cout1, cout2, k, width) == \
        (1, 16, 32, 5, 128) and height % 4 == 0


def decoder3_supported(dtype: torch.dtype, cin: int, cout1: int, cout2: int, k: int,
                       width: int) -> bool:
    """specenh_decoder3's configuration: the reference model's decoder on 128-wide images."""
    return dtype in (torch.float16, torch.bfloat16) and (cin, cout1, cout2, k, width) == \
        (64, 32, 16, 5, 32)


def tail_supported(dtype: torch.dtype, cin: int, cout: int, kt: int, ko: int,
                   w_in: int | None = None) -> bool:
    """specenh_convt_conv_out's configurations: the reference model's last two layers
    (32 -> 16, k 5, any width), and the 32 -> 32 tails of the hyperparameter-scan models
    (k = 3 / 5 / 7) and manual_scan.py's 32 -> 64 (k = 3 / 5) on 64-position-wide inputs
    (csrc/tail_rows_g.hip)."""
    if dtype not in (torch.float16, torch.bfloat16):
        return False
    if (cin, cout, kt, ko) == (32, 16, 5, 5):
        return True
    return w_in == 64 and cin == 32 and kt == ko and ((cout == 32 and kt in (3, 5, 7)) or
                                                       (cout == 64 and kt in (3, 5)))


# ---------------------------------------------------------------- pooling, loss, optimizer
def _pool_out(x, out, argmax):
    _need(x, "x")
    N, H, W, C = x.shape
    if tuple(out.shape) != (N, H // 2, W // 2, C) or out.dtype != x.dtype:
        raise ValueError("out must be [N, H/2, W/2, C] in x's dtype")
    if argmax.dtype != torch.uint8 or argmax.shape != out.shape:
        raise ValueError("argmax must be uint8 like out")
    _lib.check(_lib.lib().specenh_maxpool2_fwd(_code(x), _vp(x), N, H, W, C, _vp(out),
                                               _vp(argmax), _st(x)), "maxpool2_fwd")


def _pool(x):
    N, H, W, C = x.shape
    out = torch.empty((N, H // 2, W // 2, C), dtype=x.dtype, device=x.device)
    am = torch.empty(out.shape, dtype=torch.uint8, device=x.device)
    _pool_out(x, out, am)
    return out, am


def _pool_bwd_out(dy, argmax, pooled, dx):
    _need(dy, "dy")
    N, H2, W2, C = dy.shape
    if tuple(dx.shape) != (N, 2 * H2, 2 * W2, C) or dx.dtype != dy.dtype:
        raise ValueError("dx must be [N, 2H, 2W, C] in dy's dtype")
    _lib.check(_lib.lib().specenh_maxpool2_bwd(_code(dy), _vp(dy), _vp(argmax), _vp(pooled), N,
                                               2 * H2, 2 * W2, C, _vp(dx), _st(dy)),
               "maxpool2_bwd")


def _pool_bwd(dy, argmax, pooled):
    N, H2, W2, C = dy.shape
    dx = torch.empty((N, 2 * H2, 2 * W2, C), dtype=dy.dtype, device=dy.device)
    _pool_bwd_out(dy, argmax, pooled, dx)
    return dx


_op("maxpool2(Tensor x) -> (Tensor, Tensor)", _pool,
    lambda x: (x.new_empty((x.shape[0], x.shape[1] // 2, x.shape[2] // 2, x.shape[3])),
               x.new_empty((x.shape[0], x.shape[1] // 2, x.shape[2] // 2, x.shape[3]),
                           dtype=torch.uint8)))
_op("maxpool2_out(Tensor x, Tensor(a!) out, Tensor(b!) argmax) -> ()", _pool_out,
    lambda *a: None)
_op("maxpool2_bwd(Tensor dy, Tensor argmax, Tensor? pooled) -> Tensor", _pool_bwd,
    lambda dy, argmax, pooled: dy.new_empty((dy.shape[0], 2 * dy.shape[1], 2 * dy.shape[2],
                                             dy.shape[3])))
_op("maxpool2_bwd_out(Tensor dy, Tensor argmax, Tensor? pooled, Tensor(a!) dx) -> ()",
    _pool_bwd_out, lambda *a: None)


def _bce_out(z, target, grad, loss_sum):
    if z.dtype != torch.float32 or target.numel() != z.numel():
        raise ValueError("z must be float32 and target the same size")
    _need(z, "z")
    _need(target, "target")
    if loss_sum.dtype != torch.float64 or loss_sum.numel() != 1:
        raise ValueError("loss_sum must be a float64 [1] accumulator")
    if grad is not None and grad.numel() != z.numel():
        raise ValueError("grad must have z's size")
    _lib.check(_lib.lib().specenh_bce_logits(
        _vp(z), _vp(target), _code(target), z.numel(), _vp(grad),
        _code(grad) if grad is not None else F32, _vp(loss_sum), _st(z)), "bce_logits")


def _bce(z, target, grad_dtype):
    loss = torch.zeros(1, dtype=torch.float64, device=z.device)
    grad = torch.empty(z.shape, dtype=grad_dtype, device=z.device)
    _bce_out(z, target, grad, loss)
    return loss, grad


_op("bce_logits(Tensor z, Tensor target, ScalarType grad_dtype) -> (Tensor, Tensor)", _bce,
    lambda z, target, grad_dtype: (z.new_empty((1,), dtype=torch.float64),
                                   z.new_empty(z.shape, dtype=grad_dtype)))
_op("bce_logits_out(Tensor z, Tensor target, Tensor(a!)? grad, Tensor(b!) loss_sum) -> ()",
    _bce_out, lambda *a: None)


def _adam(w, g, m, v, lr_t, beta_1, beta_2, epsilon, grad_scale, w_lowp):
    n = w.numel()
    for t, nm in ((g, "g"), (m, "m"), (v, "v")):
        if t.numel() != n or t.dtype != torch.float32:
            raise ValueError(f"{nm} must be float32 like w")
    if w_lowp is not None and w_lowp.numel() != n:
        raise ValueError("w_lowp must have w's size")
    _lib.check(_lib.lib().specenh_adam_step(
        _vp(w), _vp(g), _vp(m), _vp(v), n, lr_t, beta_1, beta_2, epsilon, grad_scale,
        _vp(w_lowp), _code(w_lowp) if w_lowp is not None else F32, _st(w)), "adam_step")


_op("adam_step_(Tensor(a!) w, Tensor g, Tensor(b!) m, Tensor(c!) v, float lr_t, float beta_1, "
    "float beta_2, float epsilon, float grad_scale, Tensor(d!)? w_lowp) -> ()", _adam,
    lambda *a: None)


def _adam_flip(w, g, m, v, lr_t, beta_1, beta_2, epsilon, grad_scale, w_lowp, seg_off, seg_kcc,
               seg_dst):
    """adam_step_ plus the flipped input-gradient weights of len(seg_dst) layers in the same
    launch (specenh_adam_step_flip): seg_off[s] is the layer's flat weight offset in w,
    seg_kcc[3s:3s+3] = (k, ci, co), seg_dst[s] its [ci][k][k][co] buffer."""
    import ctypes
    n = w.numel()
    for t, nm in ((g, "g"), (m, "m"), (v, "v")):
        if t.numel() != n or t.dtype != torch.float32:
            raise ValueError(f"{nm} must be float32 like w")
    if w_lowp is not None and w_lowp.numel() != n:
        raise ValueError("w_lowp must have w's size")
    ns = len(seg_dst)
    if len(seg_off) != ns or len(seg_kcc) != 3 * ns:
        raise ValueError("segment lists")
    want = w_lowp.dtype if w_lowp is not None else torch.float32
    for s, d in enumerate(seg_dst):
        k, ci, co = seg_kcc[3 * s:3 * s + 3]
        if d.dtype != want or d.numel() != k * k * ci * co or not d.is_contiguous():
            raise ValueError(f"segment {s}: destination must be contiguous {want} [{ci}][{k}][{k}][{co}]")
    off = (ctypes.c_longlong * max(ns, 1))(*seg_off)
    kcc = (ctypes.c_int * max(3 * ns, 1))(*seg_kcc)
    dst = (ctypes.c_void_p * max(ns, 1))(*[d.data_ptr() for d in seg_dst])
    _lib.check(_lib.lib().specenh_adam_step_flip(
        _vp(w), _vp(g), _vp(m), _vp(v), n, lr_t, beta_1, beta_2, epsilon, grad_scale,
        _vp(w_lowp), _code(w_lowp) if w_lowp is not None else F32, ns, off, kcc, dst, _st(w)),
        "adam_step_flip")


_op("adam_step_flip_(Tensor(a!) w, Tensor g, Tensor(b!) m, Tensor(c!) v, float lr_t, "
    "float beta_1, float beta_2, float epsilon, float grad_scale, Tensor(d!)? w_lowp, "
    "int[] seg_off, int[] seg_kcc, Tensor(e!)[] seg_dst) -> ()", _adam_flip, lambda *a: None)


def _flip_out(bt, k, ci, co, out):
    if bt.numel() != co * k * k * ci or out.numel() != bt.numel() or out.dtype != bt.dtype:
        raise ValueError("bt / out sizes")
    _lib.check(_lib.lib().specenh_weight_flip_transpose(_code(bt), _vp(bt), k, ci, co, _vp(out),
                                                        _st(bt)), "flip_transpose")


def _flip(bt, k, ci, co):
    out = torch.empty((ci, k, k, co), dtype=bt.dtype, device=bt.device)
    _flip_out(bt, k, ci, co, out)
    return out


_op("weight_flip_transpose(Tensor bt, int k, int ci, int co) -> Tensor", _flip,
    lambda bt, k, ci, co: bt.new_empty((ci, k, k, co)))
_op("weight_flip_transpose_out(Tensor bt, int k, int ci, int co, Tensor(a!) out) -> ()",
    _flip_out, lambda *a: None)


def _cast_out(x, out):
    if out.numel() != x.numel():
        raise ValueError("out must have x's size")
    _need(x, "x")
    _need(out, "out")
    _lib.check(_lib.lib().specenh_cast(_code(x), _vp(x), _code(out), _vp(out), x.numel(), _st(x)),
               "cast")


def _cast(x, dtype):
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    _cast_out(x, out)
    return out


_op("cast(Tensor x, ScalarType dtype) -> Tensor", _cast,
    lambda x, dtype: x.new_empty(x.shape, dtype=dtype))
_op("cast_out(Tensor x, Tensor(a!) out) -> ()", _cast_out, lambda *a: None)


# ---------------------------------------------------------------- label filters
def _batch3(S):
    if S.dim() != 3:
        raise ValueError("S must be [batch, rows, cols]")
    _need(S, "S")
    return S.shape


def _filter(S, op):
    B, rows, cols = _batch3(S)
    L = _lib.lib()
    out = torch.empty_like(S)
    ws = torch.empty(max(16, int(L.specenh_filter_workspace_bytes(B, rows))), dtype=torch.uint8,
                     device=S.device)
    _lib.check(L.specenh_filter(int(op), _code(S, (F32, F64)), _vp(S), B, rows, cols, rows * cols,
                                _vp(out), _vp(ws), _st(S)), "filter")
    return out


def _quantfilt(S, thr):
    B, rows, cols = _batch3(S)
    out = torch.empty_like(S)
    _lib.check(_lib.lib().specenh_quantfilt(_code(S, (F32, F64)), _vp(S), B, rows, cols,
                                            rows * cols, float(thr), _vp(out), _st(S)), "quantfilt")
    return out


def _u8ws(S):
    B, rows, cols = S.shape
    n = int(_lib.lib().specenh_u8filter_workspace_bytes(B, rows, cols))
    return torch.empty(max(16, n), dtype=torch.uint8, device=S.device)


def _gaussblr(S, kw, kh, sigma):
    B, rows, cols = _batch3(S)
    out = torch.empty_like(S)
    _lib.check(_lib.lib().specenh_gaussblr(_code(S, (F32, F64)), _vp(S), B, rows, cols,
                                           rows * cols, int(kw), int(kh), float(sigma), _vp(out),
                                           _vp(_u8ws(S)), _st(S)), "gaussblr")
    return out


def _morph(S):
    B, rows, cols = _batch3(S)
    out = torch.empty_like(S)
    _lib.check(_lib.lib().specenh_morph(_code(S, (F32, F64)), _vp(S), B, rows, cols, rows * cols,
                                        _vp(out), _vp(_u8ws(S)), _st(S)), "morph")
    return out


_op("label_filter(Tensor S, int op) -> Tensor", _filter, lambda S, op: torch.empty_like(S))
_op("quantfilt(Tensor S, float thr) -> Tensor", _quantfilt, lambda S, thr: torch.empty_like(S))
_op("gaussblr(Tensor S, int kw, int kh, float sigma) -> Tensor", _gaussblr,
    lambda S, kw, kh, sigma: torch.empty_like(S))
_op("morph(Tensor S) -> Tensor", _morph, lambda S: torch.empty_like(S))


# ---------------------------------------------------------------- strip glue
def _pack_out(S, rows, width, n_strips, out):
    if S.dim() != 3 or S.dtype != torch.float32 or S.stride(2) != 1 or S.stride(1) != S.shape[2]:
        raise ValueError("S must be float32 [batch, F, T] with row-major spectrograms")
    B, F, T = S.shape
    if (out.numel() != B * n_strips * rows * width or not out.is_contiguous()
            or out.device != S.device or out.dtype not in (torch.float32, torch.bfloat16,
                                                          torch.float16)):
        raise ValueError(f"out must be a contiguous float32/bfloat16/float16 tensor of "
                         f"{B * n_strips} x {rows} x {width} elements on S's device")
    _lib.check(_lib.lib().specenh_strips_pack(
        _code(out), _vp(S), B, F, T, S.stride(0), rows, width, n_strips, _vp(out), _st(S)),
        "strips_pack")


def _pack(S, rows, width, n_strips, dtype):
    out = torch.empty((S.shape[0] * n_strips, rows, width, 1), dtype=dtype, device=S.device)
    _pack_out(S, rows, width, n_strips, out)
    return out


def _unpack_out(strips, rows, width, n_strips, out):
    _need(strips, "strips")
    if strips.shape[0] % n_strips or tuple(strips.shape[1:3]) != (rows, width):
        raise ValueError(f"strips must be [k*{n_strips}, {rows}, {width}(, 1)]")
    B = strips.shape[0] // n_strips
    if (out.numel() != B * rows * n_strips * width or not out.is_contiguous()
            or out.device != strips.device or out.dtype != torch.float32):
        raise ValueError(f"out must be a contiguous float32 tensor of {B} x {rows} x "
                         f"{n_strips * width} elements on the strips' device")
    _lib.check(_lib.lib().specenh_strips_unpack(_code(strips), _vp(strips), B, rows, width,
                                                n_strips, _vp(out), _st(strips)), "strips_unpack")


def _unpack(strips, rows, width, n_strips):
    out = torch.empty((strips.shape[0] // n_strips, rows, n_strips * width), dtype=torch.float32,
                      device=strips.device)
    _unpack_out(strips, rows, width, n_strips, out)
    return out


_op("strips_pack(Tensor S, int rows, int width, int n_strips, ScalarType dtype) -> Tensor", _pack,
    lambda S, rows, width, n_strips, dtype:
    S.new_empty((S.shape[0] * n_strips, rows, width, 1), dtype=dtype))
_op("strips_unpack(Tensor strips, int rows, int width, int n_strips) -> Tensor", _unpack,
    lambda strips, rows, width, n_strips:
    strips.new_empty((strips.shape[0] // n_strips, rows, n_strips * width), dtype=torch.float32))
_op("strips_pack_out(Tensor S, int rows, int width, int n_strips, Tensor(a!) out) -> ()",
    _pack_out, lambda *a: None)
_op("strips_unpack_out(Tensor strips, int rows, int width, int n_strips, Tensor(a!) out) -> ()",
    _unpack_out, lambda *a: None)

ops = torch.ops.specenh
