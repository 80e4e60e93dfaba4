"""ctypes binding of libspecenh.so (the C-ABI declared in include/specenh.h).

torch is imported first so that the HIP runtime already mapped by torch
(torch/lib/libamdhip64.so, SONAME libamdhip64.so.7) is the one libspecenh.so
binds to: device pointers and streams from torch are then valid in the library.

There is no fallback: if the library is missing or fails to load, every op
raises ExtensionNotLoaded.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen below; see module docstring)

# SPECENH_LIB: development A/B builds only (tools/build_variant.sh); default = in-tree build
LIB_PATH = os.environ.get("SPECENH_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                         "libspecenh.so")

SPECENH_OK = 0
SPECENH_EINVAL = -1
SPECENH_EUNSUPPORTED = -2
SPECENH_EHIP = -3
SPECENH_ENOMEM = -4
SPECENH_ERANGE = -5
SVD_OPTIMAL = 0
FILTER_NORM = 0
FILTER_RESCALE = 1
FILTER_MEANSUB = 2
SVD_COMPUTE = 1

STFT_LOG = 1
STFT_NORMALIZE = 2
STFT_DROP_NYQUIST = 4
STFT_EXACT = 8  # one frame per FFT (include/specenh.h SPECENH_STFT_EXACT)

DETREND = {False: 0, None: 0, "constant": 1, "c": 1, "linear": 2, "l": 2}
SCALING = {"density": 0, "spectrum": 1}


class ExtensionNotLoaded(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None

# name -> (restype, argtypes); must match include/specenh.h exactly
_c = ctypes
SIGNATURES = {
    "specenh_last_error": (_c.c_char_p, []),
    "specenh_version": (_c.c_char_p, []),
    "specenh_set_variant": (_c.c_int, [_c.c_char_p, _c.c_int]),
    "specenh_get_variant": (_c.c_int, [_c.c_char_p, _c.POINTER(_c.c_int)]),
    "specenh_last_kernel_name": (_c.c_char_p, []),
    "specenh_launch_count": (_c.c_longlong, []),
    "specenh_kernel_name_at": (_c.c_char_p, [_c.c_longlong]),
    "specenh_stream_wait": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int]),
    "specenh_stft_frames": (_c.c_longlong, [_c.c_longlong, _c.c_int, _c.c_int]),
    "specenh_stft_plan_create": (_c.c_int, [_c.POINTER(_c.c_void_p), _c.c_int, _c.c_int,
                                            _c.POINTER(_c.c_double), _c.c_double, _c.c_int,
                                            _c.c_int, _c.c_double]),
    "specenh_stft_plan_destroy": (_c.c_int, [_c.c_void_p]),
    "specenh_stft_workspace_bytes": (_c.c_size_t, [_c.c_void_p, _c.c_longlong]),
    "specenh_stft_psd_f16": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_longlong, _c.c_longlong,
                                        _c.c_longlong, _c.c_void_p, _c.c_int, _c.c_void_p]),
    "specenh_stft_psd": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_longlong, _c.c_longlong,
                                    _c.c_longlong, _c.c_void_p, _c.c_int, _c.c_void_p,
                                    _c.c_void_p]),
    "specenh_csd_plan_create": (_c.c_int, [_c.POINTER(_c.c_void_p), _c.c_int, _c.c_int,
                                           _c.POINTER(_c.c_double), _c.c_double, _c.c_int,
                                           _c.c_int]),
    "specenh_csd_plan_destroy": (_c.c_int, [_c.c_void_p]),
    "specenh_csd": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_longlong,
                               _c.c_longlong, _c.c_longlong, _c.c_longlong, _c.c_void_p, _c.c_int,
                               _c.c_void_p]),
    "specenh_svd_workspace_bytes": (_c.c_size_t, [_c.c_longlong, _c.c_int, _c.c_int, _c.c_int]),
    "specenh_svd_denoise_workspace_bytes": (_c.c_size_t, [_c.c_longlong, _c.c_int, _c.c_int,
                                                          _c.c_int, _c.c_int]),
    "specenh_svd_denoise": (_c.c_int, [_c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                       _c.c_longlong, _c.c_int, _c.c_int, _c.c_void_p,
                                       _c.c_void_p, _c.c_void_p]),
    "specenh_svd_denoise_ex": (_c.c_int, [_c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                          _c.c_longlong, _c.c_int, _c.c_int, _c.c_void_p,
                                          _c.c_int, _c.c_void_p, _c.c_void_p]),
    "specenh_svd_optimal_workspace_bytes": (_c.c_size_t, [_c.c_longlong, _c.c_int, _c.c_int]),
    "specenh_svd_denoise_optimal": (_c.c_int, [_c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                               _c.c_longlong, _c.c_int, _c.c_void_p,
                                               _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                               _c.c_void_p]),
    "specenh_conv2d": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                  _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                                  _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                  _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_int,
                                  _c.c_int, _c.c_void_p, _c.c_void_p]),
    "specenh_conv2d_wgrad": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                        _c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                        _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                        _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                        _c.c_void_p]),
    "specenh_conv2d_wgrad_ex": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                           _c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                           _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                           _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int,
                                           _c.c_void_p, _c.c_void_p]),
    "specenh_conv2d_wgrad_workspace_bytes": (_c.c_size_t, [_c.c_int] * 7),
    "specenh_conv2d_wgrad_pooled": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int,
                                               _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p,
                                               _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                               _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                               _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                               _c.c_void_p]),
    "specenh_conv2d_pooled_in": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                            _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                                            _c.c_int, _c.c_int, _c.c_int, _c.c_void_p, _c.c_int,
                                            _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                                            _c.c_void_p, _c.c_void_p]),
    "specenh_convt_conv_out": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                          _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int,
                                          _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p,
                                          _c.c_void_p]),
    "specenh_convt_conv_out_train": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int,
                                                _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p,
                                                _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p,
                                                _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                                _c.c_void_p]),
    "specenh_decoder3": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                    _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p,
                                    _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p,
                                    _c.c_void_p]),
    "specenh_decoder3_ex": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                       _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p,
                                       _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_int,
                                       _c.c_void_p, _c.c_int, _c.c_void_p]),
    "specenh_encoder2": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                    _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p,
                                    _c.c_int, _c.c_int, _c.c_void_p, _c.c_void_p]),
    "specenh_maxpool2_fwd": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int,
                                        _c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p]),
    "specenh_maxpool2_bwd": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                        _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                                        _c.c_void_p]),
    "specenh_bce_logits": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _c.c_longlong,
                                      _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_void_p]),
    "specenh_adam_step": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                     _c.c_longlong, _c.c_float, _c.c_float, _c.c_float,
                                     _c.c_float, _c.c_float, _c.c_void_p, _c.c_int,
                                     _c.c_void_p]),
    "specenh_adam_step_flip": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                          _c.c_longlong, _c.c_float, _c.c_float, _c.c_float,
                                          _c.c_float, _c.c_float, _c.c_void_p, _c.c_int, _c.c_int,
                                          _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p]),
    "specenh_weight_flip_transpose": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int,
                                                 _c.c_int, _c.c_void_p, _c.c_void_p]),
    "specenh_cast": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_longlong,
                                _c.c_void_p]),
    "specenh_filter_workspace_bytes": (_c.c_size_t, [_c.c_longlong, _c.c_int]),
    "specenh_filter": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _c.c_longlong, _c.c_int,
                                  _c.c_int, _c.c_longlong, _c.c_void_p, _c.c_void_p,
                                  _c.c_void_p]),
    "specenh_quantfilt": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                     _c.c_longlong, _c.c_double, _c.c_void_p, _c.c_void_p]),
    "specenh_u8filter_workspace_bytes": (_c.c_size_t, [_c.c_longlong, _c.c_int, _c.c_int]),
    "specenh_gaussblr": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                    _c.c_longlong, _c.c_int, _c.c_int, _c.c_double, _c.c_void_p,
                                    _c.c_void_p, _c.c_void_p]),
    "specenh_morph": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                 _c.c_longlong, _c.c_void_p, _c.c_void_p, _c.c_void_p]),
    "specenh_strips_pack": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                       _c.c_longlong, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p,
                                       _c.c_void_p]),
    "specenh_strips_unpack": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_longlong, _c.c_int, _c.c_int,
                                         _c.c_int, _c.c_void_p, _c.c_void_p]),
}


def lib():
    """Load (once) and return the ctypes handle; raise ExtensionNotLoaded on failure."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ExtensionNotLoaded(
                f"{LIB_PATH} not found: build it with `python spectrogram-enhancement_amd/build.py` "
                "(there is no CPU fallback)")
        try:
            h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise ExtensionNotLoaded(f"failed to load {LIB_PATH}: {e}") from e
        dev_build = bool(os.environ.get("SPECENH_LIB"))
        for name, (res, args) in SIGNATURES.items():
            if dev_build and not hasattr(h, name):
                continue  # an older revision's build for an A/B run (tools/build_rev_lib.sh)
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def last_error() -> str:
    return lib().specenh_last_error().decode(errors="replace")


def check(rc: int, what: str = "") -> int:
    """Map a C-ABI return code onto the reference's Python exception types."""
    if rc >= 0:
        return rc
    msg = f"{what}: {last_error()}" if what else last_error()
    if rc == SPECENH_EINVAL:
        raise ValueError(msg)
    if rc == SPECENH_EUNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == SPECENH_ENOMEM:
        raise MemoryError(msg)
    if rc == SPECENH_ERANGE:
        raise IndexError(msg)
    raise RuntimeError(msg)


def current_stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def get_variant(name: str) -> int:
    v = ctypes.c_int(0)
    check(lib().specenh_get_variant(name.encode(), ctypes.byref(v)), "get_variant")
    return v.value


def set_variant(name: str, value: int) -> None:
    """Select a kernel variant (runtime.hpp: the A/B switches; SPECENH_<name> in the
    environment sets the process default, read once)."""
    check(lib().specenh_set_variant(name.encode(), int(value)), "set_variant")


class variant:
    """Context manager: ``with _lib.variant("CONV_NO_S2", 1): ...`` restores the old value."""

    def __init__(self, name: str, value: int):
        self.name, self.value = name, int(value)

    def __enter__(self):
        self.old = get_variant(self.name)
        set_variant(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_variant(self.name, self.old)
        return False


def stream_wait(waiter, signaler, device_scope: bool = True) -> None:
    """``waiter`` (torch.cuda.Stream) waits for the work enqueued on ``signaler`` so far, through
    a library event recorded with a device-scope release (specenh_stream_wait)."""
    check(lib().specenh_stream_wait(waiter.cuda_stream, signaler.cuda_stream,
                                    1 if device_scope else 0), "stream_wait")


def last_kernel_name() -> str:
    """Mangled symbol of the last kernel the calling thread launched through the library."""
    return lib().specenh_last_kernel_name().decode(errors="replace")


def launch_count() -> int:
    """Kernels the calling thread has launched through the library so far."""
    return int(lib().specenh_launch_count())


def kernel_names(first: int, end: int) -> list:
    """Symbols of this thread's launches [first, end) (specenh_launch_count numbering)."""
    L = lib()
    return [L.specenh_kernel_name_at(i).decode(errors="replace") for i in range(first, end)]
