"""specenh — MI355X-native spectrogram-enhancement hot path (gfx950, HIP via a C-ABI).

Reference-compatible entry points (same names/arguments as the reference):
  specenh.pipeline_data : specgr, norm, rescale, quantfilt, meansub (+ specgr_batch)
Device fast path:
  specenh.stft.stft_psd / torch.ops.specenh.stft_psd

Importing the package does not touch the GPU; the HIP library is loaded on the
first op call and its absence raises specenh._lib.ExtensionNotLoaded.
"""
__version__ = "0.1.0"


def load_library():
    """Load libspecenh.so now (raises ExtensionNotLoaded if it is missing)."""
    from . import _lib

    return _lib.lib()
