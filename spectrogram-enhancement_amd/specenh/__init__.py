"""specenh — MI355X-native spectrogram-enhancement hot path (gfx950, HIP via a C-ABI).

Reference-compatible entry points (same names/arguments as the reference):
  specenh.pipeline_data : specgr, norm, rescale, quantfilt, gaussblr, meansub, morph
  specenh.svd           : omega, denoiseSignal, computeSignal
  specenh.strips        : patch, unpatch, reshape
  specenh.keras         : layers / Model / compile / fit / predict / save / load_model
Device fast paths: specgr_batch, denoise_batch, cross_spectrogram_batch, and
specenh.autograd (differentiable Conv2D / Conv2DTranspose / MaxPooling2D / BCE).
Every one of them reaches the HIP kernels through the ``torch.ops.specenh`` operators
(specenh/ops.py, registered when the package is imported) and the C-ABI.

Importing the package does not touch the GPU; the HIP library is loaded on the
first op call and its absence raises specenh._lib.ExtensionNotLoaded.
"""
__version__ = "0.2.0"

from . import ops  # noqa: E402,F401  (registers torch.ops.specenh.*)


def load_library():
    """Load libspecenh.so now (raises ExtensionNotLoaded if it is missing)."""
    from . import _lib

    return _lib.lib()
