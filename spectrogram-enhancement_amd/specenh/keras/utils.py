"""keras.utils subset."""
import numpy as np

_rng = np.random.default_rng()


def set_random_seed(seed):
    """Seed the host RNG used for glorot_uniform initialisation and fit() shuffling."""
    global _rng
    _rng = np.random.default_rng(seed)


def rng():
    return _rng
