"""Keras-shaped facade over the MI355X conv-autoencoder engine (specenh.ae).

The reference builds and trains its model with
    from keras import layers
    from keras.models import Model, load_model
    from keras.callbacks import EarlyStopping          (VAE/manual_scan_3layers.py:21-25)
A notebook switches by importing the same names from here:
    from specenh.keras import layers
    from specenh.keras.models import Model, load_model
    from specenh.keras.callbacks import EarlyStopping
Supported graph: a single chain of Input -> Conv2D / MaxPooling2D / Conv2DTranspose
(the only layers the reference uses, manual_scan_3layers.py:186-199; manual_scan.py
:190-199; hyperparam_scan.py:153-164), compiled with optimizer "adam" and loss
"binary_crossentropy". Everything runs on the GPU; there is no CPU fallback.
"""
from . import callbacks, layers, mixed_precision, models, optimizers, utils  # noqa: F401
from .models import Model, load_model  # noqa: F401
