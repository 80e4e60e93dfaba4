"""keras.layers subset used by the reference model (VAE/manual_scan_3layers.py:186-199):
Input, Conv2D, MaxPooling2D, Conv2DTranspose. Layers are called on symbolic tensors
to build a chain; specenh.keras.models.Model compiles the chain onto the GPU engine."""
from __future__ import annotations

import math
from collections import defaultdict

import numpy as np

from . import utils

_name_counts = defaultdict(int)


def _auto_name(base):
    n = _name_counts[base]
    _name_counts[base] += 1
    return base if n == 0 else f"{base}_{n}"


def _pair(v, what):
    if isinstance(v, int):
        return v, v
    v = tuple(v)
    if len(v) != 2:
        raise ValueError(f"{what} must be an int or a pair")
    return int(v[0]), int(v[1])


class KerasTensor:
    """Symbolic tensor: a shape (None, H, W, C) and the layer that produced it."""

    def __init__(self, shape, layer=None, inbound=None):
        self.shape = tuple(shape)
        self._layer = layer
        self._inbound = inbound

    def __repr__(self):
        return f"<KerasTensor shape={self.shape}>"


class Layer:
    trainable = True

    def __init__(self, name=None, **kwargs):
        unknown = set(kwargs) - {"dtype", "input_shape"}
        if unknown:
            raise TypeError(f"unsupported arguments {sorted(unknown)}")
        self.name = name or _auto_name(self._base_name)
        self.input_shape = None
        self.output_shape = None

    def __call__(self, x):
        if not isinstance(x, KerasTensor):
            raise TypeError("layers are called on symbolic tensors (layers.Input)")
        self.input_shape = x.shape
        self.output_shape = (None,) + self.compute_output_shape(x.shape[1:])
        return KerasTensor(self.output_shape, self, x)

    def count_params(self):
        return 0

    def get_config(self):
        return {"name": self.name}


class InputLayer(Layer):
    _base_name = "input"

    def __init__(self, shape, name=None):
        super().__init__(name=name)
        self.output_shape = (None,) + tuple(shape)

    def get_config(self):
        return {"name": self.name, "shape": list(self.output_shape[1:])}


def Input(shape=None, batch_size=None, name=None, dtype=None, **kwargs):
    """layers.Input(shape=(H, W, C)) (manual_scan_3layers.py:186)."""
    if shape is None or len(shape) != 3:
        raise ValueError("Input shape must be (height, width, channels)")
    lay = InputLayer(tuple(int(s) for s in shape), name=name)
    return KerasTensor(lay.output_shape, lay, None)


_ACTS = (None, "linear", "relu", "sigmoid")


class _ConvBase(Layer):
    def __init__(self, filters, kernel_size, strides, padding, activation, use_bias,
                 kernel_initializer, bias_initializer, name, **kwargs):
        super().__init__(name=name, **kwargs)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size, "kernel_size")
        if self.kernel_size[0] != self.kernel_size[1]:
            raise NotImplementedError("non-square kernels")
        self.strides = _pair(strides, "strides")
        if self.strides[0] != self.strides[1]:
            raise NotImplementedError("anisotropic strides")
        self.padding = padding.lower()
        if activation not in _ACTS:
            raise NotImplementedError(f"activation {activation!r} (supported: {_ACTS})")
        self.activation = activation
        if not use_bias:
            raise NotImplementedError("use_bias=False")
        if kernel_initializer != "glorot_uniform" or bias_initializer != "zeros":
            raise NotImplementedError("only glorot_uniform kernels / zero biases")
        self.use_bias = True
        self.kernel = None
        self.bias = None

    @property
    def k(self):
        return self.kernel_size[0]

    def _glorot(self, shape):
        receptive = shape[0] * shape[1]
        fan_in, fan_out = receptive * shape[2], receptive * shape[3]
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        return utils.rng().uniform(-lim, lim, shape).astype(np.float32)

    def count_params(self):
        cin = self.input_shape[-1]
        return self.k * self.k * cin * self.filters + self.filters

    def get_config(self):
        return {"name": self.name, "filters": self.filters, "kernel_size": list(self.kernel_size),
                "strides": list(self.strides), "padding": self.padding,
                "activation": self.activation}


class Conv2D(_ConvBase):
    """layers.Conv2D(filters, kernel_size, activation=, padding="same") — stride 1."""
    _base_name = "conv2d"

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 name=None, **kwargs):
        super().__init__(filters, kernel_size, strides, padding, activation, use_bias,
                         kernel_initializer, bias_initializer, name, **kwargs)
        if self.strides != (1, 1):
            raise NotImplementedError("Conv2D with strides != 1")
        if self.padding not in ("same", "valid"):
            raise ValueError(f"padding {padding!r}")

    def compute_output_shape(self, s):
        h, w, _ = s
        if self.padding == "valid":
            h, w = h - self.k + 1, w - self.k + 1
        return (h, w, self.filters)

    def build_weights(self):
        cin = self.input_shape[-1]
        self.kernel = self._glorot((self.k, self.k, cin, self.filters))
        self.bias = np.zeros(self.filters, np.float32)


class Conv2DTranspose(_ConvBase):
    """layers.Conv2DTranspose(filters, kernel_size, strides=2, activation=, padding="same")."""
    _base_name = "conv2d_transpose"

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 name=None, output_padding=None, **kwargs):
        super().__init__(filters, kernel_size, strides, padding, activation, use_bias,
                         kernel_initializer, bias_initializer, name, **kwargs)
        if self.padding != "same" or output_padding is not None:
            raise NotImplementedError("Conv2DTranspose supports padding='same' only")
        if self.k < self.strides[0]:
            raise NotImplementedError("Conv2DTranspose with kernel_size < strides")

    def compute_output_shape(self, s):
        h, w, _ = s
        return (h * self.strides[0], w * self.strides[1], self.filters)

    def build_weights(self):
        cin = self.input_shape[-1]
        self.kernel = self._glorot((self.k, self.k, self.filters, cin))  # Keras [k,k,out,in]
        self.bias = np.zeros(self.filters, np.float32)


class MaxPooling2D(Layer):
    """layers.MaxPooling2D((2, 2), padding="same") on even sizes (= 2x2, stride 2)."""
    _base_name = "max_pooling2d"

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.pool_size = _pair(pool_size, "pool_size")
        self.strides = self.pool_size if strides is None else _pair(strides, "strides")
        self.padding = padding.lower()
        if self.pool_size != (2, 2) or self.strides != (2, 2):
            raise NotImplementedError("MaxPooling2D supports pool_size=strides=(2, 2)")

    def compute_output_shape(self, s):
        h, w, c = s
        if h % 2 or w % 2:
            raise NotImplementedError("MaxPooling2D on odd spatial sizes")
        return (h // 2, w // 2, c)

    def get_config(self):
        return {"name": self.name, "pool_size": list(self.pool_size), "padding": self.padding}
