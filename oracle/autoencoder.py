"""ORACLE (test infrastructure only): PyTorch-CPU restatement of the Keras conv autoencoder.

PARITY UNPINNED: TensorFlow/Keras are not installed and the trained model
(VAE/best_model) is absent, so no reference-side fixture exists. This file restates
the Keras semantics the reference relies on (VAE/manual_scan_3layers.py:186-212;
variants manual_scan.py:190-213, hyperparam_scan.py:153-184, graphs.ipynb:234-278):

* NHWC tensors, ``layers.Conv2D(f, k, activation, padding="same")`` (stride 1, TF SAME:
  pad_top = (k-1)//2, pad_bottom = k-1-pad_top), kernel HWIO ``[k, k, Cin, Cout]``.
* ``layers.MaxPooling2D((2, 2), padding="same")`` on even sizes = 2x2/2 max pool.
* ``layers.Conv2DTranspose(f, k, strides=2, padding="same")``: the gradient of a
  stride-2 SAME conv; equals ``conv_transpose2d(stride=2, padding=(k-2)//2)`` with the
  trailing row/column cropped; kernel ``[k, k, Cout, Cin]`` (SURVEY.md §7 hard parts).
* ``compile(optimizer="adam", loss="binary_crossentropy")``: in graph mode Keras
  computes BCE from the pre-sigmoid logits (``sigmoid_cross_entropy_with_logits``),
  mean over all elements; Adam lr=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-7 (Keras
  form ``w -= lr_t * m / (sqrt(v) + eps)``, ``lr_t = lr*sqrt(1-b2^t)/(1-b1^t)``).
* ``glorot_uniform`` kernels, zero biases.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# layer spec: ("conv", Cin, Cout, k, act) | ("pool",) | ("convT", Cin, Cout, k, act)


def ae_spec(conv1=16, conv2=32, conv3=64, k=5, layers3=True):
    """The 3-layer AE of manual_scan_3layers.py:186-199 (2-layer variants drop conv3)."""
    if layers3:
        return [("conv", 1, conv1, k, "relu"), ("pool",), ("conv", conv1, conv2, k, "relu"),
                ("pool",), ("conv", conv2, conv3, k, "relu"), ("pool",),
                ("convT", conv3, conv3, k, "relu"), ("convT", conv3, conv2, k, "relu"),
                ("convT", conv2, conv1, k, "relu"), ("conv", conv1, 1, k, "sigmoid")]
    return [("conv", 1, conv1, k, "relu"), ("pool",), ("conv", conv1, conv2, k, "relu"),
            ("pool",), ("convT", conv2, conv2, k, "relu"), ("convT", conv2, conv1, k, "relu"),
            ("conv", conv1, 1, k, "sigmoid")]


def glorot_params(spec, seed=0):
    """Keras-shaped parameters: conv W[k,k,Cin,Cout], convT W[k,k,Cout,Cin], zero biases."""
    rng = np.random.default_rng(seed)
    params = []
    for layer in spec:
        if layer[0] == "pool":
            params.append(None)
            continue
        kind, cin, cout, k, _ = layer
        shape = (k, k, cin, cout) if kind == "conv" else (k, k, cout, cin)
        fan_in, fan_out = k * k * shape[2], k * k * shape[3]
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        params.append({"W": rng.uniform(-lim, lim, shape).astype(np.float32),
                       "b": np.zeros(cout, np.float32)})
    return params


def _same_pads(k):
    t = (k - 1) // 2
    return t, k - 1 - t


def conv2d_same(x, W, b):
    """x NHWC, W [k,k,Cin,Cout] -> NHWC (stride 1, TF SAME)."""
    k = W.shape[0]
    t, bo = _same_pads(k)
    xt = F.pad(x.permute(0, 3, 1, 2), (t, bo, t, bo))
    y = F.conv2d(xt, W.permute(3, 2, 0, 1).contiguous(), b)
    return y.permute(0, 2, 3, 1)


def conv2d_transpose_same(x, W, b):
    """x NHWC [N,H,W,Cin], W [k,k,Cout,Cin] -> NHWC [N,2H,2W,Cout] (stride 2, TF SAME)."""
    k = W.shape[0]
    p = (k - 2) // 2
    y = F.conv_transpose2d(x.permute(0, 3, 1, 2), W.permute(3, 2, 0, 1).contiguous(), b, stride=2,
                           padding=p)
    H, Wd = 2 * x.shape[1], 2 * x.shape[2]
    return y[:, :, :H, :Wd].permute(0, 2, 3, 1)


def maxpool2(x):
    return F.max_pool2d(x.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)


def forward(spec, params, x, return_logits=False):
    """x NHWC float tensor -> sigmoid output (and the final pre-activation)."""
    h = x
    z = None
    for layer, p in zip(spec, params):
        if layer[0] == "pool":
            h = maxpool2(h)
            continue
        W = torch.as_tensor(p["W"]) if not isinstance(p["W"], torch.Tensor) else p["W"]
        b = torch.as_tensor(p["b"]) if not isinstance(p["b"], torch.Tensor) else p["b"]
        z = conv2d_same(h, W, b) if layer[0] == "conv" else conv2d_transpose_same(h, W, b)
        h = torch.relu(z) if layer[4] == "relu" else torch.sigmoid(z)
    return (h, z) if return_logits else h


def bce_from_logits(z, t):
    """Keras graph-mode binary_crossentropy after a sigmoid layer (mean over all elements)."""
    return (torch.clamp(z, min=0) - z * t + torch.log1p(torch.exp(-torch.abs(z)))).mean()


class KerasAdam:
    def __init__(self, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7):
        self.lr, self.b1, self.b2, self.eps, self.t = lr, b1, b2, eps, 0
        self.m, self.v = {}, {}

    def step(self, named):
        self.t += 1
        lr_t = self.lr * math.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        with torch.no_grad():
            for name, p in named:
                g = p.grad
                m = self.m.setdefault(name, torch.zeros_like(p))
                v = self.v.setdefault(name, torch.zeros_like(p))
                m.mul_(self.b1).add_(g, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                p.sub_(lr_t * m / (v.sqrt() + self.eps))


def train_step(spec, params, x, y, opt: KerasAdam):
    """One Keras fit() step (forward, BCE, backward, Adam); params updated in place
    (torch tensors with requires_grad). Returns the loss."""
    named = []
    for i, p in enumerate(params):
        if p is None:
            continue
        named += [(f"{i}.W", p["W"]), (f"{i}.b", p["b"])]
    for _, t in named:
        t.grad = None
    _, z = forward(spec, params, x, return_logits=True)
    loss = bce_from_logits(z, y)
    loss.backward()
    opt.step(named)
    return float(loss)
