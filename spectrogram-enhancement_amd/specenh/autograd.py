"""Differentiable functional API over the ``torch.ops.specenh`` convolution, pooling and loss
operators: build the reference's autoencoder (or any other chain of its
layers) as ordinary PyTorch code and train it with ``torch.autograd``.

    from specenh import autograd as F
    h = F.conv2d_same(x, W1, b1, "relu")                 # layers.Conv2D(16, 5, "relu", "same")
    h = F.max_pool2(h)                                   # layers.MaxPooling2D((2, 2), "same")
    h = F.conv2d_transpose_same(h, W2, b2, "relu")        # layers.Conv2DTranspose(.., strides=2)
    z = F.conv2d_same(h, W3, b3, None)                    # last layer's logits
    loss = F.binary_crossentropy_with_logits(z, y)        # Keras graph-mode BCE after a sigmoid
    loss.backward()

Tensors are NHWC on the GPU; kernels are Keras-shaped (Conv2D ``[k, k, Cin, Cout]``,
Conv2DTranspose ``[k, k, Cout, Cin]``, VAE/manual_scan_3layers.py:186-199) in the compute
dtype of ``x`` (float32 / bfloat16 / float16); biases float32. Forward and every gradient
are the HIP kernels of csrc/conv_ae.hip (implicit-GEMM conv with fused bias + activation,
deterministic split-K weight gradient, the input gradient as a conv over flipped weights,
maxpool with argmax, BCE from logits); the activation derivative (``dy * (y > 0)`` /
``dy * y (1 - y)``) and the Keras <-> GEMM weight permutation are PyTorch element ops.
The Keras facade (specenh.keras) uses the fused engine in specenh.ae instead, which keeps
all buffers resident and fuses pooling into the convolutions.
"""
from __future__ import annotations

import torch

from .ae import ACT, ConvOp
from .ops import ops


def _to_gemm(kind: str, kernel: torch.Tensor) -> torch.Tensor:
    """Keras kernel -> [CO][KH][KW][C] (differentiable; the inverse permutation on backward)."""
    if kind == "conv":
        return kernel.permute(3, 0, 1, 2).contiguous()
    return kernel.flip(0, 1).permute(2, 0, 1, 3).contiguous()


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_gemm, bias, kind, act):
        k, cout, cin = w_gemm.shape[1], w_gemm.shape[0], w_gemm.shape[3]
        op = ConvOp(kind, cin, cout, k, act, stride=2 if kind == "convT" else 1)
        if x.dim() != 4 or x.shape[3] != cin:
            raise ValueError(f"x must be NHWC with {cin} channels")
        x = x.contiguous()
        oh, ow = op.out_hw(x.shape[1], x.shape[2])
        s, pt, pl, dil = op.fwd_geom()
        y = ops.conv2d(x, w_gemm.to(x.dtype).contiguous(), bias, k, k, cout, s, pt, pl, dil, oh,
                       ow, ACT[act])
        ctx.op = op
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, w_gemm, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_gemm, y = ctx.saved_tensors
        op = ctx.op
        if op.act == "relu":
            dz = dy * (y > 0)
        elif op.act == "sigmoid":
            yf = y.float()
            dz = dy.float() * yf * (1.0 - yf)
        else:
            dz = dy
        dz = dz.to(x.dtype).contiguous()
        s, pt, pl, dil = op.fwd_geom()
        dw, db = ops.conv2d_wgrad(x, dz, op.k, op.k, s, pt, pl, dil)
        dx = None
        if ctx.needs_input_grad[0]:
            wd = ops.weight_flip_transpose(w_gemm.to(x.dtype).contiguous(), op.k, op.cin, op.cout)
            s2, pt2, pl2, dil2 = op.dgrad_geom()
            dx = ops.conv2d(dz, wd, None, op.k, op.k, op.cin, s2, pt2, pl2, dil2, x.shape[1],
                            x.shape[2], ACT[None])
        return dx, dw.to(w_gemm.dtype), (db if ctx.has_bias else None), None, None


def conv2d_same(x, kernel, bias=None, activation=None):
    """layers.Conv2D(filters, k, activation, padding="same") on NHWC x; kernel [k, k, Cin, Cout]."""
    return _Conv.apply(x, _to_gemm("conv", kernel), bias, "conv", activation)


def conv2d_transpose_same(x, kernel, bias=None, activation=None):
    """layers.Conv2DTranspose(filters, k, strides=2, activation, padding="same");
    kernel [k, k, Cout, Cin]."""
    if kernel.shape[0] < 2:
        raise NotImplementedError("Conv2DTranspose with kernel_size < strides")
    return _Conv.apply(x, _to_gemm("convT", kernel), bias, "convT", activation)


class _Pool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        if x.shape[1] % 2 or x.shape[2] % 2:
            raise NotImplementedError("MaxPooling2D on odd spatial sizes")
        y, am = ops.maxpool2(x.contiguous())
        ctx.save_for_backward(am)
        ctx.mark_non_differentiable(am)
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        return ops.maxpool2_bwd(dy.contiguous(), am, None)


def max_pool2(x):
    """layers.MaxPooling2D((2, 2), padding="same") on even H, W (NHWC)."""
    return _Pool.apply(x)


class _BCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, target):
        if z.dtype != torch.float32:
            raise TypeError("logits must be float32")
        loss_sum, grad = ops.bce_logits(z.contiguous(), target.contiguous(), torch.float32)
        ctx.save_for_backward(grad)
        return (loss_sum / z.numel()).to(torch.float32).reshape(())

    @staticmethod
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        return grad * gout, None


def binary_crossentropy_with_logits(z, target):
    """compile(loss="binary_crossentropy") after a sigmoid layer, as Keras evaluates it in graph
    mode: mean over all elements of max(z, 0) - z t + log1p(exp(-|z|)) from the logits z.
    bfloat16 / float16 logits (a low-precision last layer) are widened to float32 first, as
    Keras' mixed-precision policy computes the loss in float32; the gradient flows back
    through the cast in z's dtype."""
    if z.dtype != torch.float32:
        z = z.float()
    return _BCE.apply(z, target)
