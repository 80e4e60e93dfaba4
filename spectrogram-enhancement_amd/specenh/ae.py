"""Device engine of the convolutional autoencoder (VAE/manual_scan_3layers.py:186-212).

The Keras facade (specenh.keras) builds a chain of layers and hands it to
:class:`AutoencoderEngine`, which owns every device buffer and sequences the kernels of
csrc/conv_ae.hip through the ``torch.ops.specenh`` operators (specenh/ops.py):

* forward   Conv2D / Conv2DTranspose = implicit-GEMM conv (+bias, relu/sigmoid fused),
            MaxPooling2D = maxpool2 with argmax;
* loss      binary_crossentropy from the last layer's fp32 logits (Keras graph mode);
* backward  per conv layer: wgrad (+bias grad) and, except for the first layer, the
            input gradient as another implicit-GEMM conv over flipped/transposed weights
            whose epilogue applies the previous ReLU's mask; pools route through argmax
            with the ReLU mask fused;
* update    one Keras-Adam launch over ONE flat fp32 parameter buffer (GEMM layout), which
            also refreshes the bf16 copy the MFMA kernels read; a data-parallel run
            all-reduces the ONE flat gradient buffer (RCCL) before it.

Weights live in "GEMM layout" Bt[co][(ky, kx, ci)] such that the forward pass is
out[m][co] = sum_k A[m][k] Bt[co][k]. For Conv2D this is the Keras HWIO kernel with the
output channel moved first; for Conv2DTranspose (Keras kernel [k, k, Cout, Cin]) it is
kernel[::-1, ::-1] with Cout moved first. Adam is elementwise, so it runs on this
layout directly.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .ops import decoder3_supported, encoder2_supported, ops, tail_supported

F32, BF16, F16 = 0, 1, 2
_DTYPES = {"float32": F32, "bfloat16": BF16, "bf16": BF16, "mixed_bfloat16": BF16,
           "float16": F16, "fp16": F16, "mixed_float16": F16}
_TORCH = {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16}
ACT = {None: 0, "linear": 0, "relu": 1, "sigmoid": 2}
_ALIGN = 64  # elements; keeps every layer's GEMM weights 16-byte aligned for bf16 x8 loads


@dataclass
class ConvOp:
    """One Conv2D (kind "conv") or Conv2DTranspose ("convT") in GEMM form."""
    kind: str
    cin: int
    cout: int
    k: int
    act: str | None
    stride: int = 1          # Conv2DTranspose stride (upsampling factor)
    padding: str = "same"    # Conv2D: "same" | "valid"
    off_w: int = 0           # offsets into the flat parameter buffer (elements)
    off_b: int = 0

    @property
    def n_w(self):
        return self.k * self.k * self.cin * self.cout

    def out_hw(self, h, w):
        if self.kind == "convT":
            return h * self.stride, w * self.stride
        if self.padding == "valid":
            return h - self.k + 1, w - self.k + 1
        return h, w

    def fwd_geom(self):
        """(stride, pad_t, pad_l, in_dil) of the forward implicit GEMM."""
        k = self.k
        if self.kind == "conv":
            p = 0 if self.padding == "valid" else (k - 1) // 2
            return 1, p, p, 1
        pt = max(k - self.stride, 0) // 2              # TF SAME for the transposed conv
        return 1, k - 1 - pt, k - 1 - pt, self.stride  # conv over the dilated input

    def dgrad_geom(self):
        """(stride, pad_t, pad_l, in_dil) of the input gradient as a conv over dOut."""
        k = self.k
        if self.kind == "conv":
            p = 0 if self.padding == "valid" else (k - 1) // 2
            return 1, k - 1 - p, k - 1 - p, 1
        pt = max(k - self.stride, 0) // 2
        return self.stride, pt, pt, 1


@dataclass
class PoolOp:
    kind: str = "pool"


def keras_to_gemm(op: ConvOp, kernel: np.ndarray) -> np.ndarray:
    """Keras kernel -> Bt[co][(ky, kx, ci)] (flattened fp32, N-major GEMM operand)."""
    kernel = np.asarray(kernel, dtype=np.float32)
    if op.kind == "conv":
        assert kernel.shape == (op.k, op.k, op.cin, op.cout), kernel.shape
        return np.ascontiguousarray(kernel.transpose(3, 0, 1, 2)).reshape(-1)
    assert kernel.shape == (op.k, op.k, op.cout, op.cin), kernel.shape
    return np.ascontiguousarray(kernel[::-1, ::-1].transpose(2, 0, 1, 3)).reshape(-1)


def gemm_to_keras(op: ConvOp, flat: np.ndarray) -> np.ndarray:
    bt = np.asarray(flat, dtype=np.float32).reshape(op.cout, op.k, op.k, op.cin)
    if op.kind == "conv":
        return np.ascontiguousarray(bt.transpose(1, 2, 3, 0))
    return np.ascontiguousarray(bt[:, ::-1, ::-1, :].transpose(1, 2, 0, 3))


class AutoencoderEngine:
    """Device state + kernel sequencing for a chain of Conv/Pool/ConvT layers."""

    def __init__(self, ops, input_shape, compute_dtype="float32", device=None):
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("specenh requires a ROCm GPU (HIP); there is no CPU fallback")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("specenh.ae runs on the GPU only (no CPU fallback)")
        self.L = _lib.lib()
        self.ops = list(ops)
        self.input_shape = tuple(input_shape)  # (H, W, C)
        if compute_dtype not in _DTYPES:
            raise ValueError(f"compute dtype {compute_dtype!r} (choose from {sorted(_DTYPES)})")
        self.dt = _DTYPES[compute_dtype]
        self.tdt = _TORCH[self.dt]
        self._validate()
        off = 0
        for op in self.ops:
            if isinstance(op, ConvOp):
                op.off_w = off
                off += -(-op.n_w // _ALIGN) * _ALIGN
                op.off_b = off
                off += -(-op.cout // _ALIGN) * _ALIGN
        self.n_flat = off
        dev = self.device
        self.w = torch.zeros(off, dtype=torch.float32, device=dev)   # fp32 master weights
        self.g = torch.zeros(off, dtype=torch.float32, device=dev)   # gradients
        self.m = torch.zeros(off, dtype=torch.float32, device=dev)   # Adam moments
        self.v = torch.zeros(off, dtype=torch.float32, device=dev)
        self.w_lp = torch.zeros(off, dtype=self.tdt, device=dev) if self.dt != F32 else None
        # flipped/transposed copies for the input gradients (compute dtype)
        self.w_d = {i: torch.zeros(op.n_w, dtype=self.tdt, device=dev)
                    for i, op in enumerate(self.ops) if isinstance(op, ConvOp) and i > 0}
        # conv i followed by MaxPooling2D: one launch (bf16/f16 LDS-patch kernel)
        # (not when the pool is the model's output: that buffer is fp32 for inference)
        self.fused = {i for i, op in enumerate(self.ops[:-2])
                      if self.dt != F32 and isinstance(op, ConvOp) and op.kind == "conv"
                      and isinstance(self.ops[i + 1], PoolOp) and op.k <= 7
                      and (op.cin in (1, 16) or op.cin % 32 == 0)}
        # inference: the last Conv2DTranspose(relu) + Conv2D(1, sigmoid) as one launch
        # (csrc/decoder_tail.hip); its 16-channel map never reaches HBM
        last2 = self.ops[-2:] if len(self.ops) >= 2 else []
        self.tail = (len(last2) == 2 and all(isinstance(o, ConvOp) for o in last2)
                     and last2[0].kind == "convT" and last2[0].act == "relu"
                     and last2[0].stride == 2 and last2[1].kind == "conv"
                     and last2[1].cout == 1 and last2[1].act == "sigmoid"
                     and last2[1].padding == "same"
                     and tail_supported(self.tdt, last2[0].cin, last2[0].cout, last2[0].k,
                                        last2[1].k, self.shapes()[len(self.ops) - 2][1])
                     and os.environ.get("SPECENH_NO_TAIL_FUSION", "0") in ("", "0"))
        # training: the same two layers as one row-sweep launch that also stores the map (the
        # backward's mask and weight-gradient input), the logits and the output
        # (decoder_tail.hip tail_rows_kernel<T, true>), at 64-position-wide inputs
        self.tail_train = (self.tail and self.shapes()[len(self.ops) - 2][1] == 64
                           and (last2[0].cin, last2[0].cout, last2[0].k, last2[1].k)
                           == (32, 16, 5, 5)
                           and os.environ.get("SPECENH_NO_TAIL_TRAIN", "0") in ("", "0"))
        # inference: the last THREE layers (Conv2DTranspose x2 + Conv2D(1)) as one launch
        # (csrc/decoder_tail.hip decoder3_kernel) when the shapes are the reference model's
        # at 128-wide inputs; both intermediate maps stay in LDS
        self.dec3 = False
        if self.tail and len(self.ops) >= 3 and isinstance(self.ops[-3], ConvOp):
            o3 = self.ops[-3]
            w_in = self.shapes()[len(self.ops) - 3][1]
            self.dec3 = (o3.kind == "convT" and o3.act == "relu" and o3.stride == 2
                         and decoder3_supported(self.tdt, o3.cin, o3.cout, self.ops[-2].cout,
                                                o3.k, w_in)
                         and o3.k == self.ops[-2].k == self.ops[-1].k
                         and _lib.get_variant("DECODER_UNFUSED") == 0)
        # inference: the FIRST two layers (Conv2D + pool, Conv2D + pool) as one launch
        # (csrc/conv_rows.hip enc2_rows_kernel) on the reference model's 128-wide one-channel
        # inputs; the pooled 16-channel map between them stays in LDS
        self.enc2 = False
        if len(self.ops) >= 4 and 0 in self.fused and 2 in self.fused:
            o1, o2 = self.ops[0], self.ops[2]
            self.enc2 = (o1.kind == o2.kind == "conv" and o1.act == o2.act == "relu"
                         and o1.padding == o2.padding == "same" and o1.k == o2.k
                         and o2.cin == o1.cout
                         and encoder2_supported(self.tdt, o1.cin, o1.cout, o2.cout, o1.k,
                                                self.input_shape[0], self.input_shape[1])
                         and _lib.get_variant("ENCODER_UNFUSED") == 0)
        # training: the first Conv2D's weight gradient straight from its pool's gradient
        # (specenh_conv2d_wgrad_pooled: no full-resolution pool-backward output)
        c0 = self.ops[0] if self.ops else None
        self.wgrad_pooled = (self.dt != F32 and isinstance(c0, ConvOp) and c0.kind == "conv"
                             and c0.cin == 1 and c0.cout % 8 == 0 and c0.stride == 1
                             and c0.k <= 5 and c0.act in (None, "linear", "relu")
                             and len(self.ops) > 1
                             and isinstance(self.ops[1], PoolOp)
                             and self.input_shape[0] % 2 == 0 and self.input_shape[1] % 2 == 0
                             and os.environ.get("SPECENH_NO_WGRAD_POOLED", "0") in ("", "0"))
        # training (round 6): the other pooled Conv2Ds' weight AND input gradients straight
        # from their pool's gradient (specenh_conv2d_wgrad_pooled, specenh_conv2d_pooled_in:
        # argmax select + ReLU mask while the tiles / patches are staged), so the pool backward
        # launch and its full-resolution gradient are gone from the input-gradient chain.
        # SPECENH_NO_POOL_ROUTED=1: the pool backward + plain conv launches (bitwise the same)
        self.pool_routed = set()
        if self.dt != F32 and os.environ.get("SPECENH_NO_POOL_ROUTED", "0") in ("", "0"):
            hw = self.input_shape[:2]
            for i, op in enumerate(self.ops):
                nxt = self.ops[i + 1] if i + 1 < len(self.ops) else None
                if (i > 0 and isinstance(op, ConvOp) and op.kind == "conv" and op.stride == 1
                        and op.padding == "same" and op.cin % 16 == 0 and op.cout % 16 == 0
                        and op.k <= 7 and op.act in (None, "linear", "relu")
                        and isinstance(nxt, PoolOp) and hw[0] % 2 == 0 and hw[1] % 2 == 0):
                    self.pool_routed.add(i)
                hw = op.out_hw(*hw) if isinstance(op, ConvOp) else (hw[0] // 2, hw[1] // 2)
        self.t = 0  # Adam iterations
        # backward: weight gradients on a second stream, off the input-gradient chain
        # (SPECENH_WGRAD_SERIAL=1: one stream, the round-4 order)
        self.wgrad_overlap = os.environ.get("SPECENH_WGRAD_SERIAL", "0") in ("", "0")
        # round 6: the weight gradients alternate over this many side streams (the side chain
        # of one stream had become the step's critical path at batch 128), and every layer's
        # weight gradient OVERWRITES its slice of self.g (no zeroing launches; the slices'
        # alignment padding is never written and stays zero). SPECENH_WGRAD_STREAMS=1 and
        # SPECENH_WGRAD_ACCUM=1 restore the round-5 schedule.
        self.wgrad_streams = max(1, int(os.environ.get("SPECENH_WGRAD_STREAMS", "2") or 2))
        self.wgrad_overwrite = os.environ.get("SPECENH_WGRAD_ACCUM", "0") in ("", "0")
        self._sides = None
        # fork / join of the weight-gradient stream: "device" (library events with a
        # device-scope release, the default), "system" (library events, system-scope
        # fence), "torch" (torch.cuda.Stream.wait_stream)
        self.fork_mode = os.environ.get("SPECENH_FORK", "device")
        self._bufs = {}
        self.infer_out_dtype = torch.float32  # set_inference_output_dtype
        self._loss = torch.zeros(1, dtype=torch.float64, device=dev)
        # per-layer views into the flat buffers (the operators take tensors, not offsets)
        lp = self.w_lp if self.dt != F32 else self.w
        self._wv, self._bv, self._gwv, self._gbv = {}, {}, {}, {}
        for i, op in enumerate(self.ops):
            if isinstance(op, ConvOp):
                self._wv[i] = lp[op.off_w:op.off_w + op.n_w]
                self._bv[i] = self.w[op.off_b:op.off_b + op.cout]
                self._gwv[i] = self.g[op.off_w:op.off_w + op.n_w]
                self._gbv[i] = self.g[op.off_b:op.off_b + op.cout]

    # ------------------------------------------------------------------ shapes
    def _validate(self):
        convs = [op for op in self.ops if isinstance(op, ConvOp)]
        if not convs:
            raise ValueError("model has no convolution layers")
        h, w, c = self.input_shape
        for i, op in enumerate(self.ops):
            if isinstance(op, PoolOp):
                if h % 2 or w % 2:
                    raise NotImplementedError("MaxPooling2D on odd spatial sizes")
                h, w = h // 2, w // 2
                continue
            if op.cin != c:
                raise ValueError(f"layer {i}: expects {op.cin} channels, gets {c}")
            if op.act not in ACT:
                raise NotImplementedError(f"activation {op.act!r}")
            if op.kind == "convT" and op.k < op.stride:
                raise NotImplementedError("Conv2DTranspose with kernel_size < strides")
            h, w = op.out_hw(h, w)
            if h <= 0 or w <= 0:
                raise ValueError(f"layer {i}: output size {h}x{w}")
            c = op.cout
        self.output_shape = (h, w, c)

    def shapes(self):
        """Per-op input shapes (H, W, C) plus the final output shape."""
        out = []
        h, w, c = self.input_shape
        for op in self.ops:
            out.append((h, w, c))
            if isinstance(op, PoolOp):
                h, w = h // 2, w // 2
            else:
                h, w = op.out_hw(h, w)
                c = op.cout
        out.append((h, w, c))
        return out

    def set_inference_output_dtype(self, dtype):
        """Precision of forward(train=False)'s output: float32 (default, what Keras predict
        returns) or float16 — BASELINE config 5's fp16 reconstructions (32,768 B per 128 x 128
        shot), stored by the fused three-layer decoder (decoder3) itself."""
        if dtype not in (torch.float32, torch.float16):
            raise ValueError("inference output dtype must be torch.float32 or torch.float16")
        if dtype != torch.float32 and not self.dec3:
            raise NotImplementedError("fp16 inference output needs the fused three-layer decoder")
        if dtype != self.infer_out_dtype:
            self.infer_out_dtype = dtype
            self._bufs = {k: v for k, v in self._bufs.items() if k[1]}  # drop inference buffers

    def _buffers(self, N, train):
        key = (N, train)
        b = self._bufs.get(key)
        if b is not None:
            return b
        dev, shp = self.device, self.shapes()
        b = {"h": [None] * (len(self.ops) + 1), "am": [None] * len(self.ops),
             "d": [None] * (len(self.ops) + 1)}
        for i in range(1, len(self.ops) + 1):
            H, W, C = shp[i]
            last = i == len(self.ops)
            dtype = self.infer_out_dtype if (last and not train) else self.tdt
            tail_map = not train and ((self.tail and i == len(self.ops) - 1) or
                                      (self.dec3 and i == len(self.ops) - 2) or
                                      (self.enc2 and i == 2))  # maps kept in LDS
            if (i - 1) not in self.fused and not tail_map:  # never-stored fused outputs
                b["h"][i] = torch.empty((N, H, W, C), dtype=dtype, device=dev)
            if train:
                b["d"][i] = torch.empty((N, H, W, C), dtype=self.tdt, device=dev)
        for i, op in enumerate(self.ops):
            if isinstance(op, PoolOp) and train:
                H, W, C = shp[i + 1]
                b["am"][i] = torch.empty((N, H, W, C), dtype=torch.uint8, device=dev)
        if train:
            H, W, C = shp[-1]
            b["z"] = torch.empty((N, H, W, C), dtype=torch.float32, device=dev)
            ws = 16
            for i, op in enumerate(self.ops):
                if isinstance(op, ConvOp):
                    OH, OW, _ = shp[i + 1]
                    ws = max(ws, int(self.L.specenh_conv2d_wgrad_workspace_bytes(
                        N, OH, OW, op.k, op.k, op.cin, op.cout)))
            b["ws"] = torch.empty(ws, dtype=torch.uint8, device=dev)
            # one more per extra weight-gradient stream
            b["wss"] = [b["ws"]] + [torch.empty(ws, dtype=torch.uint8, device=dev)
                                    for _ in range(self.wgrad_streams - 1)]
            # the first convolution's weight gradient runs on the current stream beside the
            # second stream's last ones (backward): a workspace of its own
            first = next((i for i, op in enumerate(self.ops) if isinstance(op, ConvOp)), None)
            ws0 = 16
            if first is not None:
                op = self.ops[first]
                OH, OW, _ = shp[first + 1]
                ws0 = max(ws0, int(self.L.specenh_conv2d_wgrad_workspace_bytes(
                    N, OH, OW, op.k, op.k, op.cin, op.cout)))
            b["ws0"] = torch.empty(ws0, dtype=torch.uint8, device=dev)
        if len(self._bufs) >= 4:  # e.g. full + partial batch for train and inference
            self._bufs.pop(next(iter(self._bufs)))
        self._bufs[key] = b
        return b

    # ------------------------------------------------------------------ weights
    def set_keras_weights(self, weights):
        """weights: [kernel0, bias0, kernel1, bias1, ...] in Keras shapes."""
        convs = [op for op in self.ops if isinstance(op, ConvOp)]
        if len(weights) != 2 * len(convs):
            raise ValueError(f"expected {2 * len(convs)} arrays, got {len(weights)}")
        host = np.zeros(self.n_flat, dtype=np.float32)
        for j, op in enumerate(convs):
            host[op.off_w:op.off_w + op.n_w] = keras_to_gemm(op, weights[2 * j])
            b = np.asarray(weights[2 * j + 1], dtype=np.float32).reshape(-1)
            if b.shape[0] != op.cout:
                raise ValueError("bias shape")
            host[op.off_b:op.off_b + op.cout] = b
        self.w.copy_(torch.from_numpy(host))
        self._refresh_lowp()

    def get_keras_weights(self):
        host = self.w.cpu().numpy()
        out = []
        for op in self.ops:
            if isinstance(op, ConvOp):
                out.append(gemm_to_keras(op, host[op.off_w:op.off_w + op.n_w]))
                out.append(host[op.off_b:op.off_b + op.cout].copy())
        return out

    def _refresh_lowp(self):
        if self.dt != F32:
            ops.cast_out(self.w, self.w_lp)
        for i, wd in self.w_d.items():
            op = self.ops[i]
            ops.weight_flip_transpose_out(self._wv[i], op.k, op.cin, op.cout, wd)

    # ------------------------------------------------------------------ passes
    def _conv(self, i, x, out, *, weights, geom, act, mask=None, logits=None, bias=True,
              out_shape=None, cout=None, pool=False, argmax=None):
        op = self.ops[i]
        OH, OW = out_shape
        s, pt, pl, dil = geom
        ops.conv2d_out(x, weights, self._bv[i] if bias else None, op.k, op.k, cout, s, pt, pl,
                       dil, OH, OW, ACT[act], mask, logits, out, pool, argmax)

    def forward(self, x, train=False, timing=None, kernels=None):
        """x: device [N, H, W, C] in the compute dtype. Returns the output buffer
        (fp32 for inference, compute dtype for training; reused between calls), except for
        an inference batch above the int32 element cap of one launch: that batch runs in
        consecutive slices and the result is a newly allocated tensor.
        ``timing``: optional list; a (start, end) pair of torch.cuda.Event recorded on the
        launch stream is appended around every convolution launch. ``kernels``: optional
        list; the symbol of each such launch's kernel is appended (the key of its PMC
        record, tools/pmc_fold.py). Neither can be given with a batch above the cap (one
        launch per layer is what they describe): ValueError."""
        N = x.shape[0]
        if x.dtype != self.tdt or not x.is_contiguous() or tuple(x.shape[1:]) != self.input_shape:
            raise ValueError(f"forward expects a contiguous {self.tdt} [N, *{self.input_shape}]")
        # one launch addresses at most 2^31 - 1 elements of a tensor: larger inference batches
        # (e.g. the 64-channel manual_scan.py model at 256 x 128) run in consecutive slices
        per = max(h * w * c for h, w, c in self.shapes())
        cap = (2 ** 31 - 1) // per
        if N > cap and (timing is not None or kernels is not None):
            raise ValueError(f"batch {N} exceeds one launch's int32 element cap ({cap} samples "
                             f"of this model): it cannot be timed or profiled as one launch "
                             f"per layer; pass at most {cap} samples")
        if N > cap and not train:
            out = None
            for s0 in range(0, N, cap):
                y = self.forward(x[s0:s0 + cap])
                if out is None:
                    out = torch.empty((N,) + tuple(y.shape[1:]), dtype=y.dtype, device=y.device)
                out[s0:s0 + y.shape[0]].copy_(y)
            return out
        b = self._buffers(N, train)
        b["h"][0] = x
        if train:
            self._last_train_N = N
        n_ops = len(self.ops)
        skip = False
        start = 0
        if self.enc2 and not train:  # conv1 + pool + conv2 + pool, one launch
            if timing is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(torch.cuda.current_stream(self.device))
            o1, o2 = self.ops[0], self.ops[2]
            ops.encoder2_out(x, self._wv[0], self._bv[0], o1.cout, self._wv[2], self._bv[2],
                             o2.cout, o1.k, b["h"][4])
            if timing is not None:
                ev[1].record(torch.cuda.current_stream(self.device))
                timing.append(ev)
            if kernels is not None:
                kernels.append(_lib.last_kernel_name())
            start = 4
        for i, op in enumerate(self.ops):
            if i < start:
                continue
            if skip:  # the pool that was fused into the previous conv
                skip = False
                continue
            hin, hout = b["h"][i], b["h"][i + 1]
            if i in self.fused:
                if timing is not None:
                    ev = (torch.cuda.Event(enable_timing=True),
                          torch.cuda.Event(enable_timing=True))
                    ev[0].record(torch.cuda.current_stream(self.device))
                _, H, W, _ = hin.shape
                self._conv(i, hin, b["h"][i + 2], weights=self._wv[i], geom=op.fwd_geom(),
                           act=op.act, out_shape=(H, W), cout=op.cout, pool=True,
                           argmax=b["am"][i + 1] if train else None)
                if timing is not None:
                    ev[1].record(torch.cuda.current_stream(self.device))
                    timing.append(ev)
                if kernels is not None:
                    kernels.append(_lib.last_kernel_name())
                skip = True
                continue
            if isinstance(op, PoolOp):
                _, H, W, C = hin.shape
                am = b["am"][i]
                if am is None:
                    am = b.setdefault("am_inf", {}).get(hin.shape)
                    if am is None:
                        am = torch.empty((N, H // 2, W // 2, C), dtype=torch.uint8,
                                         device=self.device)
                        b["am_inf"][hin.shape] = am
                ops.maxpool2_out(hin, hout, am)
                continue
            last = i == n_ops - 1
            if timing is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(torch.cuda.current_stream(self.device))
            if self.dec3 and not train and i == n_ops - 3:  # three-layer decoder, then done
                o2, o3 = self.ops[i + 1], self.ops[i + 2]
                ops.decoder3_out(hin, self._wv[i], self._bv[i], op.cout, self._wv[i + 1],
                                 self._bv[i + 1], o2.cout, self._wv[i + 2], self._bv[i + 2],
                                 op.k, b["h"][n_ops])
                if timing is not None:
                    ev[1].record(torch.cuda.current_stream(self.device))
                    timing.append(ev)
                if kernels is not None:
                    kernels.append(_lib.last_kernel_name())
                break
            if self.tail_train and train and i == n_ops - 2:  # fused tail with stores, done
                o2 = self.ops[i + 1]
                ops.convt_conv_out_train_out(hin, self._wv[i], self._bv[i], op.cout, op.k,
                                             self._wv[i + 1], self._bv[i + 1], o2.k, hout,
                                             b["z"], b["h"][n_ops])
                if timing is not None:
                    ev[1].record(torch.cuda.current_stream(self.device))
                    timing.append(ev)
                if kernels is not None:
                    kernels.append(_lib.last_kernel_name())
                break
            if self.tail and not train and i == n_ops - 2:  # fused decoder tail, then done
                o2 = self.ops[i + 1]
                ops.convt_conv_out_out(hin, self._wv[i], self._bv[i], op.cout, op.k,
                                       self._wv[i + 1], self._bv[i + 1], o2.k, b["h"][n_ops])
                if timing is not None:
                    ev[1].record(torch.cuda.current_stream(self.device))
                    timing.append(ev)
                if kernels is not None:
                    kernels.append(_lib.last_kernel_name())
                break
            self._conv(i, hin, hout, weights=self._wv[i], geom=op.fwd_geom(), act=op.act,
                       logits=b["z"] if (train and last) else None,
                       out_shape=hout.shape[1:3], cout=op.cout)
            if timing is not None:
                ev[1].record(torch.cuda.current_stream(self.device))
                timing.append(ev)
            if kernels is not None:
                kernels.append(_lib.last_kernel_name())
        return b["h"][n_ops]

    def last_logits(self):
        """fp32 pre-sigmoid output of the last forward(train=True) (device, reused buffer)."""
        return self._buffers(self._last_train_N, True)["z"]

    def loss_and_grad(self, y, want_grad=True, accumulate=None):
        """BCE of the last forward(train=True) against y (device, same shape).

        The fp64 sum over elements is added to ``accumulate`` (a device fp64 [1] tensor)
        when given, else to self._loss after zeroing it; the tensor is returned (the
        mean is sum / y.numel()). Fills the last layer's gradient when want_grad."""
        if tuple(y.shape) != (self._last_train_N,) + self.output_shape:
            raise ValueError(f"targets must have shape (N, *{self.output_shape})")
        if y.dtype not in _TORCH.values() or not y.is_contiguous():
            raise TypeError("targets must be contiguous float32, bfloat16 or float16")
        b = self._buffers(self._last_train_N, True)
        if accumulate is None:
            accumulate = self._loss
            accumulate.zero_()
        ops.bce_logits_out(b["z"], y, b["d"][-1] if want_grad else None, accumulate)
        return accumulate

    def grad_bucket_split(self):
        """(op index j, flat offset): the gradients of layers >= j (the decoder: from the first
        Conv2DTranspose, else the second half of the convolutions) occupy self.g[offset:] and
        are final once backward() has run layer j's weight gradient — a data-parallel step
        all-reduces that bucket while the encoder's backward still runs."""
        convs = [i for i, op in enumerate(self.ops) if isinstance(op, ConvOp)]
        dec = [i for i in convs if self.ops[i].kind == "convT"]
        j = dec[0] if dec else convs[len(convs) // 2]
        return j, self.ops[j].off_w

    def sync_state(self, group=None, src=0):
        """Broadcast the master weights, the Adam moments and the step count from rank
        ``src`` (data-parallel start: ranks may have initialised differently), then refresh
        the low-precision and flipped weight copies."""
        import torch.distributed as dist
        for t in (self.w, self.m, self.v):
            dist.broadcast(t, src, group=group)
        tt = torch.tensor([self.t], dtype=torch.float64, device=self.device)
        dist.broadcast(tt, src, group=group)
        self.t = int(tt.item())
        self._refresh_lowp()

    def backward(self, on_layer_done=None):
        """Gradients of the last loss_and_grad() into self.g (overwritten).
        ``on_layer_done(i)`` (optional) is called once layer i's weight gradient is enqueued
        (layers in reverse order), with the stream that gradient was enqueued on current:
        self.g[ops[i].off_w:] is final in that stream's order.

        The input-gradient chain (dgrad, pool backward) stays on the current stream; each
        layer's weight gradient (wgrad + its ordered partial sum) is enqueued on a side
        stream (round-robin over self.wgrad_streams of them, each with its own workspace) as
        soon as the layer's output gradient exists, so the under-filled wgrad launches of a
        128-sample step run beside the chain and beside each other instead of after each
        link. The current stream waits for the side streams before returning: the same
        kernels on the same inputs, bitwise the serial result (tests/test_ae_gpu.py)."""
        N = self._last_train_N
        b = self._buffers(N, True)
        main = torch.cuda.current_stream(self.device)
        ow = self.wgrad_overwrite
        sides = []
        if self.wgrad_overlap:
            if self._sides is None or len(self._sides) != self.wgrad_streams:
                self._sides = [torch.cuda.Stream(device=self.device)
                               for _ in range(self.wgrad_streams)]
            sides = self._sides
        elif not ow:
            self.g.zero_()
        zeroed = not sides or ow
        while len(b["wss"]) < len(sides):  # (wgrad_streams raised after the buffers were made)
            b["wss"].append(torch.empty_like(b["ws"]))
        used = []  # side streams that received work, in issue order
        n_ops = len(self.ops)
        first = next((i for i, op in enumerate(self.ops) if isinstance(op, ConvOp)), -1)
        # the first convolution's gradient slice g[:g0_end] (the layers' slices follow the op
        # order; zero unless a second convolution exists: then the whole buffer is one slice)
        second = next((i for i, op in enumerate(self.ops) if isinstance(op, ConvOp) and i > first),
                      None)
        g0_end = self.ops[second].off_w if second is not None else 0
        for i in range(n_ops - 1, -1, -1):
            op = self.ops[i]
            d_out = b["d"][i + 1]
            hin = b["h"][i]
            prev = self.ops[i - 1] if i > 0 else None
            prev_relu = isinstance(prev, ConvOp) and prev.act == "relu"
            relu_mask = hin if prev_relu else None
            if isinstance(op, PoolOp):
                if i == 0 or (i == 1 and self.wgrad_pooled) or (i - 1) in self.pool_routed:
                    continue  # nothing upstream needs it / the conv reads d[i + 1] directly
                _, H, W, C = d_out.shape
                # ReLU mask of the pool's input at its argmax == (pooled output > 0)
                ops.maxpool2_bwd_out(d_out, b["am"][i], b["h"][i + 1] if prev_relu else None,
                                     b["d"][i])
                continue
            if op.act == "sigmoid" and i != n_ops - 1:
                raise NotImplementedError("sigmoid activation before the last layer")
            _, IH, IW, C = hin.shape
            OH, OW = d_out.shape[1:3]
            s, pt, pl, dil = op.fwd_geom()
            if not sides:
                if i == 0:
                    self._wgrad0(b, hin, d_out, op, s, pt, pl, dil, b["ws"])
                else:
                    self._wgrad(b, i, hin, d_out, op, s, pt, pl, dil, b["ws"])
                if on_layer_done is not None:
                    on_layer_done(i)
            elif i == first and zeroed:
                # no input gradient follows: the current stream is idle, so this weight
                # gradient runs there, beside the side streams' remaining ones
                if not (self.wgrad_pooled or ow):  # (overwriting forms need no zeroing)
                    self.g[:g0_end].zero_()
                self._wgrad0(b, hin, d_out, op, s, pt, pl, dil, b["ws0"])
                if on_layer_done is not None:
                    on_layer_done(i)
            else:
                k = len(used) % len(sides)
                side = sides[k]
                self._wait(side, main)  # d_out is ready
                with torch.cuda.stream(side):
                    if not zeroed:  # zeroed off the input-gradient chain (but the first
                        self.g[g0_end:].zero_()  # layer's slice: its wgrad runs on `main`)
                        zeroed = True
                    if i == 0:
                        self._wgrad0(b, hin, d_out, op, s, pt, pl, dil, b["wss"][k])
                    else:
                        self._wgrad(b, i, hin, d_out, op, s, pt, pl, dil, b["wss"][k])
                    if on_layer_done is not None:
                        # every weight gradient enqueued so far is final in this stream's order
                        for o in sides:
                            if o is not side and o in used:
                                self._wait(side, o)
                        on_layer_done(i)
                used.append(side)
            if i == 0:
                continue
            if i in self.pool_routed:
                _, dpt, dpl, _ = op.dgrad_geom()
                ops.conv2d_pooled_in_out(b["d"][i + 2], b["am"][i + 1],
                                         b["h"][i + 2] if op.act == "relu" else None,
                                         self.w_d[i], None, op.k, op.k, op.cin, dpt, dpl, IH, IW,
                                         0, relu_mask, b["d"][i])
                continue
            self._conv(i, d_out, b["d"][i], weights=self.w_d[i], geom=op.dgrad_geom(),
                       act=None, mask=relu_mask, bias=False, out_shape=(IH, IW), cout=op.cin)
        if not zeroed:  # no convolution reported a gradient
            self.g.zero_()
        for side in sides:
            if side in used:
                self._wait(main, side)

    def _wgrad0(self, b, hin, d_out, op, s, pt, pl, dil, ws):
        """Weight gradient of op 0: from its pool's gradient d[2] (argmax + ReLU mask of the
        pooled output) when wgrad_pooled, else from d_out = d[1]."""
        if self.wgrad_pooled:
            ops.conv2d_wgrad_pooled_out(hin, b["d"][2], b["am"][1],
                                        b["h"][2] if op.act == "relu" else None, op.k, op.k, s,
                                        pt, pl, dil, self._gwv[0], self._gbv[0], ws)
        else:
            ops.conv2d_wgrad_out(hin, d_out, op.k, op.k, s, pt, pl, dil, self._gwv[0],
                                 self._gbv[0], ws, self.wgrad_overwrite)

    def _wgrad(self, b, i, hin, d_out, op, s, pt, pl, dil, ws):
        """Weight gradient of op i > 0: from its pool's gradient d[i + 2] when i is pool-routed
        (d_out = d[i + 1] is then never formed), else from d_out. The routed form overwrites
        the layer's slice, the other accumulates into it (zeroed beforehand): same values."""
        if i in self.pool_routed:
            ops.conv2d_wgrad_pooled_out(hin, b["d"][i + 2], b["am"][i + 1],
                                        b["h"][i + 2] if op.act == "relu" else None, op.k, op.k,
                                        s, pt, pl, dil, self._gwv[i], self._gbv[i], ws)
        else:
            ops.conv2d_wgrad_out(hin, d_out, op.k, op.k, s, pt, pl, dil, self._gwv[i],
                                 self._gbv[i], ws, self.wgrad_overwrite)

    def _wait(self, waiter, signaler):
        if self.fork_mode == "torch":
            waiter.wait_stream(signaler)
        else:
            _lib.stream_wait(waiter, signaler, device_scope=self.fork_mode != "system")

    def adam(self, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7, grad_scale=1.0):
        """Keras Adam on the fp32 master weights; the low-precision copy and every layer's
        flipped input-gradient weights are written by the same launch (adam_step_flip_)."""
        self.t += 1
        lr_t = lr * math.sqrt(1.0 - beta_2 ** self.t) / (1.0 - beta_1 ** self.t)
        if len(self.w_d) <= 8:
            seg = sorted(self.w_d.items())
            ops.adam_step_flip_(self.w, self.g, self.m, self.v, lr_t, beta_1, beta_2, epsilon,
                                grad_scale, self.w_lp, [self.ops[i].off_w for i, _ in seg],
                                [x for i, _ in seg for x in (self.ops[i].k, self.ops[i].cin,
                                                              self.ops[i].cout)],
                                [wd for _, wd in seg])
            return
        ops.adam_step_(self.w, self.g, self.m, self.v, lr_t, beta_1, beta_2, epsilon, grad_scale,
                       self.w_lp)
        for i, wd in self.w_d.items():
            op = self.ops[i]
            ops.weight_flip_transpose_out(self._wv[i], op.k, op.cin, op.cout, wd)

    def train_step(self, x, y, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7,
                   process_group=None):
        """One fit() step: forward, BCE, backward, [gradient all-reduce], Adam. Returns the
        device fp64 loss sum of this rank (divide by y.numel() for the mean).

        With ``process_group`` (an initialised torch.distributed group, RCCL on the GPU)
        the flat gradient buffer is SUM-all-reduced and Adam scales it by 1/world_size:
        every rank then applies the identical update. The decoder's
        bucket is all-reduced asynchronously while the encoder's backward runs
        (dp_backward). Without it the step is rank-local even when a default process
        group is initialised."""
        self.forward(x, train=True)
        loss = self.loss_and_grad(y)
        scale = dp_backward(self, process_group)
        self.adam(lr, beta_1, beta_2, epsilon, grad_scale=scale)
        return loss

    def to_compute(self, x):
        """Host/device array -> contiguous device tensor in the compute dtype."""
        t = torch.as_tensor(x)
        if t.device != self.device:
            if t.dtype != torch.float32:
                t = t.float()
            t = t.contiguous().to(self.device, non_blocking=False)
        t = t.contiguous()
        if t.dtype == self.tdt:
            return t
        if t.dtype != torch.float32:
            raise TypeError(f"unsupported input dtype {t.dtype}")
        return ops.cast(t, self.tdt)


def dp_backward(eng, group=None, dist=None) -> float:
    """eng.backward() with the data-parallel gradient exchange: two
    buckets of the ONE flat gradient buffer, SUM-all-reduced over ``group``. The decoder
    bucket (eng.grad_bucket_split) goes out asynchronously as soon as its weight gradients
    are enqueued and overlaps the encoder's backward; the encoder bucket follows when
    backward ends; both are awaited before returning. Returns Adam's grad_scale
    (1/world_size), or 1.0 (plain backward) without a process group.

    The exchange is opt-in: it runs only when the caller names a group or passes the
    ``torch.distributed`` module (Model.fit does, under an initialised default group). An
    initialised default group alone never turns a single-model step into a collective, so
    rank-local training (a per-rank sweep task, the bench's rank-0 stages) cannot
    deadlock against ranks that are not stepping."""
    if dist is None and group is not None:
        import torch.distributed as dist
    if dist is None:
        eng.backward()
        return 1.0
    j, off = eng.grad_bucket_split()
    works = []

    def ready(i):
        if i == j:
            works.append(dist.all_reduce(eng.g[off:], group=group, async_op=True))

    eng.backward(on_layer_done=ready)
    if not works:  # layer j never reported (cannot happen for a conv layer): whole buffer
        off = eng.g.numel()
    if off > 0:
        works.append(dist.all_reduce(eng.g[:off], group=group, async_op=True))
    for w in works:
        w.wait()
    return 1.0 / dist.get_world_size(group)
