"""keras.models subset: Model(inputs, outputs) with compile / fit / predict / evaluate /
save / summary / get_weights / set_weights, and load_model.

Call sites replaced (VAE/manual_scan_3layers.py): Model(input, x) :200, compile :201,
fit(...) -> hist.history['val_loss'] :203-216, predict :239,264,295, summary :249,
save :257. Semantics kept from Keras:
  * fit(): per-epoch shuffle of the training set (host RNG, specenh.keras.utils), batches
    of ``batch_size`` with a final partial batch, history['loss'] = batch-size-weighted
    mean of the batch losses, history['val_loss'] = evaluate() on validation_data,
    callbacks (EarlyStopping) after each epoch, returns a History.
  * predict(): float32 numpy, same NHWC shape as the model output. Results do not depend
    on ``batch_size`` (every sample is computed independently), so the engine uses
    larger internal chunks.
  * Data parallel: when torch.distributed is initialised with world_size > 1 (one process
    per GPU, RCCL), fit() behaves like Keras under MirroredStrategy: ``batch_size`` is
    the GLOBAL batch, each rank takes its 1/world slice, the flat gradient buffer is
    all-reduced once per step (a final partial batch is truncated to a multiple of
    world_size) and every rank applies the same Adam update.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time

import numpy as np
import torch

from .. import ae as _ae
from . import callbacks as _cb
from . import layers as _layers
from . import mixed_precision, optimizers, utils

_PRED_CHUNK = 512


def _chain(inputs, outputs):
    """Walk back from the output tensor to the input: the reference model is a chain."""
    seq = []
    t = outputs
    while t is not None and t._inbound is not None:
        seq.append(t._layer)
        t = t._inbound
    if t is not inputs:
        raise ValueError("outputs are not connected to inputs by a single chain of layers")
    return inputs._layer, seq[::-1]


def _to_op(layer):
    if isinstance(layer, _layers.MaxPooling2D):
        return _ae.PoolOp()
    cin = layer.input_shape[-1]
    if isinstance(layer, _layers.Conv2DTranspose):
        return _ae.ConvOp("convT", cin, layer.filters, layer.k, layer.activation,
                          stride=layer.strides[0])
    if isinstance(layer, _layers.Conv2D):
        return _ae.ConvOp("conv", cin, layer.filters, layer.k, layer.activation,
                          padding=layer.padding)
    raise NotImplementedError(f"layer type {type(layer).__name__}")


_local = threading.local()


@contextlib.contextmanager
def rank_local():
    """Within this context fit/evaluate ignore an initialised process group: each rank trains
    its own model with no collective (the sweep's one-task-per-GPU mode, specenh.sweep)."""
    prev = getattr(_local, "on", False)
    _local.on = True
    try:
        yield
    finally:
        _local.on = prev


def _dist():
    """torch.distributed when a process group is initialised (any world size: a 1-rank RCCL
    group still runs the exchange) and not inside rank_local(), else None."""
    if getattr(_local, "on", False):
        return None
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist
    return None


class Model:
    def __init__(self, inputs=None, outputs=None, name=None):
        if inputs is None or outputs is None:
            raise NotImplementedError("only the functional Model(inputs, outputs) form")
        self.inputs, self.outputs = inputs, outputs
        self.name = name or _layers._auto_name("model")
        inp, seq = _chain(inputs, outputs)
        self.layers = [inp] + seq
        self.input_shape = inputs.shape
        self.output_shape = outputs.shape
        for lay in seq:
            if hasattr(lay, "build_weights") and lay.kernel is None:
                lay.build_weights()
        self._ops = [_to_op(lay) for lay in seq]
        self._engine = None
        self.optimizer = None
        self.loss = None
        self.stop_training = False
        self.history = None
        self._policy = mixed_precision.global_policy().name

    # ------------------------------------------------------------------ engine
    @property
    def _conv_layers(self):
        return [lay for lay in self.layers[1:] if isinstance(lay, _layers._ConvBase)]

    def _get_engine(self):
        if self._engine is None:
            eng = _ae.AutoencoderEngine(self._ops, self.input_shape[1:],
                                        compute_dtype=mixed_precision.Policy(
                                            self._policy).compute_dtype)
            ws = []
            for lay in self._conv_layers:
                ws += [lay.kernel, lay.bias]
            eng.set_keras_weights(ws)
            self._engine = eng
        return self._engine

    def get_weights(self):
        if self._engine is not None:
            return self._engine.get_keras_weights()
        out = []
        for lay in self._conv_layers:
            out += [lay.kernel.copy(), lay.bias.copy()]
        return out

    def set_weights(self, weights):
        weights = [np.asarray(w, dtype=np.float32) for w in weights]
        convs = self._conv_layers
        if len(weights) != 2 * len(convs):
            raise ValueError(f"expected {2 * len(convs)} arrays, got {len(weights)}")
        for j, lay in enumerate(convs):
            if weights[2 * j].shape != lay.kernel.shape or weights[2 * j + 1].shape != lay.bias.shape:
                raise ValueError(f"weight shape mismatch for layer {lay.name}")
            lay.kernel, lay.bias = weights[2 * j].copy(), weights[2 * j + 1].copy()
        if self._engine is not None:
            self._engine.set_keras_weights(weights)

    def count_params(self):
        return sum(lay.count_params() for lay in self.layers)

    # ------------------------------------------------------------------ compile / fit
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, **kwargs):
        opt = optimizers.get(optimizer)
        if loss not in ("binary_crossentropy",):
            raise NotImplementedError(f"loss {loss!r}: only 'binary_crossentropy'")
        if self._ops and (not isinstance(self._ops[-1], _ae.ConvOp)
                          or self._ops[-1].act != "sigmoid"):
            raise NotImplementedError("binary_crossentropy needs a final sigmoid Conv layer")
        if metrics:
            raise NotImplementedError("metrics")
        self.optimizer, self.loss = opt, loss

    def _check_xy(self, x, y=None):
        want = tuple(self.input_shape[1:])
        x = x if isinstance(x, torch.Tensor) else np.asarray(x)
        if tuple(x.shape[1:]) != want:
            raise ValueError(f"expected input shape (N, {want}), got {tuple(x.shape)}")
        if y is not None:
            y = y if isinstance(y, torch.Tensor) else np.asarray(y)
            if tuple(y.shape) != (x.shape[0],) + tuple(self.output_shape[1:]):
                raise ValueError(f"target shape {tuple(y.shape)} does not match the output")
        return x, y

    def _upload(self, a, eng):
        """Host or device array -> device tensor in the compute dtype (chunked)."""
        if isinstance(a, torch.Tensor) and a.device == eng.device and a.dtype == eng.tdt:
            return a.contiguous()
        out = torch.empty(tuple(a.shape), dtype=eng.tdt, device=eng.device)
        step = 4096
        for s in range(0, a.shape[0], step):
            chunk = a[s:s + step]
            if not isinstance(chunk, torch.Tensor):
                chunk = torch.from_numpy(np.ascontiguousarray(chunk, dtype=np.float32))
            out[s:s + step] = eng.to_compute(chunk)
        return out

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose="auto", callbacks=None,
            validation_split=0.0, validation_data=None, shuffle=True, initial_epoch=0, **kwargs):
        if self.optimizer is None:
            raise RuntimeError("You must compile your model before training/testing.")
        if kwargs:
            raise NotImplementedError(f"fit arguments {sorted(kwargs)}")
        batch_size = 32 if batch_size is None else int(batch_size)
        x, y = self._check_xy(x, y)
        if validation_split and validation_data is None:
            cut = int(x.shape[0] * (1.0 - validation_split))
            validation_data = (x[cut:], y[cut:])
            x, y = x[:cut], y[:cut]
        eng = self._get_engine()
        xd, yd = self._upload(x, eng), self._upload(y, eng)
        n = xd.shape[0]
        dist = _dist()
        world = dist.get_world_size() if dist else 1
        rank = dist.get_rank() if dist else 0
        group = dist.group.WORLD if dist else None
        opt = self.optimizer
        hist = _cb.History()
        hist.params = {"verbose": verbose, "epochs": epochs, "steps": -(-n // batch_size)}
        cbs = [hist] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
            cb.on_train_begin()
        self.stop_training = False
        hwc = int(np.prod(self.output_shape[1:]))
        acc = torch.zeros(1, dtype=torch.float64, device=eng.device)
        if dist:  # every rank starts from rank 0's weights and optimizer state
            eng.sync_state(group)
        for epoch in range(initial_epoch, epochs):
            t0 = time.time()
            order = utils.rng().permutation(n) if shuffle else np.arange(n)
            order_d = torch.from_numpy(order).to(eng.device)
            if dist and shuffle:  # one epoch permutation for all ranks: rank 0's
                dist.broadcast(order_d, 0, group=group)
            acc.zero_()
            seen = 0
            for s in range(0, n, batch_size):
                idx = order_d[s:s + batch_size]
                bs = idx.shape[0] - idx.shape[0] % world
                if bs == 0:
                    continue
                per = bs // world
                idx = idx[rank * per:(rank + 1) * per]
                xb = xd.index_select(0, idx)
                yb = yd.index_select(0, idx)
                eng.forward(xb, train=True)
                eng.loss_and_grad(yb, accumulate=acc)
                scale = _ae.dp_backward(eng, group, dist)  # bucketed RCCL all-reduce under DP
                eng.adam(opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon,
                         grad_scale=scale)
                seen += bs
            if dist:
                dist.all_reduce(acc, group=group)
            logs = {"loss": float(acc.item()) / (hwc * max(seen, 1))}
            if validation_data is not None:
                logs["val_loss"] = self.evaluate(validation_data[0], validation_data[1],
                                                 batch_size=batch_size, verbose=0)
            if verbose and rank == 0:
                extra = "".join(f" - {k}: {v:.4f}" for k, v in logs.items())
                print(f"Epoch {epoch + 1}/{epochs} - {time.time() - t0:.1f}s{extra}", flush=True)
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in cbs:
            cb.on_train_end()
        self.history = hist
        return hist

    def evaluate(self, x=None, y=None, batch_size=None, verbose="auto", **kwargs):
        """Mean binary_crossentropy over (x, y) (float). Sharded over ranks under DP."""
        if self.loss is None:
            raise RuntimeError("You must compile your model before training/testing.")
        x, y = self._check_xy(x, y)
        eng = self._get_engine()
        batch_size = max(32 if batch_size is None else int(batch_size), _PRED_CHUNK)
        dist = _dist()
        world = dist.get_world_size() if dist else 1
        rank = dist.get_rank() if dist else 0
        n = x.shape[0]
        lo, hi = rank * n // world, (rank + 1) * n // world
        acc = torch.zeros(1, dtype=torch.float64, device=eng.device)
        for s in range(lo, hi, batch_size):
            xb = self._upload(x[s:min(s + batch_size, hi)], eng)
            yb = self._upload(y[s:min(s + batch_size, hi)], eng)
            eng.forward(xb, train=True)
            eng.loss_and_grad(yb, want_grad=False, accumulate=acc)
        if dist:
            dist.all_reduce(acc)
        return float(acc.item()) / (n * int(np.prod(self.output_shape[1:])))

    def predict(self, x, batch_size=None, verbose="auto", **kwargs):
        """Forward pass -> float32 numpy (N, H, W, C)."""
        x, _ = self._check_xy(x)
        eng = self._get_engine()
        n = x.shape[0]
        out = np.empty((n,) + tuple(self.output_shape[1:]), dtype=np.float32)
        for s in range(0, n, _PRED_CHUNK):
            xb = self._upload(x[s:s + _PRED_CHUNK], eng)
            out[s:s + xb.shape[0]] = eng.forward(xb, train=False).cpu().numpy()
        return out

    def predict_on_device(self, x):
        """Device fast path: x device [N, H, W, C] -> device fp32 output (engine buffer)."""
        eng = self._get_engine()
        return eng.forward(self._upload(x, eng), train=False)

    __call__ = predict_on_device

    # ------------------------------------------------------------------ save / summary
    def save(self, filepath, overwrite=True, **kwargs):
        """Directory format: config.json (architecture, policy, optimizer) + weights.npz
        (Keras-shaped kernels/biases and the Adam state). Not Keras' own file format."""
        if os.path.exists(filepath) and not overwrite:
            raise FileExistsError(filepath)
        os.makedirs(filepath, exist_ok=True)
        cfg = {"format": "specenh-keras-1", "name": self.name, "policy": self._policy,
               "input_shape": list(self.input_shape[1:]),
               "layers": [{"class_name": type(lay).__name__, "config": lay.get_config()}
                          for lay in self.layers[1:]],
               "loss": self.loss,
               "optimizer": self.optimizer.get_config() if self.optimizer else None}
        arrays = {}
        for lay, (k, b) in zip(self._conv_layers, _pairs(self.get_weights())):
            arrays[f"{lay.name}/kernel"] = k
            arrays[f"{lay.name}/bias"] = b
        if self._engine is not None and self._engine.t > 0:
            cfg["optimizer_iterations"] = self._engine.t
            arrays["optimizer/m"] = self._engine.m.cpu().numpy()
            arrays["optimizer/v"] = self._engine.v.cpu().numpy()
        with open(os.path.join(filepath, "config.json"), "w") as f:
            json.dump(cfg, f, indent=1)
        np.savez(os.path.join(filepath, "weights.npz"), **arrays)

    def summary(self, print_fn=None):
        pf = print_fn or print
        line = "_" * 90
        pf(f'Model: "{self.name}"')
        pf(line)
        pf(f" {'Layer (type)':<44}{'Output Shape':<30}{'Param #':<10}")
        pf("=" * 90)
        for lay in self.layers:
            shape = f"[{lay.output_shape}]" if isinstance(lay, _layers.InputLayer) else \
                str(lay.output_shape)
            pf(f" {lay.name + ' (' + type(lay).__name__ + ')':<44}{shape:<30}"
               f"{lay.count_params():<10}")
        pf("=" * 90)
        total = self.count_params()
        pf(f"Total params: {total:,}")
        pf(f"Trainable params: {total:,}")
        pf("Non-trainable params: 0")
        pf(line)


def _pairs(ws):
    return [(ws[i], ws[i + 1]) for i in range(0, len(ws), 2)]


_LAYER_TYPES = {"Conv2D": _layers.Conv2D, "Conv2DTranspose": _layers.Conv2DTranspose,
                "MaxPooling2D": _layers.MaxPooling2D}


def load_model(filepath, compile=True, **kwargs):
    """Inverse of Model.save (directory with config.json + weights.npz)."""
    with open(os.path.join(filepath, "config.json")) as f:
        cfg = json.load(f)
    if cfg.get("format") != "specenh-keras-1":
        raise ValueError(f"{filepath}: not a model saved by specenh.keras")
    prev = mixed_precision.global_policy().name
    mixed_precision.set_global_policy(cfg["policy"])
    try:
        t = _layers.Input(shape=tuple(cfg["input_shape"]))
        inp = t
        for spec in cfg["layers"]:
            c = dict(spec["config"])
            cls = _LAYER_TYPES[spec["class_name"]]
            if cls is _layers.MaxPooling2D:
                lay = cls(tuple(c["pool_size"]), padding=c["padding"], name=c["name"])
            else:
                lay = cls(c["filters"], tuple(c["kernel_size"]), strides=tuple(c["strides"]),
                          padding=c["padding"], activation=c["activation"], name=c["name"])
            t = lay(t)
        model = Model(inp, t, name=cfg["name"])
    finally:
        mixed_precision.set_global_policy(prev)
    with np.load(os.path.join(filepath, "weights.npz")) as z:  # allow_pickle=False
        ws = []
        for lay in model._conv_layers:
            ws += [z[f"{lay.name}/kernel"], z[f"{lay.name}/bias"]]
        model.set_weights(ws)
        if compile and cfg.get("loss"):
            opt = cfg.get("optimizer") or {}
            opt.pop("name", None)
            model.compile(optimizer=optimizers.Adam(**opt), loss=cfg["loss"])
            if "optimizer_iterations" in cfg:
                eng = model._get_engine()
                eng.m.copy_(torch.from_numpy(z["optimizer/m"]))
                eng.v.copy_(torch.from_numpy(z["optimizer/v"]))
                eng.t = int(cfg["optimizer_iterations"])
    return model
