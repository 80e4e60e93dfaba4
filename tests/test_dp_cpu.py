"""Data-parallel fit() on CPU with gloo, world_size 2.

Model.fit under torch.distributed broadcasts rank 0's weights and optimizer state, uses
rank 0's epoch permutation on every rank, takes each global batch, gives every rank its
slice, SUM-all-reduces the ONE flat gradient buffer in two buckets (the decoder's
asynchronously, overlapping the encoder's backward; specenh.ae.dp_backward), scales it by
1/world inside Adam and all-reduces the epoch loss. These tests run that orchestration with
a test-only engine: the oracle's autograd on CPU behind the engine interface (the HIP
engine under a real RCCL group is tests/test_dp_gpu.py). Two gloo ranks must then end with
the weights and history a single process gets on the same global batches, and unseeded
ranks (different initial weights) must still end identical.
"""
import math
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import autoencoder as ora


class OracleEngine:
    """CPU stand-in for specenh.ae.AutoencoderEngine (same methods fit() calls)."""

    def __init__(self, ops, input_shape, compute_dtype="float32", device=None):
        self.ops = ops
        self.input_shape = tuple(input_shape)
        self.device = torch.device("cpu")
        self.tdt = torch.float64
        self.spec = [("pool",) if op.kind == "pool" else (op.kind, op.cin, op.cout, op.k, op.act)
                     for op in ops]
        self.t = 0
        self.params = None

    def set_keras_weights(self, ws):
        it = iter(ws)
        self.params = []
        for s in self.spec:
            if s[0] == "pool":
                self.params.append(None)
            else:
                self.params.append({"W": torch.tensor(next(it), dtype=torch.float64),
                                    "b": torch.tensor(next(it), dtype=torch.float64)})
        flat = self._flat()
        self.g = torch.zeros_like(flat)
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)

    def _tensors(self):
        return [t for p in self.params if p is not None for t in (p["W"], p["b"])]

    def _flat(self):
        return torch.cat([t.reshape(-1) for t in self._tensors()])

    def get_keras_weights(self):
        return [t.detach().numpy().astype(np.float32) for t in self._tensors()]

    def to_compute(self, x):
        return torch.as_tensor(x).to(torch.float64)

    def forward(self, x, train=False):
        for t in self._tensors():
            t.requires_grad_(train)
            t.grad = None
        out, self._z = ora.forward(self.spec, self.params, x, return_logits=True)
        return out

    def loss_and_grad(self, y, want_grad=True, accumulate=None):
        z = self._z
        per = torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-torch.abs(z)))
        if want_grad:
            per.mean().backward()
        accumulate += per.sum().detach()
        return accumulate

    def backward(self, on_layer_done=None):
        self.g = torch.cat([t.grad.reshape(-1) for t in self._tensors()])
        if on_layer_done is not None:
            for i in reversed(range(len(self.spec))):
                if self.spec[i][0] != "pool":
                    on_layer_done(i)

    def grad_bucket_split(self):
        convs = [i for i, s in enumerate(self.spec) if s[0] != "pool"]
        dec = [i for i in convs if self.spec[i][0] == "convT"]
        j = dec[0] if dec else convs[len(convs) // 2]
        off = sum(p["W"].numel() + p["b"].numel() for p in self.params[:j] if p is not None)
        return j, off

    def sync_state(self, group=None, src=0):
        with torch.no_grad():
            for t in self._tensors() + [self.m, self.v]:
                dist.broadcast(t, src, group=group)

    def adam(self, lr, b1, b2, eps, grad_scale=1.0):
        self.t += 1
        lr_t = lr * math.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t)
        g = self.g * grad_scale
        self.m = b1 * self.m + (1 - b1) * g
        self.v = b2 * self.v + (1 - b2) * g * g
        flat = self._flat().detach() - lr_t * self.m / (self.v.sqrt() + eps)
        off = 0
        with torch.no_grad():
            for t in self._tensors():
                n = t.numel()
                t.copy_(flat[off:off + n].reshape(t.shape))
                off += n


def _build(seed=0):
    from specenh.keras import layers, utils
    from specenh.keras.models import Model
    if seed is not None:
        utils.set_random_seed(seed)
    inp = layers.Input(shape=(16, 16, 1))
    x = layers.Conv2D(4, 3, activation="relu", padding="same")(inp)
    x = layers.MaxPooling2D((2, 2), padding="same")(x)
    x = layers.Conv2DTranspose(4, 3, strides=2, activation="relu", padding="same")(x)
    x = layers.Conv2D(1, 3, activation="sigmoid", padding="same")(x)
    m = Model(inp, x)
    m.compile(optimizer="adam", loss="binary_crossentropy")
    return m


def _data():
    rng = np.random.default_rng(42)
    x = rng.uniform(0, 1, (24, 16, 16, 1)).astype(np.float32)
    y = (x > 0.6).astype(np.float32)
    return x, y


def _fit(out_q=None, rank=0, world=1, port=0, seed=0):
    from specenh import ae
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    real_engine = ae.AutoencoderEngine
    ae.AutoencoderEngine = OracleEngine  # test-only: CPU autograd behind the engine API
    try:
        m = _build(seed)
        x, y = _data()
        w0 = [w.copy() for w in m.get_weights()]
        hist = m.fit(x, y, epochs=2, batch_size=8, shuffle=True, validation_data=(x[:8], y[:8]),
                     verbose=0)
        res = ([w.copy() for w in m.get_weights()], dict(hist.history), w0)
    finally:
        ae.AutoencoderEngine = real_engine
        if world > 1:
            dist.destroy_process_group()
    if out_q is not None:
        out_q.put((rank, res))
    return res


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world2(seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit, args=(q, r, 2, port, seed)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


def test_dp_fit_world2_matches_single_process():
    ref_w, ref_h, _ = _fit()
    results = _run_world2(0)
    for rank in (0, 1):
        w, h, _ = results[rank]
        for a, b in zip(w, ref_w):
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)
        for key in ("loss", "val_loss"):
            np.testing.assert_allclose(h[key], ref_h[key], rtol=1e-10)
    # every rank applied the identical update
    for a, b in zip(results[0][0], results[1][0]):
        np.testing.assert_array_equal(a, b)


def test_dp_fit_unseeded_ranks_stay_in_lockstep():
    """No set_random_seed on any rank (the reference scripts never seed): the ranks start
    from different glorot weights, fit() broadcasts rank 0's, and they end identical."""
    results = _run_world2(None)
    w0_0, w0_1 = results[0][2], results[1][2]
    assert any(not np.array_equal(a, b) for a, b in zip(w0_0, w0_1))
    for a, b in zip(results[0][0], results[1][0]):
        np.testing.assert_array_equal(a, b)
    h = results[0][1]
    assert h["loss"][-1] < h["loss"][0]


def _rank_local_steps(out_q, rank, world, port):
    """Only rank 0 trains (as bench.py's rank-0 stages and a per-rank sweep task do) while
    rank 1 waits in the final barrier: with no group named, the step must stay rank-local
    even though a default group is initialised (no collective that rank 1 never joins)."""
    from specenh import ae
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scales = []
        if rank == 0:
            m = _build(0)
            eng = OracleEngine(_oracle_ops(), (16, 16, 1))
            eng.set_keras_weights(m.get_weights())
            x, y = _data()
            for s in range(3):
                eng.forward(torch.as_tensor(x[:8], dtype=torch.float64), train=True)
                eng.loss_and_grad(torch.as_tensor(y[:8], dtype=torch.float64),
                                  accumulate=torch.zeros(1, dtype=torch.float64))
                scales.append(ae.dp_backward(eng))
                eng.adam(1e-3, 0.9, 0.999, 1e-7, grad_scale=scales[-1])
        dist.barrier()
        # both ranks: an explicit group does exchange (and averages over the world)
        eng2 = _TwoLayerGrad(rank)
        sc = ae.dp_backward(eng2, group=dist.group.WORLD)
        out_q.put((rank, scales, sc, eng2.g.tolist()))
    finally:
        dist.destroy_process_group()


class _TwoLayerGrad:
    """Minimal engine: backward() writes a rank-dependent flat gradient."""

    def __init__(self, rank):
        self.rank = rank
        self.g = torch.zeros(6, dtype=torch.float64)

    def grad_bucket_split(self):
        return 1, 3

    def backward(self, on_layer_done=None):
        self.g = torch.arange(6, dtype=torch.float64) + 10 * self.rank
        if on_layer_done is not None:
            on_layer_done(1)
            on_layer_done(0)


def _oracle_ops():
    from specenh import ae
    return [ae.ConvOp("conv", 1, 4, 3, "relu"), ae.PoolOp(),
            ae.ConvOp("convT", 4, 4, 3, "relu", stride=2), ae.ConvOp("conv", 4, 1, 3, "sigmoid")]


def test_rank_local_step_under_initialised_group_does_not_collect():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_local_steps, args=(q, r, 2, port)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert results[0][0] == [1.0, 1.0, 1.0] and results[1][0] == []
    for r in (0, 1):
        scale, g = results[r][1], results[r][2]
        assert scale == 0.5
        np.testing.assert_array_equal(g, 2 * np.arange(6) + 10)  # SUM over the two ranks
