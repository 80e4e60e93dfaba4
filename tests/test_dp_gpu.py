"""The data-parallel training path on the GPU with a real RCCL process group:
Model.fit and AutoencoderEngine.train_step under a 1-rank "nccl" (= RCCL) group run the
state broadcast, the permutation broadcast and the bucketed asynchronous gradient
all-reduce (specenh.ae.dp_backward) through RCCL with the HIP engine, and must give
bit-identical weights and history to the same training without a group. (World sizes > 1
are the driver's 8-GPU runs; the multi-rank arithmetic is tests/test_dp_cpu.py over gloo.)"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(policy):
    from specenh.keras import layers, mixed_precision, utils
    from specenh.keras.models import Model
    utils.set_random_seed(7)
    mixed_precision.set_global_policy(policy)
    try:
        inp = layers.Input(shape=(32, 32, 1))
        x = layers.Conv2D(16, 5, activation="relu", padding="same")(inp)
        x = layers.MaxPooling2D((2, 2), padding="same")(x)
        x = layers.Conv2D(32, 5, activation="relu", padding="same")(x)
        x = layers.MaxPooling2D((2, 2), padding="same")(x)
        x = layers.Conv2DTranspose(32, 5, strides=2, activation="relu", padding="same")(x)
        x = layers.Conv2DTranspose(16, 5, strides=2, activation="relu", padding="same")(x)
        x = layers.Conv2D(1, 5, activation="sigmoid", padding="same")(x)
        m = Model(inp, x)
    finally:
        mixed_precision.set_global_policy("float32")
    m.compile(optimizer="adam", loss="binary_crossentropy")
    return m


def _train(policy):
    rng = np.random.default_rng(3)
    x = rng.uniform(0, 1, (48, 32, 32, 1)).astype(np.float32)
    y = (x > 0.55).astype(np.float32)
    m = _model(policy)
    h = m.fit(x, y, epochs=2, batch_size=16, shuffle=True, validation_data=(x[:16], y[:16]),
              verbose=0)
    return m.get_weights(), h.history


@pytest.mark.parametrize("policy", ["float32", "mixed_bfloat16"])
def test_fit_under_rccl_group_is_bit_identical(gpu_device, policy):
    import torch.distributed as dist

    ref_w, ref_h = _train(policy)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu_device)
    try:
        assert dist.get_backend() == "nccl"
        w, h = _train(policy)
        # the engine's own train_step with an explicit group
        from specenh import ae
        from specenh.keras.models import Model  # noqa: F401
        m = _model(policy)
        eng = m._get_engine()
        xb = eng.to_compute(torch.rand(8, 32, 32, 1, device=gpu_device))
        yb = eng.to_compute((torch.rand(8, 32, 32, 1, device=gpu_device) > 0.5).float())
        eng.sync_state(dist.group.WORLD)
        loss = eng.train_step(xb, yb, process_group=dist.group.WORLD)
        assert torch.isfinite(loss).all()
        j, off = eng.grad_bucket_split()
        assert isinstance(eng.ops[j], ae.ConvOp) and eng.ops[j].kind == "convT" and 0 < off
    finally:
        dist.destroy_process_group()
    for a, b in zip(w, ref_w):
        np.testing.assert_array_equal(a, b)
    assert h == ref_h
