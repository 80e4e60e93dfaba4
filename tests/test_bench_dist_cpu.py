"""bench.py's multi-GPU logic over gloo, world size 2, on CPU: per-rank shards are disjoint
and cover the job, seeds differ, the timed region is the MAX over ranks, and the reported
value is all ranks' spectrograms over that time (SURVEY.md §8 E1, weak scaling)."""
import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import REPO


def _rank(q, rank, world, port):
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = bench.shard(world, rank, 4096)
        el = bench.max_over_ranks(0.25 + 0.5 * rank, dist, "cpu")
        q.put((rank, sh, el, bench.throughput(world, 4096, 10, el)))
    finally:
        dist.destroy_process_group()


def test_bench_shard_and_max_elapsed_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(q, r, 2, port)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (sh, el, v)) for r, sh, el, v in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (sh0, el0, v0), (sh1, el1, v1) = res[0], res[1]
    assert sh0["seed"] != sh1["seed"]
    ids = set(range(sh0["first_shot"], sh0["first_shot"] + sh0["shots"]))
    ids1 = set(range(sh1["first_shot"], sh1["first_shot"] + sh1["shots"]))
    assert not ids & ids1 and ids | ids1 == set(range(2 * 4096))
    assert el0 == el1 == 0.75          # the slowest rank's time, on every rank
    assert v0 == v1 == 2 * 4096 * 10 / 0.75


def _c4_rank(q, rank, world, port):
    """bench.ae_train_c4_stage on gloo with the oracle's CPU engine (test_dp_cpu.OracleEngine)
    in both modes: per-GPU batch (global batch = batch x world) and global batch."""
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import bench
    from specenh import ae
    from test_dp_cpu import OracleEngine, _oracle_ops

    class C4Oracle(OracleEngine):
        def train_step(self, x, y, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7,
                       process_group=None):  # specenh.ae.AutoencoderEngine.train_step
            self.forward(x, train=True)
            loss = self.loss_and_grad(y, accumulate=torch.zeros(1, dtype=torch.float64))
            scale = ae.dp_backward(self, process_group)
            self.adam(lr, beta_1, beta_2, epsilon, grad_scale=scale)
            return loss

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def make(r):
            rng = np.random.default_rng(100 + r)  # every rank its own pairs
            eng = C4Oracle(_oracle_ops(), (16, 16, 1))
            ws = []
            wrng = np.random.default_rng(7 + 31 * r)  # unseeded-style: ranks differ at start
            for op in eng.ops:
                if op.kind == "pool":
                    continue
                shape = (op.k, op.k, op.cin, op.cout) if op.kind == "conv" else \
                    (op.k, op.k, op.cout, op.cin)
                ws += [(0.3 * wrng.standard_normal(shape)).astype(np.float32),
                       np.zeros(op.cout, np.float32)]
            eng.set_keras_weights(ws)
            X = torch.as_tensor(rng.uniform(0, 1, (16, 16, 16, 1)), dtype=torch.float64)
            return eng, X, (X > 0.6).to(torch.float64)

        holder = {}

        def make_keep(r):
            holder["eng"], X, Y = make(r)
            return holder["eng"], X, Y

        res = bench.ae_train_c4_stage("cpu", dist, batch=8, steps=3, make=make_keep,
                                      sync=lambda: None)
        w = [t.copy() for t in holder["eng"].get_keras_weights()]
        q.put((rank, res, w))
    finally:
        dist.destroy_process_group()


def test_c4_train_stage_world2_both_modes():
    import numpy as np
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c4_rank, args=(q, r, 2, port)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (st, w)) for r, st, w in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        st = res[r][0]
        assert st["world"] == 2
        assert st["per_gpu_batch"]["samples_per_rank"] == 8
        assert st["per_gpu_batch"]["global_batch"] == 16
        assert st["global_batch"]["samples_per_rank"] == 4       # Keras parity: 8 / world
        assert st["global_batch"]["global_batch"] == 8
        for mode in ("per_gpu_batch", "global_batch"):
            assert st[mode]["ms_per_step"] > 0 and np.isfinite(st[mode]["samples_per_s"])
        assert st["allreduce"]["bytes"] > 0
    # the max-over-ranks times are the same on both ranks
    assert res[0][0]["per_gpu_batch"]["ms_per_step"] == res[1][0]["per_gpu_batch"]["ms_per_step"]
    # rank 0's start weights were broadcast and every step applied the all-reduced gradient:
    # both ranks end bit-identical although they started apart and trained on their own pairs
    for a, b in zip(res[0][1], res[1][1]):
        np.testing.assert_array_equal(a, b)
