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
