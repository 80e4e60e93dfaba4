"""The sweep harness (specenh.sweep) on CPU: task assignment as a SLURM
array (hyperparam_scan.py:122) or one process per rank, rank-local training (no gradient
collective between ranks training different models), the reference's per-task files
(val_loss.txt, t_pred.txt, keras_model/) and the sweep-level arrays of
manual_scan_3layers.py:279-350, gathered on rank 0 over gloo (world 2). The engine is the
oracle's CPU autograd behind the engine interface (test_dp_cpu.OracleEngine)."""
import json
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dp_cpu import OracleEngine, _data, _free_port


def _small_grid():
    from specenh import sweep
    return sweep.hyperparam_scan_grid(((3, 3), (5, 5), (7, 7)))


def _dataset():
    x, y = _data()
    return (x[:16], y[:16], x[16:], y[16:])


def _run(out_q, rank, world, port, out_root):
    from specenh import ae, sweep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    real = ae.AutoencoderEngine
    ae.AutoencoderEngine = OracleEngine
    try:
        mine, summ = sweep.run_sweep(_small_grid(), _dataset(), out_root, epochs=2,
                                     batch_size=8)
        dist.barrier()
        out_q.put((rank, [r["name"] for r in mine], None if summ is None else
                   (summ["val_losses"].tolist(), summ["best"]["name"])))
    finally:
        ae.AutoencoderEngine = real
        dist.destroy_process_group()


def test_sweep_world2_rank_local_tasks_and_summary(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(q, r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == ["kernel_3_32_32", "kernel_7_32_32"]
    assert res[1][0] == ["kernel_5_32_32"] and res[1][1] is None
    val, best = res[0][1]
    assert len(val) == 3 and best == ["kernel_3_32_32", "kernel_5_32_32",
                                      "kernel_7_32_32"][int(np.argmin(val))]
    for name in ("kernel_3_32_32", "kernel_5_32_32", "kernel_7_32_32"):
        d = tmp_path / name
        hist = np.loadtxt(d / "val_loss.txt")
        assert hist.shape == (2,) and np.all(np.isfinite(hist))
        assert float(open(d / "t_pred.txt").read()) > 0
        assert (d / "keras_model" / "config.json").exists()
    s = json.load(open(tmp_path / "sweep.json"))
    assert s["world"] == 2 and len(s["records"]) == 3
    np.testing.assert_array_equal(np.load(tmp_path / "val_losses.npy"), val)
    comps = np.load(tmp_path / "loss_comparisons.npz")
    np.testing.assert_allclose(comps["ker_loss"].ravel(), val)


def test_slurm_array_task_runs_its_one_config(tmp_path, monkeypatch):
    from specenh import ae, sweep
    monkeypatch.setenv("SLURM_ARRAY_TASK_ID", "1")
    monkeypatch.setattr(ae, "AutoencoderEngine", OracleEngine)
    assert sweep.task_assignment(3) == [1]
    mine, summ = sweep.run_sweep(_small_grid(), _dataset(), str(tmp_path), epochs=1,
                                 batch_size=8, dist=None)
    assert [r["name"] for r in mine] == ["kernel_5_32_32"] and summ is None
    assert (tmp_path / "kernel_5_32_32" / "val_loss.txt").exists()
    assert not (tmp_path / "val_losses.npy").exists()


def test_manual3_grid_order_and_parameter_averages():
    from specenh import sweep
    grid = sweep.manual_scan_3layers_grid(((3, 3), (5, 5)), (16, 32), (32,), (16, 64))
    assert len(grid) == 8
    assert grid[0].grid_index == (0, 0, 0, 0) and grid[1].grid_index == (0, 0, 0, 1)
    assert grid[-1].filters == (32, 32, 64) and grid[-1].kernel == 5
    recs = [{"config": {"grid_index": list(c.grid_index)}, "final_val_loss": float(i),
             "t_pred_per_strip": 10.0 + i, "name": c.name} for i, c in enumerate(grid)]
    val, pred, best, comps = sweep.summarize(recs, (2, 2, 1, 2))
    assert val.shape == (2, 2, 1, 2) and best["name"] == grid[0].name
    np.testing.assert_allclose(comps["ker_loss"].ravel(), [1.5, 5.5])      # mean of 0..3, 4..7
    np.testing.assert_allclose(comps["conv1_loss"].ravel(), [2.5, 4.5])
    np.testing.assert_allclose(comps["conv3_loss"].ravel(), [3.0, 4.0])
    np.testing.assert_allclose(comps["ker_time"].ravel(), [11.5, 15.5])


@pytest.mark.parametrize("filters", [(32, 32), (16, 32, 64)])
def test_build_model_matches_reference_graphs(filters):
    from specenh import sweep
    m = sweep.build_model(sweep.SweepConfig(5, filters), (256, 128, 1))
    kinds = [(op.kind, getattr(op, "cout", None)) for op in m._ops]
    n = len(filters)
    want = []
    for f in filters:
        want += [("conv", f), ("pool", None)]
    want += [("convT", f) for f in reversed(filters)] + [("conv", 1)]
    assert kinds == want and n in (2, 3)
    assert m.output_shape[1:] == (256, 128, 1)
