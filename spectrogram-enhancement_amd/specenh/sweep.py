"""Hyper-parameter sweep harness, one process per GPU.

The reference sweeps architectures two ways:

* ``VAE/hyperparam_scan.py:120-123`` — a SLURM task array: task ``SLURM_ARRAY_TASK_ID``
  picks ``kernel_vals[idx]`` of ``[(3,3), (5,5), (7,7)]`` for a 2-layer 32/32 model
  (:153-164), fits it (:174-181), saves the model, ``val_loss.txt`` and the mean predict
  time per channel ``t_pred.txt`` under ``kernel_<k>/`` (:186-247);
* ``VAE/manual_scan_3layers.py:120-123, 160-247`` — nested loops over ``ker_vals x
  conv1_vals x conv2_vals x conv3_vals`` of the 3-layer model, keeping each config's final
  ``val_loss`` and per-strip predict time in arrays, the best model, ``val_losses.npy`` and
  the per-parameter averages ``loss_comparisons.npz`` (:279-350).

Here both are one task list: ``hyperparam_scan_grid()`` / ``manual_scan_3layers_grid()``.
Launched under ``torch.distributed.run`` (one process per GPU) rank r runs tasks r, r +
world, ...; under a SLURM array the task id picks one task, as the reference does. Each task
trains rank-locally (specenh.keras.models.rank_local: no gradient collective between ranks
training different models) and writes the reference's per-task files; rank 0 then gathers
every rank's records (all_gather_object) and writes the sweep-level arrays.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m specenh.sweep --grid kernel --out sweep_out --epochs 15 --synthetic 4096
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import time
from dataclasses import asdict, dataclass

import numpy as np


@dataclass(frozen=True)
class SweepConfig:
    kernel: int                  # square kernel size (ker_vals / kernel_vals)
    filters: tuple               # (32, 32) for hyperparam_scan; (conv1, conv2, conv3)
    grid_index: tuple = ()       # position in the reference's nested loops

    @property
    def name(self):
        return f"kernel_{self.kernel}_" + "_".join(str(f) for f in self.filters)


def hyperparam_scan_grid(kernel_vals=((3, 3), (5, 5), (7, 7))):
    """hyperparam_scan.py:123 — one task per kernel size, 2-layer 32/32 model."""
    return [SweepConfig(k[0], (32, 32), (i,)) for i, k in enumerate(kernel_vals)]


def manual_scan_3layers_grid(ker_vals=((5, 5),), conv1_vals=(16,), conv2_vals=(32,),
                             conv3_vals=(64,)):
    """manual_scan_3layers.py:120-123 — the nested loops' order (:161-164)."""
    out = []
    for (a, k), (b, c1), (c, c2), (d, c3) in itertools.product(
            enumerate(ker_vals), enumerate(conv1_vals), enumerate(conv2_vals),
            enumerate(conv3_vals)):
        out.append(SweepConfig(k[0], (c1, c2, c3), (a, b, c, d)))
    return out


def build_model(cfg: SweepConfig, input_shape=(256, 128, 1)):
    """The reference graph of the config: hyperparam_scan.py:153-164 (two filters) or
    manual_scan_3layers.py:166-180 (three)."""
    from .keras import layers
    from .keras.models import Model
    k = cfg.kernel
    inp = layers.Input(shape=tuple(input_shape))
    x = inp
    for f in cfg.filters:
        x = layers.Conv2D(f, (k, k), activation="relu", padding="same")(x)
        x = layers.MaxPooling2D((2, 2), padding="same")(x)
    for f in reversed(cfg.filters):
        x = layers.Conv2DTranspose(f, (k, k), strides=2, activation="relu", padding="same")(x)
    x = layers.Conv2D(1, (k, k), activation="sigmoid", padding="same")(x)
    m = Model(inp, x)
    m.compile(optimizer="adam", loss="binary_crossentropy")
    return m


def task_assignment(n_tasks, world=None, rank=None):
    """Task indices this process runs: the SLURM array task (hyperparam_scan.py:122) when
    SLURM_ARRAY_TASK_ID is set, else rank, rank + world, ... of torch.distributed.run."""
    if "SLURM_ARRAY_TASK_ID" in os.environ:
        return [int(os.environ["SLURM_ARRAY_TASK_ID"])]
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    return list(range(rank, n_tasks, world))


def run_task(cfg: SweepConfig, data, out_dir, epochs=15, batch_size=128, pred_sets=None,
             verbose=0, save_model=True):
    """Train one config and write the reference's per-task files under ``out_dir``:
    ``keras_model/`` (specenh's directory format), ``val_loss.txt`` (np.savetxt of the
    per-epoch history, hyperparam_scan.py:235) and ``t_pred.txt`` (mean seconds of
    ``predict`` per prediction set, :238-247; manual_scan_3layers.py:226-245 divides by
    the strips per set, reported as ``t_pred_per_strip``). Returns the task record."""
    from .keras.models import rank_local
    x_tr, y_tr, x_val, y_val = data
    os.makedirs(out_dir, exist_ok=True)
    with rank_local():
        model = build_model(cfg, x_tr.shape[1:])
        t0 = time.perf_counter()
        hist = model.fit(x=x_tr, y=y_tr, epochs=epochs, batch_size=batch_size, shuffle=True,
                         validation_data=(x_val, y_val), verbose=verbose)
        fit_s = time.perf_counter() - t0
        val_loss = [float(v) for v in hist.history["val_loss"]]
        np.savetxt(os.path.join(out_dir, "val_loss.txt"), val_loss)
        sets = pred_sets if pred_sets is not None else [x_val]
        t_pred, t_strip = 0.0, 0.0
        model.predict(sets[0])  # engine buffers for this shape
        for s in sets:
            t1 = time.perf_counter()
            model.predict(s)
            dt = time.perf_counter() - t1
            t_pred += dt
            t_strip += dt / len(s)
        t_pred /= len(sets)
        t_strip /= len(sets)
        with open(os.path.join(out_dir, "t_pred.txt"), "w") as fh:
            fh.write(str(t_pred))
        if save_model:
            model.save(os.path.join(out_dir, "keras_model"))
    return {"config": asdict(cfg), "name": cfg.name, "val_loss": val_loss,
            "final_val_loss": val_loss[-1], "t_pred": t_pred, "t_pred_per_strip": t_strip,
            "fit_seconds": fit_s, "out_dir": out_dir}


def summarize(records, grid_shape=None):
    """Sweep-level arrays (manual_scan_3layers.py:279-350): final val_loss and per-strip
    predict time per config in the nested-loop shape, the best config, and the
    per-parameter averages over all other parameters."""
    records = sorted(records, key=lambda r: tuple(r["config"]["grid_index"]))
    if grid_shape is None:
        grid_shape = (len(records),)
    val = np.full(grid_shape, np.nan)
    pred = np.full(grid_shape, np.nan)
    for r in records:
        val[tuple(r["config"]["grid_index"])] = r["final_val_loss"]
        pred[tuple(r["config"]["grid_index"])] = r["t_pred_per_strip"]
    best = min(records, key=lambda r: r["final_val_loss"])
    comps = {}
    names = ["ker", "conv1", "conv2", "conv3"] if len(grid_shape) == 4 else ["ker"]
    for ax, nm in enumerate(names):
        others = tuple(i for i in range(len(grid_shape)) if i != ax)
        comps[f"{nm}_loss"] = np.nanmean(val, axis=others).reshape(-1, 1) if others else \
            val.reshape(-1, 1)
        comps[f"{nm}_time"] = np.nanmean(pred, axis=others).reshape(-1, 1) if others else \
            pred.reshape(-1, 1)
    return val, pred, best, comps


def run_sweep(configs, data, out_root, epochs=15, batch_size=128, pred_sets=None,
              grid_shape=None, verbose=0, dist=None):
    """This process's share of ``configs`` (task_assignment), then, on rank 0, the
    sweep-level files from every rank's records. Returns (my records, summary or None)."""
    if dist is None:
        import torch.distributed as tdist
        dist = tdist if (tdist.is_available() and tdist.is_initialized()) else None
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    mine = []
    for i in task_assignment(len(configs), world, rank):
        cfg = configs[i]
        mine.append(run_task(cfg, data, os.path.join(out_root, cfg.name), epochs, batch_size,
                             pred_sets, verbose))
    if dist:
        allrec = [None] * world
        dist.all_gather_object(allrec, mine)
        records = [r for part in allrec for r in part]
    else:
        records = mine
    summary = None
    if rank == 0 and records and "SLURM_ARRAY_TASK_ID" not in os.environ:
        val, pred, best, comps = summarize(records, grid_shape)
        os.makedirs(out_root, exist_ok=True)
        np.save(os.path.join(out_root, "val_losses.npy"), val)
        np.save(os.path.join(out_root, "pred_times.npy"), pred)
        np.savez(os.path.join(out_root, "loss_comparisons.npz"), **comps)
        with open(os.path.join(out_root, "sweep.json"), "w") as fh:
            json.dump({"records": records, "best": best["name"],
                       "best_model": os.path.join(best["out_dir"], "keras_model"),
                       "world": world}, fh, indent=1)
        summary = {"val_losses": val, "pred_times": pred, "best": best, "comparisons": comps}
    return mine, summary


def _synthetic_data(n, device, seed=0):
    """C4 pairs generated on the device (specenh.synthetic.c4_pairs_torch), split 60 / 25 / 15
    as manual_scan_3layers.py:153-154 splits its strips (train / tune / test)."""
    from .synthetic import c4_pairs_torch
    x, y = c4_pairs_torch(n, seed=seed, device=device)
    a, b = int(n * 0.6), int(n * 0.85)
    return (x[:a], y[:a], x[a:b], y[a:b]), [x[b:]]


def _store_data(path):
    """The dataset store (specenh.dataset: ece_<shot>/chn_<n>/{spec, pipeline_out}) as the
    reference reads it (:140-154): 30 strips of 128 columns per spectrogram, split 60/25/15."""
    from .dataset import SpectrogramStore
    from .strips import patch, reshape
    with SpectrogramStore(path, mode="r") as st:
        spec = [st[g]["spec"] for g in st.groups()]
        final = [st[g]["pipeline_out"] for g in st.groups()]
    s, f = patch(spec), patch(final)
    a, b = int(len(s) * 0.6), int(len(s) * 0.85)
    data = (reshape(s[:a]).astype(np.float32), reshape(f[:a]).astype(np.float32),
            reshape(s[a:b]).astype(np.float32), reshape(f[a:b]).astype(np.float32))
    return data, [reshape(s[b:]).astype(np.float32)]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--grid", choices=["kernel", "manual3"], default="kernel")
    ap.add_argument("--out", required=True)
    ap.add_argument("--epochs", type=int, default=15)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--synthetic", type=int, default=0, help="N device C4 pairs (128x128)")
    ap.add_argument("--store", default=None, help="dataset store root (specenh.dataset)")
    ap.add_argument("--policy", default="float32", help="keras mixed-precision policy")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    from .keras import mixed_precision
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    if use_dist:
        dist.init_process_group("nccl", device_id=dev)
    mixed_precision.set_global_policy(a.policy)
    if a.store:
        data, pred_sets = _store_data(a.store)
    else:
        data, pred_sets = _synthetic_data(a.synthetic or 1024, dev)
    if a.grid == "kernel":
        cfgs, shape = hyperparam_scan_grid(), None
    else:
        cfgs = manual_scan_3layers_grid()
        shape = (1, 1, 1, 1)
    mine, summ = run_sweep(cfgs, data, a.out, a.epochs, a.batch_size, pred_sets, shape,
                           dist=dist if use_dist else None)
    for r in mine:
        print(f"[sweep] {r['name']}: val_loss {r['final_val_loss']:.5f} "
              f"t_pred {r['t_pred']:.4f} s", flush=True)
    if summ:
        print(f"[sweep] best {summ['best']['name']}", flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
