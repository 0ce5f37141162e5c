"""The reference training loop (Training_VAE.py:316-394) on the HIP engine.

Same inputs, prints, loss history, CSV and checkpoint as the reference ``__main__`` in
``mode='training'``; what changes is underneath:

* the dataset is uploaded once and stays resident in HBM; each step hands the kernel the
  batch's row indices and the gather + relative transform (:345-348) happen in its loader;
* the step (zero_grad → forward → conditional_vae_loss → backward → Adam, :351-363) is ONE
  ``cvae_train_step`` call (two kernels) — or fwd/bwd → RCCL all-reduce → Adam under DP;
* the five ``loss.item()`` per step (:366-370) become a device accumulator read once per
  epoch, so the step loop never synchronises with the host.

RNG: ``torch.utils.data.DataLoader(shuffle=True)`` over row indices consumes the global CPU
generator exactly as the reference's loader does.  ``eps="host"`` draws each step's
``randn(B, Z)`` from that same generator (the reference's ``randn_like`` at :205 on CPU), so a
seeded run replays the reference's stream; ``eps="philox"`` generates eps in-kernel instead
(Philox4x32-10, keyed by the engine seed, the device step counter and the GLOBAL row: under data
parallelism each rank passes its first row, so the global batch draws what one process would)
and is the throughput mode.

Precision: the dataset stays fp32 on the device whatever the operand dtype; the kernels subtract
the start point in fp32 and round the RELATIVE coordinates once (Training_VAE.py:345-348), so a
bf16 run on real data (absolute coordinates of ~200 m) does not quantise its offsets to ~1 m.

Outputs (Training_VAE.py:373-394, Tools.py:747-771): one line per epoch in the reference
format; ``loss_history`` (per-epoch means) and its weighted copy; the loss CSV (header = the
five keys, one row per epoch) next to ``loss_save_path``; ``torch.save`` of the 24-key
state_dict (CPU tensors).  The matplotlib figure of ``plot_losses`` is not drawn.
"""
from __future__ import annotations

import csv
import os
from collections import OrderedDict

import numpy as np
import torch

from . import dist as dp
from .model import ConditionalTrajectoryVAE, TrajectoryDataset

LOSS_KEYS = ("total_loss", "recon_loss", "kld_loss", "start_loss", "time_loss")  # :337


class _Rows(torch.utils.data.Dataset):
    """Row indices 0..n-1: the DataLoader then draws the reference's permutation, not the data."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


def loader_permutation(n):
    """The row order of one epoch of ``DataLoader(dataset_of_n, shuffle=True)`` (Training_VAE.py:327,
    num_workers=0), drawn from the global CPU generator exactly as iterating that loader draws it:
    the iterator's base seed (``_BaseDataLoaderIter``: one int64 ``random_()``), then
    ``RandomSampler``'s own seed (a second one) for a fresh generator's ``randperm(n)``.  Nothing
    else of the loader touches the global generator, so a run that draws its epochs ahead replays
    the reference's stream (tests/test_train_dp.py checks it against the DataLoader)."""
    torch.empty((), dtype=torch.int64).random_()                    # the iterator's _base_seed
    seed = int(torch.empty((), dtype=torch.int64).random_().item())  # RandomSampler.__iter__
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g)


def epoch_line(epoch, means):
    """Training_VAE.py:373 print format."""
    t, r, k, s, ti = means
    return (f"Epoch {epoch + 1}: Loss={t:.4f}, Recon={r:.4f}, KLD={k:.4f}, Start={s:.4f}, Time={ti:.4f}")


def weighted_history(loss_history, weights):
    """Training_VAE.py:385-388: component curves scaled by their loss weights."""
    out = {k: list(v) for k, v in loss_history.items()}
    for key, w in zip(LOSS_KEYS[1:], weights):
        out[key] = [x * w for x in out[key]]
    return out


def save_loss_csv(loss_history, save_path):
    """Tools.py:747-771: ``<save_path stem>.csv``, header = keys, one row per epoch."""
    csv_path = os.path.splitext(save_path)[0] + ".csv"
    d = os.path.dirname(csv_path)
    if d:
        os.makedirs(d, exist_ok=True)
    keys = list(loss_history.keys())
    with open(csv_path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(keys)
        for i in range(len(loss_history[keys[0]])):
            w.writerow([loss_history[k][i] for k in keys])
    return csv_path


def cpu_state_dict(model):
    """The 24-key state_dict as CPU fp32 tensors (loadable by Tools.py:39-41 on any device)."""
    return OrderedDict((k, v.detach().to("cpu", torch.float32).clone()) for k, v in model.state_dict().items())


def save_checkpoint(path, model, eng, epoch, loss_history):
    """Resume point (the reference saves only the final state_dict, Training_VAE.py:393): the
    24-key state_dict, the Adam state in torch's Adam.state_dict() format, the epoch, the loss
    history, the Philox offset and the global CPU RNG state (DataLoader order and host eps)."""
    from .engine import optimizer_state_dict
    d = os.path.dirname(str(path))
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save({"model": cpu_state_dict(model), "optimizer": optimizer_state_dict(eng), "epoch": int(epoch),
                "loss_history": {k: list(v) for k, v in loss_history.items()},
                "rng_offset": int(eng.rng_offset), "cpu_rng_state": torch.get_rng_state()}, path)


def train(data, seq_len, dim, latent_dim, batch_size=32, lr=1e-3, epochs=1, hidden_dim=128,
          weights=(0.1, 0.1, 1.0, 1.0), model_save_path=None, loss_save_path=None, dtype="fp32",
          eps="host", device=None, seed=None, engine_seed=0, log=print, model=None, buckets=1,
          checkpoint_path=None, resume=None, classes=None, class_dim=0, exchange="auto", epochs_per_call=64,
          shard_adam=False):
    """Train like ``python Training_VAE.py`` (mode='training').

    data: path to the (N, seq_len, dim) ``.npy`` (TrajectoryDataset, :105-115) or an array; or a
    LIST of paths (scenes) — their rows are concatenated and, with ``class_dim`` > 0 and more than
    one file, each row's class is its file's index (BASELINE cfg4: one model over the Town04/Town05
    scenes); the default ``class_dim=0`` trains the reference's 24-key model on the rows.
    classes: per-row class ids (cfg4 class embedding, ``class_dim`` wide); None = the reference model.
    weights: (recon, kld, start, time) — the values of :300-306.
    seed: if given, ``torch.manual_seed(seed)`` first (the reference leaves it unseeded).
    Under ``torch.distributed`` every rank runs this with the same arguments; batch_size is
    then per rank (global batch = batch_size · world) and rank 0 logs and saves; ``exchange``
    picks the gradient exchange ("auto": the in-kernel peer exchange where the configuration has
    it — cvae_amd.peer — else the RCCL all-reduce; "rccl"; "peer"); ``buckets=2`` overlaps the
    decoder gradients' all-reduce with the rest of the dW GEMMs (rccl); ``shard_adam`` replaces the
    all-reduce and the whole Adam on every rank by a reduce-scatter, Adam on the rank's 1/world of
    the flat state and an all-gather of the parameters (rccl, one bucket).

    checkpoint_path: write a resume point (save_checkpoint) after every epoch; resume: continue
    from one — ``epochs`` counts the total, so train(epochs=4, resume=ckpt_after_2) runs epochs 3-4
    and ends where an uninterrupted 4-epoch run ends.

    On one device (no data parallelism, no class embedding) up to ``epochs_per_call`` epochs run as
    ONE C call (cvae_train_epochs): their permutations (loader_permutation) and host eps are drawn
    ahead in the reference's RNG order and uploaded once, the steps are enqueued without host work,
    and the per-epoch loss sums are read once per call (so the epoch lines of a call print
    together); with ``checkpoint_path`` a call is one epoch.

    Returns (model, loss_history, weighted_loss_history).
    """
    if seed is not None:
        torch.manual_seed(seed)
    rank, world_size = dp.world()
    if isinstance(data, (list, tuple)) and data and isinstance(data[0], (str, os.PathLike)):
        parts = [TrajectoryDataset(p).data for p in data]
        arr = np.ascontiguousarray(np.concatenate(parts, 0))
        if classes is None and class_dim and len(parts) > 1:
            classes = np.concatenate([np.full(len(a), i, np.int32) for i, a in enumerate(parts)])
    elif isinstance(data, (str, os.PathLike)):
        arr = TrajectoryDataset(data).data
    else:
        arr = np.ascontiguousarray(np.asarray(data, dtype=np.float32))
    n = len(arr)
    if rank == 0 and log:
        log(f"Training parameters: seq_len={seq_len}, latent_dim={latent_dim}, batch_size={batch_size}, lr={lr}")
        log(f"Dataset size: {n} trajectories")
    n_classes = 0
    if classes is not None:
        classes = np.ascontiguousarray(np.asarray(classes, dtype=np.int32))
        if classes.shape != (n,):
            raise ValueError(f"classes must hold one id per trajectory ({n}), got {classes.shape}")
        n_classes = int(classes.max()) + 1
    if model is None:  # init from the global RNG
        model = ConditionalTrajectoryVAE(seq_len, dim, latent_dim, hidden_dim, n_classes=n_classes,
                                         class_dim=class_dim)
    eng = model.__dict__.get("_engine") or model.attach(dtype=dtype, max_batch=batch_size, device=device,
                                                        seed=engine_seed)
    if eng.max_batch < batch_size:
        raise ValueError(f"engine max_batch {eng.max_batch} < batch_size {batch_size}")
    eng.set_optimizer(lr=lr)
    eng.weights = tuple(float(w) for w in weights)
    eng.keep_f32 = True                                   # relative transform in fp32 (see above)
    step = dp.DataParallelStep(eng, buckets=buckets, exchange="rccl" if classes is not None or shard_adam else exchange,
                               shard_adam=shard_adam)
    step.broadcast_params()
    x_dev = eng.as_input(torch.from_numpy(arr), keep_f32=True)  # resident for the whole run
    cls_dev = None if classes is None else torch.from_numpy(classes).to(x_dev.device)
    Z = latent_dim
    gb = batch_size * world_size
    loader = torch.utils.data.DataLoader(_Rows(n), batch_size=gb, shuffle=True)
    eng.loss_accum.zero_()
    loss_history = {k: [] for k in LOSS_KEYS}
    first = 0
    if resume is not None:
        from .engine import load_optimizer_state_dict
        ck = torch.load(resume, weights_only=True)
        model.load_state_dict(ck["model"])
        load_optimizer_state_dict(eng, ck["optimizer"])
        eng.set_optimizer(lr=lr, betas=eng.betas, eps=eng.eps)  # the checkpoint's betas / eps stay
        eng.rng_offset = ck["rng_offset"]
        torch.set_rng_state(ck["cpu_rng_state"])
        loss_history = {k: list(ck["loss_history"][k]) for k in LOSS_KEYS}
        first = ck["epoch"]
        step.broadcast_params()
        step.counters_changed()  # the peer exchange counts its flag epochs from the device step counter
    fused = world_size == 1 and classes is None and not step.split and step.px is None
    if fused:  # whole epochs per C call: the host draws, uploads once, and reads the losses once
        chunk = 1 if checkpoint_path else max(1, int(epochs_per_call))
        spe = (n + gb - 1) // gb
        if eps not in ("host", "philox"):
            raise ValueError("eps must be 'host' or 'philox'")

        def draw(k):
            """k epochs' host draws, in the reference's order: each epoch's DataLoader permutation
            (:340), then reparameterize's randn_like per batch (:205)."""
            perms, eps_rows = [], []
            for _ in range(k):
                perms.append(loader_permutation(n))
                if eps == "host":
                    for lo in range(0, n, gb):
                        eps_rows.append(torch.randn(min(gb, n - lo), Z))
            return k, torch.stack(perms), torch.cat(eps_rows) if eps == "host" else None

        epoch = first
        nxt = draw(min(chunk, epochs - epoch)) if epoch < epochs else None
        while nxt is not None:
            k, idx, e = nxt
            acc = eng.train_epochs(x_dev, idx, gb, n_steps=k * spe, eps=e)  # uploads queue behind the kernels
            # the next chunk's draws while the device runs this one (they come next in the generator's
            # stream either way; a checkpoint run draws after saving, so its saved RNG state is exact)
            nxt = None
            if epoch + k < epochs and not checkpoint_path:
                nxt = draw(min(chunk, epochs - epoch - k))
            sums = acc.cpu().numpy()                      # the only host sync of the k epochs
            for j in range(k):
                means = sums[j] / n
                for key, v in zip(LOSS_KEYS, means):
                    loss_history[key].append(float(v))
                if log:
                    log(epoch_line(epoch + j, means))
            epoch += k
            if checkpoint_path:
                save_checkpoint(checkpoint_path, model, eng, epoch, loss_history)
                nxt = draw(min(chunk, epochs - epoch)) if epoch < epochs else None
    for epoch in range(first, epochs if not fused else first):
        for rows in loader:                               # (:340) one global batch
            g = rows.numel()
            lo, hi = dp.split_rows(g, world_size, rank)
            e = None
            if eps == "host":
                e_all = torch.randn(g, Z)                 # reparameterize's randn_like (:205)
                e = e_all[lo:hi]
            elif eps != "philox":
                raise ValueError("eps must be 'host' or 'philox'")
            step.step(x_dev, idx=rows[lo:hi], eps=e, batch=hi - lo, global_batch=g, row0=lo, classes=cls_dev)
        sums = step.epoch_loss_sums().double().cpu().numpy()  # the only host sync of the epoch
        means = sums / n
        for k, v in zip(LOSS_KEYS, means):
            loss_history[k].append(float(v))
        if rank == 0 and log:
            log(epoch_line(epoch, means))
        if checkpoint_path:
            step.sync_state()  # every rank (a collective under the peer exchange)
            if rank == 0:
                save_checkpoint(checkpoint_path, model, eng, epoch + 1, loss_history)
    step.sync_state()
    step.close()
    weighted = weighted_history(loss_history, weights)
    if rank == 0:
        if loss_save_path:
            p = save_loss_csv(weighted, loss_save_path)
            if log:
                log(f"Loss history saved to CSV: {p}")
        if model_save_path:
            d = os.path.dirname(model_save_path)
            if d:
                os.makedirs(d, exist_ok=True)
            torch.save(cpu_state_dict(model), model_save_path)
            if log:
                log(f"Model saved to {model_save_path}")
    return model, loss_history, weighted


def default_paths(data_path, latent_dim, epochs):
    """The reference's save paths (Training_VAE.py:283-287): model and loss names from the dataset
    file name ('trajectory_sce1_cond.npy' → 'vae_offset_sce1_cond_ld8_epoch3000_loss2.*')."""
    name = os.path.splitext(os.path.basename(data_path))[0].replace("trajectory_", "", 1)
    stem = f"vae_offset_{name}_ld{latent_dim}_epoch{epochs}_loss2"
    return os.path.join("training", "models", stem + ".pth"), os.path.join("training", "loss", stem + ".png")


def main(argv=None):
    """``python -m cvae_amd.train --data training/DefensiveDataProcessed/trajectory_sce1_cond.npy``:
    the reference's ``__main__`` in mode='training' (Training_VAE.py:271-394) with its parameters
    as flags (same defaults: seq_len 10, dim 3, latent 8, batch 38, lr 1e-3, 3000 epochs, weights
    0.1/0.1/1.0/1.0).  Under ``torch.distributed.run`` every rank trains its share over RCCL."""
    import argparse
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("--data", required=True, nargs="+",
                    help="(N, seq_len, dim) .npy (Traj_Data_Process output); several = several scenes")
    ap.add_argument("--class-dim", type=int, default=0,
                    help="BASELINE cfg4: with several --data files, a scene-class embedding this wide (the "
                         "file index is the class)")
    ap.add_argument("--seq-len", type=int, default=10)
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--latent", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--batch-size", type=int, default=38, help="per rank under data parallelism")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--epochs", type=int, default=3000)
    ap.add_argument("--weights", type=float, nargs=4, default=(0.1, 0.1, 1.0, 1.0),
                    metavar=("RECON", "KLD", "START", "TIME"))
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="GEMM operand dtype; the dataset stays fp32 and the relative transform runs in fp32")
    ap.add_argument("--eps", default="host", choices=["host", "philox"])
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--model-out", default=None)
    ap.add_argument("--checkpoint", default=None, help="write a resume point (model + Adam + RNG) every epoch")
    ap.add_argument("--resume", default=None, help="continue from a --checkpoint file (--epochs = total)")
    ap.add_argument("--loss-out", default=None)
    a = ap.parse_args(argv)
    model_out, loss_out = default_paths(a.data[0], a.latent, a.epochs)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    device = None
    if world_size > 1:
        import torch.distributed as tdist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        tdist.init_process_group("nccl", device_id=device)
    try:
        data = a.data if len(a.data) > 1 else a.data[0]
        train(data, a.seq_len, a.dim, a.latent, batch_size=a.batch_size, lr=a.lr, epochs=a.epochs,
              hidden_dim=a.hidden, weights=tuple(a.weights), model_save_path=a.model_out or model_out,
              loss_save_path=a.loss_out or loss_out, dtype=a.dtype, eps=a.eps, device=device, seed=a.seed,
              checkpoint_path=a.checkpoint, resume=a.resume, class_dim=a.class_dim if len(a.data) > 1 else 0)
    finally:
        if world_size > 1:
            torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
