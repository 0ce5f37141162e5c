"""Data parallelism for the training step: one process per GPU, RCCL over xGMI.

The reference trains in one process (Training_VAE.py:326-370).  Every loss term is a mean over
batch elements (:240-264), so the gradient of the global-batch mean is the batch-weighted mean
of the per-rank gradients — one exchange per step:

    rank r:  forward_backward(rows of global batch assigned to r)   → grads_r (mean over B_r)
             grads_r *= B_r / B_global      (skipped when every rank has the same B_r)
             all_reduce(grads, SUM)                                 → global-mean gradient
             adam_step(grad_scale = 1/world  or 1)                  → identical params on every rank

Parameters and Adam moments are replicated (1.1 MB each at cfg2 — sharding them buys nothing);
the only collective on the data path is the 1.1 MB fp32 gradient all-reduce, plus one 5-float
all-reduce per epoch for the loss log.

Row assignment (``shard_rows``): every rank draws the same global permutation, cuts it into
global batches of ``batch_size * world`` and takes a contiguous slice of each, so a run over
``world`` ranks processes exactly the batches a single process with the global batch would.

The trainer only needs an engine with ``forward_backward / adam_step / grads / loss_accum``
(``CVAEEngine`` on the GPU; the CPU tests substitute an oracle-backed engine under gloo).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    """(rank, world_size) of the default group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def split_rows(n, world_size, rank):
    """[lo, hi) of ``rank``'s contiguous share of ``n`` rows (first ``n % world`` ranks get one more)."""
    q, r = divmod(n, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard_rows(perm, batch_size, world_size, rank):
    """Per-step (local_rows, global_batch) for one epoch of ``perm`` (1-D index tensor).

    Global batches are consecutive ``batch_size*world_size`` slices of ``perm`` (drop_last=False,
    like the reference DataLoader :327); a ragged last global batch is split as evenly as possible.
    """
    gb = batch_size * world_size
    out = []
    for s in range(0, perm.numel(), gb):
        g = perm[s:s + gb]
        lo, hi = split_rows(g.numel(), world_size, rank)
        out.append((g[lo:hi], g.numel()))
    return out


class DataParallelStep:
    """fwd+bwd → gradient all-reduce → Adam on every rank (the fused single-GPU step split in two)."""

    def __init__(self, engine, group=None):
        self.engine = engine
        self.group = group
        self.rank, self.world_size = world()
        if group is not None:
            self.rank, self.world_size = dist.get_rank(group), dist.get_world_size(group)

    def broadcast_params(self, src=0):
        """Start every rank from rank ``src``'s parameters (call once after init / load)."""
        if self.world_size > 1:
            dist.broadcast(self.engine.params, src, group=self.group)
            self.engine.pack()

    def step(self, x, idx=None, eps=None, batch=None, global_batch=None, weights=None):
        """One data-parallel training step; ``batch`` = this rank's rows, ``global_batch`` = Σ over ranks."""
        eng = self.engine
        if batch is None:
            batch = idx.numel() if idx is not None else x.shape[0]
        batch = int(batch)
        if global_batch is None:
            global_batch = batch * self.world_size
        if self.world_size == 1:
            if batch > 0:
                eng.train_step(x, idx=idx, eps=eps, batch=batch, weights=weights)
            return eng.loss
        if batch > 0:
            eng.forward_backward(x, idx=idx, eps=eps, batch=batch, weights=weights)
            if batch * self.world_size != global_batch:
                eng.grads.mul_(batch / global_batch)
                scale = 1.0
            else:
                scale = 1.0 / self.world_size
        else:  # an empty share of a ragged last batch still joins the collective
            eng.grads.zero_()
            scale = 1.0
        dist.all_reduce(eng.grads, op=dist.ReduceOp.SUM, group=self.group)
        eng.adam_step(grad_scale=scale)
        return eng.loss

    def epoch_loss_sums(self):
        """Σ over ranks of the device Σ loss·batch accumulators (5 floats); resets them."""
        acc = self.engine.loss_accum.clone()
        if self.world_size > 1:
            dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        self.engine.loss_accum.zero_()
        return acc
