"""Data parallelism for the training step: one process per GPU, RCCL over xGMI.

The reference trains in one process (Training_VAE.py:326-370).  Every loss term is a mean over
batch elements (:240-264), so the gradient of the global-batch mean is the batch-weighted mean
of the per-rank gradients — one exchange per step:

    rank r:  forward_backward(rows lo_r..hi_r of global batch)          → grads_r (mean over B_r)
             grads_r *= B_r / B_global      (skipped when every rank has the same B_r)
             all_reduce(grads, SUM)                                    → global-mean gradient
             adam_step(grad_scale = 1/world  or 1)                     → identical params on every rank

Parameters and Adam moments are replicated (1.1 MB each at cfg2 — sharding them buys nothing);
the only collective on the data path is the 1.1 MB fp32 gradient all-reduce, plus one 5-double
all-reduce per epoch for the loss log.

eps: the in-kernel Philox draw is keyed by the GLOBAL row (``row0`` = lo_r, the rank's first row
of the global batch) and every rank advances the same device offset, so the ranks of a global
batch draw exactly the noise one process with that batch draws — not rank 0's noise B_r times.

The all-reduce itself: the library's own RCCL communicator (``NativeRccl``: include/cvae.h
cvae_rccl_*; the unique id broadcast over the group with rank 0's status, the ranks agreeing on
success before any uses it) issues ncclAllReduce on the stream the step's kernels run on — no
framework stream between the dW and Adam launches, so a captured step graph is the chain, dW, the
RCCL kernels and Adam on one stream.  It is the default at world 1 (``bench.py --dp``) and opt-in
(``native=True``) at world > 1, where torch.distributed's all_reduce (RCCL under the nccl backend)
runs until a multi-GPU run has checked the library's communicator; the CPU tests' engine uses it too.

Two-bucket overlap (``buckets=2``): the dW launch is split into the decoder layers (a contiguous
tail of the flat gradient, ready first) and the rest; the decoder bucket's all-reduce runs on a
communication stream (every all-reduce of the communicator on that one stream, in one order on
every rank) while the rest of the dW GEMMs run on the compute stream, then the second bucket
follows on the communication stream and Adam waits for both.

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


class NativeRccl:
    """The gradient all-reduce issued by libcvae_hip on a given stream (cvae_rccl_init /
    cvae_rccl_allreduce): rank 0 makes the RCCL unique id, the group broadcasts it (any backend),
    every rank joins the communicator on its engine's device."""

    def __init__(self, engine, group=None):
        import ctypes as C
        from ._lib import check, lib
        self.engine = engine
        L = lib()
        n = C.c_int64()
        check(L.cvae_rccl_id_bytes(C.byref(n)), "cvae_rccl_id_bytes")
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        idb = (C.c_uint8 * n.value)()
        ok, why = 1, ""
        if rank == 0:
            rc = L.cvae_rccl_unique_id(idb)
            if rc < 0:
                ok, why = 0, f"cvae_rccl_unique_id failed ({rc}): {L.cvae_last_error().decode(errors='replace')}"
        if world > 1:
            # the id travels with rank 0's status: a rank-0 failure reaches every rank in
            # the same broadcast, so no rank is left waiting in a collective the others skipped
            dev = engine.device if dist.get_backend(group) == "nccl" else "cpu"
            t = torch.tensor([ok] + list(bytes(idb)), dtype=torch.uint8, device=dev)
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(t, src=src, group=group)
            tl = t.cpu().tolist()
            ok = tl[0]
            idb = (C.c_uint8 * n.value)(*tl[1:])
        if not ok:
            raise RuntimeError(why or "rank 0 could not create the RCCL unique id")
        rc = L.cvae_rccl_init(engine._h, idb, world, rank)
        if world > 1:
            # every rank joins the library's communicator or none does: one agreed flag
            dev = engine.device if dist.get_backend(group) == "nccl" else "cpu"
            f = torch.tensor([1 if rc >= 0 else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MIN, group=group)
            if int(f.item()) == 0:
                if rc >= 0:
                    L.cvae_rccl_close(engine._h)
                raise RuntimeError("cvae_rccl_init failed on at least one rank")
        check(rc, "cvae_rccl_init")
        self.world, self.rank = world, rank

    def all_reduce(self, buf, stream=None):
        """In-place float32 sum of ``buf`` over the ranks, enqueued on ``stream`` (default: the
        current stream of the engine's device)."""
        import ctypes as C
        from ._lib import check, lib
        st = stream if stream is not None else torch.cuda.current_stream(self.engine.device)
        check(lib().cvae_rccl_allreduce(self.engine._h, C.c_void_p(buf.data_ptr()), buf.numel(),
                                        C.c_void_p(st.cuda_stream)), "cvae_rccl_allreduce")

    def close(self):
        from ._lib import lib
        lib().cvae_rccl_close(self.engine._h)


class DataParallelStep:
    """fwd+bwd → gradient all-reduce → Adam on every rank (the fused single-GPU step split in two).

    ``force_split``: run the split path (and its all-reduce) even at world 1 — the route every rank
    of a multi-GPU run takes, measurable on one GPU (``bench.py --dp``).
    ``buckets``: 1 = one all-reduce after the whole dW launch; 2 = decoder bucket overlapped with
    the rest of the dW GEMMs (see the module docstring)."""

    def __init__(self, engine, group=None, force_split=False, buckets=1, exchange="rccl", native=None,
                 shard_adam=False):
        self.engine = engine
        # shard_adam (the RCCL path, one bucket): reduce-scatter of the flat gradient, Adam on this rank's
        # 1/world of the flat state (cvae_adam_flat), all-gather of the parameters, repack — instead of an
        # all-reduce and the whole Adam on every rank (ZeRO-1: m, v current on their shard only)
        self.shard_adam = bool(shard_adam)
        self._sh = None
        self.group = group
        self.rank, self.world_size = world()
        if group is not None:
            self.rank, self.world_size = dist.get_rank(group), dist.get_world_size(group)
        self.force_split = force_split
        if buckets not in (1, 2):
            raise ValueError("buckets must be 1 or 2")
        self.buckets = buckets
        # exchange: "rccl" = all-reduce of the flat gradient, then Adam; "peer" = the in-kernel
        # exchange over IPC-mapped peer memory (cvae_amd.peer); "auto" = peer where it serves the
        # configuration and its set-up probe passes, else rccl.  self.exchange says which runs.
        self.px = None
        self.exchange = "rccl"
        self.exchange_note = ""
        if exchange not in ("rccl", "peer", "auto"):
            raise ValueError("exchange must be 'rccl', 'peer' or 'auto'")
        if exchange != "rccl" and self.world_size > 1:
            try:
                from .peer import PeerExchange
                if getattr(engine, "train_kernel", None) != "ring":
                    raise ValueError(f"the peer exchange serves the ring chain, this engine runs "
                                     f"{getattr(engine, 'train_kernel', None)!r}")
                self.px = PeerExchange(engine, group)
                self.exchange = "peer"
            except Exception as e:  # noqa: BLE001 — "auto" falls back, "peer" re-raises
                if exchange == "peer":
                    raise
                self.exchange_note = f"peer exchange unavailable ({type(e).__name__}: {e}); rccl"
        # the all-reduce path: the library's own RCCL communicator on the step's stream (native), or
        # torch.distributed's all_reduce (native=False; engines without a HIP handle)
        self.rccl = None
        self._comm_stream = None
        if native is None:
            # a lone rank (world 1: bench --dp, the split step's measurement).  At world > 1 the library's
            # communicator is opt-in (native=True) until a multi-GPU run has checked it against
            # torch's all-reduce bit for bit: torch.distributed's RCCL all-reduce by default
            native = hasattr(engine, "_h") and torch.cuda.is_available() and self.world_size == 1 and self.px is None
        if self.shard_adam and (buckets != 1 or self.px is not None):
            raise ValueError("shard_adam is the one-bucket RCCL path")
        if native and self.split and not self.shard_adam:
            try:
                self.rccl = NativeRccl(engine, group)
            except Exception as e:  # noqa: BLE001 — torch's all_reduce takes over, and the line says so
                if native is True:  # asked for explicitly: every rank raises (NativeRccl agrees on failure)
                    raise
                self.exchange_note = (self.exchange_note + "; " if self.exchange_note else "") + \
                    f"native RCCL unavailable ({type(e).__name__}: {e}); torch all_reduce"

    @property
    def split(self):
        return self.world_size > 1 or self.force_split

    def broadcast_params(self, src=0):
        """Start every rank from rank ``src``'s parameters (call once after init / load)."""
        if self.world_size > 1:
            dist.broadcast(self.engine.params, src, group=self.group)
            self.engine.pack()

    def step(self, x, idx=None, eps=None, batch=None, global_batch=None, weights=None, row0=None, classes=None,
             sizes=None):
        """One data-parallel training step; ``batch`` = this rank's rows, ``global_batch`` = Σ over
        ranks, ``row0`` = this rank's first row in the global batch (default: the sum of the lower
        ranks' ``sizes``, else this rank's ``split_rows`` share of ``global_batch`` — rank · batch
        for equal shares); ``sizes`` = every rank's rows (peer exchange; default: ``split_rows``
        shares)."""
        eng = self.engine
        if batch is None:
            batch = idx.numel() if idx is not None else x.shape[0]
        batch = int(batch)
        if global_batch is None:
            global_batch = batch * self.world_size
        if row0 is None:  # rank · batch is wrong for ragged shares (7 rows over 2 ranks)
            row0 = (split_rows(global_batch, self.world_size, self.rank)[0] if sizes is None
                    else sum(sizes[:self.rank]))
        if self.px is not None:
            if classes is not None:
                raise ValueError("the peer exchange serves the reference model (no class embedding)")
            return self.px.step(x, idx=idx, eps=eps, batch=batch, global_batch=global_batch, weights=weights,
                                row0=row0, sizes=sizes)
        if not self.split:
            if batch > 0:
                eng.train_step(x, idx=idx, eps=eps, batch=batch, weights=weights, row0=row0,
                               **({"classes": classes} if classes is not None else {}))
            return eng.loss
        two = self.buckets == 2  # every rank issues the same collectives, empty shares included
        if batch > 0:
            parts = 3 if two else 7  # CVAE_PART_CHAIN | DW_DEC, or CVAE_PART_ALL
            eng.forward_backward(x, idx=idx, eps=eps, batch=batch, weights=weights, row0=row0, parts=parts,
                                 **({"classes": classes} if classes is not None else {}))
            ragged = batch * self.world_size != global_batch
            scale = 1.0 if ragged else 1.0 / self.world_size
        else:  # an empty share of a ragged last batch still joins the collectives, and its device
            eng.grads.zero_()  # step counters advance as the other ranks' launches advance theirs
            eng.skip_step()
            ragged, scale = True, 1.0
        g = eng.grads
        if self.shard_adam:
            if ragged and batch > 0:
                g.mul_(batch / global_batch)
            self._sharded_update(g, scale)
            return eng.loss
        if two and self.rccl is not None:  # the communication stream: both buckets, in order
            main = torch.cuda.current_stream(eng.device)
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(device=eng.device)
            cs = self._comm_stream
            dec, rest = g[eng.bucket_split:], g[:eng.bucket_split]
            if ragged:
                dec.mul_(batch / global_batch)
            cs.wait_stream(main)
            self.rccl.all_reduce(dec, cs)
            if batch > 0:
                eng.wgrad_rest(batch)  # beside the decoder bucket's all-reduce
            if ragged:
                rest.mul_(batch / global_batch)
            cs.wait_stream(main)
            self.rccl.all_reduce(rest, cs)
            main.wait_stream(cs)
        elif two:
            dec, rest = g[eng.bucket_split:], g[:eng.bucket_split]
            if ragged:
                dec.mul_(batch / global_batch)
            w1 = dist.all_reduce(dec, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if batch > 0:
                eng.wgrad_rest(batch)  # beside the decoder bucket's all-reduce
            if ragged:
                rest.mul_(batch / global_batch)
            w2 = dist.all_reduce(rest, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            w1.wait()
            w2.wait()
        else:
            if ragged and batch > 0:
                g.mul_(batch / global_batch)
            if self.rccl is not None:
                self.rccl.all_reduce(g)  # on the compute stream, between the dW and Adam launches
            else:
                dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
        eng.adam_step(grad_scale=scale)
        return eng.loss

    # ---- the sharded optimizer (shard_adam)
    def _shard_bufs(self):
        """(n, shard, lo, count): the flat state cut into world slices of ``shard`` elements (a multiple
        of 64), this rank's [lo, lo + count); buffers for the padded collectives."""
        eng = self.engine
        n, w = eng.n_params, self.world_size
        shard = -(-(-(-n // w)) // 64) * 64
        lo = self.rank * shard
        cnt = max(0, min(shard, n - lo))
        if self._sh is None:
            kw = dict(device=eng.params.device, dtype=torch.float32)
            self._sh = {"gpad": torch.zeros(w * shard, **kw), "gsh": torch.zeros(shard, **kw),
                        "ppad": torch.zeros(w * shard, **kw), "psh": torch.zeros(shard, **kw)}
        return n, shard, lo, cnt

    def _reduce_scatter(self, out, inp):
        if not dist.is_initialized():
            out.copy_(inp)
        elif dist.get_backend(self.group) == "nccl":
            dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group)
        else:  # gloo has no reduce-scatter: the all-reduced sum, this rank's slice of it
            t = inp.clone()
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            out.copy_(t[self.rank * out.numel():(self.rank + 1) * out.numel()])

    def _all_gather(self, out, inp):
        if not dist.is_initialized():
            out.copy_(inp)
        elif dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, inp, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world_size)), inp, group=self.group)

    def _gather_flat(self, t):
        """Whole ``t`` (a flat n-element state buffer current on each rank's shard) on every rank."""
        n, shard, lo, cnt = self._shard_bufs()
        b = self._sh
        b["psh"].zero_()
        b["psh"][:cnt].copy_(t[lo:lo + cnt])
        self._all_gather(b["ppad"], b["psh"])
        t.copy_(b["ppad"][:n])

    def _sharded_update(self, g, grad_scale):
        """reduce-scatter(grads) → Adam on this rank's shard → all-gather(params) → repack."""
        eng = self.engine
        n, shard, lo, cnt = self._shard_bufs()
        b = self._sh
        b["gpad"][:n].copy_(g)
        self._reduce_scatter(b["gsh"], b["gpad"])
        if cnt > 0:
            eng.adam_flat(b["gsh"][:cnt], lo, grad_scale)
        else:
            eng.adam_flat(b["gsh"][:0], 0, grad_scale)  # no elements: nothing to update
        self._gather_flat(eng.params)
        eng.pack()

    def sync_state(self):
        """Whole parameters and Adam moments on every rank (the peer exchange keeps each element
        current on its owner only, shard_adam keeps m and v current on their shard); a no-op for the
        all-reduce path, where every rank holds all."""
        if self.px is not None:
            self.px.gather_state()
        if self.shard_adam and self.world_size > 1:
            self._gather_flat(self.engine.m)
            self._gather_flat(self.engine.v)

    def counters_changed(self):
        """The device step counter was set from outside the step (a resume, a restore): the peer
        exchange counts its flag epochs from it and must be re-armed (collective)."""
        if self.px is not None:
            self.px.reset()

    def verify_exchange(self, fallback=True):
        """The peer exchange's self-check (``PeerExchange.verify``).  On a failure with ``fallback``
        every rank closes it together, clears its fault word and continues on the RCCL all-reduce:
        the master state was made whole by the check, so the ranks agree, and a fault word left set
        would fail the RCCL path's first call.  Returns True or the failure, which
        ``exchange_note`` keeps."""
        if self.px is None:
            return True
        ok = self.px.verify()
        if ok is not True and fallback:
            self.px.close()
            self.px = None
            self.engine.clear_fault()
            self.exchange = "rccl"
            self.exchange_note = f"peer exchange failed its warm-up check ({ok}); rccl"
        return ok

    def close(self):
        if self.px is not None:
            self.px.close()
            self.px = None
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None

    def epoch_loss_sums(self):
        """Σ over ranks of the device Σ loss·batch accumulators (5 doubles); resets them."""
        acc = self.engine.loss_accum.clone()
        if self.world_size > 1:
            dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        self.engine.loss_accum.zero_()
        return acc


class GraphedStep:
    """A training step captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed.

    Replay is correct because every per-step quantity lives on the device: the Philox offset and
    the Adam step are the engine's device counters, advanced by the kernels themselves; inputs
    must sit in fixed device buffers (``x`` resident, ``idx`` a fixed tensor the caller refills).
    ``fn`` is the step (e.g. ``lambda: dp.step(x, batch=B)``); ``n`` steps per replay.  Before the
    capture ``warmup`` eager steps run on a side stream (torch's capture recipe); they are real
    training steps.  The capture itself executes nothing."""

    def __init__(self, engine, fn, n=1, warmup=1):
        self.engine, self.fn, self.n = engine, fn, int(n)
        s = torch.cuda.Stream(device=engine.device)
        s.wait_stream(torch.cuda.current_stream(engine.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream(engine.device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for _ in range(self.n):
                fn()
        # the capture launched nothing; the host mirrors counted the captured calls: undo that
        self.engine.sync_counters()

    def replay(self):
        self.graph.replay()
        self.engine._ctr[0] += self.n
        self.engine._ctr[1] += self.n
