"""The data-parallel exchange over xGMI without a collective library (include/cvae.h cvae_px_*,
csrc/cvae_peer.h; SURVEY §8e — the gradient exchange the reference's single process never needs,
Training_VAE.py:362-363 across ranks).

One process per GPU.  At set-up every rank exports its workspace and an uncached mailbox through
HIP IPC, the descriptors are all-gathered over the process group (any backend: gloo or RCCL) and
every rank maps every other rank's buffers.  From then on a training step is two launches per
rank — the row chain on its rows, and the weight-gradient launch that pushes each dW tile's fp32
partial to the tile's owner (rank = tile mod world), lets the owner sum the partials in rank
order and apply Adam, and has the owner write the new operand copies into every rank's
workspace.  No collective call, no host synchronisation, no per-step host values (the step's
epoch is the device counter), so steps replay from a hipGraph as well.

State ownership: the fp32 master parameters and Adam moments of a weight are current only on the
rank owning its tile; ``gather_state`` (masked sum over the group: exact, one non-zero term per
element) makes them whole on every rank — before a checkpoint, a state_dict, the end of training.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from ._lib import CVAE_X_OPERAND, check, lib, ptr


class PeerExchange:
    def __init__(self, engine, group=None, probe=True):
        """Collective over the group: every rank constructs it together.  A failure on any rank
        (export, import, the probe) is agreed on by all ranks before anyone raises, so no rank
        is left waiting in a collective the others skipped."""
        self.engine = engine
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._open = False
        if self.world < 2:
            raise ValueError("the peer exchange needs world >= 2 (one GPU trains with the fused step)")
        h = engine._h

        def agree(ok, what):
            oks = [None] * self.world
            dist.all_gather_object(oks, ok, group=group)
            bad = [r for r, v in enumerate(oks) if v is not True]
            if bad:
                lib().cvae_px_close(h)
                raise RuntimeError(f"peer exchange {what} failed on ranks {bad}: "
                                   f"{[oks[r] for r in bad][:2]}")

        blob = b""
        try:
            n = C.c_int64()
            check(lib().cvae_px_blob_bytes(C.byref(n)))
            buf = (C.c_char * n.value)()
            check(lib().cvae_px_export(h, self.world, self.rank, buf), "cvae_px_export")
            blob, ok = bytes(buf), True
        except Exception as e:  # noqa: BLE001
            ok = f"{type(e).__name__}: {e}"
        agree(ok, "export")
        blobs = [None] * self.world
        dist.all_gather_object(blobs, blob, group=group)
        # the step epoch is counted from here: every rank must be at the same optimizer step
        base = engine.sync_counters()[1]
        steps = [None] * self.world
        dist.all_gather_object(steps, base, group=group)
        agree(True if len(set(steps)) == 1 else f"optimizer steps differ {steps}", "set-up")
        try:
            allb = b"".join(blobs)
            cbuf = (C.c_char * len(allb)).from_buffer_copy(allb)
            check(lib().cvae_px_import(h, cbuf, int(base)), "cvae_px_import")
            ok = True
        except Exception as e:  # noqa: BLE001
            ok = f"{type(e).__name__}: {e}"
        agree(ok, "import")
        dist.barrier(group=group)  # every mailbox is zeroed and mapped before anyone stores into it
        if probe:
            try:
                good = C.c_int()
                check(lib().cvae_px_probe(h, C.byref(good)), "cvae_px_probe")
                ok = True if good.value == 1 else "tags did not arrive"
            except Exception as e:  # noqa: BLE001
                ok = f"{type(e).__name__}: {e}"
            agree(ok, "probe")
        mask = (C.c_uint8 * engine.n_params)()
        check(lib().cvae_px_owned(h, mask), "cvae_px_owned")
        self.owned = torch.frombuffer(bytearray(mask), dtype=torch.uint8).to(engine.device).bool()
        self._open = True

    def layout(self):
        """(ranks on this rank's GPU, tile blocks of the exchange launch) — cvae_px_layout: the
        residency precondition the launch was sized for (csrc/cvae_peer.h)."""
        k, g = C.c_int(), C.c_int()
        check(lib().cvae_px_layout(self.engine._h, C.byref(k), C.byref(g)), "cvae_px_layout")
        return k.value, g.value

    def reset(self):
        """Re-arm the exchange (collective): after a resume or a restore changed the device step
        counter, or after a bounded wait timed out (the fault word; make the state whole first —
        ``gather_state``).  Every rank synchronises, meets a barrier, zeroes its arrival flags and
        done counter, counts the step epoch from the current counters[1] (which must agree on every
        rank) and clears its fault word; a second barrier keeps anyone from pushing early."""
        eng = self.engine
        torch.cuda.synchronize(eng.device)
        base = eng.sync_counters()[1]
        steps = [None] * self.world
        dist.all_gather_object(steps, base, group=self.group)
        if len(set(steps)) != 1:
            raise RuntimeError(f"peer exchange reset: optimizer steps differ across ranks {steps}")
        dist.barrier(group=self.group)
        check(lib().cvae_px_reset(eng._h, int(base)), "cvae_px_reset")
        dist.barrier(group=self.group)

    def step(self, x, idx=None, eps=None, batch=None, global_batch=None, weights=None, row0=None, accumulate=True,
             sizes=None):
        """One data-parallel step: this rank's ``batch`` rows (0 allowed) of a global batch.

        ``sizes``: every rank's row count.  Without it the shares are the ones ``dist.split_rows``
        gives (as every rank computes them alike: no collective); a rank whose batch differs from
        its share there raises instead of weighting its partial wrongly."""
        eng = self.engine
        if batch is None:
            batch = idx.numel() if idx is not None else x.shape[0]
        batch = int(batch)
        if global_batch is None:
            global_batch = batch * self.world
        global_batch = int(global_batch)
        if sizes is None:
            q, r = divmod(global_batch, self.world)
            sizes = [q + (1 if k < r else 0) for k in range(self.world)]
            if sizes[self.rank] != batch:
                raise ValueError(f"rank {self.rank}: batch {batch} is not its split_rows share {sizes[self.rank]} of "
                                 f"global batch {global_batch}; pass sizes= (every rank's rows)")
        sizes = [int(s) for s in sizes]
        if len(sizes) != self.world or sum(sizes) != global_batch or sizes[self.rank] != batch:
            raise ValueError(f"sizes {sizes} do not describe rank {self.rank}'s batch {batch} of {global_batch}")
        if row0 is None:
            row0 = sum(sizes[:self.rank])
        scales = None
        if any(s != sizes[0] for s in sizes):  # ragged: the partials are weighted by B_r / B_global
            scales = (C.c_float * self.world)(*[s / global_batch for s in sizes])
        xp = idxp = ep = None
        xfl = CVAE_X_OPERAND
        if batch > 0:
            x, idx, batch = eng._prep(x, idx, batch)
            xp, idxp, xfl = ptr(x), ptr(idx), eng._xflags(x)
            e = eng._eps(eps, batch)
            ep = ptr(e)
        eng.ensure_packed()
        check(lib().cvae_px_train_step(
            eng._h, xp, idxp, batch, xfl, ep, eng.seed, int(row0), C.byref(eng._weights(weights)), ptr(eng.params),
            ptr(eng.m), ptr(eng.v), C.byref(eng._adam()), scales, ptr(eng.loss),
            ptr(eng.loss_accum) if accumulate else None, ptr(eng.counters), eng._stream()), "cvae_px_train_step")
        eng._ctr[0] += 1
        eng._ctr[1] += 1
        return eng.loss

    def prepare(self, x, batch):
        """``run(k)``: k equal-share steps on rows 0..batch-1 of the resident ``x``, Philox eps
        (bench.py's timed call: every argument converted once)."""
        eng = self.engine
        x = eng.as_input(x)
        B = int(batch)
        eng._check_rows(x, None, B)
        eng.ensure_packed()
        f = lib().cvae_px_train_step
        w, a = eng._weights(None), eng._adam()
        args = (eng._h, C.c_void_p(x.data_ptr()), None, C.c_int(B), C.c_int(eng._xflags(x)), None,
                C.c_uint64(eng.seed), C.c_int64(self.rank * B), C.byref(w), ptr(eng.params), ptr(eng.m),
                ptr(eng.v), C.byref(a), None, ptr(eng.loss), ptr(eng.loss_accum), ptr(eng.counters), eng._stream())
        ctr = eng._ctr

        def run(k, _f=f, _args=args, _keep=(x, w, a), _ctr=ctr):
            for _ in range(k):
                rc = _f(*_args)
                if rc < 0:
                    check(rc, "cvae_px_train_step")
            _ctr[0] += k
            _ctr[1] += k
        return run

    def stats(self, reset=False):
        """This rank's exchange waits (cvae_px_stats), in microseconds: the longest owner-tile
        wait for the partials, the longest end-of-launch wait, the mean owner-tile wait."""
        out = (C.c_uint64 * 4)()
        check(lib().cvae_px_stats(self.engine._h, out, 1 if reset else 0), "cvae_px_stats")
        return {"owner_wait_max_us": out[0] / 100.0, "end_wait_max_us": out[1] / 100.0,
                "owner_wait_mean_us": out[2] / 100.0 / max(out[3], 1), "owner_waits": int(out[3])}

    def verify(self, rows=64):
        """Self-check outside any timed region (bench.py runs it after warm-up AND after the timed
        steps); collective over the group.  Passes when
          * no rank's fault word is set (no bounded wait gave up);
          * every rank's operand copies — written by the tiles' owners — have the same checksum
            (cvae_operand_checksum over every byte of W, Wᵀ and the biases), and that checksum is
            unchanged by ``gather_state()``'s repack from the whole master state: the broadcast
            delivered the owners' update, byte for byte, everywhere;
          * a forward pass over seeded rows (eps = 0) gives identical outputs before and after.
        Returns True, or the first failing rank's reason (the same value on every rank; a local
        error becomes a reason, so no rank is left in a collective)."""
        eng = self.engine
        S, D, Z = eng.shape[:3]
        rows = min(int(rows), eng.max_batch)
        reason = before = None
        ck_before = 0

        def outs(probe, eps):
            return torch.cat([t.flatten() for t in eng.forward(probe, eps=eps, batch=rows, offset=0)])
        try:
            torch.cuda.synchronize(eng.device)
            f = eng.fault()
            if f:
                reason = f"fault word {f:#x} (a bounded wait gave up)"
            else:
                ck_before = eng.operand_checksum()
                probe = eng.as_input(torch.randn(rows, S, D, generator=torch.Generator().manual_seed(7)))
                eps = torch.zeros(rows, Z, device=eng.device, dtype=torch.float32)
                before = outs(probe, eps)
        except Exception as e:  # noqa: BLE001
            reason = f"{type(e).__name__}: {e}"
        cks = [None] * self.world
        dist.all_gather_object(cks, ck_before, group=self.group)
        if reason is None and len(set(cks)) != 1:
            reason = f"operand-copy checksums differ across ranks {[hex(c) for c in cks]}"
        self.gather_state()
        if reason is None:
            try:
                ck_after = eng.operand_checksum()
                if ck_after != ck_before:
                    reason = (f"operand-copy checksum {ck_before:#x} (broadcast) != {ck_after:#x} (repacked from "
                              f"the gathered master state)")
                else:
                    after = outs(probe, eps)
                    if not torch.equal(before, after):
                        n = int((before != after).sum())
                        reason = f"{n} forward outputs differ between the broadcast and the repacked operand copies"
            except Exception as e:  # noqa: BLE001
                reason = f"{type(e).__name__}: {e}"
        reasons = [None] * self.world
        dist.all_gather_object(reasons, reason, group=self.group)
        bad = [(r, v) for r, v in enumerate(reasons) if v]
        self.last_checksum = cks[0]
        return True if not bad else f"rank {bad[0][0]}: {bad[0][1]}"

    def gather_state(self):
        """Whole fp32 params / Adam moments on every rank (each element from its owner), and the
        operand copies repacked from them."""
        eng = self.engine
        with torch.no_grad():
            for t in (eng.params, eng.m, eng.v):
                t.copy_(torch.where(self.owned, t, torch.zeros_like(t)))
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        eng.pack()

    def close(self):
        """Unmap the peers and free the mailbox; every rank calls it (it barriers first)."""
        if not self._open:
            return
        torch.cuda.synchronize(self.engine.device)
        dist.barrier(group=self.group)
        lib().cvae_px_close(self.engine._h)
        self._open = False
