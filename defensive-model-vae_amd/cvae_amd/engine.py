"""Device engine: one C-ABI handle + the flat fp32 parameter / Adam / gradient buffers.

The engine owns what the reference spreads over ``ConditionalTrajectoryVAE``
parameters, ``torch.optim.Adam`` state and autograd (Training_VAE.py:331-363):

* ``params``  flat fp32, state_dict order; the bound module's parameters are views
* ``m, v``    Adam moments (torch ``exp_avg``/``exp_avg_sq``), same layout
* ``grads``   flat fp32 gradient (data-parallel path); bound ``p.grad`` are views
* ``loss``    fp32[5] last step's (total, recon, kld, start, time)  — on device
* ``loss_accum`` fp64[5] running Σ loss·batch for the epoch (Python-double sums of the
  reference, Training_VAE.py:366-370)                             — on device
* ``counters`` int64[2] device step counters (include/cvae.h): [0] the Philox offset of the
  next training step, [1] optimizer steps begun.  Every training call reads and advances them
  ON THE DEVICE, so a captured step (hipGraph) replays correctly; ``rng_offset`` /
  ``step_count`` are host mirrors kept in step with every call the host issues.

Every call enqueues HIP kernels on torch's current stream and returns without
synchronising.  Nothing falls back to torch compute.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import (CVAE_BF16, CVAE_F32, CVAE_FP8, CVAE_PART_ALL, CVAE_PART_CHAIN, CVAE_PART_DW_DEC,
                   CVAE_PART_DW_REST, CVAE_X_F32, CVAE_X_OPERAND, CvaeAdamConfig, CvaeConfig, CvaeLossWeights,
                   check, lib, ptr)

# "fp8": bf16 activations with OCP e4m3 forward GEMM operands (BASELINE cfg5; cvae.h CVAE_FP8)
DTYPES = {"fp32": (CVAE_F32, torch.float32), "bf16": (CVAE_BF16, torch.bfloat16),
          "fp8": (CVAE_FP8, torch.bfloat16)}
DEFAULT_WEIGHTS = (0.1, 0.1, 1.0, 1.0)  # Training_VAE.py:300-306


def config_info(seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4, dtype="fp32", max_batch=1,
                n_classes=0, class_dim=0):
    """Host-only query: (n_params, n_tensors, lds_bytes) — works without a GPU."""
    cfg = CvaeConfig(seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec, DTYPES[dtype][0], max_batch, n_classes,
                     class_dim)
    n = C.c_int64()
    nt = C.c_int()
    lds = C.c_int()
    check(lib().cvae_config_info(C.byref(cfg), C.byref(n), C.byref(nt), C.byref(lds)), "cvae_config_info")
    return n.value, nt.value, lds.value


class CVAEEngine:
    def __init__(self, seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4, dtype="fp32",
                 max_batch=1024, device=None, seed=0, n_classes=0, class_dim=0):
        if not torch.cuda.is_available():
            raise RuntimeError("CVAEEngine needs a HIP device (MI355X); there is no CPU fallback")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.dtype_name = dtype
        self.cdtype, self.tdtype = DTYPES[dtype]
        self.shape = (seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec)
        self.n_classes, self.class_dim = int(n_classes), int(class_dim)
        self.max_batch = max_batch
        cfg = CvaeConfig(seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec, self.cdtype, max_batch, self.n_classes,
                         self.class_dim)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().cvae_create(C.byref(cfg), self.device.index, C.byref(h)), "cvae_create")
        self._h = h
        n = C.c_int64()
        nt = C.c_int()
        check(lib().cvae_num_params(h, C.byref(n), C.byref(nt)))
        self.n_params = n.value
        self.tensors = []
        for i in range(nt.value):
            off, numel, rows, cols = C.c_int64(), C.c_int64(), C.c_int(), C.c_int()
            check(lib().cvae_param_info(h, i, C.byref(off), C.byref(numel), C.byref(rows), C.byref(cols)))
            shape = (rows.value, cols.value) if cols.value > 0 else (rows.value,)
            self.tensors.append((off.value, numel.value, shape))
        split = C.c_int64()
        check(lib().cvae_bucket_split(h, C.byref(split)))
        self.bucket_split = split.value  # decoder.0.weight: grads[split:] is the decoder bucket
        kw = dict(device=self.device, dtype=torch.float32)
        self.params = torch.zeros(self.n_params, **kw)
        self.m = torch.zeros(self.n_params, **kw)
        self.v = torch.zeros(self.n_params, **kw)
        self.grads = torch.zeros(self.n_params, **kw)
        self.loss = torch.zeros(5, **kw)
        self.loss_accum = torch.zeros(5, device=self.device, dtype=torch.float64)
        # [offset, steps begun, Adam scalars of that step (2 x fp32), reserved] — include/cvae.h
        self.counters = torch.zeros(4, device=self.device, dtype=torch.int64)
        self._ctr = [0, 0]  # host mirrors of counters
        self.seed = int(seed)
        self.lr, self.betas, self.eps = 1e-3, (0.9, 0.999), 1e-8
        self.weights = DEFAULT_WEIGHTS
        self._module = None
        self._packed_version = None
        # fp32 trajectories handed to a bf16/fp8 engine: False = rounded to the operand dtype on upload
        # (synthetic N(0,1) data), True = kept fp32, relative transform in fp32 (real data; train())
        self.keep_f32 = False

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            # the handle's arena and buffers are freed below: let every launch queued on this
            # engine's device finish first (an engine dropped right after an asynchronous step)
            try:
                torch.cuda.synchronize(self.device)
            except Exception:
                pass
            lib().cvae_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def views(self, flat):
        return [flat[o:o + n].view(shape) for (o, n, shape) in self.tensors]

    def bind(self, module):
        """Make ``module``'s parameters (state_dict order) views of ``self.params``."""
        plist = list(module.parameters())
        if len(plist) != len(self.tensors):
            raise ValueError(f"module has {len(plist)} parameters, engine layout has {len(self.tensors)}")
        with torch.no_grad():
            for p, view, gview in zip(plist, self.views(self.params), self.views(self.grads)):
                if tuple(p.shape) != tuple(view.shape):
                    raise ValueError(f"parameter shape {tuple(p.shape)} != layout {tuple(view.shape)}")
                view.copy_(p.detach().to(self.device, torch.float32))
                p.data = view
                p.grad = gview
        self._module = module
        self.pack()
        return self

    def _param_version(self):
        m = self._module
        return None if m is None else sum(p._version for p in m.parameters())

    def pack(self):
        """Refresh the device operand copies (W, Wᵀ, bias) after parameters were written."""
        check(lib().cvae_pack_weights(self._h, ptr(self.params), self._stream()), "cvae_pack_weights")
        self._packed_version = self._param_version()

    def ensure_packed(self):
        """Repack if the bound parameters were modified in place since the last pack (an optimizer
        outside this library, e.g. torch.optim.Adam over model.parameters())."""
        if self._module is not None and self._param_version() != self._packed_version:
            self.pack()

    def set_optimizer(self, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)

    def _adam(self):
        return CvaeAdamConfig(self.lr, self.betas[0], self.betas[1], self.eps)

    def reset_optimizer(self):
        self.m.zero_()
        self.v.zero_()
        self.step_count = 0

    # ------------------------------------------------------------------ optimizer state (resume)
    def optimizer_state_dict(self):
        """Adam state in torch.optim.Adam.state_dict() format (CPU tensors): per parameter index
        {'step', 'exp_avg', 'exp_avg_sq'} and one param group — loadable by torch's Adam over
        model.parameters(), and by load_optimizer_state_dict."""
        return optimizer_state_dict(self)

    def load_optimizer_state_dict(self, sd):
        load_optimizer_state_dict(self, sd)

    # ------------------------------------------------------------------ step counters
    @property
    def rng_offset(self):
        return self._ctr[0]

    @rng_offset.setter
    def rng_offset(self, v):
        self._ctr[0] = int(v)
        self.counters[0].fill_(int(v))

    @property
    def step_count(self):
        return self._ctr[1]

    @step_count.setter
    def step_count(self, v):
        self._ctr[1] = int(v)
        self.counters[1].fill_(int(v))

    def sync_counters(self):
        """Host mirrors ← device counters (after graph replays the host did not count)."""
        c = self.counters[:2].cpu().tolist()
        self._ctr = [int(c[0]), int(c[1])]
        return tuple(self._ctr)

    # ------------------------------------------------------------------ inputs
    def as_input(self, x, keep_f32=False):
        """Trajectories on the device, contiguous: in the operand dtype, or — keep_f32 with an fp32
        tensor — left fp32 so the kernels subtract the start point in fp32 before rounding (real
        data with absolute coordinates, Training_VAE.py:345-348)."""
        x = torch.as_tensor(x)
        want = torch.float32 if (keep_f32 and x.dtype in (torch.float32, torch.float64)) else self.tdtype
        if x.device != self.device or x.dtype != want or not x.is_contiguous():
            x = x.to(device=self.device, dtype=want).contiguous()
        return x

    def _xflags(self, x):
        if x.dtype == self.tdtype:
            return CVAE_X_OPERAND
        if x.dtype == torch.float32:
            return CVAE_X_F32
        raise ValueError(f"trajectories must be {self.tdtype} or float32, got {x.dtype}")

    def _check_rows(self, x, idx, batch):
        S, D = self.shape[0], self.shape[1]
        if x.dim() != 3 or x.shape[1] != S or x.shape[2] != D:
            raise ValueError(f"expected (N,{S},{D}) trajectories, got {tuple(x.shape)}")
        if idx is None and batch > x.shape[0]:
            raise ValueError("batch larger than the trajectory tensor")
        if idx is not None and idx.numel() < batch:
            raise ValueError(f"idx holds {idx.numel()} rows, the batch needs {batch}")
        if batch > self.max_batch:
            raise ValueError(f"batch {batch} > max_batch {self.max_batch}")

    def _dev(self, t, dtype):
        """``t`` on the device, contiguous, as ``dtype``.  A host tensor goes through pinned memory
        with a non-blocking copy: the upload then queues on the stream behind the kernels already
        there instead of waiting for them, so the host can prepare its next call meanwhile (the
        pinned staging block stays allocated until the copy has run: torch's host allocator)."""
        t = torch.as_tensor(t)
        if t.device.type == "cpu":
            return t.to(dtype).contiguous().pin_memory().to(self.device, non_blocking=True)
        return t.to(device=self.device, dtype=dtype).contiguous()

    def _idx(self, idx, n_rows):
        """int64 row indices on the device.  A host index tensor is range-checked before the upload
        (the kernels gather x[idx[b]] without bounds checks); a device one is trusted."""
        if idx is None:
            return None
        idx = torch.as_tensor(idx)
        if idx.device.type == "cpu" and idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= n_rows):
            raise IndexError(f"row index out of range [0, {n_rows})")
        if idx.device != self.device or idx.dtype != torch.int64:
            idx = self._dev(idx, torch.int64)
        return idx.contiguous()

    def _eps(self, eps, batch):
        if eps is None:
            return None
        eps = self._dev(eps, torch.float32)
        if eps.shape != (batch, self.shape[2]):
            raise ValueError(f"eps must be ({batch},{self.shape[2]})")
        return eps

    def _classes(self, classes, n_rows):
        """int32 class ids per row of x on the device (cfg4); None for the reference model."""
        if not self.n_classes:
            if classes is not None:
                raise ValueError("this model has no class embedding (n_classes=0)")
            return None
        if classes is None:
            raise ValueError(f"a class-embedding model (n_classes={self.n_classes}) needs class ids per row")
        c = torch.as_tensor(classes)
        if c.device.type == "cpu" and c.numel() and (int(c.min()) < 0 or int(c.max()) >= self.n_classes):
            raise IndexError(f"class id out of range [0, {self.n_classes})")
        if c.numel() < n_rows:
            raise ValueError(f"{c.numel()} class ids for {n_rows} rows")
        return c.to(device=self.device, dtype=torch.int32).contiguous()

    def _weights(self, weights):
        w = self.weights if weights is None else weights
        return CvaeLossWeights(*[float(v) for v in w])

    def _prep(self, x, idx, batch):
        x = self.as_input(x, keep_f32=self.keep_f32)
        idx = self._idx(idx, x.shape[0])
        B = int(batch if batch is not None else (idx.numel() if idx is not None else x.shape[0]))
        self._check_rows(x, idx, B)
        return x, idx, B

    # ------------------------------------------------------------------ training
    def train_step(self, x, idx=None, eps=None, batch=None, weights=None, accumulate=True, row0=0, classes=None):
        """Fused step (fwd + loss + bwd + Adam) — Training_VAE.py:345-370 for one batch.

        ``x``: (B,S,D) absolute trajectories, or the whole dataset with ``idx`` the rows.
        ``row0``: global row of this batch's first row (Philox eps keying under data parallelism).
        Returns the device loss tensor (total, recon, kld, start, time); no host sync.
        """
        x, idx, B = self._prep(x, idx, batch)
        e = self._eps(eps, B)
        cl = self._classes(classes, x.shape[0])
        self.ensure_packed()
        w = self._weights(weights)
        a = self._adam()
        check(lib().cvae_train_step(
            self._h, ptr(x), ptr(idx), ptr(cl), B, self._xflags(x), ptr(e), self.seed, 0, int(row0), C.byref(w),
            ptr(self.params), ptr(self.m), ptr(self.v), 0, C.byref(a), ptr(self.loss),
            ptr(self.loss_accum) if accumulate else None, ptr(self.counters), self._stream()), "cvae_train_step")
        self._ctr[0] += 1
        self._ctr[1] += 1
        return self.loss

    def train_steps(self, x, n_steps, idx=None, eps=None, batch=None, weights=None, accumulate=True, row0=0,
                    classes=None):
        """``n_steps`` fused steps in one C call (cvae_train_steps): the loop body of
        Training_VAE.py:340-370 over a run of equal-size batches, with no host work per step.

        ``idx``: (n_steps·batch) rows of ``x`` (step i takes idx[i·batch:(i+1)·batch]); without it
        every step uses rows 0..batch-1.  ``eps``: (n_steps·batch, Z) or None (Philox).
        Returns the device loss tensor of the last step; no host sync.
        """
        x = self.as_input(x, keep_f32=self.keep_f32)
        idx = self._idx(idx, x.shape[0])
        n_steps = int(n_steps)
        if batch is None:
            batch = idx.numel() // max(n_steps, 1) if idx is not None else x.shape[0]
        B = int(batch)
        self._check_rows(x, None if idx is None else idx[:B], B)
        if idx is not None and idx.numel() < n_steps * B:
            raise ValueError(f"idx holds {idx.numel()} rows, {n_steps} steps of {B} need {n_steps * B}")
        e = None
        if eps is not None:
            e = self._dev(eps, torch.float32)
            if e.shape != (n_steps * B, self.shape[2]):
                raise ValueError(f"eps must be ({n_steps * B},{self.shape[2]})")
        cl = self._classes(classes, x.shape[0])
        self.ensure_packed()
        w = self._weights(weights)
        a = self._adam()
        check(lib().cvae_train_steps(
            self._h, ptr(x), ptr(idx), ptr(cl), B, n_steps, self._xflags(x), ptr(e), self.seed, 0, int(row0), C.byref(w),
            ptr(self.params), ptr(self.m), ptr(self.v), 0, C.byref(a), ptr(self.loss),
            ptr(self.loss_accum) if accumulate else None, ptr(self.counters), self._stream()), "cvae_train_steps")
        self._ctr[0] += n_steps
        self._ctr[1] += n_steps
        return self.loss

    def train_epochs(self, x, idx, batch, n_steps=None, eps=None, loss_accum=None, weights=None, row0=0):
        """Shuffled epochs of the reference loop (Training_VAE.py:338-370) in ONE C call
        (cvae_train_epochs): ``idx`` holds E epochs' permutations of the ``n_rows`` rows of ``x``
        ((E, n_rows) or flat, device or host int64); epoch e runs the DataLoader's batches of
        ``batch`` rows over its permutation (the last one ragged), ``n_steps`` steps in all (default
        every step of the E epochs; step s is batch s % spe of epoch s // spe).  ``eps``: one row per
        visited row ((E·n_rows, Z)) or None (Philox).  ``loss_accum``: a device fp64 (E, 5) tensor
        that receives each epoch's Σ loss·batch (zeroed here; default a fresh one).  Returns it; no
        host sync.  Only the last epoch may be cut short by ``n_steps``."""
        x = self.as_input(x, keep_f32=self.keep_f32)
        idx = torch.as_tensor(idx)
        E = idx.shape[0] if idx.dim() == 2 else 1
        n_rows = idx.shape[1] if idx.dim() == 2 else idx.numel()
        idx = self._idx(idx.reshape(-1), x.shape[0])
        B = int(batch)
        spe = (n_rows + B - 1) // B
        n_steps = E * spe if n_steps is None else int(n_steps)
        if n_steps > E * spe:
            raise ValueError(f"{n_steps} steps > the {E * spe} steps of {E} epochs")
        self._check_rows(x, idx[:min(B, n_rows)], min(B, n_rows))
        e = None
        if eps is not None:
            e = self._dev(eps, torch.float32)
            if e.shape != (E * n_rows, self.shape[2]):
                raise ValueError(f"eps must be ({E * n_rows},{self.shape[2]})")
        if loss_accum is None:
            loss_accum = torch.zeros(E, 5, device=self.device, dtype=torch.float64)
        elif loss_accum.shape != (E, 5) or loss_accum.dtype != torch.float64 or loss_accum.device != self.device:
            raise ValueError(f"loss_accum must be a ({E}, 5) float64 tensor on {self.device}")
        else:
            loss_accum.zero_()
        self.ensure_packed()
        w = self._weights(weights)
        a = self._adam()
        check(lib().cvae_train_epochs(
            self._h, ptr(x), ptr(idx), None, n_rows, B, n_steps, self._xflags(x), ptr(e), self.seed, 0, int(row0),
            C.byref(w), ptr(self.params), ptr(self.m), ptr(self.v), 0, C.byref(a), ptr(self.loss), ptr(loss_accum),
            ptr(self.counters), self._stream()), "cvae_train_epochs")
        self._ctr[0] += n_steps
        self._ctr[1] += n_steps
        return loss_accum

    def prepare_steps(self, x, batch=None, weights=None, accumulate=True, row0=0, classes=None):
        """A callable ``run(n)`` that enqueues ``n`` fused steps on rows 0..batch-1 of the resident
        ``x`` with Philox eps (cvae_train_steps) — what ``train_steps(x, n, batch=batch)`` does,
        with every argument converted once here instead of per call.

        train_steps spends ~40 µs of Python (input checks, the parameter-version scan of
        ensure_packed, ctypes conversion of 21 arguments, the current-stream lookup) before its
        first launch; a timed run of a few steps pays that once (short runs).  The
        prepared call is bound to this stream, x, batch and these optimizer/loss settings; the
        parameters must not be written from outside the engine between calls (call
        ``ensure_packed`` / prepare again after ``load_state_dict`` or an external optimizer)."""
        x = self.as_input(x, keep_f32=self.keep_f32)
        B = int(batch if batch is not None else x.shape[0])
        self._check_rows(x, None, B)
        cl = self._classes(classes, x.shape[0])  # cfg4: class ids per row of x (None for the reference model)
        self.ensure_packed()
        f = lib().cvae_train_steps
        w = self._weights(weights)
        a = self._adam()
        keep = (x, w, a, cl)  # referenced by the closure: the pointers stay valid
        pre = (self._h, C.c_void_p(x.data_ptr()), None, ptr(cl), C.c_int(B))
        post = (C.c_int(self._xflags(x)), None, C.c_uint64(self.seed), C.c_uint64(0), C.c_int64(int(row0)),
                C.byref(w), ptr(self.params), ptr(self.m), ptr(self.v), C.c_int64(0), C.byref(a), ptr(self.loss),
                ptr(self.loss_accum) if accumulate else None, ptr(self.counters), self._stream())
        ctr = self._ctr

        def run(n, _f=f, _pre=pre, _post=post, _keep=keep, _ctr=ctr, _i=C.c_int):
            rc = _f(*_pre, _i(n), *_post)
            if rc < 0:
                check(rc, "cvae_train_steps")
            _ctr[0] += n
            _ctr[1] += n
        return run

    def forward_backward(self, x, idx=None, eps=None, batch=None, weights=None, accumulate=True, row0=0,
                         parts=CVAE_PART_ALL, classes=None):
        """fwd + loss + bwd into ``self.grads`` (means over this batch) — the DP half-step.

        ``parts``: CVAE_PART_ALL, or CHAIN|DW_DEC then (separately) ``wgrad_rest()`` — the two-bucket
        split that lets the decoder bucket's all-reduce run beside the rest of the dW GEMMs."""
        x, idx, B = self._prep(x, idx, batch)
        e = self._eps(eps, B)
        cl = self._classes(classes, x.shape[0])
        self.ensure_packed()
        w = self._weights(weights)
        a = self._adam()
        check(lib().cvae_train_fwd_bwd(
            self._h, ptr(x), ptr(idx), ptr(cl), B, self._xflags(x), ptr(e), self.seed, 0, int(row0), C.byref(w),
            ptr(self.grads), ptr(self.loss), ptr(self.loss_accum) if accumulate else None, ptr(self.counters),
            C.byref(a), int(parts), self._stream()), "cvae_train_fwd_bwd")
        self._ctr[0] += 1
        self._ctr[1] += 1
        self._last_batch = B
        return self.loss

    def forward_backward_outputs(self, x, idx=None, eps=None, batch=None, weights=None, row0=0):
        """``forward_backward`` whose row chain also returns what its epilogues computed — recon
        (B,S,D), mu and logvar (B,Z), fp32 — at the training step's own rounding points
        (cvae_tap_outputs; the ring chain only).  Parity checks of the bf16 headline path."""
        S, D, Z = self.shape[:3]
        B = int(batch if batch is not None else (len(idx) if idx is not None else x.shape[0]))
        kw = dict(device=self.device, dtype=torch.float32)
        recon, mu, lv = torch.empty(B, S, D, **kw), torch.empty(B, Z, **kw), torch.empty(B, Z, **kw)
        check(lib().cvae_tap_outputs(self._h, ptr(recon), ptr(mu), ptr(lv)), "cvae_tap_outputs")
        try:
            self.forward_backward(x, idx=idx, eps=eps, batch=B, weights=weights, row0=row0)
        finally:
            lib().cvae_tap_outputs(self._h, None, None, None)  # one-shot even if the call failed early
        return recon, mu, lv

    def activation(self, layer, which="x", rows=None):
        """The arena matrix the last training row chain wrote for ``layer`` (state_dict layer order:
        C0, C1, E0.., fc, D0..): ``which="x"`` its input, ``"g"`` the gradient of its pre-activation —
        as a (rows, features) fp32 tensor (cvae_read_activation; parity tests)."""
        w = 0 if which == "x" else 1
        rows = int(self.max_batch if rows is None else rows)
        f = C.c_int()
        check(lib().cvae_read_activation(self._h, int(layer), w, rows, None, C.byref(f), None), "cvae_read_activation")
        r16 = (rows + 15) // 16 * 16
        buf = torch.empty(r16 * f.value, device=self.device, dtype=self.tdtype)
        check(lib().cvae_read_activation(self._h, int(layer), w, rows, ptr(buf), C.byref(f), self._stream()),
              "cvae_read_activation")
        # tile-major [rows/16][features][16] → (rows, features)
        return buf.view(r16 // 16, f.value, 16).permute(0, 2, 1).reshape(r16, f.value)[:rows].float()

    def operand_checksum(self):
        """cvae_operand_checksum of the device operand copies (W, Wᵀ, biases) as a Python int
        (synchronises): equal on every rank of the peer exchange, and to its value after a repack."""
        out = torch.zeros(1, device=self.device, dtype=torch.int64)
        check(lib().cvae_operand_checksum(self._h, ptr(out), self._stream()), "cvae_operand_checksum")
        return int(out.item()) & (2 ** 64 - 1)

    def wgrad_rest(self, batch=None):
        """The second dW bucket (condition encoder, encoder, fc) of the batch the last
        ``forward_backward(parts=CHAIN|DW_DEC)`` ran."""
        B = int(batch if batch is not None else self._last_batch)
        check(lib().cvae_train_fwd_bwd(
            self._h, None, None, None, B, 0, None, 0, 0, 0, None, ptr(self.grads), None, None, None, None,
            CVAE_PART_DW_REST, self._stream()), "cvae_train_fwd_bwd(rest)")

    def adam_step(self, grad_scale=1.0):
        """optimizer.step() on the flat buffers with g = grads * grad_scale (Training_VAE.py:363);
        the step number is the device counter the preceding forward_backward advanced."""
        a = self._adam()
        check(lib().cvae_adam(self._h, ptr(self.params), ptr(self.grads), ptr(self.m), ptr(self.v), 0,
                              C.byref(a), float(grad_scale), ptr(self.counters), self._stream()), "cvae_adam")

    def adam_flat(self, grads, lo, grad_scale=1.0):
        """Adam on params/m/v[lo, lo + len(grads)) from the summed gradient shard ``grads``
        (cvae_adam_flat: the sharded optimizer of the RCCL data-parallel step); the step number is
        the device counter.  The operand copies are left stale: ``pack()`` after the all-gather."""
        a = self._adam()
        check(lib().cvae_adam_flat(self._h, ptr(self.params), ptr(grads), ptr(self.m), ptr(self.v), int(lo),
                                   int(grads.numel()), 0, C.byref(a), float(grad_scale), ptr(self.counters),
                                   self._stream()), "cvae_adam_flat")

    def skip_step(self):
        """A data-parallel step with no rows on this rank (cvae_step_skip): the device counters
        advance as a forward_backward would (step begun + its Adam scalars, Philox offset), so the
        following adam_step matches every other rank's."""
        check(lib().cvae_step_skip(self._h, ptr(self.counters), C.byref(self._adam()), self._stream()),
              "cvae_step_skip")
        self._ctr[0] += 1
        self._ctr[1] += 1

    def fault(self):
        """The handle's sticky fault word (cvae_fault): non-zero after a launch gave up a bounded wait."""
        w = C.c_uint()
        check(lib().cvae_fault(self._h, C.byref(w)), "cvae_fault")
        return w.value

    def clear_fault(self):
        check(lib().cvae_clear_fault(self._h), "cvae_clear_fault")

    def adam_host_step(self, step, grad_scale=1.0, grads=None):
        """Adam with a host step number (no device counters): grads default ``self.grads``."""
        a = self._adam()
        g = self.grads if grads is None else grads
        check(lib().cvae_adam(self._h, ptr(self.params), ptr(g), ptr(self.m), ptr(self.v), int(step),
                              C.byref(a), float(grad_scale), None, self._stream()), "cvae_adam")

    # ------------------------------------------------------------------ inference / autograd
    def forward(self, x, start=None, idx=None, eps=None, batch=None, outputs=("recon", "mu", "logvar", "hc"),
                row0=0, offset=None, classes=None):
        """Training_VAE.py:217-226.  start=None: x absolute (transform in-kernel); else x relative.
        eps None: in-kernel Philox at ``offset`` (default: the next host offset, then advanced)."""
        S, D, Z, H = self.shape[:4]
        x, idx, B = self._prep(x, idx, batch)
        e = self._eps(eps, B)
        cl = self._classes(classes, x.shape[0])
        self.ensure_packed()
        st = None
        if start is not None:
            st = torch.as_tensor(start).to(device=self.device, dtype=torch.float32).contiguous()
        if offset is None:
            offset = self.rng_offset
            self.rng_offset = offset + 1
        kw = dict(device=self.device, dtype=torch.float32)
        out = {"recon": torch.empty(B, S, D, **kw) if "recon" in outputs else None,
               "mu": torch.empty(B, Z, **kw) if "mu" in outputs else None,
               "logvar": torch.empty(B, Z, **kw) if "logvar" in outputs else None,
               "hc": torch.empty(B, H, **kw) if "hc" in outputs else None,
               "eps": torch.empty(B, Z, **kw) if "eps" in outputs else None}
        check(lib().cvae_forward(self._h, ptr(x), ptr(idx), ptr(cl), B, self._xflags(x), ptr(st), ptr(e), self.seed,
                                 int(offset), int(row0), ptr(out["recon"]), ptr(out["mu"]), ptr(out["logvar"]),
                                 ptr(out["hc"]), ptr(out["eps"]), self._stream()), "cvae_forward")
        if "eps" in outputs:
            return out["recon"], out["mu"], out["logvar"], out["hc"], out["eps"]
        return out["recon"], out["mu"], out["logvar"], out["hc"]

    def backward(self, x, start, eps, offset, d_recon, d_mu=None, d_logvar=None, d_hc=None, row0=0, grads=None,
                 classes=None):
        """Gradient of the forward (x relative, start, eps / Philox offset) w.r.t. every parameter from
        the output gradients (cvae_backward: recompute + backward).  Writes ``grads`` (default a
        fresh flat buffer) and returns it."""
        x, _, B = self._prep(x, None, None)
        st = None if start is None else torch.as_tensor(start).to(device=self.device,
                                                                    dtype=torch.float32).contiguous()
        e = self._eps(eps, B)
        cl = self._classes(classes, B)
        f = lambda t: None if t is None else t.to(device=self.device, dtype=torch.float32).contiguous()  # noqa: E731
        out = torch.empty(self.n_params, device=self.device, dtype=torch.float32) if grads is None else grads
        self.ensure_packed()
        dr, dm, dl, dh = f(d_recon), f(d_mu), f(d_logvar), f(d_hc)
        check(lib().cvae_backward(self._h, ptr(x), None, ptr(cl), B, self._xflags(x), ptr(st), ptr(e), self.seed, int(offset),
                                  int(row0), ptr(dr), ptr(dm), ptr(dl), ptr(dh), ptr(out), self._stream()),
              "cvae_backward")
        return out

    def condition(self, start):
        """condition_encoder(start) — Training_VAE.py:132-137."""
        st = torch.as_tensor(start).to(device=self.device, dtype=torch.float32).contiguous()
        B = st.shape[0]
        hc = torch.empty(B, self.shape[3], device=self.device, dtype=torch.float32)
        self.ensure_packed()
        check(lib().cvae_condition(self._h, ptr(st), B, ptr(hc), self._stream()), "cvae_condition")
        return hc

    def decode(self, z, start=None, hc=None, classes=None):
        """decode(z, h_c) (Training_VAE.py:208-215) or decode from absolute start points."""
        S, D, Z, H = self.shape[:4]
        z = torch.as_tensor(z).to(device=self.device, dtype=torch.float32).contiguous()
        B = z.shape[0]
        st = None if start is None else torch.as_tensor(start).to(device=self.device, dtype=torch.float32).contiguous()
        h = None if hc is None else torch.as_tensor(hc).to(device=self.device, dtype=torch.float32).contiguous()
        cl = self._classes(classes, B)
        out = torch.empty(B, S, D, device=self.device, dtype=torch.float32)
        self.ensure_packed()
        check(lib().cvae_decode(self._h, ptr(z), ptr(st), ptr(h), ptr(cl), B, ptr(out), self._stream()), "cvae_decode")
        return out

    # ------------------------------------------------------------------ timing
    def set_timing(self, on=True):
        check(lib().cvae_set_timing(self._h, 1 if on else 0))

    def kernel_times(self):
        """{name: (avg_ms, count)} over all calls since set_timing(True) (stream must be synchronised)."""
        names = C.create_string_buffer(1024)
        ms = (C.c_float * 16)()
        n = check(lib().cvae_kernel_times(self._h, names, 1024, ms, 16))
        out = {}
        for i, item in enumerate(names.value.decode().split(",")[:n]):
            k, c = item.rsplit(":", 1)
            out[k] = (ms[i], int(c))
        return out

    def bench_kernels(self, x, reps, idx=None, batch=None):
        """{'rowchain', 'wgrad_adam', 'step'}: average device ms of ``reps`` back-to-back launches
        (cvae_bench_kernels; synchronises; updates params like training steps)."""
        x, idx, B = self._prep(x, idx, batch)
        if self.n_classes:
            raise ValueError("bench_kernels measures the reference model (n_classes=0)")
        ms = (C.c_float * 3)()
        check(lib().cvae_bench_kernels(self._h, ptr(x), ptr(idx), B, int(reps), ptr(self.params), ptr(self.m),
                                       ptr(self.v), self.step_count + 1, ms, self._stream()), "cvae_bench_kernels")
        self.step_count = self.step_count + 2 * int(reps)
        return {"rowchain": ms[0], "wgrad_adam": ms[1], "step": ms[2]}

    @property
    def train_kernel(self):
        """'generic', 'fast' / 'ring' (reference architecture, bf16; 'ring' = the single weight-stream
        chain, S=100 D=6), 'wide' (BASELINE cfg5 shape, bf16) or 'f32' (the reference's own
        configuration in fp32: S=10 D=3, the fp32-MFMA ring chain):
        the training row chain this engine runs (cvae_train_kernel)."""
        k = C.c_int()
        check(lib().cvae_train_kernel(self._h, C.byref(k)))
        return ("generic", "fast", "wide", "ring", "f32")[k.value]

    @property
    def dw_kernel(self):
        """'generic' (tile list from memory) or the compile-time tile decode the dW ⊕ Adam launch
        uses: 'fast', 'wide', 'f32' or 'cls' (cvae_dw_kernel)."""
        k = C.c_int()
        check(lib().cvae_dw_kernel(self._h, C.byref(k)))
        return ("generic", "fast", "wide", "f32", "cls")[k.value]

    def chain_rows(self, batch):
        """Rows per workgroup of the training row chain a call of ``batch`` rows launches
        (cvae_chain_rows: 4 or 16 for the fp32 chain, 16 for the bf16 ones)."""
        r = C.c_int()
        check(lib().cvae_chain_rows(self._h, int(batch), C.byref(r)), "cvae_chain_rows")
        return r.value

    def workspace_bytes(self):
        b = C.c_int64()
        check(lib().cvae_workspace_bytes(self._h, C.byref(b)))
        return b.value


def optimizer_state_dict(eng):
    """torch.optim.Adam.state_dict() of the engine's flat m / v (works for any engine with
    tensors/m/v/step_count/lr/betas/eps: the CPU oracle stand-in too)."""
    steps = float(eng.step_count)
    state = {}
    for i, (o, n, shape) in enumerate(eng.tensors):
        state[i] = {"step": torch.tensor(steps),
                    "exp_avg": eng.m[o:o + n].detach().view(shape).cpu().clone(),
                    "exp_avg_sq": eng.v[o:o + n].detach().view(shape).cpu().clone()}
    group = {"lr": eng.lr, "betas": tuple(eng.betas), "eps": eng.eps, "weight_decay": 0, "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
             "decoupled_weight_decay": False, "params": list(range(len(eng.tensors)))}
    return {"state": state, "param_groups": [group]}


def load_optimizer_state_dict(eng, sd):
    """Inverse of optimizer_state_dict (also accepts torch Adam's own state_dict of the same
    parameter order); sets m, v, the step count and the hyper-parameters."""
    g = sd["param_groups"][0]
    eng.set_optimizer(lr=g["lr"], betas=g["betas"], eps=g["eps"])
    steps = set()
    with torch.no_grad():
        for i, (o, n, shape) in enumerate(eng.tensors):
            st = sd["state"].get(i) or sd["state"].get(str(i))
            if st is None:  # a parameter torch never stepped
                eng.m[o:o + n].zero_()
                eng.v[o:o + n].zero_()
                continue
            eng.m[o:o + n].copy_(st["exp_avg"].reshape(-1).to(eng.m.device, torch.float32))
            eng.v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1).to(eng.v.device, torch.float32))
            steps.add(int(float(st["step"])))
    if len(steps) > 1:
        raise ValueError(f"parameters carry different Adam step counts {sorted(steps)}")
    eng.step_count = steps.pop() if steps else 0


def adam_scalars(n, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, device="cuda"):
    """The device's (−lr/(1−β1^t), sqrt(1−β2^t)) for t = 1..n (cvae_adam_scalars), as an (n, 2)
    fp32 tensor — the check of the device-counter Adam path against torch's Python doubles."""
    out = torch.empty(n, 2, device=device, dtype=torch.float32)
    a = CvaeAdamConfig(float(lr), float(betas[0]), float(betas[1]), float(eps))
    check(lib().cvae_adam_scalars(C.byref(a), int(n), ptr(out),
                                  C.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)), "cvae_adam_scalars")
    return out


__all__ = ["CVAEEngine", "config_info", "adam_scalars", "optimizer_state_dict", "load_optimizer_state_dict", "DTYPES", "DEFAULT_WEIGHTS", "CVAE_PART_ALL",
           "CVAE_PART_CHAIN", "CVAE_PART_DW_DEC", "CVAE_PART_DW_REST"]
