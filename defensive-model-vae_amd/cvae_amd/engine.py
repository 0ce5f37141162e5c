"""Device engine: one C-ABI handle + the flat fp32 parameter / Adam / gradient buffers.

The engine owns what the reference spreads over ``ConditionalTrajectoryVAE``
parameters, ``torch.optim.Adam`` state and autograd (Training_VAE.py:331-363):

* ``params``  flat fp32, state_dict order; the bound module's parameters are views
* ``m, v``    Adam moments (torch ``exp_avg``/``exp_avg_sq``), same layout
* ``grads``   flat fp32 gradient (data-parallel path); bound ``p.grad`` are views
* ``loss``    fp32[5] last step's (total, recon, kld, start, time)  — on device
* ``loss_accum`` fp32[5] running Σ loss·batch for the epoch       — on device

Every call enqueues HIP kernels on torch's current stream and returns without
synchronising.  Nothing falls back to torch compute.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import CVAE_BF16, CVAE_F32, CVAE_FP8, CvaeConfig, CvaeLossWeights, check, lib, ptr

# "fp8": bf16 activations with OCP e4m3 forward GEMM operands (BASELINE cfg5; cvae.h CVAE_FP8)
DTYPES = {"fp32": (CVAE_F32, torch.float32), "bf16": (CVAE_BF16, torch.bfloat16),
          "fp8": (CVAE_FP8, torch.bfloat16)}
DEFAULT_WEIGHTS = (0.1, 0.1, 1.0, 1.0)  # Training_VAE.py:300-306


def config_info(seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4, dtype="fp32", max_batch=1):
    """Host-only query: (n_params, n_tensors, lds_bytes) — works without a GPU."""
    cfg = CvaeConfig(seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec, DTYPES[dtype][0], max_batch)
    n = C.c_int64()
    nt = C.c_int()
    lds = C.c_int()
    check(lib().cvae_config_info(C.byref(cfg), C.byref(n), C.byref(nt), C.byref(lds)), "cvae_config_info")
    return n.value, nt.value, lds.value


class CVAEEngine:
    def __init__(self, seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4, dtype="fp32",
                 max_batch=1024, device=None, seed=0):
        if not torch.cuda.is_available():
            raise RuntimeError("CVAEEngine needs a HIP device (MI355X); there is no CPU fallback")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.dtype_name = dtype
        self.cdtype, self.tdtype = DTYPES[dtype]
        self.shape = (seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec)
        self.max_batch = max_batch
        cfg = CvaeConfig(seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec, self.cdtype, max_batch)
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
        kw = dict(device=self.device, dtype=torch.float32)
        self.params = torch.zeros(self.n_params, **kw)
        self.m = torch.zeros(self.n_params, **kw)
        self.v = torch.zeros(self.n_params, **kw)
        self.grads = torch.zeros(self.n_params, **kw)
        self.loss = torch.zeros(5, **kw)
        self.loss_accum = torch.zeros(5, **kw)
        self.step_count = 0
        self.seed = int(seed)
        self.rng_offset = 0
        self.lr, self.betas, self.eps = 1e-3, (0.9, 0.999), 1e-8
        self.weights = DEFAULT_WEIGHTS
        self._module = None

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
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

    def pack(self):
        """Refresh the device operand copies (W, Wᵀ, bias) after parameters were written."""
        check(lib().cvae_pack_weights(self._h, ptr(self.params), self._stream()), "cvae_pack_weights")

    def set_optimizer(self, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)

    def reset_optimizer(self):
        self.m.zero_()
        self.v.zero_()
        self.step_count = 0

    # ------------------------------------------------------------------ inputs
    def as_input(self, x):
        """Trajectories in the operand dtype, contiguous on the device."""
        x = torch.as_tensor(x)
        if x.device != self.device or x.dtype != self.tdtype or not x.is_contiguous():
            x = x.to(device=self.device, dtype=self.tdtype).contiguous()
        return x

    def _check_rows(self, x, idx, batch):
        S, D = self.shape[0], self.shape[1]
        if x.dim() != 3 or x.shape[1] != S or x.shape[2] != D:
            raise ValueError(f"expected (N,{S},{D}) trajectories, got {tuple(x.shape)}")
        if idx is None and batch > x.shape[0]:
            raise ValueError("batch larger than the trajectory tensor")
        if batch > self.max_batch:
            raise ValueError(f"batch {batch} > max_batch {self.max_batch}")

    def _idx(self, idx):
        if idx is None:
            return None
        idx = torch.as_tensor(idx)
        if idx.device != self.device or idx.dtype != torch.int64:
            idx = idx.to(device=self.device, dtype=torch.int64)
        return idx.contiguous()

    def _eps(self, eps, batch):
        if eps is None:
            return None
        eps = torch.as_tensor(eps).to(device=self.device, dtype=torch.float32).contiguous()
        if eps.shape != (batch, self.shape[2]):
            raise ValueError(f"eps must be ({batch},{self.shape[2]})")
        return eps

    def _weights(self, weights):
        w = self.weights if weights is None else weights
        return CvaeLossWeights(*[float(v) for v in w])

    def _next_offset(self):
        o = self.rng_offset
        self.rng_offset += 1
        return o

    # ------------------------------------------------------------------ training
    def train_step(self, x, idx=None, eps=None, batch=None, weights=None, accumulate=True):
        """Fused step (fwd + loss + bwd + Adam) — Training_VAE.py:345-370 for one batch.

        ``x``: (B,S,D) absolute trajectories, or the whole dataset with ``idx`` the rows.
        Returns the device loss tensor (total, recon, kld, start, time); no host sync.
        """
        x = self.as_input(x)
        idx = self._idx(idx)
        B = int(batch if batch is not None else (idx.numel() if idx is not None else x.shape[0]))
        self._check_rows(x, idx, B)
        e = self._eps(eps, B)
        self.step_count += 1
        w = self._weights(weights)
        check(lib().cvae_train_step(
            self._h, ptr(x), ptr(idx), B, ptr(e), C.c_uint64(self.seed), C.c_uint64(self._next_offset()),
            C.byref(w), ptr(self.params), ptr(self.m), ptr(self.v), self.step_count, self.lr, self.betas[0],
            self.betas[1], self.eps, ptr(self.loss), ptr(self.loss_accum) if accumulate else None,
            self._stream()), "cvae_train_step")
        return self.loss

    def train_steps(self, x, n_steps, idx=None, eps=None, batch=None, weights=None, accumulate=True):
        """``n_steps`` fused steps in one C call (cvae_train_steps): the loop body of
        Training_VAE.py:340-370 over a run of equal-size batches, with no host work per step.

        ``idx``: (n_steps·batch) rows of ``x`` (step i takes idx[i·batch:(i+1)·batch]); without it
        every step uses rows 0..batch-1.  ``eps``: (n_steps·batch, Z) or None (Philox).
        Returns the device loss tensor of the last step; no host sync.
        """
        x = self.as_input(x)
        idx = self._idx(idx)
        n_steps = int(n_steps)
        if batch is None:
            batch = idx.numel() // max(n_steps, 1) if idx is not None else x.shape[0]
        B = int(batch)
        self._check_rows(x, idx, B)
        if idx is not None and idx.numel() < n_steps * B:
            raise ValueError(f"idx holds {idx.numel()} rows, {n_steps} steps of {B} need {n_steps * B}")
        e = None
        if eps is not None:
            e = torch.as_tensor(eps).to(device=self.device, dtype=torch.float32).contiguous()
            if e.shape != (n_steps * B, self.shape[2]):
                raise ValueError(f"eps must be ({n_steps * B},{self.shape[2]})")
        w = self._weights(weights)
        step0 = self.step_count + 1
        offset = self.rng_offset
        check(lib().cvae_train_steps(
            self._h, ptr(x), ptr(idx), B, n_steps, ptr(e), C.c_uint64(self.seed), C.c_uint64(offset), C.byref(w),
            ptr(self.params), ptr(self.m), ptr(self.v), step0, self.lr, self.betas[0], self.betas[1], self.eps,
            ptr(self.loss), ptr(self.loss_accum) if accumulate else None, self._stream()), "cvae_train_steps")
        self.step_count += n_steps
        self.rng_offset += n_steps
        return self.loss

    def forward_backward(self, x, idx=None, eps=None, batch=None, weights=None, accumulate=True):
        """fwd + loss + bwd into ``self.grads`` (means over this batch) — the DP half-step."""
        x = self.as_input(x)
        idx = self._idx(idx)
        B = int(batch if batch is not None else (idx.numel() if idx is not None else x.shape[0]))
        self._check_rows(x, idx, B)
        e = self._eps(eps, B)
        w = self._weights(weights)
        check(lib().cvae_train_fwd_bwd(
            self._h, ptr(x), ptr(idx), B, ptr(e), C.c_uint64(self.seed), C.c_uint64(self._next_offset()),
            C.byref(w), ptr(self.grads), ptr(self.loss), ptr(self.loss_accum) if accumulate else None,
            self._stream()), "cvae_train_fwd_bwd")
        return self.loss

    def adam_step(self, grad_scale=1.0):
        """optimizer.step() on the flat buffers with g = grads * grad_scale (Training_VAE.py:363)."""
        self.step_count += 1
        check(lib().cvae_adam(self._h, ptr(self.params), ptr(self.grads), ptr(self.m), ptr(self.v),
                              self.step_count, self.lr, self.betas[0], self.betas[1], self.eps,
                              float(grad_scale), self._stream()), "cvae_adam")

    # ------------------------------------------------------------------ inference
    def forward(self, x, start=None, idx=None, eps=None, batch=None, outputs=("recon", "mu", "logvar", "hc")):
        """Training_VAE.py:217-226.  start=None: x absolute (transform in-kernel); else x relative."""
        S, D, Z, H = self.shape[:4]
        x = self.as_input(x)
        idx = self._idx(idx)
        B = int(batch if batch is not None else (idx.numel() if idx is not None else x.shape[0]))
        self._check_rows(x, idx, B)
        e = self._eps(eps, B)
        st = None
        if start is not None:
            st = torch.as_tensor(start).to(device=self.device, dtype=torch.float32).contiguous()
        kw = dict(device=self.device, dtype=torch.float32)
        out = {"recon": torch.empty(B, S, D, **kw) if "recon" in outputs else None,
               "mu": torch.empty(B, Z, **kw) if "mu" in outputs else None,
               "logvar": torch.empty(B, Z, **kw) if "logvar" in outputs else None,
               "hc": torch.empty(B, H, **kw) if "hc" in outputs else None}
        check(lib().cvae_forward(self._h, ptr(x), ptr(idx), B, ptr(st), ptr(e), C.c_uint64(self.seed),
                                 C.c_uint64(self._next_offset()), ptr(out["recon"]), ptr(out["mu"]),
                                 ptr(out["logvar"]), ptr(out["hc"]), self._stream()), "cvae_forward")
        return out["recon"], out["mu"], out["logvar"], out["hc"]

    def condition(self, start):
        """condition_encoder(start) — Training_VAE.py:132-137."""
        st = torch.as_tensor(start).to(device=self.device, dtype=torch.float32).contiguous()
        B = st.shape[0]
        hc = torch.empty(B, self.shape[3], device=self.device, dtype=torch.float32)
        check(lib().cvae_condition(self._h, ptr(st), B, ptr(hc), self._stream()), "cvae_condition")
        return hc

    def decode(self, z, start=None, hc=None):
        """decode(z, h_c) (Training_VAE.py:208-215) or decode from absolute start points."""
        S, D, Z, H = self.shape[:4]
        z = torch.as_tensor(z).to(device=self.device, dtype=torch.float32).contiguous()
        B = z.shape[0]
        st = None if start is None else torch.as_tensor(start).to(device=self.device, dtype=torch.float32).contiguous()
        h = None if hc is None else torch.as_tensor(hc).to(device=self.device, dtype=torch.float32).contiguous()
        out = torch.empty(B, S, D, device=self.device, dtype=torch.float32)
        check(lib().cvae_decode(self._h, ptr(z), ptr(st), ptr(h), B, ptr(out), self._stream()), "cvae_decode")
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
        x = self.as_input(x)
        idx = self._idx(idx)
        B = int(batch if batch is not None else (idx.numel() if idx is not None else x.shape[0]))
        self._check_rows(x, idx, B)
        ms = (C.c_float * 3)()
        check(lib().cvae_bench_kernels(self._h, ptr(x), ptr(idx), B, int(reps), ptr(self.params), ptr(self.m),
                                       ptr(self.v), self.step_count + 1, ms, self._stream()), "cvae_bench_kernels")
        self.step_count += 2 * int(reps)
        return {"rowchain": ms[0], "wgrad_adam": ms[1], "step": ms[2]}

    def sync_words(self):
        """The fused launch's hand-off words (cvae_sync_words): [group0, group1, group2, finished
        tiles, time-out flag], all 0 between launches."""
        out = (C.c_uint * 5)()
        check(lib().cvae_sync_words(self._h, out), "cvae_sync_words")
        return list(out)

    def workspace_bytes(self):
        b = C.c_int64()
        check(lib().cvae_workspace_bytes(self._h, C.byref(b)))
        return b.value
