"""CPU stand-in for ``CVAEEngine`` built on the oracle — TEST INFRASTRUCTURE ONLY.

It exposes the engine surface ``cvae_amd.train`` and ``cvae_amd.dist`` drive (flat fp32
params/grads/m/v, device-style loss accumulators, train_step / forward_backward / adam_step),
so the host logic (loader RNG, DP sharding, gradient weighting, epoch bookkeeping) can be
tested on the CPU under gloo.  The arithmetic is the oracle's torch-CPU restatement of
Training_VAE.py (oracle/cvae_oracle.py); Adam follows torch ``_single_tensor_adam`` op order
on the flat buffer, which is elementwise-identical to the per-tensor optimizer.
"""
import torch

from oracle.cvae_oracle import DEFAULT_WEIGHTS, OracleCVAE, oracle_loss, relative


class OracleEngine:
    def __init__(self, model, max_batch=1 << 30):
        self.model = model
        self.max_batch = max_batch
        self.plist = list(model.parameters())
        self.params = torch.cat([p.detach().reshape(-1) for p in self.plist]).clone()
        n = self.params.numel()
        self.grads = torch.zeros(n)
        self.m = torch.zeros(n)
        self.v = torch.zeros(n)
        self.loss = torch.zeros(5)
        self.loss_accum = torch.zeros(5, dtype=torch.float64)
        self.bucket_split = sum(p.numel() for p in self.plist[:-2 * 4])  # decoder.* = the last 8 tensors
        self.step_count = 0
        self.lr, self.betas, self.eps = 1e-3, (0.9, 0.999), 1e-8
        self.weights = DEFAULT_WEIGHTS
        self.calls = []
        self.rng_offset = 0
        o, self.tensors = 0, []
        for p in self.plist:
            self.tensors.append((o, p.numel(), tuple(p.shape)))
            o += p.numel()

    # --- engine surface
    def set_optimizer(self, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.betas, self.eps = lr, betas, eps

    keep_f32 = True

    def as_input(self, x, keep_f32=False):
        return torch.as_tensor(x, dtype=torch.float32).contiguous()

    def pack(self):
        o = 0
        with torch.no_grad():
            for p in self.plist:
                p.copy_(self.params[o:o + p.numel()].view_as(p))
                o += p.numel()

    def forward_backward(self, x, idx=None, eps=None, batch=None, weights=None, accumulate=True, row0=0, parts=7,
                         classes=None):
        # the device-counter path: the launch that begins a step advances steps-begun and the offset;
        # adam_step then takes its step number from that counter (CVAEEngine / include/cvae.h)
        self.step_count += 1
        self.rng_offset += 1
        self.calls.append(("fb", None if idx is None else idx.clone(), batch, row0, parts))
        rows = x[idx] if idx is not None else x[:batch]
        cls = None if classes is None else (classes[idx] if idx is not None else classes[:batch]).long()
        rel, start = relative(rows)
        for p in self.plist:
            p.grad = None
        mu, lv, hc = self.model.encode(rel, start, cls)
        recon = self.model.decode(self.model.reparameterize(mu, lv, eps), hc, cls)
        w = dict(zip(("recon_weight", "kld_weight", "start_weight", "time_weight"), weights or self.weights))
        ls = oracle_loss(recon, rel, mu, lv, hc, **w)
        ls[0].backward()
        self.grads.copy_(torch.cat([p.grad.reshape(-1) for p in self.plist]))
        self.loss.copy_(torch.stack([v.detach() for v in ls]))
        if accumulate:  # the reference's loss.item() * B in Python doubles
            self.loss_accum += self.loss.double() * float(rows.shape[0])
        return self.loss

    def wgrad_rest(self, batch=None):
        self.calls.append(("rest", None, batch, None, 4))

    def skip_step(self):
        """cvae_step_skip: an empty share advances the counters as a forward_backward would."""
        self.calls.append(("skip", None, 0, None, 0))
        self.step_count += 1
        self.rng_offset += 1

    def adam_step(self, grad_scale=1.0):
        b1, b2 = self.betas
        g = self.grads * grad_scale if grad_scale != 1.0 else self.grads
        self.m.lerp_(g, 1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        denom = (self.v.sqrt() / (bc2 ** 0.5)).add_(self.eps)
        self.params.addcdiv_(self.m, denom, value=-(self.lr / bc1))
        self.pack()

    @property
    def n_params(self):
        return self.params.numel()

    def adam_flat(self, grads, lo, grad_scale=1.0):
        """cvae_adam_flat: adam_step's arithmetic on params/m/v[lo, lo + len(grads)) only."""
        b1, b2 = self.betas
        hi = lo + grads.numel()
        g = grads * grad_scale if grad_scale != 1.0 else grads
        m, v, p = self.m[lo:hi], self.v[lo:hi], self.params[lo:hi]
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        denom = (v.sqrt() / (bc2 ** 0.5)).add_(self.eps)
        p.addcdiv_(m, denom, value=-(self.lr / bc1))

    def train_step(self, x, idx=None, eps=None, batch=None, weights=None, accumulate=True, row0=0, classes=None):
        self.forward_backward(x, idx=idx, eps=eps, batch=batch, weights=weights, accumulate=accumulate,
                              classes=classes)
        self.adam_step()
        return self.loss

    def train_epochs(self, x, idx, batch, n_steps=None, eps=None, loss_accum=None, weights=None, row0=0):
        """cvae_train_epochs' schedule: epoch e's permutation idx[e], DataLoader batches of ``batch``
        rows (the last ragged), eps rows in visiting order, epoch e's Σ loss·batch in row e."""
        idx = torch.as_tensor(idx)
        idx = idx.view(1, -1) if idx.dim() == 1 else idx
        E, n = idx.shape
        spe = (n + batch - 1) // batch
        n_steps = E * spe if n_steps is None else int(n_steps)
        acc = torch.zeros(E, 5, dtype=torch.float64)
        saved = self.loss_accum
        for s in range(n_steps):
            e, k = divmod(s, spe)
            lo, b = k * batch, min(batch, n - k * batch)
            self.loss_accum = acc[e]
            self.train_step(x, idx=idx[e, lo:lo + b], eps=None if eps is None else eps[e * n + lo:e * n + lo + b],
                            batch=b, weights=weights)
        self.loss_accum = saved
        if loss_accum is not None:
            loss_accum.copy_(acc)
            return loss_accum
        return acc


class OracleModel(OracleCVAE):
    """An OracleCVAE already 'attached' to an OracleEngine (what cvae_amd.train expects)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.__dict__["_engine"] = OracleEngine(self)

    def load_state_dict(self, sd, strict=True, assign=False):
        res = super().load_state_dict(sd, strict=strict, assign=assign)
        eng = self.__dict__["_engine"]
        eng.params.copy_(torch.cat([p.detach().reshape(-1) for p in eng.plist]))
        return res
