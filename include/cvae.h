/*
 * cvae.h — C-ABI of the MI355X-native conditional trajectory VAE training path.
 *
 * This is the drop-in boundary for the reference's hot path
 * (yslf2035/Defensive-Model-VAE, Training_VAE.py).  The reference has no FFI of
 * its own (it is torch-CPU Python); each entry point below names the reference
 * code it replaces.  Plain pointers and sizes only — no torch types: every
 * device pointer is a HIP device allocation owned by the CALLER (torch tensors
 * pass data_ptr()), every `stream` is a hipStream_t (torch's current stream).
 * The library owns only its workspace (padded weight copies + activation
 * arena), allocated in cvae_create and sized by cfg->max_batch.
 *
 * Errors: every function returns 0 on success or a negative CVAE_E* code; it
 * never aborts.  cvae_last_error() returns a thread-local message.
 * Threading: one handle per device per process; a handle is not thread-safe.
 * No call synchronises the device: all work is queued on `stream`, so every
 * call is capturable into a hipGraph.  With device step counters (below) a
 * captured training step can be REPLAYED: nothing in it is a host value that
 * changes from step to step.
 *
 * ABI 2 (round 2): Adam hyper-parameters are doubles (torch computes its step
 * size and bias corrections in Python doubles, torch/optim/adam.py), loss
 * accumulators are fp64 (the reference sums loss.item()*B in Python doubles,
 * Training_VAE.py:366-370), eps rows are keyed by a global row offset, and the
 * training calls take optional device step counters.
 *
 * ABI 3 (rounds 5-6): the library's own RCCL communicator (cvae_rccl_*), an armed
 * tap consumed by cvae_train_fwd_bwd only, the fp32 chain's kernel id
 * (CVAE_KERNEL_F32), arena introspection (cvae_read_activation), whole shuffled
 * epochs in one call (cvae_train_epochs) and Adam over a flat range
 * (cvae_adam_flat, the sharded-Adam data-parallel step), which dW kernel and how
 * many rows per row-chain workgroup a handle runs (cvae_dw_kernel, cvae_chain_rows).
 */
#ifndef CVAE_H
#define CVAE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CVAE_ABI_VERSION 3

enum cvae_dtype {
  CVAE_F32 = 0,
  CVAE_BF16 = 1,
  CVAE_FP8 = 2  /* bf16 activations + OCP e4m3 forward GEMM operands with per-layer scales (BASELINE cfg5) */
};

enum cvae_status {
  CVAE_OK = 0,
  CVAE_E_INVALID = -1,   /* bad argument / unsupported configuration        */
  CVAE_E_HIP = -2,       /* a HIP runtime call failed (message has details) */
  CVAE_E_CAPACITY = -3,  /* batch larger than cfg.max_batch                  */
  CVAE_E_NOMEM = -4,
  CVAE_E_TIMEOUT = -5    /* an earlier launch gave up a bounded wait and skipped work (fault word) */
};

/* Input flags (the `xflags` argument of the calls that read trajectories). */
enum cvae_xflags {
  CVAE_X_OPERAND = 0,  /* x is in the operand dtype (fp32 / bf16)                                   */
  CVAE_X_F32 = 1       /* x is fp32 whatever the operand dtype: the relative transform
                          (Training_VAE.py:345-348) runs in fp32 and rounds once — real data with
                          absolute coordinates of ~200 m stays exact in the relative frame       */
};

/* fwd/bwd parts (cvae_train_fwd_bwd `parts`): a data-parallel caller can split the weight-gradient
 * launch in two buckets and all-reduce the decoder bucket while the rest is computed. */
enum cvae_parts {
  CVAE_PART_CHAIN = 1,    /* forward + loss + every dX (the row chain)                         */
  CVAE_PART_DW_DEC = 2,   /* dW/db of the decoder layers (a contiguous tail of the flat buffer)  */
  CVAE_PART_DW_REST = 4,  /* dW/db of condition encoder, encoder, fc_mu, fc_logvar               */
  CVAE_PART_ALL = 7
};

/* Model shape.  Training_VAE.py:124 ConditionalTrajectoryVAE(seq_len, dim,
 * latent_dim, hidden_dim=128); n_enc/n_dec are 4/4 in the reference
 * (:141-167) and may be raised for the wide config. */
typedef struct cvae_config {
  int seq_len;     /* S */
  int dim;         /* D (channel 0 = time, 1:3 = x,y; Training_VAE.py:250-262) */
  int latent_dim;  /* Z */
  int hidden_dim;  /* H */
  int n_enc;       /* Linear layers in `encoder`  (reference: 4) */
  int n_dec;       /* Linear layers in `decoder`  (reference: 4) */
  int dtype;       /* cvae_dtype: GEMM operand / activation type; master weights, Adam and loss are fp32 */
  int max_batch;   /* rows per call the workspace is sized for */
  int n_classes;   /* BASELINE cfg4: scenario classes of the class embedding (0 = the reference model) */
  int class_dim;   /* width of the class embedding (a multiple of 4), concatenated beside h_c in the fc
                      input [h_traj ‖ h_c ‖ e] and the decoder input [z ‖ h_c ‖ e] (Training_VAE.py:193, :214);
                      its table is the LAST parameter tensor, nn.Embedding layout (n_classes, class_dim) */
} cvae_config;

typedef struct cvae_handle cvae_handle;

/* Loss weights in the reference's order (Training_VAE.py:229, call site :356-359). */
typedef struct cvae_loss_weights {
  float recon, kld, start, time;
} cvae_loss_weights;

/* torch.optim.Adam(lr, betas=(beta1, beta2), eps) hyper-parameters, as the Python doubles torch
 * computes with (amsgrad=False, weight_decay=0). */
typedef struct cvae_adam_config {
  double lr, beta1, beta2, eps;
} cvae_adam_config;

/* Device step counters (caller-owned device memory, 4 x uint64, zero-initialised by the caller or
 * set to a resume point):
 *   counters[0] = Philox offset of the next training step's eps draw,
 *   counters[1] = optimizer steps begun,
 *   counters[2] = the Adam scalars of step counters[1] (two fp32: -lr/(1-beta1^t), sqrt(1-beta2^t),
 *                 written by the library), counters[3] reserved.
 * A training call given counters reads them ON THE DEVICE and advances them: the row chain that
 * begins a step adds 1 to counters[1] and (given the Adam config) stores that step's scalars, the
 * Adam update uses t = counters[1] and those scalars, and the dW launch adds 1 to counters[0].  The
 * `offset` / `step` arguments are then ignored.  With counters == NULL the host values are used. */

/* Create/destroy.  Replaces ConditionalTrajectoryVAE.__init__ (Training_VAE.py:124-167)
 * for the device side; parameters themselves live in the caller's flat fp32 buffer. */
int cvae_create(const cvae_config* cfg, int device, cvae_handle** out);
int cvae_destroy(cvae_handle* h);

/* Flat fp32 parameter layout = the reference's state_dict order and shapes
 * (Training_VAE.py:132-167; 24 tensors at 4+4 layers).  Tensor i occupies
 * [offset, offset+numel) of the flat buffer, row-major nn.Linear (out,in). */
int cvae_num_params(const cvae_handle* h, int64_t* total, int* n_tensors);
int cvae_param_info(const cvae_handle* h, int i, int64_t* offset, int64_t* numel, int* rows, int* cols);

/* Host-only query (no device needed): parameter count / tensor count of the
 * flat layout, and the LDS bytes one row-chain workgroup needs (0 < lds <=
 * 163840 when the configuration is supported). */
int cvae_config_info(const cvae_config* cfg, int64_t* total_params, int* n_tensors, int* lds_bytes);

/* Workspace bytes the handle allocated (informational). */
int cvae_workspace_bytes(const cvae_handle* h, int64_t* bytes);

/* First flat index of the decoder's parameters (decoder.0.weight): the CVAE_PART_DW_DEC bucket is
 * [split, total), CVAE_PART_DW_REST is [0, split). */
int cvae_bucket_split(const cvae_handle* h, int64_t* split);

/* Which training row chain this handle runs for the usual call (16-B aligned operand-dtype x, no
 * external gradients): CVAE_KERNEL_GENERIC (the step interpreter, any shape), CVAE_KERNEL_FAST
 * (bf16, the reference architecture: hidden 128, latent 8, 4+4 layers, seq_len*dim 600) or
 * CVAE_KERNEL_WIDE (bf16, BASELINE cfg5's shape: seq_len 200, dim 6, latent 512, 8+8 layers) or
 * CVAE_KERNEL_RING (the fast configuration at seq_len 100, dim 6 on the single-ring weight-stream
 * chain: the default at that shape; CVAE_RING=0 at creation keeps CVAE_KERNEL_FAST) or
 * CVAE_KERNEL_F32 (fp32, the reference's own configuration Training_VAE.py:274-282: seq_len 10, dim 3,
 * latent 8, hidden 128, 4+4 layers, on the fp32-MFMA ring chain).
 * Introspection only (no reference counterpart); CVAE_GENERIC=1 at creation forces the generic. */
enum cvae_train_kernel_kind {
  CVAE_KERNEL_GENERIC = 0, CVAE_KERNEL_FAST = 1, CVAE_KERNEL_WIDE = 2, CVAE_KERNEL_RING = 3, CVAE_KERNEL_F32 = 4
};
int cvae_train_kernel(const cvae_handle* h, int* kind);

/* Which dW ⊕ Adam kernel the handle's training step launches (after the row chain,
 * Training_VAE.py:362-363): CVAE_DW_GENERIC (tile descriptors and layer records read from memory),
 * or a compile-time tile decode — CVAE_DW_FAST (the reference architecture, bf16, S*D = 600),
 * CVAE_DW_WIDE (BASELINE cfg5's shape), CVAE_DW_F32 (the reference's own configuration in fp32),
 * CVAE_DW_CLS (BASELINE cfg4's class embedding at S=100, D=6).  Introspection only;
 * CVAE_F32_DW=generic / CVAE_CLS_DW=generic at creation keep the generic kernel for A/B. */
enum cvae_dw_kernel_kind {
  CVAE_DW_GENERIC = 0, CVAE_DW_FAST = 1, CVAE_DW_WIDE = 2, CVAE_DW_F32 = 3, CVAE_DW_CLS = 4
};
int cvae_dw_kernel(const cvae_handle* h, int* kind);

/* Rows per workgroup of the training row chain a call of `batch` rows (1 <= batch <= max_batch, 16-B
 * aligned inputs) launches: 16 for the bf16 chains and the generic fp32 one (or what fits its LDS);
 * the fp32 chain of the reference's configuration runs 4-row workgroups up to
 * CVAE_F32_R4_MAX_BATCH rows (default 1024) and 16-row ones above (CVAE_F32_ROWS=4 / 16 at creation:
 * one tiling at every batch).  Introspection only. */
int cvae_chain_rows(const cvae_handle* h, int batch, int* rows);

/* Rebuild the device copies of the weights (padded operand-dtype W and Wᵀ,
 * padded fp32 biases) from the flat fp32 master `params`.  Call after the
 * caller writes parameters (init, load_state_dict, an optimizer outside this
 * library).  cvae_adam/cvae_train_step keep the copies current themselves. */
int cvae_pack_weights(cvae_handle* h, const float* params, void* stream);

/* Inference: encode → reparameterise → decode.  Replaces
 * ConditionalTrajectoryVAE.forward (Training_VAE.py:217-226).
 *   x      (N_total,S,D) trajectories, operand dtype (or fp32 with CVAE_X_F32), row-major.
 *          With start == NULL x holds ABSOLUTE coordinates and the relative
 *          transform of :345-348 is applied in-kernel (condition = x[:,0,1:3]);
 *          with start != NULL x is used as given (already relative, as
 *          model(batch_rel, start_points) at :352) and start fp32 (batch,2) is
 *          the condition.
 *   idx    optional int64[batch] row gather into x (NULL = rows 0..batch-1)
 *   classes cfg4 only: int32 class id per row of x (gathered by idx like x; NULL = class 0)
 *   eps    optional fp32 (batch,Z); NULL = in-kernel Philox(seed, offset) keyed by the global
 *          row eps_row0 + b (a data-parallel rank passes its first global row, so the ranks of
 *          a global batch draw what one process with that batch draws)
 *   recon  fp32 (batch,S,D) relative trajectories; mu, logvar fp32 (batch,Z);
 *   hc     fp32 (batch,H) condition features; eps_out fp32 (batch,Z) the eps each row used
 *          (any output may be NULL).                                                           */
int cvae_forward(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                 const float* start, const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0,
                 float* recon, float* mu, float* logvar, float* hc, float* eps_out, void* stream);

/* Condition encoder only: h_c = condition_encoder(start)
 * (Training_VAE.py:132-137, called at :190 and Tools.py:55).
 *   start fp32 (batch,2) absolute start points → hc fp32 (batch,H). */
int cvae_condition(cvae_handle* h, const float* start, int batch, float* hc, void* stream);

/* Decode (generation).  Replaces ConditionalTrajectoryVAE.decode
 * (Training_VAE.py:208-215) and the sampling of Tools.py:46-63.
 *   z fp32 (batch,Z); exactly the condition given:
 *     hc    fp32 (batch,H) condition features (decode(z, h_c) semantics), or
 *     start fp32 (batch,2) absolute start points (condition encoder fused in);
 *   classes (cfg4) int32 (batch) class ids;
 *   out fp32 (batch,S,D) relative trajectories (caller adds start for global). */
int cvae_decode(cvae_handle* h, const float* z, const float* start, const float* hc, const int32_t* classes,
                int batch, float* out, void* stream);

/* Forward + conditional_vae_loss + full backward for one batch, gradients into
 * the flat fp32 `grads` (overwritten, same layout as params).  Replaces
 * Training_VAE.py:351-362 (zero_grad, model(), conditional_vae_loss(),
 * loss.backward()).  `loss_out` fp32[5] = (total, recon, kld, start, time) as
 * returned by conditional_vae_loss (:268); `loss_accum` (nullable) fp64[5]
 * += (double)loss * batch (the per-epoch accumulators of :366-370, kept on device).
 * Means are over this call's batch, so a data-parallel caller all-reduces
 * `grads` and passes grad_scale = 1/world to cvae_adam.
 * parts: CVAE_PART_ALL, or CVAE_PART_CHAIN|CVAE_PART_DW_DEC followed by a CVAE_PART_DW_REST call
 * on the same batch (the two-bucket overlap; loss and counters advance in the first call).
 * counters + adam (nullable): the step this call begins, with its Adam scalars precomputed for the
 * cvae_adam(counters) that completes it — a data-parallel step is capturable as one graph. */
int cvae_train_fwd_bwd(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch,
                       int xflags,
                       const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0,
                       const cvae_loss_weights* w, float* grads, float* loss_out, double* loss_accum,
                       uint64_t* counters, const cvae_adam_config* adam, int parts, void* stream);

/* Backward of model.forward from caller-supplied output gradients (the autograd path: the
 * reference loop's loss.backward(), Training_VAE.py:362, when conditional_vae_loss and the
 * model are separate autograd nodes).  Recomputes the forward of (x relative, start, eps or
 * Philox(seed, offset, eps_row0)) — bit-identical to the cvae_forward that produced the
 * outputs — and back-propagates d_recon fp32 (batch,S,D), d_mu / d_logvar fp32 (batch,Z) and
 * d_hc fp32 (batch,H) (any may be NULL = zero) into the flat fp32 `grads` (overwritten). */
int cvae_backward(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                  const float* start, const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0,
                  const float* d_recon, const float* d_mu, const float* d_logvar, const float* d_hc,
                  float* grads, void* stream);

/* torch.optim.Adam step (amsgrad=False, weight_decay=0) over the flat buffers
 * — replaces optimizer.step() (Training_VAE.py:363; torch/optim/adam.py
 * _single_tensor_adam).  step is the 1-based step count after increment; with counters, t and its
 * scalars come from the cvae_train_fwd_bwd(counters, adam) that began the step.
 * g_eff = grads * grad_scale.  Also refreshes the device weight copies. */
int cvae_adam(cvae_handle* h, float* params, const float* grads, float* m, float* v, int64_t step,
              const cvae_adam_config* adam, float grad_scale, const uint64_t* counters, void* stream);

/* Adam on one contiguous range of the flat fp32 state — the sharded optimizer of the RCCL data-
 * parallel step (cvae_amd.dist, shard_adam): after a reduce-scatter of the flat gradient each rank
 * updates params/m/v[lo, lo + count) from `grads` (its summed shard, count floats, times
 * grad_scale), torch's op order (as cvae_adam); the step's scalars from `counters` (or `step`).  The
 * operand copies are NOT rewritten: the caller all-gathers the parameters and calls
 * cvae_pack_weights.  Replaces optimizer.step() (Training_VAE.py:363) for one shard. */
int cvae_adam_flat(cvae_handle* h, float* params, const float* grads, float* m, float* v, int64_t lo, int64_t count,
                   int64_t step, const cvae_adam_config* adam, float grad_scale, const uint64_t* counters,
                   void* stream);

/* Fused single-device step: cvae_train_fwd_bwd + cvae_adam with the weight
 * gradient GEMMs and Adam in one kernel (the gradient never round-trips HBM).
 * Replaces the whole body of Training_VAE.py:345-370 for one batch. */
int cvae_train_step(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                    const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0,
                    const cvae_loss_weights* w, float* params, float* m, float* v, int64_t step,
                    const cvae_adam_config* adam, float* loss_out, double* loss_accum,
                    uint64_t* counters, void* stream);

/* n_steps consecutive fused steps (cvae_train_step) enqueued by one call: step i uses the rows
 * idx[i*batch .. (i+1)*batch) of x (idx == NULL: rows 0..batch-1 every step), eps rows
 * eps[i*batch ..] (NULL: Philox(seed, offset + i)) and Adam step step0 + i (with counters: the
 * device counters, advanced per step).  Replaces the inner `for batch in dataloader` loop of
 * Training_VAE.py:340-370 for a run of equal-size batches (an epoch's permutation uploaded
 * once); loss_out = the last step's losses, loss_accum += every step's loss * batch.  No host
 * work per step beyond the two kernel launches. */
int cvae_train_steps(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch,
                     int n_steps, int xflags,
                     const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0,
                     const cvae_loss_weights* w, float* params, float* m, float* v, int64_t step0,
                     const cvae_adam_config* adam, float* loss_out, double* loss_accum,
                     uint64_t* counters, void* stream);

/* The reference's shuffled epochs (Training_VAE.py:340-370 under `for epoch in range(epochs)`),
 * n_steps fused steps enqueued by one call: epoch e visits the n_rows rows idx[e*n_rows ..
 * (e+1)*n_rows) of x (that epoch's permutation, uploaded once) in DataLoader order — batches of
 * `batch` rows, the last one ragged (drop_last=False) — and step s is batch s % spe of epoch s / spe
 * (spe = ceil(n_rows / batch) steps per epoch), so an epoch may be split across calls.  eps: one
 * row per visited row in the same order (NULL: Philox(seed, offset + s)).  loss_accum (NULL, or
 * fp64[5 * epochs]) receives epoch e's Σ loss * batch at 5 * e; loss_out = the last step's losses.
 * The host draws the permutations and eps with the reference's RNG order (cvae_amd.train): the
 * host does no work per step. */
int cvae_train_epochs(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int n_rows,
                      int batch, int n_steps, int xflags, const float* eps, uint64_t seed, uint64_t offset,
                      int64_t eps_row0, const cvae_loss_weights* w, float* params, float* m, float* v, int64_t step0,
                      const cvae_adam_config* adam, float* loss_out, double* loss_accum, uint64_t* counters,
                      void* stream);

/* Standalone conditional_vae_loss (Training_VAE.py:229-268), forward only, for
 * callers holding (recon, x, mu, logvar) fp32 device tensors; x is the RELATIVE
 * batch as at the reference call site (:356-359).  loss_out fp32[5] =
 * (total, recon, kld, start, time); workspace: >= 8*ceil(batch/32) fp32 on device.
 * Handle-free.  The training entry points fuse the loss and do not need this. */
int cvae_loss(const float* recon, const float* x, const float* mu, const float* logvar,
              int batch, int seq_len, int dim, int latent_dim, const cvae_loss_weights* w,
              float* loss_out, float* workspace, void* stream);

/* Backward of cvae_loss (autograd of Training_VAE.py:240-267): given the upstream
 * gradients g_out fp32[5] of (total, recon, kld, start, time) on the device, writes
 * d_recon fp32 (batch,S,D), d_mu and d_logvar fp32 (batch,Z) (overwritten).  Handle-free. */
int cvae_loss_backward(const float* recon, const float* x, const float* mu, const float* logvar,
                       int batch, int seq_len, int dim, int latent_dim, const cvae_loss_weights* w,
                       const float* g_out, float* d_recon, float* d_mu, float* d_logvar, void* stream);

/* Per-kernel device time, measured with HIP events recorded on `stream`
 * around every kernel of every call made while timing is enabled (no
 * synchronisation is added; read after the stream is synchronised).
 * cvae_set_timing(h, 1) enables and resets the record.  cvae_kernel_times
 * writes, per kernel name ("rowchain", "wgrad", "wgrad_adam", "adam"), the
 * AVERAGE duration in ms to ms[i] and "name:count" comma-separated to names;
 * returns the number of kernel names. */
int cvae_set_timing(cvae_handle* h, int enabled);
int cvae_kernel_times(cvae_handle* h, char* names, int names_len, float* ms, int max_n);

/* Measurement: average device time (ms) of `reps` back-to-back launches of each kernel of the
 * fused training step on the batch (x, idx, batch): ms[0] = the row chain (forward + loss + every
 * dX), ms[1] = the dW + Adam kernel, ms[2] = the whole step.  Two HIP events per measurement on
 * `stream`; SYNCHRONISES the stream (measurement only).  The row-chain and step runs update
 * params/m/v like training steps (step numbers step0..). */
int cvae_bench_kernels(cvae_handle* h, const void* x, const int64_t* idx, int batch, int reps,
                       float* params, float* m, float* v, int64_t step0, float* ms, void* stream);

/* The handle's sticky fault word.  A kernel that waits on a hand-off (the peer exchange) waits a
 * bounded time; on a time-out it skips its update and sets this word in pinned host memory.  Every later training call (cvae_train_step[s], cvae_train_fwd_bwd, cvae_adam)
 * then returns CVAE_E_TIMEOUT without launching; the check reads host memory and does not
 * synchronise, so it sees a time-out once the faulting launch has run.  cvae_fault reads the word,
 * cvae_clear_fault resets it (after the caller restored consistent parameters). */
int cvae_fault(const cvae_handle* h, unsigned* word);
int cvae_clear_fault(cvae_handle* h);

/* Checksum of the handle's device operand copies (every layer's padded W and Wᵀ in the operand
 * dtype and the padded fp32 biases — what the row chain multiplies by): Σ over their 8-B words w_i
 * of splitmix64(w_i ^ i·0x9E3779B97F4A7C15) mod 2^64, written to the DEVICE word `out`.  Under the
 * peer exchange every rank's copies are written by the tiles' owners: equal checksums on every
 * rank, and equal to the checksum after a repack from the gathered master state, show the
 * broadcast delivered every byte.  Queued on `stream`. */
int cvae_operand_checksum(cvae_handle* h, uint64_t* out, void* stream);

/* Parity introspection (tests): copy the arena matrix of layer `layer` (state_dict layer order: C0, C1,
 * E0.., fc, D0..) that the last training row chain wrote — which = 0: its input xT, 1: the gradient of
 * its pre-activation gT — for the first roundup(rows, 16) batch rows, in the arena's own layout
 * (tile-major [rows/16][features][16 rows], the operand dtype: fp32, or bf16 for CVAE_BF16/CVAE_FP8),
 * to the device buffer `dst` (NULL: only report).  *features = the matrix's padded feature count. */
int cvae_read_activation(cvae_handle* h, int layer, int which, int rows, void* dst, int* features, void* stream);

/* Parity taps (tests): the NEXT training call's row chain also writes what its epilogues computed
 * at the training step's own rounding points — recon fp32 (batch,S,D) (the last decoder layer's
 * output, Training_VAE.py:215, before the loss), mu and logvar fp32 (batch,Z) (:195-196); any may be
 * NULL.  One-shot, and consumed by cvae_train_fwd_bwd only: while a tap is armed every other
 * training call (cvae_train_step(s), the peer step, cvae_bench_kernels) fails with CVAE_E_INVALID
 * and launches nothing; disarm it by passing NULLs.  Served by the ring chain (CVAE_KERNEL_RING)
 * only: on another handle this call fails (CVAE_E_INVALID) unless every pointer is NULL. */
int cvae_tap_outputs(cvae_handle* h, float* recon, float* mu, float* logvar);

/* ---- Data parallelism over xGMI without a collective library (Training_VAE.py:362-363
 * across ranks): the "peer exchange".  One process per GPU; every rank's workspace and a mailbox
 * are mapped into every other rank through HIP IPC, and the weight-gradient launch of each step
 * does dW ⊕ reduce-scatter ⊕ Adam ⊕ all-gather itself: tile t of the padded weights is owned by
 * rank t mod world, the other ranks push their fp32 partial of t into the owner's mailbox, the
 * owner sums the world partials in rank order, applies Adam to its fp32 master state and writes
 * the new operand copies into every rank's workspace.  Serves the reference architecture at
 * seq_len 100, dim 6, bf16 (cvae_train_kernel == CVAE_KERNEL_RING).
 *   cvae_px_blob_bytes: size of one rank's exchange descriptor (handle-free).
 *   cvae_px_export: allocate this rank's mailbox (zeroed) and write its descriptor to `blob`.
 *   cvae_px_import: `blobs` = the world descriptors in rank order (all-gathered by the caller, who
 *     must also barrier after every rank's import and before any rank's first step); `base` =
 *     counters[1] at this point, the same on every rank.
 *   cvae_px_train_step: one training step of this rank's rows (batch may be 0: an empty share of
 *     a ragged global batch), the exchange included; rank_scales = host float[world] of
 *     B_r / B_global for a ragged batch, NULL for equal shares (gradient = sum / world).  Every
 *     rank must call it for every step.  Master parameters and moments are current on the OWNER
 *     of each element only (cvae_px_owned: host uint8[n_params] mask of this rank's elements);
 *     the caller gathers them (e.g. masked sum across ranks) before reading them.
 *   cvae_px_close: unmap the peers and free the mailbox (after a barrier). */
int cvae_px_blob_bytes(int64_t* bytes);
int cvae_px_export(cvae_handle* h, int world, int rank, void* blob);
int cvae_px_import(cvae_handle* h, const void* blobs, uint64_t base);
int cvae_px_owned(const cvae_handle* h, uint8_t* mask);
int cvae_px_train_step(cvae_handle* h, const void* x, const int64_t* idx, int batch, int xflags, const float* eps,
                       uint64_t seed, int64_t eps_row0, const cvae_loss_weights* w, float* params, float* m, float* v,
                       const cvae_adam_config* adam, const float* rank_scales, float* loss_out, double* loss_accum,
                       uint64_t* counters, void* stream);
int cvae_px_close(cvae_handle* h);
/* The residency precondition (csrc/cvae_peer.h): a waiting owner block holds a workgroup slot, so
 * the blocks of every rank on one GPU must fit that GPU's slots together.  cvae_px_import counts
 * the ranks on this rank's GPU (PCI address in the blobs) and sizes the exchange launch: one rank
 * per GPU runs one block per tile; k sharing ranks run 2·CUs/k − 1 tile blocks each (a block
 * pushes all its tiles before it waits on any it owns), and import fails when the row chain alone
 * needs more than 2·CUs/k blocks.  *ranks_on_gpu = k, *tile_blocks = the launch's tile blocks. */
int cvae_px_layout(const cvae_handle* h, int* ranks_on_gpu, int* tile_blocks);
/* Re-arm the exchange after every rank synchronised and met a barrier (collective by contract):
 * zero this rank's arrival flags and done counter, count the step epoch from `base` (= counters[1]
 * now, the same on every rank: after a resume or a restore) and clear the fault word.  A timed-out
 * step leaves the flag epochs short; restore consistent state (gather it), then call this on every
 * rank before the next step.  Synchronises the device. */
int cvae_px_reset(cvae_handle* h, uint64_t base);
/* Set-up check after cvae_px_import (every rank calls it once, concurrently): each rank stores a
 * tagged word into every peer's mailbox and waits (bounded, ~1 s) for theirs; *ok = 1 when every
 * peer's tag arrived intact.  Synchronises the device. */
int cvae_px_probe(cvae_handle* h, int* ok);
/* This rank's exchange wait statistics since set-up or the last reset, in 10-ns ticks: out[0] the
 * longest owner-tile wait for the other ranks' partials, out[1] the longest end-of-launch wait for
 * the other owners' operand copies, out[2] the sum and out[3] the number of owner-tile waits.
 * Every wait is bounded by CVAE_PX_TIMEOUT_MS (default 10000); a time-out sets the fault word to 2
 * (owner tile) or 3 (end of launch).  Synchronises the device. */
int cvae_px_stats(cvae_handle* h, uint64_t* out, int reset);

/* ---- The gradient all-reduce over RCCL on the caller's stream (Training_VAE.py:362-363
 * across ranks; BASELINE configs[2] "RCCL grad all-reduce over xGMI"): the data-parallel split
 * step's collective, issued by this library on the stream its kernels run on, so a captured step
 * graph holds the RCCL kernels between the dW and Adam launches with no stream of a framework in
 * between (cvae_amd.dist.DataParallelStep, exchange "rccl").  One communicator per handle.
 *   cvae_rccl_id_bytes: size of the unique id (handle-free);
 *   cvae_rccl_unique_id: a new id (rank 0; the caller broadcasts it to the other ranks);
 *   cvae_rccl_init: join the world-rank communicator of that id on the handle's device (collective);
 *   cvae_rccl_allreduce: in-place float32 sum over the ranks of `count` elements of `buf` (device);
 *   cvae_rccl_close: destroy the communicator (also done by cvae_destroy). */
int cvae_rccl_id_bytes(int64_t* bytes);
int cvae_rccl_unique_id(void* id);
int cvae_rccl_init(cvae_handle* h, const void* id, int world, int rank);
int cvae_rccl_allreduce(cvae_handle* h, float* buf, int64_t count, void* stream);
int cvae_rccl_close(cvae_handle* h);

/* A data-parallel step in which this rank has no rows (a ragged last global batch shorter than the
 * world): advances the device counters exactly as a training step's launches would — counters[1]
 * += 1 with that step's Adam scalars, counters[0] += 1 — so the rank's following cvae_adam uses the
 * same step number and scalars as every other rank, and its later eps draws stay in step
 * (Training_VAE.py:363, the step every rank takes). */
int cvae_step_skip(cvae_handle* h, uint64_t* counters, const cvae_adam_config* adam, void* stream);

/* Adam's per-step scalars as the device computes them from a step counter (t = 1..n): writes
 * out[2*(t-1)] = -lr/(1-beta1^t) and out[2*(t-1)+1] = sqrt(1-beta2^t), both rounded to fp32 —
 * the values torch's CPU Adam forms in Python doubles.  Check/diagnostic entry point for the
 * device-counter path (the host path computes them on the host). */
int cvae_adam_scalars(const cvae_adam_config* adam, int64_t n, float* out, void* stream);

/* Trajectory extraction (Traj_Data_Process.process_csv :72-122) for n_files parsed
 * CSV logs at once, handle-free.  cols: float64 [9][n_rows] on the device, the columns
 * (ego_x, ego_y, sv1_x, sv1_y, sv1_vx, sv1_vy, sv1_yaw, sv2_vx, sv2_vy) of all files stacked,
 * file f owning rows [file_offsets[f], file_offsets[f+1]) (int64 [n_files+1], device).
 * scene: CVAE_SCENE_* (SCENE_CONFIG :8-25); point_mode 0 = 'normal', 1 = 'extend_mid'.
 * Writes out float64 [n_files][target_points][3] (time, ego_x, ego_y) and valid int32 [n_files]
 * (0 where process_csv returns None: no start row, or fewer than target_points rows). */
enum cvae_scene { CVAE_SCENE_STATIC = 0, CVAE_SCENE_DYNAMIC = 1, CVAE_SCENE_PREDICTABLE = 2,
                  CVAE_SCENE_UNPREDICTABLE = 3 };
int cvae_extract_trajectories(const double* cols, int64_t n_rows, const int64_t* file_offsets, int n_files,
                              int scene, int target_points, int point_mode, double time_interval,
                              double* out, int32_t* valid, void* stream);

/* Batched MPC path tracking (MPC/MPC_Tracking.py), handle-free, float64 throughout.
 * The configuration mirrors PathTracker / MPCController / VehicleModel's parameters
 * (MPC_Tracking.py:26, :283-306, :421-423); cvae_mpc_default_config fills the reference's values
 * (wheelbase 2.8, max_steer 0.5, max_accel 7, dt 0.01, N 10, control horizon 5,
 * Q = Qf = diag(20, 5), R = diag(1, 50)).  Limits: 1 <= control_horizon <= min(N, 32), N <= 63,
 * 2..64 waypoints per path with strictly increasing times. */
typedef struct cvae_mpc_config {
  double wheelbase, max_steer, max_accel, dt;
  double q_theta, q_v, qf_theta, qf_v, r_accel, r_steer;
  double tol;            /* projected-gradient stationarity of the sub-problem solve */
  int prediction_horizon, control_horizon, max_iter, reserved;
} cvae_mpc_config;
int cvae_mpc_default_config(cvae_mpc_config* cfg);

/* PathTracker(waypoints, initial_state).run_simulation for n_paths paths at once (MPC_Tracking.py
 * :418-523).  Device arrays: waypoints float64 [sum n_wp][3] (x, y, t), wp_offsets int32 [n_paths+1],
 * initial_states float64 [n_paths][5] (x, y, theta, vx, vy; theta already wrapped as :435-436 does),
 * n_steps int32 [n_paths] (= int(total_time / dt)), step_offsets int64 [n_paths+1] (prefix sums of
 * n_steps).  Writes states float64 rows [step_offsets[p] + p .. + n_steps[p]] x 4 (x, y, theta, v;
 * row 0 = the initial state), controls float64 rows [step_offsets[p] ..) x 2 (accel, steer) and,
 * if non-null, iters int32 [sum n_steps] (Newton iterations of each sub-problem). */
int cvae_mpc_track(const cvae_mpc_config* cfg, int n_paths, const double* waypoints, const int32_t* wp_offsets,
                   const double* initial_states, const int32_t* n_steps, const int64_t* step_offsets,
                   double* states, double* controls, int32_t* iters, void* stream);

/* MPCController.solve_mpc (:311-415) for n independent sub-problems: state [n][4], ref [n][N+1][2]
 * (theta_ref, v_ref), last [n][2] (previous control, NaN = none).  Writes the control sequence
 * u [n][control_horizon][2], its cost [n] and (if non-null) iters [n]. */
int cvae_mpc_solve(const cvae_mpc_config* cfg, int n, const double* state, const double* ref, const double* last,
                   double* u, double* cost, int32_t* iters, void* stream);

/* PathInterpolator (:89-277) queries: out [n_paths][n_t][5] = get_reference(t) (x, y, vx, vy) and
 * get_reference_heading(t); scalars [n_paths][6] = start_theta, end_vx, end_vy, end_theta, end_x,
 * end_y.  Same waypoint/initial-state layout as cvae_mpc_track; t float64 [n_t]. */
int cvae_mpc_reference(int n_paths, const double* waypoints, const int32_t* wp_offsets,
                       const double* initial_states, const double* t, int n_t, double* out, double* scalars,
                       void* stream);

const char* cvae_last_error(void);
int cvae_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CVAE_H */
