// cvae_capi.hip — host side of the C-ABI (include/cvae.h): planning, workspace,
// launches.  All launches go to the caller's stream; nothing here synchronises.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <array>
#include <cstring>
#include <cstdlib>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/cvae.h"
#include "cvae_device.h"
#include "cvae_rowchain.h"
#include "cvae_wgrad.h"
#include "cvae_loss.h"
#include "cvae_fastwgrad.h"
#include "cvae_widechain.h"
#include "cvae_widewgrad.h"
#include "cvae_f32chain.h"
#include "cvae_f32wgrad.h"
#include "cvae_extract.h"
#include "cvae_mpc.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCK(call)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return fail(CVAE_E_HIP, std::string(#call) + " failed: " + hipGetErrorString(e_));      \
  } while (0)

struct ParamInfo {
  int64_t offset, numel;
  int rows, cols;
};

}  // namespace

struct cvae_handle {
  cvae_config cfg{};
  int device = 0;
  int R = 32;               // rows per row-chain workgroup
  int tsize = 2;
  NetDev net{};
  std::vector<ParamInfo> params;
  int64_t nparams = 0;
  std::vector<TileDesc> tiles;
  TileDesc* d_tiles = nullptr;
  // the two dW buckets (CVAE_PART_DW_DEC / CVAE_PART_DW_REST): tiles of the decoder layers and of the rest
  std::vector<TileDesc> tiles_part[2];
  TileDesc* d_tiles_part[2] = {nullptr, nullptr};
  // the generic dW kernel's tile list for a whole step: tiles, or (a long 16-bit list) with 32 × 64
  // tiles where a layer's K pairs up (wtiles_ni2)
  std::vector<TileDesc> wtiles;
  TileDesc* d_wtiles = nullptr;
  bool wtiles_ni2 = false;
  int64_t bucket_split = 0;   // flat index of decoder.0.weight
  // split-K of the dW launch for large batches (cvae_wgrad.h SplitK): partial workspace + tickets
  int splitk_max = 1;
  float* splitk_ws = nullptr;
  unsigned* splitk_tickets = nullptr;
  char* arena = nullptr;    // weight copies + activations
  // sticky fault word in pinned, device-mapped host memory: a kernel that gives up a bounded spin
  // sets it (system scope); the next training call reads it WITHOUT synchronising and fails
  unsigned* fault_host = nullptr;
  unsigned* fault_dev = nullptr;
  // data-parallel peer exchange (cvae_peer.h): this rank's mailbox (uncached, IPC-exported) and
  // every rank's arena / mailbox as mapped into this process
  int px_world = 0, px_rank = 0;
  char* px_mbox = nullptr;
  ncclComm_t rccl = nullptr;   // cvae_rccl_init: this rank's communicator (the gradient all-reduce)
  int rccl_world = 0, rccl_rank = 0;
  int64_t px_mbox_bytes = 0, px_done_off = 0, px_inbox_off = 0;
  char* px_arena[PX_MAX] = {};
  char* px_mb[PX_MAX] = {};
  bool px_ready = false;
  uint64_t px_base = 0;
  int px_share = 1;            // ranks of the exchange on this rank's GPU (cvae_px_import)
  int px_grid = 0;             // tile blocks of px_wgrad_kernel (the residency precondition, cvae_peer.h)
  // one-shot outputs of the next training row chain (cvae_tap_outputs): recon, mu, logvar
  float* tap[3] = {nullptr, nullptr, nullptr};
  int64_t arena_bytes = 0;
  float* d_partials = nullptr;
  int max_row_tiles = 0;
  // step tables of the row-chain interpreter, one per mode (device copies in the arena)
  enum { ST_TRAIN = 0, ST_FWD, ST_DEC, ST_DEC_HC, ST_COND, ST_N };
  StepDesc* d_steps[ST_N] = {};
  int n_steps[ST_N] = {};
  unsigned long long* d_stamps = nullptr;  // diagnostic builds only
  int lds_bytes = 0;
  int fast_nki = 0;         // > 0: bf16 training runs fchain::fastchain_kernel<fast_nki>
  int fast_lds = 0;
  bool fast_buckets = false;  // the two dW buckets run fchain::fastwgrad_bucket_kernel
  bool wide = false;        // bf16 training at BASELINE cfg5's shape runs wchain::widechain_kernel<Cfg5>
  bool wide_dw = false;     // ... and its dW ⊕ Adam runs wchain::widewgrad_kernel (compile-time tile decode)
  bool wide_mx = false;     // CVAE_FP8 at that shape: the large dX GEMMs e4m3 + MX scales (Cfg5F8), else bf16 (Cfg5F8B)
  bool wide_mxw = false;    // ... and (CVAE_FP8_DW=mx) its dW GEMMs e4m3 + MX scales along the batch
  int wide_lds = 0;
  bool ring = false;        // the fast configuration's training chain runs wchain::widechain_kernel<Cfg2>
  bool ring_cls = false;    // cfg4 (class embedding) at cfg2's shape: widechain_kernel<Cfg4>, generic dW
  int ring_lds = 0;
  bool f32c = false;        // fp32 training at the reference's own shape (seq_len 10, dim 3): f32c::f32chain_kernel<Cfg1>
  int f32c_lds = 0;
  bool cls_dw = false;       // BASELINE cfg4's dW ⊕ Adam with the compile-time decode (wchain::clswgrad_kernel)
  int f32c_r4_max = 0;
  int f32c_spread = 8;       // XCDs the fp32 chain's row tiles occupy (CVAE_F32_SPREAD, A/B)       // ... on 4-row workgroups up to this batch (f32c_rows), 16-row above
  bool f32c_dw = false;      // ... and its dW ⊕ Adam with the compile-time tile decode (f32c::f32wgrad_kernel)
  bool timing = false;
  // timing: per call, a chain of events on the caller's stream; segment i of a
  // call spans ev[i] → ev[i+1] and is named by the kernel launched after ev[i]
  std::vector<hipEvent_t> pool;
  int n_used = 0;
  struct Seg { int e0, e1; std::string name; };
  std::vector<Seg> segs;
  const char* pending = nullptr;  // name of the next timed launch (tmark)
};

namespace {

int rup_i(int v, int a) { return (v + a - 1) / a * a; }
// 16-bit activation/arena types: bf16, and CVAE_FP8 (bf16 activations, e4m3 forward operands)
inline bool is16(const cvae_handle* h) { return h->cfg.dtype != CVAE_F32; }

// The wide chain's e4m3 dX GEMMs (wchain::Cfg5F8): CVAE_FP8 at exactly BASELINE cfg5's shape, the
// specialised kernels allowed, and not CVAE_FP8_DX=bf16 (the bf16-dX fallback, wchain::Cfg5F8B).
// Only such a handle reserves and writes the e4m3 Wᵀ copies (LayerDev::f8b) — ADVICE r04.
bool wide_fp8_mx(const cvae_config& c) {
  using A = wchain::Cfg5F8;
  const char* gen = std::getenv("CVAE_GENERIC");
  const char* dx = std::getenv("CVAE_FP8_DX");
  return c.dtype == CVAE_FP8 && !(gen && gen[0] == '1') && !(dx && std::strcmp(dx, "bf16") == 0) &&
         c.n_classes == 0 && c.hidden_dim == wchain::H && c.seq_len == A::S && c.dim == A::D &&
         c.latent_dim == A::Z && c.n_enc == A::NE && c.n_dec == A::ND;
}

int build_plan(cvae_handle* h) {
  const cvae_config& c = h->cfg;
  NetDev& n = h->net;
  n.S = c.seq_len; n.D = c.dim; n.Z = c.latent_dim; n.H = c.hidden_dim;
  n.I = c.seq_len * c.dim;
  n.n_enc = c.n_enc; n.n_dec = c.n_dec;
  n.n_layers = 2 + c.n_enc + 1 + c.n_dec + (c.n_classes > 0 ? 1 : 0);
  // cfg4 class embedding: e = table[class] (class_dim wide) joins both concatenations
  n.n_cls = c.n_classes > 0 ? c.n_classes : 0;
  n.cls_dim = n.n_cls ? c.class_dim : 0;
  n.Clsp = n.n_cls ? rup_i(n.n_cls, 32) : 0;
  const int E = n.cls_dim;
  n.Ip = rup_i(n.I, 32); n.Hp = rup_i(n.H, 32); n.Hcp = rup_i(2 * n.H + E, 32);
  n.ZHp = rup_i(n.Z + n.H + E, 32); n.Zp2 = rup_i(2 * n.Z, 32); n.Cp = 32;
  n.dtype = c.dtype;
  h->tsize = c.dtype == CVAE_F32 ? 4 : 2;  // CVAE_FP8 keeps bf16 activations (only forward W/X operands are e4m3)
  // arena rows: whole row tiles, and a multiple of the K chunk of the wgrad GEMM
  n.Bp = rup_i(c.max_batch, 32);

  // layer table (in = K, out = N) in state_dict order
  struct LD { int K, N, relu; };
  std::vector<LD> ld;
  ld.push_back({2, n.H, 1});
  ld.push_back({n.H, n.H, 1});
  for (int i = 0; i < n.n_enc; ++i) ld.push_back({i == 0 ? n.I : n.H, n.H, 1});
  ld.push_back({2 * n.H + E, 2 * n.Z, 0});                       // [h_traj ‖ h_c (‖ e)] → mu ‖ logvar
  for (int i = 0; i < n.n_dec; ++i) {
    const bool last = i == n.n_dec - 1;
    ld.push_back({i == 0 ? n.Z + n.H + E : n.H, last ? n.I : n.H, last ? 0 : 1});  // [z ‖ h_c (‖ e)] first
  }
  if (n.n_cls) ld.push_back({n.n_cls, E, 0});                    // one-hot(class) → e (the table)
  if ((int)ld.size() > CVAE_MAX_LAYERS) return fail(CVAE_E_INVALID, "too many layers");

  // flat parameter table (state_dict order; fc splits into fc_mu / fc_logvar)
  h->params.clear();
  int64_t off = 0;
  auto add = [&](int rows, int cols) {
    ParamInfo p{off, (int64_t)rows * (cols > 0 ? cols : 1), rows, cols};
    h->params.push_back(p);
    off += p.numel;
    return p.offset;
  };
  for (int l = 0; l < (int)ld.size(); ++l) {
    LayerDev& L = n.L[l];
    L.K = ld[l].K; L.N = ld[l].N; L.Kp = rup_i(L.K, 32); L.Np = rup_i(L.N, 32); L.relu = ld[l].relu;
    L.f8 = c.dtype == CVAE_FP8 && L.Kp % 64 == 0;  // fp8 forward GEMM where K pairs up (cvae_device.h)
    // e4m3 copy of Wᵀ for the wide chain's MX dX GEMMs (wchain::Arch::f8b): the backward K pairs up,
    // the layer has a dX, and it is one of the large ones
    L.f8b = wide_fp8_mx(c) && L.f8 && L.Np % 64 == 0 && l != lC0(n) && l != lE(n, 0) && (L.Np >= 512 || L.Kp >= 512)
                ? 1 : 0;
    L.has_bias = 1;
    L.wt = 0;
    if (n.n_cls && l == lCE(n)) {  // nn.Embedding(n_classes, class_dim).weight: [K][N], no bias
      L.f8 = 0;
      L.f8b = 0;
      L.wt = 1;
      L.has_bias = 0;
      L.nseg = 1; L.seg_rows0 = L.N;
      L.pw[0] = L.pw[1] = add(n.n_cls, E);
      L.pb[0] = L.pb[1] = -1;
    } else if (l == lFC(n)) {
      L.nseg = 2; L.seg_rows0 = n.Z;
      L.pw[0] = add(n.Z, L.K); L.pb[0] = add(n.Z, 0);
      L.pw[1] = add(n.Z, L.K); L.pb[1] = add(n.Z, 0);
    } else {
      L.nseg = 1; L.seg_rows0 = L.N;
      L.pw[0] = add(L.N, L.K); L.pb[0] = add(L.N, 0);
      L.pw[1] = L.pw[0]; L.pb[1] = L.pb[0];
    }
  }
  h->nparams = off;

  // all padded biases back to back (copied into LDS by the row-chain prologue)
  n.nbias = 0;
  for (int l = 0; l < n.n_layers; ++l) {
    n.bias_off[l] = n.nbias;
    n.nbias += n.L[l].Np;
  }
  // LDS budget of the row-chain kernel: the largest row tile (16, 8 or 4 rows) whose state fits
  // in 160 KiB.  Tiles under 16 rows leave MFMA rows idle (duplicated rows), so they only serve
  // the wide configurations (latent 512, seq_len 200: SURVEY cfg5) that need them.
  // CVAE_ROW_TILE=<4|8|16> in the environment caps the tile (A/B measurements)
  const char* rt_env = std::getenv("CVAE_ROW_TILE");
  const int rt_cap = rt_env ? std::atoi(rt_env) : CVAE_ROWS;
  h->R = 0;
  for (int R : {CVAE_ROWS, 8, 4}) {
    if (R > CVAE_ROWS || (R > rt_cap && R > 4)) continue;
    const LdsPlan lp = lds_plan(n, R, h->tsize);
    if (lp.total <= 160 * 1024) { h->R = R; h->lds_bytes = lp.total; break; }
  }
  if (!h->R)
    return fail(CVAE_E_INVALID, "configuration needs " + std::to_string(lds_plan(n, 4, h->tsize).total) +
                                    " B of LDS per 4-row tile (> 160 KiB); reduce seq_len*dim or latent_dim");
  h->max_row_tiles = rup_i(c.max_batch, 32) / 4;  // loss partials of the smallest row tile any chain runs
  if (c.dim < 3) return fail(CVAE_E_INVALID, "dim must be >= 3 (channel 0 = time, 1:3 = x,y)");
  if (c.hidden_dim % 4 || c.latent_dim % 4)
    return fail(CVAE_E_INVALID, "hidden_dim and latent_dim must be multiples of 4 (4-feature epilogue vectors)");
  if (c.n_classes < 0 || (c.n_classes > 0 && (c.class_dim < 4 || c.class_dim % 4)))
    return fail(CVAE_E_INVALID, "class_dim must be a positive multiple of 4 when n_classes > 0");

  // Weight-gradient / parameter tiles: 32×32 over each layer's padded (Np × Kp), laid out for
  // the 8 XCDs.  Workgroup b runs on XCD b % 8 and every XCD has its own L2, so a tile's G rows
  // (shared along its o-block) and X rows (shared along its i-block) are re-fetched from the
  // fabric by every XCD that needs them.  The tiles are listed layer by layer with the longer
  // dimension outermost, cut into 8 contiguous chunks, and chunk x is placed at blockIdx
  // 8j + x: each XCD then covers compact regions of few layers and fetches their rows once.
  std::vector<TileDesc> seq;
  for (int l = 0; l < n.n_layers; ++l) {
    const LayerDev& L = n.L[l];
    if (L.Kp > L.Np) {
      for (int i = 0; i < L.Kp; i += 32)
        for (int o = 0; o < L.Np; o += 32) seq.push_back({l, o, i, 0});
    } else {
      for (int o = 0; o < L.Np; o += 32)
        for (int i = 0; i < L.Kp; i += 32) seq.push_back({l, o, i, 0});
    }
  }
  auto xcd_order = [](const std::vector<TileDesc>& list) {
    const int nt = (int)list.size(), q = nt / 8, r = nt % 8;
    std::vector<TileDesc> out(nt);
    for (int b = 0; b < nt; ++b) {
      const int x = b % 8, j = b / 8;
      const int start = x * q + (x < r ? x : r);  // chunk x = list[start, start + q + (x < r))
      out[b] = list[start + j];
    }
    return out;
  };
  h->tiles = xcd_order(seq);
  // more 32 × 32 tiles than workgroup slots (2 dW workgroups per CU, 256 CUs): the generic dW
  // launch takes 32 × 64 tiles where the layer's padded K is a multiple of 64 — fewer workgroups,
  // and each G row is read by half as many tiles (BASELINE cfg5: 868 → 442 tiles)
  h->wtiles = h->tiles;
  h->wtiles_ni2 = false;
  const char* ni2_env = std::getenv("CVAE_DW_NI2");  // "0": 32 × 32 tiles only (A/B)
  if (c.dtype != CVAE_F32 && seq.size() > 512 && !(ni2_env && ni2_env[0] == '0')) {
    std::vector<TileDesc> wseq;
    for (int l = 0; l < n.n_layers; ++l) {
      const LayerDev& L = n.L[l];
      const int ni = (L.Kp % 64 == 0 && !L.wt) ? 2 : 1;
      if (L.Kp > L.Np) {
        for (int i = 0; i < L.Kp; i += 32 * ni)
          for (int o = 0; o < L.Np; o += 32) wseq.push_back({l, o, i, ni});
      } else {
        for (int o = 0; o < L.Np; o += 32)
          for (int i = 0; i < L.Kp; i += 32 * ni) wseq.push_back({l, o, i, ni});
      }
      h->wtiles_ni2 = h->wtiles_ni2 || ni == 2;
    }
    h->wtiles = xcd_order(wseq);
  }
  std::vector<TileDesc> dec, rest;
  for (const TileDesc& t : seq) (t.layer >= lD(n, 0) ? dec : rest).push_back(t);
  h->tiles_part[0] = xcd_order(dec);
  h->tiles_part[1] = xcd_order(rest);
  h->bucket_split = n.L[lD(n, 0)].pw[0];
  return CVAE_OK;
}

// Step tables (see cvae_rowchain.h).  Masks: C0=0, C1=1, E_i=2+i, D_i=2+n_enc+i.
std::vector<StepSpec> build_steps(const NetDev& n, int mode) {
  const bool train = mode == cvae_handle::ST_TRAIN;
  const int ne = n.n_enc, nd = n.n_dec, Z = n.Z, H = n.H;
  auto arena = [&](void* p) -> void* { return train ? p : nullptr; };
  auto blank = [&]() {
    StepSpec s{};
    s.mask_out = -1; s.mask_in = -1; s.dst1 = B_NONE; s.dst2 = B_NONE;
    return s;
  };
  auto fwd = [&](int l, int xbuf, int epi) {
    StepSpec s = blank();
    const LayerDev& L = n.L[l];
    s.W = L.Wf; s.bias_off = n.bias_off[l]; s.Kp = L.Kp; s.Np = L.Np; s.N = L.N; s.f8 = L.f8;
    s.xbuf = xbuf; s.epi = epi;
    return s;
  };
  auto bwd = [&](int l, int xbuf, int epi) {
    StepSpec s = blank();
    const LayerDev& L = n.L[l];
    s.W = L.Wb; s.bias_off = -1; s.Kp = L.Np; s.Np = L.Kp; s.N = L.K; s.xbuf = xbuf;
    s.epi = epi;
    return s;
  };
  auto pb = [](int i) { return (i & 1) ? B_P1 : B_P0; };
  std::vector<StepSpec> v;
#ifdef CVAE_DIAG_SIMPLE
  // microbenchmark (diagnostic builds only): CVAE_DIAG_SIMPLE copies of one plain 128x128
  // forward step (encoder layer 1, ping-ponging P0 ↔ P1) — the per-step cost without special steps
  if (train) {
    for (int k = 0; k < CVAE_DIAG_SIMPLE; ++k) {
      StepSpec s = fwd(lE(n, 1), pb(k), E_RELU);
      s.mask_out = 3; s.dst1 = pb(k + 1); s.g1 = n.L[lE(n, 2)].xT;
      v.push_back(s);
    }
    return v;
  }
#endif
  if (mode != cvae_handle::ST_DEC_HC) {
    StepSpec s = fwd(lC0(n), B_CIN, E_RELU);
    s.mask_out = 0; s.dst1 = B_P0; s.g1 = arena(n.L[lC1(n)].xT);
    v.push_back(s);
    s = fwd(lC1(n), B_P0, E_RELU);
    s.mask_out = 1; s.concat = 1;
    s.dst1 = B_HC; s.off1 = H; s.dst2 = B_DEC; s.off2 = Z;
    s.g1 = arena(n.L[lFC(n)].xT); s.goff1 = H; s.g2 = arena(n.L[lD(n, 0)].xT); s.goff2 = Z;
    s.hc_out = train ? 0 : 1;
    v.push_back(s);
  }
  if (mode == cvae_handle::ST_COND) return v;
  if (n.n_cls) {  // cfg4: e = table[class] → [.. ‖ e] of the fc input and of the decoder input
    StepSpec s = fwd(lCE(n), B_CLS, E_RELU);
    s.linear = 1; s.concat = 1;
    s.dst1 = B_HC; s.off1 = 2 * H; s.dst2 = B_DEC; s.off2 = Z + H;
    s.g1 = arena(n.L[lFC(n)].xT); s.goff1 = 2 * H; s.g2 = arena(n.L[lD(n, 0)].xT); s.goff2 = Z + H;
    v.push_back(s);
  }
  if (mode == cvae_handle::ST_TRAIN || mode == cvae_handle::ST_FWD) {
    for (int i = 0; i < ne; ++i) {
      StepSpec s = fwd(lE(n, i), i == 0 ? B_XIN : pb(i - 1), E_RELU);
      s.mask_out = 2 + i;
      if (i == ne - 1) {
        s.dst1 = B_HC; s.off1 = 0; s.concat = 1; s.g1 = arena(n.L[lFC(n)].xT);
      } else {
        s.dst1 = pb(i); s.g1 = arena(n.L[lE(n, i + 1)].xT);
      }
      v.push_back(s);
    }
    v.push_back(fwd(lFC(n), B_HC, E_FC));
  }
  for (int i = 0; i < nd - 1; ++i) {
    StepSpec s = fwd(lD(n, i), i == 0 ? B_DEC : pb(i - 1), E_RELU);
    s.mask_out = 2 + ne + i; s.dst1 = pb(i); s.g1 = arena(n.L[lD(n, i + 1)].xT);
    v.push_back(s);
  }
  {
    StepSpec s = fwd(lD(n, nd - 1), nd == 1 ? B_DEC : pb(nd - 2), train ? E_LOSS : E_RECON);
    if (train) s.g1 = n.L[lD(n, nd - 1)].gT;
    v.push_back(s);
  }
  if (!train) return v;
  // backward: decoder → reparameterisation → fc → encoder / condition encoder
  int cur = B_XIN, pp = 0;
  for (int i = nd - 1; i >= 1; --i) {
    StepSpec s = bwd(lD(n, i), cur, E_BWD);
    s.mask_in = 2 + ne + i - 1; s.dst1 = pp ? B_P1 : B_P0; s.g1 = n.L[lD(n, i - 1)].gT;
    v.push_back(s);
    cur = s.dst1;
    pp ^= 1;
  }
  v.push_back(bwd(lD(n, 0), cur, E_D0B));
  {
    StepSpec s = bwd(lFC(n), B_P0, E_FCB);
    s.g1 = n.L[lE(n, ne - 1)].gT; s.g2 = n.L[lC1(n)].gT;
    v.push_back(s);
  }
  cur = B_P1;
  int p = 0;
  for (int i = ne - 1; i >= 1; --i) {
    StepSpec s = bwd(lE(n, i), cur, E_BWD);
    s.mask_in = 2 + i - 1; s.dst1 = i > 1 ? (p ? B_P1 : B_P0) : B_NONE; s.g1 = n.L[lE(n, i - 1)].gT;
    v.push_back(s);
    cur = s.dst1;
    p ^= 1;
  }
  {
    StepSpec s = bwd(lC1(n), B_HC, E_BWD);
    s.mask_in = 0; s.g1 = n.L[lC0(n)].gT;
    v.push_back(s);
  }
  return v;
}

int alloc_arena(cvae_handle* h) {
  NetDev& n = h->net;
  const int ts = h->tsize;
  std::vector<int64_t> offs;
  int64_t total = 0;
  auto take = [&](int64_t bytes) { int64_t o = total; total += (bytes + 255) / 256 * 256; return o; };
  struct Off { int64_t wf, wb, wb8, bias, xT, gT; };
  std::vector<Off> lo(n.n_layers);
  for (int l = 0; l < n.n_layers; ++l) {
    LayerDev& L = n.L[l];
    lo[l].wf = take((int64_t)L.Np * L.Kp * ts + (L.f8 ? (int64_t)sizeof(F8Scale) : 0));
    lo[l].wb = take((int64_t)L.Kp * L.Np * ts);
    lo[l].wb8 = L.f8b ? take((int64_t)L.Kp * L.Np) : -1;
    lo[l].bias = n.bias_off[l];  // planned in build_plan
  }
  const int64_t bias_base = take((int64_t)n.nbias * 4);
  // activations: every layer has its own xT and gT (inputs that are concatenations
  // are written by their producers at column offsets)
  for (int l = 0; l < n.n_layers; ++l) {
    LayerDev& L = n.L[l];
    lo[l].xT = take((int64_t)L.Kp * n.Bp * ts);
    lo[l].gT = take((int64_t)L.Np * n.Bp * ts);
  }
  int maxnp = 32;
  for (int l = 0; l < n.n_layers; ++l) maxnp = std::max(maxnp, std::max(n.L[l].Np, n.L[l].Kp));
  const int64_t zb_off = take((int64_t)maxnp * 4);
  const int64_t part_off = take((int64_t)h->max_row_tiles * 8 * 4);
  // split-K for batches of >= 8192 rows: up to 16 splits of >= 2048 rows (cvae_wgrad.h SplitK)
  h->splitk_max = std::max(1, std::min(16, rup_i(h->cfg.max_batch, 32) / 2048));
  if (rup_i(h->cfg.max_batch, 32) < 8192) h->splitk_max = 1;
  // split-K partials: [tile][split][pw] for either tile list (pw = 32·TW + 32 of its widest tile)
  const int64_t skw_floats = std::max((int64_t)h->tiles.size() * (32 * 32 + 32),
                                      (int64_t)h->wtiles.size() * (h->wtiles_ni2 ? 32 * 64 + 32 : 32 * 32 + 32));
  const int64_t skw_off = h->splitk_max > 1 ? take(skw_floats * h->splitk_max * 4) : 0;
  const int64_t skt_off = h->splitk_max > 1 ? take((int64_t)std::max(h->tiles.size(), h->wtiles.size()) * 4) : 0;
  const int64_t tile_off = take((int64_t)h->tiles.size() * sizeof(TileDesc));
  const int64_t wtile_off = take((int64_t)h->wtiles.size() * sizeof(TileDesc));
  const int64_t tp_off0 = take((int64_t)h->tiles_part[0].size() * sizeof(TileDesc));
  const int64_t tp_off1 = take((int64_t)h->tiles_part[1].size() * sizeof(TileDesc));
  int64_t step_off[cvae_handle::ST_N];
  for (int m = 0; m < cvae_handle::ST_N; ++m) step_off[m] = take(64 * (int64_t)sizeof(StepDesc));
  HIPCK(hipMalloc(&h->arena, total));
  HIPCK(hipMemset(h->arena, 0, total));
  HIPCK(hipHostMalloc((void**)&h->fault_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(h->fault_host, 0, 64);
  HIPCK(hipHostGetDevicePointer((void**)&h->fault_dev, h->fault_host, 0));
  h->arena_bytes = total;
  for (int l = 0; l < n.n_layers; ++l) {
    LayerDev& L = n.L[l];
    L.Wf = h->arena + lo[l].wf + (L.f8 ? sizeof(F8Scale) : 0);  // f8: F8Scale header in front
    L.Wb = h->arena + lo[l].wb;
    L.Wb8 = L.f8b ? h->arena + lo[l].wb8 : nullptr;
    L.bias = (float*)(h->arena + bias_base) + lo[l].bias;
    L.xT = h->arena + lo[l].xT;
    L.gT = h->arena + lo[l].gT;
  }
  n.zbias = (const float*)(h->arena + zb_off);
  n.bias_all = (const float*)(h->arena + bias_base);
  h->d_partials = (float*)(h->arena + part_off);
  if (h->splitk_max > 1) {  // tickets start at zero (the arena memset) and return to zero after every launch
    h->splitk_ws = (float*)(h->arena + skw_off);
    h->splitk_tickets = (unsigned*)(h->arena + skt_off);
  }
  h->d_tiles = (TileDesc*)(h->arena + tile_off);
  HIPCK(hipMemcpy(h->d_tiles, h->tiles.data(), h->tiles.size() * sizeof(TileDesc), hipMemcpyHostToDevice));
  h->d_wtiles = (TileDesc*)(h->arena + wtile_off);
  HIPCK(hipMemcpy(h->d_wtiles, h->wtiles.data(), h->wtiles.size() * sizeof(TileDesc), hipMemcpyHostToDevice));
  const int64_t tp_off[2] = {tp_off0, tp_off1};
  for (int k = 0; k < 2; ++k) {
    h->d_tiles_part[k] = (TileDesc*)(h->arena + tp_off[k]);
    HIPCK(hipMemcpy(h->d_tiles_part[k], h->tiles_part[k].data(), h->tiles_part[k].size() * sizeof(TileDesc),
                    hipMemcpyHostToDevice));
  }
  for (int m = 0; m < cvae_handle::ST_N; ++m) {
    const std::vector<StepSpec> spec = build_steps(n, m);
    std::vector<StepDesc> st;
    for (StepSpec x : spec) {
      // feature rows of the arena matrices g1 / g2 point into (xT: Kp, gT: Np of their layer)
      auto kf_of = [&](const void* g) {
        for (int l = 0; l < n.n_layers; ++l) {
          if (g == n.L[l].xT) return n.L[l].Kp;
          if (g == n.L[l].gT) return n.L[l].Np;
        }
        return 0;
      };
      x.kf1 = x.g1 ? kf_of(x.g1) : 0;
      x.kf2 = x.g2 ? kf_of(x.g2) : 0;
      if ((x.g1 && !x.kf1) || (x.g2 && !x.kf2)) return fail(CVAE_E_INVALID, "step arena target is not a layer matrix");
      if (x.goff1 < 0 || x.goff1 > 0xFFFF || x.goff2 < 0 || x.goff2 > 0xFFFF || x.mask_out > 62 || x.mask_in > 62)
        return fail(CVAE_E_INVALID, "step descriptor field out of range");
      st.push_back(encode_step(x));
    }
    if (st.empty() || st.size() > 64) return fail(CVAE_E_INVALID, "bad step table");
    h->d_steps[m] = (StepDesc*)(h->arena + step_off[m]);
    h->n_steps[m] = (int)st.size();
    HIPCK(hipMemcpy(h->d_steps[m], st.data(), st.size() * sizeof(StepDesc), hipMemcpyHostToDevice));
  }
  return CVAE_OK;
}

template <typename T, int R, bool F8>
int set_lds_attrs_rf(cvae_handle* h) {
  HIPCK(hipFuncSetAttribute((const void*)rowchain_kernel<T, R, RC_TRAIN, F8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytes));
  HIPCK(hipFuncSetAttribute((const void*)rowchain_kernel<T, R, RC_FWD, F8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytes));
  HIPCK(hipFuncSetAttribute((const void*)rowchain_kernel<T, R, RC_DECODE, F8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, h->lds_bytes));
  return CVAE_OK;
}
// CVAE_FP8 runs its own instantiation (F8 = true): the bf16/fp32 kernels carry no fp8 code
template <typename T, int R>
int set_lds_attrs_r(cvae_handle* h) {
  if constexpr (std::is_same<T, __bf16>::value)
    if (h->cfg.dtype == CVAE_FP8) return set_lds_attrs_rf<T, R, true>(h);
  return set_lds_attrs_rf<T, R, false>(h);
}
template <typename T>
int set_lds_attrs(cvae_handle* h) {
  if (h->R == CVAE_ROWS) return set_lds_attrs_r<T, CVAE_ROWS>(h);
  if (h->R == 8) return set_lds_attrs_r<T, 8>(h);
  if (h->R == 4) return set_lds_attrs_r<T, 4>(h);
  return fail(CVAE_E_INVALID, "no row-chain instance for this row tile");
}

// ---- timing helpers (no syncs).  With timing on, tmark(name) names the next kernel launch and
// klaunch records that launch's own start/end timestamps (hipExtLaunchKernelGGL's event pair: the
// dispatch packet's begin/end, the interval rocprofv3's kernel trace reports) — events recorded
// between kernels would add the dispatch gap and their own overhead to every duration.
void tbegin(cvae_handle* h) { h->pending = nullptr; }
int tmark(cvae_handle* h, hipStream_t, const char* name) {
  h->pending = (h->timing && std::strcmp(name, "end") != 0) ? name : nullptr;
  return CVAE_OK;
}
int tevent(cvae_handle* h) {
  if (h->n_used >= (int)h->pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    h->pool.push_back(e);
  }
  return h->n_used++;
}
template <typename... KArgs, typename... Args>
int klaunch(cvae_handle* h, void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t shm, hipStream_t s,
            Args... args) {
  if (h->timing && h->pending) {
    const int e0 = tevent(h), e1 = tevent(h);
    if (e0 < 0 || e1 < 0) return fail(CVAE_E_HIP, "hipEventCreate failed");
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)shm, s, h->pool[e0], h->pool[e1], 0, args...);
    h->segs.push_back({e0, e1, h->pending});
    h->pending = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shm, s, args...);
  }
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

template <typename T, int MODE, int R>
int launch_rowchain_r(cvae_handle* h, RowArgs a, hipStream_t s) {
  // the grid covers roundup(batch, 32) rows: the wgrad K range (a multiple of the 32-deep bf16
  // chunk) then only reads rows this launch wrote (zeros past the batch)
  const int grid = rup_i(a.batch, 32) / R;
  int st = cvae_handle::ST_TRAIN;
  if (MODE == RC_FWD) st = cvae_handle::ST_FWD;
  if (MODE == RC_DECODE) st = a.hc_in ? cvae_handle::ST_DEC_HC : (a.z_in ? cvae_handle::ST_DEC : cvae_handle::ST_COND);
  a.steps = h->d_steps[st];
  a.nsteps = h->n_steps[st];
  a.stamps = h->d_stamps;
  if constexpr (std::is_same<T, __bf16>::value)
    if (h->cfg.dtype == CVAE_FP8)
      return klaunch(h, rowchain_kernel<T, R, MODE, true>, dim3(grid), dim3(RC_THREADS), h->lds_bytes, s, h->net, a);
  return klaunch(h, rowchain_kernel<T, R, MODE, false>, dim3(grid), dim3(RC_THREADS), h->lds_bytes, s, h->net, a);
}
template <typename T, int MODE>
int launch_rowchain(cvae_handle* h, RowArgs a, hipStream_t s) {
  if (h->R == CVAE_ROWS) return launch_rowchain_r<T, MODE, CVAE_ROWS>(h, a, s);
  if (h->R == 8) return launch_rowchain_r<T, MODE, 8>(h, a, s);
  if (h->R == 4) return launch_rowchain_r<T, MODE, 4>(h, a, s);
  return fail(CVAE_E_INVALID, "no row-chain instance for this row tile");
}

int check_batch(cvae_handle* h, int batch) {
  if (batch <= 0) return fail(CVAE_E_INVALID, "batch must be > 0");
  if (batch > h->cfg.max_batch)
    return fail(CVAE_E_CAPACITY, "batch " + std::to_string(batch) + " > max_batch " + std::to_string(h->cfg.max_batch));
  return CVAE_OK;
}

AdamArgs make_adam(float* params, float* grads, float* m, float* v, int64_t step, const cvae_adam_config& c,
                   float grad_scale, const uint64_t* ctr) {
  AdamArgs a{};
  a.params = params; a.grads = grads; a.m = m; a.v = v;
  a.grad_scale = grad_scale;
  // torch computes these in Python doubles, then the tensor ops take them as float
  // (torch/optim/adam.py _single_tensor_adam): step_size = lr / (1 - beta1**step), bias_correction2**0.5
  if (!ctr) {
    const double bc1 = 1.0 - std::pow(c.beta1, (double)step);
    const double bc2 = 1.0 - std::pow(c.beta2, (double)step);
    a.lr_neg_step = (float)(-(c.lr / bc1));
    a.bc2_sqrt = (float)std::pow(bc2, 0.5);
  }
  a.beta1_w = (float)(1.0 - c.beta1);   // exp_avg.lerp_(grad, 1 - beta1)
  a.beta2 = (float)c.beta2;             // exp_avg_sq.mul_(beta2)
  a.one_m_beta2 = (float)(1.0 - c.beta2);  // .addcmul_(grad, grad, value=1 - beta2)
  a.eps = (float)c.eps;
  a.ctr = ctr;
  a.lr = c.lr; a.beta1d = c.beta1; a.beta2d = c.beta2;
  return a;
}

// The specialised bf16 training chain (cvae_fastchain.h) covers the reference architecture:
// hidden 128, latent 8, 4+4 layers, S·D a multiple of 8 padding to one of the instantiated chunk
// counts.  CVAE_GENERIC=1 in the environment forces the interpreter (A/B comparisons).
constexpr int kFastNki[] = {19};
// the compile-time arena layout the fast kernel addresses (fchain::Layout) is the handle's
template <int NKI>
bool fast_layout_matches(const cvae_handle* h) {
  using LY = fchain::Layout<NKI>;
  const NetDev& n = h->net;
  if (n.n_layers != LY::NL || n.nbias != LY::nbias || n.Bp % 32 != 0 ||
      (const char*)n.bias_all != h->arena + LY::bias_base)
    return false;
  const int64_t Bp2 = 2 * (int64_t)n.Bp;
  // the fast kernel's tiles (some 64 inputs wide) cover exactly the handle's 32×32 tile set
  std::vector<std::array<int, 3>> mine, theirs;
  for (int b = 0; b < fchain::Tiles<NKI>::total(); ++b) {
    const TileDesc t = fchain::Tiles<NKI>::at(b);
    for (int s = 0; s < fchain::Tiles<NKI>::ni(t.layer); ++s) mine.push_back({t.layer, t.o0, t.i0 + 32 * s});
  }
  for (const TileDesc& t : h->tiles) theirs.push_back({t.layer, t.o0, t.i0});
  std::sort(mine.begin(), mine.end());
  std::sort(theirs.begin(), theirs.end());
  if (mine != theirs) return false;
  for (int l = 0; l < LY::NL; ++l) {
    const LayerDev& L = n.L[l];
    const LayerDev F = fchain::fast_layer<NKI>(l, h->arena, n.Bp, n.I);
    if (F.K != L.K || F.N != L.N || F.Kp != L.Kp || F.Np != L.Np || F.relu != L.relu || F.nseg != L.nseg ||
        F.seg_rows0 != L.seg_rows0 || F.Wf != L.Wf || F.Wb != L.Wb || F.bias != L.bias || F.xT != L.xT ||
        F.gT != L.gT)
      return false;
    for (int g = 0; g < 2; ++g)
      if (F.pw[g] != L.pw[g] || F.pb[g] != L.pb[g]) return false;
    if (L.Kp != LY::Kp(l) || L.Np != LY::Np(l) || n.bias_off[l] != LY::bias_off(l) ||
        (char*)L.Wf != h->arena + LY::wf(l) || (char*)L.Wb != h->arena + LY::wb(l) ||
        (char*)L.xT != h->arena + LY::act0 + Bp2 * LY::xrows(l) ||
        (char*)L.gT != h->arena + LY::act0 + Bp2 * LY::grows(l))
      return false;
  }
  return true;
}

// the bucket kernel's tiles (fastwgrad_bucket_kernel) are the handle's bucket lists, in order
template <int NKI>
bool fast_buckets_match(const cvae_handle* h) {
  using T = fchain::Tiles<NKI>;
  for (int k = 0; k < 2; ++k) {
    const int n = T::bucket_count(k);
    if ((int)h->tiles_part[k].size() != n) return false;
    for (int b = 0; b < n; ++b) {
      const TileDesc a = T::decode(T::bucket_first(k) + T::slot(b, n)), &t = h->tiles_part[k][b];
      if (a.layer != t.layer || a.o0 != t.o0 || a.i0 != t.i0) return false;
    }
  }
  return true;
}

int plan_fast(cvae_handle* h) {
  const cvae_config& c = h->cfg;
  const NetDev& n = h->net;
  h->fast_nki = 0;
  h->fast_buckets = false;
  const char* env = std::getenv("CVAE_GENERIC");
  if ((env && env[0] == '1') || c.dtype != CVAE_BF16 || c.n_classes > 0 || c.hidden_dim != fchain::H ||
      c.latent_dim != fchain::Z ||
      c.n_enc != 4 || c.n_dec != 4 || n.I % 8 != 0 || n.nbias > 16 * fchain::NT || h->R != 16)
    return CVAE_OK;
  for (int nki : kFastNki) {
    if (n.Ip != 32 * nki) continue;
    const fchain::Lds lp = fchain::lds_layout(n.Ip, n.S, n.nbias);
    if (lp.total > 160 * 1024) return CVAE_OK;
    if (nki == 19 && !fast_layout_matches<19>(h)) return CVAE_OK;
    h->fast_nki = nki;
    h->fast_lds = lp.total;
    const char* gb = std::getenv("CVAE_GENERIC_BUCKETS");  // "1": the buckets on the generic kernel (A/B)
    h->fast_buckets = nki == 19 && fast_buckets_match<19>(h) && !(gb && gb[0] == '1');
    if (nki == 19) {
      HIPCK(hipFuncSetAttribute((const void*)fchain::fastchain_kernel<19>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lp.total));
    }
  }
  return CVAE_OK;
}

// The specialised wide chain (cvae_widechain.h) covers exactly BASELINE cfg5's shape in bf16:
// S=200, D=6, latent 512, 8+8 layers, hidden 128.  Its compile-time arena offsets are checked
// against the handle's layout before it is enabled (as fast_layout_matches).
template <class A>
bool wide_layout_matches(const cvae_handle* h) {
  const NetDev& n = h->net;
  if (n.n_layers != A::NL || n.nbias != A::nbias || n.Bp % 32 != 0 ||
      (const char*)n.bias_all != h->arena + A::bias_base)
    return false;
  const int64_t Bp2 = 2 * (int64_t)n.Bp;
  for (int l = 0; l < A::NL; ++l) {
    const LayerDev& L = n.L[l];
    if (L.Kp != A::Kp(l) || L.Np != A::Np(l) || n.bias_off[l] != A::bias_off(l) || (L.f8 != 0) != A::f8(l) ||
        (char*)L.Wf != h->arena + A::wf(l) || (char*)L.Wb != h->arena + A::wb(l) ||
        (char*)L.xT != h->arena + A::act0 + Bp2 * A::xrows(l) ||
        (char*)L.gT != h->arena + A::act0 + Bp2 * A::grows(l) || (L.f8b != 0) != A::f8b(l) ||
        (L.f8b && (char*)L.Wb8 != h->arena + A::wb8(l)))
      return false;
    const bool relu = !(l == A::LFC || l == A::LDL || l == A::LCE);
    if (L.relu != (relu ? 1 : 0)) return false;
  }
  return true;
}

// The reference architecture (the fast configuration, S=100: BASELINE cfg2) on the single-ring
// weight-stream chain (cvae_widechain.h, small-latent form) instead of fastchain_kernel's per-step
// register prefetch: the per-CU L2 stream stays busy across step barriers.  The default for this
// shape (row chain 17.8 vs 18.35 us at B = 1024); CVAE_RING=0 at creation keeps
// fastchain_kernel.
// the chain instance for the rows' format: bf16 rows (the bench's and the peer step's data) run the
// form with the fp32-row loads compiled out (wchain::wide_body's XB)
template <class A>
auto chain_for(const RowArgs& ra) {
  return ra.x_f32 ? wchain::widechain_kernel<A> : wchain::widechain_kernel<A, false, true>;
}

int plan_ring(cvae_handle* h) {
  using A = wchain::Cfg2;
  const cvae_config& c = h->cfg;
  h->ring = false;
  const char* env = std::getenv("CVAE_RING");
  if ((env && env[0] == '0') || h->fast_nki != 19 || c.seq_len != A::S || c.dim != A::D) return CVAE_OK;
  if (!wide_layout_matches<A>(h) || h->arena_bytes >= ((int64_t)1 << 31)) return CVAE_OK;
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            A::L_TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, A::L_TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, A::L_TOTAL));
  h->ring = true;
  h->ring_lds = A::L_TOTAL;
  return CVAE_OK;
}

// cfg4's compile-time dW decode (cvae_widewgrad.h CTiles / cls_layer) restates the handle's tile list
// (order included) and every layer record for this handle's n_classes and class_dim
template <class A>
bool cls_dw_matches(const cvae_handle* h) {
  using CT = wchain::CTiles<A>;
  if (h->wtiles_ni2 || (int)h->wtiles.size() != CT::total()) return false;
  for (int b = 0; b < CT::total(); ++b) {
    const TileDesc t = CT::at(b), u = h->wtiles[b];
    if (t.layer != u.layer || t.o0 != u.o0 || t.i0 != u.i0 || u.ni > 1) return false;
  }
  for (int l = 0; l < A::NL; ++l) {
    const LayerDev& L = h->net.L[l];
    const LayerDev F = wchain::cls_layer<A>(l, h->arena, h->net.Bp, h->cfg.n_classes, h->cfg.class_dim);
    if (F.K != L.K || F.N != L.N || F.Kp != L.Kp || F.Np != L.Np || F.relu != L.relu || F.nseg != L.nseg ||
        F.seg_rows0 != L.seg_rows0 || F.f8 != L.f8 || F.wt != L.wt || F.has_bias != L.has_bias || F.Wf != L.Wf ||
        F.Wb != L.Wb || F.bias != L.bias || F.xT != L.xT || F.gT != L.gT || F.f8b != L.f8b || F.Wb8 != L.Wb8)
      return false;
    for (int g = 0; g < 2; ++g)
      if (F.pw[g] != L.pw[g] || F.pb[g] != L.pb[g]) return false;
  }
  return true;
}

// BASELINE cfg4 (the class embedding) at cfg2's shape on the ring chain (wchain::Cfg4), its dW ⊕ Adam
// on the compile-time decode (wchain::clswgrad_kernel; CVAE_CLS_DW=generic keeps the tile list)
int plan_ring_cls(cvae_handle* h) {
  using A = wchain::Cfg4;
  const cvae_config& c = h->cfg;
  h->ring_cls = false;
  const char* env = std::getenv("CVAE_RING");
  const char* gen = std::getenv("CVAE_GENERIC");
  if ((env && env[0] == '0') || (gen && gen[0] == '1') || c.dtype != CVAE_BF16 || c.n_classes < 1 ||
      c.n_classes > A::CLS_NMAX || c.class_dim < 4 || c.class_dim > A::CLS_EMAX || c.class_dim % 4 ||
      c.seq_len != A::S || c.dim != A::D || c.latent_dim != A::Z || c.hidden_dim != wchain::H || c.n_enc != A::NE ||
      c.n_dec != A::ND || h->R != wchain::R)
    return CVAE_OK;
  if (!wide_layout_matches<A>(h) || h->arena_bytes >= ((int64_t)1 << 31)) return CVAE_OK;
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            A::L_TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, A::L_TOTAL));
  h->ring_cls = true;
  h->ring_lds = A::L_TOTAL;
  const char* dw = std::getenv("CVAE_CLS_DW");
  h->cls_dw = !(dw && std::strcmp(dw, "generic") == 0) && cls_dw_matches<A>(h);
  return CVAE_OK;
}

// The reference's own configuration in fp32 (Training_VAE.py:274-282: seq_len 10, dim 3, latent 8,
// hidden 128, 4+4 layers; BASELINE configs[0]) on the fp32 ring chain (cvae_f32chain.h) instead of the
// generic interpreter.  Its compile-time arena offsets are checked against the handle's layout.
template <class A>
bool f32c_layout_matches(const cvae_handle* h) {
  const NetDev& n = h->net;
  if (n.n_layers != f32c::NL || n.nbias != A::nbias || n.Bp % 32 != 0 ||
      (const char*)n.bias_all != h->arena + A::bias_base)
    return false;
  const int64_t Bp4 = 4 * (int64_t)n.Bp;
  for (int l = 0; l < f32c::NL; ++l) {
    const LayerDev& L = n.L[l];
    if (L.Kp != A::Kp(l) || L.Np != A::Np(l) || n.bias_off[l] != A::bias_off(l) || L.f8 || L.f8b ||
        (char*)L.Wf != h->arena + A::wf(l) || (char*)L.Wb != h->arena + A::wb(l) ||
        (char*)L.xT != h->arena + A::act0 + Bp4 * A::xrows(l) || (char*)L.gT != h->arena + A::act0 + Bp4 * A::grows(l))
      return false;
    const bool relu = !(l == f32c::LFC || l == f32c::LD3);
    if (L.relu != (relu ? 1 : 0)) return false;
  }
  return true;
}

// the fp32 chain's compile-time dW decode (cvae_f32wgrad.h) covers the handle's 32 × 32 tile list
// exactly (as a set: each tile is one independent wgrad_body) and restates every layer record
template <class A>
bool f32c_dw_matches(const cvae_handle* h) {
  using WT = f32c::WTiles<A>;
  if (h->wtiles_ni2 || (int)h->wtiles.size() != WT::total()) return false;
  std::vector<int> seen(WT::total(), 0);
  for (int b = 0; b < WT::total(); ++b) {
    const TileDesc t = WT::at(b);
    int hit = -1;
    for (int u = 0; u < (int)h->wtiles.size(); ++u) {
      const TileDesc& w = h->wtiles[u];
      if (w.layer == t.layer && w.o0 == t.o0 && w.i0 == t.i0 && w.ni <= 1) hit = u;
    }
    if (hit < 0 || seen[hit]++) return false;
  }
  for (int l = 0; l < f32c::NL; ++l) {
    const LayerDev& L = h->net.L[l];
    const LayerDev F = f32c::f32_layer<A>(l, h->arena, h->net.Bp);
    if (F.K != L.K || F.N != L.N || F.Kp != L.Kp || F.Np != L.Np || F.relu != L.relu || F.nseg != L.nseg ||
        F.seg_rows0 != L.seg_rows0 || F.f8 != L.f8 || F.wt != L.wt || F.has_bias != L.has_bias || F.Wf != L.Wf ||
        F.Wb != L.Wb || F.bias != L.bias || F.xT != L.xT || F.gT != L.gT || F.f8b != L.f8b || F.Wb8 != L.Wb8)
      return false;
    for (int g = 0; g < 2; ++g)
      if (F.pw[g] != L.pw[g] || F.pb[g] != L.pb[g]) return false;
  }
  return true;
}

int plan_f32c(cvae_handle* h) {
  using A = f32c::Cfg1;
  const cvae_config& c = h->cfg;
  h->f32c = false;
  const char* gen = std::getenv("CVAE_GENERIC");
  if ((gen && gen[0] == '1') || c.dtype != CVAE_F32 || c.n_classes > 0 || c.hidden_dim != f32c::H ||
      c.latent_dim != f32c::Z || c.n_enc != 4 || c.n_dec != 4 || c.seq_len != A::S || c.dim != A::D)
    return CVAE_OK;
  // the chain stores to the arena and streams its weights through 32-bit buffer offsets
  if (!f32c_layout_matches<A>(h) || h->arena_bytes >= ((int64_t)1 << 31)) return CVAE_OK;
  HIPCK(hipFuncSetAttribute((const void*)f32c::f32chain_kernel<A, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            A::L_TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)f32c::f32chain_kernel<A, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            A::L_TOTAL));
  h->f32c = true;
  // CVAE_F32_ROWS=16 / =4: one row tiling at every batch (A/B); default: 4-row workgroups up to
  // CVAE_F32_R4_MAX_BATCH rows (each workgroup streams all weights, so many small ones cost L2 traffic)
  const char* rows = std::getenv("CVAE_F32_ROWS");
  const char* r4max = std::getenv("CVAE_F32_R4_MAX_BATCH");
  h->f32c_r4_max = rows && std::atoi(rows) == 16 ? 0 : rows && std::atoi(rows) == 4 ? (1 << 30)
                 : r4max ? std::atoi(r4max) : CVAE_F32_R4_MAX;
  const char* spread = std::getenv("CVAE_F32_SPREAD");
  h->f32c_spread = spread && (std::atoi(spread) == 1 || std::atoi(spread) == 2 || std::atoi(spread) == 4) ? std::atoi(spread) : 8;
  h->f32c_lds = A::L_TOTAL;
  const char* dw = std::getenv("CVAE_F32_DW");  // "generic": the tile-list kernel (A/B)
  h->f32c_dw = !(dw && std::strcmp(dw, "generic") == 0) && f32c_dw_matches<A>(h);
  return CVAE_OK;
}

// the compile-time dW decode of the wide shape (cvae_widewgrad.h) restates the handle's 32 × 64 tile
// list and layer table exactly (CVAE_DW_NI2=0 or any other difference keeps the generic kernel)
template <class A>
bool wide_dw_matches(const cvae_handle* h) {
  using WT = wchain::WTiles<A>;
  if (!h->wtiles_ni2 || (int)h->wtiles.size() != WT::total()) return false;
  for (int b = 0; b < WT::total(); ++b) {
    const TileDesc t = WT::at(b), u = h->wtiles[b];
    if (t.layer != u.layer || t.o0 != u.o0 || t.i0 != u.i0 || t.ni != u.ni) return false;
  }
  for (int l = 0; l < A::NL; ++l) {
    const LayerDev& L = h->net.L[l];
    const LayerDev F = wchain::wide_layer<A>(l, h->arena, h->net.Bp);
    if (F.K != L.K || F.N != L.N || F.Kp != L.Kp || F.Np != L.Np || F.relu != L.relu || F.nseg != L.nseg ||
        F.seg_rows0 != L.seg_rows0 || F.f8 != L.f8 || F.wt != L.wt || F.has_bias != L.has_bias || F.Wf != L.Wf ||
        F.Wb != L.Wb || F.bias != L.bias || F.xT != L.xT || F.gT != L.gT || F.f8b != L.f8b || F.Wb8 != L.Wb8)
      return false;
    for (int g = 0; g < 2; ++g)
      if (F.pw[g] != L.pw[g] || F.pb[g] != L.pb[g]) return false;
  }
  return true;
}

template <class A>
int plan_wide_as(cvae_handle* h) {
  // the wide chain stores to the arena through a buffer resource of 2^31 - 1 bytes
  if (!wide_layout_matches<A>(h) || h->arena_bytes >= ((int64_t)1 << 31)) return CVAE_OK;
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            A::L_TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)wchain::widechain_kernel<A, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, A::L_TOTAL));
  h->wide = true;
  h->wide_lds = A::L_TOTAL;
  const char* g = std::getenv("CVAE_GENERIC_DW");  // "1": the generic tile-list dW kernel (A/B)
  h->wide_dw = !(g && g[0] == '1') && wide_dw_matches<A>(h);
  // the MX dW (measured slower than the bf16 dW at B = 1024, DESIGN §4.5: an option, not the default)
  const char* mw = std::getenv("CVAE_FP8_DW");
  h->wide_mxw = std::is_same<A, wchain::Cfg5F8>::value && h->wide_dw && mw && std::strcmp(mw, "mx") == 0;
  return CVAE_OK;
}

// bf16 runs wchain::Cfg5, CVAE_FP8 wchain::Cfg5F8 (e4m3 forward GEMMs and MX dX GEMMs) or, with
// CVAE_FP8_DX=bf16, wchain::Cfg5F8B (e4m3 forward, bf16 dX)
int plan_wide(cvae_handle* h) {
  using A = wchain::Cfg5;
  const cvae_config& c = h->cfg;
  h->wide = false;
  const char* env = std::getenv("CVAE_GENERIC");
  if ((env && env[0] == '1') || (c.dtype != CVAE_BF16 && c.dtype != CVAE_FP8) || c.n_classes > 0 ||
      c.hidden_dim != wchain::H || c.seq_len != A::S || c.dim != A::D || c.latent_dim != A::Z || c.n_enc != A::NE ||
      c.n_dec != A::ND)
    return CVAE_OK;
  if (c.dtype != CVAE_FP8) return plan_wide_as<A>(h);
  h->wide_mx = wide_fp8_mx(c);
  return h->wide_mx ? plan_wide_as<wchain::Cfg5F8>(h) : plan_wide_as<wchain::Cfg5F8B>(h);
}

// What every training / inference call hands the row chain.
struct CallX {
  const void* x;
  const int64_t* idx;
  const int32_t* classes;
  int batch;
  int xflags;
  const float* eps;
  uint64_t seed, offset;
  int64_t eps_row0;
  const cvae_loss_weights* w;
  uint64_t* ctr;
  const cvae_adam_config* adam;  // with ctr: the chain precomputes the step's Adam scalars
};

RowArgs row_args(cvae_handle* h, const CallX& c) {
  RowArgs ra{};
  ra.x = c.x; ra.idx = c.idx; ra.classes = c.classes; ra.batch = c.batch; ra.eps = c.eps; ra.seed = c.seed; ra.offset = c.offset;
  ra.eps_row0 = c.eps_row0;
  ra.x_f32 = (c.xflags & CVAE_X_F32) && is16(h) ? 1 : 0;
  ra.ctr = c.ctr;
  if (c.ctr && c.adam) {
    ra.adam_pre = 1;
    ra.lr = c.adam->lr; ra.beta1 = c.adam->beta1; ra.beta2 = c.adam->beta2;
  }
  ra.w_recon = c.w ? c.w->recon : 0.1f; ra.w_kld = c.w ? c.w->kld : 0.1f;
  ra.w_start = c.w ? c.w->start : 1.0f; ra.w_time = c.w ? c.w->time : 1.0f;
  ra.partials = h->d_partials;
  ra.ncls = h->net.n_cls;
  ra.cdim = h->net.cls_dim;
  return ra;
}

bool fast_ok(const cvae_handle* h, const RowArgs& ra) {
  return h->fast_nki > 0 && (((uintptr_t)ra.x) & 15) == 0 && !ra.x_f32 && !ra.ext && !ra.x_relative;
}
// the ring and wide chains (cvae_widechain.h Cfg2 / Cfg4 / Cfg5*) also take fp32 rows (CVAE_X_F32,
// the train loop's real data): the prologue subtracts the start point in fp32 and rounds once
bool ring_ok(const cvae_handle* h, const RowArgs& ra) {
  return h->ring && h->fast_nki > 0 && (((uintptr_t)ra.x) & 15) == 0 && (((uintptr_t)ra.eps) & 15) == 0 && !ra.ext &&
         !ra.x_relative;
}
bool ring_cls_ok(const cvae_handle* h, const RowArgs& ra) {
  return h->ring_cls && (((uintptr_t)ra.x) & 15) == 0 && (((uintptr_t)ra.eps) & 15) == 0 && !ra.ext &&
         !ra.x_relative;
}
// fp32 rows of S·D = 30 floats are 8-B aligned (the x-tile loads are feature pairs)
bool f32c_ok(const cvae_handle* h, const RowArgs& ra) {
  return h->f32c && (((uintptr_t)ra.x) & 7) == 0 && (((uintptr_t)ra.eps) & 15) == 0 && !ra.ext && !ra.x_relative;
}
int f32c_rows(const cvae_handle* h, int batch) { return batch <= h->f32c_r4_max ? 4 : 16; }
bool wide_ok(const cvae_handle* h, const RowArgs& ra) {
  return h->wide && (((uintptr_t)ra.x) & 15) == 0 && (((uintptr_t)ra.eps) & 15) == 0 && !ra.ext &&
         !ra.x_relative;
}
// rows per workgroup of the training row chain a call runs (its loss partials are per workgroup)
int chain_rows(const cvae_handle* h, const RowArgs& ra) {
  if (fast_ok(h, ra)) return fchain::R;
  if (ring_ok(h, ra) || ring_cls_ok(h, ra)) return wchain::R;
  if (wide_ok(h, ra)) return wchain::R;
  if (f32c_ok(h, ra)) return f32c_rows(h, ra.batch);
  return h->R;
}

// the training row chain (forward + loss + every dX): the specialised bf16 chain where it applies
// tap_ok: the caller is cvae_train_fwd_bwd, the one entry point that consumes an armed parity tap
// (cvae_tap_outputs); every other training call fails while one is armed, so a tap whose buffers a
// caller freed is never written by a later step or by a captured graph
template <typename T>
int launch_train_chain(cvae_handle* h, RowArgs ra, hipStream_t s, bool tap_ok = false) {
  const bool tap = h->tap[0] || h->tap[1] || h->tap[2];
  if (tap && !tap_ok)
    return fail(CVAE_E_INVALID, "cvae_tap_outputs is armed: only cvae_train_fwd_bwd consumes it (disarm with NULLs)");
  int rc = tmark(h, s, "rowchain");
  if (rc) return rc;
  if (tap) {  // one-shot (cvae_tap_outputs): this launch only
    ra.recon_out = h->tap[0];
    ra.mu_out = h->tap[1];
    ra.lv_out = h->tap[2];
    h->tap[0] = h->tap[1] = h->tap[2] = nullptr;
    if (!(std::is_same<T, __bf16>::value && ring_ok(h, ra)))
      return fail(CVAE_E_INVALID, "cvae_tap_outputs: only the ring chain (seq_len 100, dim 6, bf16) writes them");
    ra.stamps = h->d_stamps;
    const int grid = rup_i(ra.batch, 32) / wchain::R;
    return klaunch(h, wchain::widechain_kernel<wchain::Cfg2, true>, dim3(grid), dim3(wchain::NT), h->ring_lds, s,
                   h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra);
  }
  if (std::is_same<T, __bf16>::value && ring_ok(h, ra)) {
    ra.stamps = h->d_stamps;
    const int grid = rup_i(ra.batch, 32) / wchain::R;
    return klaunch(h, chain_for<wchain::Cfg2>(ra), dim3(grid), dim3(wchain::NT), h->ring_lds, s,
                   h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra);
  }
  if (std::is_same<T, __bf16>::value && ring_cls_ok(h, ra)) {
    ra.stamps = h->d_stamps;
    const int grid = rup_i(ra.batch, 32) / wchain::R;
    return klaunch(h, chain_for<wchain::Cfg4>(ra), dim3(grid), dim3(wchain::NT), h->ring_lds, s,
                   h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra);
  }
  if (std::is_same<T, __bf16>::value && fast_ok(h, ra)) {
    ra.steps = h->d_steps[cvae_handle::ST_TRAIN];
    ra.nsteps = h->n_steps[cvae_handle::ST_TRAIN];
    ra.stamps = h->d_stamps;
    const int grid = rup_i(ra.batch, 32) / fchain::R;
    return klaunch(h, fchain::fastchain_kernel<19>, dim3(grid), dim3(fchain::NT), h->fast_lds, s, h->arena, ra.x,
                   ra.idx, h->net.Bp, ra.batch, h->net.S, h->net.D, h->net.I, ra);
  }
  if (std::is_same<T, __bf16>::value && wide_ok(h, ra)) {
    ra.stamps = h->d_stamps;
    const int grid = rup_i(ra.batch, 32) / wchain::R;
    if (h->cfg.dtype == CVAE_FP8 && h->wide_mx)
      return klaunch(h, chain_for<wchain::Cfg5F8>(ra), dim3(grid), dim3(wchain::NT), h->wide_lds, s,
                     h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra);
    if (h->cfg.dtype == CVAE_FP8)
      return klaunch(h, chain_for<wchain::Cfg5F8B>(ra), dim3(grid), dim3(wchain::NT), h->wide_lds, s,
                     h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra);
    return klaunch(h, chain_for<wchain::Cfg5>(ra), dim3(grid), dim3(wchain::NT), h->wide_lds, s,
                   h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra);
  }
  if (std::is_same<T, float>::value && f32c_ok(h, ra)) {
    ra.stamps = h->d_stamps;
    const int rows = f32c_rows(h, ra.batch), tiles = rup_i(ra.batch, 32) / rows;
    // CVAE_F32_SPREAD=1|2|4: the tiles on that many XCDs (A/B; 8 = every XCD, the plain grid)
    const int spread = h->f32c_spread < 8 && tiles % h->f32c_spread == 0 && tiles / h->f32c_spread <= 32 ? h->f32c_spread : 8;
    const int grid = spread < 8 ? tiles / spread * 8 : tiles;
    return klaunch(h, rows == 4 ? f32c::f32chain_kernel<f32c::Cfg1, 4> : f32c::f32chain_kernel<f32c::Cfg1, 16>,
                   dim3(grid), dim3(f32c::NT), h->f32c_lds, s, h->arena, ra.x, ra.idx, h->net.Bp, ra.batch, ra.ctr, ra,
                   spread);
  }
  return launch_rowchain<T, RC_TRAIN>(h, ra, s);
}

LossArgs make_loss(cvae_handle* h, const RowArgs& ra, float* loss_out, double* loss_accum) {
  LossArgs la{};
  la.partials = h->d_partials;
  la.ntiles = rup_i(ra.batch, 32) / chain_rows(h, ra);
  la.batch = ra.batch;
  la.w_recon = ra.w_recon; la.w_kld = ra.w_kld; la.w_start = ra.w_start; la.w_time = ra.w_time;
  la.loss_out = loss_out; la.loss_accum = loss_accum;
  la.ctr = ra.ctr;
  return la;
}

int bk_of(cvae_handle*, int batch) { return rup_i(batch, 32); }

// the dW (⊕ Adam) launch of a training step: the fast kernel for the fast configuration, the
// generic kernel over a bucket's tile list for a split (two-bucket) step
// splits of the dW launch's K (= batch) range: 1 below 8192 rows, else >= 2048 rows per split
int splits_of(const cvae_handle* h, int batch) {
  const int Bk = rup_i(batch, 32);
  if (h->splitk_max <= 1 || Bk < 8192) return 1;
  const char* env = std::getenv("CVAE_SPLITK");  // A/B measurements: force a split count
  const int want = env ? std::atoi(env) : Bk / 2048;
  return std::max(1, std::min(h->splitk_max, want));
}

template <int MODE>
int launch_wgrad(cvae_handle* h, int batch, const AdamArgs& aa, const LossArgs& la, hipStream_t s,
                 int parts = CVAE_PART_DW_DEC | CVAE_PART_DW_REST) {
  const int dw = parts & (CVAE_PART_DW_DEC | CVAE_PART_DW_REST);
  SplitK sk{splits_of(h, batch), 0, h->splitk_ws, h->splitk_tickets, 0};
  if (dw != (CVAE_PART_DW_DEC | CVAE_PART_DW_REST)) {
    const int k = dw == CVAE_PART_DW_DEC ? 0 : 1;
    if (h->fast_buckets) {
      using T = fchain::Tiles<19>;
      return klaunch(h, fchain::fastwgrad_bucket_kernel<19, MODE>, dim3(T::bucket_count(k) * sk.S + 1),
                     dim3(WG_THREADS), 0, s, h->arena, aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), h->net.S,
                     h->net.D, h->net.I, aa, la, sk, T::bucket_first(k), T::bucket_count(k));
    }
    const int nt = (int)h->tiles_part[k].size();
    if (is16(h))
      return klaunch(h, wgrad_kernel<__bf16, MODE>, dim3(nt * sk.S), dim3(WG_THREADS), 0, s, h->net,
                     (const TileDesc*)h->d_tiles_part[k], bk_of(h, batch), aa, la, sk);
    return klaunch(h, wgrad_kernel<float, MODE>, dim3(nt * sk.S), dim3(WG_THREADS), 0, s, h->net,
                   (const TileDesc*)h->d_tiles_part[k], bk_of(h, batch), aa, la, sk);
  }
  const int nt = (int)h->wtiles.size();
  if (h->wide_dw) {  // BASELINE cfg5: the compile-time tile decode (cvae_widewgrad.h)
    sk.pw = 32 * 64 + 32;
    const int g = wchain::WTiles<wchain::Cfg5>::total() * sk.S + 1;
    static_assert(wchain::WTiles<wchain::Cfg5>::total() == wchain::WTiles<wchain::Cfg5F8>::total(), "tile lists");
    if (h->cfg.dtype == CVAE_FP8 && h->wide_mxw && batch % 128 == 0)  // the MX dW: 128-row chunks
      return klaunch(h, wchain::widewgrad_kernel<wchain::Cfg5F8, MODE, true>, dim3(g), dim3(WG_THREADS), 0, s,
                     h->arena, aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), aa, la, sk);
    if (h->cfg.dtype == CVAE_FP8 && h->wide_mx)
      return klaunch(h, wchain::widewgrad_kernel<wchain::Cfg5F8, MODE>, dim3(g), dim3(WG_THREADS), 0, s, h->arena,
                     aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), aa, la, sk);
    if (h->cfg.dtype == CVAE_FP8)
      return klaunch(h, wchain::widewgrad_kernel<wchain::Cfg5F8B, MODE>, dim3(g), dim3(WG_THREADS), 0, s, h->arena,
                     aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), aa, la, sk);
    return klaunch(h, wchain::widewgrad_kernel<wchain::Cfg5, MODE>, dim3(g), dim3(WG_THREADS), 0, s, h->arena,
                   aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), aa, la, sk);
  }
  if (h->cls_dw)
    return klaunch(h, wchain::clswgrad_kernel<wchain::Cfg4, MODE>, dim3(wchain::CTiles<wchain::Cfg4>::total() * sk.S + 1),
                   dim3(WG_THREADS), 0, s, h->arena, aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch),
                   h->cfg.n_classes, h->cfg.class_dim, aa, la, sk);
  if (h->f32c_dw)
    return klaunch(h, f32c::f32wgrad_kernel<f32c::Cfg1, MODE>, dim3(f32c::WTiles<f32c::Cfg1>::total() * sk.S + 1),
                   dim3(WG_THREADS), 0, s, h->arena, aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), aa, la, sk);
  if (h->fast_nki == 19)
    return klaunch(h, fchain::fastwgrad_kernel<19, MODE>, dim3(fchain::Tiles<19>::total() * sk.S + 1),
                   dim3(WG_THREADS), 0, s, h->arena, aa.params, aa.m, aa.v, h->net.Bp, bk_of(h, batch), h->net.S,
                   h->net.D, h->net.I, aa, la, sk);
  if (is16(h) && h->wtiles_ni2) {
    sk.pw = 32 * 64 + 32;
    return klaunch(h, wgrad_kernel<__bf16, MODE, true>, dim3(nt * sk.S), dim3(WG_THREADS), 0, s, h->net,
                   (const TileDesc*)h->d_wtiles, bk_of(h, batch), aa, la, sk);
  }
  if (is16(h))
    return klaunch(h, wgrad_kernel<__bf16, MODE>, dim3(nt * sk.S), dim3(WG_THREADS), 0, s, h->net,
                   (const TileDesc*)h->d_wtiles, bk_of(h, batch), aa, la, sk);
  return klaunch(h, wgrad_kernel<float, MODE>, dim3(nt * sk.S), dim3(WG_THREADS), 0, s, h->net,
                 (const TileDesc*)h->d_wtiles, bk_of(h, batch), aa, la, sk);
}

// a training call fails while the handle's fault word is set (a kernel of an earlier call gave up
// a bounded spin and skipped work: that step's parameters are incomplete).  A host read of pinned
// memory the device writes at system scope: no synchronisation
int check_fault(const cvae_handle* h) {
  if (h->fault_host && __atomic_load_n(h->fault_host, __ATOMIC_ACQUIRE))
    return fail(CVAE_E_TIMEOUT, "an earlier training launch timed out waiting for a hand-off and skipped its "
                                "update (fault word set); the parameters are incomplete — cvae_clear_fault after "
                                "restoring them (with the peer exchange open: cvae_px_reset on every rank, which "
                                "also re-arms its mailbox)");
  return CVAE_OK;
}

// a step with no rows on this rank (a ragged global batch shorter than the world): advance the
// device counters exactly as a row chain + dW launch would (steps begun + that step's Adam scalars,
// Philox offset), so this rank's Adam and eps stay in step with the others
__global__ void step_skip_kernel(uint64_t* c, double lr, double b1, double b2) {
  adam_precompute(c, lr, b1, b2, true);
  c[0] = c[0] + 1;
}

int check_adam(const cvae_adam_config* adam) {
  if (!adam) return fail(CVAE_E_INVALID, "null adam config");
  if (!(adam->beta1 >= 0.0 && adam->beta1 < 1.0 && adam->beta2 >= 0.0 && adam->beta2 < 1.0))
    return fail(CVAE_E_INVALID, "betas must lie in [0, 1)");
  return CVAE_OK;
}

int fwd_bwd_impl(cvae_handle* h, const CallX& c, float* grads, float* loss_out, double* loss_accum, int parts,
                 hipStream_t s) {
  tbegin(h);
  const RowArgs ra = row_args(h, c);
  int rc = CVAE_OK;
  if (parts & CVAE_PART_CHAIN)
    rc = is16(h) ? launch_train_chain<__bf16>(h, ra, s, true) : launch_train_chain<float>(h, ra, s, true);
  if (rc) return rc;
  AdamArgs aa{};
  aa.grads = grads;
  LossArgs la{};
  if (parts & CVAE_PART_CHAIN) la = make_loss(h, ra, loss_out, loss_accum);  // the loss belongs to the chain's call
  const int dw = parts & (CVAE_PART_DW_DEC | CVAE_PART_DW_REST);
  if ((rc = tmark(h, s, dw == CVAE_PART_DW_DEC ? "wgrad_dec" : dw == CVAE_PART_DW_REST ? "wgrad_rest" : "wgrad")))
    return rc;
  return launch_wgrad<PM_GRAD>(h, c.batch, aa, la, s, parts);
}

int train_step_impl(cvae_handle* h, const CallX& c, float* params, float* m, float* v, int64_t step,
                    const cvae_adam_config* adam, float* loss_out, double* loss_accum, hipStream_t s) {
  tbegin(h);
  AdamArgs aa = make_adam(params, nullptr, m, v, step, *adam, 1.f, c.ctr);
  CallX ca = c;
  ca.adam = adam;
  const RowArgs ra = row_args(h, ca);
  int rc = is16(h) ? launch_train_chain<__bf16>(h, ra, s) : launch_train_chain<float>(h, ra, s);
  if (rc) return rc;
  const LossArgs la = make_loss(h, ra, loss_out, loss_accum);
  if ((rc = tmark(h, s, "wgrad_adam"))) return rc;
  return launch_wgrad<PM_ADAM>(h, c.batch, aa, la, s);
}

}  // namespace

extern "C" {

const char* cvae_last_error(void) { return g_err.c_str(); }
int cvae_abi_version(void) { return CVAE_ABI_VERSION; }

int cvae_create(const cvae_config* cfg, int device, cvae_handle** out) {
  if (!cfg || !out) return fail(CVAE_E_INVALID, "null argument");
  if (cfg->seq_len < 1 || cfg->dim < 1 || cfg->latent_dim < 1 || cfg->hidden_dim < 1 || cfg->n_enc < 1 ||
      cfg->n_dec < 1 || cfg->max_batch < 1 ||
      (cfg->dtype != CVAE_F32 && cfg->dtype != CVAE_BF16 && cfg->dtype != CVAE_FP8))
    return fail(CVAE_E_INVALID, "invalid cvae_config");
  cvae_handle* h = new cvae_handle();
  h->cfg = *cfg;
  h->device = device;
  int rc = build_plan(h);
  if (rc) { delete h; return rc; }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete h; return fail(CVAE_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)); }
  rc = alloc_arena(h);
  if (!rc) rc = is16(h) ? set_lds_attrs<__bf16>(h) : set_lds_attrs<float>(h);
  if (!rc) rc = plan_fast(h);
  if (!rc) rc = plan_wide(h);
  if (!rc) rc = plan_ring(h);
  if (!rc) rc = plan_ring_cls(h);
  if (!rc) rc = plan_f32c(h);
  if (rc) { cvae_destroy(h); return rc; }
  *out = h;
  return CVAE_OK;
}

int cvae_destroy(cvae_handle* h) {
  if (!h) return CVAE_OK;
  for (auto e : h->pool) (void)hipEventDestroy(e);
  if (h->arena) (void)hipFree(h->arena);
  if (h->fault_host) (void)hipHostFree(h->fault_host);
  cvae_px_close(h);
  cvae_rccl_close(h);
  delete h;
  return CVAE_OK;
}

int cvae_num_params(const cvae_handle* h, int64_t* total, int* n_tensors) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  if (total) *total = h->nparams;
  if (n_tensors) *n_tensors = (int)h->params.size();
  return CVAE_OK;
}

int cvae_param_info(const cvae_handle* h, int i, int64_t* offset, int64_t* numel, int* rows, int* cols) {
  if (!h || i < 0 || i >= (int)h->params.size()) return fail(CVAE_E_INVALID, "bad param index");
  const ParamInfo& p = h->params[i];
  if (offset) *offset = p.offset;
  if (numel) *numel = p.numel;
  if (rows) *rows = p.rows;
  if (cols) *cols = p.cols;
  return CVAE_OK;
}

int cvae_config_info(const cvae_config* cfg, int64_t* total_params, int* n_tensors, int* lds_bytes) {
  if (!cfg) return fail(CVAE_E_INVALID, "null argument");
  cvae_handle tmp;
  tmp.cfg = *cfg;
  const int rc = build_plan(&tmp);
  if (total_params) *total_params = tmp.nparams;
  if (n_tensors) *n_tensors = (int)tmp.params.size();
  if (lds_bytes) *lds_bytes = tmp.lds_bytes;
  return rc;
}

int cvae_workspace_bytes(const cvae_handle* h, int64_t* bytes) {
  if (!h || !bytes) return fail(CVAE_E_INVALID, "null argument");
  *bytes = h->arena_bytes;
  return CVAE_OK;
}

int cvae_train_kernel(const cvae_handle* h, int* kind) {
  if (!h || !kind) return fail(CVAE_E_INVALID, "null argument");
  *kind = h->ring || h->ring_cls ? CVAE_KERNEL_RING
           : h->fast_nki > 0      ? CVAE_KERNEL_FAST
           : h->wide              ? CVAE_KERNEL_WIDE
           : h->f32c              ? CVAE_KERNEL_F32
                                  : CVAE_KERNEL_GENERIC;
  return CVAE_OK;
}

int cvae_dw_kernel(const cvae_handle* h, int* kind) {
  if (!h || !kind) return fail(CVAE_E_INVALID, "null argument");
  *kind = h->wide_dw        ? CVAE_DW_WIDE
          : h->cls_dw       ? CVAE_DW_CLS
          : h->f32c_dw      ? CVAE_DW_F32
          : h->fast_nki == 19 ? CVAE_DW_FAST
                            : CVAE_DW_GENERIC;
  return CVAE_OK;
}

int cvae_chain_rows(const cvae_handle* h, int batch, int* rows) {
  if (!h || !rows) return fail(CVAE_E_INVALID, "null argument");
  if (batch < 1 || batch > h->cfg.max_batch) return fail(CVAE_E_INVALID, "batch must be in [1, max_batch]");
  RowArgs ra{};  // a call with 16-B aligned rows and host-relative-free input
  ra.batch = batch;
  *rows = chain_rows(h, ra);
  return CVAE_OK;
}

int cvae_bucket_split(const cvae_handle* h, int64_t* split) {
  if (!h || !split) return fail(CVAE_E_INVALID, "null argument");
  *split = h->bucket_split;
  return CVAE_OK;
}

int cvae_pack_weights(cvae_handle* h, const float* params, void* stream) {
  if (!h || !params) return fail(CVAE_E_INVALID, "null argument");
  hipStream_t s = (hipStream_t)stream;
  AdamArgs aa{};
  aa.params = (float*)params;
  const int nt = (int)h->tiles.size();
  if (h->cfg.dtype == CVAE_FP8)  // per-layer e4m3 weight scales first: the pack reads them
    hipLaunchKernelGGL(f8_scale_kernel, dim3(h->net.n_layers), dim3(CVAE_THREADS), 0, s, h->net, (const float*)params);
  if (is16(h))
    hipLaunchKernelGGL((param_kernel<__bf16, PM_PACK>), dim3(nt), dim3(CVAE_THREADS), 0, s, h->net, h->d_tiles, aa);
  else
    hipLaunchKernelGGL((param_kernel<float, PM_PACK>), dim3(nt), dim3(CVAE_THREADS), 0, s, h->net, h->d_tiles, aa);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_forward(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                 const float* start,
                 const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0, float* recon, float* mu,
                 float* logvar, float* hc, float* eps_out, void* stream) {
  if (!h || !x) return fail(CVAE_E_INVALID, "null argument");
  int rc = check_batch(h, batch);
  if (rc) return rc;
  RowArgs a = row_args(h, CallX{x, idx, classes, batch, xflags, eps, seed, offset, eps_row0, nullptr, nullptr, nullptr});
  a.start_in = start; a.x_relative = start ? 1 : 0;
  a.recon_out = recon; a.mu_out = mu; a.lv_out = logvar; a.hc_out = hc; a.eps_out = eps_out;
  hipStream_t s = (hipStream_t)stream;
  return is16(h) ? launch_rowchain<__bf16, RC_FWD>(h, a, s) : launch_rowchain<float, RC_FWD>(h, a, s);
}

int cvae_condition(cvae_handle* h, const float* start, int batch, float* hc, void* stream) {
  if (!h || !start || !hc) return fail(CVAE_E_INVALID, "null argument");
  int rc = check_batch(h, batch);
  if (rc) return rc;
  RowArgs a{};
  a.batch = batch; a.start_in = start; a.hc_out = hc;
  a.partials = h->d_partials;
  hipStream_t s = (hipStream_t)stream;
  return is16(h) ? launch_rowchain<__bf16, RC_DECODE>(h, a, s)
                                   : launch_rowchain<float, RC_DECODE>(h, a, s);
}

int cvae_decode(cvae_handle* h, const float* z, const float* start, const float* hc, const int32_t* classes, int batch,
                float* out, void* stream) {
  if (!h || !z || !out || (!start && !hc)) return fail(CVAE_E_INVALID, "null argument");
  int rc = check_batch(h, batch);
  if (rc) return rc;
  RowArgs a{};
  a.batch = batch; a.z_in = z; a.start_in = start; a.hc_in = hc; a.recon_out = out; a.classes = classes;
  a.partials = h->d_partials;
  hipStream_t s = (hipStream_t)stream;
  return is16(h) ? launch_rowchain<__bf16, RC_DECODE>(h, a, s)
                                   : launch_rowchain<float, RC_DECODE>(h, a, s);
}

int cvae_train_fwd_bwd(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                       const float* eps,
                       uint64_t seed, uint64_t offset, int64_t eps_row0, const cvae_loss_weights* w, float* grads,
                       float* loss_out, double* loss_accum, uint64_t* counters, const cvae_adam_config* adam,
                       int parts, void* stream) {
  if (!h || !grads || ((parts & CVAE_PART_CHAIN) && !x)) return fail(CVAE_E_INVALID, "null argument");
  if (parts != CVAE_PART_ALL && parts != (CVAE_PART_CHAIN | CVAE_PART_DW_DEC) && parts != CVAE_PART_DW_REST)
    return fail(CVAE_E_INVALID, "parts must be CVAE_PART_ALL, CHAIN|DW_DEC, or DW_REST");
  int rc = check_batch(h, batch);
  if (!rc) rc = check_fault(h);
  if (rc) return rc;
  if (adam && (rc = check_adam(adam))) return rc;
  return fwd_bwd_impl(h, CallX{x, idx, classes, batch, xflags, eps, seed, offset, eps_row0, w, counters, adam}, grads,
                      loss_out, loss_accum, parts, (hipStream_t)stream);
}

int cvae_backward(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                  const float* start,
                  const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0, const float* d_recon,
                  const float* d_mu, const float* d_logvar, const float* d_hc, float* grads, void* stream) {
  if (!h || !x || !grads) return fail(CVAE_E_INVALID, "null argument");
  int rc = check_batch(h, batch);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  tbegin(h);
  RowArgs ra = row_args(h, CallX{x, idx, classes, batch, xflags, eps, seed, offset, eps_row0, nullptr, nullptr, nullptr});
  ra.start_in = start; ra.x_relative = start ? 1 : 0;
  ra.ext = 1;
  ra.d_recon = d_recon; ra.d_mu = d_mu; ra.d_lv = d_logvar; ra.d_hc = d_hc;
  if ((rc = tmark(h, s, "rowchain_bwd"))) return rc;
  rc = is16(h) ? launch_rowchain<__bf16, RC_TRAIN>(h, ra, s) : launch_rowchain<float, RC_TRAIN>(h, ra, s);
  if (rc) return rc;
  AdamArgs aa{};
  aa.grads = grads;
  if ((rc = tmark(h, s, "wgrad"))) return rc;
  return launch_wgrad<PM_GRAD>(h, batch, aa, LossArgs{}, s);
}

int cvae_adam(cvae_handle* h, float* params, const float* grads, float* m, float* v, int64_t step,
              const cvae_adam_config* adam, float grad_scale, const uint64_t* counters, void* stream) {
  if (!h || !params || !grads || !m || !v) return fail(CVAE_E_INVALID, "null argument");
  if (!counters && step < 1) return fail(CVAE_E_INVALID, "step must be >= 1");
  int rc = check_adam(adam);
  if (!rc) rc = check_fault(h);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  AdamArgs aa = make_adam(params, (float*)grads, m, v, step, *adam, grad_scale, counters);
  const int nt = (int)h->tiles.size();
  if ((rc = tmark(h, s, "adam"))) return rc;
  if (h->fast_nki == 19)
    return klaunch(h, fchain::fastadam_kernel<19>, dim3(fchain::Tiles<19>::total()), dim3(CVAE_THREADS), 0, s,
                   h->arena, params, m, v, grads, h->net.Bp, h->net.I, aa);
  if (is16(h))
    return klaunch(h, param_kernel<__bf16, PM_ADAM>, dim3(nt), dim3(CVAE_THREADS), 0, s, h->net,
                   (const TileDesc*)h->d_tiles, aa);
  return klaunch(h, param_kernel<float, PM_ADAM>, dim3(nt), dim3(CVAE_THREADS), 0, s, h->net,
                 (const TileDesc*)h->d_tiles, aa);
}

namespace {
// elementwise Adam over params/m/v[lo, lo + count) with the shard's gradient g[0, count) (cvae_adam_flat)
__global__ void adam_flat_kernel(float* params, const float* g, float* m, float* v, int64_t lo, int64_t count,
                                 AdamArgs a) {
  adam_resolve(a, adam_step_load(a));
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    float mm = m[lo + i], vv = v[lo + i];
    const float p = adam_math(params[lo + i], g[i] * a.grad_scale, mm, vv, a);
    params[lo + i] = p;
    m[lo + i] = mm;
    v[lo + i] = vv;
  }
}
}  // namespace

int cvae_adam_flat(cvae_handle* h, float* params, const float* grads, float* m, float* v, int64_t lo, int64_t count,
                   int64_t step, const cvae_adam_config* adam, float grad_scale, const uint64_t* counters,
                   void* stream) {
  if (!h || !params || !m || !v || (count > 0 && !grads)) return fail(CVAE_E_INVALID, "null argument");
  if (lo < 0 || count < 0 || lo + count > h->nparams) return fail(CVAE_E_INVALID, "range outside the parameters");
  if (!counters && step < 1) return fail(CVAE_E_INVALID, "step must be >= 1");
  int rc = check_adam(adam);
  if (!rc) rc = check_fault(h);
  if (rc || count == 0) return rc;
  hipStream_t s = (hipStream_t)stream;
  const AdamArgs aa = make_adam(params, (float*)grads, m, v, step, *adam, grad_scale, counters);
  if ((rc = tmark(h, s, "adam_flat"))) return rc;
  const int blocks = (int)std::min<int64_t>((count + 255) / 256, 2048);
  return klaunch(h, adam_flat_kernel, dim3(blocks), dim3(256), 0, s, params, grads, m, v, lo, count, aa);
}

int cvae_train_step(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int xflags,
                    const float* eps,
                    uint64_t seed, uint64_t offset, int64_t eps_row0, const cvae_loss_weights* w, float* params,
                    float* m, float* v, int64_t step, const cvae_adam_config* adam, float* loss_out,
                    double* loss_accum, uint64_t* counters, void* stream) {
  if (!h || !x || !params || !m || !v) return fail(CVAE_E_INVALID, "null argument");
  if (!counters && step < 1) return fail(CVAE_E_INVALID, "step must be >= 1");
  int rc = check_batch(h, batch);
  if (!rc) rc = check_adam(adam);
  if (!rc) rc = check_fault(h);
  if (rc) return rc;
  return train_step_impl(h, CallX{x, idx, classes, batch, xflags, eps, seed, offset, eps_row0, w, counters, adam}, params, m, v,
                         step, adam, loss_out, loss_accum, (hipStream_t)stream);
}

int cvae_train_steps(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int batch, int n_steps,
                     int xflags,
                     const float* eps, uint64_t seed, uint64_t offset, int64_t eps_row0,
                     const cvae_loss_weights* w, float* params, float* m, float* v, int64_t step0,
                     const cvae_adam_config* adam, float* loss_out, double* loss_accum, uint64_t* counters,
                     void* stream) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  if (n_steps < 0) return fail(CVAE_E_INVALID, "n_steps must be >= 0");
  const int Z = h->cfg.latent_dim;
  for (int i = 0; i < n_steps; ++i) {
    const int rc = cvae_train_step(h, x, idx ? idx + (size_t)i * batch : nullptr, classes, batch, xflags,
                                   eps ? eps + (size_t)i * batch * Z : nullptr, seed, offset + (uint64_t)i, eps_row0,
                                   w, params, m, v, step0 + i, adam, loss_out, loss_accum, counters, stream);
    if (rc) return rc;
  }
  return CVAE_OK;
}

int cvae_train_epochs(cvae_handle* h, const void* x, const int64_t* idx, const int32_t* classes, int n_rows,
                      int batch, int n_steps, int xflags, const float* eps, uint64_t seed, uint64_t offset,
                      int64_t eps_row0, const cvae_loss_weights* w, float* params, float* m, float* v, int64_t step0,
                      const cvae_adam_config* adam, float* loss_out, double* loss_accum, uint64_t* counters,
                      void* stream) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  if (!idx || n_rows < 1 || batch < 1 || n_steps < 0) return fail(CVAE_E_INVALID, "idx, n_rows >= 1, batch >= 1, n_steps >= 0");
  const int Z = h->cfg.latent_dim;
  const int spe = (n_rows + batch - 1) / batch;
  for (int s = 0; s < n_steps; ++s) {
    const int e = s / spe, k = s % spe;
    const int64_t r0 = (int64_t)e * n_rows + (int64_t)k * batch;  // first visited row of this step
    const int b = std::min(batch, n_rows - k * batch);
    const int rc = cvae_train_step(h, x, idx + r0, classes, b, xflags, eps ? eps + r0 * Z : nullptr, seed,
                                   offset + (uint64_t)s, eps_row0, w, params, m, v, step0 + s, adam, loss_out,
                                   loss_accum ? loss_accum + 5 * (int64_t)e : nullptr, counters, stream);
    if (rc) return rc;
  }
  return CVAE_OK;
}

int cvae_bench_kernels(cvae_handle* h, const void* x, const int64_t* idx, int batch, int reps, float* params,
                       float* m, float* v, int64_t step0, float* ms, void* stream) {
  if (!h || !x || !params || !m || !v || !ms || reps < 1) return fail(CVAE_E_INVALID, "bad argument");
  int rc = check_batch(h, batch);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const bool timing = h->timing;
  h->timing = false;
  hipEvent_t e0, e1;
  HIPCK(hipEventCreate(&e0));
  HIPCK(hipEventCreate(&e1));
  const cvae_loss_weights w{0.1f, 0.1f, 1.0f, 1.0f};
  const cvae_adam_config ac{1e-3, 0.9, 0.999, 1e-8};
  auto timed = [&](int which, float* out) -> int {
    HIPCK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) {
      int rc2 = CVAE_OK;
      const CallX c{x, idx, nullptr, batch, 0, nullptr, 1, (uint64_t)r, 0, &w, nullptr, nullptr};
      if (which == 0) {
        rc2 = is16(h) ? launch_train_chain<__bf16>(h, row_args(h, c), s) : launch_train_chain<float>(h, row_args(h, c), s);
      } else if (which == 1) {
        AdamArgs aa = make_adam(params, nullptr, m, v, step0 + r, ac, 1.f, nullptr);
        rc2 = launch_wgrad<PM_ADAM>(h, batch, aa, LossArgs{}, s);
      } else {
        rc2 = train_step_impl(h, c, params, m, v, step0 + r, &ac, nullptr, nullptr, s);
      }
      if (rc2) return rc2;
    }
    HIPCK(hipEventRecord(e1, s));
    HIPCK(hipEventSynchronize(e1));
    HIPCK(hipEventElapsedTime(out, e0, e1));
    *out /= reps;
    return CVAE_OK;
  };
  for (int k = 0; k < 3 && !rc; ++k) rc = timed(k, ms + k);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  h->timing = timing;
  return rc;
}

int cvae_step_skip(cvae_handle* h, uint64_t* counters, const cvae_adam_config* adam, void* stream) {
  if (!h || !counters) return fail(CVAE_E_INVALID, "null argument");
  int rc = check_adam(adam);
  if (rc) return rc;
  hipLaunchKernelGGL(step_skip_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counters, adam->lr, adam->beta1,
                     adam->beta2);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

// ---------------------------------------------------------------- data parallel: peer exchange
namespace {
struct PxBlob {
  int magic, world, rank, nt;
  int64_t arena_bytes, mbox_bytes;
  int pci_domain, pci_bus, pci_device, cus;  // which GPU (ranks sharing one: the residency precondition)
  int chain_blocks, pad;                     // row-chain workgroups at the batch capacity
  hipIpcMemHandle_t arena, mbox;
};
constexpr int PX_MAGIC = 0x43505832;  // "CPX2"
int px_tiles(const cvae_handle*) { return fchain::Tiles<19>::total(); }
// bound of every exchange wait: CVAE_PX_TIMEOUT_MS (default 10000 ms: ranks of a real
// multi-GPU job may enter their first exchange seconds apart), in s_memrealtime ticks
uint64_t px_timeout_ticks() {
  const char* e = std::getenv("CVAE_PX_TIMEOUT_MS");
  const double ms = e ? std::atof(e) : 10000.0;
  return (uint64_t)(std::max(1.0, ms) * 1e5);
}

// set-up check of the mapping and the protocol's primitives: every rank stores a tagged word into
// every peer's probe slot, releases it and counts one arrival there; then waits (bounded) for the
// world − 1 arrivals in its own mailbox and checks every tag.  The probe area follows the done
// counter: [done_off + 64] arrivals, [done_off + 128 + 8·r] rank r's tag.
__global__ void px_probe_kernel(PeerArgs p, int* ok) {
  if (threadIdx.x != 0) return;
  const uint64_t tag = 0x5EED000000000000ull;
  for (int r = 0; r < p.world; ++r) {
    if (r == p.rank) continue;
    char* pr = p.mbox[r] + p.done_off;
    __hip_atomic_store((uint64_t*)(pr + 128) + p.rank, tag | (uint64_t)(p.rank + 1), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_fetch_add((uint64_t*)(pr + 64), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  char* mine = p.mbox[p.rank] + p.done_off;
  int good = px_wait((const uint64_t*)(mine + 64), (uint64_t)(p.world - 1), nullptr, p.timeout) ? 1 : 0;
  for (int r = 0; r < p.world && good; ++r)
    if (r != p.rank &&
        __hip_atomic_load((const uint64_t*)(mine + 128) + r, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) !=
            (tag | (uint64_t)(r + 1)))
      good = 0;
  *ok = good;
}
}  // namespace

int cvae_px_blob_bytes(int64_t* bytes) {
  if (!bytes) return fail(CVAE_E_INVALID, "null argument");
  *bytes = (int64_t)sizeof(PxBlob);
  return CVAE_OK;
}

int cvae_px_export(cvae_handle* h, int world, int rank, void* blob) {
  if (!h || !blob) return fail(CVAE_E_INVALID, "null argument");
  if (world < 2 || world > PX_MAX || rank < 0 || rank >= world)
    return fail(CVAE_E_INVALID, "peer exchange: 2 <= world <= " + std::to_string(PX_MAX) + ", 0 <= rank < world");
  if (h->fast_nki != 19 || !h->ring)
    return fail(CVAE_E_INVALID, "peer exchange serves the reference architecture at seq_len 100, dim 6, bf16 "
                                "(the ring chain and fastwgrad tiles); use the collective path otherwise");
  cvae_px_close(h);
  const int nt = px_tiles(h);
  h->px_done_off = ((int64_t)nt * 8 + 255) / 256 * 256;
  h->px_inbox_off = h->px_done_off + 512;  // done, probe words, statistics (cvae_peer.h)
  h->px_mbox_bytes = h->px_inbox_off + (int64_t)nt * world * PX_PW * 4;
  HIPCK(hipSetDevice(h->device));
  HIPCK(hipExtMallocWithFlags((void**)&h->px_mbox, h->px_mbox_bytes, hipDeviceMallocUncached));
  HIPCK(hipMemset(h->px_mbox, 0, h->px_mbox_bytes));
  HIPCK(hipDeviceSynchronize());
  PxBlob b{};
  b.magic = PX_MAGIC; b.world = world; b.rank = rank; b.nt = nt;
  b.arena_bytes = h->arena_bytes; b.mbox_bytes = h->px_mbox_bytes;
  hipDeviceProp_t prop;
  HIPCK(hipGetDeviceProperties(&prop, h->device));
  b.pci_domain = prop.pciDomainID; b.pci_bus = prop.pciBusID; b.pci_device = prop.pciDeviceID;
  b.cus = prop.multiProcessorCount;
  b.chain_blocks = rup_i(h->cfg.max_batch, 32) / wchain::R;
  HIPCK(hipIpcGetMemHandle(&b.arena, h->arena));
  HIPCK(hipIpcGetMemHandle(&b.mbox, h->px_mbox));
  std::memcpy(blob, &b, sizeof(b));
  h->px_world = world;
  h->px_rank = rank;
  h->px_ready = false;
  return CVAE_OK;
}

// Workgroups of the exchange's launches one CU holds at once, from the compiled kernels' resources
// (the residency precondition of cvae_peer.h was a constant): the minimum of what the
// occupancy calculator gives the row chain (both row formats, its dynamic LDS) and both px_wgrad
// forms, capped at PX_SLOTS_PER_CU.  Falls below 2 only if a kernel's VGPRs or LDS grow past the
// two-per-CU budget.
int px_slots_per_cu(const cvae_handle* h, int* out) {
  int a = 0, a2 = 0, b = 0, c = 0;
  HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, (const void*)wchain::widechain_kernel<wchain::Cfg2>,
                                                     wchain::NT, h->ring_lds));
  HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &a2, (const void*)wchain::widechain_kernel<wchain::Cfg2, false, true>, wchain::NT, h->ring_lds));
  a = std::min(a, a2);
  HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, (const void*)fchain::px_wgrad_kernel<19, true>,
                                                     WG_THREADS, 0));
  HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, (const void*)fchain::px_wgrad_kernel<19>, WG_THREADS, 0));
  *out = std::min(PX_SLOTS_PER_CU, std::min(a, std::min(b, c)));
  return CVAE_OK;
}

int cvae_px_import(cvae_handle* h, const void* blobs, uint64_t base) {
  if (!h || !blobs || !h->px_mbox) return fail(CVAE_E_INVALID, "peer exchange: export first");
  const PxBlob* b = (const PxBlob*)blobs;
  HIPCK(hipSetDevice(h->device));
  for (int r = 0; r < h->px_world; ++r)
    if (b[r].magic != PX_MAGIC || b[r].world != h->px_world || b[r].rank != r || b[r].nt != px_tiles(h) ||
        b[r].arena_bytes != h->arena_bytes || b[r].mbox_bytes != h->px_mbox_bytes)
      return fail(CVAE_E_INVALID, "peer exchange: rank " + std::to_string(r) +
                                      "'s blob does not match this configuration (same model, batch capacity, world)");
  // the residency precondition (cvae_peer.h): the k ranks on this rank's GPU share its 2·CUs slots
  const PxBlob& me = b[h->px_rank];
  int share = 0;
  for (int r = 0; r < h->px_world; ++r)
    share += b[r].pci_domain == me.pci_domain && b[r].pci_bus == me.pci_bus && b[r].pci_device == me.pci_device;
  int per_cu = 0;
  if (int rc = px_slots_per_cu(h, &per_cu)) return rc;
  const int nt = px_tiles(h);
  // one rank per GPU: the launch's nt tile blocks + the end block must all be resident at once
  if (per_cu * me.cus < nt + 1)
    return fail(CVAE_E_INVALID, "peer exchange: the kernels fit " + std::to_string(per_cu) +
                                    " workgroup(s) per CU, the exchange launch needs " + std::to_string(nt + 1) +
                                    " resident workgroups on " + std::to_string(me.cus) + " CUs");
  const int slots = per_cu * me.cus / std::max(share, 1);
  if (share > 1 && me.chain_blocks > slots)
    return fail(CVAE_E_INVALID, "peer exchange: " + std::to_string(share) + " ranks share one GPU; each may hold " +
                                    std::to_string(slots) + " resident workgroups, its row chain needs " +
                                    std::to_string(me.chain_blocks) + " (lower max_batch or the ranks per GPU)");
  h->px_share = std::max(share, 1);
  h->px_grid = share > 1 ? std::max(1, std::min(nt, slots - 1)) : nt;
  for (int r = 0; r < h->px_world; ++r) {
    if (r == h->px_rank) {
      h->px_arena[r] = h->arena;
      h->px_mb[r] = h->px_mbox;
      continue;
    }
    HIPCK(hipIpcOpenMemHandle((void**)&h->px_arena[r], b[r].arena, hipIpcMemLazyEnablePeerAccess));
    HIPCK(hipIpcOpenMemHandle((void**)&h->px_mb[r], b[r].mbox, hipIpcMemLazyEnablePeerAccess));
  }
  h->px_base = base;
  h->px_ready = true;
  return CVAE_OK;
}

int cvae_px_probe(cvae_handle* h, int* ok) {
  if (!h || !ok) return fail(CVAE_E_INVALID, "null argument");
  if (!h->px_ready) return fail(CVAE_E_INVALID, "peer exchange not set up");
  PeerArgs px{};
  px.world = h->px_world;
  px.rank = h->px_rank;
  for (int r = 0; r < px.world; ++r) px.mbox[r] = h->px_mb[r];
  px.done_off = h->px_done_off;
  px.timeout = px_timeout_ticks();
  int* d_ok = (int*)(h->fault_dev + 4);  // a spare word of the pinned fault page
  h->fault_host[4] = 0;
  hipLaunchKernelGGL(px_probe_kernel, dim3(1), dim3(64), 0, 0, px, d_ok);
  HIPCK(hipGetLastError());
  HIPCK(hipDeviceSynchronize());
  *ok = (int)__atomic_load_n(h->fault_host + 4, __ATOMIC_ACQUIRE);
  return CVAE_OK;
}

int cvae_px_stats(cvae_handle* h, uint64_t* out, int reset) {
  if (!h || !out) return fail(CVAE_E_INVALID, "null argument");
  if (!h->px_mbox) return fail(CVAE_E_INVALID, "peer exchange not set up");
  char* st = h->px_mbox + h->px_done_off + PX_STATS_OFF;
  HIPCK(hipDeviceSynchronize());
  HIPCK(hipMemcpy(out, st, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (reset) {
    HIPCK(hipMemset(st, 0, 4 * sizeof(uint64_t)));
    HIPCK(hipDeviceSynchronize());
  }
  return CVAE_OK;
}

int cvae_px_close(cvae_handle* h) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  for (int r = 0; r < PX_MAX; ++r) {
    if (r != h->px_rank) {
      if (h->px_arena[r]) (void)hipIpcCloseMemHandle(h->px_arena[r]);
      if (h->px_mb[r]) (void)hipIpcCloseMemHandle(h->px_mb[r]);
    }
    h->px_arena[r] = h->px_mb[r] = nullptr;
  }
  if (h->px_mbox) (void)hipFree(h->px_mbox);
  h->px_mbox = nullptr;
  h->px_ready = false;
  h->px_world = 0;
  return CVAE_OK;
}

int cvae_px_owned(const cvae_handle* h, uint8_t* mask) {
  if (!h || !mask) return fail(CVAE_E_INVALID, "null argument");
  if (!h->px_world) return fail(CVAE_E_INVALID, "peer exchange not set up");
  std::memset(mask, 0, (size_t)h->nparams);
  const int nt = px_tiles(h);
  for (int b = 0; b < nt; ++b) {
    if (px_owner(b, h->px_world) != h->px_rank) continue;
    const TileDesc td = fchain::Tiles<19>::at(b);
    const LayerDev& L = h->net.L[td.layer];
    for (int o = td.o0; o < td.o0 + 32 && o < L.N; ++o) {
      const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
      const int orow = seg ? o - L.seg_rows0 : o;
      for (int i = td.i0; i < td.i0 + 32 && i < L.K; ++i) mask[L.pw[seg] + (int64_t)orow * L.K + i] = 1;
      if (td.i0 == 0) mask[L.pb[seg] + orow] = 1;
    }
  }
  return CVAE_OK;
}

int cvae_px_train_step(cvae_handle* h, const void* x, const int64_t* idx, int batch, int xflags, const float* eps,
                       uint64_t seed, int64_t eps_row0, const cvae_loss_weights* w, float* params, float* m, float* v,
                       const cvae_adam_config* adam, const float* rank_scales, float* loss_out, double* loss_accum,
                       uint64_t* counters, void* stream) {
  if (!h || !params || !m || !v || !counters) return fail(CVAE_E_INVALID, "null argument");
  if (!h->px_ready) return fail(CVAE_E_INVALID, "peer exchange not set up (cvae_px_export / cvae_px_import)");
  if (batch < 0 || batch > h->cfg.max_batch) return fail(CVAE_E_CAPACITY, "batch out of range");
  if (batch > 0 && !x) return fail(CVAE_E_INVALID, "null x");
  int rc = check_adam(adam);
  if (!rc) rc = check_fault(h);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  tbegin(h);
  PeerArgs px{};
  px.world = h->px_world;
  px.rank = h->px_rank;
  px.ragged = rank_scales ? 1 : 0;
  for (int r = 0; r < px.world; ++r) {
    px.c[r] = rank_scales ? rank_scales[r] : 0.f;
    px.arena[r] = h->px_arena[r];
    px.mbox[r] = h->px_mb[r];
  }
  const int nt = px_tiles(h);
  int own = 0;
  for (int b = 0; b < nt; ++b) own += px_owner(b, px.world) == px.rank;
  px.n_remote = nt - own;
  px.done_off = h->px_done_off;
  px.inbox_off = h->px_inbox_off;
  px.base = h->px_base;
  px.fault = h->fault_dev;
  px.timeout = px_timeout_ticks();
  LossArgs la{};
  if (batch > 0) {
    CallX c{x, idx, nullptr, batch, xflags, eps, seed, 0, eps_row0, w, counters, adam};
    const RowArgs ra = row_args(h, c);
    if (!ring_ok(h, ra)) return fail(CVAE_E_INVALID, "peer exchange: x must be 16-B aligned rows (operand dtype or fp32)");
    if ((rc = launch_train_chain<__bf16>(h, ra, s))) return rc;
    la = make_loss(h, ra, loss_out, loss_accum);
  } else {  // no rows on this rank this step: the counters advance as a chain + dW launch would
    hipLaunchKernelGGL(step_skip_kernel, dim3(1), dim3(1), 0, s, counters, adam->lr, adam->beta1, adam->beta2);
    HIPCK(hipGetLastError());
  }
  const AdamArgs aa = make_adam(params, nullptr, m, v, 0, *adam, rank_scales ? 1.f : 1.f / (float)px.world, counters);
  if ((rc = tmark(h, s, "px_wgrad"))) return rc;
  const int grid = h->px_grid > 0 ? h->px_grid : nt;
  if (grid < nt)  // ranks sharing this GPU: fewer blocks, each looping over its tiles (cvae_peer.h)
    return klaunch(h, fchain::px_wgrad_kernel<19, true>, dim3(grid + 1), dim3(WG_THREADS), 0, s, h->arena, params,
                   m, v, h->net.Bp, bk_of(h, batch), h->net.S, h->net.D, h->net.I, aa, la, px);
  return klaunch(h, fchain::px_wgrad_kernel<19>, dim3(nt + 1), dim3(WG_THREADS), 0, s, h->arena, params, m, v,
                 h->net.Bp, bk_of(h, batch), h->net.S, h->net.D, h->net.I, aa, la, px);
}

int cvae_px_layout(const cvae_handle* h, int* ranks_on_gpu, int* tile_blocks) {
  if (!h || !ranks_on_gpu || !tile_blocks) return fail(CVAE_E_INVALID, "null argument");
  if (!h->px_ready) return fail(CVAE_E_INVALID, "peer exchange not set up");
  *ranks_on_gpu = h->px_share;
  *tile_blocks = h->px_grid;
  return CVAE_OK;
}

int cvae_px_reset(cvae_handle* h, uint64_t base) {
  if (!h) return fail(CVAE_E_INVALID, "null argument");
  if (!h->px_ready) return fail(CVAE_E_INVALID, "peer exchange not set up");
  HIPCK(hipSetDevice(h->device));
  HIPCK(hipDeviceSynchronize());
  // arrival flags, the done counter and the probe words; the wait statistics stay
  HIPCK(hipMemset(h->px_mbox, 0, h->px_done_off + PX_STATS_OFF));
  HIPCK(hipDeviceSynchronize());
  h->px_base = base;
  if (h->fault_host) __atomic_store_n(h->fault_host, 0u, __ATOMIC_RELEASE);
  return CVAE_OK;
}

// ---- the gradient all-reduce over RCCL, issued by the library on the caller's stream (include/cvae.h)
#define RCCLCK(x)                                                                       \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) return fail(CVAE_E_HIP, std::string(#x ": ") + ncclGetErrorString(r_)); \
  } while (0)

int cvae_rccl_id_bytes(int64_t* bytes) {
  if (!bytes) return fail(CVAE_E_INVALID, "null argument");
  *bytes = (int64_t)sizeof(ncclUniqueId);
  return CVAE_OK;
}

int cvae_rccl_unique_id(void* id) {
  if (!id) return fail(CVAE_E_INVALID, "null argument");
  ncclUniqueId u;
  RCCLCK(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return CVAE_OK;
}

int cvae_rccl_init(cvae_handle* h, const void* id, int world, int rank) {
  if (!h || !id) return fail(CVAE_E_INVALID, "null argument");
  if (world < 1 || rank < 0 || rank >= world) return fail(CVAE_E_INVALID, "rank must lie in [0, world)");
  cvae_rccl_close(h);
  HIPCK(hipSetDevice(h->device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  RCCLCK(ncclCommInitRank(&h->rccl, world, u, rank));
  h->rccl_world = world;
  h->rccl_rank = rank;
  return CVAE_OK;
}

int cvae_rccl_allreduce(cvae_handle* h, float* buf, int64_t count, void* stream) {
  if (!h || (!buf && count > 0) || count < 0) return fail(CVAE_E_INVALID, "null argument or negative count");
  if (!h->rccl) return fail(CVAE_E_INVALID, "cvae_rccl_init first");
  if (count == 0) return CVAE_OK;
  RCCLCK(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, h->rccl, (hipStream_t)stream));
  return CVAE_OK;
}

int cvae_rccl_close(cvae_handle* h) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  if (h->rccl) {
    (void)hipSetDevice(h->device);
    (void)ncclCommDestroy(h->rccl);
    h->rccl = nullptr;
  }
  h->rccl_world = h->rccl_rank = 0;
  return CVAE_OK;
}

int cvae_tap_outputs(cvae_handle* h, float* recon, float* mu, float* logvar) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  if ((recon || mu || logvar) && !h->ring)
    return fail(CVAE_E_INVALID, "cvae_tap_outputs: the outputs are tapped from the ring chain only "
                                "(the reference architecture at S=100, D=6, bf16)");
  h->tap[0] = recon;
  h->tap[1] = mu;
  h->tap[2] = logvar;
  return CVAE_OK;
}

namespace {
// Σ over the 8-B words w_i of the operand copies of splitmix64(w_i ^ i·φ) (mod 2^64): order-free,
// so the block sums may meet in any order, and any change of any word moves it
__global__ __launch_bounds__(256) void checksum_kernel(const uint64_t* __restrict__ w, int64_t n,
                                                      unsigned long long* out) {
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t z = w[i] ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    s += z ^ (z >> 31);
  }
  for (int k = 32; k > 0; k >>= 1) s += __shfl_xor(s, k, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}
}  // namespace

int cvae_operand_checksum(cvae_handle* h, uint64_t* out, void* stream) {
  if (!h || !out) return fail(CVAE_E_INVALID, "null argument");
  hipStream_t s = (hipStream_t)stream;
  // the operand copies (Wf, Wb of every layer, padding included) and the padded biases: the arena's
  // head up to the end of the bias block (alloc_arena)
  const int64_t bytes = (const char*)(h->net.bias_all + h->net.nbias) - h->arena;
  HIPCK(hipMemsetAsync(out, 0, sizeof(uint64_t), s));
  hipLaunchKernelGGL(checksum_kernel, dim3(64), dim3(256), 0, s, (const uint64_t*)h->arena, bytes / 8,
                     (unsigned long long*)out);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_read_activation(cvae_handle* h, int layer, int which, int rows, void* dst, int* features, void* stream) {
  if (!h || layer < 0 || layer >= h->net.n_layers || (which != 0 && which != 1) || rows < 0)
    return fail(CVAE_E_INVALID, "bad argument");
  const LayerDev& L = h->net.L[layer];
  const int kf = which ? L.Np : L.Kp;
  if (features) *features = kf;
  if (!dst) return CVAE_OK;
  const int r16 = rup_i(rows, 16);
  if (r16 > h->net.Bp) return fail(CVAE_E_CAPACITY, "rows beyond the arena's row capacity");
  HIPCK(hipMemcpyAsync(dst, which ? L.gT : L.xT, (size_t)r16 * kf * h->tsize, hipMemcpyDeviceToDevice,
                       (hipStream_t)stream));
  return CVAE_OK;
}

int cvae_fault(const cvae_handle* h, unsigned* word) {
  if (!h || !word) return fail(CVAE_E_INVALID, "null argument");
  *word = h->fault_host ? __atomic_load_n(h->fault_host, __ATOMIC_ACQUIRE) : 0u;
  return CVAE_OK;
}

int cvae_clear_fault(cvae_handle* h) {
  if (!h) return fail(CVAE_E_INVALID, "null argument");
  if (h->fault_host) __atomic_store_n(h->fault_host, 0u, __ATOMIC_RELEASE);
  return CVAE_OK;
}

int cvae_loss(const float* recon, const float* x, const float* mu, const float* logvar, int batch, int seq_len,
              int dim, int latent_dim, const cvae_loss_weights* w, float* loss_out, float* workspace,
              void* stream) {
  if (!recon || !x || !mu || !logvar || !loss_out || !workspace || !w)
    return fail(CVAE_E_INVALID, "null argument");
  if (batch < 1 || seq_len < 1 || dim < 3 || latent_dim < 1) return fail(CVAE_E_INVALID, "bad shape");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (batch + 31) / 32;
  hipLaunchKernelGGL(loss_partial_kernel, dim3(nb), dim3(CVAE_THREADS), 0, s, recon, x, mu, logvar, batch, seq_len,
                     dim, latent_dim, workspace);
  HIPCK(hipGetLastError());
  LossArgs la{};
  la.partials = workspace; la.ntiles = nb; la.batch = batch;
  la.w_recon = w->recon; la.w_kld = w->kld; la.w_start = w->start; la.w_time = w->time;
  la.loss_out = loss_out;
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(64), 0, s, la, seq_len, dim, latent_dim);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_loss_backward(const float* recon, const float* x, const float* mu, const float* logvar, int batch,
                       int seq_len, int dim, int latent_dim, const cvae_loss_weights* w, const float* g_out,
                       float* d_recon, float* d_mu, float* d_logvar, void* stream) {
  if (!recon || !x || !mu || !logvar || !w || !g_out || !d_recon || !d_mu || !d_logvar)
    return fail(CVAE_E_INVALID, "null argument");
  if (batch < 1 || seq_len < 1 || dim < 3 || latent_dim < 1) return fail(CVAE_E_INVALID, "bad shape");
  const int64_t n = (int64_t)batch * (seq_len * dim + latent_dim);
  const int grid = (int)std::min<int64_t>((n + CVAE_THREADS - 1) / CVAE_THREADS, 4096);
  hipLaunchKernelGGL(loss_backward_kernel, dim3(grid), dim3(CVAE_THREADS), 0, (hipStream_t)stream, recon, x, mu,
                     logvar, batch, seq_len, dim, latent_dim, *w, g_out, d_recon, d_mu, d_logvar);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_adam_scalars(const cvae_adam_config* adam, int64_t n, float* out, void* stream) {
  int rc = check_adam(adam);
  if (rc) return rc;
  if (!out || n < 1) return fail(CVAE_E_INVALID, "bad argument");
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(adam_scalars_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, adam->lr, adam->beta1,
                     adam->beta2, n, out);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_extract_trajectories(const double* cols, int64_t n_rows, const int64_t* file_offsets, int n_files,
                              int scene, int target_points, int point_mode, double time_interval, double* out,
                              int32_t* valid, void* stream) {
  if (n_files < 0 || n_rows < 0) return fail(CVAE_E_INVALID, "bad size");
  if (n_files == 0) return CVAE_OK;
  if (!cols || !file_offsets || !out || !valid) return fail(CVAE_E_INVALID, "null argument");
  if (scene < CVAE_SCENE_STATIC || scene > CVAE_SCENE_UNPREDICTABLE) return fail(CVAE_E_INVALID, "bad scene");
  if (target_points < 2 || (point_mode != 0 && point_mode != 1)) return fail(CVAE_E_INVALID, "bad resampling");
  hipLaunchKernelGGL(extract_kernel, dim3(n_files), dim3(EX_THREADS), 0, (hipStream_t)stream, cols, n_rows,
                     file_offsets, scene, target_points, point_mode, time_interval, out, (int*)valid);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_mpc_default_config(cvae_mpc_config* cfg) {
  if (!cfg) return fail(CVAE_E_INVALID, "null argument");
  cfg->wheelbase = 2.8; cfg->max_steer = 0.5; cfg->max_accel = 7.0; cfg->dt = 0.01;
  cfg->q_theta = 20.0; cfg->q_v = 5.0; cfg->qf_theta = 20.0; cfg->qf_v = 5.0; cfg->r_accel = 1.0; cfg->r_steer = 50.0;
  cfg->tol = 1e-10;
  cfg->prediction_horizon = 10; cfg->control_horizon = 5; cfg->max_iter = 50; cfg->reserved = 0;
  return CVAE_OK;
}

static int mpc_cfg(const cvae_mpc_config* in, MpcCfg* c) {
  if (!in) return fail(CVAE_E_INVALID, "null config");
  if (in->prediction_horizon < 1 || in->prediction_horizon > MPC_MAXH)
    return fail(CVAE_E_INVALID, "prediction_horizon must be in [1, 63]");
  if (in->control_horizon < 1 || in->control_horizon > MPC_MAXCH || in->control_horizon > in->prediction_horizon)
    return fail(CVAE_E_INVALID, "control_horizon must be in [1, min(prediction_horizon, 32)]");
  if (!(in->dt > 0.0) || !(in->wheelbase > 0.0) || !(in->max_steer >= 0.0) || !(in->max_accel >= 0.0) ||
      in->max_iter < 0 || !(in->tol >= 0.0))
    return fail(CVAE_E_INVALID, "bad MPC parameter");
  c->L = in->wheelbase; c->max_steer = in->max_steer; c->max_accel = in->max_accel; c->dt = in->dt;
  c->q_th = in->q_theta; c->q_v = in->q_v; c->qf_th = in->qf_theta; c->qf_v = in->qf_v;
  c->r_a = in->r_accel; c->r_d = in->r_steer; c->tol = in->tol;
  c->N = in->prediction_horizon; c->CH = in->control_horizon; c->max_iter = in->max_iter; c->pad_ = 0;
  return CVAE_OK;
}

static size_t mpc_spline_bytes() { return (sizeof(MpcSpline) + 7) / 8 * 8; }

int cvae_mpc_track(const cvae_mpc_config* cfg, int n_paths, const double* waypoints, const int32_t* wp_offsets,
                   const double* initial_states, const int32_t* n_steps, const int64_t* step_offsets,
                   double* states, double* controls, int32_t* iters, void* stream) {
  MpcCfg c;
  int rc = mpc_cfg(cfg, &c);
  if (rc) return rc;
  if (n_paths < 0) return fail(CVAE_E_INVALID, "bad size");
  if (n_paths == 0) return CVAE_OK;
  if (!waypoints || !wp_offsets || !initial_states || !n_steps || !step_offsets || !states || !controls)
    return fail(CVAE_E_INVALID, "null argument");
  const size_t lds = mpc_spline_bytes() + mpc_ws_doubles(c.N, c.CH) * 8;
  HIPCK(hipFuncSetAttribute((const void*)mpc_track_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(mpc_track_kernel, dim3(n_paths), dim3(64), lds, (hipStream_t)stream, c, waypoints, wp_offsets,
                     initial_states, n_steps, step_offsets, states, controls, iters);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_mpc_solve(const cvae_mpc_config* cfg, int n, const double* state, const double* ref, const double* last,
                   double* u, double* cost, int32_t* iters, void* stream) {
  MpcCfg c;
  int rc = mpc_cfg(cfg, &c);
  if (rc) return rc;
  if (n < 0) return fail(CVAE_E_INVALID, "bad size");
  if (n == 0) return CVAE_OK;
  if (!state || !ref || !last || !u || !cost) return fail(CVAE_E_INVALID, "null argument");
  const size_t lds = mpc_ws_doubles(c.N, c.CH) * 8;
  HIPCK(hipFuncSetAttribute((const void*)mpc_solve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(mpc_solve_kernel, dim3(n), dim3(64), lds, (hipStream_t)stream, c, state, ref, last, u, cost,
                     iters);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

int cvae_mpc_reference(int n_paths, const double* waypoints, const int32_t* wp_offsets,
                       const double* initial_states, const double* t, int n_t, double* out, double* scalars,
                       void* stream) {
  if (n_paths < 0 || n_t < 0) return fail(CVAE_E_INVALID, "bad size");
  if (n_paths == 0) return CVAE_OK;
  if (!waypoints || !wp_offsets || !initial_states || (n_t && (!t || !out)) || !scalars)
    return fail(CVAE_E_INVALID, "null argument");
  const size_t lds = mpc_spline_bytes() + (size_t)4 * 5 * MPC_MAXWP * 8;
  HIPCK(hipFuncSetAttribute((const void*)mpc_reference_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds));
  hipLaunchKernelGGL(mpc_reference_kernel, dim3(n_paths), dim3(64), lds, (hipStream_t)stream, waypoints, wp_offsets,
                     initial_states, t, n_t, out, scalars);
  HIPCK(hipGetLastError());
  return CVAE_OK;
}

#if CVAE_DIAG_MPC
int cvae_diag_mpc_prof(unsigned long long* host8) {
  HIPCK(hipDeviceSynchronize());
  HIPCK(hipMemcpyFromSymbol(host8, HIP_SYMBOL(mpc_prof), 8 * sizeof(unsigned long long)));
  unsigned long long z[8] = {0};
  HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(mpc_prof), z, sizeof(z)));
  return CVAE_OK;
}
#endif

#if CVAE_DIAG_SUB
int cvae_diag_set_sub(unsigned long long* dev_buf) {
  HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(g_sub), &dev_buf, sizeof(dev_buf)));
  return CVAE_OK;
}
#endif

#if CVAE_DIAG_STAMPS
// diagnostic builds only: per-block step stamps (s_memrealtime, 100 MHz) of the next launches
int cvae_diag_set_stamps(cvae_handle* h, unsigned long long* dev_buf) {
  h->d_stamps = dev_buf;
  return CVAE_OK;
}
int cvae_diag_set_wstamps(unsigned long long* dev_buf) {
  HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(g_wstamps), &dev_buf, sizeof(dev_buf)));
  return CVAE_OK;
}
#endif

int cvae_set_timing(cvae_handle* h, int enabled) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  h->timing = enabled != 0;
  h->segs.clear();
  h->n_used = 0;
  h->pending = nullptr;
  return CVAE_OK;
}

int cvae_kernel_times(cvae_handle* h, char* names, int names_len, float* ms, int max_n) {
  if (!h) return fail(CVAE_E_INVALID, "null handle");
  std::vector<std::string> keys;
  std::vector<double> tot;
  std::vector<int> cnt;
  for (const auto& sg : h->segs) {
    if (sg.e1 < 0) continue;
    float t = 0.f;
    HIPCK(hipEventElapsedTime(&t, h->pool[sg.e0], h->pool[sg.e1]));
    size_t k = 0;
    while (k < keys.size() && keys[k] != sg.name) ++k;
    if (k == keys.size()) { keys.push_back(sg.name); tot.push_back(0.0); cnt.push_back(0); }
    tot[k] += t;
    cnt[k] += 1;
  }
  std::string all;
  int n = 0;
  for (size_t k = 0; k < keys.size() && n < max_n; ++k, ++n) {
    if (ms) ms[n] = (float)(tot[k] / cnt[k]);
    if (!all.empty()) all += ",";
    all += keys[k] + ":" + std::to_string(cnt[k]);
  }
  if (names && names_len > 0) {
    std::strncpy(names, all.c_str(), names_len - 1);
    names[names_len - 1] = 0;
  }
  return n;
}

}  // extern "C"
