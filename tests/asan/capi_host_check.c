/* Host-side check of the C-ABI under AddressSanitizer ("-fsanitize=address host build of
 * the C-ABI shim").  Linked against a build of csrc/cvae_capi.hip whose HOST code is compiled with
 * -fsanitize=address (cvae_amd._build.build_asan; the gfx950 device code is not instrumented, and
 * nothing here launches a kernel); drives every entry point's host logic that runs without a GPU —
 * the planner (build_plan: layer table, tile lists, LDS budget) over the BASELINE shapes and
 * invalid ones, argument validation of every handle call with NULL / bad arguments, the error
 * strings, and cvae_create's failure path (no device here) that must free what it allocated.
 * Exit status 0 = every expectation held; ASan aborts the process on any memory error. */
#include <stdio.h>
#include <string.h>

#include "../../include/cvae.h"

static int fails = 0;
#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                      \
    }                                                               \
  } while (0)

static cvae_config cfg(int S, int D, int Z, int H, int ne, int nd, int dt, int B, int nc, int cd) {
  cvae_config c;
  c.seq_len = S; c.dim = D; c.latent_dim = Z; c.hidden_dim = H; c.n_enc = ne; c.n_dec = nd;
  c.dtype = dt; c.max_batch = B; c.n_classes = nc; c.class_dim = cd;
  return c;
}

int main(void) {
  EXPECT(cvae_abi_version() == CVAE_ABI_VERSION);
  /* the planner over the BASELINE configurations (Training_VAE.py:124-167 shapes) */
  const cvae_config good[] = {
      cfg(10, 3, 8, 128, 4, 4, CVAE_F32, 32, 0, 0),     /* cfg1 */
      cfg(100, 6, 8, 128, 4, 4, CVAE_BF16, 1024, 0, 0), /* cfg2 */
      cfg(100, 6, 8, 128, 4, 4, CVAE_BF16, 65536, 0, 0),
      cfg(100, 6, 8, 128, 4, 4, CVAE_BF16, 1024, 4, 16), /* cfg4 */
      cfg(200, 6, 512, 128, 8, 8, CVAE_BF16, 1024, 0, 0), /* cfg5 */
      cfg(200, 6, 512, 128, 8, 8, CVAE_FP8, 1024, 0, 0),
      cfg(10, 3, 8, 16, 4, 4, CVAE_F32, 8, 0, 0), /* every dimension padded */
      cfg(37, 5, 12, 64, 2, 3, CVAE_BF16, 77, 0, 0),
  };
  const long long want_params[] = {128942, 275432, 275432, -1, -1, -1, -1, -1};
  for (unsigned i = 0; i < sizeof(good) / sizeof(good[0]); ++i) {
    int64_t n = 0;
    int nt = 0, lds = 0;
    EXPECT(cvae_config_info(&good[i], &n, &nt, &lds) == CVAE_OK);
    /* 2 tensors per Linear, fc = fc_mu + fc_logvar, the class table (no bias) last */
    const cvae_config* g = &good[i];
    EXPECT(nt == 2 * (3 + g->n_enc + g->n_dec) + 2 + (g->n_classes > 0 ? 1 : 0));
    EXPECT(n > 0 && lds > 0 && lds <= 163840);
    if (want_params[i] > 0) EXPECT(n == want_params[i]);
  }
  /* invalid configurations: a negative code and a message, no crash */
  const cvae_config bad[] = {
      cfg(10, 2, 8, 128, 4, 4, CVAE_F32, 32, 0, 0),   /* dim < 3 */
      cfg(10, 3, 6, 128, 4, 4, CVAE_F32, 32, 0, 0),   /* latent not a multiple of 4 */
      cfg(10, 3, 8, 128, 4, 4, CVAE_F32, 32, 3, 6),   /* class_dim not a multiple of 4 */
      cfg(4000, 6, 8, 128, 4, 4, CVAE_F32, 32, 0, 0), /* tile state beyond 160 KiB of LDS */
      cfg(10, 3, 8, 128, 40, 40, CVAE_F32, 32, 0, 0), /* too many layers */
  };
  for (unsigned i = 0; i < sizeof(bad) / sizeof(bad[0]); ++i) {
    int64_t n = 0;
    int nt = 0, lds = 0;
    EXPECT(cvae_config_info(&bad[i], &n, &nt, &lds) < 0);
    EXPECT(strlen(cvae_last_error()) > 0);
  }
  EXPECT(cvae_config_info(NULL, NULL, NULL, NULL) == CVAE_E_INVALID);
  /* cvae_create: invalid configurations are refused before any device call; a valid one fails on
   * this GPU-less host (or succeeds on a GPU host: then destroy it) */
  cvae_handle* h = NULL;
  cvae_config c = cfg(0, 6, 8, 128, 4, 4, CVAE_BF16, 1024, 0, 0);
  EXPECT(cvae_create(&c, 0, &h) == CVAE_E_INVALID && h == NULL);
  c = good[1];
  c.dtype = 7;
  EXPECT(cvae_create(&c, 0, &h) == CVAE_E_INVALID && h == NULL);
  EXPECT(cvae_create(NULL, 0, &h) == CVAE_E_INVALID);
  int rc = cvae_create(&good[1], 0, &h);
  if (rc == CVAE_OK) cvae_destroy(h);
  else EXPECT(h == NULL && strlen(cvae_last_error()) > 0);
  EXPECT(cvae_destroy(NULL) == CVAE_OK);
  /* argument validation of the handle calls (NULL handle / outputs) */
  int64_t i64 = 0;
  int i32 = 0;
  unsigned u = 0;
  uint64_t u64[4];
  EXPECT(cvae_num_params(NULL, &i64, &i32) < 0);
  EXPECT(cvae_param_info(NULL, 0, &i64, &i64, &i32, &i32) < 0);
  EXPECT(cvae_workspace_bytes(NULL, &i64) < 0);
  EXPECT(cvae_bucket_split(NULL, &i64) < 0);
  EXPECT(cvae_train_kernel(NULL, &i32) < 0);
  EXPECT(cvae_pack_weights(NULL, NULL, NULL) < 0);
  EXPECT(cvae_fault(NULL, &u) < 0);
  EXPECT(cvae_clear_fault(NULL) < 0);
  EXPECT(cvae_tap_outputs(NULL, NULL, NULL, NULL) < 0);
  EXPECT(cvae_operand_checksum(NULL, NULL, NULL) < 0);
  EXPECT(cvae_px_export(NULL, 2, 0, NULL) < 0);
  EXPECT(cvae_px_import(NULL, NULL, 0) < 0);
  EXPECT(cvae_px_layout(NULL, &i32, &i32) < 0);
  EXPECT(cvae_px_reset(NULL, 0) < 0);
  EXPECT(cvae_px_stats(NULL, u64, 0) < 0);
  EXPECT(cvae_px_probe(NULL, &i32) < 0);
  EXPECT(cvae_px_close(NULL) < 0);
  EXPECT(cvae_px_owned(NULL, NULL) < 0);
  EXPECT(cvae_set_timing(NULL, 1) < 0);
  EXPECT(cvae_px_blob_bytes(&i64) == CVAE_OK && i64 > 0 && i64 < 4096);
  EXPECT(cvae_px_blob_bytes(NULL) < 0);
  cvae_adam_config a = {1e-3, 0.9, 0.999, 1e-8};
  EXPECT(cvae_step_skip(NULL, NULL, &a, NULL) < 0);
  EXPECT(cvae_adam_scalars(NULL, 4, NULL, NULL) < 0);
  /* the MPC configuration defaults (MPC_Tracking.py:26, :283-306) */
  cvae_mpc_config m;
  memset(&m, 0, sizeof(m));
  EXPECT(cvae_mpc_default_config(&m) == CVAE_OK);
  EXPECT(m.prediction_horizon == 10 && m.control_horizon == 5 && m.wheelbase == 2.8 && m.dt == 0.01);
  EXPECT(cvae_mpc_default_config(NULL) < 0);
  if (fails) {
    fprintf(stderr, "%d expectation(s) failed\n", fails);
    return 1;
  }
  printf("capi host check ok\n");
  return 0;
}
