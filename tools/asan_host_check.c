/* Host AddressSanitizer / UBSan check of libadmmq's host code (optional
 * -fsanitize=address host build). Built by `make -C admm-quantization_amd/csrc asan`
 * against build/asan/libadmmq_asan.so, whose host code is instrumented (-Xarch_host
 * -fsanitize=address,undefined; device code untouched). Runs without a GPU: it drives the
 * host-only planners (workspace-size queries: problem layout, tile lists and their CU
 * ordering, stage-1 chunking, the finalize / small-job plans) over the bench configs
 * C3 / C4 / C5 and seeded random batches, and the argument-validation error paths. Any
 * heap / stack overflow or UB in that code aborts with a sanitizer report.
 * usage: build/asan/asan_host_check   (exit 0 = clean) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/admmq.h"

static uint64_t rng = 88172645463325252ull;
static int rnd(int lo, int hi) { /* xorshift64, inclusive range */
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return lo + (int)(rng % (uint64_t)(hi - lo + 1));
}

static size_t ws_of(const int (*ir)[2], int n) {
  admmq_problem* p = calloc((size_t)n, sizeof(admmq_problem));
  for (int i = 0; i < n; ++i) { p[i].I = ir[i][0]; p[i].R = ir[i][1]; }
  size_t b = admmq_admm_workspace_size(p, n, 200);
  free(p);
  return b;
}

int main(void) {
  int fails = 0;
  /* C3: resnet18 16 3x3 convs, every mode (I_m, R) */
  static const int r18[16][3] = {{64, 64, 134}, {64, 64, 134}, {64, 64, 134}, {64, 64, 134}, {128, 64, 183},
                                 {128, 128, 278}, {128, 128, 278}, {128, 128, 278}, {256, 128, 375},
                                 {256, 256, 566}, {256, 256, 566}, {256, 256, 566}, {512, 256, 759},
                                 {512, 512, 1141}, {512, 512, 1141}, {512, 512, 1141}};
  for (int m = 0; m < 3; ++m) {
    int ir[16][2];
    for (int l = 0; l < 16; ++l) { ir[l][0] = m == 2 ? 9 : r18[l][m]; ir[l][1] = r18[l][2]; }
    size_t b = ws_of((const int(*)[2])ir, 16);
    printf("C3 mode %d: workspace %zu B\n", m, b);
    fails += b == 0;
  }
  /* C5: one Llama-7B decoder layer, both modes (the wide-tile plan) */
  static const int ll[7][3] = {{4096, 4096, 1024}, {4096, 4096, 1024}, {4096, 4096, 1024}, {4096, 4096, 1024},
                               {11008, 4096, 1492}, {11008, 4096, 1492}, {4096, 11008, 1492}};
  for (int m = 0; m < 2; ++m) {
    int ir[7][2];
    for (int l = 0; l < 7; ++l) { ir[l][0] = ll[l][m]; ir[l][1] = ll[l][2]; }
    size_t b = ws_of((const int(*)[2])ir, 7);
    printf("C5 mode %d: workspace %zu B\n", m, b);
    fails += b == 0;
  }
  /* seeded random batches: thin (I <= 16), 32-row, 64x64 and wide mixes, ragged R */
  size_t tot = 0;
  for (int t = 0; t < 400; ++t) {
    int n = rnd(1, 48), ir[48][2];
    for (int i = 0; i < n; ++i) {
      const int cls = rnd(0, 3);
      ir[i][0] = cls == 0 ? rnd(1, 16) : (cls == 1 ? rnd(17, 32) : (cls == 2 ? rnd(33, 700) : rnd(700, 4096)));
      ir[i][1] = rnd(1, t % 50 == 0 ? 3000 : 1200);
    }
    size_t b = ws_of((const int(*)[2])ir, n);
    fails += b == 0;
    tot += b;
  }
  printf("400 random batches: total workspace %zu B\n", tot);
  /* quantizer planner: ragged tensors */
  for (int t = 0; t < 200; ++t) {
    admmq_qtensor q[8] = {0};
    const int n = rnd(1, 8);
    for (int i = 0; i < n; ++i) { q[i].rows = rnd(1, 3000); q[i].cols = rnd(1, 3000); }
    fails += admmq_quantize_workspace_size(q, n, rnd(1, 400)) == 0;
  }
  /* argument validation: each must fail cleanly (no device call is reached) */
  admmq_problem bad = {0};
  bad.I = 0; bad.R = 5;
  fails += admmq_admm_workspace_size(&bad, 1, 200) != 0;
  bad.I = 5; bad.R = -1;
  fails += admmq_admm_workspace_size(&bad, 1, 200) != 0;
  bad.I = 1 << 16; bad.R = 1 << 15;
  fails += admmq_admm_workspace_size(&bad, 1, 200) != 0;
  fails += admmq_admm_workspace_size(NULL, 3, 200) != 0;
  bad.I = 8; bad.R = 8;
  fails += admmq_admm_workspace_size(&bad, 1, 0) != 0;
  fails += admmq_admm_prepare(&bad, 1, 200, NULL, 0, NULL) == ADMMQ_OK;
  fails += admmq_quantize_batched(NULL, 1, 4, 99, 200, NULL, 0, NULL) != ADMMQ_ERR_SCHEME;
  printf("last error: %s\n", admmq_last_error());
  printf("%s (%d failures)\n", fails ? "FAIL" : "OK", fails);
  return fails ? 1 : 0;
}
