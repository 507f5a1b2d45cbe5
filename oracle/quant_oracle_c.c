/* ORACLE — test infrastructure only (never linked into the product path).
 *
 * C restatement of oracle/quant_oracle.py's MSE-minmax candidate search, for
 * full-size parity checks (a 11008 x 1492 Llama factor is 3.3 G candidate-elements:
 * minutes in numpy, about a second here with OpenMP). Every function follows the
 * numpy restatement line by line, which in turn restates the reference:
 *
 *   candidate grid      source/quantization.py:130 (torch.linspace, pinned by F5)
 *   _quantize           source/quantization.py:123-126
 *   mse + argmin        source/quantization.py:136-141
 *
 * Two argmin rules are exposed:
 *   rule 0  canonical fixed-point SSE (uint64 sums of floor(g 2^K) per quad), first
 *           index on ties - the rule of quant_oracle.py and of the HIP kernels in
 *           round 1;
 *   rule 1  the same sums converted to the reference's float32 mean
 *           (fl32(fl32(S) / fl32(n)), S = sse 2^-K; source/quantization.py:138 is
 *           torch's CPU sum followed by one division), first index on ties of those
 *           float32 values (torch.argmin over the float32 `mses`).
 * Pinned against the numpy oracle and the reference fixtures by
 * tests/test_oracle_c.py. Build: oracle/Makefile (gcc; -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float cand_t(float mx, int c, int n) {
  const float s = (float)(0.2 * (double)mx);
  const float e = (float)(1.2 * (double)mx);
  if (n == 1) return s;
  const float step = (e - s) / (float)(n - 1);
  if (c < n / 2) return fmaf(step, (float)c, s);
  return fmaf(-step, (float)(n - 1 - c), e);
}

static int fixed_exponent(float mx, int64_t nq) {
  int e;
  (void)frexp((double)mx, &e);
  int bl = 0;
  uint64_t v = nq > 1 ? (uint64_t)(nq - 1) : 0;
  while (v) { ++bl; v >>= 1; }
  return 56 - bl - 2 * e;
}

static float qround(float x, float scale, float qlo, float qhi) {
  float q = rintf(x / scale);
  if (q != q) return q;
  if (q < qlo) q = qlo;
  if (q > qhi) q = qhi;
  return q;
}

/* max(|min x|, |max x|) as the reference computes it (NaN propagates). */
float oq_absmax(const float* x, int64_t n) {
  if (n <= 0) return 0.f;
  float mn = x[0], mxv = x[0];
  int nan = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float v = x[i];
    if (v != v) nan = 1;
    if (v < mn) mn = v;
    if (v > mxv) mxv = v;
  }
  if (nan) return NAN;
  const float a = fabsf(mn), b = fabsf(mxv);
  return a > b ? a : b;
}

/* Canonical SSE table of x viewed as (rows, cols), quads of 4 consecutive row
 * elements (last quad zero padded). Returns the fixed-point exponent K; grid_out
 * (may be NULL) receives the candidates. */
int oq_sse_table(const float* x, int64_t rows, int64_t cols, int bits, int ncand, uint64_t* sse_out,
                 float* grid_out, float* mx_out) {
  const int64_t qpr = (cols + 3) / 4;
  const int64_t nq = rows * qpr;
  const float mx = oq_absmax(x, rows * cols);
  const int q = 1 << (bits - 1);
  const float den = (float)(2 * q - 1), qlo = (float)(-q), qhi = (float)(q - 1);
  const int K = fixed_exponent(mx, nq);
  const double sc = ldexp(1.0, K);
  if (mx_out) *mx_out = mx;
#pragma omp parallel for schedule(dynamic, 1)
  for (int c = 0; c < ncand; ++c) {
    const float t = cand_t(mx, c, ncand);
    if (grid_out) grid_out[c] = t;
    const float scale = (2.0f * t) / den;
    uint64_t acc = 0;
    for (int64_t r = 0; r < rows; ++r) {
      const float* xr = x + r * cols;
      for (int64_t k = 0; k < qpr; ++k) {
        float d2[4];
        for (int j = 0; j < 4; ++j) {
          const int64_t col = 4 * k + j;
          const float v = col < cols ? xr[col] : 0.f;
          const float qv = qround(v, scale, qlo, qhi);
          const float p = qv * scale;
          const float d = v - p;
          d2[j] = d * d;
        }
        const float a = d2[0] + d2[1];
        const float b = d2[2] + d2[3];
        const float g = a + b;
        acc += (uint64_t)floor((double)g * sc);
      }
    }
    sse_out[c] = acc;
  }
  return K;
}

/* float32 mean of candidate c under rule 1. */
static float rule1_mean(uint64_t sse, int K, int64_t n) {
  const float s = (float)ldexp((double)(float)sse, -K);   /* uint64 -> f32 (one rounding), exact scale */
  return s / (float)n;
}

/* Argmin of the table under `rule` (0 canonical integer, 1 float32 mean). */
int oq_argmin(const uint64_t* sse, int ncand, int rule, int K, int64_t nelem) {
  int best = 0;
  if (rule == 0) {
    for (int c = 1; c < ncand; ++c)
      if (sse[c] < sse[best]) best = c;
    return best;
  }
  float bm = rule1_mean(sse[0], K, nelem);
  for (int c = 1; c < ncand; ++c) {
    const float m = rule1_mean(sse[c], K, nelem);
    if (m < bm) { bm = m; best = c; }
  }
  return best;
}

/* quantize_tensor_mse (source/quantization.py:118-144) under `rule`; returns the
 * chosen candidate index (-1: degenerate range, every output NaN). */
int oq_quantize_mse(const float* x, int64_t rows, int64_t cols, int bits, int ncand, int rule, float* y) {
  const int64_t n = rows * cols;
  uint64_t* sse = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(ncand > 0 ? ncand : 1));
  float mx;
  const int K = oq_sse_table(x, rows, cols, bits, ncand, sse, NULL, &mx);
  int idx = -1;
  if (!(mx > 0.f && mx < INFINITY)) {
    for (int64_t i = 0; i < n; ++i) y[i] = NAN;
  } else {
    idx = oq_argmin(sse, ncand, rule, K, n);
    const int q = 1 << (bits - 1);
    const float den = (float)(2 * q - 1);
    const float scale = (2.0f * cand_t(mx, idx, ncand)) / den;
#pragma omp parallel for
    for (int64_t i = 0; i < n; ++i) y[i] = qround(x[i], scale, (float)(-q), (float)(q - 1)) * scale;
  }
  free(sse);
  return idx;
}
