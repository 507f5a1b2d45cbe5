// Device helpers of the two-stage MSE search shared by mse_search.hip (the per-launch
// search kernels) and thin_loop.hip (the persistent loop of the thin factors).
#pragma once
#include "quant_device.h"

namespace admmq {

// Closed form of level_threshold(s, k) (s > 0 normal, k >= 1): rint(fl(a/s)) >= k
// <=> fl(a/s) >= H with H = k - 1/2 (k even: rint(H) = k) or H = next float above
// k - 1/2 (k odd: the tie rounds down). fl(a/s) >= H <=> a/s >= m, the midpoint of
// H and the float below it, where a/s == m rounds to H iff H's last mantissa bit is
// 0 (round half to even). s * m is exact in fp64 (24 + 25 significant bits), so the
// threshold is the smallest float >= s m, one float higher on a tie that rounds
// down. Checked against level_threshold by admmq_debug_check_thresholds.
__device__ __forceinline__ float level_threshold_fast(float s, int k) {
  float H = (float)k - 0.5f;
  if (k & 1) H = __uint_as_float(__float_as_uint(H) + 1u);
  const float Hm = __uint_as_float(__float_as_uint(H) - 1u);
  const double m = 0.5 * ((double)H + (double)Hm);
  const double prod = (double)s * m;
  float a = (float)prod;                                   // round to nearest
  if ((double)a < prod) a = __uint_as_float(__float_as_uint(a) + 1u);
  else if ((double)a > prod) {                             // nearest went up: is the float below still >= prod?
    const float b = __uint_as_float(__float_as_uint(a) - 1u);
    if ((double)b >= prod) a = b;
  }
  if ((double)a == prod && (__float_as_uint(H) & 1u)) a = __uint_as_float(__float_as_uint(a) + 1u);
  return a;
}

// Threshold table of one job into LDS: thr[(k-1) n + c] = smallest a with
// |q_c(a)| >= k, for k = 1..qmax (increasing in c and in k).
__device__ __forceinline__ void fill_thresholds(float* thr, float mx, int n, int qmax, int nt) {
  const float den = (float)(2 * qmax - 1);
  for (int e = threadIdx.x; e < qmax * n; e += nt) {
    const int k = 1 + e / n, c = e - (k - 1) * n;
    thr[e] = level_threshold_fast((2.0f * cand_t(mx, c, n)) / den, k);
  }
}

__device__ __forceinline__ int hist_fixed_exp(float mx, long long nelem, int qmax) {
  int emx;
  (void)__builtin_frexpf(mx, &emx);
  const long long nterm = nelem * qmax;
  const int clt = 64 - __builtin_clzll((unsigned long long)(nterm > 1 ? nterm - 1 : 1));
  return 61 - emx - clt;
}

// Rigorous bounds of the stage-1 SSE model of one candidate: A(c) = S2 - 2 s T1 + s^2 T2
// (exact-arithmetic SSE from the level sums) and E(c), a bound on |canonical - A|
// (oracle/stage1_model.py); S = {c : A - E <= min(A + E)} holds the argmin.
struct SelCtx {
  double S2, fixu, u, Kterm, Nterm, tiny;
  float mx, denf;
  int n;
  __device__ void bounds(int c, unsigned long long T1i, unsigned long long T2i, double& lo, double& hi) const {
    bounds_s((double)((2.0f * cand_t(mx, c, n)) / denf), T1i, T2i, lo, hi);
  }
  // the same with the candidate's scale s_c = fl(2 t_c / den) already at hand
  __device__ void bounds_s(double s, unsigned long long T1i, unsigned long long T2i, double& lo, double& hi) const {
    const double T1 = (double)T1i * fixu;
    const double T2 = (double)T2i;
    const double A = S2 - 2.0 * s * T1 + s * s * T2;
    const double mag = S2 + 2.0 * s * T1 + s * s * T2;
    const double slack = 1e-10 * mag;
    const double sh = fmax(A, 0.0) + slack;
    const double B1 = 2.0 * u * (1.0 + u) * (s * sqrt(T2 * sh) + sh) + 2.0 * u * u * (1.0 + u) * (1.0 + u) * (s * s * T2 + sh);
    const double E = B1 + 3.0000002 * u * (sh + B1) + Kterm + 2.0 * s * Nterm * fixu + slack + tiny;
    lo = A - E;
    hi = A + E;
  }
};

// Stage 1 of one element x (a = |x|) into a block's level-sum bins (k_mse_hist and the
// thin-factor loop): level k is reached by candidate c iff a >= thr[k][c] (x > 0 reaches
// at most QMAX - 1 levels). Levels k <= kfull are reached by every candidate (summed in
// registers: full1 / full2, bin n); levels kfull < k <= k0 have a breakpoint b_k in
// [1, n-1] = #{c : level k reached}: a linear estimate from t_c ~ S0 + c step (off by at
// most one), checked against its two neighbouring thresholds (exact -> added at once;
// inactive lanes add 0 to their private dummy bin, no branch), else a rare binary search.
// h1[b] += to_fixed(a, K1), h2[b] += 2k - 1 per (level, breakpoint b); s2 += x^2.
template <int QMAX>
__device__ __forceinline__ void hist_insert_elem(float x, const float* thr, int n, float S0, float inv_step, int K1,
                                                 int dummy, const float* tlo0, const float* thin,
                                                 unsigned long long* h1, unsigned* h2, double& s2,
                                                 unsigned long long& full1, unsigned& full2) {
  s2 += (double)x * (double)x;
  const float a = __builtin_fabsf(x);
  const int cap = (x > 0.f) ? QMAX - 1 : QMAX;
  int k0 = 0, kfull = 0;
#pragma unroll
  for (int k = 1; k <= QMAX; ++k) {
    k0 += (k <= cap && a >= tlo0[k - 1]) ? 1 : 0;
    kfull += (k <= cap && a >= thin[k - 1]) ? 1 : 0;
  }
  if (x == 0.f) k0 = 0;
  const unsigned long long af = to_fixed(a, K1);
  full1 += af * (unsigned long long)kfull;
  full2 += (unsigned)(kfull * kfull);              // sum_{k<=kfull} (2k-1)
  unsigned slow = 0u;
  if constexpr (QMAX <= 8) {
    // every level's estimate and its two neighbouring thresholds first, so the 2 QMAX LDS
    // reads are in flight together (read at their compare, each was waited for on its
    // own), then the compares, then the adds (QMAX = 16 keeps the per-level form: the
    // batched form's 32 reads spill in the thin loop)
    int bk[QMAX];
    float tlo[QMAX], thi[QMAX];
#pragma unroll
    for (int k = 1; k <= QMAX; ++k) {
      const float tau = a * ((float)(2 * QMAX - 1) / (float)(2 * k - 1));   // estimate only
      const float ce = (tau - S0) * inv_step;
      int b = (ce >= (float)(n - 1)) ? n - 1 : (ce < 0.f ? 1 : (int)ce + 1);
      b = max(min(b, n - 1), 1);
      bk[k - 1] = b;
      const float* tk = thr + (k - 1) * n;
      tlo[k - 1] = tk[b - 1];
      thi[k - 1] = tk[b];
    }
#pragma unroll
    for (int k = 1; k <= QMAX; ++k) {
      const bool act = (k > kfull && k <= k0);
      const bool exact = (a >= tlo[k - 1]) && (a < thi[k - 1]);
      slow |= (act && !exact) ? (1u << k) : 0u;
      // only the lanes whose level k is active add (1-2 of the QMAX levels of an
      // element): the masked-off lanes cost no LDS atomic
      if (act && exact) {
        atomicAdd(&h1[bk[k - 1]], af);
        atomicAdd(&h2[bk[k - 1]], (unsigned)(2 * k - 1));
      }
    }
  } else {
#pragma unroll
    for (int k = 1; k <= QMAX; ++k) {
      const bool act = (k > kfull && k <= k0);
      const float tau = a * ((float)(2 * QMAX - 1) / (float)(2 * k - 1));   // estimate only
      const float ce = (tau - S0) * inv_step;
      int b = (ce >= (float)(n - 1)) ? n - 1 : (ce < 0.f ? 1 : (int)ce + 1);
      b = max(min(b, n - 1), 1);
      const float* tk = thr + (k - 1) * n;
      const bool exact = (a >= tk[b - 1]) && (a < tk[b]);
      slow |= (act && !exact) ? (1u << k) : 0u;
      if (act && exact) {
        atomicAdd(&h1[b], af);
        atomicAdd(&h2[b], (unsigned)(2 * k - 1));
      }
    }
  }
  (void)dummy;
  if (slow) {   // rare: exact breakpoint by binary search (largest b with thr[k][b-1] <= a)
#pragma unroll 1
    for (int k = 1; k <= QMAX; ++k) {
      if (!((slow >> k) & 1u)) continue;
      const float* tk = thr + (k - 1) * n;
      int lo = 1, hi = n - 1;   // a >= tk[0] and a < tk[n-1]: answer in [1, n-1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a >= tk[mid - 1]) lo = mid; else hi = mid - 1;
      }
      atomicAdd(&h1[lo], af);
      atomicAdd(&h2[lo], (unsigned)(2 * k - 1));
    }
  }
}

}  // namespace admmq
