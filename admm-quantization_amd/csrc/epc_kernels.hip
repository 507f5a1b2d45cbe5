// The EPC step's Lagrange multiplier on the device (cp_anc, source/parafac_epc.py:61-74;
// admmq.parafac_epc): the scalar root search that ran on the host after every mode step's
// R x R eigendecomposition, with two host synchronisations per step.
#include <cmath>
#include <cstdint>

#include "../../include/admmq.h"
#include "admmq_internal.h"

namespace admmq {

// The root mu >= 0 of normY2 - sum_i c_i (s_i + 2 mu) / (s_i + mu)^2 = delta2 by doubling
// the bracket from max(s) and 200 bisection steps to fp64 resolution; the sum over i in a
// fixed order (thread-strided partials, then the 4 waves' sums in order). One workgroup:
// the host no longer waits for c and s every mode step.
__device__ double epc_err(const double* c, const double* sv, int n, double mu, double normY2, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double acc = 0.0;
  for (int i = tid; i < n; i += 256) {
    const double d = sv[i] + mu;
    acc += c[i] * (sv[i] + 2.0 * mu) / (d * d);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __syncthreads();   // red reused across calls
  if (lane == 0) red[w] = acc;
  __syncthreads();
  return normY2 - (((red[0] + red[1]) + red[2]) + red[3]);
}

__global__ __launch_bounds__(256) void k_epc_mu(const double* __restrict__ c, const double* __restrict__ sv, int n,
                                                double normY2, double delta2, double* __restrict__ mu_out) {
  __shared__ double red[4];
  __shared__ double smax[4];
  double mx = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) mx = fmax(mx, sv[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmax(fmax(smax[0], smax[1]), fmax(smax[2], smax[3]));
  double result = 0.0;
  if (!(epc_err(c, sv, n, 0.0, normY2, red) >= delta2)) {
    double hi = fmax(mx, 1e-300);
    while (epc_err(c, sv, n, hi, normY2, red) < delta2 && hi < 1e300) hi *= 2.0;
    double lo = 0.0;
    for (int it = 0; it < 200; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (mid <= lo || mid >= hi) break;
      if (epc_err(c, sv, n, mid, normY2, red) < delta2) lo = mid;
      else hi = mid;
    }
    result = lo;
  }
  if (threadIdx.x == 0) *mu_out = result;
}

// ---------------------------------------------------------------------------
// The R x R normal-equation solves of the CP-ALS / EPC initialiser on one workgroup
// (n <= kSpdSmallMax: the fp64 matrix in LDS), replacing tensorly parafac's solve and
// cp_anc's eigendecomposition (source/parafac_epc.py:42, :61-74; admmq.parafac_epc):
//
//   k_spd_solve64   X = F G^-1 (the CP-ALS update U_m = F G^-1, G = Hadamard of the Grams);
//   k_epc_step64    X = F (G + mu I)^-1 with mu >= 0 the root of the EPC error equation
//                   e(mu) = ||Y||^2 - <F, X> - mu ||X||^2 = delta^2 (the eigen form's
//                   ||Y||^2 - sum_j c_j (s_j + 2 mu) / (s_j + mu)^2 with G = V diag(s) V^T,
//                   c_j = |F v_j|^2), found by Newton steps on e, e'(mu) = 2 mu ||X L^-T||^2,
//                   safeguarded by the bracket [lo, hi] (bisection / doubling), each from a
//                   fresh Cholesky of G + mu I; mu = 0 when e(0) >= delta^2 already (the LS
//                   step keeps the error).
//
// The inverse (G + shift I)^-1 in LDS by blocked Gauss-Jordan without pivoting (G + shift I
// SPD: positive pivots), then the right-hand sides as one dense product X = F (G + shift I)^-1.
// At this size a factorization's time is its sequential depth, not its arithmetic: a
// column-at-a-time Cholesky plus two triangular solves per right-hand side made 3 n dependent
// steps (~0.5 ms at n = 134); Gauss-Jordan on 8 x 8 pivot blocks has n / 8 steps of four
// workgroup barriers, each step a rank-8 update of the whole matrix, and the products have
// no sequential chain at all.
//   pivot block  wave 0 inverts P = A[kb][kb] in registers (lane = row, v_readlane for the
//                pivot row) into sP;
//   row block    B' = P^-1 A[kb][j] for the columns j outside kb (loads, barrier, stores);
//   the rest     A[i][j] -= A[i][kb] B'[kb][j] and A[i][kb] <- -A[i][kb] P^-1 for every row i
//                outside kb (a wave per row, lanes on columns; each row's loads before its
//                stores), then A[kb][kb] <- P^-1.
// Rows are lda = n + 1 doubles apart.
constexpr int kSpdSmallMax = 136;   // 136 rows of 137 doubles (146 KB) + the pivot-block scratch
constexpr int kSpdThreads = 1024;
constexpr int kGJ = 8;              // pivot block
constexpr int kSpdCols = 16;        // lanes per right-hand-side row in the products (a DPP row)
constexpr int kSpdRowsPerPass = kSpdThreads / kSpdCols;   // 64 rows at a time
constexpr int kSpdPer = (kSpdSmallMax + kSpdCols - 1) / kSpdCols;   // columns per lane (9)
__host__ __device__ inline int spd_lda(int n) { return n + 1; }

// Diagnostics (make TRACE=1; admmq_debug_spd_trace): s_memrealtime at {start, G in LDS,
// inverse done, products done} of the last k_spd_solve64
__device__ unsigned long long g_spd_trace[16];   // [4 + k]: s_memtime (shader clocks) at the same points; [8 + k]: inverse phase sums
#define ADMMQ_SPD_STAMP(k)                                         \
  if (ADMMQ_TRACE && threadIdx.x == 0) {                           \
    g_spd_trace[k] = ADMMQ_NOW();                                  \
    g_spd_trace[4 + (k)] = __builtin_amdgcn_s_memtime();           \
  }

__device__ __forceinline__ double readlane_f64(double v, int src) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// A <- (G + shift I)^-1 (full n x n, row stride spd_lda(n)); sP: kGJ x kGJ doubles, Cb: n x kGJ
// doubles of LDS. false (uniform over the workgroup) if a pivot is not positive and finite.
// A block step (pivot rows / columns kb = [p, p + pb)), three workgroup barriers:
//   1. wave 0: P^-1 (P = A[kb][kb]) by Gauss-Jordan in registers (lane = row) into sP; the
//      others copy the column block A[:][kb] into Cb;
//   2. thread (row group g, column j): B'[.][j] = P^-1 A[kb][j] in registers (its column of
//      the new row block, computed by each of the 8 row groups that update column j);
//   3. the row block's new values written (g = 0), and for every row i = g (mod 8) outside
//      kb: A[i][j] -= Cb[i][.] B'[.][j] (j outside kb), A[i][j] = -(Cb[i][.] P^-1)[j - p]
//      (j in kb); A[kb][kb] <- P^-1.
template <int NT>
__device__ __forceinline__ bool spd_inverse_lds(const double* __restrict__ G, int n, double shift, double* A,
                                                double* sP, double* Cb) {
  constexpr int kRG = NT / 128;   // row groups
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lda = spd_lda(n);
  const int g = tid >> 7, js = tid & 127;   // NT / 128 row groups x 128 column slots (columns js, js + 128)
  __shared__ int s_bad;
  for (int e = tid; e < n * n; e += NT) {
    const int i = e / n, k = e - i * n;
    A[i * lda + k] = G[e] + (i == k ? shift : 0.0);
  }
  if (tid == 0) s_bad = 0;
  __syncthreads();
  ADMMQ_SPD_STAMP(1);
  unsigned long long ph[4] = {0ull, 0ull, 0ull, 0ull}, tp = ADMMQ_NOW();
#define ADMMQ_GJ_PH(k)                                \
  if (ADMMQ_TRACE) {                                  \
    const unsigned long long tn_ = ADMMQ_NOW();       \
    ph[k] += tn_ - tp;                                \
    tp = tn_;                                         \
  }
  for (int p = 0; p < n; p += kGJ) {
    const int pb = min(kGJ, n - p);
    if (w == 0) {   // P^-1 by Gauss-Jordan in registers: lane r < pb holds row r of P
      double pr[kGJ];
#pragma unroll
      for (int t = 0; t < kGJ; ++t) pr[t] = (lane < pb && t < pb) ? A[(p + lane) * lda + p + t] : (lane == t ? 1.0 : 0.0);
      int bad = 0;
#pragma unroll
      for (int t = 0; t < kGJ; ++t) {
        if (t < pb) {
          const double piv = __shfl(pr[t], t, 64);
          if (!(piv > 0.0) || !(piv < __builtin_huge_val())) bad = 1;
          const double ip = 1.0 / piv;
          double rt[kGJ];   // pivot row, scaled (its pivot entry 1 / piv)
#pragma unroll
          for (int u = 0; u < kGJ; ++u) rt[u] = u == t ? ip : __shfl(pr[u], t, 64) * ip;
          const double f = pr[t];
#pragma unroll
          for (int u = 0; u < kGJ; ++u) {
            if (lane == t) pr[u] = rt[u];
            else pr[u] = u == t ? -f * ip : pr[u] - f * rt[u];
          }
        }
      }
      if (lane < kGJ)
#pragma unroll
        for (int t = 0; t < kGJ; ++t) sP[lane * kGJ + t] = pr[t];
      if (bad && lane == 0) s_bad = 1;
    } else {
      for (int e = tid - 64; e < n * kGJ; e += NT - 64) {
        const int i = e >> 3, t = e & (kGJ - 1);
        Cb[e] = t < pb ? A[i * lda + p + t] : 0.0;
      }
    }
    __syncthreads();
    ADMMQ_GJ_PH(0);
    if (s_bad) return false;
    double bk[2][kGJ];   // B'[.][j] for j = js, js + 128
    {
      double ak[2][kGJ];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = min(js + 128 * h, n - 1);
#pragma unroll
        for (int s2 = 0; s2 < kGJ; ++s2) ak[h][s2] = s2 < pb ? A[(p + s2) * lda + j] : 0.0;
      }
#pragma unroll
      for (int t = 0; t < kGJ; ++t) {   // one row of P^-1 at a time (all 64 hoisted would spill)
        double pt[kGJ];
#pragma unroll
        for (int s2 = 0; s2 < kGJ; ++s2) pt[s2] = sP[t * kGJ + s2];
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int s2 = 0; s2 < kGJ; ++s2) { a0 += pt[s2] * ak[0][s2]; a1 += pt[s2] * ak[1][s2]; }
        bk[0][t] = a0; bk[1][t] = a1;
        asm volatile("" ::: "memory");
      }
    }
    __syncthreads();
    ADMMQ_GJ_PH(1);
    if (g == 0) {   // the new row block (columns outside kb) and A[kb][kb] = P^-1
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = js + 128 * h;
        if (j < n) {
          const bool inb = j >= p && j < p + pb;
#pragma unroll
          for (int t = 0; t < kGJ; ++t)
            if (t < pb) A[(p + t) * lda + j] = inb ? sP[t * kGJ + (j - p)] : bk[h][t];
        }
      }
    }
    // rows i = g (mod kRG) outside kb, two at a time: both rows' loads before their stores (the
    // compiler cannot tell rows i and i + kRG of A apart); Cb and sP are separate arrays
    for (int i0 = g; i0 < n; i0 += 2 * kRG) {
      double ci[2][kGJ], a[2][2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int i = min(i0 + kRG * b, n - 1);
#pragma unroll
        for (int t = 0; t < kGJ; ++t) ci[b][t] = Cb[i * kGJ + t];
#pragma unroll
        for (int h = 0; h < 2; ++h) a[b][h] = A[i * lda + min(js + 128 * h, n - 1)];
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int i = i0 + kRG * b;
        if (i >= n || (i >= p && i < p + pb)) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = js + 128 * h;
          if (j < n) {
            double v;
            if (j >= p && j < p + pb) {   // C' = -C P^-1
              v = 0.0;
#pragma unroll
              for (int s2 = 0; s2 < kGJ; ++s2) v -= ci[b][s2] * sP[s2 * kGJ + (j - p)];
            } else {                      // D -= C B'
              v = a[b][h];
#pragma unroll
              for (int t = 0; t < kGJ; ++t) v -= ci[b][t] * bk[h][t];
            }
            A[i * lda + j] = v;
          }
        }
      }
    }
    __syncthreads();
    ADMMQ_GJ_PH(2);
  }
#undef ADMMQ_GJ_PH
  if (ADMMQ_TRACE && threadIdx.x == 0)
    for (int k = 0; k < 3; ++k) g_spd_trace[8 + k] = ph[k];
  return true;
}

// y = x Ainv for one row per 16-lane group: lane c holds x_k and y_k for k = c + 16 q; x_k is
// taken from its owner lane of the group (ds_bpermute), Ainv's row k read from LDS
// (consecutive lanes, consecutive columns)
__device__ __forceinline__ void spd_row_times(const double* A, int n, const double (&x)[kSpdPer], double (&y)[kSpdPer]) {
  const int lane = threadIdx.x & 63, c = lane & (kSpdCols - 1), base = lane & ~(kSpdCols - 1);
  const int lda = spd_lda(n);
#pragma unroll
  for (int q = 0; q < kSpdPer; ++q) y[q] = 0.0;
#pragma unroll
  for (int kq = 0; kq < kSpdPer; ++kq) {
    const int kn = min(kSpdCols, n - kSpdCols * kq);   // uniform
    for (int kc = 0; kc < kn; ++kc) {
      const int k = kc + kSpdCols * kq;
      const double xk = __shfl(x[kq], base + kc, 64);
      const double* Ak = A + k * lda;
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int j = c + kSpdCols * q;
        y[q] += xk * Ak[min(j, n - 1)] * (j < n ? 1.0 : 0.0);
      }
    }
  }
}

__device__ __forceinline__ void spd_load_row(const double* __restrict__ F, int row, int m, int n, double (&x)[kSpdPer]) {
  const int c = threadIdx.x & (kSpdCols - 1);
#pragma unroll
  for (int q = 0; q < kSpdPer; ++q) {
    const int i = c + kSpdCols * q;
    x[q] = (row < m && i < n) ? F[(size_t)row * n + i] : 0.0;
  }
}

// Block sum (every thread's v; the result in every thread), NT / 64 waves
template <int NT>
__device__ __forceinline__ double spd_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += red[w];
  return t;
}

__global__ __launch_bounds__(kSpdThreads) void k_spd_solve64(const double* __restrict__ G, const double* __restrict__ F,
                                                             int m, int n, double* __restrict__ X,
                                                             int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double sP[kGJ * kGJ];
  ADMMQ_SPD_STAMP(0);
  __shared__ double Cb[kSpdSmallMax * kGJ];
  const bool ok = spd_inverse_lds<kSpdThreads>(G, n, 0.0, A, sP, Cb);
  ADMMQ_SPD_STAMP(2);
  if (!ok) {
    if (threadIdx.x == 0 && info) *info = 1;
    return;
  }
  const int c = threadIdx.x & (kSpdCols - 1);
  for (int r0 = 0; r0 < m; r0 += kSpdRowsPerPass) {
    const int row = r0 + (int)(threadIdx.x / kSpdCols);
    if (r0 + 4 * (int)(threadIdx.x >> 6) >= m) continue;   // every row of this wave past the end
    double f[kSpdPer], x[kSpdPer];
    spd_load_row(F, row, m, n, f);
    spd_row_times(A, n, f, x);
    if (row < m)
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int i = c + kSpdCols * q;
        if (i < n) X[(size_t)row * n + i] = x[q];
      }
  }
  ADMMQ_SPD_STAMP(3);
  if (threadIdx.x == 0 && info) *info = 0;
}

// Diagnostics (admmq_debug_epc_evals): evaluations (inverses) made by k_epc_step64 since the
// last reset
__device__ unsigned long long g_epc_evals = 0ull;

// e(mu), e'(mu) and X = F (G + mu I)^-1 (into X when `store`); false if G + mu I is not SPD.
// With A = G + mu I: <F, X> and ||X||^2 give e = normY2 - <F, X> - mu ||X||^2 (the eigen form
// normY2 - sum_j c_j (s_j + 2 mu) / (s_j + mu)^2), and e' = 2 mu <X, X A^-1>.
constexpr int kEpcThreads = 1024;   // (512 threads: no spills, but the rank-8 updates at half the width: 6.3 vs 5.4 s per parafac_epc)
__device__ __forceinline__ bool epc_eval(const double* __restrict__ G, const double* __restrict__ F, int m, int n,
                                         double mu, double normY2, double* A, double* sP, double* Cb, double* red,
                                         double* X, double& e, double& de) {
  if (threadIdx.x == 0) atomicAdd(&g_epc_evals, 1ull);
  if (!spd_inverse_lds<kEpcThreads>(G, n, mu, A, sP, Cb)) return false;
  double fx = 0.0, xx = 0.0, ww = 0.0;
  const int c = threadIdx.x & (kSpdCols - 1);
  for (int r0 = 0; r0 < m; r0 += kEpcThreads / kSpdCols) {   // X = F A^-1 (stored), <F, X>, ||X||^2
    const int row = r0 + (int)(threadIdx.x / kSpdCols);
    if (r0 + 4 * (int)(threadIdx.x >> 6) >= m) continue;   // every row of this wave past the end
    double f[kSpdPer], x[kSpdPer];
    spd_load_row(F, row, m, n, f);
    spd_row_times(A, n, f, x);
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) { fx += f[q] * x[q]; xx += x[q] * x[q]; }
    if (row < m)
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int i = c + kSpdCols * q;
        if (i < n) X[(size_t)row * n + i] = x[q];
      }
  }
  if (mu > 0.0) {   // <X, X A^-1>, X read back (this thread's own stores)
    for (int r0 = 0; r0 < m; r0 += kEpcThreads / kSpdCols) {
      const int row = r0 + (int)(threadIdx.x / kSpdCols);
      if (r0 + 4 * (int)(threadIdx.x >> 6) >= m) continue;
      double x[kSpdPer], y[kSpdPer];
      spd_load_row(X, row, m, n, x);
      spd_row_times(A, n, x, y);
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) ww += x[q] * y[q];
    }
  }
  fx = spd_block_sum<kEpcThreads>(fx, red);
  xx = spd_block_sum<kEpcThreads>(xx, red);
  ww = spd_block_sum<kEpcThreads>(ww, red);
  e = normY2 - fx - mu * xx;
  de = 2.0 * mu * ww;
  return true;
}

// mu to 1e-12 relative: X = F (G + mu I)^-1 moves by at most mu_err / (lambda_min + mu) <= 1e-12
// relative (mu itself is ill-determined where e is flat, e'(0) = 0: there only X matters)
constexpr double kEpcMuTol = 1e-12;

__global__ __launch_bounds__(kEpcThreads) void k_epc_step64(const double* __restrict__ G, const double* __restrict__ F,
                                                            int m, int n, double normY2, double delta2,
                                                            double* __restrict__ mu_io, double* __restrict__ X,
                                                            int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double sP[kGJ * kGJ];
  __shared__ double Cb[kSpdSmallMax * kGJ];
  __shared__ double red[kSpdThreads / 64];   // (>= the epc kernel's waves)
  double tr = 0.0;   // trace(G) / n: the scale of the bracket's first step
  for (int i = threadIdx.x; i < n; i += kEpcThreads) tr += G[(size_t)i * n + i];
  tr = spd_block_sum<kEpcThreads>(tr, red) / (double)n;
  const double warm = *mu_io;
  // One evaluation site (a state machine: every branch below is uniform over the workgroup):
  //   WARM   the warm start, when > 0: e < delta2 puts the root above it (mu > 0 for sure);
  //   ZERO   mu = 0: e(0) >= delta2 means the LS step keeps the error (mu = 0, done);
  //   GROW   no upper end yet: from max(lo, trace / n 2^-20), doubling / Newton steps;
  //   NEWTON safeguarded Newton inside [lo, hi] until the step is below fp64 resolution, the
  //          bracket has collapsed or e is at its rounding floor (e is flat near mu = 0,
  //          e'(0) = 0, so a small |e - delta2| alone does not fix mu: the step decides);
  //   FINAL  one more evaluation when X is not that of the returned mu.
  enum { WARM, ZERO, GROW, NEWTON, FINAL, DONE };
  // the search state lives in LDS (uniform; thread 0 updates it between evaluations), so the
  // evaluation's registers are not shared with it (128 VGPRs at 1024 threads)
  struct St { double e, de, mu, lo, hi, xmu, at; int state, have, need0; };
  __shared__ St st;
  if (threadIdx.x == 0) {
    st.e = st.de = st.mu = st.lo = 0.0; st.hi = __builtin_huge_val(); st.xmu = -1.0;
    st.state = warm > 0.0 ? WARM : ZERO; st.have = 0; st.need0 = 1;
  }
  __syncthreads();
  for (int guard = 0; guard < 400; ++guard) {
    if (threadIdx.x == 0) {   // where to evaluate next (or DONE)
      for (;;) {
        const int state = st.state;
        if (state == WARM) { st.at = warm; break; }
        if (state == ZERO) { st.at = 0.0; break; }
        if (state == GROW) {
          double at = st.have ? 2.0 * fmax(st.mu, st.lo) : (tr > 0.0 ? tr * 0x1p-20 : 1e-300);
          if (st.have && st.de > 0.0) {   // a Newton step from below (lands above the root: e convex near it)
            const double nx = st.mu - (st.e - delta2) / st.de;
            if (nx > st.mu && nx < at) at = nx;
            if (fabs(nx - st.mu) <= kEpcMuTol * st.mu) { st.state = FINAL; continue; }   // converged from below
          }
          if (!(at < 1e300)) { st.state = FINAL; continue; }
          st.at = at;
          break;
        }
        if (state == NEWTON) {
          if (!(st.hi - st.lo > kEpcMuTol * st.hi)) { st.state = FINAL; continue; }   // collapsed bracket
          double nx = st.de > 0.0 ? st.mu - (st.e - delta2) / st.de : -1.0;
          if (!(nx > st.lo && nx < st.hi)) nx = 0.5 * (st.lo + st.hi);
          if (fabs(nx - st.mu) <= kEpcMuTol * st.mu) { st.state = FINAL; continue; }   // converged
          st.at = nx;
          break;
        }
        if (state == FINAL) {
          if (!st.have || st.xmu == st.mu) { st.state = DONE; break; }
          st.at = st.mu;
          break;
        }
        break;   // DONE
      }
    }
    __syncthreads();
    if (st.state == DONE) break;
    double en, dn;
    const double at = st.at;
    const bool ok = epc_eval(G, F, m, n, at, normY2, A, sP, Cb, red, X, en, dn);
    if (threadIdx.x == 0) {   // (epc_eval ends with a block sum: every thread is past its reads of st)
      if (ok) st.xmu = at;
      const int state = st.state;
      if (state == WARM) {
        if (ok) {
          st.mu = at; st.e = en; st.de = dn; st.have = 1;
          if (en < delta2) { st.lo = at; st.need0 = 0; }
          else st.hi = at;
        }
        st.state = st.need0 ? ZERO : GROW;
      } else if (state == ZERO) {
        if (ok && en >= delta2) { st.mu = 0.0; st.have = 0; st.state = DONE; }   // the LS step: mu = 0
        else st.state = (st.have && st.hi < __builtin_huge_val()) ? NEWTON : GROW;
      } else if (state == GROW) {
        if (!ok) st.lo = at;
        else {
          st.mu = at; st.e = en; st.de = dn; st.have = 1;
          if (en < delta2) st.lo = at;
          else { st.hi = at; st.state = NEWTON; }
        }
      } else if (state == NEWTON) {
        if (!ok) st.lo = at;
        else {
          st.mu = at; st.e = en; st.de = dn;
          if (en < delta2) st.lo = at; else st.hi = at;
          if (fabs(en - delta2) <= 16.0 * 0x1p-52 * normY2) st.state = FINAL;   // at the rounding floor of e
        }
      } else {
        st.state = DONE;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { *mu_io = st.mu; if (info) *info = (st.have || st.mu == 0.0) ? 0 : 1; }
}

}  // namespace admmq

using namespace admmq;

extern "C" {

int32_t admmq_epc_mu(const double* c, const double* s, int64_t n, double normY2, double delta2, double* mu,
                     void* stream) {
  if (!c || !s || !mu || n <= 0 || n > (1LL << 30)) return set_error(ADMMQ_ERR_ARG, "epc_mu: bad arguments");
  hipLaunchKernelGGL(k_epc_mu, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), c, s, (int)n, normY2, delta2, mu);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_mu: launch failed");
}

int32_t admmq_debug_epc_evals(unsigned long long* out, int32_t reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_epc_evals), sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z = 0ull;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_epc_evals), &z, sizeof(z)) != hipSuccess) return -1;
  }
  return ADMMQ_OK;
}

int32_t admmq_debug_spd_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spd_trace), sizeof(g_spd_trace)) == hipSuccess ? ADMMQ_OK : -1;
}

int32_t admmq_spd_solve64(const double* G, const double* F, int64_t m, int64_t n, double* X, int32_t* info,
                          void* stream) {
  if (!G || !F || !X || m < 0 || n <= 0 || n > kSpdSmallMax || m > (1LL << 24))
    return set_error(ADMMQ_ERR_ARG, "spd_solve64: bad arguments (1 <= n <= 136)");
  if (m == 0) return ADMMQ_OK;
  const size_t lds = (size_t)n * spd_lda((int)n) * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_spd_solve64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(k_spd_solve64, dim3(1), dim3(kSpdThreads), lds, static_cast<hipStream_t>(stream), G, F, (int)m,
                     (int)n, X, info);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "spd_solve64: launch failed");
}

int32_t admmq_epc_step64(const double* G, const double* F, int64_t m, int64_t n, double normY2, double delta2,
                         double* mu, double* X, int32_t* info, void* stream) {
  if (!G || !F || !X || !mu || m <= 0 || n <= 0 || n > kSpdSmallMax || m > (1LL << 24))
    return set_error(ADMMQ_ERR_ARG, "epc_step64: bad arguments (1 <= n <= 136)");
  const size_t lds = (size_t)n * spd_lda((int)n) * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_epc_step64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(k_epc_step64, dim3(1), dim3(kEpcThreads), lds, static_cast<hipStream_t>(stream), G, F, (int)m,
                     (int)n, normY2, delta2, mu, X, info);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_step64: launch failed");
}

}  // extern "C"
