// The EPC step's Lagrange multiplier on the device (cp_anc, source/parafac_epc.py:61-74;
// admmq.parafac_epc): the scalar root search that ran on the host after every mode step's
// R x R eigendecomposition, with two host synchronisations per step.
#include <cmath>
#include <cstdint>

#include "../../include/admmq.h"
#include "admmq_internal.h"
#include "epc_search.h"

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
//                   c_j = |F v_j|^2), found by Newton steps on e, e'(mu) = 2 mu <X, X (G + mu I)^-1>,
//                   safeguarded by the bracket [lo, hi] (bisection / doubling; epc_search.h),
//                   each evaluation on tridiagonal L D L^T recurrences after one Householder
//                   reduction of G per call (below); mu = 0 when e(0) >= delta^2 already (the
//                   LS step keeps the error).
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

// rel_shift > 0: X = F (G + rel_shift (trace(G) / n) I)^-1 (the regularised retry of a CP-ALS
// update whose G was not numerically positive definite; admmq.parafac_epc)
__global__ __launch_bounds__(kSpdThreads) void k_spd_solve64(const double* __restrict__ G, const double* __restrict__ F,
                                                             int m, int n, double rel_shift, double* __restrict__ X,
                                                             int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double sP[kGJ * kGJ];
  ADMMQ_SPD_STAMP(0);
  __shared__ double Cb[kSpdSmallMax * kGJ];
  double shift = 0.0;
  if (rel_shift > 0.0) {
    __shared__ double red[kSpdThreads / 64];
    double t = 0.0;
    for (int i = threadIdx.x; i < n; i += kSpdThreads) t += G[(size_t)i * n + i];
    shift = rel_shift * spd_block_sum<kSpdThreads>(t, red) / (double)n;
  }
  const bool ok = spd_inverse_lds<kSpdThreads>(G, n, shift, A, sP, Cb);
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

// Diagnostics (admmq_debug_epc_evals): evaluations of e(mu) made by k_epc_step64 since the
// last reset; TRACE builds (admmq_debug_epc_trace): s_memrealtime of the last k_epc_step64 at
// {start, G in LDS, tridiagonal, Z = F Q, search done, X written}
__device__ unsigned long long g_epc_evals = 0ull;
__device__ unsigned long long g_epc_trace[16];   // [8 + k]: tridiagonalisation phase sums (wave 0's view)
#define ADMMQ_EPC_STAMP(k) \
  if (ADMMQ_TRACE && threadIdx.x == 0) g_epc_trace[k] = ADMMQ_NOW();

// ---------------------------------------------------------------------------
// The EPC mode update through one tridiagonal reduction per call. G = Q T Q^T (Householder,
// T symmetric tridiagonal, Q = H_0 ... H_{n-3}) once; with Z = F Q every evaluation of the
// error equation is a set of independent tridiagonal recurrences:
//   <F, X> = z (T + mu)^-1 z^T,  ||X||^2 = z (T + mu)^-2 z^T,  <X, X (G + mu)^-1> = z (T + mu)^-3 z^T
// summed over the rows z of Z. With T + mu = L D L^T (L unit lower bidiagonal) and u = L^-1 z,
// s(mu) = sum_i u_i^2 / D_i is the first; the other two are -s' and s'' / 2, carried through
// the same forward recurrence as derivatives in mu (D', D'', L', L'' once per evaluation, by
// one thread; u', u'' per row). One evaluation is O(m n) work with an n-step dependency
// chain (a few microseconds), where an explicit (G + mu I)^-1 was O(n^3) on one workgroup;
// the final X = (Z (T + mu)^-1) Q^T is one forward / backward pass and the reflectors applied
// in reverse.
constexpr int kEpcPad = 16 * kSpdPer;   // zeroed doubles after the matrix (unclamped reads past the last row)
// 1024 threads: at 512 (256 VGPRs) half the lanes sat out the rank-2 updates and the reflector
// products took two passes over 64 rows (0.79 vs 0.71 ms per step)
constexpr int kEpcThreads = 1024;

// Householder tridiagonalisation of the symmetric A (LDS, n x n, lda = n + 1) in place:
// dd (diagonal), ee (off-diagonal), tau_k and v_k (v_k[k + 1] = 1, stored in row k from
// column k + 1: that row is not touched after step k). Step k: p = tau A22 v,
// w = p - (tau / 2)(p . v) v, A22 -= v w^T + w v^T on the trailing (n - k - 1)^2 block (both
// triangles). Two workgroup barriers per step: the reflector of step k + 1 is formed by wave 0
// right after its own rows of step k's update (it owns row k + 1), into the other half of the
// double-buffered vb.
// Cross-lane sums without LDS round trips: DPP within a row of 16 lanes (xor 1, xor 2, half
// mirror, mirror: every lane of the row ends with the row's sum), v_readlane across the four
// rows. At this size every step is a latency chain; a ds_bpermute shuffle costs an LDS round
// trip per level.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double sum16(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  v += dpp_f64<0x141>(v);   // row_half_mirror
  v += dpp_f64<0x140>(v);   // row_mirror
  return v;
}
__device__ __forceinline__ double sum64(double v) {   // the wave's sum, in every lane
  v = sum16(v);
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

__device__ __forceinline__ void tri_reflector(double* A, int n, int k, double* vb, double* tau, double* dd,
                                              double* ee) {
  const int lane = threadIdx.x & 63, lda = spd_lda(n);
  double* row = A + k * lda;
  const double alpha = row[k + 1], dk = row[k];
  double x[3], sig = 0.0;
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int j = k + 2 + lane + 64 * h;
    const double xr = row[min(j, n - 1)];
    x[h] = j < n ? xr : 0.0;
    sig += x[h] * x[h];
  }
  sig = sum64(sig);
  double t = 0.0, beta = alpha, scale = 0.0;
  if (sig > 0.0) {
    const double nrm = sqrt(alpha * alpha + sig);
    beta = alpha <= 0.0 ? nrm : -nrm;
    t = (beta - alpha) / beta;
    scale = 1.0 / (alpha - beta);
  }
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int j = k + 2 + lane + 64 * h;
    if (j < n) {
      const double v = x[h] * scale;
      vb[j - k - 1] = v;
      row[j] = v;
    }
  }
  for (int j = lane; j <= k; j += 64) row[j] = 0.0;   // v_k over the whole row (tri_apply_q)
  if (lane == 0) {
    dd[k] = dk;
    vb[0] = 1.0;
    row[k + 1] = 1.0;
    tau[k] = t;
    ee[k] = beta;
  }
}

constexpr int kRegRows = (kSpdSmallMax + 15) / 16;   // rows per wave (9)

template <int NT>
__device__ __forceinline__ void tridiag_regs(const double* __restrict__ G, int n, double* A, double* dd, double* ee,
                                             double* tau, double* vb2, double* pb) {
  static_assert(NT == 1024, "16 waves x kRegRows rows");
  constexpr int kW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lda = spd_lda(n);
  double a[kRegRows][3];
#pragma unroll
  for (int t = 0; t < kRegRows; ++t) {
    const int r = w + kW * t;
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int j = lane + 64 * h;
      a[t][h] = (r < n && j < n) ? G[(size_t)r * n + j] : 0.0;
    }
  }
  auto store_row = [&](int t, int r) {   // this wave's row a[t] (wave-uniform t) into row r of A
#pragma unroll
    for (int tt = 0; tt < kRegRows; ++tt)
      if (tt == t)
#pragma unroll
        for (int h = 0; h < 3; ++h) {
          const int j = lane + 64 * h;
          if (j < n) A[r * lda + j] = a[tt][h];
        }
  };
  if (n >= 3 && w == 0) {
    store_row(0, 0);
    asm volatile("" ::: "memory");
    tri_reflector(A, n, 0, vb2, tau, dd, ee);
  }
  unsigned long long ph[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull}, tp = ADMMQ_NOW();
#define ADMMQ_TRI_PH(q)                               \
  if (ADMMQ_TRACE) {                                  \
    const unsigned long long tn_ = ADMMQ_NOW();       \
    ph[q] += tn_ - tp;                                \
    tp = tn_;                                         \
  }
  for (int k = 0; k + 3 <= n; ++k) {
    const int m = n - k - 1;
    const double* vb = vb2 + (k & 1) * kSpdSmallMax;
    double* part = A + (k + 1) * lda;   // rows k + 1 .. (and the pad) are free until their reflectors
    __syncthreads();   // v_k, tau_k visible
    ADMMQ_TRI_PH(0);
    const double t_ = tau[k];
    {   // this wave's partial column sums of A22 v over its rows r >= k + 1
      double ps[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int t = 0; t < kRegRows; ++t) {
        const int r = w + kW * t;
        if (r >= k + 1 && r < n) {
          const double vr = vb[r - k - 1];
#pragma unroll
          for (int h = 0; h < 3; ++h) ps[h] = fma(a[t][h], vr, ps[h]);
        }
      }
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int j = lane + 64 * h;
        if (j >= k + 1 && j < n) part[w * m + (j - k - 1)] = ps[h];
      }
    }
    ADMMQ_TRI_PH(1);
    __syncthreads();
    if (tid < m) {   // p = tau A22 v: the 16 waves' partials in wave order
      double sacc = 0.0;
#pragma unroll
      for (int ww = 0; ww < kW; ++ww) sacc += part[ww * m + tid];
      pb[tid] = t_ * sacc;
    }
    __syncthreads();
    ADMMQ_TRI_PH(2);
    double vj[3], wj[3], pv = 0.0;
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int i = lane + 64 * h - k - 1;
      const int ic = min(max(i, 0), m - 1);
      const double xv = vb[ic], xw = pb[ic];
      vj[h] = (i >= 0 && i < m) ? xv : 0.0;
      wj[h] = (i >= 0 && i < m) ? xw : 0.0;
      pv = fma(vj[h], wj[h], pv);
    }
    const double K = 0.5 * t_ * sum64(pv);
#pragma unroll
    for (int h = 0; h < 3; ++h) wj[h] = fma(-K, vj[h], wj[h]);
#pragma unroll
    for (int t = 0; t < kRegRows; ++t) {   // A22 -= v w^T + w v^T on this wave's rows
      const int r = w + kW * t;
      if (r >= k + 1 && r < n) {
        const double vr = vb[r - k - 1], wr = fma(-K, vr, pb[r - k - 1]);
#pragma unroll
        for (int h = 0; h < 3; ++h) a[t][h] = fma(-vr, wj[h], fma(-wr, vj[h], a[t][h]));
      }
    }
    ADMMQ_TRI_PH(3);
    if (k + 4 <= n && w == (k + 1) % kW) {   // the owner of row k + 1: the next reflector, from
      store_row((k + 1) / kW, k + 1);         // its row put where the reflector will be stored
      asm volatile("" ::: "memory");
      tri_reflector(A, n, k + 1, vb2 + ((k + 1) & 1) * kSpdSmallMax, tau, dd, ee);
    }
    ADMMQ_TRI_PH(4);
  }
#undef ADMMQ_TRI_PH
  if (ADMMQ_TRACE && tid == 0)
    for (int q = 0; q < 5; ++q) g_epc_trace[8 + q] = ph[q];
  // the last diagonal / off-diagonal entries, from their owners' registers (via rows n - 2,
  // n - 1 of A, free: no reflector goes there)
  __syncthreads();
  if (n >= 2 && w == (n - 2) % kW) store_row((n - 2) / kW, n - 2);
  if (w == (n - 1) % kW) store_row((n - 1) / kW, n - 1);
  __syncthreads();
  if (tid == 0) {
    if (n >= 2) {
      dd[n - 2] = A[(n - 2) * lda + n - 2];
      ee[n - 2] = A[(n - 2) * lda + n - 1];
    }
    dd[n - 1] = A[(n - 1) * lda + n - 1];
  }
  // rows n - 2, n - 1 and the pad held partials: zero them (tri_apply_q's crossing chunk
  // reads past the last reflector row) and so did the pad column of rows 1 .. n - 3; row 0's
  // was never written: all of them to 0 (tri_apply_q's unclamped reads meet only zeros there)
  __syncthreads();
  const int r0 = max(n - 2, 0);
  for (int e = tid; e < (n - r0) * lda + kEpcPad; e += NT) A[r0 * lda + e] = 0.0;
  for (int i = tid; i < r0; i += NT) A[i * lda + n] = 0.0;
  __syncthreads();
}

// One row of F -> F Q (dir = +1: H_0 first) or one row of Y -> Y Q^T (dir = -1: H_{n-3}
// first), 16 lanes per row, lane c holding coordinates c + 16 q. Row k of A holds v_k over
// every column (zeros up to k, 1 at k + 1: tri_reflector), so a lane reads v_k[c + 16 q]
// with an immediate offset and no clamp or select; only the chunk that crosses n masks (its
// reads past the row's end are the next row's values, or 0 past the LDS allocation).
// Issue-bound: ~60 wave-instructions per reflector and wave before, ~35 now.
__device__ __forceinline__ void tri_apply_q(const double* A, int n, const double* tau, int dir, double (&f)[kSpdPer]) {
  const int c = threadIdx.x & 15, lda = spd_lda(n);
  for (int s = 0; s + 3 <= n; ++s) {
    const int k = dir > 0 ? s : n - 3 - s;
    const double* v = A + k * lda + c;
    double vq[kSpdPer], d3[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) {
      double x = v[16 * q];
      if (16 * q + 15 >= n) x = c + 16 * q < n ? x : 0.0;   // (uniform test: the crossing chunk only)
      vq[q] = x;
      d3[q % 3] = fma(f[q], x, d3[q % 3]);
    }
    const double d = sum16((d3[0] + d3[1]) + d3[2]) * tau[k];
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) f[q] = fma(-d, vq[q], f[q]);
  }
}

// The LDL^T recurrence of T + mu I with its first and second derivatives in mu (thread 0),
// packed per step i (8 doubles, two 16-byte loads and one more): P[i] = {L_{i-1}, L_{i-1}',
// L_{i-1}'' (0 for i = 0), 1 / D_i, D_i' / D_i^2, D_i'' / D_i^2 - 2 D_i'^2 / D_i^3}. The
// dependency chain per step is one division and one fma (D_{i+1} = d_{i+1} + mu - e_i^2 / D_i,
// fp64 ops cost ~30 clocks each in a chain); d and e come one step ahead, everything else is
// off the chain. false if a pivot is not positive and finite.
constexpr int kTriP = 8;
constexpr int kTriChunk = 4;                                                     // recurrence steps per prefetched chunk
constexpr int kTriPad = (kSpdSmallMax + 2 * kTriChunk - 1) / (2 * kTriChunk) * (2 * kTriChunk);   // P rows (144)
__device__ __forceinline__ bool tri_ldl(const double* __restrict__ dd, const double* __restrict__ ee, int n, double mu,
                                        double* __restrict__ P) {
  double D = dd[0] + mu, D1 = 1.0, D2 = 0.0, L = 0.0, L1 = 0.0, L2 = 0.0;
  double e = ee[0], an = dd[min(1, n - 1)] + mu;
  bool bad = false;   // (no branch per step: a bad pivot only spoils the rest, which is then unused)
#pragma unroll 2
  for (int i = 0; i < n; ++i) {
    bad |= !(D > 0.0) || !(D < __builtin_huge_val());
    const double e_next = ee[min(i + 1, kSpdSmallMax - 1)], a_next = dd[min(i + 2, n - 1)] + mu;   // (prefetch)
    const double gi = 1.0 / D;
    const double g2 = gi * gi;
    double* Pi = P + kTriP * i;
    Pi[0] = L;
    Pi[1] = L1;
    Pi[2] = L2;
    Pi[3] = gi;
    Pi[4] = D1 * g2;
    Pi[5] = D2 * g2 - 2.0 * D1 * D1 * g2 * gi;
    L = e * gi;
    L1 = -e * D1 * g2;
    L2 = e * (2.0 * D1 * D1 * g2 * gi - D2 * g2);
    D = fma(-e * e, gi, an);   // the chain: one division and one fma per step
    D1 = fma(-e, L1, 1.0);
    D2 = -e * L2;
    e = e_next;
    an = a_next;
  }
  for (int i = n; i < kTriPad; ++i)   // zero steps past n: the row recurrences run whole chunks
#pragma unroll
    for (int q = 0; q < 6; ++q) P[kTriP * i + q] = 0.0;
  return !bad;
}

// The same coefficients streamed for a running evaluation: producer A (one thread) runs the
// D chain (one division and one fma per step) and writes L_{i-1} and 1 / D_i; producer B (a
// thread of another wave) follows it with the derivative chains and the other four entries;
// the row recurrences (tri_row_sums) follow B. Progress counters in LDS, advanced every
// kTriChunk steps behind a workgroup release fence; waits are bounded (a stalled partner
// leaves garbage and sets the stall flag, which the step reports through info; never a hang). Rows past n are zero (kTriPad), as in tri_ldl.
__device__ __forceinline__ void tri_wait(const volatile int* prog, int need, int* stall) {
  int guard = 0;
  for (; *prog < need && guard < (1 << 22); ++guard) __builtin_amdgcn_s_sleep(1);
  if (guard == (1 << 22)) *stall = 1;   // reported through info (the step's result is not trusted)
  // (a wave's LDS operations complete in order, so the loads below see what the producer
  // stored before its release; only the compiler must not hoist them above the poll)
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void tri_publish(volatile int* prog, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  *prog = v;
}
__device__ __forceinline__ bool tri_ldl_a(const double* __restrict__ dd, const double* __restrict__ ee, int n,
                                          double mu, double* __restrict__ P, volatile int* progA) {
  double D = dd[0] + mu, L = 0.0;
  double e = ee[0], an = dd[min(1, n - 1)] + mu;
  bool bad = false;
  for (int i = 0; i < n; ++i) {
    bad |= !(D > 0.0) || !(D < __builtin_huge_val());
    const double e_next = ee[min(i + 1, kSpdSmallMax - 1)], a_next = dd[min(i + 2, n - 1)] + mu;
    const double gi = 1.0 / D;
    double* Pi = P + kTriP * i;
    Pi[0] = L;
    Pi[3] = gi;
    L = e * gi;
    D = fma(-e * e, gi, an);
    e = e_next;
    an = a_next;
    if ((i & (kTriChunk - 1)) == kTriChunk - 1) tri_publish(progA, i + 1);
  }
  for (int i = n; i < kTriPad; ++i) { P[kTriP * i] = 0.0; P[kTriP * i + 3] = 0.0; }
  tri_publish(progA, kTriPad);
  return !bad;
}
__device__ __forceinline__ void tri_ldl_b(const double* __restrict__ ee, int n, double* __restrict__ P,
                                          const volatile int* progA, volatile int* progB, int* stall) {
  double D1 = 1.0, D2 = 0.0, L1 = 0.0, L2 = 0.0;
  for (int i = 0; i < n; ++i) {
    if ((i & (kTriChunk - 1)) == 0) tri_wait(progA, min(i + kTriChunk, kTriPad), stall);
    double* Pi = P + kTriP * i;
    const double gi = Pi[3], g2 = gi * gi, e = ee[min(i, kSpdSmallMax - 1)];
    Pi[1] = L1;
    Pi[2] = L2;
    Pi[4] = D1 * g2;
    Pi[5] = D2 * g2 - 2.0 * D1 * D1 * g2 * gi;
    L1 = -e * D1 * g2;
    L2 = e * (2.0 * D1 * D1 * g2 * gi - D2 * g2);
    D1 = fma(-e, L1, 1.0);
    D2 = -e * L2;
    if ((i & (kTriChunk - 1)) == kTriChunk - 1) tri_publish(progB, i + 1);
  }
  tri_wait(progA, kTriPad, stall);
  for (int i = n; i < kTriPad; ++i) {
    double* Pi = P + kTriP * i;
    Pi[1] = Pi[2] = Pi[4] = Pi[5] = 0.0;
  }
  tri_publish(progB, kTriPad);
}

// Block sums of three values (every thread's; the results in every thread)
template <int NT>
__device__ __forceinline__ void block_sum3(double& a, double& b, double& c, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = a;
    red[NT / 64 + (threadIdx.x >> 6)] = b;
    red[2 * NT / 64 + (threadIdx.x >> 6)] = c;
  }
  __syncthreads();
  a = b = c = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    a += red[w];
    b += red[NT / 64 + w];
    c += red[2 * NT / 64 + w];
  }
  __syncthreads();   // red reused
}

// s, s', s'' of one row z (Zt: n x m, column `row`) from the packed coefficients P at the
// current mu. z is read a chunk of kTriChunk ahead and P one step ahead of the recurrence;
// the empty asm between steps keeps the compiler from hoisting every step's P loads to the
// top of the chunk (they would take ~100 VGPRs).
struct TriCoef { double L, L1, L2, a1, a2, a3; };
__device__ __forceinline__ TriCoef tri_coef(const double* P, int i) {
  const double* Pi = P + kTriP * i;
  return TriCoef{Pi[0], Pi[1], Pi[2], Pi[3], Pi[4], Pi[5]};
}
__device__ __forceinline__ void tri_row_sums(const double* __restrict__ Zt, int m, int n, int row, const double* P,
                                             const volatile int* progB, int* stall, double& s0, double& s1,
                                             double& s2) {
  // every recurrence is one fma deep per step (the terms from the other chains formed off
  // it), and the sums alternate between two accumulators: a chained fp64 op costs ~30 clocks
  double u = 0.0, u1 = 0.0, u2 = 0.0;
  double a0[2] = {0.0, 0.0}, a1[2] = {0.0, 0.0}, a2[2] = {0.0, 0.0};
  tri_wait(progB, min(kTriChunk, kTriPad), stall);
  TriCoef cur = tri_coef(P, 0);
  auto steps = [&](const double (&zz)[kTriChunk], int i0) {   // (steps past n: P = 0, so no terms)
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) {
      const int i = i0 + q;
      const TriCoef nxt = tri_coef(P, min(i + 1, kTriPad - 1));
      const double c2 = fma(2.0 * cur.L1, u1, cur.L2 * u), c1 = cur.L1 * u;
      u2 = fma(-cur.L, u2, -c2);
      u1 = fma(-cur.L, u1, -c1);
      u = fma(-cur.L, u, zz[q]);
      const double uu = u * u, uu1 = u * u1;
      const double t0 = uu * cur.a1;
      const double t1 = fma(2.0 * uu1, cur.a1, -uu * cur.a2);
      const double t2 = fma(2.0 * fma(u1, u1, u * u2), cur.a1, fma(-4.0 * uu1, cur.a2, -uu * cur.a3));
      a0[q & 1] += t0;
      a1[q & 1] += t1;
      a2[q & 1] += t2;
      cur = nxt;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // two chunk buffers in turn: one being read while the other's loads are in flight (the
  // indices clamped, not predicated: straight-line loads keep counted vmcnt waits)
  double za[kTriChunk], zb[kTriChunk];
#pragma unroll
  for (int q = 0; q < kTriChunk; ++q) za[q] = Zt[(size_t)min(q, n - 1) * m + row];
  for (int i0 = 0; i0 < n; i0 += 2 * kTriChunk) {
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) zb[q] = Zt[(size_t)min(i0 + kTriChunk + q, n - 1) * m + row];
    tri_wait(progB, min(i0 + 2 * kTriChunk + 1, kTriPad), stall);   // (a step reads the next step's coefficients)
    steps(za, i0);
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) za[q] = Zt[(size_t)min(i0 + 2 * kTriChunk + q, n - 1) * m + row];
    steps(zb, i0 + kTriChunk);
  }
  s0 += a0[0] + a0[1];
  s1 += a1[0] + a1[1];
  s2 += a2[0] + a2[1];
}

// Y = Z (T + mu I)^-1 for one row: forward (u / D) from Zt into Wt, backward from Wt into Zt;
// both transposed (n x m), chunks read ahead as in tri_row_sums
__device__ __forceinline__ void tri_row_solve(double* __restrict__ Zt, double* __restrict__ Wt, int m, int n, int row,
                                              const double* P) {
  double u = 0.0;
  auto fwd = [&](const double (&zz)[kTriChunk], int i0) {
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) {
      const int i = i0 + q;
      if (i < n) {
        u = fma(-P[kTriP * i], u, zz[q]);   // (L_{-1} = 0)
        Wt[(size_t)i * m + row] = u * P[kTriP * i + 3];
      }
    }
  };
  double za[kTriChunk], zb[kTriChunk];
#pragma unroll
  for (int q = 0; q < kTriChunk; ++q) za[q] = Zt[(size_t)min(q, n - 1) * m + row];
  for (int i0 = 0; i0 < n; i0 += 2 * kTriChunk) {
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) zb[q] = Zt[(size_t)min(i0 + kTriChunk + q, n - 1) * m + row];
    fwd(za, i0);
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) za[q] = Zt[(size_t)min(i0 + 2 * kTriChunk + q, n - 1) * m + row];
    fwd(zb, i0 + kTriChunk);
  }
  __builtin_amdgcn_s_waitcnt(0);   // this thread's Wt stores complete before it reads them back
  double y = 0.0;
  auto bwd = [&](const double (&ww)[kTriChunk], int i1) {
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) {
      const int i = i1 - q;
      if (i >= 0) {
        y = i + 1 < n ? fma(-P[kTriP * (i + 1)], y, ww[q]) : ww[q];
        Zt[(size_t)i * m + row] = y;
      }
    }
  };
#pragma unroll
  for (int q = 0; q < kTriChunk; ++q) za[q] = Wt[(size_t)max(n - 1 - q, 0) * m + row];
  for (int i1 = n - 1; i1 >= 0; i1 -= 2 * kTriChunk) {
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) zb[q] = Wt[(size_t)max(i1 - kTriChunk - q, 0) * m + row];
    bwd(za, i1);
#pragma unroll
    for (int q = 0; q < kTriChunk; ++q) za[q] = Wt[(size_t)max(i1 - 2 * kTriChunk - q, 0) * m + row];
    bwd(zb, i1 - kTriChunk);
  }
}

__global__ __launch_bounds__(kEpcThreads) void k_epc_step64(const double* __restrict__ G, const double* __restrict__ F,
                                                            int m, int n, double normY2, double delta2,
                                                            double* __restrict__ mu_io, double* __restrict__ X,
                                                            double* __restrict__ Zt, int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double dd[kSpdSmallMax], ee[kSpdSmallMax], tau[kSpdSmallMax];
  __shared__ __attribute__((aligned(16))) double cf[kTriP * kTriPad];   // the tridiagonalisation's vb (2 x n) and pb, then the LDL coefficients
  __shared__ double red[3 * kEpcThreads / 64];
  __shared__ int s_ok, s_stall;
  __shared__ int s_prog[2];   // the streamed coefficients' progress (producers A, B)
  const int tid = threadIdx.x;
  if (tid == 0) s_stall = 0;
  ADMMQ_EPC_STAMP(0);
  double tr = 0.0;   // trace(G) / n: the scale of the bracket's first step
  for (int i = tid; i < n; i += kEpcThreads) tr += G[(size_t)i * n + i];
  {
    double z1 = 0.0, z2 = 0.0;
    block_sum3<kEpcThreads>(tr, z1, z2, red);
  }
  tr /= (double)n;
  ADMMQ_EPC_STAMP(1);
  tridiag_regs<kEpcThreads>(G, n, A, dd, ee, tau, cf, cf + 2 * kSpdSmallMax);
  ADMMQ_EPC_STAMP(2);
  // Z = F Q, stored transposed (Zt[i * m + row]: the row recurrences read it coalesced)
  for (int r0 = 0; r0 < m; r0 += kEpcThreads / 16) {
    const int row = r0 + (tid >> 4), c = tid & 15;
    if (r0 + 4 * (tid >> 6) >= m) continue;   // every row of this wave past the end
    double f[kSpdPer];
    spd_load_row(F, row, m, n, f);
    tri_apply_q(A, n, tau, +1, f);
    if (row < m)
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int j = c + 16 * q;
        if (j < n) Zt[(size_t)j * m + row] = f[q];
      }
  }
  ADMMQ_EPC_STAMP(3);
  const double warm = *mu_io;
  // the search (epc_search.h: a state machine in LDS, thread 0 deciding between evaluations;
  // every branch below uniform over the workgroup)
  __shared__ EpcSearch st;
  if (tid == 0) epc_search_init(st, warm);
  unsigned long long ev_ph[3] = {0ull, 0ull, 0ull};   // (TRACE: thread 0's LDL, row sums, block sum)
  for (int guard = 0; guard < 400; ++guard) {
    if (tid == 0) {   // where to evaluate next (or DONE)
      epc_search_next(st, warm, tr, delta2);
      if (st.state != EPC_DONE) atomicAdd(&g_epc_evals, 1ull);
    }
    if (tid == 0) { s_prog[0] = 0; s_prog[1] = 0; }
    __syncthreads();   // (also: Zt written, before the first evaluation)
    if (st.state == EPC_DONE) break;
    const double at = st.at;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const unsigned long long t1 = ADMMQ_NOW();
    // the coefficients streamed by two producers (waves 1 and 2, lane 0) while the rows'
    // recurrences (the other waves) follow them; ok (s_ok) is known after the block sum
    if (tid == 64) {
      s_ok = tri_ldl_a(dd, ee, n, at, cf, &s_prog[0]) ? 1 : 0;
    } else if (tid == 128) {
      tri_ldl_b(ee, n, cf, &s_prog[0], &s_prog[1], &s_stall);
    } else if (tid < 64 || tid >= 192) {
      for (int row = tid < 64 ? tid : tid - 128; row < m; row += kEpcThreads - 128)
        tri_row_sums(Zt, m, n, row, cf, &s_prog[1], &s_stall, s0, s1, s2);
    }
    const unsigned long long t2 = ADMMQ_NOW();
    block_sum3<kEpcThreads>(s0, s1, s2, red);
    ev_ph[1] += t2 - t1;
    ev_ph[2] += ADMMQ_NOW() - t2;
    if (tid == 0)   // e = ||Y||^2 - <F, X> - mu ||X||^2 with <F, X> = s, ||X||^2 = -s'; e' = mu s''
      epc_search_absorb(st, s_ok != 0, normY2 - s0 + at * s1, at * s2, 0.5 * s2, delta2, normY2);
  }
  ADMMQ_EPC_STAMP(4);
  if (ADMMQ_TRACE && tid == 0)
    for (int q = 0; q < 3; ++q) g_epc_trace[13 + q] = ev_ph[q];
  // X = (Z (T + mu I)^-1) Q^T at the returned mu (X first holds the forward pass, transposed)
  if (tid == 0 && !(st.pmu == st.mu)) s_ok = tri_ldl(dd, ee, n, st.mu, cf) ? 1 : 0;   // (else: the last evaluation's, ok)
  if (tid == 0 && st.pmu == st.mu) s_ok = 1;
  __syncthreads();
  const bool ok = s_ok != 0;
  if (ok)
    for (int row = tid; row < m; row += kEpcThreads) tri_row_solve(Zt, X, m, n, row, cf);   // (X: scratch here)
  __syncthreads();
  for (int r0 = 0; r0 < m; r0 += kEpcThreads / 16) {
    const int row = r0 + (tid >> 4), c = tid & 15;
    if (r0 + 4 * (tid >> 6) >= m) continue;
    double y[kSpdPer];
#pragma unroll
    for (int q = 0; q < kSpdPer; ++q) {
      const int j = c + 16 * q;
      y[q] = (row < m && j < n) ? Zt[(size_t)j * m + row] : 0.0;
    }
    tri_apply_q(A, n, tau, -1, y);
    if (row < m)
#pragma unroll
      for (int q = 0; q < kSpdPer; ++q) {
        const int j = c + 16 * q;
        if (j < n) X[(size_t)row * n + j] = ok ? y[q] : __builtin_nan("");
      }
  }
  // info 1: no positive definite G + mu I on the bracket, the search's evaluation budget
  // spent, or a stalled coefficient hand-off (a bounded wait expired: its sums are not trusted)
  if (tid == 0) {
    *mu_io = st.mu;
    if (info) *info = ok && st.state == EPC_DONE && !s_stall && (st.have || st.mu == 0.0) ? 0 : 1;
  }
  ADMMQ_EPC_STAMP(5);
}

// cp_anc's normalisation of the factors other than the updated one (one launch for both,
// instead of a norm, a clamp and a division per factor): out = U / max(||U[:, r]||, 1e-300)
// per column, a thread per column (coalesced across columns), the rows in order.
struct CpColNorm { const double* src[2]; double* dst[2]; int rows[2]; };
__global__ __launch_bounds__(256) void k_cp_colnorm(CpColNorm a, int R) {
  const int r = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
  if (r >= R) return;
  const double* src = a.src[f];
  double* dst = a.dst[f];
  const int I = a.rows[f];
  double acc = 0.0;
#pragma unroll 8
  for (int i = 0; i < I; ++i) {
    const double v = src[(size_t)i * R + r];
    acc = fma(v, v, acc);
  }
  const double nrm = fmax(sqrt(acc), 1e-300);
#pragma unroll 8
  for (int i = 0; i < I; ++i) dst[(size_t)i * R + r] = src[(size_t)i * R + r] / nrm;
}

void launch_spd_solve64_small(const double* G, const double* F, int m, int n, double rel_shift, double* X, int* info,
                              hipStream_t s) {
  const size_t lds = (size_t)n * spd_lda(n) * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_spd_solve64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(k_spd_solve64, dim3(1), dim3(kSpdThreads), lds, s, G, F, m, n, rel_shift, X, info);
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

int32_t admmq_cp_colnorm64(const double* A, int64_t rowsA, const double* B, int64_t rowsB, int64_t R, double* outA,
                           double* outB, void* stream) {
  if (!A || !outA || rowsA < 1 || R < 1 || R > (1 << 24) || rowsA > (1 << 24) || (B && (!outB || rowsB < 1 || rowsB > (1 << 24))))
    return set_error(ADMMQ_ERR_ARG, "cp_colnorm64: bad arguments");
  CpColNorm a;
  a.src[0] = A; a.dst[0] = outA; a.rows[0] = (int)rowsA;
  a.src[1] = B; a.dst[1] = outB; a.rows[1] = B ? (int)rowsB : 0;
  hipLaunchKernelGGL(k_cp_colnorm, dim3((unsigned)((R + 255) / 256), B ? 2u : 1u), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a, (int)R);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "cp_colnorm64: launch failed");
}

int32_t admmq_debug_epc_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_epc_trace), sizeof(g_epc_trace)) == hipSuccess ? ADMMQ_OK : -1;
}

int32_t admmq_debug_spd_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spd_trace), sizeof(g_spd_trace)) == hipSuccess ? ADMMQ_OK : -1;
}

int32_t admmq_spd_solve64(const double* G, const double* F, int64_t m, int64_t n, double* X, int32_t* info,
                          void* stream) {
  if (!G || !F || !X || m < 0 || n <= 0 || n > kSpdSmallMax || m > (1LL << 24))
    return set_error(ADMMQ_ERR_ARG, "spd_solve64: bad arguments (1 <= n <= 136)");
  if (m == 0) return ADMMQ_OK;
  launch_spd_solve64_small(G, F, (int)m, (int)n, 0.0, X, info, static_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "spd_solve64: launch failed");
}

int32_t admmq_epc_step64(const double* G, const double* F, int64_t m, int64_t n, double normY2, double delta2,
                         double* mu, double* X, double* work, int32_t* info, void* stream) {
  if (!G || !F || !X || !mu || !work || m <= 0 || n <= 0 || n > kSpdSmallMax || m > (1LL << 24))
    return set_error(ADMMQ_ERR_ARG, "epc_step64: bad arguments (1 <= n <= 136)");
  const size_t lds = ((size_t)n * spd_lda((int)n) + kEpcPad) * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_epc_step64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(k_epc_step64, dim3(1), dim3(kEpcThreads), lds, static_cast<hipStream_t>(stream), G, F, (int)m,
                     (int)n, normY2, delta2, mu, X, work, info);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_step64: launch failed");
}

}  // extern "C"
