// The R x R solves of the CP-ALS / EPC initialiser for any rank (source/parafac_epc.py:42-74:
// tensorly parafac's torch.linalg.solve, musco cp_anc's eigendecomposition; admmq.parafac_epc).
// The one-workgroup kernels of epc_kernels.hip hold G in LDS and stop at n = 136; every larger
// rank of the resnet layers (183 ... 1141, 12 of resnet18's 16 convs) runs here, spread over
// the chip:
//
//   A  = G + shift I                       k_s64_fill (fp64, identity padding to 32 x 32 blocks)
//   L  = chol(A), Linv = L^-1              spd_kernels.hip (the blocked fp64 Cholesky and
//                                           triangular inverse of the ADMM prepare, 32 x 32
//                                           blocks: launch_spd_linv)
//   W1 = F Linv^T, X = W1 Linv             two fp64 GEMMs on v_mfma_f64_16x16x4_f64 (k_cp64
//                                           plain-GEMM jobs, the triangle of Linv masked and
//                                           its empty K range skipped; split-K in fixed order)
//
// i.e. X = F A^-1. The CP-ALS update is one such solve (shift 0, or a relative shift on
// request). The EPC update X = F (G + mu I)^-1 repeats it inside the multiplier search of
// epc_search.h: every evaluation round is the solve at the search's next mu plus
//   W2 = X Linv^T, and f = ||W1||^2 = <F, X>, g = ||X||^2, h = ||W2||^2 = <X, X A^-1>
// (k_s64_sumsq: fixed-order partials), from which k_s64_state forms e(mu) = ||Y||^2 - f - mu g
// and e'(mu) = 2 mu h and decides the next mu (one thread). A round after the search is done
// costs only launch overhead: the state kernel zeroes the Cholesky's block count in the
// descriptor and raises the gate every other launch of the round checks first. The host asks
// for rounds and reads the done flag when it wants (admmq.panel.epc_step64: a few rounds per
// read); the state never leaves the device.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "../../include/admmq.h"
#include "admmq_internal.h"
#include "cp64.h"
#include "epc_search.h"

namespace admmq {

constexpr int kS64SumBlocks = 64;
constexpr int kS64MaxEvals = 96;   // the search's evaluation budget (the one-workgroup step: 400 cheap ones)

// Diagnostics (admmq_debug_s64_evals): evaluation rounds that did work since the last reset
__device__ unsigned long long g_s64_evals = 0ull;

struct Solve64State {
  EpcSearch st;
  double warm, tr, normY2, delta2;
  double part[3 * kS64SumBlocks];
  int gate;        // nonzero: the search is done, a round's launches return at once
  int nbk;         // the Cholesky's 32 x 32 block count
  int evals;       // evaluations made
  int exhausted;   // the budget ran out before the search converged
  int flags[4];    // ProbDesc flags of the Cholesky: [2] a non-positive pivot
};

static inline size_t s64_al(size_t v) { return (v + 255) / 256 * 256; }

struct S64Layout {
  int m, n, ldm, nbk;
  Solve64State* S;
  ProbDesc* desc;
  char* cp;        // the GEMM plan's tables and partial planes
  double *A64, *L64, *D64, *W1, *W2;
  size_t bytes;
};

// Deterministic carve (a function of m, n only) and the GEMM plan: job 0 W1 = F Linv^T,
// job 1 X = W1 Linv, job 2 W2 = X Linv^T.
static void s64_layout(int64_t m, int64_t n, const double* F, double* X, void* base, S64Layout& L, Cp64Plan& pl) {
  L.m = (int)m; L.n = (int)n;
  L.ldm = (int)((n + 31) / 32 * 32);
  L.nbk = L.ldm / 32;
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b ? b + off : nullptr; off += s64_al(nbytes); return p; };
  L.S = reinterpret_cast<Solve64State*>(take(sizeof(Solve64State)));
  L.desc = reinterpret_cast<ProbDesc*>(take(sizeof(ProbDesc)));
  const size_t ldm2 = (size_t)L.ldm * L.ldm, mn = (size_t)m * n;
  L.A64 = reinterpret_cast<double*>(take(ldm2 * 8));
  L.L64 = reinterpret_cast<double*>(take(ldm2 * 8));
  L.D64 = reinterpret_cast<double*>(take((size_t)L.ldm * 32 * 8));
  L.W1 = reinterpret_cast<double*>(take(mn * 8));
  L.W2 = reinterpret_cast<double*>(take(mn * 8));
  pl.jobs.clear(); pl.units.clear(); pl.split_ids.clear();
  const int* gate = b ? &L.S->gate : nullptr;
  cp64_plan_gemm(pl, F, n, L.L64, L.ldm, 1, 1, L.W1, (int)m, (int)n, (int)n, gate);
  cp64_plan_gemm(pl, L.W1, n, L.L64, L.ldm, 0, 2, X, (int)m, (int)n, (int)n, gate);
  cp64_plan_gemm(pl, X, n, L.L64, L.ldm, 1, 1, L.W2, (int)m, (int)n, (int)n, gate);
  L.cp = b ? b + off : nullptr;
  off += cp64_carve(pl, L.cp);
  L.bytes = off + 256;
}

__device__ __forceinline__ double s64_block_sum(double v, double* red) {   // 256 threads, fixed order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double t = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return t;
}

// trace(G) / n, the search's initial state and first mu (epc), or the solve's shift (ALS)
__global__ __launch_bounds__(256) void k_s64_begin(Solve64State* S, ProbDesc* d, const double* __restrict__ G, int n,
                                                   int nbk, const double* __restrict__ mu_warm, double normY2,
                                                   double delta2, double rel_shift, int epc) {
  __shared__ double red[4];
  double t = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) t += G[(size_t)i * n + i];
  const double tr = s64_block_sum(t, red) / (double)n;
  if (threadIdx.x == 0) {
    S->tr = tr; S->normY2 = normY2; S->delta2 = delta2;
    S->evals = 0; S->exhausted = 0;
    for (int q = 0; q < 4; ++q) S->flags[q] = 0;
    const double warm = epc ? *mu_warm : 0.0;
    S->warm = warm;
    epc_search_init(S->st, warm);
    if (epc) epc_search_next(S->st, warm, tr, delta2);
    else S->st.at = rel_shift * tr;
    S->gate = 0;
    S->nbk = nbk;
    d->nbk = nbk;
  }
}

// A64 = G + at I (the search's mu, or the solve's shift) in fp64, identity past n
__global__ __launch_bounds__(256) void k_s64_fill(const Solve64State* __restrict__ S, const ProbDesc* __restrict__ d,
                                                  const double* __restrict__ G, int n) {
  if (S->gate) return;
  const double at = S->st.at;
  const int ldm = d->ldm;
  double* A = d->A64;
  const long long total = (long long)ldm * ldm;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int r = (int)(e / ldm), c = (int)(e - (long long)r * ldm);
    double v;
    if (r < n && c < n) v = G[(size_t)r * n + c] + (r == c ? at : 0.0);
    else v = r == c ? 1.0 : 0.0;
    A[e] = v;
  }
}

// Fixed-order partial sums of squares of W1, X, W2 (kS64SumBlocks blocks)
__global__ __launch_bounds__(256) void k_s64_sumsq(Solve64State* S, const double* __restrict__ a,
                                                   const double* __restrict__ b, const double* __restrict__ c,
                                                   long long len) {
  if (S->gate) return;
  __shared__ double red[4];
  double x = 0.0, y = 0.0, z = 0.0;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < len; e += (long long)kS64SumBlocks * 256) {
    const double va = a[e], vb = b[e], vc = c[e];
    x = fma(va, va, x);
    y = fma(vb, vb, y);
    z = fma(vc, vc, z);
  }
  x = s64_block_sum(x, red);
  y = s64_block_sum(y, red);
  z = s64_block_sum(z, red);
  if (threadIdx.x == 0) {
    S->part[3 * blockIdx.x] = x;
    S->part[3 * blockIdx.x + 1] = y;
    S->part[3 * blockIdx.x + 2] = z;
  }
}

// One thread: absorb the round's evaluation, decide the next mu (or done)
__global__ __launch_bounds__(64) void k_s64_state(Solve64State* S, ProbDesc* d, int* done_out) {
  if (threadIdx.x != 0) return;
  if (!S->gate) {
    double f = 0.0, g = 0.0, h = 0.0;
    for (int q = 0; q < kS64SumBlocks; ++q) {
      f += S->part[3 * q];
      g += S->part[3 * q + 1];
      h += S->part[3 * q + 2];
    }
    const bool ok = S->flags[2] == 0 && f < __builtin_huge_val() && g < __builtin_huge_val() && h < __builtin_huge_val();
    S->flags[2] = 0;
    ++S->evals;
    atomicAdd(&g_s64_evals, 1ull);
    EpcSearch& st = S->st;
    if (st.state == EPC_FINAL) {   // X at the returned mu, recomputed
      st.pmu = ok ? st.at : __builtin_nan("");
      st.state = EPC_DONE;
    } else {
      const double at = st.at;
      epc_search_absorb(st, ok, S->normY2 - f - at * g, 2.0 * at * h, h, S->delta2, S->normY2);
      epc_search_next(st, S->warm, S->tr, S->delta2);
      // X holds the last evaluated point's solve: another round at mu when that is not mu
      if (st.state == EPC_DONE && !(st.pmu == st.mu)) { st.state = EPC_FINAL; st.at = st.mu; }
    }
    if (st.state != EPC_DONE && S->evals >= kS64MaxEvals) { st.state = EPC_DONE; S->exhausted = 1; }
    S->gate = st.state == EPC_DONE;
    d->nbk = S->gate ? 0 : S->nbk;
  }
  if (done_out) *done_out = S->gate;
}

// info: 0 converged (X at mu); 1 no positive definite G + mu I found / budget spent; 2 not done
// yet (more rounds needed). ALS solve (epc = 0): 0, or 1 on a non-positive pivot.
__global__ __launch_bounds__(64) void k_s64_end(const Solve64State* __restrict__ S, double* mu_io, int* info, int epc) {
  if (threadIdx.x != 0) return;
  if (!epc) {
    if (info) *info = S->flags[2] ? 1 : 0;
    return;
  }
  if (mu_io) *mu_io = S->st.mu;
  if (info) *info = !S->gate ? 2 : (epc_search_ok(S->st) && !S->exhausted ? 0 : 1);
}

// Host side --------------------------------------------------------------------------

static bool s64_args_ok(const double* G, const double* F, int64_t m, int64_t n, const double* X) {
  return G && F && X && m >= 1 && n >= 1 && n <= 8192 && m <= (1LL << 24) && m * n < (1LL << 31);
}

static int s64_begin(const double* G, const double* F, int64_t m, int64_t n, double* X, const double* mu,
                     double normY2, double delta2, double rel_shift, int epc, void* ws, size_t wsb, hipStream_t s,
                     S64Layout& L, Cp64Plan& pl) {
  s64_layout(m, n, F, X, ws, L, pl);
  if (!ws || wsb < L.bytes) return set_error(ADMMQ_ERR_WORKSPACE, "solve64: workspace too small");
  ProbDesc d;
  std::memset(&d, 0, sizeof(d));
  d.A64 = L.A64; d.L64 = L.L64; d.D64 = L.D64;
  d.flags = L.S->flags;
  d.R = L.n; d.ldm = L.ldm; d.nbk = L.nbk;
  if (upload_async(L.desc, &d, sizeof(d), s) != ADMMQ_OK || cp64_upload(pl, L.cp, s) != ADMMQ_OK)
    return set_error(ADMMQ_ERR_HIP, "solve64: descriptor upload failed");
  hipLaunchKernelGGL(k_s64_begin, dim3(1), dim3(256), 0, s, L.S, L.desc, G, L.n, L.nbk, mu, normY2, delta2, rel_shift,
                     epc);
  return ADMMQ_OK;
}

// One solve at the state's mu / shift (+ the EPC round's products, sums and state update)
static int s64_round(const S64Layout& L, const Cp64Plan& pl, const double* G, const double* X, int epc, int* done,
                     hipStream_t s) {
  const long long tot = (long long)L.ldm * L.ldm;
  const int fb = (int)std::min<long long>(1024, (tot + 255) / 256);
  hipLaunchKernelGGL(k_s64_fill, dim3(fb), dim3(256), 0, s, L.S, L.desc, G, L.n);
  launch_spd_linv(L.desc, 1, L.nbk, s);
  if (cp64_launch_job(pl, L.cp, 0, s) != ADMMQ_OK || cp64_launch_job(pl, L.cp, 1, s) != ADMMQ_OK)
    return set_error(ADMMQ_ERR_HIP, "solve64: GEMM launch failed");
  if (epc) {
    if (cp64_launch_job(pl, L.cp, 2, s) != ADMMQ_OK) return set_error(ADMMQ_ERR_HIP, "solve64: GEMM launch failed");
    hipLaunchKernelGGL(k_s64_sumsq, dim3(kS64SumBlocks), dim3(256), 0, s, L.S, L.W1, X, L.W2,
                       (long long)L.m * L.n);
    hipLaunchKernelGGL(k_s64_state, dim3(1), dim3(64), 0, s, L.S, L.desc, done);
  }
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "solve64: launch failed");
}

void launch_spd_solve64_small(const double* G, const double* F, int m, int n, double rel_shift, double* X, int* info,
                              hipStream_t s);

}  // namespace admmq

using namespace admmq;

extern "C" {

int32_t admmq_debug_s64_evals(unsigned long long* out, int32_t reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_s64_evals), sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z = 0ull;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_s64_evals), &z, sizeof(z)) != hipSuccess) return -1;
  }
  return ADMMQ_OK;
}

size_t admmq_solve64_workspace_size(int64_t m, int64_t n) {
  if (m < 1 || n < 1 || n > 8192 || m > (1LL << 24) || m * n >= (1LL << 31)) return 0;
  S64Layout L;
  Cp64Plan pl;
  s64_layout(m, n, nullptr, nullptr, nullptr, L, pl);
  return L.bytes;
}

int32_t admmq_spd_solve64_ws(const double* G, const double* F, int64_t m, int64_t n, double rel_shift, double* X,
                             int32_t* info, void* workspace, size_t workspace_bytes, void* stream) {
  if (!s64_args_ok(G, F, m, n, X) || !(rel_shift >= 0.0) || !(rel_shift < 1e300))
    return set_error(ADMMQ_ERR_ARG, "spd_solve64_ws: bad arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n <= 136) {   // the one-workgroup Gauss-Jordan form (epc_kernels.hip); no workspace needed
    launch_spd_solve64_small(G, F, (int)m, (int)n, rel_shift, X, info, s);
    return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "spd_solve64_ws: launch failed");
  }
  S64Layout L;
  Cp64Plan pl;
  int rc = s64_begin(G, F, m, n, X, nullptr, 0.0, 0.0, rel_shift, 0, workspace, workspace_bytes, s, L, pl);
  if (rc) return rc;
  rc = s64_round(L, pl, G, X, 0, nullptr, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_s64_end, dim3(1), dim3(64), 0, s, L.S, nullptr, info, 0);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "spd_solve64_ws: launch failed");
}

int32_t admmq_epc_begin64(const double* G, const double* F, int64_t m, int64_t n, double normY2, double delta2,
                          const double* mu, double* X, void* workspace, size_t workspace_bytes, void* stream) {
  if (!s64_args_ok(G, F, m, n, X) || !mu) return set_error(ADMMQ_ERR_ARG, "epc_begin64: bad arguments");
  S64Layout L;
  Cp64Plan pl;
  return s64_begin(G, F, m, n, X, mu, normY2, delta2, 0.0, 1, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream), L, pl);
}

int32_t admmq_epc_rounds64(const double* G, const double* F, int64_t m, int64_t n, double* X, int32_t rounds,
                           int32_t* done, void* workspace, size_t workspace_bytes, void* stream) {
  if (!s64_args_ok(G, F, m, n, X) || rounds < 0 || rounds > 1024) return set_error(ADMMQ_ERR_ARG, "epc_rounds64: bad arguments");
  S64Layout L;
  Cp64Plan pl;
  s64_layout(m, n, F, X, workspace, L, pl);
  if (!workspace || workspace_bytes < L.bytes) return set_error(ADMMQ_ERR_WORKSPACE, "epc_rounds64: workspace too small");
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int r = 0; r < rounds; ++r) {
    const int rc = s64_round(L, pl, G, X, 1, done, s);
    if (rc) return rc;
  }
  return ADMMQ_OK;
}

int32_t admmq_epc_end64(int64_t m, int64_t n, double* mu, int32_t* info, void* workspace, size_t workspace_bytes,
                        void* stream) {
  if (m < 1 || n < 1 || !mu) return set_error(ADMMQ_ERR_ARG, "epc_end64: bad arguments");
  S64Layout L;
  Cp64Plan pl;
  s64_layout(m, n, nullptr, nullptr, workspace, L, pl);
  if (!workspace || workspace_bytes < L.bytes) return set_error(ADMMQ_ERR_WORKSPACE, "epc_end64: workspace too small");
  hipLaunchKernelGGL(k_s64_end, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), L.S, mu, info, 1);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "epc_end64: launch failed");
}

}  // extern "C"
