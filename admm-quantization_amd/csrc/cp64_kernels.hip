// fp64 per-mode contractions of the CP-ALS / EPC initialiser (admmq.parafac_epc; the
// reference's source/parafac_epc.py:42-74 runs them inside tensorly `parafac` and musco
// `cp_anc` on the fp64 tensor):
//
//   MTTKRP  F[a, r] = sum_k Y_(n)[a, k] KR[k, r]      KR = Khatri-Rao product of the other factors
//   Gram    G = hadamard over o != n of (U_o^T U_o)
//
// on v_mfma_f64_16x16x4_f64: a 64 x 64 output tile per workgroup of 4 waves (each wave a
// 32 x 32 sub-tile = 2 x 2 MFMA blocks), K-step 16 staged through registers into
// double-buffered k-major LDS images (one barrier per step). As in the fp32 ALS kernels
// (als_kernels.hip), the Khatri-Rao operand is formed while the K-step is staged and the
// unfolding is addressed in place - nothing is materialised; long reductions are split
// into K chunks whose partial planes k_cp64_reduce sums in chunk order (deterministic).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/admmq.h"
#include "admmq_internal.h"
#include "cp64.h"

namespace admmq {

__device__ __forceinline__ double c64_opA(const Cp64Job& j, int which, int m, int k) {
  if (j.kind == 0) {
    const int kq = k / j.K2, kr = k - kq * j.K2;
    return j.W[(long long)m * j.sm + (long long)kq * j.s1 + (long long)kr * j.s2];
  }
  return (which ? j.Y : j.X)[(long long)k * j.R + m];   // A(m = r1, k = i) = U[i, r1]
}
__device__ __forceinline__ double c64_opB(const Cp64Job& j, int which, int k, int n) {
  if (j.kind == 0) {
    if (j.K2 == 1) {   // (also the plain GEMM: B row-major k x n, or transposed; tri masks a triangle)
      const double v = j.bt ? j.X[(long long)n * j.ldb + k] : j.X[(long long)k * j.ldb + n];
      return j.tri == 0 ? v : ((j.tri == 1 ? k <= n : k >= n) ? v : 0.0);
    }
    const int kq = k / j.K2, kr = k - kq * j.K2;
    return j.X[(long long)kq * j.N + n] * j.Y[(long long)kr * j.N + n];
  }
  return (which ? j.Y : j.X)[(long long)k * j.R + n];
}

// acc[i][c] (the 16 x 16 MFMA block (i, c) of this wave's 32 x 32 sub-tile of the tile at
// (m0, n0)) += sum over k in [kb, ke) of A(m, k) B(k, n).
__device__ __forceinline__ void c64_core(const Cp64Job& j, int which, int m0, int n0, int kb, int ke, int Mrows,
                                         int Ncols, f64x4 (&acc)[2][2], double (*sA)[kC64BK * kC64LD],
                                         double (*sB)[kC64BK * kC64LD]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const bool afast = j.afast != 0, bfast = j.bt != 0;   // bfast: B staged along k (B^T rows contiguous)
  // two register sets: the loads of K-step k + 2 are issued before step k's MFMAs, so each has
  // a whole step of MFMAs plus the barrier to land (one set: the step's own MFMAs only, and
  // every step then waited on its loads; the same MFMA sequence either way: same bits)
  double ra[2][kC64PA], rb[2][kC64PB];
  // the plain GEMM (kind 0, K2 = 1): per-element base pointers formed once, so a K-step's
  // load is a pointer plus an offset (the generic operand functions divide k by K2 and form
  // 64-bit products per element and step: VALU work on the MFMA's pipe)
  const bool plain = j.kind == 0 && j.K2 == 1;
  const double* pa[kC64PA];
  const double* pb[kC64PB];
  int ka[kC64PA], kbq[kC64PB], nb_[kC64PB];
  long long sa = 0, sb = 0;
  if (plain) {
#pragma unroll
    for (int e = 0; e < kC64PA; ++e) {
      const int x = tid + kC64NT * e;
      const int r = afast ? x % kC64BM : x / kC64BK, kk = afast ? x / kC64BM : x % kC64BK;
      const int m = min(m0 + r, Mrows - 1);
      pa[e] = j.W + (long long)m * j.sm + (long long)kk * j.s1;
      ka[e] = m0 + r < Mrows ? kk : (1 << 30);   // past the rows: never loaded
    }
    sa = j.s1;
#pragma unroll
    for (int e = 0; e < kC64PB; ++e) {
      const int x = tid + kC64NT * e;
      const int c = bfast ? x / kC64BK : x % kC64BN, kk = bfast ? x % kC64BK : x / kC64BN;
      const int n = min(n0 + c, Ncols - 1);
      pb[e] = j.bt ? j.X + (long long)n * j.ldb + kk : j.X + (long long)kk * j.ldb + n;
      kbq[e] = n0 + c < Ncols ? kk : (1 << 30);
      nb_[e] = n0 + c;
    }
    sb = j.bt ? 1 : j.ldb;
  }
  auto load = [&](int set, int k0) {
    if (plain) {
#pragma unroll
      for (int e = 0; e < kC64PA; ++e) ra[set][e] = k0 + ka[e] < ke ? pa[e][(long long)k0 * sa] : 0.0;
#pragma unroll
      for (int e = 0; e < kC64PB; ++e) {
        const int k = k0 + kbq[e];
        const bool in = k < ke && (j.tri == 0 || (j.tri == 1 ? k <= nb_[e] : k >= nb_[e]));
        rb[set][e] = in ? pb[e][(long long)k0 * sb] : 0.0;
      }
      return;
    }
#pragma unroll
    for (int e = 0; e < kC64PA; ++e) {
      const int x = tid + kC64NT * e;
      const int r = afast ? x % kC64BM : x / kC64BK, kk = afast ? x / kC64BM : x % kC64BK;
      const int m = m0 + r, k = k0 + kk;
      ra[set][e] = (m < Mrows && k < ke) ? c64_opA(j, which, m, k) : 0.0;
    }
#pragma unroll
    for (int e = 0; e < kC64PB; ++e) {
      const int x = tid + kC64NT * e;
      const int c = bfast ? x / kC64BK : x % kC64BN, kk = bfast ? x % kC64BK : x / kC64BN;
      const int n = n0 + c, k = k0 + kk;
      rb[set][e] = (n < Ncols && k < ke) ? c64_opB(j, which, k, n) : 0.0;
    }
  };
  auto store = [&](int set, int buf) {
#pragma unroll
    for (int e = 0; e < kC64PA; ++e) {
      const int x = tid + kC64NT * e;
      const int r = afast ? x % kC64BM : x / kC64BK, kk = afast ? x / kC64BM : x % kC64BK;
      sA[buf][kk * kC64LD + r] = ra[set][e];
    }
#pragma unroll
    for (int e = 0; e < kC64PB; ++e) {
      const int x = tid + kC64NT * e;
      const int c = bfast ? x / kC64BK : x % kC64BN, kk = bfast ? x % kC64BK : x / kC64BN;
      sB[buf][kk * kC64LD + c] = rb[set][e];
    }
  };
  if (kb >= ke) return;
  load(0, kb);
  __syncthreads();   // the previous use of the images (an earlier core call) is done
  store(0, 0);
  __syncthreads();
  if (kb + kC64BK < ke) load(0, kb + kC64BK);
  int buf = 0;
  const int fr = lane & 15, fk = lane >> 4;   // f64 16x16x4 operands: A[fr][fk], B[fk][fr]
  auto mfmas = [&](int bf) {
    const double* a = sA[bf] + 32 * wm + fr;
    const double* b = sB[bf] + 32 * wn + fr;
#pragma unroll
    for (int q = 0; q < kC64BK / 4; ++q) {
      const int kk = (4 * q + fk) * kC64LD;
      const double a0 = a[kk], a1 = a[kk + 16], b0 = b[kk], b1 = b[kk + 16];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
  };
  // step k0 reads LDS image buf; register set s holds step k0 + BK, set s ^ 1 receives k0 + 2 BK
  for (int k0 = kb; k0 < ke; k0 += 2 * kC64BK) {
    {
      const bool more1 = k0 + kC64BK < ke, more2 = k0 + 2 * kC64BK < ke;
      if (more2) load(1, k0 + 2 * kC64BK);
      mfmas(buf);
      if (more1) store(0, buf ^ 1);
      __syncthreads();
      buf ^= 1;
      if (!more1) break;
    }
    {
      const int k1 = k0 + kC64BK;
      const bool more1 = k1 + kC64BK < ke, more2 = k1 + 2 * kC64BK < ke;
      if (more2) load(0, k1 + 2 * kC64BK);
      mfmas(buf);
      if (more1) store(1, buf ^ 1);
      __syncthreads();
      buf ^= 1;
      if (!more1) break;
    }
  }
}

__device__ __forceinline__ void c64_zero(f64x4 (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[i][c] = f64x4{0.0, 0.0, 0.0, 0.0};
}

// One 64 x 64 output tile (and K chunk) per workgroup. C/D map of v_mfma_f64_16x16x4_f64:
// col = lane & 15, row = (lane >> 4) + 4 reg (cdna_hip_programming.md, fragment layout).
__global__ __launch_bounds__(kC64NT) void k_cp64(const Cp64Job* __restrict__ jobs, const Cp64Unit* __restrict__ units) {
  __shared__ __attribute__((aligned(16))) double sA[2][kC64BK * kC64LD];
  __shared__ __attribute__((aligned(16))) double sB[2][kC64BK * kC64LD];
  const Cp64Unit u = units[blockIdx.x];
  const Cp64Job& j = jobs[u.job];
  if (j.gate && *j.gate) return;   // a round of the blocked EPC step after its search is done
  const int m0 = u.tm * kC64BM, n0 = u.tn * kC64BN;
  f64x4 acc[2][2];
  c64_zero(acc);
  double* dst;
  if (j.kind == 0) {
    // the chunk, clipped to the rows of B a triangular operand can have nonzero (tri 1: k <= n,
    // so k < n0 + 64; tri 2: k >= n0); an empty chunk leaves its partial plane zero
    const int kb = max(u.ks * j.kchunk, j.tri == 2 ? n0 : 0);
    const int ke = min(min(j.K, u.ks * j.kchunk + j.kchunk), j.tri == 1 ? n0 + kC64BN : j.K);
    c64_core(j, 0, m0, n0, kb, ke, j.M, j.N, acc, sA, sB);
    dst = j.nsplit > 1 ? j.part + (size_t)u.ks * j.M * j.N : j.out;
  } else {
    c64_core(j, 0, m0, n0, 0, j.Kx, j.R, j.R, acc, sA, sB);
    if (j.Ky > 0) {   // Hadamard product with the second Gram (same tile)
      f64x4 acc2[2][2];
      c64_zero(acc2);
      c64_core(j, 1, m0, n0, 0, j.Ky, j.R, j.R, acc2, sA, sB);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[i][c] *= acc2[i][c];
    }
    dst = j.out;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int col = n0 + 32 * wn + 16 * c + (lane & 15);
      if (col >= j.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 32 * wm + 16 * i + (lane >> 4) + 4 * r;
        if (row < j.M) dst[(size_t)row * j.N + col] = acc[i][c][r];
      }
    }
}

// MTTKRP split-K: F = sum over chunks s (in order) of part[s]. grid.y = job.
__global__ __launch_bounds__(256) void k_cp64_reduce(const Cp64Job* __restrict__ jobs, const int* __restrict__ ids) {
  const Cp64Job& j = jobs[ids[blockIdx.y]];
  if (j.gate && *j.gate) return;
  const size_t n = (size_t)j.M * j.N;
  for (size_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (size_t)gridDim.x * 256) {
    double s = j.part[e];
    for (int q = 1; q < j.nsplit; ++q) s += j.part[(size_t)q * n + e];
    j.out[e] = s;
  }
}

// ---------------------------------------------------------------------------------
// Host planning

static inline size_t al64(size_t v) { return (v + 255) / 256 * 256; }
static inline int cdiv64(long long a, long long b) { return (int)((a + b - 1) / b); }

static bool layer64_ok(const admmq_cp_layer_f64& L) {
  if (!L.W || (L.ndim != 2 && L.ndim != 3) || L.R < 1) return false;
  for (int d = 0; d < L.ndim; ++d)
    if (L.dims[d] < 1 || !L.factors[d]) return false;
  return true;
}

// Carve order: [jobs][units][split ids][partials]. Per layer: the mode's Gram(-Hadamard)
// job, then its MTTKRP job (K chunks: enough units to fill the chip, chunks >= 64 rows).
static int plan_cp64(const admmq_cp_layer_f64* layers, int n, int mode, void* base, Cp64Plan& pl, std::string& err) {
  pl.jobs.clear(); pl.units.clear(); pl.split_ids.clear();
  for (int l = 0; l < n; ++l) {
    const admmq_cp_layer_f64& L = layers[l];
    if (!layer64_ok(L)) { err = "cp64 layer " + std::to_string(l) + ": bad W/factors/dims/ndim/R"; return ADMMQ_ERR_ARG; }
    if (mode < 0 || mode >= L.ndim) { err = "mode out of range"; return ADMMQ_ERR_ARG; }
    const int I = L.dims[0], J = L.dims[1], Kd = L.ndim == 3 ? L.dims[2] : 1, R = L.R;
    if ((long long)I * J * Kd >= (1LL << 31)) { err = "cp64 layer too large"; return ADMMQ_ERR_ARG; }
    if (base && (!L.F || !L.G)) { err = "cp64 layer: F / G output missing"; return ADMMQ_ERR_ARG; }
    Cp64Job g;
    std::memset(&g, 0, sizeof(g));
    g.kind = 1; g.R = R; g.M = g.N = R; g.afast = 1; g.ldb = R;
    int o[2], no = 0;
    for (int d = 0; d < L.ndim; ++d)
      if (d != mode) o[no++] = d;
    g.X = L.factors[o[0]]; g.Kx = L.dims[o[0]];
    if (no == 2) { g.Y = L.factors[o[1]]; g.Ky = L.dims[o[1]]; }
    g.out = L.G;
    const int gid = (int)pl.jobs.size();
    g.unit0 = (int)pl.units.size();
    for (int a = 0; a < cdiv64(R, kC64BM); ++a)
      for (int b = 0; b < cdiv64(R, kC64BN); ++b) pl.units.push_back({gid, a, b, 0});
    g.nunits = (int)pl.units.size() - g.unit0;
    pl.jobs.push_back(g);
    Cp64Job f;
    std::memset(&f, 0, sizeof(f));
    f.kind = 0; f.N = R; f.ldb = R; f.W = L.W; f.M = L.dims[mode];
    const long long JK = (long long)J * Kd;
    if (L.ndim == 3) {   // k runs over the other two modes in their order (torch unfold / Khatri-Rao order)
      if (mode == 0) { f.K = J * Kd; f.K2 = Kd; f.sm = JK; f.s1 = Kd; f.s2 = 1; f.X = L.factors[1]; f.Y = L.factors[2]; }
      if (mode == 1) { f.K = I * Kd; f.K2 = Kd; f.sm = Kd; f.s1 = JK; f.s2 = 1; f.X = L.factors[0]; f.Y = L.factors[2]; }
      if (mode == 2) { f.K = I * J; f.K2 = J; f.sm = 1; f.s1 = JK; f.s2 = Kd; f.X = L.factors[0]; f.Y = L.factors[1]; f.afast = 1; }
    } else {
      f.K2 = 1;
      if (mode == 0) { f.K = J; f.sm = J; f.s1 = 1; f.X = L.factors[1]; }
      else { f.K = I; f.sm = 1; f.s1 = J; f.X = L.factors[0]; f.afast = 1; }
    }
    f.out = L.F;
    const int tm = cdiv64(f.M, kC64BM), tn = cdiv64(f.N, kC64BN);
    // chunks of >= 64 K (4 K-steps): a unit's time is its chain of K-steps, each waiting on
    // the next step's global loads (the Khatri-Rao operand formed in flight), so the short
    // reductions of the small EPC layers are cut as finely as the chip can hold (R = 134,
    // (9, 64, 64): mode 0 24 -> 192 units, modes 1 / 2 3 -> 27)
    const int by_k = std::max(1, f.K / 64), by_fill = std::max(1, 512 / std::max(tm * tn, 1));
    f.nsplit = std::max(1, std::min(by_k, by_fill));
    f.kchunk = cdiv64(cdiv64(f.K, f.nsplit), kC64BK) * kC64BK;
    f.nsplit = cdiv64(f.K, f.kchunk);
    const int fid = (int)pl.jobs.size();
    if (f.nsplit > 1) pl.split_ids.push_back(fid);
    f.unit0 = (int)pl.units.size();
    for (int ks = 0; ks < f.nsplit; ++ks)
      for (int a = 0; a < tm; ++a)
        for (int b = 0; b < tn; ++b) pl.units.push_back({fid, a, b, ks});
    f.nunits = (int)pl.units.size() - f.unit0;
    pl.jobs.push_back(f);
  }
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b ? b + off : nullptr; off += al64(nbytes); return p; };
  take(pl.jobs.size() * sizeof(Cp64Job));
  take(pl.units.size() * sizeof(Cp64Unit));
  take(pl.split_ids.size() * sizeof(int) + 4);
  for (auto& j : pl.jobs)
    if (j.kind == 0 && j.nsplit > 1) j.part = reinterpret_cast<double*>(take((size_t)j.nsplit * j.M * j.N * 8));
  pl.bytes = off + 256;
  return ADMMQ_OK;
}

static int run_cp64(const Cp64Plan& pl, void* base, size_t wsb, hipStream_t s, std::string& err) {
  if (!base || wsb < pl.bytes) { err = "workspace too small"; return ADMMQ_ERR_WORKSPACE; }
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b + off; off += al64(nbytes); return p; };
  Cp64Job* djobs = reinterpret_cast<Cp64Job*>(take(pl.jobs.size() * sizeof(Cp64Job)));
  Cp64Unit* dunits = reinterpret_cast<Cp64Unit*>(take(pl.units.size() * sizeof(Cp64Unit)));
  int* dids = reinterpret_cast<int*>(take(pl.split_ids.size() * sizeof(int) + 4));
  auto up = [&](void* dst, const void* src, size_t nbytes) {
    return upload_async(dst, src, nbytes, s) == ADMMQ_OK;   // pinned staging: never waits for the stream
  };
  if (!up(djobs, pl.jobs.data(), pl.jobs.size() * sizeof(Cp64Job)) ||
      !up(dunits, pl.units.data(), pl.units.size() * sizeof(Cp64Unit)) ||
      !up(dids, pl.split_ids.data(), pl.split_ids.size() * sizeof(int))) {
    err = "cp64 descriptor upload failed";
    return ADMMQ_ERR_HIP;
  }
  if (!pl.units.empty())
    hipLaunchKernelGGL(k_cp64, dim3((unsigned)pl.units.size()), dim3(kC64NT), 0, s, djobs, dunits);
  if (!pl.split_ids.empty()) {
    size_t mx = 0;
    for (int id : pl.split_ids) mx = std::max(mx, (size_t)pl.jobs[id].M * pl.jobs[id].N);
    const int nb = (int)std::min<size_t>(256, (mx + 255) / 256);
    hipLaunchKernelGGL(k_cp64_reduce, dim3(nb, (unsigned)pl.split_ids.size()), dim3(256), 0, s, djobs, dids);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("cp64 launch: ") + hipGetErrorString(e); return ADMMQ_ERR_HIP; }
  return ADMMQ_OK;
}

// ---------------------------------------------------------------------------------
// Plain fp64 GEMMs (the blocked R x R solves of solve64.hip)

void cp64_plan_gemm(Cp64Plan& pl, const double* A, long long lda, const double* B, long long ldb, int bt, int tri,
                    double* C, int M, int N, int K, const int* gate) {
  Cp64Job f;
  std::memset(&f, 0, sizeof(f));
  f.kind = 0; f.M = M; f.N = N; f.K = K; f.K2 = 1;
  f.W = A; f.sm = lda; f.s1 = 1; f.s2 = 0;
  f.X = B; f.ldb = ldb; f.bt = bt; f.tri = tri;
  f.out = C; f.gate = gate;
  const int tm = cdiv64(M, kC64BM), tn = cdiv64(N, kC64BN);
  // K chunks of >= 64 to bring the units to ~1024 (4 per CU): a 64 x 64 tile's K chain is
  // latency-bound at these sizes (each K-step of k_cp64 waits on its staging loads), so short
  // chains side by side beat long ones; the fixed-order reduction reads the extra planes once
  // (with a triangular B most chunks of the early column tiles are empty and return at once)
  const int by_k = std::max(1, K / 64), by_fill = std::max(1, 1024 / std::max(tm * tn, 1));
  f.nsplit = std::max(1, std::min(by_k, by_fill));
  f.kchunk = cdiv64(cdiv64(K, f.nsplit), kC64BK) * kC64BK;
  f.nsplit = cdiv64(K, f.kchunk);
  const int fid = (int)pl.jobs.size();
  if (f.nsplit > 1) pl.split_ids.push_back(fid);
  f.unit0 = (int)pl.units.size();
  for (int ks = 0; ks < f.nsplit; ++ks)
    for (int a = 0; a < tm; ++a)
      for (int b = 0; b < tn; ++b) pl.units.push_back({fid, a, b, ks});
  f.nunits = (int)pl.units.size() - f.unit0;
  pl.jobs.push_back(f);
}

// Carve order: [jobs][units][split ids][partials] (as plan_cp64).
size_t cp64_carve(Cp64Plan& pl, void* base) {
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b ? b + off : nullptr; off += al64(nbytes); return p; };
  take(pl.jobs.size() * sizeof(Cp64Job));
  take(pl.units.size() * sizeof(Cp64Unit));
  take(pl.split_ids.size() * sizeof(int) + 4);
  for (auto& j : pl.jobs)
    if (j.kind == 0 && j.nsplit > 1) j.part = reinterpret_cast<double*>(take((size_t)j.nsplit * j.M * j.N * 8));
  pl.bytes = off + 256;
  return pl.bytes;
}

struct Cp64Tables { Cp64Job* jobs; Cp64Unit* units; int* ids; };
static Cp64Tables cp64_tables(const Cp64Plan& pl, void* base) {
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b + off; off += al64(nbytes); return p; };
  Cp64Tables t;
  t.jobs = reinterpret_cast<Cp64Job*>(take(pl.jobs.size() * sizeof(Cp64Job)));
  t.units = reinterpret_cast<Cp64Unit*>(take(pl.units.size() * sizeof(Cp64Unit)));
  t.ids = reinterpret_cast<int*>(take(pl.split_ids.size() * sizeof(int) + 4));
  return t;
}

int cp64_upload(const Cp64Plan& pl, void* base, hipStream_t s) {
  const Cp64Tables t = cp64_tables(pl, base);
  if (upload_async(t.jobs, pl.jobs.data(), pl.jobs.size() * sizeof(Cp64Job), s) != ADMMQ_OK ||
      upload_async(t.units, pl.units.data(), pl.units.size() * sizeof(Cp64Unit), s) != ADMMQ_OK ||
      upload_async(t.ids, pl.split_ids.data(), pl.split_ids.size() * sizeof(int), s) != ADMMQ_OK)
    return ADMMQ_ERR_HIP;
  return ADMMQ_OK;
}

int cp64_launch_job(const Cp64Plan& pl, void* base, int job, hipStream_t s) {
  const Cp64Tables t = cp64_tables(pl, base);
  const Cp64Job& j = pl.jobs[job];
  if (j.nunits > 0) hipLaunchKernelGGL(k_cp64, dim3((unsigned)j.nunits), dim3(kC64NT), 0, s, t.jobs, t.units + j.unit0);
  if (j.nsplit > 1) {
    int pos = 0;
    while (pl.split_ids[pos] != job) ++pos;
    const size_t mn = (size_t)j.M * j.N;
    const int nb = (int)std::min<size_t>(2048, (mn + 255) / 256);   // (one element per thread up to 512 K)
    hipLaunchKernelGGL(k_cp64_reduce, dim3(nb, 1), dim3(256), 0, s, t.jobs, t.ids + pos);
  }
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : ADMMQ_ERR_HIP;
}

}  // namespace admmq

using namespace admmq;

extern "C" {

size_t admmq_cp64_workspace_size(const admmq_cp_layer_f64* layers, int32_t n, int32_t mode) {
  Cp64Plan pl;
  std::string err;
  if (n < 0 || (n > 0 && !layers) || plan_cp64(layers, n, mode, nullptr, pl, err)) return 0;
  return pl.bytes;
}

int32_t admmq_cp64_gram_mttkrp(const admmq_cp_layer_f64* layers, int32_t n, int32_t mode, void* workspace,
                               size_t workspace_bytes, void* stream) {
  if (n < 0 || (n > 0 && !layers)) return set_error(ADMMQ_ERR_ARG, "cp64_gram_mttkrp: bad layer array");
  Cp64Plan pl;
  std::string err;
  int rc = plan_cp64(layers, n, mode, workspace, pl, err);
  if (!rc) rc = run_cp64(pl, workspace, workspace_bytes, static_cast<hipStream_t>(stream), err);
  if (rc) return set_error(rc, ("cp64_gram_mttkrp: " + err).c_str());
  return ADMMQ_OK;
}

}  // extern "C"
