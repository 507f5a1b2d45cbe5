// ALS-sweep contractions of scripts/factorize.py on fp32 MFMA, batched over layers:
//
//   G1  Gram∘Gram      G = (X^T X) ∘ (Y^T Y)                   :215,226,236  (2-way :276,:285  G = X^T X)
//   M1  MTTKRP         F[m,r] = sum_k W_(mode)[m,k] KR[k,r]     :217,227,237  (2-way :277,:286  W B, W^T A)
//   E1  rel-Frob error ||W - [[A,B(,C)]]||_F / ||W||_F          :246-253, source/admm.py:14-15
//
// All three are one LDS-tiled GEMM core (v_mfma_f32_32x32x2_f32, 32x32 sub-tile per
// wave, K-step 16, register prefetch of the next K-step + double-buffered LDS, one
// barrier per step) with operand loaders that never materialise an intermediate:
//   * the Khatri-Rao operand KR[k,r] = X[k / K2, r] * Y[k % K2, r] is formed while the
//     K-step is staged (the reference's einsum builds a (I,J,R) tensor, 1.2 GB at layer4);
//   * the mode-n unfolding of W is addressed in place: W_(n)[m,k] = W[m sm + (k/K2) s1 + (k%K2) s2],
//     with the k order chosen per mode so the loads run along contiguous memory;
//   * E1 forms [[A,B,C]] tile by tile in registers and folds (W - rec)^2 and W^2 into
//     fp64 block partials; nothing of the I x J x K reconstruction is stored.
// MTTKRP splits long reductions (the 9-row spatial mode has K = I J up to 262144) into
// K chunks whose partial planes are summed in chunk order by k_als_reduce; every sum
// is in a fixed order, so results are deterministic run to run.
// 3-way layers with a 3 x 3 spatial mode (KD = 9) take k_als_mttkrp_sp instead: the KD
// spatial slices are KD GEMMs that share one factor operand, W is staged in its own
// contiguous (row, k, s) runs, and the third factor is applied in the epilogue - no
// Khatri-Rao operand, no padded 9-row tiles, no K = I J reduction.
#include <algorithm>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/admmq.h"
#include "admmq_internal.h"

namespace admmq {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kAlsBK = 16;   // K-step
constexpr int kAlsBN = 64;   // tile columns
constexpr int kSpatialKD = 9;   // k_als_mttkrp_sp: the flattened 3 x 3 kernel

// One contraction of the batch (device descriptor).
struct AlsJob {
  int kind;            // 0 MTTKRP, 1 Gram(-Hadamard), 2 reconstruction error
  int M, N, K;         // output rows / cols, reduction length
  int nsplit, kchunk;  // MTTKRP: K chunks and their length (multiple of kAlsBK)
  int K2, afast;       // MTTKRP: Khatri-Rao inner extent; 1 = W_(n) rows are the contiguous index
  float invK2;         // 1 / K2 (fast exact div/mod)
  int R, Kx;           // Gram: R, rows of Y (0: 2-way, no Hadamard factor)
  long long sm, s1, s2;
  const float* W;      // MTTKRP / error: the layer tensor
  const float* X;      // MTTKRP: KR outer factor; Gram: first factor; error: factor 0
  const float* Y;      // MTTKRP: KR inner factor (nullptr 2-way); Gram: second factor; error: factor 1
  const float* Z;      // error: factor 2 (nullptr 2-way)
  float* part;         // MTTKRP: [nsplit][M][N] partial planes (nsplit > 1)
  float* out;          // MTTKRP: F (M x N); Gram: G (R x R)
  double* epart;       // error: per-unit {sum (W-rec)^2, sum W^2}
  double* eout;        // error: caller's result slot
  int unit0, nunits;   // error: this job's unit range
  int epi;             // MTTKRP (spatial form): 0 F = sum_s acc_s . E[s,:], 1 F[s,:] = sum_rows E . acc_s
};
struct AlsUnit { int job, tm, tn, ks; };

// q = k / d, r = k % d for 0 <= k < 2^24 and d >= 1 by a float reciprocal estimate and
// one correction step each way (exact: k * (1/d) is within one of the true quotient).
__device__ __forceinline__ int divmod(int k, int d, float inv, int& r) {
  int q = (int)((float)k * inv);
  r = k - q * d;
  if (r < 0) { q -= 1; r += d; }
  if (r >= d) { q += 1; r -= d; }
  return q;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 a;
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
  return a;
}

// Operand value at (row, k) of the A side and (k, col) of the B side, per kind.
// Callers guarantee the indices are in range.
__device__ __forceinline__ float opA(const AlsJob& j, int kind, int m, int k, int which) {
  if (kind == 0) {
    int kr = 0;
    const int kq = j.K2 == 1 ? k : divmod(k, j.K2, j.invK2, kr);
    return j.W[(long long)m * j.sm + (long long)kq * j.s1 + (long long)kr * j.s2];
  }
  if (kind == 1) return (which ? j.Y : j.X)[(long long)k * j.R + m];   // X^T: A(m=r1, k=i) = X[i, r1]
  return j.X[(long long)m * j.R + k];                                   // error: A(m=a, k=r) = A[a, r]
}
__device__ __forceinline__ float opB(const AlsJob& j, int kind, int k, int n, int which) {
  if (kind == 0) {
    if (!j.Y) return j.X[(long long)k * j.N + n];
    int kr;
    const int kq = divmod(k, j.K2, j.invK2, kr);
    return j.X[(long long)kq * j.N + n] * j.Y[(long long)kr * j.N + n];
  }
  if (kind == 1) return (which ? j.Y : j.X)[(long long)k * j.R + n];
  // error: B(k=r, n) = B[n / Kc, r] * C[n % Kc, r]   (Kc = K2 here)
  if (!j.Z) return j.Y[(long long)n * j.R + k];
  int nr;
  const int nq = divmod(n, j.K2, j.invK2, nr);
  return j.Y[(long long)nq * j.R + k] * j.Z[(long long)nr * j.R + k];
}

// The GEMM core: acc (this wave's 32 x 32 sub-tile at (32 wm, 32 wn) of the BM x 64
// tile at (m0, n0)) += sum over k in [kb, ke) of A(m, k) B(k, n).
// Operand images in LDS are k-major ([k][row], rows contiguous): the MFMA fragment of
// lane (i, h) is image[2q + h][32 w + i], 32 consecutive floats per half-wave, and the
// row stride is 32 mod 64 floats so the two half-waves use disjoint banks.
// A-side staging maps threads along rows when `afast` (W_(n) rows contiguous in
// memory) and along k otherwise; the B side always runs along its columns, which are
// contiguous for every kind except the error's KR operand (along k).
template <int BM>
struct Stage {
  static constexpr int NT = 2 * BM * 2;          // 4 waves (BM 64) or 2 waves (BM 32)
  static constexpr int LDA = BM % 64 == 0 ? BM + 32 : BM, LDB = kAlsBN + 32;   // row stride = 32 mod 64 floats
  static constexpr int PA = kAlsBK * BM / NT;     // A elements per thread per K-step
  static constexpr int PB = kAlsBK * kAlsBN / NT; // B elements per thread per K-step
};

template <int BM>
__device__ __forceinline__ void als_core(const AlsJob& j, int kind, int which, bool afast, bool bfast, int m0,
                                         int n0, int kb, int ke, int Mrows, int Ncols, f32x16& acc,
                                         float (*sA)[kAlsBK * Stage<BM>::LDA],
                                         float (*sB)[kAlsBK * Stage<BM>::LDB]) {
  using S = Stage<BM>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (BM == 64) ? (wave >> 1) : 0, wn = wave & 1;
  const int i = lane & 31, h = lane >> 5;
  float ra[S::PA], rb[S::PB];
  auto load = [&](int k0) {
#pragma unroll
    for (int e = 0; e < S::PA; ++e) {
      const int x = tid + S::NT * e;
      const int r = afast ? x % BM : x / kAlsBK, kk = afast ? x / BM : x % kAlsBK;
      const int m = m0 + r, k = k0 + kk;
      ra[e] = (m < Mrows && k < ke) ? opA(j, kind, m, k, which) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < S::PB; ++e) {
      const int x = tid + S::NT * e;
      const int c = bfast ? x % kAlsBN : x / kAlsBK, kk = bfast ? x / kAlsBN : x % kAlsBK;
      const int n = n0 + c, k = k0 + kk;
      rb[e] = (n < Ncols && k < ke) ? opB(j, kind, k, n, which) : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < S::PA; ++e) {
      const int x = tid + S::NT * e;
      const int r = afast ? x % BM : x / kAlsBK, kk = afast ? x / BM : x % kAlsBK;
      sA[buf][kk * S::LDA + r] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < S::PB; ++e) {
      const int x = tid + S::NT * e;
      const int c = bfast ? x % kAlsBN : x / kAlsBK, kk = bfast ? x / kAlsBN : x % kAlsBK;
      sB[buf][kk * S::LDB + c] = rb[e];
    }
  };
  if (kb >= ke) return;
  load(kb);
  __syncthreads();   // the previous use of the LDS images (an earlier core call) is done
  store(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += kAlsBK) {
    const bool more = k0 + kAlsBK < ke;
    if (more) load(k0 + kAlsBK);
    const float* a = sA[buf] + 32 * wm + i;
    const float* b = sB[buf] + 32 * wn + i;
#pragma unroll
    for (int q = 0; q < kAlsBK / 2; ++q)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[(2 * q + h) * S::LDA], b[(2 * q + h) * S::LDB], acc, 0, 0, 0);
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
}

// C/D map of v_mfma_f32_32x32x2_f32: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#define ALS_ROW(r) ((r & 3) + 8 * (r >> 2) + 4 * h)

template <int BM>
__global__ __launch_bounds__(Stage<BM>::NT) void k_als_mttkrp(const AlsJob* __restrict__ jobs,
                                                              const AlsUnit* __restrict__ units) {
  __shared__ __attribute__((aligned(16))) float sA[2][kAlsBK * Stage<BM>::LDA];
  __shared__ __attribute__((aligned(16))) float sB[2][kAlsBK * Stage<BM>::LDB];
  const AlsUnit u = units[blockIdx.x];
  const AlsJob& j = jobs[u.job];
  const int m0 = u.tm * BM, n0 = u.tn * kAlsBN;
  const int kb = u.ks * j.kchunk, ke = min(j.K, kb + j.kchunk);
  f32x16 acc = zero16();
  als_core<BM>(j, 0, 0, j.afast != 0, true, m0, n0, kb, ke, j.M, j.N, acc, sA, sB);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (BM == 64) ? (wave >> 1) : 0, wn = wave & 1, i = lane & 31, h = lane >> 5;
  const int col = n0 + 32 * wn + i;
  float* dst = j.nsplit > 1 ? j.part + (size_t)u.ks * j.M * j.N : j.out;
  if (col < j.N) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + 32 * wm + ALS_ROW(r);
      if (row < j.M) dst[(size_t)row * j.N + col] = acc[r];
    }
  }
}

// MTTKRP of a 3-way layer W[I][J][KD] (KD = 9, the flattened 3 x 3 kernel) as KD GEMMs
// over one shared factor operand (scripts/factorize.py:217,227,237, the einsum of W with
// the Khatri-Rao product of the other two factors, regrouped):
//   mode 0: acc_s[i,r] = sum_j W[i,j,s] B[j,r]     F[i,r] = sum_s acc_s[i,r] C[s,r]
//   mode 1: acc_s[j,r] = sum_i W[i,j,s] A[i,r]     F[j,r] = sum_s acc_s[j,r] C[s,r]
//   mode 2: acc_s[i,r] = sum_j W[i,j,s] B[j,r]     F[s,r] = sum_i A[i,r] acc_s[i,r]
// (job: rows M, reduction K, X = the MFMA factor (K x R), Y = the epilogue factor E).
// Per K-step the tile's W block is BM x 16 x KD floats: modes 0, 2 read each row's
// 16 KD contiguous floats, mode 1 each reduction row's BM KD contiguous floats; it is
// stored as KD k-major planes (the als_core image, one per s), and each B fragment read
// from LDS feeds KD MFMAs. Mode 2 reduces over the tile's rows in the epilogue (fixed
// order: lane rows, half-waves, waves) into one partial plane per row tile, summed in
// tile order by k_als_reduce.
template <int BM, int KD>
__global__ __launch_bounds__(Stage<BM>::NT) __attribute__((amdgpu_waves_per_eu(2)))
void k_als_mttkrp_sp(const AlsJob* __restrict__ jobs, const AlsUnit* __restrict__ units) {
  using S = Stage<BM>;
  static_assert(S::NT == 4 * BM && KD == 9, "36 floats (9 float4) of W per thread per K-step");
  constexpr int PL = kAlsBK * S::LDA + 8;                 // plane stride (staggers the s planes' banks)
  __shared__ __attribute__((aligned(16))) float sA[KD * PL];
  __shared__ __attribute__((aligned(16))) float sB[kAlsBK * S::LDB];
  __shared__ float red[2][KD][32];
  const AlsUnit u = units[blockIdx.x];
  const AlsJob& j = jobs[u.job];
  const int m0 = u.tm * BM, n0 = u.tn * kAlsBN;
  const int M = j.M, N = j.N, K = j.K;
  const float* __restrict__ X = j.X;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (BM == 64) ? (wave >> 1) : 0, wn = wave & 1, i = lane & 31, h = lane >> 5;
  // Each thread stages 36 contiguous floats of W per K-step (9 float4; the planner
  // guarantees K % 16 == 0, M % 4 == 0, 16-byte aligned runs). Modes 0, 2 (rows are the
  // runs): BM rows x 144 floats, thread -> row tid % BM, quarter q = tid / BM (reduction
  // rows 4q..4q+3, all s); a wave's LDS stores then hit 64 consecutive rows. Mode 1
  // (reduction rows are the runs): 16 runs x 9 BM floats, thread -> run tid / (BM / 4),
  // q = tid % (BM / 4) (tile rows 4q..4q+3, all s).
  const bool rmaj = j.afast == 0;   // block-uniform
  int run, q;
  if (rmaj) { run = tid % BM; q = tid / BM; }
  else { run = tid / (BM / 4); q = tid % (BM / 4); }
  const bool wvalid = rmaj ? (m0 + run < M) : (m0 + 4 * q < M);
  const float* wp = rmaj ? j.W + (long long)(m0 + run) * j.sm + 36 * q
                         : j.W + (long long)run * j.s1 + (long long)m0 * KD + 36 * q;
  const long long kstep = rmaj ? (long long)kAlsBK * KD : (long long)kAlsBK * j.s1;   // W floats per K-step
  // LDS image of float t (0..35) of the run: plane t % 9, at sbase + (t / 9) * (rmaj ? LDA : 1)
  float* const sbase = sA + (rmaj ? 4 * q * S::LDA + run : run * S::LDA + 4 * q);
  float4 ra[9];
  float rb[S::PB];
  auto load = [&](int ks) {
    const float* p = wp + ks * kstep;
#pragma unroll
    for (int e = 0; e < 9; ++e) ra[e] = wvalid ? gld4(p + 4 * e) : make_float4(0.f, 0.f, 0.f, 0.f);
    const int k0 = ks * kAlsBK;
#pragma unroll
    for (int e = 0; e < S::PB; ++e) {
      const int x = tid + S::NT * e;
      const int c = x % kAlsBN, kk = x / kAlsBN;
      const int n = n0 + c;
      rb[e] = n < N ? *(gcf32*)(X + (long long)(k0 + kk) * N + n) : 0.f;
    }
  };
  f32x16 acc[KD];
#pragma unroll
  for (int s = 0; s < KD; ++s) acc[s] = zero16();
  const int nks = K / kAlsBK;
  load(0);
  for (int ks = 0; ks < nks; ++ks) {
    __syncthreads();   // the previous K-step's fragment reads are done
    auto stage = [&](auto step) {   // step: LDS distance of consecutive reduction / tile rows
#pragma unroll
      for (int e = 0; e < 9; ++e) {
        const float f[4] = {ra[e].x, ra[e].y, ra[e].z, ra[e].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int t = 4 * e + c;
          sbase[(t % 9) * PL + (t / 9) * decltype(step)::value] = f[c];
        }
      }
    };
    if (rmaj) stage(std::integral_constant<int, S::LDA>());
    else stage(std::integral_constant<int, 1>());
#pragma unroll
    for (int e = 0; e < S::PB; ++e) {
      const int x = tid + S::NT * e;
      sB[(x / kAlsBN) * S::LDB + x % kAlsBN] = rb[e];
    }
    __syncthreads();
    if (ks + 1 < nks) load(ks + 1);   // in flight under the MFMAs
    const float* a = sA + 32 * wm + i;
    const float* b = sB + 32 * wn + i;
#pragma unroll
    for (int q = 0; q < kAlsBK / 2; ++q) {
      const float bv = b[(2 * q + h) * S::LDB];
#pragma unroll
      for (int s = 0; s < KD; ++s)
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s * PL + (2 * q + h) * S::LDA], bv, acc[s], 0, 0, 0);
    }
  }
  const int col = n0 + 32 * wn + i;
  const float* __restrict__ E = j.Y;
  if (j.epi == 0) {   // modes 0, 1: F[row, col] = sum_s acc_s[row, col] E[s, col]
    if (col >= N) return;
    float ev[KD];
#pragma unroll
    for (int s = 0; s < KD; ++s) ev[s] = E[(long long)s * N + col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row < M) {
        float v = acc[0][r] * ev[0];
#pragma unroll
        for (int s = 1; s < KD; ++s) v += acc[s][r] * ev[s];
        j.out[(long long)row * N + col] = v;
      }
    }
    return;
  }
  // mode 2: F[s, col] (partial over this tile's rows) = sum_row E[row, col] acc_s[row, col]
  float ev[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
    ev[r] = (row < M && col < N) ? E[(long long)row * N + col] : 0.f;
  }
  float v[KD];
#pragma unroll
  for (int s = 0; s < KD; ++s) {
    float t = acc[s][0] * ev[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) t += acc[s][r] * ev[r];
    v[s] = t + __shfl_xor(t, 32);   // the two half-waves' rows (same sum on both)
  }
  if (BM == 64) {
    if (wm == 1 && h == 0) {
#pragma unroll
      for (int s = 0; s < KD; ++s) red[wn][s][i] = v[s];
    }
    __syncthreads();
    if (wm == 1) return;
#pragma unroll
    for (int s = 0; s < KD; ++s) v[s] += red[wn][s][i];
  }
  if (h != 0 || col >= N) return;
  float* dst = j.nsplit > 1 ? j.part + (size_t)u.ks * KD * N : j.out;
#pragma unroll
  for (int s = 0; s < KD; ++s) dst[(size_t)s * N + col] = v[s];
}

template <int BM>
__global__ __launch_bounds__(Stage<BM>::NT) void k_als_gram(const AlsJob* __restrict__ jobs,
                                                            const AlsUnit* __restrict__ units) {
  __shared__ __attribute__((aligned(16))) float sA[2][kAlsBK * Stage<BM>::LDA];
  __shared__ __attribute__((aligned(16))) float sB[2][kAlsBK * Stage<BM>::LDB];
  const AlsUnit u = units[blockIdx.x];
  const AlsJob& j = jobs[u.job];
  const int m0 = u.tm * BM, n0 = u.tn * kAlsBN;
  f32x16 acc = zero16();
  als_core<BM>(j, 1, 0, true, true, m0, n0, 0, j.K, j.R, j.R, acc, sA, sB);
  if (j.Kx > 0) {   // Hadamard factor (scripts/factorize.py:215: B.T @ B * (C.T @ C)), its own fp32 Gram first
    f32x16 acc2 = zero16();
    als_core<BM>(j, 1, 1, true, true, m0, n0, 0, j.Kx, j.R, j.R, acc2, sA, sB);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc[r] * acc2[r];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (BM == 64) ? (wave >> 1) : 0, wn = wave & 1, i = lane & 31, h = lane >> 5;
  const int col = n0 + 32 * wn + i;
  if (col < j.R) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + 32 * wm + ALS_ROW(r);
      if (row < j.R) j.out[(size_t)row * j.R + col] = acc[r];
    }
  }
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// E1: per unit, the BM x 64 tile of rec = A (B ⊙ C)^T, then sum (W - rec)^2 and W^2
// over the tile's valid entries into fp64 (lane, wave, block in fixed order).
template <int BM>
__global__ __launch_bounds__(Stage<BM>::NT) void k_als_error(const AlsJob* __restrict__ jobs,
                                                             const AlsUnit* __restrict__ units) {
  using S = Stage<BM>;
  __shared__ __attribute__((aligned(16))) float sA[2][kAlsBK * S::LDA];
  __shared__ __attribute__((aligned(16))) float sB[2][kAlsBK * S::LDB];
  __shared__ double red[2][S::NT / 64];
  const AlsUnit u = units[blockIdx.x];
  const AlsJob& j = jobs[u.job];
  const int m0 = u.tm * BM, n0 = u.tn * kAlsBN;
  f32x16 acc = zero16();
  als_core<BM>(j, 2, 0, false, false, m0, n0, 0, j.R, j.M, j.N, acc, sA, sB);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (BM == 64) ? (wave >> 1) : 0, wn = wave & 1, i = lane & 31, h = lane >> 5;
  const int col = n0 + 32 * wn + i;
  double e2 = 0.0, w2 = 0.0;
  if (col < j.N) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + 32 * wm + ALS_ROW(r);
      if (row < j.M) {
        const float w = j.W[(size_t)row * j.N + col];
        const float d = w - acc[r];
        e2 += (double)d * (double)d;
        w2 += (double)w * (double)w;
      }
    }
  }
  e2 = wave_sum_f64(e2);
  w2 = wave_sum_f64(w2);
  if (lane == 0) { red[0][wave] = e2; red[1][wave] = w2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < S::NT / 64; ++w) { a += red[0][w]; b += red[1][w]; }
    j.epart[2 * (size_t)blockIdx.x] = a;
    j.epart[2 * (size_t)blockIdx.x + 1] = b;
  }
}
#undef ALS_ROW

// MTTKRP split-K: F = sum over chunks s (in order) of part[s]. grid.y = job.
__global__ __launch_bounds__(256) void k_als_reduce(const AlsJob* __restrict__ jobs, const int* __restrict__ ids) {
  const AlsJob& j = jobs[ids[blockIdx.y]];
  const size_t n = (size_t)(j.kind == 3 ? j.K2 : j.M) * j.N;   // spatial form: KD x R planes
  for (size_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (size_t)gridDim.x * 256) {
    float s = j.part[e];
    for (int q = 1; q < j.nsplit; ++q) s += j.part[(size_t)q * n + e];
    j.out[e] = s;
  }
}

// E1: per job, sqrt(sum e2 / sum w2) over its units in unit order (source/admm.py:15).
__global__ __launch_bounds__(64) void k_als_error_final(const AlsJob* __restrict__ jobs, int njobs) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= njobs) return;
  const AlsJob& j = jobs[t];
  double a = 0.0, b = 0.0;
  for (int q = 0; q < j.nunits; ++q) { a += j.epart[2 * (size_t)(j.unit0 + q)]; b += j.epart[2 * (size_t)(j.unit0 + q) + 1]; }
  j.eout[0] = sqrt(a / b);
}

// ---------------------------------------------------------------------------------
// Host planning

static inline size_t al(size_t v) { return (v + 255) / 256 * 256; }
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

struct AlsPlan {
  std::vector<AlsJob> jobs;
  std::vector<AlsUnit> units[2][4];   // [BM 32 / 64][kind] (kind 3: MTTKRP, spatial form)
  std::vector<int> split_ids;         // MTTKRP jobs with nsplit > 1
  size_t bytes = 0;
};

static int bm_index(int M) { return M <= 32 ? 0 : 1; }

// Tiles x K chunks: enough units to fill the chip twice over (~2048), chunks of at
// least 512 reduction rows.
static int choose_split(int tiles, int K) {
  const int by_k = std::max(1, K / 512);
  const int by_fill = std::max(1, 2048 / std::max(tiles, 1));
  return std::max(1, std::min(by_k, by_fill));
}

static bool layer_ok(const admmq_cp_layer& L) {
  if (!L.W || (L.ndim != 2 && L.ndim != 3) || L.R < 1) return false;
  for (int d = 0; d < L.ndim; ++d)
    if (L.dims[d] < 1 || !L.factors[d]) return false;
  return true;
}

// Carve order: [jobs][units x 6][split ids][partials | error partials]
static int plan_als(const admmq_cp_layer* layers, int n, int mode, int kind, double* eout, void* base, AlsPlan& pl,
                    std::string& err) {
  pl.jobs.clear();
  for (auto& a : pl.units)
    for (auto& b : a) b.clear();
  pl.split_ids.clear();
  int err_units = 0;
  for (int l = 0; l < n; ++l) {
    const admmq_cp_layer& L = layers[l];
    if (!layer_ok(L)) { err = "cp layer " + std::to_string(l) + ": bad W/factors/dims/ndim/R"; return ADMMQ_ERR_ARG; }
    const int I = L.dims[0], J = L.dims[1], Kd = L.ndim == 3 ? L.dims[2] : 1, R = L.R;
    if ((long long)I * J * Kd >= (1LL << 31)) { err = "cp layer too large"; return ADMMQ_ERR_ARG; }
    if (kind != 2 && (mode < 0 || mode >= L.ndim)) { err = "mode out of range"; return ADMMQ_ERR_ARG; }
    AlsJob j;
    std::memset(&j, 0, sizeof(j));
    j.kind = kind;
    j.W = L.W;
    const int sp_rows = mode == 1 ? J : I, sp_red = mode == 1 ? I : J;
    if (kind == 0 && L.ndim == 3 && Kd == kSpatialKD && sp_red % kAlsBK == 0 && sp_rows % 4 == 0 && J % 4 == 0 &&
        (reinterpret_cast<uintptr_t>(L.W) & 15) == 0) {   // MTTKRP, spatial form (k_als_mttkrp_sp)
      const long long JK = (long long)J * Kd;
      j.kind = 3; j.N = R; j.K2 = Kd; j.epi = mode == 2;
      if (mode == 1) { j.M = J; j.K = I; j.sm = Kd; j.s1 = JK; j.X = L.factors[0]; j.Y = L.factors[2]; j.afast = 1; }
      else { j.M = I; j.K = J; j.sm = JK; j.s1 = Kd; j.X = L.factors[1]; j.Y = L.factors[mode == 0 ? 2 : 0]; j.afast = 0; }
      if (base && !L.F) { err = "cp layer: F output missing"; return ADMMQ_ERR_ARG; }
      j.out = L.F;
      const int bi = bm_index(j.M), BM = bi ? 64 : 32;
      const int tm = cdiv(j.M, BM), tn = cdiv(j.N, kAlsBN);
      j.nsplit = mode == 2 ? tm : 1;   // mode 2: one partial plane per row tile
      if (j.nsplit > 1) pl.split_ids.push_back(l);
      for (int a = 0; a < tm; ++a)
        for (int b = 0; b < tn; ++b) pl.units[bi][3].push_back({l, a, b, a});
    } else if (kind == 0) {   // MTTKRP of mode `mode` (k order: see the file header)
      const long long JK = (long long)J * Kd;
      j.N = R;
      if (L.ndim == 3) {
        j.M = L.dims[mode];
        if (mode == 0) { j.K = J * Kd; j.K2 = Kd; j.sm = JK; j.s1 = Kd; j.s2 = 1; j.X = L.factors[1]; j.Y = L.factors[2]; j.afast = 0; }
        if (mode == 1) { j.K = I * Kd; j.K2 = Kd; j.sm = Kd; j.s1 = JK; j.s2 = 1; j.X = L.factors[0]; j.Y = L.factors[2]; j.afast = 0; }
        if (mode == 2) { j.K = I * J; j.K2 = J; j.sm = 1; j.s1 = JK; j.s2 = Kd; j.X = L.factors[0]; j.Y = L.factors[1]; j.afast = 1; }
      } else {
        j.K2 = 1; j.s2 = 0;
        if (mode == 0) { j.M = I; j.K = J; j.sm = J; j.s1 = 1; j.X = L.factors[1]; j.afast = 0; }
        else           { j.M = J; j.K = I; j.sm = 1; j.s1 = J; j.X = L.factors[0]; j.afast = 1; }
      }
      if (base && !L.F) { err = "cp layer: F output missing"; return ADMMQ_ERR_ARG; }
      j.out = L.F;
      const int bi = bm_index(j.M), BM = bi ? 64 : 32;
      const int tm = cdiv(j.M, BM), tn = cdiv(j.N, kAlsBN);
      j.nsplit = choose_split(tm * tn, j.K);
      j.kchunk = cdiv(cdiv(j.K, j.nsplit), kAlsBK) * kAlsBK;
      j.nsplit = cdiv(j.K, j.kchunk);
      if (j.nsplit > 1) pl.split_ids.push_back(l);
      for (int ks = 0; ks < j.nsplit; ++ks)
        for (int a = 0; a < tm; ++a)
          for (int b = 0; b < tn; ++b) pl.units[bi][0].push_back({l, a, b, ks});
    } else if (kind == 1) {   // Gram(-Hadamard) of the factors other than `mode`
      int o[2], no = 0;
      for (int d = 0; d < L.ndim; ++d)
        if (d != mode) o[no++] = d;
      if (base && !L.G) { err = "cp layer: G output missing"; return ADMMQ_ERR_ARG; }
      j.R = R; j.M = j.N = R;
      j.X = L.factors[o[0]]; j.K = L.dims[o[0]];
      if (no == 2) { j.Y = L.factors[o[1]]; j.Kx = L.dims[o[1]]; }
      j.out = L.G;
      const int bi = bm_index(R), BM = bi ? 64 : 32;
      for (int a = 0; a < cdiv(R, BM); ++a)
        for (int b = 0; b < cdiv(R, kAlsBN); ++b) pl.units[bi][1].push_back({l, a, b, 0});
    } else {   // reconstruction error: rec (I x J*K) = A . (B ⊙ C)^T
      j.R = R; j.M = I; j.N = J * Kd; j.K2 = Kd;
      j.X = L.factors[0]; j.Y = L.factors[1]; j.Z = L.ndim == 3 ? L.factors[2] : nullptr;
      j.eout = eout + l;
      const int bi = bm_index(I), BM = bi ? 64 : 32;
      j.unit0 = (int)pl.units[bi][2].size();
      for (int a = 0; a < cdiv(I, BM); ++a)
        for (int b = 0; b < cdiv(j.N, kAlsBN); ++b) pl.units[bi][2].push_back({l, a, b, 0});
      j.nunits = (int)pl.units[bi][2].size() - j.unit0;
    }
    j.invK2 = 1.0f / (float)std::max(j.K2, 1);
    if (j.kind != 3 && j.K2 > 1 && (kind == 0 ? j.K : j.N) >= (1 << 24)) {   // divmod's exact range
      err = "cp layer " + std::to_string(l) + ": Khatri-Rao index range >= 2^24";
      return ADMMQ_ERR_ARG;
    }
    pl.jobs.push_back(j);
  }
  // carve
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b ? b + off : nullptr; off += al(nbytes); return p; };
  char* djobs = take(pl.jobs.size() * sizeof(AlsJob));
  size_t nu = 0;
  for (auto& a : pl.units)
    for (auto& u : a) nu += u.size();
  take(nu * sizeof(AlsUnit));
  take(pl.split_ids.size() * sizeof(int) + 4);
  // error units index epart by their launch's blockIdx: one array per BM class
  size_t eunits[2] = {pl.units[0][2].size(), pl.units[1][2].size()};
  double* ep[2];
  ep[0] = reinterpret_cast<double*>(take(2 * eunits[0] * sizeof(double) + 16));
  ep[1] = reinterpret_cast<double*>(take(2 * eunits[1] * sizeof(double) + 16));
  (void)djobs;
  (void)err_units;
  for (auto& j : pl.jobs) {
    if (j.kind == 0 && j.nsplit > 1) j.part = reinterpret_cast<float*>(take((size_t)j.nsplit * j.M * j.N * 4));
    if (j.kind == 3 && j.nsplit > 1) j.part = reinterpret_cast<float*>(take((size_t)j.nsplit * j.K2 * j.N * 4));
    if (j.kind == 2) j.epart = ep[bm_index(j.M)];
  }
  pl.bytes = off + 256;
  return ADMMQ_OK;
}

static int run_als(const AlsPlan& pl, void* base, size_t wsb, hipStream_t s, std::string& err) {
  if (!base || wsb < pl.bytes) { err = "workspace too small"; return ADMMQ_ERR_WORKSPACE; }
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t nbytes) -> char* { char* p = b + off; off += al(nbytes); return p; };
  AlsJob* djobs = reinterpret_cast<AlsJob*>(take(pl.jobs.size() * sizeof(AlsJob)));
  size_t nu = 0;
  for (auto& a : pl.units)
    for (auto& u : a) nu += u.size();
  AlsUnit* dunits = reinterpret_cast<AlsUnit*>(take(nu * sizeof(AlsUnit)));
  int* dids = reinterpret_cast<int*>(take(pl.split_ids.size() * sizeof(int) + 4));
  auto up = [&](void* dst, const void* src, size_t nbytes) {
    return upload_async(dst, src, nbytes, s) == ADMMQ_OK;   // pinned staging: never waits for the stream
  };
  std::vector<AlsUnit> all;
  all.reserve(nu);
  size_t first[2][4];
  for (int bi = 0; bi < 2; ++bi)
    for (int k = 0; k < 4; ++k) { first[bi][k] = all.size(); all.insert(all.end(), pl.units[bi][k].begin(), pl.units[bi][k].end()); }
  if (!up(djobs, pl.jobs.data(), pl.jobs.size() * sizeof(AlsJob)) || !up(dunits, all.data(), nu * sizeof(AlsUnit)) ||
      !up(dids, pl.split_ids.data(), pl.split_ids.size() * sizeof(int))) {
    err = "als descriptor upload failed";
    return ADMMQ_ERR_HIP;
  }
  for (int bi = 0; bi < 2; ++bi)
    for (int k = 0; k < 4; ++k) {
      const int n = (int)pl.units[bi][k].size();
      if (!n) continue;
      const AlsUnit* u = dunits + first[bi][k];
      const dim3 g(n), t(bi ? Stage<64>::NT : Stage<32>::NT);
      if (k == 0) {
        if (bi) hipLaunchKernelGGL(k_als_mttkrp<64>, g, t, 0, s, djobs, u);
        else hipLaunchKernelGGL(k_als_mttkrp<32>, g, t, 0, s, djobs, u);
      } else if (k == 1) {
        if (bi) hipLaunchKernelGGL(k_als_gram<64>, g, t, 0, s, djobs, u);
        else hipLaunchKernelGGL(k_als_gram<32>, g, t, 0, s, djobs, u);
      } else if (k == 2) {
        if (bi) hipLaunchKernelGGL(k_als_error<64>, g, t, 0, s, djobs, u);
        else hipLaunchKernelGGL(k_als_error<32>, g, t, 0, s, djobs, u);
      } else {
        if (bi) hipLaunchKernelGGL((k_als_mttkrp_sp<64, kSpatialKD>), g, t, 0, s, djobs, u);
        else hipLaunchKernelGGL((k_als_mttkrp_sp<32, kSpatialKD>), g, t, 0, s, djobs, u);
      }
    }
  if (!pl.split_ids.empty()) {
    size_t mx = 0;
    for (int id : pl.split_ids) mx = std::max(mx, (size_t)pl.jobs[id].M * pl.jobs[id].N);
    const int nb = (int)std::min<size_t>(256, (mx + 255) / 256);
    hipLaunchKernelGGL(k_als_reduce, dim3(nb, (unsigned)pl.split_ids.size()), dim3(256), 0, s, djobs, dids);
  }
  if (!pl.jobs.empty() && pl.jobs[0].kind == 2)
    hipLaunchKernelGGL(k_als_error_final, dim3(cdiv((long long)pl.jobs.size(), 64)), dim3(64), 0, s, djobs,
                       (int)pl.jobs.size());
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("als launch: ") + hipGetErrorString(e); return ADMMQ_ERR_HIP; }
  return ADMMQ_OK;
}

}  // namespace admmq

using namespace admmq;

extern "C" {

size_t admmq_cp_workspace_size(const admmq_cp_layer* layers, int32_t n, int32_t mode) {
  AlsPlan g, f, e;
  std::string err;
  if (plan_als(layers, n, mode, 1, nullptr, nullptr, g, err) || plan_als(layers, n, mode, 0, nullptr, nullptr, f, err))
    return 0;
  if (plan_als(layers, n, 0, 2, nullptr, nullptr, e, err)) return 0;
  return std::max(std::max(g.bytes, f.bytes), e.bytes);
}

int32_t admmq_cp_gram_mttkrp(const admmq_cp_layer* layers, int32_t n, int32_t mode, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (n < 0 || (n > 0 && !layers)) return set_error(ADMMQ_ERR_ARG, "cp_gram_mttkrp: bad layer array");
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int kind = 1; kind >= 0; --kind) {
    AlsPlan pl;
    std::string err;
    int rc = plan_als(layers, n, mode, kind, nullptr, workspace, pl, err);
    if (!rc) rc = run_als(pl, workspace, workspace_bytes, s, err);
    if (rc) return set_error(rc, ("cp_gram_mttkrp: " + err).c_str());
  }
  return ADMMQ_OK;
}

int32_t admmq_cp_rel_error(const admmq_cp_layer* layers, int32_t n, double* out, void* workspace,
                           size_t workspace_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!layers || !out))) return set_error(ADMMQ_ERR_ARG, "cp_rel_error: bad arguments");
  AlsPlan pl;
  std::string err;
  int rc = plan_als(layers, n, 0, 2, out, workspace, pl, err);
  if (!rc) rc = run_als(pl, workspace, workspace_bytes, static_cast<hipStream_t>(stream), err);
  if (rc) return set_error(rc, ("cp_rel_error: " + err).c_str());
  return ADMMQ_OK;
}

}  // extern "C"
