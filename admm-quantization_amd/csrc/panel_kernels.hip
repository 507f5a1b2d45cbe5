// Panel products of the low-rank projection (scripts/factorize_lowrank.py:80-82: the rank-r
// truncation of every inner step, done on the device by admmq.lowrank.KrylovProjector):
//
//   admmq_panel_xtq    Y = X^T Q   (n x k)   X: m x n float32 (the iterate), Q: m x k float64
//   admmq_panel_xy     Z = X Y     (m x k)   Y: n x k float64
//   admmq_panel_outer  O = A B^T   (m x n)   A: m x r, B: n x r float64, O float32 (rounded once)
//
// Block Krylov applies X X^T to a k = 32 column panel per block and K^T X / X V at its
// Rayleigh-Ritz checks. Each is one pass over X (64 MB for the notebook's 4096 x 4096
// q_proj) with ~32 fp64 FMAs per element: on v_mfma_f64_16x16x4_f64 the pass is balanced
// between HBM (64 MB at ~5 TB/s) and the fp64 matrix rate (m n k FMAs at 78.6 TF/s), and X
// is read as float32 and widened in registers (exact), never materialised in fp64. The
// library GEMMs this replaces read an fp64 copy of X (128 MB, made once per call).
//
// Work split (both products): a wave owns a 64 x 32 output tile (4 x 2 MFMA tiles, 64
// accumulator VGPRs) and one of 4G slices of the reduction; the 4 waves of a workgroup take
// consecutive slices of the same tile and are summed in wave order through LDS; the G
// workgroups of a tile hand their partials over (16-B sc1 stores, vmcnt(0), an agent-scope
// arrival counter that advances by G per call) and the last to arrive sums them in slice
// order. Every result is fixed by (m, n, k): no atomics on data, no schedule dependence.
//
// MFMA lane maps (cdna_hip_programming.md, f64 16x16x4): A[fr][fk], B[fk][fr] with
// fr = lane & 15, fk = lane >> 4; D: col = lane & 15, row = (lane >> 4) + 4 reg.
//   xtq: M = column j of X, N = column c of Q, K = row i.  Lane (fr, fk) loads the float4
//        X[i0 + fk][j0 + 4 fr .. + 3]; element t is the A operand of M-tile t, whose row r
//        is column j0 + 4 r + t (a permutation of the strip: coalesced 256-B rows).
//   xy:  M = row i of X, N = column c of Y, K = column j.  Lane (fr, fk) loads the float4
//        X[i0 + fr][j0 + 4 fk .. + 3]; element t is the A operand of the t-th MFMA of the
//        16-column chunk, whose K index fk is column j0 + 4 fk + t (B loads the same rows).
#include <algorithm>
#include <cstdint>

#include "../../include/admmq.h"
#include "admmq_internal.h"

namespace admmq {

typedef double f64x4p __attribute__((ext_vector_type(4)));
typedef unsigned u32x4p __attribute__((ext_vector_type(4)));

constexpr int kPanG = 4;          // workgroups per output tile (each 4 reduction slices)
constexpr int kPanSlices = 4 * kPanG;

__device__ __forceinline__ f64x4p pan_mfma(double a, double b, f64x4p c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// In-workgroup sum of the 4 waves' tiles (wave order), then the cross-workgroup hand-off.
// Returns true in wave 0 of the workgroup that holds the final sum in acc. ctr: the END of
// the counter array (tile t counts at ctr[-1 - t]).
__device__ __forceinline__ bool pan_combine(f64x4p (&acc)[4][2], double* part, unsigned* ctr, int tile) {
  __shared__ double red[3][32][64];   // 48 KB: [wave - 1][value][lane] (lane-contiguous: no conflicts)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w > 0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) red[w - 1][(a * 2 + u) * 4 + v][lane] = acc[a][u][v];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll 1
    for (int q = 0; q < 3; ++q)   // (one wave's 32 values in flight at a time)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[a][u][v] = acc[a][u][v] + red[q][(a * 2 + u) * 4 + v][lane];
    // publish this workgroup's partial: slot blockIdx.y of the tile, 16 x 16 B per lane
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(part + (size_t)tile * kPanG * 64 * 32, 0, kPanG * 64 * 32 * 8, 0x00020000);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const double d0 = acc[a][u][2 * h], d1 = acc[a][u][2 * h + 1];
          const u32x4p x = {(unsigned)__double_as_longlong(d0), (unsigned)(__double_as_longlong(d0) >> 32),
                            (unsigned)__double_as_longlong(d1), (unsigned)(__double_as_longlong(d1) >> 32)};
          const int q = (a * 2 + u) * 2 + h;   // 0..15
          __builtin_amdgcn_raw_buffer_store_b128(x, rs, ((blockIdx.y * 16 + q) * 64 + lane) * 16, 0, 16);   // sc1
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) {
      const unsigned old = __hip_atomic_fetch_add(ctr - 1 - tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = ((old + 1u) % (unsigned)kPanG) == 0u ? 1 : 0;
    }
    if (!__builtin_amdgcn_readfirstlane(last)) return false;   // (lane 0 is active: its value)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");     // the sc1 loads below stay after the arrival
    f64x4p sum[4][2];
#pragma unroll 1
    for (int g = 0; g < kPanG; ++g) {   // (one slot's 16 loads in flight at a time)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int q = (a * 2 + u) * 2 + h;
            double d0, d1;
            if (g == (int)blockIdx.y) {
              d0 = acc[a][u][2 * h]; d1 = acc[a][u][2 * h + 1];
            } else {
              const u32x4p x = __builtin_amdgcn_raw_buffer_load_b128(rs, ((g * 16 + q) * 64 + lane) * 16, 0, 16);
              d0 = __longlong_as_double((long long)(((unsigned long long)x[1] << 32) | x[0]));
              d1 = __longlong_as_double((long long)(((unsigned long long)x[3] << 32) | x[2]));
            }
            if (g == 0) { sum[a][u][2 * h] = d0; sum[a][u][2 * h + 1] = d1; }
            else { sum[a][u][2 * h] += d0; sum[a][u][2 * h + 1] += d1; }
          }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[a][u] = sum[a][u];
    return true;
  }
  return false;
}

// Y = X^T Q. grid (ceil(n / 64), kPanG, ceil(k / 32)), 256 threads.
template <bool V4>
__global__ __launch_bounds__(256, 2) void k_panel_xtq(const float* __restrict__ X, int m, int n, int ldx,
                                                   const double* __restrict__ Q, int k, double* __restrict__ Y,
                                                   double* __restrict__ part, unsigned* __restrict__ ctr) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int j0 = blockIdx.x * 64, c0 = blockIdx.z * 32;
  const int steps = (m + 3) >> 2;                       // K-steps of 4 rows
  const int per = (steps + kPanSlices - 1) / kPanSlices;
  const int slice = blockIdx.y * 4 + w;
  const int s0 = min(steps, slice * per), s1 = min(steps, s0 + per);
  const int jl = j0 + 4 * fr;
  const int cq0 = c0 + fr, cq1 = c0 + 16 + fr;
  f64x4p acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[a][u] = f64x4p{0.0, 0.0, 0.0, 0.0};
  auto load = [&](int s, float4& xv, double& q0, double& q1) {
    const int i = 4 * s + fk;
    xv = make_float4(0.f, 0.f, 0.f, 0.f);
    q0 = 0.0; q1 = 0.0;
    if (i < m) {
      const float* xr = X + (size_t)i * ldx;
      if constexpr (V4) {
        if (jl < n) xv = *reinterpret_cast<const float4*>(xr + jl);
      } else {
        if (jl < n) xv.x = xr[jl];
        if (jl + 1 < n) xv.y = xr[jl + 1];
        if (jl + 2 < n) xv.z = xr[jl + 2];
        if (jl + 3 < n) xv.w = xr[jl + 3];
      }
      if (cq0 < k) q0 = Q[(size_t)i * k + cq0];
      if (cq1 < k) q1 = Q[(size_t)i * k + cq1];
    }
  };
  float4 xv; double q0, q1;
  if (s0 < s1) load(s0, xv, q0, q1);
  for (int s = s0; s < s1; ++s) {
    const float4 xc = xv;
    const double b0 = q0, b1 = q1;
    if (s + 1 < s1) load(s + 1, xv, q0, q1);   // next step's operands in flight under this step's MFMAs
    const double av[4] = {(double)xc.x, (double)xc.y, (double)xc.z, (double)xc.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t][0] = pan_mfma(av[t], b0, acc[t][0]);
      acc[t][1] = pan_mfma(av[t], b1, acc[t][1]);
    }
  }
  const int tile = blockIdx.z * gridDim.x + blockIdx.x;
  if (!pan_combine(acc, part, ctr, tile)) return;
  // D of M-tile t, N-tile u: row r = (lane >> 4) + 4 v -> column j0 + 4 r + t; col -> c0 + 16 u + (lane & 15)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = c0 + 16 * u + (lane & 15);
      if (c >= k) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int j = j0 + 4 * ((lane >> 4) + 4 * v) + t;
        if (j < n) Y[(size_t)j * k + c] = acc[t][u][v];
      }
    }
}

// Z = X Y. grid (ceil(m / 64), kPanG, ceil(k / 32)), 256 threads.
template <bool V4>
__global__ __launch_bounds__(256, 2) void k_panel_xy(const float* __restrict__ X, int m, int n, int ldx,
                                                  const double* __restrict__ Yp, int k, double* __restrict__ Z,
                                                  double* __restrict__ part, unsigned* __restrict__ ctr) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int i0 = blockIdx.x * 64, c0 = blockIdx.z * 32;
  const int steps = (n + 15) >> 4;                      // K-steps of 16 columns
  const int per = (steps + kPanSlices - 1) / kPanSlices;
  const int slice = blockIdx.y * 4 + w;
  const int s0 = min(steps, slice * per), s1 = min(steps, s0 + per);
  const int cq0 = c0 + fr, cq1 = c0 + 16 + fr;
  f64x4p acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[a][u] = f64x4p{0.0, 0.0, 0.0, 0.0};
  auto load = [&](int s, float4 (&xv)[4], double (&yb)[4][2]) {
    const int jb = 16 * s + 4 * fk;   // this lane's 4 columns of the chunk
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int i = i0 + 16 * a + fr;
      xv[a] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < m) {
        const float* xr = X + (size_t)i * ldx;
        if constexpr (V4) {
          if (jb < n) xv[a] = *reinterpret_cast<const float4*>(xr + jb);
        } else {
          if (jb < n) xv[a].x = xr[jb];
          if (jb + 1 < n) xv[a].y = xr[jb + 1];
          if (jb + 2 < n) xv[a].z = xr[jb + 2];
          if (jb + 3 < n) xv[a].w = xr[jb + 3];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = jb + t;
      yb[t][0] = (j < n && cq0 < k) ? Yp[(size_t)j * k + cq0] : 0.0;
      yb[t][1] = (j < n && cq1 < k) ? Yp[(size_t)j * k + cq1] : 0.0;
    }
  };
  float4 xv[4];
  double yb[4][2];
  if (s0 < s1) load(s0, xv, yb);
  for (int s = s0; s < s1; ++s) {
    double av[4][4], bv[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      av[a][0] = xv[a].x; av[a][1] = xv[a].y; av[a][2] = xv[a].z; av[a][3] = xv[a].w;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) { bv[t][0] = yb[t][0]; bv[t][1] = yb[t][1]; }
    if (s + 1 < s1) load(s + 1, xv, yb);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[a][0] = pan_mfma(av[a][t], bv[t][0], acc[a][0]);
        acc[a][1] = pan_mfma(av[a][t], bv[t][1], acc[a][1]);
      }
  }
  const int tile = blockIdx.z * gridDim.x + blockIdx.x;
  if (!pan_combine(acc, part, ctr, tile)) return;
  // D of M-tile a, N-tile u: row (lane >> 4) + 4 v -> X row i0 + 16 a + ...; col -> c0 + 16 u + (lane & 15)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = c0 + 16 * u + (lane & 15);
      if (c >= k) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = i0 + 16 * a + (lane >> 4) + 4 * v;
        if (i < m) Z[(size_t)i * k + c] = acc[a][u][v];
      }
    }
}

// O = A B^T rounded to float32 once: thread (j4 = 4 columns) x 16 rows, B rows of its columns
// held in registers (RB = r rounded up to 8, 16 or 32: compile-time trip counts, so the
// rows stay in VGPRs), the A row broadcast. grid (ceil(n / 1024), ceil(m / 16)), 256 threads.
constexpr int kOuterRows = 16;
constexpr int kOuterMaxR = 32;
template <int RB>
__global__ __launch_bounds__(256) void k_panel_outer(const double* __restrict__ A, const double* __restrict__ B,
                                                     int m, int n, int r, float* __restrict__ O, int ldo) {
  const int j = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (j >= n) return;
  double bj[4][RB];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < RB; ++c) bj[q][c] = (c < r && j + q < n) ? B[(size_t)(j + q) * r + c] : 0.0;
  const int i0 = blockIdx.y * kOuterRows;
  for (int ii = 0; ii < kOuterRows; ++ii) {
    const int i = i0 + ii;
    if (i >= m) break;
    const double* ar = A + (size_t)i * r;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < RB; ++c) {
      const double a = c < r ? ar[c] : 0.0;   // (c >= r: b = 0 too, so the sum is unchanged)
#pragma unroll
      for (int q = 0; q < 4; ++q) s[q] = fma(a, bj[q][c], s[q]);
    }
    float* orow = O + (size_t)i * ldo;
    if (j + 3 < n && (ldo & 3) == 0) {
      *reinterpret_cast<float4*>(orow + j) = make_float4((float)s[0], (float)s[1], (float)s[2], (float)s[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j + q < n) orow[j + q] = (float)s[q];
    }
  }
}

// C = A^T B (p x q, float64) for tall A (m x p) and B (m x q): the Gram / cross products of
// the Krylov panels (Z^T Z of a block's Cholesky QR, K^T Z of the re-orthogonalization,
// B B^T of the Rayleigh-Ritz step). A wave owns a 32 x 32 tile (2 x 2 MFMA tiles) over
// m / (4 S) rows, the 4 waves of a workgroup consecutive row ranges (summed in wave order
// in LDS); grid (tiles, S); k_gram64_sum adds the S workgroup partials in order. Library
// GEMMs ran these (m = 4096, p = q = 32) on one workgroup: ~220 us each.
constexpr int kGramMaxS = 64;
__global__ __launch_bounds__(256) void k_gram64(const double* __restrict__ A, int lda, const double* __restrict__ B,
                                                int ldb, int m, int p, int q, double* __restrict__ part) {
  __shared__ double red[3][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int tq = (q + 31) / 32;
  const int p0 = (blockIdx.x / tq) * 32, q0 = (blockIdx.x % tq) * 32;
  const int S = gridDim.y;
  const int steps = (m + 3) >> 2;
  const int per = (steps + 4 * S - 1) / (4 * S);
  const int s0 = min(steps, (blockIdx.y * 4 + w) * per), s1 = min(steps, s0 + per);
  f64x4p acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[a][u] = f64x4p{0.0, 0.0, 0.0, 0.0};
  for (int st = s0; st < s1; ++st) {
    const int i = 4 * st + fk;
    double av[2], bv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int pc = p0 + 16 * t + fr, qc = q0 + 16 * t + fr;
      av[t] = (i < m && pc < p) ? A[(size_t)i * lda + pc] : 0.0;
      bv[t] = (i < m && qc < q) ? B[(size_t)i * ldb + qc] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[a][u] = pan_mfma(av[a], bv[u], acc[a][u]);
  }
  if (w > 0) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) red[w - 1][(a * 2 + u) * 4 + v][lane] = acc[a][u][v];
  }
  __syncthreads();
  if (w != 0) return;
  double* o = part + ((size_t)blockIdx.x * S + blockIdx.y) * 16 * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int x = (a * 2 + u) * 4 + v;
        o[x * 64 + lane] = ((acc[a][u][v] + red[0][x][lane]) + red[1][x][lane]) + red[2][x][lane];
      }
}

// the S partials of a tile in slice order: thread v of 256 sums values v, v + 256, ... of the
// tile's 1024 (x = value / 64, lane = value % 64), loads issued 8 slices ahead; then the D
// map (row (lane >> 4) + 4 v of the p-tile a, column lane & 15 of the q-tile u)
__global__ __launch_bounds__(256) void k_gram64_sum(const double* __restrict__ part, int S, int p, int q,
                                                    double* __restrict__ C, int ldc) {
  const int tq = (q + 31) / 32;
  const int p0 = (blockIdx.x / tq) * 32, q0 = (blockIdx.x % tq) * 32;
  const double* src = part + (size_t)blockIdx.x * S * 16 * 64;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int val = threadIdx.x + 256 * k;
    double sum = src[val];
#pragma unroll 8
    for (int g = 1; g < S; ++g) sum += src[(size_t)g * 1024 + val];
    const int x = val >> 6, lane = val & 63;
    const int a = x >> 3, u = (x >> 2) & 1, v = x & 3;
    const int r = p0 + 16 * a + (lane >> 4) + 4 * v, c = q0 + 16 * u + (lane & 15);
    if (r < p && c < q) C[(size_t)r * ldc + c] = sum;
  }
}

static int gram_slices(int64_t m) { return (int)std::max<int64_t>(1, std::min<int64_t>(kGramMaxS, (m + 255) / 256)); }
static size_t gram_bytes(int64_t m, int64_t p, int64_t q) {
  return (size_t)((p + 31) / 32) * (size_t)((q + 31) / 32) * gram_slices(m) * 16 * 64 * sizeof(double);
}

static size_t pan_align(size_t v) { return (v + 255) / 256 * 256; }

static size_t pan_tiles(int64_t rows, int64_t k) { return (size_t)((rows + 63) / 64) * (size_t)((k + 31) / 32); }

// Workspace: the partials from offset 0, the arrival counters at the END, counter t at
// end - 4 (t + 1): a tile's counter has the same address in every call on the workspace
// whatever the call's tile count (a later call with more tiles extends the counter region
// downwards, into bytes no call's partials reach: every call checks partials + counters fit).
static size_t pan_bytes(int64_t m, int64_t n, int64_t k) {
  const size_t tiles = std::max(pan_tiles(m, k), pan_tiles(n, k));
  return tiles * kPanG * 64 * 32 * sizeof(double) + pan_align(tiles * sizeof(unsigned));
}

static int pan_args(const float* X, int64_t m, int64_t n, int64_t ldx, const double* P, int64_t k, const double* Out,
                    void* ws, size_t wsb) {
  if (!X || !P || !Out || m <= 0 || n <= 0 || k <= 0 || ldx < n) return set_error(ADMMQ_ERR_ARG, "panel: bad arguments");
  if (m >= (1LL << 31) || n >= (1LL << 31) || k > 32LL * 65535 || (m + 63) / 64 > 2147483647LL)
    return set_error(ADMMQ_ERR_ARG, "panel: sizes out of range");
  if (!ws || wsb < pan_bytes(m, n, k)) return set_error(ADMMQ_ERR_WORKSPACE, "panel: workspace too small");
  return ADMMQ_OK;
}

}  // namespace admmq

using namespace admmq;

extern "C" {

size_t admmq_panel_workspace_size(int64_t m, int64_t n, int64_t k) {
  return (m <= 0 || n <= 0 || k <= 0) ? 0 : pan_bytes(m, n, k);
}

int32_t admmq_panel_xtq(const float* X, int64_t m, int64_t n, int64_t ldx, const double* Q, int64_t k, double* Y,
                        void* workspace, size_t workspace_bytes, void* stream) {
  if (const int rc = pan_args(X, m, n, ldx, Q, k, Y, workspace, workspace_bytes)) return rc;
  unsigned* ctr = reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + (workspace_bytes & ~(size_t)3));
  double* part = static_cast<double*>(workspace);
  const dim3 grid((unsigned)((n + 63) / 64), kPanG, (unsigned)((k + 31) / 32));
  const bool v4 = n % 4 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (v4)
    hipLaunchKernelGGL(k_panel_xtq<true>, grid, dim3(256), 0, s, X, (int)m, (int)n, (int)ldx, Q, (int)k, Y, part, ctr);
  else
    hipLaunchKernelGGL(k_panel_xtq<false>, grid, dim3(256), 0, s, X, (int)m, (int)n, (int)ldx, Q, (int)k, Y, part, ctr);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "panel_xtq: launch failed");
}

int32_t admmq_panel_xy(const float* X, int64_t m, int64_t n, int64_t ldx, const double* Y, int64_t k, double* Z,
                       void* workspace, size_t workspace_bytes, void* stream) {
  if (const int rc = pan_args(X, m, n, ldx, Y, k, Z, workspace, workspace_bytes)) return rc;
  unsigned* ctr = reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + (workspace_bytes & ~(size_t)3));
  double* part = static_cast<double*>(workspace);
  const dim3 grid((unsigned)((m + 63) / 64), kPanG, (unsigned)((k + 31) / 32));
  const bool v4 = n % 4 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (v4)
    hipLaunchKernelGGL(k_panel_xy<true>, grid, dim3(256), 0, s, X, (int)m, (int)n, (int)ldx, Y, (int)k, Z, part, ctr);
  else
    hipLaunchKernelGGL(k_panel_xy<false>, grid, dim3(256), 0, s, X, (int)m, (int)n, (int)ldx, Y, (int)k, Z, part, ctr);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "panel_xy: launch failed");
}

size_t admmq_gram64_workspace_size(int64_t m, int64_t p, int64_t q) {
  return (m <= 0 || p <= 0 || q <= 0) ? 0 : gram_bytes(m, p, q);
}

int32_t admmq_gram64(const double* A, int64_t lda, const double* B, int64_t ldb, int64_t m, int64_t p, int64_t q,
                     double* C, void* workspace, size_t workspace_bytes, void* stream) {
  if (!A || !B || !C || m <= 0 || p <= 0 || q <= 0 || lda < p || ldb < q)
    return set_error(ADMMQ_ERR_ARG, "gram64: bad arguments");
  if (m >= (1LL << 31) || p > 8192 || q > 8192) return set_error(ADMMQ_ERR_ARG, "gram64: sizes out of range");
  if (!workspace || workspace_bytes < gram_bytes(m, p, q)) return set_error(ADMMQ_ERR_WORKSPACE, "gram64: workspace too small");
  const int S = gram_slices(m);
  const unsigned tiles = (unsigned)(((p + 31) / 32) * ((q + 31) / 32));
  hipStream_t s = static_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(workspace);
  hipLaunchKernelGGL(k_gram64, dim3(tiles, S), dim3(256), 0, s, A, (int)lda, B, (int)ldb, (int)m, (int)p, (int)q, part);
  hipLaunchKernelGGL(k_gram64_sum, dim3(tiles), dim3(256), 0, s, part, S, (int)p, (int)q, C, (int)q);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "gram64: launch failed");
}

int32_t admmq_panel_outer(const double* A, const double* B, int64_t m, int64_t n, int64_t r, float* O, int64_t ldo,
                          void* stream) {
  if (!A || !B || !O || m <= 0 || n <= 0 || r <= 0 || ldo < n) return set_error(ADMMQ_ERR_ARG, "panel_outer: bad arguments");
  if (r > kOuterMaxR) return set_error(ADMMQ_ERR_ARG, "panel_outer: rank above 32");
  if (m >= (1LL << 31) || n >= (1LL << 31)) return set_error(ADMMQ_ERR_ARG, "panel_outer: sizes out of range");
  const dim3 grid((unsigned)((n + 1023) / 1024), (unsigned)((m + kOuterRows - 1) / kOuterRows));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (r <= 8)
    hipLaunchKernelGGL(k_panel_outer<8>, grid, dim3(256), 0, s, A, B, (int)m, (int)n, (int)r, O, (int)ldo);
  else if (r <= 16)
    hipLaunchKernelGGL(k_panel_outer<16>, grid, dim3(256), 0, s, A, B, (int)m, (int)n, (int)r, O, (int)ldo);
  else
    hipLaunchKernelGGL(k_panel_outer<32>, grid, dim3(256), 0, s, A, B, (int)m, (int)n, (int)r, O, (int)ldo);
  return hipGetLastError() == hipSuccess ? ADMMQ_OK : set_error(ADMMQ_ERR_HIP, "panel_outer: launch failed");
}

}  // extern "C"
