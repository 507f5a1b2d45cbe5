// ADMM primal solve (source/admm.py:56-57):  H_T = (F + rho(H+U)) (G + rho I)^-1
// as one grouped fp32-MFMA GEMM  HT[Ip x ld] = P[Ip x ld] . M[ld x ld]  over every
// active (layer, mode) problem. P is produced by the previous iteration's
// finalize kernel; M is symmetric, so the B operand is read as rows of M.
//
// Tile (32*WM) x 64 per workgroup of 2*WM waves; wave (wm, wn) owns the 32 x 32
// sub-tile at (32 wm, 32 wn) with one v_mfma_f32_32x32x2_f32 accumulator chain
// (16 accumulator registers). WM = 2 (64 x 64 tiles, 256 threads) for factors with
// I > 32, WM = 1 (32 x 64, 128 threads) for the 9-row mode-C factors.
// K-step 32 = 16 MFMAs per wave between barriers, double-buffered through LDS with
// register prefetch of the next K-step. The LDS images keep k permuted as
// [row][h][m] (k = 2m + h) so a lane's 16 operands for a K-step are 64 contiguous
// bytes (4 x ds_read_b128); rows padded to 144 B (conflict-free b128 reads).
//
// Epilogue: store HT, X = HT - U, and fold max|X|, min X, max X of the valid
// region into the problem's per-iteration stat slot (one atomic each per block).
#include "quant_device.h"

namespace admmq {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BN = 64, BK = 32, LROW = 36;  // LDS row = 32 floats + 4 pad

__device__ __forceinline__ bool converged_before(const ProbDesc& p, int slot_prev, int iter, float eps) {
  if (iter == 0) return false;
  const double* r = p.res + 4 * slot_prev;
  const double rr = r[0] / r[1];
  const double ss = r[2] / r[3];
  return (rr < (double)eps) && (ss < (double)eps);
}

template <int WM>
__global__ __launch_bounds__(128 * WM) void k_gemm(const ProbDesc* __restrict__ probs, const GemmTile* __restrict__ tiles,
                                                   int slot, int iter, float eps, int ncand) {
  constexpr int BM = 32 * WM;
  constexpr int NT = 128 * WM;                 // threads
  constexpr int AV = BM * (BK / 4) / NT;       // float4 loads of A per thread per K-step (= 2)
  constexpr int BV = BN * (BK / 4) / NT;       // float4 loads of B per thread per K-step (= 4 / WM)
  const GemmTile tl = tiles[blockIdx.x];
  const ProbDesc& p = probs[tl.prob];
  if (p.flags[0]) return;
  if (converged_before(p, slot ^ 1, iter, eps)) {
    if (tl.first && threadIdx.x == 0) p.flags[0] = 1;   // sticky "break" (source/admm.py:64-65)
    return;
  }
  if (tl.first) {   // this iteration's quantizer-search accumulators start at zero
    unsigned long long* sse = p.mv.sse + (size_t)slot * ncand;
    unsigned long long* h1 = p.mv.h1 + (size_t)slot * kHistRep * (ncand + 1);
    unsigned long long* h2 = p.mv.h2 + (size_t)slot * kHistRep * (ncand + 1);
    for (int c = threadIdx.x; c < ncand; c += NT) sse[c] = 0ull;
    for (int c = threadIdx.x; c < kHistRep * (ncand + 1); c += NT) { h1[c] = 0ull; h2[c] = 0ull; }
    if (threadIdx.x == 0) p.mv.s2[slot] = 0.0;
  }

  __shared__ __attribute__((aligned(16))) float As[2][BM * LROW];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / 2, wn = wave & 1;
  const int ld = p.ld, ldm = p.ldm;
  const int row0 = tl.tm * BM, col0 = tl.tn * BN;
  const float* __restrict__ P = p.P;
  const float* __restrict__ M = p.M;

  // staging: element v of thread t covers row (t + v*NT) / 8, k-quad (t % 8)
  const int kq = tid & 7;
  const int r0 = tid >> 3;
  float4 ra[AV], rb[BV];
  auto gload = [&](int k0) {
#pragma unroll
    for (int v = 0; v < AV; ++v)
      ra[v] = *reinterpret_cast<const float4*>(P + (size_t)(row0 + r0 + v * (NT / 8)) * ld + k0 + 4 * kq);
#pragma unroll
    for (int v = 0; v < BV; ++v)
      rb[v] = *reinterpret_cast<const float4*>(M + (size_t)(col0 + r0 + v * (NT / 8)) * ldm + k0 + 4 * kq);
  };
  auto sstore = [&](int b) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      float* a = &As[b][(r0 + v * (NT / 8)) * LROW + 2 * kq];
      *reinterpret_cast<float2*>(a) = make_float2(ra[v].x, ra[v].z);
      *reinterpret_cast<float2*>(a + 16) = make_float2(ra[v].y, ra[v].w);
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      float* bb = &Bs[b][(r0 + v * (NT / 8)) * LROW + 2 * kq];
      *reinterpret_cast<float2*>(bb) = make_float2(rb[v].x, rb[v].z);
      *reinterpret_cast<float2*>(bb + 16) = make_float2(rb[v].y, rb[v].w);
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  const int i = lane & 31, h = lane >> 5;
  const int nk = ld / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const float4* ap = reinterpret_cast<const float4*>(&As[cur][(32 * wm + i) * LROW + 16 * h]);
    const float4* bp = reinterpret_cast<const float4*>(&Bs[cur][(32 * wn + i) * LROW + 16 * h]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a = ap[q], b = bp[q];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int col = col0 + 32 * wn + i;
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  if (col < ld) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + 32 * wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      const size_t off = (size_t)row * ld + col;
      const float ht = acc[r];
      const float x = ht - p.U[off];
      p.HT[off] = ht;
      p.X[off] = x;
      if (row < p.I && col < p.R) {
        amax = max(amax, __float_as_uint(x) & 0x7FFFFFFFu);
        const unsigned e = enc_ord(x);
        mn = min(mn, e);
        mxo = max(mxo, e);
      }
    }
  }
  amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
  __shared__ unsigned red[3][2 * WM];
  if (lane == 0) { red[0][wave] = amax; red[1][wave] = mn; red[2][wave] = mxo; }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < 2 * WM; ++w) {
      red[0][0] = max(red[0][0], red[0][w]); red[1][0] = min(red[1][0], red[1][w]); red[2][0] = max(red[2][0], red[2][w]);
    }
    unsigned* st = p.mv.stat + 4 * slot;
    atomicMax(&st[0], red[0][0]);
    atomicMin(&st[1], red[1][0]);
    atomicMax(&st[2], red[2][0]);
  }
}

void launch_gemm(const ProbDesc* d, const GemmTile* tiles, int ntiles_small, int ntiles_big, int slot, int iter,
                 float eps, int ncand, hipStream_t s) {
  // tiles[0 .. ntiles_big) are 64x64 (WM=2), then ntiles_small 32x64 tiles (WM=1)
  if (ntiles_big > 0)
    hipLaunchKernelGGL(k_gemm<2>, dim3(ntiles_big), dim3(256), 0, s, d, tiles, slot, iter, eps, ncand);
  if (ntiles_small > 0)
    hipLaunchKernelGGL(k_gemm<1>, dim3(ntiles_small), dim3(128), 0, s, d, tiles + ntiles_big, slot, iter, eps, ncand);
}

}  // namespace admmq
