// ADMM primal solve (source/admm.py:56-57):  H_T = (F + rho(H+U)) (G + rho I)^-1
// as one grouped fp32-MFMA GEMM  HT[Ip x ld] = P[Ip x ld] . M[ld x ld]  over every
// active (layer, mode) problem. P is produced by the previous iteration's
// finalize kernel; M is symmetric, so the B operand is read as rows of M.
//
// Tile 32 x 64 per 128-thread workgroup; wave w owns the 32 x 32 sub-tile at
// columns 32w with one v_mfma_f32_32x32x2_f32 accumulator chain (16 AGPRs).
// K-step 16 = 8 MFMAs per wave, double-buffered through LDS. The LDS images keep
// k permuted as [row][h][m] (k = 2m + h) so every lane's 8 operands for a K-step
// are 32 contiguous bytes (2 x ds_read_b128); rows padded to 80 B.
//
// Epilogue: store HT, X = HT - U, and fold max|X|, min X, max X of the valid
// region into the problem's per-iteration stat slot (one atomic each per block).
#include "quant_device.h"

namespace admmq {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 32, BN = 64, BK = 16, LROW = 20;  // LDS row = 16 floats + 4 pad

__device__ __forceinline__ bool converged_before(const ProbDesc& p, int slot_prev, int iter, float eps) {
  if (iter == 0) return false;
  const double* r = p.res + 4 * slot_prev;
  const double rr = r[0] / r[1];
  const double ss = r[2] / r[3];
  return (rr < (double)eps) && (ss < (double)eps);
}

__global__ __launch_bounds__(128) void k_gemm(const ProbDesc* __restrict__ probs, const GemmTile* __restrict__ tiles,
                                              int slot, int iter, float eps, int ncand) {
  const GemmTile tl = tiles[blockIdx.x];
  const ProbDesc& p = probs[tl.prob];
  if (p.flags[0]) return;
  if (converged_before(p, slot ^ 1, iter, eps)) {
    if (tl.first && threadIdx.x == 0) p.flags[0] = 1;   // sticky "break" (source/admm.py:64-65)
    return;
  }
  if (tl.first) {   // this iteration's quantizer-search accumulators start at zero
    unsigned long long* sse = p.mv.sse + (size_t)slot * ncand;
    unsigned long long* h1 = p.mv.h1 + (size_t)slot * (ncand + 1);
    unsigned long long* h2 = p.mv.h2 + (size_t)slot * (ncand + 1);
    for (int c = threadIdx.x; c <= ncand; c += blockDim.x) {
      if (c < ncand) sse[c] = 0ull;
      h1[c] = 0ull;
      h2[c] = 0ull;
    }
    if (threadIdx.x == 0) p.mv.s2[slot] = 0.0;
  }

  __shared__ __attribute__((aligned(16))) float As[2][BM * LROW];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ld = p.ld, ldm = p.ldm;
  const int row0 = tl.tm * BM, col0 = tl.tn * BN;
  const float* __restrict__ P = p.P;
  const float* __restrict__ M = p.M;

  // global -> register staging indices
  const int ar = tid >> 2, aq = tid & 3;            // A: 32 rows x 4 float4
  const float* aptr = P + (size_t)(row0 + ar) * ld + 4 * aq;
  const float* bptr0 = M + (size_t)(col0 + ar) * ldm + 4 * aq;        // B rows ar and ar+32
  const float* bptr1 = M + (size_t)(col0 + ar + 32) * ldm + 4 * aq;

  float4 ra, rb0, rb1;
  auto gload = [&](int k0) {
    ra = *reinterpret_cast<const float4*>(aptr + k0);
    rb0 = *reinterpret_cast<const float4*>(bptr0 + k0);
    rb1 = *reinterpret_cast<const float4*>(bptr1 + k0);
  };
  auto sstore = [&](int b) {
    float* a = &As[b][ar * LROW + 2 * aq];
    *reinterpret_cast<float2*>(a) = make_float2(ra.x, ra.z);
    *reinterpret_cast<float2*>(a + 8) = make_float2(ra.y, ra.w);
    float* b0 = &Bs[b][ar * LROW + 2 * aq];
    *reinterpret_cast<float2*>(b0) = make_float2(rb0.x, rb0.z);
    *reinterpret_cast<float2*>(b0 + 8) = make_float2(rb0.y, rb0.w);
    float* b1 = &Bs[b][(ar + 32) * LROW + 2 * aq];
    *reinterpret_cast<float2*>(b1) = make_float2(rb1.x, rb1.z);
    *reinterpret_cast<float2*>(b1 + 8) = make_float2(rb1.y, rb1.w);
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
    const float4* ap = reinterpret_cast<const float4*>(&As[cur][i * LROW + 8 * h]);
    const float4* bp = reinterpret_cast<const float4*>(&Bs[cur][(32 * wave + i) * LROW + 8 * h]);
    const float4 a0 = ap[0], a1 = ap[1], b0 = bp[0], b1 = bp[1];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b0.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b0.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, b0.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, b0.w, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b1.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b1.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, b1.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, b1.w, acc, 0, 0, 0);
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int col = col0 + 32 * wave + i;
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  if (col < ld) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
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
  __shared__ unsigned red[3][2];
  if (lane == 0) { red[0][wave] = amax; red[1][wave] = mn; red[2][wave] = mxo; }
  __syncthreads();
  if (tid == 0) {
    unsigned* st = p.mv.stat + 4 * slot;
    atomicMax(&st[0], max(red[0][0], red[0][1]));
    atomicMin(&st[1], min(red[1][0], red[1][1]));
    atomicMax(&st[2], max(red[2][0], red[2][1]));
  }
}

void launch_gemm(const ProbDesc* d, const GemmTile* tiles, int ntiles, int slot, int iter, float eps, int ncand,
                 hipStream_t s) {
  if (ntiles > 0) hipLaunchKernelGGL(k_gemm, dim3(ntiles), dim3(128), 0, s, d, tiles, slot, iter, eps, ncand);
}

}  // namespace admmq
