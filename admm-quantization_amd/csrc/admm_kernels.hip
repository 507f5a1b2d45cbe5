// ADMM per-call setup and per-iteration finalize (source/admm.py:51-67).
//
//   k_rho        rho = trace(G)/R                       (admm.py:53; trace accumulated in fp64 like torch-CPU)
//   k_pack       padded Fp/H/U copies, P = F + rho(H+U)  (admm.py:56, first iteration's right-hand side)
//   k_fill_a64   A = G + rho I in fp64 for the SPD inverse (admm.py:54)
//   k_finalize   H = Q(X), X = H_T - U re-formed here, with the chosen scale, U += H - H_T, next P = F + rho(H+U),
//                residual sums for the r/s stop test  (admm.py:59-65)
//   k_unpack     padded H/U -> caller tensors
#include "quant_device.h"

namespace admmq {

__global__ __launch_bounds__(256) void k_rho(const ProbDesc* __restrict__ probs) {
  const ProbDesc& p = probs[blockIdx.x];
  double s = 0.0;
  for (int i = threadIdx.x; i < p.R; i += blockDim.x) s += (double)p.G_user[(size_t)i * p.R + i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    // sequential-order fp64 sum is not required: trace of <= 1500 fp32 values is exact in fp64
    const double tr = red[0] + red[1] + red[2] + red[3];
    p.rho[0] = (float)tr / (float)p.R;
    p.flags[0] = 0; p.flags[1] = 0; p.flags[2] = 0; p.flags[3] = 0;
    for (int sl = 0; sl < 2; ++sl) {
      unsigned* st = p.mv.stat + 4 * sl;
      st[0] = 0u; st[1] = 0xFFFFFFFFu; st[2] = 0u; st[3] = 0u;
      for (int k = 0; k < 4 * kResRep; ++k) p.res[4 * kResRep * sl + k] = 0.0;
    }
  }
}

__global__ __launch_bounds__(256) void k_pack(const ProbDesc* __restrict__ probs) {
  const ProbDesc& p = probs[blockIdx.y];
  const float rho = p.rho[0];
  const long long total = (long long)p.Ip * p.ld;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / p.ld), c = (int)(e - (long long)r * p.ld);
    float f = 0.f, h = 0.f, u = 0.f, pv = 0.f;
    if (r < p.I && c < p.R) {
      const size_t o = (size_t)r * p.R + c;
      f = p.F_user[o]; h = p.H0_user[o]; u = p.U_user[o];
      pv = f + rho * (h + u);
    }
    p.Fp[e] = f; p.H[e] = h; p.U[e] = u; p.P[e] = pv; p.X[e] = 0.f; p.HT[e] = 0.f;
  }
}

__global__ __launch_bounds__(256) void k_fill_a64(const ProbDesc* __restrict__ probs) {
  const ProbDesc& p = probs[blockIdx.y];
  const float rho = p.rho[0];
  const long long total = (long long)p.ldm * p.ldm;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / p.ldm), c = (int)(e - (long long)r * p.ldm);
    double v;
    if (r < p.R && c < p.R) {
      const float g = p.G_user[(size_t)r * p.R + c];
      v = (r == c) ? (double)(g + rho * 1.0f) : (double)(g + rho * 0.0f);   // G + rho*eye, in fp32
    } else {
      v = (r == c) ? 1.0 : 0.0;
    }
    p.A64[e] = v;
  }
}

// Work unit = whole rows [start / ld, total / ld) of one problem (at most 1024 G
// elements), so a split problem's next P gets its exact per-row exponent in one pass.
template <int G>   // float4 groups per thread: 256 G * 4 elements per work unit
__global__ __launch_bounds__(256) void k_finalize_admm(const ProbDesc* __restrict__ probs, const Chunk* __restrict__ chunks,
                                                       int ncand, int bits, int scheme, int slot, int iter) {
  constexpr int kMaxRows = 1024 * G / 32;   // ld >= 32
  __shared__ unsigned rmax[kMaxRows];
  const Chunk ck = chunks[blockIdx.x];
  // float4 group g of thread t at start + 4 t + 1024 g. The stop flag and the search
  // record (max|x|, |S| and its first entry: the chosen candidate whenever |S| = 1), then
  // the element loads, straight from the unit (no descriptor read first; past the end a
  // clamped address, never used): one level of dependent loads before everything is in
  // flight. The rare |S| > 1 record is resolved by block_qparams (canonical SSEs).
  const long long total = ck.total;   // end of this unit
  const int stopped = gld_i32(ck.done);
  const unsigned ab = gld_u32(ck.stat + 4 * slot);
  const int* selp = ck.sel + (size_t)slot * (2 + kMaxSel);
  const int nsel = gld_i32(selp), sel0 = gld_i32(selp + 2);
  float4 t4[G], h4[G], u4[G], f4[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const long long e = (long long)ck.start + 4LL * threadIdx.x + 1024LL * g;
    const long long ec = e < total ? e : 0;
    t4[g] = gld4(ck.X + ec);
    h4[g] = gld4(ck.H + ec);
    u4[g] = gld4(ck.U + ec);
    f4[g] = gld4(ck.F + ec);
  }
  const ProbDesc& p = probs[ck.job];
  if (stopped) return;   // converged earlier (sticky break)
  const QParams qp = (scheme == kMse && nsel == 1 && !mse_degenerate(__uint_as_float(ab)))
                         ? qparams_mse(bits, cand_t(__uint_as_float(ab), sel0, ncand))
                         : block_qparams(scheme, bits, p.mv, slot, ncand, 0, 0.f, 0.f);   // (ends with a barrier)
  admm_finalize_block<256, G>(p, ck.start, total, t4, u4, h4, f4, qp, slot, iter, blockIdx.x & (kResRep - 1), rmax);
}

__global__ __launch_bounds__(256) void k_unpack(const ProbDesc* __restrict__ probs) {
  const ProbDesc& p = probs[blockIdx.y];
  const long long total = (long long)p.I * p.R;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / p.R), c = (int)(e - (long long)r * p.R);
    const size_t o = (size_t)r * p.ld + c;
    if (p.H_out) p.H_out[e] = p.H[o];
    if (p.U_user) p.U_user[e] = p.U[o];
    if (p.HT_dbg) p.HT_dbg[e] = p.HT[o];
    if (p.X_dbg) p.X_dbg[e] = p.X[o];
  }
}

void launch_rho(const ProbDesc* d, int nprob, hipStream_t s) {
  hipLaunchKernelGGL(k_rho, dim3(nprob), dim3(256), 0, s, d);
}
void launch_pack(const ProbDesc* d, int nprob, int maxIp, int maxld, hipStream_t s) {
  const long long tot = (long long)maxIp * maxld;
  const int nb = (int)std::min<long long>(1024, (tot + 255) / 256);
  hipLaunchKernelGGL(k_pack, dim3(nb, nprob), dim3(256), 0, s, d);
}
void launch_fill_a64(const ProbDesc* d, int nprob, int maxldm, hipStream_t s) {
  const long long tot = (long long)maxldm * maxldm;
  const int nb = (int)std::min<long long>(1024, (tot + 255) / 256);
  hipLaunchKernelGGL(k_fill_a64, dim3(nb, nprob), dim3(256), 0, s, d);
}
void launch_finalize_admm(const ProbDesc* d, const Chunk* chunks, int nchunks, int groups, int ncand, int bits,
                          int qscheme, int slot, int iter, hipStream_t s) {
  if (nchunks <= 0) return;
#define ADMMQ_FIN(G) \
  hipLaunchKernelGGL(k_finalize_admm<G>, dim3(nchunks), dim3(256), 0, s, d, chunks, ncand, bits, qscheme, slot, iter)
  switch (groups) {
    case 1: ADMMQ_FIN(1); break;
    case 2: ADMMQ_FIN(2); break;
    case 4: ADMMQ_FIN(4); break;
    default: ADMMQ_FIN(8); break;
  }
#undef ADMMQ_FIN
}
void launch_unpack(const ProbDesc* d, int nprob, int maxI, int maxR, hipStream_t s) {
  const long long tot = (long long)maxI * maxR;
  const int nb = (int)std::min<long long>(1024, (tot + 255) / 256);
  hipLaunchKernelGGL(k_unpack, dim3(nb, nprob), dim3(256), 0, s, d);
}

}  // namespace admmq
