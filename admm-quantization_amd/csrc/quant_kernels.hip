// Standalone quantize_tensor kernels (source/quantization.py:69-115): pack + tensor
// statistics, and the final elementwise quantization with the resolved parameters.
// The MSE-minmax candidate search itself lives in mse_search.hip.
#include "quant_device.h"

namespace admmq {

// Standalone statistics of a tensor (source/quantization.py:72-76: min, max, abs max) and,
// when cols % 4 != 0, the zero-padded copy rows x ld. One unit = kPackElems elements; each
// unit's block writes its three partials (plain stores, no same-address atomics: 16 k blocks
// of one 4096 x 4096 tensor serialized on three words took 565 us); k_qstat folds them.
__global__ __launch_bounds__(256) void k_qpack(const QJob* __restrict__ jobs, const Chunk* __restrict__ chunks) {
  const Chunk ck = chunks[blockIdx.x];
  const QJob& j = jobs[ck.job];
  const long long total = (long long)j.rows * j.ld;
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  auto acc = [&](float v) {
    amax = max(amax, __float_as_uint(v) & 0x7FFFFFFFu);
    mn = min(mn, enc_ord(v));
    mxo = max(mxo, enc_ord(v));
  };
  if (!j.copy) {   // rows are already ld wide (ld == cols): read in place, 16 float4 per thread
    float4 v[kPackElems / 1024];
#pragma unroll
    for (int k = 0; k < kPackElems / 1024; ++k) {
      const long long e = (long long)ck.start + 4LL * threadIdx.x + 1024LL * k;
      v[k] = e < total ? *reinterpret_cast<const float4*>(j.src + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < kPackElems / 1024; ++k) {
      const long long e = (long long)ck.start + 4LL * threadIdx.x + 1024LL * k;
      if (e < total) { acc(v[k].x); acc(v[k].y); acc(v[k].z); acc(v[k].w); }
    }
  } else {
    for (int k = 0; k < kPackElems / 1024; ++k) {
      const long long e = (long long)ck.start + 4LL * threadIdx.x + 1024LL * k;
      if (e >= total) break;
      const int row = (int)(e / j.ld);
      const int c0 = (int)(e - (long long)row * j.ld);
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + q;
        v[q] = c < j.cols ? j.src[(size_t)row * j.cols + c] : 0.f;
        if (c < j.cols) acc(v[q]);
      }
      *reinterpret_cast<float4*>(j.Xp + e) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  __shared__ unsigned red[3][4];
  amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = amax; red[1][w] = mn; red[2][w] = mxo; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      amax = max(amax, red[0][k]); mn = min(mn, red[1][k]); mxo = max(mxo, red[2][k]);
    }
    unsigned* o = j.pstat + 3 * (size_t)(blockIdx.x - j.pu0);
    o[0] = amax; o[1] = mn; o[2] = mxo;
  }
}

// one block per tensor: its units' partials -> stat[0..2] (max / min / max: order-free)
__global__ __launch_bounds__(256) void k_qstat(const QJob* __restrict__ jobs) {
  const QJob& j = jobs[blockIdx.x];
  unsigned amax = 0u, mn = 0xFFFFFFFFu, mxo = 0u;
  for (int u = threadIdx.x; u < j.pun; u += blockDim.x) {
    amax = max(amax, j.pstat[3 * u + 0]);
    mn = min(mn, j.pstat[3 * u + 1]);
    mxo = max(mxo, j.pstat[3 * u + 2]);
  }
  __shared__ unsigned red[3][4];
  amax = wave_max_u32(amax); mn = wave_min_u32(mn); mxo = wave_max_u32(mxo);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = amax; red[1][w] = mn; red[2][w] = mxo; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      amax = max(amax, red[0][k]); mn = min(mn, red[1][k]); mxo = max(mxo, red[2][k]);
    }
    j.mv.stat[0] = amax; j.mv.stat[1] = mn; j.mv.stat[2] = mxo;
  }
}

__global__ __launch_bounds__(256) void k_qfinal(const QJob* __restrict__ jobs, const Chunk* __restrict__ chunks,
                                                int ncand, int bits, int scheme) {
  const Chunk ck = chunks[blockIdx.x];
  const QJob& j = jobs[ck.job];
  const QParams qp = block_qparams(scheme, bits, j.mv, 0, ncand, j.has_kw, j.tmin_kw, j.tmax_kw);
  const long long total = (long long)j.rows * j.ld;
  const long long e = (long long)ck.start + 4LL * threadIdx.x;
  if (e >= total) return;
  const int row = (int)(e / j.ld);
  const int c0 = (int)(e - (long long)row * j.ld);
  const float4 v = *reinterpret_cast<const float4*>(j.Xp + e);
  const float xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + k;
    if (c < j.cols) j.dst[(size_t)row * j.cols + c] = apply_quant(xv[k], qp);
  }
}

// Per-channel schemes (channel_symmetric / channel_affine with an explicit dim,
// source/quantization.py:29-33, 91-106). The tensor is viewed as (A, C, B) around the
// channel dimension dim (C = shape[dim]); channel r = row r of unfold(x, dim)
// (source/utils.py:60-74). gridDim.y blocks per channel (large channels split over
// several), merged by atomics into stats zeroed beforehand: {~min, max} as order-preserving
// encodings (min stored complemented so every word starts at 0), plus a NaN flag (torch's
// max / min propagate NaN).
__global__ __launch_bounds__(256) void k_channel_stats(const float* __restrict__ x, long long A, int C, long long B,
                                                       unsigned* __restrict__ stats) {
  const int r = blockIdx.x;
  const long long n = A * B;
  unsigned mn = 0xFFFFFFFFu, mxo = 0u, nan = 0u;
  const long long step = (long long)blockDim.x * gridDim.y;
  for (long long t = (long long)blockIdx.y * blockDim.x + threadIdx.x; t < n; t += step) {
    const long long a = t / B, b = t - a * B;
    const float v = x[(a * C + r) * B + b];
    if (v != v) {
      nan = 1u;
    } else {
      const unsigned e = enc_ord(v);
      mn = min(mn, e);
      mxo = max(mxo, e);
    }
  }
  __shared__ unsigned red[3][4];
  mn = wave_min_u32(mn); mxo = wave_max_u32(mxo); nan = wave_max_u32(nan);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = mn; red[1][w] = mxo; red[2][w] = nan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      mn = min(mn, red[0][k]); mxo = max(mxo, red[1][k]); nan = max(nan, red[2][k]);
    }
    atomicMax(&stats[3 * r + 0], ~mn);
    atomicMax(&stats[3 * r + 1], mxo);
    atomicMax(&stats[3 * r + 2], nan);
  }
}

// y (outer x Lo) = the scheme applied to x (outer x L) with the statistics of channel
// (C == 1 ? 0 : j) for output column j: torch broadcasts the (C,) statistics against the
// tensor's last dimension (the host checked L == C or one of them is 1; Lo = max(L, C)).
// Grid-stride over the outputs (the grid is capped; outputs may exceed 2^32).
__device__ __noinline__ void channel_quant_one(const float* __restrict__ x, float* __restrict__ y, long long i, int L,
                                               int Lo, int C, const unsigned* __restrict__ stats, int bits, int scheme) {
  const long long o = i / Lo;
  const int j = (int)(i - o * Lo);
  const int ci = C == 1 ? 0 : j;
  const float tmin = dec_ord(~stats[3 * ci + 0]), tmax = dec_ord(stats[3 * ci + 1]);
  const QParams qp = qparams_stats(scheme, bits, tmin, tmax, (int)stats[3 * ci + 2], 0, 0.f, 0.f);
  y[i] = apply_quant(x[o * L + (L == 1 ? 0 : j)], qp);
}
__global__ __launch_bounds__(256) void k_channel_quant(const float* __restrict__ x, float* __restrict__ y,
                                                       long long nout, int L, int Lo, int C,
                                                       const unsigned* __restrict__ stats, int bits, int scheme) {
  const long long step = (long long)blockDim.x * gridDim.x;
  for (long long i0 = (long long)blockIdx.x * blockDim.x; i0 < nout; i0 += step) {
    const long long i = i0 + threadIdx.x;
    if (i >= nout) break;
    channel_quant_one(x, y, i, L, Lo, C, stats, bits, scheme);
  }
}

void launch_channel_quant(const float* x, float* y, long long A, int C, long long B, long long outer, int L, int Lo,
                          unsigned* stats, int bits, int scheme, hipStream_t s) {
  // blocks per channel: about 16 k elements each, at most 2048 blocks in all beyond one per channel
  const long long n = A * B;
  long long per = (n + 16383) / 16384;
  const long long cap = 2048LL / C > 1 ? 2048LL / C : 1;
  if (per > cap) per = cap;
  if (per < 1) per = 1;
  (void)hipMemsetAsync(stats, 0, (size_t)3 * C * sizeof(unsigned), s);
  hipLaunchKernelGGL(k_channel_stats, dim3(C, (unsigned)per), dim3(256), 0, s, x, A, C, B, stats);
  const long long nout = outer * Lo;
  long long nblk = (nout + 255) / 256;
  if (nblk > (1LL << 20)) nblk = 1LL << 20;
  if (nblk < 1) nblk = 1;
  hipLaunchKernelGGL(k_channel_quant, dim3((unsigned)nblk), dim3(256), 0, s, x, y, nout, L, Lo, C,
                     stats, bits, scheme);
}

void launch_qpack(const QJob* jobs, int njobs, const Chunk* chunks, int nchunks, hipStream_t s) {
  if (nchunks > 0) hipLaunchKernelGGL(k_qpack, dim3(nchunks), dim3(256), 0, s, jobs, chunks);
  if (njobs > 0) hipLaunchKernelGGL(k_qstat, dim3(njobs), dim3(256), 0, s, jobs);
}
void launch_qfinal(const QJob* jobs, const Chunk* chunks, int nchunks, int ncand, int bits, int qscheme,
                   hipStream_t s) {
  if (nchunks > 0)
    hipLaunchKernelGGL(k_qfinal, dim3(nchunks), dim3(256), 0, s, jobs, chunks, ncand, bits, qscheme);
}

}  // namespace admmq
