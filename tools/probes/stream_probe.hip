// Probe: per-CU read rate of one workgroup streaming its own region, by
//   mode 0: global_load_lds_dwordx4 into an NS-stage LDS ring (the GEMM's staging)
//   mode 1: global_load_dwordx4 into registers, NS-1 chunks in flight, then ds_write_b128
//   mode 2: as mode 0 with the GEMM's access pattern: per step 128 rows x 128 B at a row
//           stride of 1152 floats (region: kb must be 576 = 128 rows x 4.5 KiB)
//   mode 3..6: the GEMM K-loop on that pattern, {no fragment reads, no MFMA}, {reads},
//           {MFMA on constants}, {reads + MFMA} (36 steps per pass)
// One chunk = 16 KiB per workgroup step (256 threads x 4 x 16 B). Region per workgroup
// `kb` KiB, read `reps` times (the first pass warms the caches); `shared` = 1: every
// workgroup reads the same region (L2 hits), 0: private regions.
// usage: stream_probe <mode> <nblk> <kb> <reps> <shared>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void glds16(const float* g, float* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(g, lds, 16, 0, 0);
#endif
}
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int NS = 3;
constexpr int CH = 4096;   // floats per chunk (16 KiB)

__global__ __launch_bounds__(256) void k_glds(const float* src, long long per, int reps, int shared,
                                              unsigned long long* t, float* out) {
  __shared__ __attribute__((aligned(16))) float ring[NS][CH];
  const float* base = src + (shared ? 0 : per * blockIdx.x);
  const int nch = (int)(per / CH);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long t0 = 0;
  for (int r = 0; r < reps; ++r) {
    if (r == 1) { __syncthreads(); t0 = __builtin_amdgcn_s_memrealtime(); }
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(base + (size_t)s * CH + (w * 4 + j) * 256 + 4 * lane, &ring[s][(w * 4 + j) * 256]);
    for (int c = 0; c < nch; ++c) {
      wait_vm<4 * (NS - 2)>();
      asm volatile("s_barrier" ::: "memory");
      const int cn = c + NS - 1 < nch ? c + NS - 1 : nch - 1;
      const int sn = (c + NS - 1) % NS;
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(base + (size_t)cn * CH + (w * 4 + j) * 256 + 4 * lane, &ring[sn][(w * 4 + j) * 256]);
    }
    wait_vm<0>();
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = ring[0][threadIdx.x] + ring[1][threadIdx.x];
}

__global__ __launch_bounds__(256) void k_vgpr(const float* src, long long per, int reps, int shared,
                                              unsigned long long* t, float* out) {
  __shared__ __attribute__((aligned(16))) float ring[2][CH];
  const float* base = src + (shared ? 0 : per * blockIdx.x);
  const int nch = (int)(per / CH);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long t0 = 0;
  f4 buf[NS - 1][4];
  for (int r = 0; r < reps; ++r) {
    if (r == 1) { __syncthreads(); t0 = __builtin_amdgcn_s_memrealtime(); }
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        buf[s][j] = *(const __attribute__((address_space(1))) f4*)(base + (size_t)s * CH + (w * 4 + j) * 256 + 4 * lane);
    for (int c = 0; c < nch; c += NS - 1) {
#pragma unroll
      for (int s = 0; s < NS - 1; ++s) {
        wait_vm<4 * (NS - 2)>();
#pragma unroll
        for (int j = 0; j < 4; ++j) *(f4*)&ring[c & 1][(w * 4 + j) * 256 + 4 * lane] = buf[s][j];
        const int cn = c + s + NS - 1 < nch ? c + s + NS - 1 : nch - 1;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          buf[s][j] = *(const __attribute__((address_space(1))) f4*)(base + (size_t)cn * CH + (w * 4 + j) * 256 + 4 * lane);
      }
    }
    wait_vm<0>();
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = ring[0][threadIdx.x] + ring[1][threadIdx.x];
}

__global__ __launch_bounds__(256) void k_rows(const float* src, long long per, int reps, int shared,
                                              unsigned long long* t, float* out) {
  // the GEMM's pattern: per step 128 rows x 128 B (row stride kLd floats), column block c
  constexpr int kLd = 1152;
  __shared__ __attribute__((aligned(16))) float ring[NS][CH];
  const float* base = src + (shared ? 0 : per * blockIdx.x);
  const int nch = kLd / 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long t0 = 0;
  for (int r = 0; r < reps; ++r) {
    if (r == 1) { __syncthreads(); t0 = __builtin_amdgcn_s_memrealtime(); }
#define ROWSRC(c, j) (base + (size_t)(8 * (w * 4 + (j)) + (lane >> 3)) * kLd + (c) * 32 + 4 * (lane & 7))
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(ROWSRC(s, j), &ring[s][(w * 4 + j) * 256]);
    for (int c = 0; c < nch; ++c) {
      wait_vm<4 * (NS - 2)>();
      asm volatile("s_barrier" ::: "memory");
      const int cn = c + NS - 1 < nch ? c + NS - 1 : nch - 1;
      const int sn = (c + NS - 1) % NS;
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(ROWSRC(cn, j), &ring[sn][(w * 4 + j) * 256]);
    }
#undef ROWSRC
    wait_vm<0>();
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = ring[0][threadIdx.x] + ring[1][threadIdx.x];
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
// The GEMM's K-loop without its epilogue: per step wait + barrier + 4 glds per wave
// (128 rows x 128 B), then (FL) 8 ds_read_b128 fragment reads and (FM) 16 MFMAs.
template <int FL, int FM>
__global__ __launch_bounds__(256) void k_gemmlike(const float* src, long long per, int reps, int shared,
                                                  unsigned long long* t, float* out) {
  constexpr int kLd = 1152;
  __shared__ __attribute__((aligned(16))) float ring[NS][CH];
  const float* base = src + (shared ? 0 : per * blockIdx.x);
  const int nch = kLd / 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 31, h = lane >> 5, swz = (i >> 1) & 7;
  const int aoff = (32 * (w >> 1) + i) * 32, boff = (64 + 32 * (w & 1) + i) * 32;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  unsigned long long t0 = 0;
  for (int r = 0; r < reps; ++r) {
    if (r == 1) { __syncthreads(); t0 = __builtin_amdgcn_s_memrealtime(); }
#define ROWSRC(c, j) (base + (size_t)(8 * (w * 4 + (j)) + (lane >> 3)) * kLd + (c) * 32 + 4 * (lane & 7))
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(ROWSRC(s, j), &ring[s][(w * 4 + j) * 256]);
    for (int c0 = 0; c0 < nch; c0 += NS) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int c = c0 + s;
        wait_vm<4 * (NS - 2)>();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        asm volatile("s_barrier" ::: "memory");
        const int cn = c + NS - 1 < nch ? c + NS - 1 : nch - 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) glds16(ROWSRC(cn, j), &ring[(s + NS - 1) % NS][(w * 4 + j) * 256]);
        const float* st = ring[s];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int cpos = ((4 * h + qq) ^ swz) * 4;
          float4 a = make_float4(1.f, 1.f, 1.f, 1.f), b = a;
          if (FL) {
            a = *reinterpret_cast<const float4*>(st + aoff + cpos);
            b = *reinterpret_cast<const float4*>(st + boff + cpos);
          }
          if (FM) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
          } else {
            acc[qq] += a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
          }
        }
      }
    }
#undef ROWSRC
    wait_vm<0>();
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
  float sacc = 0.f;
  for (int r = 0; r < 16; ++r) sacc += acc[r];
  out[blockIdx.x * 256 + threadIdx.x] = sacc;
}

int main(int argc, char** argv) {
  if (argc < 6) { printf("usage: stream_probe mode nblk kb reps shared\n"); return 1; }
  const int mode = atoi(argv[1]), nblk = atoi(argv[2]), kb = atoi(argv[3]), reps = atoi(argv[4]), shared = atoi(argv[5]);
  const long long per = (long long)kb * 256;   // floats
  const size_t total = (size_t)per * (shared ? 1 : nblk);
  float* src; unsigned long long* t; float* out;
  if (hipMalloc(&src, total * 4) != hipSuccess || hipMalloc(&t, nblk * 8) != hipSuccess ||
      hipMalloc(&out, (size_t)nblk * 256 * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(src, 0, total * 4);
  for (int it = 0; it < 2; ++it) {
    if (mode == 0) hipLaunchKernelGGL(k_glds, dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    else if (mode == 1) hipLaunchKernelGGL(k_vgpr, dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    else if (mode == 2) hipLaunchKernelGGL(k_rows, dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    else if (mode == 3) hipLaunchKernelGGL((k_gemmlike<0, 0>), dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    else if (mode == 4) hipLaunchKernelGGL((k_gemmlike<1, 0>), dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    else if (mode == 5) hipLaunchKernelGGL((k_gemmlike<0, 1>), dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    else hipLaunchKernelGGL((k_gemmlike<1, 1>), dim3(nblk), dim3(256), 0, 0, src, per, reps, shared, t, out);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  }
  std::vector<unsigned long long> h(nblk);
  hipMemcpy(h.data(), t, nblk * 8, hipMemcpyDeviceToHost);
  double sum = 0, mx = 0;
  for (auto v : h) { sum += v; mx = v > mx ? v : mx; }
  const double bytes = (mode >= 2 ? 128.0 * 1152 * 4 : (double)per * 4) * (reps - 1);
  const double avg_us = sum / nblk / 100.0;
  printf("mode %d nblk %d kb %d shared %d: avg %.2f us/block -> %.1f GB/s per workgroup, aggregate %.2f TB/s,"
         " %.3f us per 36-step pass\n", mode, nblk, kb, shared, avg_us, bytes / (avg_us * 1e3),
         bytes * nblk / (mx / 100.0 * 1e6), avg_us / (reps - 1));
  return 0;
}
