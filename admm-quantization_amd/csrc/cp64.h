// fp64 contraction jobs on v_mfma_f64_16x16x4_f64 (cp64_kernels.hip): the CP-ALS / EPC
// initialiser's MTTKRP and Gram-Hadamard products, and plain fp64 GEMMs for the blocked
// R x R solves (solve64.hip).
#pragma once

#include <string>
#include <vector>

#include <hip/hip_runtime.h>

namespace admmq {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kC64BM = 64, kC64BN = 64, kC64BK = 16, kC64NT = 256;
constexpr int kC64LD = kC64BM + 8;   // LDS row stride (doubles): the 4 k rows of a fragment read on distinct banks
constexpr int kC64PA = kC64BK * kC64BM / kC64NT;   // A elements per thread per K-step
constexpr int kC64PB = kC64BK * kC64BN / kC64NT;   // B elements per thread per K-step

struct Cp64Job {
  int kind;             // 0 MTTKRP (and the plain GEMM: K2 = 1), 1 Gram(-Hadamard)
  int M, N, K;          // output rows / cols, reduction length (MTTKRP)
  int nsplit, kchunk;   // MTTKRP: K chunks and their length (multiple of kC64BK)
  int K2;               // MTTKRP: Khatri-Rao inner extent (1: one other factor, 2-way / GEMM)
  int afast;            // A side staged along rows (rows contiguous in memory)
  int R, Kx, Ky;        // Gram: rank, rows of X, rows of Y (0: no Hadamard factor)
  int bt, tri;          // K2 = 1: B transposed (B(k, n) = X[n ldb + k]); tri 1 / 2: B(k, n) = 0 unless k <= n / k >= n
  long long ldb;        // K2 = 1: B's row stride
  long long sm, s1, s2; // MTTKRP: Y_(n)[a, k] = W[a sm + (k / K2) s1 + (k % K2) s2]
  const double* W;
  const double* X;      // MTTKRP: KR outer factor ((K / K2) x N); Gram: first factor (Kx x R)
  const double* Y;      // MTTKRP: KR inner factor (K2 x N) or nullptr; Gram: second factor or nullptr
  double* part;         // MTTKRP: [nsplit][M][N] partial planes (nsplit > 1)
  double* out;          // MTTKRP: F (M x N); Gram: G (R x R)
  const int* gate;      // nullptr, or a device int: the job's units return at once while it is nonzero
  int unit0, nunits;    // the job's units in the plan (contiguous)
};
struct Cp64Unit { int job, tm, tn, ks; };

struct Cp64Plan {
  std::vector<Cp64Job> jobs;
  std::vector<Cp64Unit> units;
  std::vector<int> split_ids;
  size_t bytes = 0;
};

// Appends C = A op(B) (A: M x K row-major with row stride lda; B: K x N row-major with row stride
// ldb, or its transpose when bt = 1 (B^T: N x K, stride ldb); tri 1 / 2: only the entries of B
// with k <= n / k >= n are nonzero (the triangle of an L^-1 or L^-T operand; the others are not
// read)) to the plan, its units after the plan's and its K chunks to fill ~512 units;
// `gate`: a device int, the units return at once while it is nonzero.
void cp64_plan_gemm(Cp64Plan& pl, const double* A, long long lda, const double* B, long long ldb, int bt, int tri,
                    double* C, int M, int N, int K, const int* gate);
// Carves the plan's tables and partial planes from `base` (nullptr: only sizes): bytes used.
size_t cp64_carve(Cp64Plan& pl, void* base);
// Uploads the tables (stream-ordered, pinned staging).
int cp64_upload(const Cp64Plan& pl, void* base, hipStream_t s);
// Launches job `job`'s units (and its split-K reduction) from the uploaded tables.
int cp64_launch_job(const Cp64Plan& pl, void* base, int job, hipStream_t s);

}  // namespace admmq
