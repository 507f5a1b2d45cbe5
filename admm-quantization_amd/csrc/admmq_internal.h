// Internal device/host structures of libadmmq (not part of the C-ABI).
//
// Memory layout in HBM (per ADMM problem = one (layer, mode) factor):
//   Fp, H, U, P, X, HT : float32 [Ip x ld] row-major, ld = roundup(R,32),
//                        Ip = 32 if I <= 32 else roundup(I, 64);
//                        pads kept at exactly 0
//   M                  : float32 [ldm x ldm], ldm = roundup(R,64); (G+rho I)^-1,
//                        symmetric, zero outside the R x R block
//   A64, L64           : float64 [ldm x ldm] SPD factor / inverse-factor scratch
//   D64                : float64 [ldm x 32] diagonal Cholesky blocks
//   res[2][kResRep][4] : per parity slot, kResRep replicas of the fp64 residual sums
//                        S1..S4 (source/admm.py:62-63), summed by the convergence test
//   flags[4]           : {done, iterations, spd_error, 0}
// and one MseView of per-slot quantizer state (below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Diagnostic per-block timelines / counters (admmq_debug_*_trace, tools/*_timeline.py):
// compiled in only with `make TRACE=1`; the production library makes no trace stores.
#ifndef ADMMQ_TRACE
#define ADMMQ_TRACE 0
#endif
#define ADMMQ_NOW() (ADMMQ_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull)

namespace admmq {

enum QScheme { kMse = 0, kMinMax = 1, kSymmetric = 2, kAffine = 3 };
enum SolveMode { kSolveF32 = 0, kSolveSplit = 1 };

constexpr int kMaxSel = 64;        // stage-2 candidate list length (else exhaustive)
constexpr int kMaxStage1 = 1024;   // num_attempts handled by the two-stage search
constexpr int kMaxStage1Bits = 6;  // bits handled by the two-stage search (threshold table in LDS)
constexpr int kHistRep = 8;        // replicas of the global stage-1 histograms (atomic spread)
constexpr int kMaxMerged = 4096;   // qmax * ncand of the merged-threshold stage 1
constexpr int kCells = 4096;       // coarse cells of the merged-threshold stage 1 (mse_search.hip)
constexpr int kResRep = 8;         // replicas of the per-problem residual sums (atomic spread)
constexpr int kThinRows = 16;      // factors with I <= kThinRows take the VALU solve of thin_loop.hip
constexpr long long kWideMinTiles = 4 * 768;   // 64x64 tiles of a launch from which I > 64 factors take wide tiles
constexpr int kWideRows = 256;                 // ... of kWideRows x 128 (k_gemm<8, 1, 3, *, 2>)

// Quantizer state of one job (an ADMM problem's X, or a standalone tensor), with
// `nslot` parity slots. The MSE-minmax search (source/quantization.py:118-144) runs in
// two exact stages: stage 1 accumulates per-candidate level sums h1 (sum |x| per
// breakpoint, fixed point) / h2 (sum 2k-1 per breakpoint) and s2 = sum x^2; select
// turns them into A(c) +- E(c) and the candidate set S; stage 2 evaluates the
// canonical SSE only on S (sel = {nS, c*, list...}); nS == ncand means exhaustive.
struct MseView {
  const float* X;              // rows x ld, zero pads (ADMM: H_T, see U)
  const float* U;              // non-null (ADMM): the quantizer input is X - U = H_T - U
  int rows, cols, ld, qpr;     // qpr = ceil(cols/4)
  int nq, nelem;               // quads of the valid region, rows*cols
  unsigned* stat;              // [slot][4] {absmax bits, min enc, max enc, 0}
  unsigned long long* sse;     // [slot][ncand] canonical fixed-point SSE
  unsigned long long* h1;      // [slot][kHistRep][ncand+1]
  unsigned long long* h2;      // [slot][kHistRep][ncand+1]
  double* s2;                  // [slot]
  int* sel;                    // [slot][2 + kMaxSel]
  unsigned* ticket;            // [slot] stage-1 blocks finished (the last one runs the selection)
  unsigned long long* ready;   // [slot] fused finalize: (iteration + 1) << 32 once the selection is published,
                               // | 1 << 31 | c* when the selection is the single candidate c*
  const int* done;             // early-exit flag (ADMM) or nullptr
  int nhist, pad_;             // stage-1 blocks of this job
};

struct ProbDesc {
  // caller buffers (I x R contiguous)
  const float* F_user;
  const float* G_user;
  const float* H0_user;
  float* H_out;
  float* U_user;
  float* HT_dbg;   // optional: last H_T (I x R)
  float* X_dbg;    // optional: last H_T - U (I x R)
  // internal padded buffers
  float* Fp; float* H; float* U; float* P; float* X; float* HT;
  float* M;
  double* A64; double* L64; double* D64;   // D64: diagonal L blocks [nbk][32][32]
  // split solve (kSolveSplit, gemm_kernels.hip): P and M as [rows][ld/32][32 hi | 32 lo]
  // fp16 planes (the bytes of the fp32 rows) with one power-of-two exponent per row
  _Float16* P2; int* eP;    // [Ip] rows
  _Float16* M2; int* eM;    // [ldm] rows
  MseView mv;
  double* res;
  int* flags;
  float* rho;
  int I, R, ld, Ip, ldm, nbk;
  int nq;          // quads of the valid (I x R) region: I * ceil(R/4)
  int split;       // 1: this problem's solve uses the split operand planes
  int fin_rows;    // split: rows per finalize unit (units hold whole rows)
  int ksplit;      // K-split pieces of each 64 x 64 solve tile (1: none); a function of (I, R) only
  float* kpart;    // K-split: partial images [tiles][ksplit][4096] floats
  unsigned* kctr;  // K-split: per-tile arrival counters (monotonic, zeroed per run)
};

// A standalone quantization job (quantize_tensor): x viewed as (rows, cols).
struct QJob {
  const float* src;   // rows x cols contiguous (user)
  float* dst;         // rows x cols contiguous (user)
  float* Xp;          // padded copy rows x ld (workspace), or src itself when cols % 4 == 0
  MseView mv;         // one slot
  int rows, cols, ld, nq;
  float tmin_kw, tmax_kw;   // affine kwargs (NaN = unset)
  int has_kw, copy;         // copy: Xp is the workspace copy (k_qpack writes it)
  unsigned* pstat;          // k_qpack's per-unit {absmax, min, max} partials (3 per unit)
  int pu0, pun;             // this job's units in the statistics launch: first, count
};

// Work-unit tables (built on the host, uploaded once per call)
// GEMM tile: rows tm, columns tn of problem prob, K-steps nk. The operands' addresses
// and strides ride along (filled at upload), so a tile's first loads depend on the
// tile entry only, not on a further descriptor read. Split form: P / M point at the
// fp16 planes (row strides in floats are unchanged), eP / eM at the row exponents.
// K-split pieces (fp32 64 x 64 tiles; the piece count np is fixed by the factor's shape:
// api.hip ksplit_pieces): piece p covers K-steps [p nk / np, (p + 1) nk / np) of the tile
// in its own accumulator chain and the tile is ((p0 + p1) + p2) + ... Two execution forms
// with the same bits: parallel (launches that leave CUs idle: np workgroups per tile, piece
// pc of np runs K-steps [k0, k0 + nk), `part` holds the tile's np partial images, `ctr` its
// arrival counter: gemm_kernels.hip ksplit_combine) or serial (one workgroup runs the whole
// tile and folds its accumulator into the running sum at each of the ser - 1 piece starts).
struct GemmTile {
  int prob, tm, tn, first, nk, bm;   // bm: tile rows of the persistent fp32 kernel (k_gemm_f32p), else 0
  const float* P; const float* M; const float* U;
  const int* eP; const int* eM;
  int ld, ldm;
  int k0, np, pc, ser;               // K-split: parallel form: first K-step, pieces, this piece (np = 1: whole tile);
                                     // serial form: pieces folded in this workgroup (1: none)
  float* part; unsigned* ctr;        // K-split: the tile's partial images [np][16 KB] and arrival counter
};
constexpr int kKsplitMax = 4;        // pieces per tile at most
constexpr int kKsplitMinSteps = 6;   // K-steps per piece at least
// Thin-factor solve workgroup (thin_loop.hip): columns [col0, col0 + cw) of problem `job`,
// the rank-th of the problem's nteam workgroups (in the persistent loop rank 0 resets the
// team's words)
struct ThinLoopUnit { int job, col0, cw, rank, nteam, pad_[3]; };
constexpr int kTLThreads = 512;
constexpr int kTLMaxCand = 256;       // num_attempts of the persistent loop
constexpr int kTLBins = 264;          // >= kTLMaxCand + 1, a whole number of 64-B lines
constexpr int kTLMaxTeam = 64;        // workgroups of a team (ld / 32 <= 36; one polling wave)
constexpr int kTLKPairs = 9;          // k pairs of M per thread and reduction chunk (ld <= 1152 per chunk)
// A team's hand-off words, one set per parity slot (zeroed by the host before the launch;
// after that rank 0 re-zeroes a slot once every reader is past it). 128-B lines apart.
struct alignas(128) ThinSync {
  unsigned bar;                          // barrier arrivals (monotonic)
  unsigned pad0_[31];
  unsigned long long mx[2];              // (unused since the barrier-1 words carry max |X|)
  unsigned long long pad1_[14];
  unsigned long long arr1[kTLMaxTeam];   // barrier 1: per team rank, (iteration + 1) << 32 | its max |X| bits
  double s2[2];                          // sum X^2 per slot (stage-1 bound)
  double res[2][4];                      // residual sums S1..S4 per slot
  double pad2_[6];
  unsigned long long h1[2][kTLBins];     // stage-1 level sums (team total)
  unsigned long long h2[2][kTLBins];
  unsigned long long sse[2][kTLBins];    // stage-2 canonical SSE of the selected candidates
};
// Work unit {job, first element}. Stage-1 units also carry the job's inputs that the
// kernel's first loads need (the search state, the stop flag, the tensor and its size),
// so those loads do not wait on a dependent descriptor read.
struct Chunk {
  int job, start;
  const unsigned* stat;
  const int* done;
  const float* X;
  const float* U;   // non-null: the element is X - U (ADMM: H_T - U)
  long long total;
  const float* H;   // ADMM finalize units: the current H and the padded F
  const float* F;
  const int* sel;   // ADMM finalize units: the job's search record [slot][2 + kMaxSel]
  // k_mse_hist3 without the fused finalize: `reps` consecutive stage-1 units of `step`
  // elements in one block (one table setup and one histogram flush for all of them;
  // `total` is then the last unit's end); `nblk` = blocks of this job in the launch
  // (the ticket count). 0 = one unit / the job's nhist.
  int reps, step, nblk, pad2_;
};

// Loads through global (not flat) pointers: flat loads also count in lgkmcnt, and a
// kernel prologue that issues all its loads before using any needs plain vmcnt order.
typedef __attribute__((address_space(1))) const float gcf32;
typedef __attribute__((address_space(1))) const int gci32;
typedef float gf32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 gld4(const float* q) {
  const gf32x4 v = *(__attribute__((address_space(1))) const gf32x4*)q;
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int gld_i32(const int* q) { return *(gci32*)q; }
__device__ __forceinline__ unsigned gld_u32(const unsigned* q) {
  return *(__attribute__((address_space(1))) const unsigned*)q;
}
__device__ __forceinline__ float4 sub4(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}

// Quantizer input elements at off..off+3: X, or H_T - U for an ADMM view (the GEMM
// does not store X = H_T - U; every reader forms it with the same float32 subtraction).
__device__ __forceinline__ float4 load_x4(const float* X, const float* U, long long off) {
  float4 x = *reinterpret_cast<const float4*>(X + off);
  if (U) {
    const float4 u = *reinterpret_cast<const float4*>(U + off);
    x.x -= u.x; x.y -= u.y; x.z -= u.z; x.w -= u.w;
  }
  return x;
}

// float <-> order-preserving unsigned encodings for atomicMin/Max
__device__ __forceinline__ unsigned enc_ord(float f) {
  unsigned b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float dec_ord(unsigned e) {
  return __uint_as_float((e & 0x80000000u) ? (e & 0x7FFFFFFFu) : ~e);
}

// Records the thread's last error text (admmq_last_error) and returns `code`.
int set_error(int code, const char* msg);
// Stream-ordered host -> device copy of n bytes through a pinned staging chunk (the host
// buffer may be reused at once; the call never waits for the stream). ADMMQ_OK or an error.
int upload_async(void* dst, const void* src, size_t n, hipStream_t s);

// Host-side launchers (each defined in its own translation unit).
void launch_rho(const ProbDesc* d, int nprob, hipStream_t s);
void launch_pack(const ProbDesc* d, int nprob, int maxIp, int maxld, hipStream_t s);
void launch_fill_a64(const ProbDesc* d, int nprob, int maxldm, hipStream_t s);
void launch_spd_inverse(const ProbDesc* d, int nprob, int maxnbk, hipStream_t s);
void launch_spd_linv(const ProbDesc* d, int nprob, int maxnbk, hipStream_t s);
void launch_thin_solve(const ProbDesc* d, const ThinLoopUnit* units, int nunits, int nr, int maxld, int slot, int iter,
                       float eps, int ncand, hipStream_t s);
void launch_gemm(const ProbDesc* d, const GemmTile* tiles, int ntiles_wide, int ntiles_small, int ntiles_big,
                 bool split, int slot, int iter, float eps, int ncand, hipStream_t s, hipEvent_t ev0 = nullptr,
                 hipEvent_t ev1 = nullptr, bool prefetch_u = false);
extern int g_gemm_ks_f32;
int set_sel_widen_search(int on);   // diagnostics (mse_search.hip / thin_loop.hip)
int set_sel_widen_thin(int on);
extern int g_gemm_f32_stage;   // fp32 64 x 64 staging form (gemm_kernels.hip)
void launch_gemm_f32t(const ProbDesc* d, const GemmTile* tiles, int ntiles, int slot, int iter, float eps, int ncand,
                      hipStream_t s);
void launch_gemm_f32p(const ProbDesc* d, const GemmTile* tiles, const int* list_off, int nslots, int slot, int iter,
                      float eps, int ncand, hipStream_t s);
void launch_split_rows(const ProbDesc* d, int nprob, int maxrows, int which, hipStream_t s);
// persistent thin-factor loop: 0 if launched, else why not (-1 unsupported shape, -2 no residency)
int launch_thin_loop(const ProbDesc* d, const ThinLoopUnit* units, int nunits, ThinSync* sync, int nr, int maxld,
                     int n_iter, float eps, int ncand, int bits, unsigned wait_polls, int ncu, hipStream_t s);
// two-stage MSE search over MseView tables (ADMM: views embedded in ProbDesc)
void launch_mse_hist(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits,
                     int slot, int nv, hipStream_t s);
size_t hist_lds_bytes(int ncand, int bits);
size_t hist3_lds_bytes(int ncand, int bits);
int copy_hist_trace(unsigned long long* host, int n);
int copy_gemm_trace(unsigned long long* host, int n);
int copy_gemm_trace2(unsigned long long* host, int n);
int copy_gemm_simd(unsigned* host, int n);
int copy_setup_trace(unsigned long long* host, int n);
int copy_fin_trace(unsigned long long* host, int n);
int copy_hist_cu(unsigned long long* host, int n);
int copy_small_trace(unsigned long long* host, int n);
int copy_thin_loop_trace(unsigned long long* host, int n);
int copy_sel_stats(unsigned long long* host, int reset);
int check_thresholds(unsigned seed, int nsamp);
int check_cells(int n, int bits, unsigned seed, int nsamp, unsigned* maxdev_out);
bool merged_ok(int ncand, int bits);
void launch_mse_hist3(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits, int slot,
                      const unsigned short* rank0, const unsigned short* groups, int ngroups, int nv, bool fin, int iter,
                      unsigned wait_polls, hipStream_t s, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// fused finalize: polls (s_sleep 2 each, ~10 ms in all) before a block gives up waiting for
// its job's selection and reports an internal fault instead of finalizing
constexpr unsigned kFinWaitPollsDefault = 1u << 17;
int hist3_fin_capacity(int ncand, int bits, int nv);
int small_admm_groups(long long maxtotal);
void launch_mse_small_admm(const ProbDesc* d, const int* jobs, int njobs, int ngr, int ncand, int bits, int slot,
                           int iter, const unsigned short* rank0, const unsigned short* groups, int ngroups,
                           hipStream_t s);
void launch_mse_select_all(const ProbDesc* d, const QJob* q, int njobs, int ncand, int slot, hipStream_t s);
void launch_mse_sse(const ProbDesc* d, const QJob* q, const Chunk* chunks, int nchunks, int ncand, int bits,
                    int slot, hipStream_t s);
void launch_finalize_admm(const ProbDesc* d, const Chunk* chunks, int nchunks, int groups, int ncand, int bits,
                          int qscheme, int slot, int iter, hipStream_t s);
void launch_unpack(const ProbDesc* d, int nprob, int maxI, int maxR, hipStream_t s);

void launch_qpack(const QJob* jobs, int njobs, const Chunk* chunks, int nchunks, hipStream_t s);
void launch_channel_quant(const float* x, float* y, long long A, int C, long long B, long long outer, int L, int Lo,
                          unsigned* stats, int bits, int scheme, hipStream_t s);
void launch_qfinal(const QJob* jobs, const Chunk* chunks, int nchunks, int ncand, int bits, int qscheme,
                   hipStream_t s);

constexpr int kSseQuads = 512;      // quads per stage-2 / exhaustive SSE work unit (8 KiB LDS)
constexpr int kHistElems = 4096;    // elements per stage-1 work unit x hist_nv (1024 x 4 legacy, 512 x 8 merged)
constexpr int kHistMultiRounds = 2;   // non-fused search: units per block sized for ~2 rounds of kHistMaxUnits blocks
constexpr int kHistMultiMaxReps = 8;  // ... at most 8 units per block
constexpr int kHistMaxUnits = 512;  // stage-1 units that fit in one round (2 per CU): above, 2x larger units
constexpr int kElemChunk = 1024;    // elements per elementwise work unit (256 threads x float4)
constexpr int kPackElems = 16384;   // elements per k_qpack unit (256 threads x 16 float4): few partials
constexpr int kFinElems = 4096;     // elements per ADMM finalize work unit when there are >= kFinMinUnits of them
constexpr int kFinMinUnits = 256;   //   (else kElemChunk: small problem sets keep their parallelism)

}  // namespace admmq
