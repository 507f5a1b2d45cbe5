/*
 * libadmmq — MI355X-native ADMM quantized tensor-factorization hot path (C ABI).
 *
 * Every entry point is stream-ordered on the caller's HIP stream (`stream` is a
 * hipStream_t passed as void*), takes plain device pointers to row-major float32
 * buffers, uses only caller-owned workspace, and returns an int32 status
 * (ADMMQ_OK = 0). No entry point allocates device memory or synchronises with the
 * device: plans (descriptor and work-unit tables) go up with hipMemcpyAsync from a pool
 * of pinned host staging chunks (per device of the stream, at most 64 MB) the library
 * grows on first use and reuses once their copies have completed, so a call returns
 * while its launches are still queued. Only when every chunk is in flight and the pool
 * is at its cap does a plan go up from pageable memory, a copy that may wait for the
 * stream (it never waits on the device otherwise).
 *
 * Reference interfaces replaced (KamikaziZen/admm-quantization @ 2024_10_08):
 *   admmq_admm_prepare + admmq_admm_run  <- source/admm.py:51-67  admm_iteration(H,U,F,G,max_iter,eps,bits,qscheme)
 *                                           (batched over independent (layer, mode) problems)
 *   admmq_quantize_batched               <- source/quantization.py:69-115  quantize_tensor(tensor,bits,qscheme,**kw)
 *                                           incl. quantize_tensor_mse :118-144, min_max_quantize :48-66
 *   admmq_quantize_channel               <- source/quantization.py:69-106 quantize_tensor(tensor,bits,
 *                                           'channel_symmetric' | 'channel_affine', dim)
 *   admmq_mse_sse_table                  <- source/quantization.py:129-141 (the candidate search, exposed
 *                                           for parity tests: canonical fixed-point SSE per candidate)
 *   admmq_cp_gram_mttkrp                 <- scripts/factorize.py:215-237 (3-way) and :276-287 (2-way):
 *                                           G = B.T @ B * (C.T @ C), F = torch.einsum('abc,cr,br->ar', W, C, B), ...
 *   admmq_cp_rel_error                   <- scripts/factorize.py:246-253 + source/admm.py:14-15
 *                                           squared_relative_diff(W, torch.einsum('ir,jr,kr->ijk', A, B, C))
 *   admmq_lowrank_pre / _post            <- scripts/factorize_lowrank.py:85-101 admm_iteration(H,U,W,H2,proj_func,
 *                                           rho,max_iter,eps): the updates around the projection, device break test
 *   admmq_panel_xtq / _xy / _outer       <- scripts/factorize_lowrank.py:80-82 (torch.linalg.svd + the rank-r
 *                                           product): the X^T Q, X Y and U S V^T products of the device projection
 *   admmq_cp64_gram_mttkrp               <- source/parafac_epc.py:42-74 (tensorly parafac / musco cp_anc's MTTKRP and
 *                                           Gram-Hadamard products, fp64)
 *   admmq_spd_solve64(_ws)               <- source/parafac_epc.py:42 (parafac's torch.linalg.solve(G, F.T).T)
 *   admmq_epc_step64 / admmq_epc_*64     <- source/parafac_epc.py:61-74 (cp_anc's mode update: eigendecomposition
 *                                           of G and the multiplier of the error constraint)
 */
#ifndef ADMMQ_H_
#define ADMMQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADMMQ_OK 0
#define ADMMQ_ERR_ARG (-1)
#define ADMMQ_ERR_HIP (-2)
#define ADMMQ_ERR_WORKSPACE (-3)
#define ADMMQ_ERR_SCHEME (-4)

/* qscheme codes (names as in source/quantization.py:91-115) */
#define ADMMQ_TENSOR_MSEMINMAX_SYMMETRIC 0
#define ADMMQ_TENSOR_MINMAX 1
#define ADMMQ_TENSOR_SYMMETRIC 2
#define ADMMQ_TENSOR_AFFINE 3

/* One ADMM problem: one factor update  H <- argmin ||F - H G|| s.t. H quantized.
 * F, H0, H_out, U: I x R; G: R x R (symmetric PSD). U is read and overwritten
 * (source/admm.py:60 mutates the caller's U in place); H0 is never written. */
typedef struct admmq_problem {
  const float* F;
  const float* G;
  const float* H0;
  float* H_out;
  float* U;
  float* HT_out; /* optional (NULL): last iteration's H_T  (debug / parity tests) */
  float* X_out;  /* optional (NULL): last iteration's H_T - U (the quantizer input) */
  int32_t I;
  int32_t R;
} admmq_problem;

/* Bytes of workspace for a batch (num_attempts: MSE candidates, 200 in the reference). */
size_t admmq_admm_workspace_size(const admmq_problem* probs, int32_t nprob, int32_t num_attempts);

/* Setup of source/admm.py:52-54 for every problem: rho = tr(G)/R, M = (G + rho I)^-1
 * (fp64 blocked Cholesky, rounded to fp32), padded copies of F/H0/U and the first
 * right-hand side. Must precede admmq_admm_run on the same workspace. */
int32_t admmq_admm_prepare(const admmq_problem* probs, int32_t nprob, int32_t num_attempts, void* workspace,
                           size_t workspace_bytes, void* stream);

/* The loop of source/admm.py:55-65: max_iter-1 iterations of {solve, quantize,
 * dual update, residual test} per problem, with the per-problem early exit when
 * r < eps and s < eps. Writes H_out and U. info (device int32[nprob*4], may be
 * NULL) receives {iterations run, converged, spd_error, internal fault} per problem
 * (internal fault: see admmq_admm_run_ex). With info == NULL the run never takes the
 * fused paths that can report an internal fault (as fused_finalize = 0), so a NULL-info
 * call always returns finalized results. Uses the solve mode its prepare recorded;
 * ADMMQ_ERR_ARG for a workspace no prepare has set up, or whose prepare planned other
 * problems or another buffer layout (the record is kept per workspace address: prepare
 * again after reallocating a workspace). */
int32_t admmq_admm_run(const admmq_problem* probs, int32_t nprob, int32_t max_iter, float eps, int32_t bits,
                       int32_t qscheme, int32_t num_attempts, void* workspace, size_t workspace_bytes,
                       int32_t* info, void* stream);

/* Per-call options of the ADMM entry points (the _ex forms). A prepare fixes the
 * operand form of the solve for its workspace: a run on that workspace must ask for the
 * same solve_mode (ADMMQ_ERR_ARG otherwise). The plain forms above take the process
 * defaults (admmq_set_solve_mode) at prepare; their run uses what its prepare recorded. */
#define ADMMQ_SOLVE_FP32 0  /* v_mfma_f32_32x32x2_f32: an fp32 FMA chain, the reference's arithmetic (default) */
#define ADMMQ_SOLVE_SPLIT 1 /* split fp16 planes on f16 MFMA (about 2^-21 relative per product; opt-in) */
typedef struct admmq_admm_options {
  int32_t solve_mode;     /* ADMMQ_SOLVE_FP32 or ADMMQ_SOLVE_SPLIT */
  int32_t fused_finalize; /* 1: projection + dual update inside the search launch where all its blocks are
                             resident at once; 0: always the separate finalize launch (same results) */
  int32_t reserved[6];    /* must be zero */
} admmq_admm_options;

/* Fills *out with the process defaults (admmq_set_solve_mode; fused finalize on). */
int32_t admmq_admm_default_options(admmq_admm_options* out);
size_t admmq_admm_workspace_size_ex(const admmq_problem* probs, int32_t nprob, int32_t num_attempts,
                                    const admmq_admm_options* opt);
int32_t admmq_admm_prepare_ex(const admmq_problem* probs, int32_t nprob, int32_t num_attempts,
                              const admmq_admm_options* opt, void* workspace, size_t workspace_bytes, void* stream);
/* info[4 p + 3] != 0: an internal fault of problem p (the fused finalize's bounded wait for
 * its job's selection timed out because the search launch's blocks were not all resident,
 * e.g. other work on the device). The affected elements were NOT finalized: H_out / U of
 * that call are invalid and the caller must restore U and re-run with fused_finalize = 0
 * (the PyTorch op does this itself). info == NULL: fused_finalize is treated as 0 (no
 * fused path runs, so no fault can go unreported). */
int32_t admmq_admm_run_ex(const admmq_problem* probs, int32_t nprob, int32_t max_iter, float eps, int32_t bits,
                          int32_t qscheme, int32_t num_attempts, const admmq_admm_options* opt, void* workspace,
                          size_t workspace_bytes, int32_t* info, void* stream);

/* prepare + run. */
int32_t admmq_admm_iteration_batched(const admmq_problem* probs, int32_t nprob, int32_t max_iter, float eps,
                                     int32_t bits, int32_t qscheme, int32_t num_attempts, void* workspace,
                                     size_t workspace_bytes, int32_t* info, void* stream);

/* One quantize_tensor call: x viewed as (rows, cols) with cols the last dimension. */
typedef struct admmq_qtensor {
  const float* x;
  float* y;
  int64_t rows;
  int64_t cols;
  float tmin; /* tensor_affine kwargs (source/quantization.py:98-101) when has_minmax */
  float tmax;
  int32_t has_minmax;
  int32_t reserved;
} admmq_qtensor;

size_t admmq_quantize_workspace_size(const admmq_qtensor* t, int32_t n, int32_t num_attempts);
int32_t admmq_quantize_batched(const admmq_qtensor* t, int32_t n, int32_t bits, int32_t qscheme, int32_t num_attempts,
                               void* workspace, size_t workspace_bytes, void* stream);

/* Per-channel schemes with an explicit dim (source/quantization.py:29-33, 91-106):
 * max / min of every row of unfold(x, dim) (source/utils.py:60-74), then the
 * tensor_symmetric / tensor_affine arithmetic with those shape[dim] statistics broadcast
 * against x's LAST dimension as torch does: requires shape[ndim-1] == shape[dim] or one of
 * them 1 (ADMMQ_ERR_ARG otherwise); y holds shape[:-1] + (max(shape[ndim-1], shape[dim]),)
 * elements. x contiguous, ndim >= 1, dim in [-ndim, ndim). */
#define ADMMQ_CHANNEL_SYMMETRIC 4
#define ADMMQ_CHANNEL_AFFINE 5
size_t admmq_quantize_channel_workspace_size(const int64_t* shape, int32_t ndim, int32_t dim);
int32_t admmq_quantize_channel(const float* x, float* y, const int64_t* shape, int32_t ndim, int32_t dim, int32_t bits,
                               int32_t qscheme, void* workspace, size_t workspace_bytes, void* stream);

/* Canonical SSE table of the MSE-minmax search for one tensor (sse_out: device uint64[num_attempts]). */
int32_t admmq_mse_sse_table(const float* x, int64_t rows, int64_t cols, int32_t bits, int32_t num_attempts,
                            uint64_t* sse_out, void* workspace, size_t workspace_bytes, void* stream);

/* A/B switch for the MSE-minmax search: 1 = evaluate the canonical SSE of every
 * candidate (the reference's 200 full passes), 0 (default) = two-stage exact search
 * (level-breakpoint bounds, then the canonical SSE only for candidates that can still
 * be the argmin). Both return bit-identical results. */
int32_t admmq_set_exhaustive_search(int32_t enable);

/* Process default of the per-iteration solve's operand form H_T = P M (the
 * cholesky_solve of source/admm.py:56) for the plain (non-_ex) entry points:
 * ADMMQ_SOLVE_FP32 (0, default) = fp32 MFMA, the reference's fp32 arithmetic;
 * ADMMQ_SOLVE_SPLIT (1) = split fp16 planes on f16 MFMA (P and M as hi + lo fp16 with a
 * power-of-two exponent per row, 3 products, fp32 accumulation; about 2^-21 relative per
 * product). Both stay within the 1e-5 rel-Frobenius solve contract of SURVEY.md §8(c) P2.
 * Read once by admmq_admm_prepare, which records it for its workspace: a later change
 * does not affect runs on an already prepared workspace. */
int32_t admmq_set_solve_mode(int32_t mode);
int32_t admmq_get_solve_mode(void);

/* Optional HIP-event timing of every launch issued by admmq_admm_prepare/run on this
 * thread between begin and end, one event pair per launch, summed per class:
 * ADMMQ_PROF_GEMM k_gemm (solve, MFMA), ADMMQ_PROF_GEMM_THIN k_gemm_thin (solve of the
 * I <= 16 factors, VALU), ADMMQ_PROF_SEARCH the multi-block MSE candidate search
 * (k_mse_hist3 / k_mse_hist / the exhaustive sweep), ADMMQ_PROF_SMALL k_mse_small_admm
 * (search + projection + dual update of the I <= 16 factors in one block each),
 * ADMMQ_PROF_FINALIZE k_finalize_admm (projection + dual update), ADMMQ_PROF_PREPARE the
 * whole prepare phase (rho, SPD inverse, operand planes), ADMMQ_PROF_THIN_LOOP k_thin_loop
 * (every iteration of a call whose factors all have I <= 16, one persistent launch, always
 * timed). Only ADMM iterations it with
 * it % sample_every == 0 are timed (each event pair adds an inter-kernel gap, so the
 * bench samples instead of timing every launch). end() synchronises on the last event
 * and fills ADMMQ_PROF_CLASSES summed milliseconds and launch counts. */
#define ADMMQ_PROF_GEMM 0
#define ADMMQ_PROF_GEMM_THIN 1
#define ADMMQ_PROF_SEARCH 2
#define ADMMQ_PROF_SMALL 3
#define ADMMQ_PROF_FINALIZE 4
#define ADMMQ_PROF_PREPARE 5
#define ADMMQ_PROF_THIN_LOOP 6
#define ADMMQ_PROF_CLASSES 8
int32_t admmq_profile_begin(int32_t max_launches, int32_t sample_every);
int32_t admmq_profile_end(double* ms_per_class, int64_t* launches_per_class);

/* One CP layer of the ALS sweep (scripts/factorize.py:207-310): W is dims[0] x dims[1]
 * (x dims[2]) row-major (a 3x3 conv reshaped to (cout, cin, 9), or a 2-D weight);
 * factors[d] is dims[d] x R row-major. G / F are outputs of admmq_cp_gram_mttkrp. */
typedef struct admmq_cp_layer {
  const float* W;
  const float* factors[3]; /* factors[2] unused (NULL) when ndim == 2 */
  float* G;                /* R x R: Hadamard product of the Grams of the factors other than `mode` */
  float* F;                /* dims[mode] x R: MTTKRP of W with the Khatri-Rao product of the others */
  int32_t dims[3];
  int32_t ndim;            /* 2 or 3 */
  int32_t R;
} admmq_cp_layer;

/* Workspace bytes for admmq_cp_gram_mttkrp (this mode) and admmq_cp_rel_error on these layers. */
size_t admmq_cp_workspace_size(const admmq_cp_layer* layers, int32_t n, int32_t mode);

/* For every layer: G = Gram∘Gram of the factors other than `mode` and F = the mode-`mode`
 * MTTKRP (fp32 MFMA, deterministic split-K). factors[mode] is not read. */
int32_t admmq_cp_gram_mttkrp(const admmq_cp_layer* layers, int32_t n, int32_t mode, void* workspace,
                             size_t workspace_bytes, void* stream);

/* out[l] (device double[n]) = ||W - [[factors]]||_F / ||W||_F per layer, without
 * materialising the reconstruction (fp32 MFMA products, fp64 sums). */
int32_t admmq_cp_rel_error(const admmq_cp_layer* layers, int32_t n, double* out, void* workspace,
                           size_t workspace_bytes, void* stream);

/* fp64 per-mode contractions of the CP-ALS / EPC initialiser (admmq.parafac_epc): the
 * reference runs them inside tensorly `parafac` and musco `cp_anc` on the fp64 tensor
 * (source/parafac_epc.py:36-74). Same layout as admmq_cp_layer, in double. */
typedef struct admmq_cp_layer_f64 {
  const double* W;
  const double* factors[3]; /* factors[2] unused (NULL) when ndim == 2 */
  double* G;                /* R x R: Hadamard product of the Grams of the factors other than `mode` */
  double* F;                /* dims[mode] x R: MTTKRP of W with the Khatri-Rao product of the others */
  int32_t dims[3];
  int32_t ndim;             /* 2 or 3 */
  int32_t R;
} admmq_cp_layer_f64;

/* Workspace bytes for admmq_cp64_gram_mttkrp (this mode) on these layers. */
size_t admmq_cp64_workspace_size(const admmq_cp_layer_f64* layers, int32_t n, int32_t mode);

/* For every layer: G and F of `mode` in fp64 (f64 MFMA, Khatri-Rao operand formed on the
 * fly, deterministic split-K). factors[mode] is not read. */
int32_t admmq_cp64_gram_mttkrp(const admmq_cp_layer_f64* layers, int32_t n, int32_t mode, void* workspace,
                               size_t workspace_bytes, void* stream);

/* Quant + low-rank ADMM (scripts/factorize_lowrank.py:85-101), one iteration =
 *   admmq_lowrank_pre   Hbar = (rho (H + U) + W - H2) / (1 + rho),  X = Hbar - U
 *   (caller)            Hn = proj(X)   (quantizer: admmq_quantize_batched; or a rank projection)
 *   admmq_lowrank_post  U += Hn - Hbar; H = Hn; residuals r, s; sticky done when r < eps and s < eps
 * All buffers are n contiguous floats. The workspace holds {done, ticket, iterations, 0}
 * (int32) at offset 0 and the fp64 partial sums; admmq_lowrank_reset zeroes the state
 * before a call's first iteration. After `done`, pre/post do nothing. */
size_t admmq_lowrank_workspace_size(int64_t n);
int32_t admmq_lowrank_reset(void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_lowrank_pre(const float* H, const float* U, const float* W, const float* H2, float* Hbar, float* X,
                          int64_t n, float rho, void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_lowrank_post(const float* Hn, const float* Hbar, float* H, float* U, int64_t n, float eps,
                           void* workspace, size_t workspace_bytes, void* stream);

/* Panel products of the rank projection (scripts/factorize_lowrank.py:80-82, the truncated
 * SVD of every low-rank inner step; admmq.lowrank.KrylovProjector builds it from these):
 *   admmq_panel_xtq    Y = X^T Q  (n x k, row-major, ld k)
 *   admmq_panel_xy     Z = X Y    (m x k, row-major, ld k)
 * X: m x n float32 with row stride ldx, read as float32 and widened exactly; Q / Y / Z
 * float64. v_mfma_f64_16x16x4_f64, fp64 accumulation in a fixed order (the result depends
 * on m, n, k only). The workspace (admmq_panel_workspace_size, zeroed once before its first
 * use) holds the cross-workgroup partials and, at its end, the arrival counters: calls on
 * one workspace must be stream-ordered and pass the same workspace_bytes (a larger
 * workspace for larger panels is a new, zeroed buffer).
 *   admmq_panel_outer  O = A B^T  (m x n float32, row stride ldo): A m x r, B n x r float64,
 * each output summed over r in fp64 and rounded once; r <= 32. */
size_t admmq_panel_workspace_size(int64_t m, int64_t n, int64_t k);
int32_t admmq_panel_xtq(const float* X, int64_t m, int64_t n, int64_t ldx, const double* Q, int64_t k, double* Y,
                        void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_panel_xy(const float* X, int64_t m, int64_t n, int64_t ldx, const double* Y, int64_t k, double* Z,
                       void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_panel_outer(const double* A, const double* B, int64_t m, int64_t n, int64_t r, float* O, int64_t ldo,
                          void* stream);
/* C = A^T B (p x q, row-major, ld q) for tall float64 A (m x p, row stride lda) and B (m x q,
 * row stride ldb): the panels' Gram / cross products (fixed summation order; the workspace,
 * admmq_gram64_workspace_size, needs no initialisation). */
size_t admmq_gram64_workspace_size(int64_t m, int64_t p, int64_t q);
int32_t admmq_gram64(const double* A, int64_t lda, const double* B, int64_t ldb, int64_t m, int64_t p, int64_t q,
                     double* C, void* workspace, size_t workspace_bytes, void* stream);

/* The EPC step's multiplier (cp_anc, source/parafac_epc.py:61-74): *mu (device double) = the
 * root mu >= 0 of normY2 - sum_i c_i (s_i + 2 mu) / (s_i + mu)^2 = delta2 (0 when already
 * below), by bracket doubling and bisection to fp64 resolution; c, s: n device doubles. */
int32_t admmq_epc_mu(const double* c, const double* s, int64_t n, double normY2, double delta2, double* mu,
                     void* stream);

/* The R x R solves of the CP-ALS / EPC initialiser on one workgroup (the fp64 matrix in LDS,
 * 1 <= n <= 136), replacing tensorly parafac's torch.linalg.solve and cp_anc's eigendecomposition
 * (source/parafac_epc.py:42, :61-74). Row-major device doubles; no host synchronisation.
 *   admmq_spd_solve64  X = F G^-1 (F, X: m x n; G: n x n SPD) by an unpivoted blocked Gauss-Jordan
 *                      inverse of G in LDS; *info (device int, may be NULL) = 0, or 1 when a pivot
 *                      is not positive (G not numerically positive definite: X untouched).
 *   admmq_epc_step64   X = F (G + mu I)^-1 with mu >= 0 the root of
 *                      normY2 - <F, X> - mu ||X||^2 = delta2 (= the eigen form
 *                      normY2 - sum_j |F v_j|^2 (s_j + 2 mu) / (s_j + mu)^2), 0 when the LS step's
 *                      error already reaches delta2; *mu (device double): in, a warm start (<= 0:
 *                      none), out, the root. work: m x n device doubles of scratch (F Q and the
 *                      solved rows, transposed: G = Q T Q^T is tridiagonalised once per call).
 *                      G is reduced to tridiagonal form once (Householder), every evaluation of
 *                      the error equation is then a set of tridiagonal L D L^T recurrences.
 *                      *info (may be NULL): 0, or 1 when no G + mu I on the search bracket was
 *                      positive definite (X NaN), the search's budget ran out or an internal
 *                      hand-off timed out. */
int32_t admmq_spd_solve64(const double* G, const double* F, int64_t m, int64_t n, double* X, int32_t* info,
                          void* stream);
int32_t admmq_epc_step64(const double* G, const double* F, int64_t m, int64_t n, double normY2, double delta2,
                         double* mu, double* X, double* work, int32_t* info, void* stream);

/* The same solves for any n (1 <= n <= 8192), spread over the chip (the resnet ranks 183 ... 1141 do
 * not fit one workgroup's LDS): A = G + shift I (fp64, shift = rel_shift * trace(G) / n), its
 * blocked Cholesky A = L L^T and L^-1 (the 32 x 32-blocked fp64 kernels of the ADMM prepare),
 * then X = (F L^-T) L^-1 as two fp64-MFMA GEMMs. Caller-owned workspace of
 * admmq_solve64_workspace_size(m, n) bytes (no initialisation; calls on one workspace must be
 * stream-ordered); no host synchronisation.
 *   admmq_spd_solve64_ws   X = F (G + shift I)^-1 (replaces source/parafac_epc.py:42, tensorly parafac's
 *                          torch.linalg.solve(G, F.T).T); *info (device int, may be NULL) = 0, or 1
 *                          when G + shift I is not numerically positive definite (X undefined). n <= 136
 *                          runs the one-workgroup kernel of admmq_spd_solve64 (no workspace used).
 *   admmq_epc_begin64 / admmq_epc_rounds64 / admmq_epc_end64
 *                          the EPC mode update of admmq_epc_step64 (replaces source/parafac_epc.py:61-74,
 *                          musco cp_anc's eigendecomposition) for any n: begin sets the multiplier
 *                          search up on the device (*mu: the warm start, <= 0 none); each round is one
 *                          evaluation (a Cholesky of G + mu I at the search's next mu, X = F (G + mu I)^-1,
 *                          and the Newton update of mu on the device); rounds after the search is done
 *                          return at once. *done (device int, may be NULL) = 1 once it is done: the
 *                          caller reads it when it chooses and asks for more rounds until then.
 *                          end writes *mu (device double) and *info (device int, may be NULL): 0
 *                          converged (X = F (G + mu I)^-1 at the returned mu), 1 no positive definite
 *                          G + mu I found or the evaluation budget (96) spent, 2 not done yet. The same
 *                          G, F, X, m, n and workspace for every call of one step. */
size_t admmq_solve64_workspace_size(int64_t m, int64_t n);
int32_t admmq_spd_solve64_ws(const double* G, const double* F, int64_t m, int64_t n, double rel_shift, double* X,
                             int32_t* info, void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_epc_begin64(const double* G, const double* F, int64_t m, int64_t n, double normY2, double delta2,
                          const double* mu, double* X, void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_epc_rounds64(const double* G, const double* F, int64_t m, int64_t n, double* X, int32_t rounds,
                           int32_t* done, void* workspace, size_t workspace_bytes, void* stream);
int32_t admmq_epc_end64(int64_t m, int64_t n, double* mu, int32_t* info, void* workspace, size_t workspace_bytes,
                        void* stream);

/* cp_anc's normalisation of the factors other than the one being updated
 * (source/parafac_epc.py:61-74, musco cp_anc): outA = A / max(||A[:, r]||_2, 1e-300) per column r
 * (A: rowsA x R row-major device doubles), and the same for B into outB when B is not NULL;
 * one launch, no host synchronisation. */
int32_t admmq_cp_colnorm64(const double* A, int64_t rowsA, const double* B, int64_t rowsB, int64_t R, double* outA,
                           double* outB, void* stream);

/* Library version (major*10000 + minor*100 + patch) and the last error text of this thread. */
int32_t admmq_version(void);
const char* admmq_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ADMMQ_H_ */
