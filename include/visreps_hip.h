/*
 * visreps_hip.h — C ABI of libvisreps_hip.so, the MI355X (gfx950) implementation of
 * the visreps RSA eval hot path: N×N Pearson RDM → upper-triangle midrank Spearman →
 * bootstrapped Spearman RSA.
 *
 * The reference (yashsmehta/visreps) has no FFI: its boundary is the Python module API
 * (visreps/analysis/rsa.py). Each entry point below names the reference function or
 * loop it replaces; the Python mirror in visreps_amd/analysis/rsa.py binds them with
 * ctypes.
 *
 * Conventions
 *  - Every function returns int status: VR_OK (0) or a negative VR_E* code; the
 *    message of the last failure on the calling thread is vr_last_error().
 *  - Array pointers marked [dev] are caller-owned device pointers (hipMalloc /
 *    torch.Tensor.data_ptr()); [host] pointers are host memory.
 *  - Scratch memory comes from a caller-provided workspace whose size is given by the
 *    matching *_workspace() query. The library never allocates caller-visible memory.
 *  - `stream` is a hipStream_t passed as void*; device work is enqueued on it. Calls whose
 *    launch geometry depends on device data (plan headers, key ranges, level counts)
 *    synchronise it once before returning; INTEGRATION.md lists them.
 *    Functions are reentrant across distinct streams and workspaces.
 *  - A statistic that is undefined (constant input, NaN input, fewer than two pairs)
 *    is returned as NaN in the output value, never as an error status — the same
 *    contract as compute_rdm_correlation (rsa.py:106-109,123-129).
 */
#ifndef VISREPS_HIP_H
#define VISREPS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_OK 0
#define VR_EINVAL (-1)    /* invalid argument (shape, pointer, size) */
#define VR_EHIP (-2)      /* HIP runtime error */
#define VR_EWORKSPACE (-3) /* workspace smaller than the *_workspace() query */
#define VR_EINTERNAL (-4)  /* an exact-arithmetic invariant of the result failed (a bug) */

/* Library version (major*10000 + minor*100 + patch). */
int vr_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* vr_last_error(void);

/* ------------------------------------------------------------------------------
 * RDM: replaces compute_rdm(X, correlation="Pearson", correction)
 *      visreps/analysis/rsa.py:59-93 (x.float(); x -= mean; std = sqrt(mean(x^2)+c);
 *      zero-variance guard; cov = x@x.T/D; corr = cov/(std_i std_j + c); clamp; diag=1;
 *      rdm = 1 - corr).
 * X [dev] fp32 row-major (n, d) with leading dimension ldx >= d.
 * rdm [dev] fp32 row-major (n, n) with leading dimension ldr >= n. Exactly symmetric,
 * diagonal exactly 0.
 * -------------------------------------------------------------------------- */
size_t vr_rdm_pearson_workspace(int64_t n, int64_t d);
int vr_rdm_pearson_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                       int64_t ldr, float correction, void* ws, size_t ws_bytes,
                       void* stream);

/* Block-distributed form (multi-GPU): the upper-triangle tiles of 128x128 are numbered
 * row-major (tile (bi,bj), bi <= bj); this computes tiles [tile_begin, tile_end) only and
 * writes each tile and its mirror into rdm. Entries of other tiles are not touched, so
 * ranks that each own a tile range and start from a zeroed rdm can combine with a sum
 * all-reduce. vr_rdm_tile_count(n) = number of tiles, vr_rdm_tile_cost(n, t) = distinct
 * (i <= j) entries of tile t, for balancing ranges. */
int64_t vr_rdm_tile_count(int64_t n);
// Super-tile rows R of the wide kernel in the full n x n launch at width d (0: the wide
// kernel is not used), and whether the 128-tile range [tile_begin, tile_end) is cut only at
// aligned boundaries (tri_start(2r, T), r <= R, or the end of the triangle): such a range's
// tiles are bit-identical to the full launch's (multi-GPU RDM pieces, pipeline.py).
int64_t vr_rdm_wide_rows(int64_t n, int64_t d);
int vr_rdm_range_aligned(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end);
int64_t vr_rdm_tile_cost(int64_t n, int64_t tile);
/* Rectangle of upper-triangle tile `tile`: rows [row0, row0+rows) x cols
 * [col0, col0+cols), col0 >= row0 (a diagonal tile covers its upper half). Host only;
 * for planners that place tile ranges on ranks (multi-GPU block-distributed RDM). */
int vr_rdm_tile_rect(int64_t n, int64_t tile, int64_t* row0, int64_t* col0, int64_t* rows,
                     int64_t* cols);
size_t vr_rdm_tiles_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end);
int vr_rdm_pearson_tiles_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                             int64_t ldr, float correction, int64_t tile_begin,
                             int64_t tile_end, void* ws, size_t ws_bytes, void* stream);

/* bf16 features (X holds the 16-bit patterns of torch.bfloat16, row-major with leading
 * dimension ldx): the same RDM as vr_rdm_pearson_f32 of X.float() (rsa.py:76 widens any
 * dtype to fp32), computed on the split bf16 MFMA Gram without an fp32 copy of X; the
 * row statistics and the centring read the bf16 values directly (cfg5: ViT / CLIP
 * features at N = 50k). Tile ranges as vr_rdm_pearson_tiles_f32. */
size_t vr_rdm_bf16_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end);
int vr_rdm_pearson_bf16(const uint16_t* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                        int64_t ldr, float correction, void* ws, size_t ws_bytes, void* stream);
int vr_rdm_pearson_tiles_bf16(const uint16_t* X, int64_t n, int64_t d, int64_t ldx, float* rdm,
                              int64_t ldr, float correction, int64_t tile_begin, int64_t tile_end,
                              void* ws, size_t ws_bytes, void* stream);

/* Plain symmetric Gram G = X X^T (fp32 out; the same MFMA kernels, tiling and accuracy
 * as the RDM, without centring or the correlation epilogue). The kernel matrix of the
 * encoding score's ridge regression: replaces the SVD inside himalaya 0.4.9's
 * RidgeCV(solver="svd") as called from visreps/analysis/encoding_score.py:47-62
 * (kernel form: X_val X_tr^T and X_tr X_tr^T are blocks of one Gram of the stacked rows).
 * Workspace: vr_rdm_pearson_workspace(n, d). G is exactly symmetric. */
int vr_gram_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* G, int64_t ldg,
                void* ws, size_t ws_bytes, void* stream);

/* Encoding-score statistic (visreps/analysis/encoding_score.py:206-224): for each of
 * `draws` row subsets (idx [dev] int32 draws x k; null = all n rows, draws = 1) the mean
 * over the v columns of the per-column Pearson r between Y and P (himalaya 0.4.9
 * correlation_score: zscore products, population std; zero variance -> NaN), in fp64.
 * Y, P [dev] fp32 (n, v) row-major with leading dimension ld. voxel_r [dev] fp64
 * (draws, v) or null. Workspace: vr_corr_score_workspace(v, draws). */
size_t vr_corr_score_workspace(int64_t v, int64_t draws);
int vr_corr_score_f32(const float* Y, const float* P, int64_t n, int64_t v, int64_t ld,
                      const int32_t* idx, int64_t k, int64_t draws, double* scores,
                      double* voxel_r, void* ws, size_t ws_bytes, void* stream);

/* Row statistics of the same RDM (rsa.py:80-87): mean[i] (fp32) and
 * std[i] = sqrt(mean((x-mean)^2) + correction) with std < 10*correction -> 1.
 * Exposed so extraction can emit them alongside the feature rows. */
int vr_row_stats_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* mean,
                     float* stdv, float correction, void* stream);

/* ------------------------------------------------------------------------------
 * Rank plans: the one-time per-RDM precompute behind every Spearman on that RDM.
 * The strict upper triangle (torch.triu_indices(n, n, 1) order, rsa.py:111) is
 * sorted by value once (LSD radix sort, -0.0 == +0.0), tie groups (equal fp32 values)
 * are marked, and the positions are cut into chunks aligned to group boundaries.
 * Replaces the per-call scipy.stats.rankdata(.., 'average') inside
 * scipy.stats.spearmanr (rsa.py:43-47,121-122).
 * plan [dev]: vr_rank_plan_bytes(n) bytes, owned by the caller, reused across calls.
 * -------------------------------------------------------------------------- */
size_t vr_rank_plan_bytes(int64_t n);
size_t vr_rank_plan_workspace(int64_t n);
int vr_rank_plan_build_f32(const float* rdm, int64_t n, int64_t ld, void* plan,
                           size_t plan_bytes, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Spearman of two RDMs' upper triangles: replaces
 * compute_rdm_correlation(rdm1, rdm2, correlation="Spearman") (rsa.py:96-129).
 * out [dev] one double. NaN if n<=1, any NaN value, or a constant triangle.
 * -------------------------------------------------------------------------- */
size_t vr_spearman_triu_workspace(int64_t n);
int vr_spearman_triu_f32(const float* A, const float* B, int64_t n, int64_t ld,
                         double* out, void* ws, size_t ws_bytes, void* stream);

/* Pearson of the two upper triangles (fp64), replacing
 * compute_rdm_correlation(.., correlation="Pearson") -> scipy.stats.pearsonr. */
size_t vr_pearson_triu_workspace(int64_t n);
int vr_pearson_triu_f32(const float* A, const float* B, int64_t n, int64_t ld,
                        double* out, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Bootstrapped Spearman RSA: replaces the loop
 *   for i in range(n_bootstrap):
 *       idx = rng.choice(n, int(0.9n), replace=False)
 *       scores[i] = compute_rdm_correlation(A[idx][:, idx], B[idx][:, idx], "Spearman")
 * visreps/evals.py:355-373 (identical copies evals.py:506-522, rsa.py:233-261).
 *
 * The engine evaluates 64 subsets per pass (one bit per subset in a per-stimulus
 * 64-bit inclusion mask); every score is exact integer midrank arithmetic on the
 * pre-sorted plans, so results do not depend on pass grouping or GPU count.
 *
 * idx [dev] int32 (n_sets, k): stimulus indices of each subset (distinct, in [0,n)).
 *   If full_first != 0 an extra first subset = all n stimuli is evaluated and its
 *   score written to scores[0] (the point estimate, evals.py:347-349), followed by the
 *   n_sets subset scores. scores [dev] double (n_sets + (full_first?1:0)).
 * -------------------------------------------------------------------------- */
size_t vr_bootstrap_workspace(int64_t n);
int vr_bootstrap_spearman_plans(const void* planA, const void* planB, int64_t n,
                                const int32_t* idx, int64_t k, int64_t n_sets,
                                int full_first, double* scores, void* ws,
                                size_t ws_bytes, void* stream);

/* Units that share one RDM: the bootstrap loop of evals.py:323-373 runs every model
 * layer against the same neural RDM with the same RandomState(42) subsets. plan_a (the
 * shared RDM) against each of the n_b plans in planBs [host array of device pointers].
 * Per pass of 64 subsets the rank walk of plan_a runs once for all n_b units. Row j of
 * scores [dev] double (n_b rows, leading dimension ld_scores >= n_sets + full_first)
 * equals vr_bootstrap_spearman_plans(planBs[j], plan_a, ...) bit for bit (Spearman is
 * symmetric and every sum is an exact integer). Workspace grows by 8 bytes per pair for
 * every B plan after the first. */
size_t vr_bootstrap_multi_workspace(int64_t n, int64_t n_b);
int vr_bootstrap_spearman_multi(const void* plan_a, const void* const* planBs, int64_t n_b,
                                int64_t n, const int32_t* idx, int64_t k, int64_t n_sets,
                                int full_first, double* scores, int64_t ld_scores, void* ws,
                                size_t ws_bytes, void* stream);
/* Shared joins for units that share their B plan across up to 4 A plans (the neural RDMs of
 * the regions one model layer is scored against; the per-unit joins of
 * vr_bootstrap_spearman_multi, evals.py:355-373's loop over regions). vr_engine_posmap4
 * interleaves the A plans' pair -> position maps into 16-B records (posmap4: workspace of
 * vr_engine_posmap4_bytes(n)); vr_engine_join4 then gives, for one B plan, posA[i][q] = the
 * position in A plan i of B's pair at position q (M u32 each) with one 16-B gather per pair,
 * where one join per unit gathers a random line per pair for each A plan. */
size_t vr_engine_posmap4_bytes(int64_t n);
int vr_engine_posmap4(const void* const* plan_as, int64_t n_a, int64_t n, void* posmap4, void* stream);
int vr_engine_join4(const void* posmap4, int64_t n_a, const void* plan_b, int64_t n, uint32_t* const* posA,
                    void* stream);
/* vr_bootstrap_spearman_multi with every unit's A positions already joined (posA[j], M u32,
 * from vr_engine_join4 against this call's A plan): the EST passes read them and skip the
 * per-unit joins. posA is in/out: an exact-form pass (a flagged EST pass re-run, or
 * VISREPS_ENGINE_EST=0) rewrites posA[j] in place, with the same values, beside its A chunks.
 * Workspace vr_bootstrap_multi_joined_workspace(n, n_b): 4 B per pair and unit less than
 * vr_bootstrap_multi_workspace (no posA arrays carved for units after the first). */
size_t vr_bootstrap_multi_joined_workspace(int64_t n, int64_t n_b);
int vr_bootstrap_spearman_multi_joined(const void* plan_a, const void* const* planBs, int64_t n_b, int64_t n,
                                       const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                                       double* scores, int64_t ld_scores, uint32_t* const* posA, void* ws,
                                       size_t ws_bytes, void* stream);
/* The units of n_a <= 4 A plans (regions) x n_b B plans (model layers) on the same subsets,
 * every unit pre-joined: posA[i * n_b + j] = B plan j's pairs in A plan i (vr_engine_join4);
 * unit (j, i)'s scores at scores + (i * n_b + j) * ld_scores. Equal bit for bit to n_a
 * vr_bootstrap_spearman_multi_joined calls (evals.py:323-373's region x layer loop, whose
 * RandomState(42) gives every region the same index sets): the EST passes walk each B plan
 * once for all regions (their window inclusion bits, group flags and B counts are the same),
 * the regions' rank tables resident together; anything off that path (exact form, masks
 * beyond LDS, giant tie groups, a flagged pass) runs the per-region calls. Workspace
 * vr_bootstrap_grid_joined_workspace(n, n_a, n_b) = n_a x the per-region joined workspace. */
size_t vr_bootstrap_grid_joined_workspace(int64_t n, int64_t n_a, int64_t n_b);
int vr_bootstrap_spearman_grid_joined(const void* const* plan_as, int64_t n_a, const void* const* planBs,
                                      int64_t n_b, int64_t n, const int32_t* idx, int64_t k, int64_t n_sets,
                                      int full_first, double* scores, int64_t ld_scores, uint32_t* const* posA,
                                      void* ws, size_t ws_bytes, void* stream);

/* Passes of the bootstrap engines run in a one-gather-per-pair form (absolute ranks kept
 * modulo 2^16 and recovered against a count estimate). A pass whose ranks the estimate
 * cannot recover (very large tie groups, adversarial orders) -- flagged by the A walk's
 * window checks, or by the tail's invariants (B-side included pairs == M', sum of the
 * gathered A ranks == M'(M'+1)) -- is re-run in the exact chunk-base form; this counter is
 * the number of such re-runs in the process so far (scores never depend on it).
 * VISREPS_ENGINE_EST=0 forces the chunk-base form; an exact-form pass that breaks the
 * invariants fails the call with VR_EINTERNAL. */
int64_t vr_engine_est_reruns(void);
/* Of those re-runs, the passes only the tail invariants flagged: the A walk's window checks
 * passed, so the B side recovered a wrong rank (0 unless a bug or a fault injection). */
int64_t vr_engine_est_tail_flags(void);
/* Test hook, not for product use: from the next engine call on, after the A walk of EST
 * pass `pass` one TB row's lanes 1..63 are corrupted (a B-side error the A walk cannot
 * see), so the tail invariants and the exact re-run can be tested. -1 (the default) = off. */
int vr_test_engine_inject(int64_t pass);
/* Engine calls whose first pass's A counts (a count pre-pass before any EST pass) already
 * put some subset's ranks outside the EST 3 window, so the call left EST 3 without spending
 * a flagged EST pass (VISREPS_ENGINE_EST_PREDICT=0 disables the check). */
int64_t vr_engine_est_predicted(void);
/* Of those, the calls run in EST 1 (per-lane count tables) instead of the exact form
 * (VISREPS_ENGINE_EST1_FALLBACK=0: exact form). */
int64_t vr_engine_est1_fallbacks(void);

// Kernel-level HIP-event timing of the hot kernels, for pricing the dominant kernel against
// its roofline on the stream it runs on (bench.py). Off by default; enabling clears the
// totals. kernel: 0 k_rankB EST forms over bootstrap subsets, 1 k_rankB exact form, 2 k_rankA,
// 3 k_join/k_join_lo, 4 k_gram3p/k_gram3w (256^2 super-tiles), 5 k_gram3/k_gram (128^2 tiles),
// 6 k_countA, 7 k_rankB EST 4 (the full-set pass: point estimates, phase-1 selections), 8 k_kwalk
// (one Kendall stream walk of one pass), 9 k_cov (fp64 MFMA covariance / ridge Gram tiles).
// units: pairs walked (engine kernels) or tile FLOPs 2 d x tile elements (Gram kernels).
// No reference counterpart (the reference has no native kernels).
int vr_ktimer_enable(int on);
int vr_ktimer_read(int kernel, double* ms, int64_t* launches, double* units);
// Trace marker: launches an empty kernel (k_trace_mark_begin if begin, else
// k_trace_mark_end) on `stream`, to bracket a region in a rocprofv3 kernel trace.
int vr_trace_mark(int begin, int tag, void* stream);

/* One-shot form: builds both plans in the workspace, then runs the engine. */
size_t vr_bootstrap_spearman_workspace(int64_t n);
int vr_bootstrap_spearman_f32(const float* A, const float* B, int64_t n, int64_t ld,
                              const int32_t* idx, int64_t k, int64_t n_sets,
                              int full_first, double* scores, void* ws, size_t ws_bytes,
                              void* stream);

/* ------------------------------------------------------------------------------
 * Kendall tau-a of two RDMs' upper triangles: replaces
 * compute_rdm_correlation(rdm1, rdm2, correlation="Kendall") -> _kendall_tau_a
 * (visreps/analysis/rsa.py:22-40,96-129): scipy.stats.kendalltau tau-b from exact
 * discordant / tie counts, converted to tau-a = tau_b sqrt((n0-tx)(n0-ty)) / n0.
 * out [dev] one double; NaN for n <= 1, NaN input or a constant triangle.
 * -------------------------------------------------------------------------- */
size_t vr_kendall_triu_workspace(int64_t n);
int vr_kendall_triu_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out,
                        void* ws, size_t ws_bytes, void* stream);

/* Kendall tau-a of two plain fp64 vectors of length m: replaces `_kendall_tau_a(x, y)`
 * itself (visreps/analysis/rsa.py:22-40; imported by the reference's
 * tests/test_rsa_bootstrap.py:46). Every unordered pair compared in fp64, exact integer
 * discordant / tie counts, then the same tau-b -> tau-a conversion as vr_kendall_triu_f32.
 * x, y, out [dev]; out = NaN for m < 2, a NaN element or a constant vector. m <= 2^22
 * (O(m^2) pair work; RDM triangles go through vr_kendall_triu_f32). */
size_t vr_kendall_vec_workspace(int64_t m);
int vr_kendall_tau_a_f64(const double* x, const double* y, int64_t m, double* out, void* ws,
                         size_t ws_bytes, void* stream);

/* The same statistic in O(m log m) for any m < 2^32 (the reference's `_kendall_tau_a` has no
 * size cap: scipy.stats.kendalltau's merge-sort counting, rsa.py:28): both vectors to dense
 * ranks (radix sorts), the (x, y)-lexicographic order, then the discordant pairs as the
 * inversions of the y ranks counted one rank bit per level (kendall_full.hip). Exact integer
 * counts, so equal bit for bit to vr_kendall_tau_a_f64 where both run. x, y, out [dev]. */
size_t vr_kendall_full_vec_workspace(int64_t m);
int vr_kendall_full_vec_f64(const double* x, const double* y, int64_t m, double* out, void* ws,
                            size_t ws_bytes, void* stream);

/* Kendall tau-a of the strict upper triangles of two RDMs beyond the rank plans' 16-bit
 * stimulus indices (compute_rdm_correlation(.., "Kendall"), rsa.py:96-129 -> rsa.py:22-40, at
 * n > 65,535): the kendall_full.hip pipeline on the M = n(n-1)/2 < 2^32 triangle elements
 * (n <= 92,681; configs[2]'s 73k RDM). A, B [dev] (n, n) row-major fp32, leading dimension
 * ld; out [dev] one double (NaN for M < 2, NaN input, a constant triangle). */
size_t vr_kendall_full_workspace(int64_t n);
int vr_kendall_full_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out, void* ws,
                        size_t ws_bytes, void* stream);
/* ... of the sub-RDMs A[idx][:, idx], B[idx][:, idx] (k rows idx [dev] int32 into the n x n
 * RDMs, never materialised): one bootstrap draw of evals.py:361-369 with compare_method=kendall
 * beyond the rank plans. Workspace: vr_kendall_full_workspace(k). */
int vr_kendall_full_subset_f32(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                               int64_t k, double* out, void* ws, size_t ws_bytes, void* stream);

/* Bootstrapped Kendall RSA on two rank plans: the bootstrap loop of evals.py:355-373 /
 * rsa.py:233-261 with compare_method="kendall". Arguments as
 * vr_bootstrap_spearman_plans; the workspace depends on the number of subsets:
 * vr_bootstrap_kendall_workspace(n, n_sets) covers up to n_sets subsets plus the full set. */
size_t vr_bootstrap_kendall_workspace(int64_t n, int64_t n_sets);
int vr_bootstrap_kendall_plans(const void* planA, const void* planB, int64_t n,
                               const int32_t* idx, int64_t k, int64_t n_sets, int full_first,
                               double* scores, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Phase-1 sparse random projection (extraction side).
 * Replaces torch.sparse.mm(P, flat.t()).t() (visreps/models/utils.py:334-336) with P the
 * CSR (k x D) components_ of sklearn SparseRandomProjection
 * (visreps/models/utils.py:297-322, visreps/analysis/sparse_random_projection.py:83-150).
 * indptr (k+1) / indices (nnz) int32, values (nnz) fp32, X (B x D, row stride ldx) fp32,
 * out (B x k, row stride ldo) fp32 -- all device. fp32 fma in CSR order per output.
 * -------------------------------------------------------------------------- */
size_t vr_srp_workspace(int64_t B, int64_t D);
int vr_srp_csr_f32(const int32_t* indptr, const int32_t* indices, const float* values,
                   int64_t k, int64_t D, const float* X, int64_t B, int64_t ldx, float* out,
                   int64_t ldo, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Full-triangle Spearman of two RDMs with up to 2^32 - 1 pairs (n <= 92681), no rank plan:
 * the compute_rdm_correlation(.., "Spearman") path above the engine's 16-bit stimulus
 * indices (rsa.py:96-129 at configs[2]'s 73k stimuli). Average ranks from per-key counts
 * of each triangle's fp32 keys (count tables over the key range, no sort) or, when the key
 * range does not fit the workspace, a radix sort of (key, triangle index); exact u128 sums
 * either way; out [device] one double. vr_spearman_full_workspace(n) covers every RDM whose
 * values span at most 2^30 + 1 fp32 keys (all correlation-distance RDMs: values in [0, 2]);
 * on a wider range the call returns VR_EWORKSPACE and vr_spearman_full_sort_workspace(n)
 * is the size that always suffices.
 * -------------------------------------------------------------------------- */
size_t vr_spearman_full_workspace(int64_t n);
size_t vr_spearman_full_sort_workspace(int64_t n);
/* Form the last vr_spearman_full_* call took: 0 bucketed count tables, 1 plain count tables,
 * 2 radix sort (-1 before any call). */
int vr_spearman_full_last_form(void);
int vr_spearman_full_f32(const float* A, const float* B, int64_t n, int64_t ld, double* out,
                         void* ws, size_t ws_bytes, void* stream);
/* ... of the sub-RDMs A[idx][:, idx], B[idx][:, idx] (k rows idx [dev] int32, never
 * materialised): one bootstrap draw of evals.py:361-369 beyond the rank plans' n <= 65,535
 * (the bootstrap engine's per-pass TB rows would need 128 B per pair: 341 GB at 73k).
 * Workspace: vr_spearman_full_workspace(k). */
int vr_spearman_full_subset_f32(const float* A, const float* B, int64_t n, int64_t ld, const int32_t* idx,
                                int64_t k, double* out, void* ws, size_t ws_bytes, void* stream);
/* Local pieces of the distributed global rank (sample sort over ranks,
 * visreps_amd/analysis/distributed_spearman.py): sortable keys of fp32 values, an in-place
 * (key, value) radix sort, doubled midranks (+ 2 base) of a sorted key run with its tie
 * term sum (k^3 - k) as a u128 {lo, hi}, and an exact u64 dot product (u128 {lo, hi}). */
/* Count-table form of the same global rank (no sort, no key exchange): per-key counts of a
 * rank's sortable keys in [kmin, kmin + bins) into cnt[bins + 1] (zeroed by the caller;
 * atomics), which the caller sums over ranks; then, on the summed table, the tie term sum
 * (c^3 - c) as a u128 {lo, hi}, the table turned into exclusive starts in place, and the
 * doubled midranks cnt[k] + cnt[k + 1] + 1 of this rank's keys. */
int vr_key_counts_u32(const uint32_t* keys, int64_t m, uint32_t kmin, int64_t bins, uint32_t* cnt, void* stream);
size_t vr_key_table_workspace(int64_t bins);
int vr_key_table_midranks(const uint32_t* keys, int64_t m, uint32_t kmin, uint32_t* cnt, int64_t bins, uint64_t* y,
                          uint64_t* tie, void* ws, size_t ws_bytes, void* stream);
int vr_f32_sort_keys(const float* v, int64_t m, uint32_t* keys, void* stream);
size_t vr_sort_pairs_workspace(int64_t m);
int vr_sort_pairs_u32(uint32_t* keys, uint32_t* vals, int64_t m, void* ws, size_t ws_bytes,
                      void* stream);
size_t vr_midranks_workspace(int64_t m);
int vr_midranks_sorted(const uint32_t* keys, int64_t m, uint64_t base, uint64_t* y, uint64_t* tie,
                       void* ws, size_t ws_bytes, void* stream);
size_t vr_dot_u64_workspace(void);
int vr_dot_u64(const uint64_t* a, const uint64_t* b, int64_t m, uint64_t* out, void* ws,
               size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Multi-GPU RDM pieces (stimulus-sharded rows); replace the
 * block-distributed use of vr_rdm_pearson_tiles_f32 + a sum all-reduce:
 *  - each rank splits its own rows (row stats + centred bf16 hi/lo plane records);
 *  - the planes and stats are all-gathered (the only feature exchange);
 *  - each rank computes its tile range from the gathered planes;
 *  - the ranges are exchanged packed (vr_rdm_tiles_pack -> all-gather -> unpack, which
 *    also writes the mirror), instead of a zero-filled n x n sum all-reduce.
 * Plane buffers hold vr_rdm_plane_rows(n) rows of vr_rdm_plane_row_bytes(d) bytes, rows
 * >= n zero. A packed tile range holds 128 x 128 floats per tile, in tile order.
 * -------------------------------------------------------------------------- */
int64_t vr_rdm_plane_rows(int64_t n);
size_t vr_rdm_plane_row_bytes(int64_t d);
int vr_rdm_split_rows_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, float correction,
                          float* mean, float* stdv, uint16_t* planes, void* stream);
/* The same split for the same `rows` rows of npts points (<= 32) in one launch (rows x npts
 * blocks): X[p] (rows, d[p]) with row stride ldx[p], outputs mean[p], stdv[p], planes[p].
 * Host arrays of device pointers. Used by bench.extract_split on each extraction batch. */
int vr_rdm_split_rows_multi_f32(int npts, const float* const* X, const int64_t* d, const int64_t* ldx,
                                int64_t rows, float correction, float* const* mean, float* const* stdv,
                                uint16_t* const* planes, void* stream);
/* Rows src[i] (host array, nrows entries) of every point's X[p] (row stride ldx[p], d[p]
 * floats) to rows dst[i] of out[p] (row stride ldo[p]): one launch per 64 rows for all
 * npts (<= 32) points. bench.extract_split keeps the phase-1 selection rows of each
 * extraction batch with it (the rows `RandomState(42).choice` picks, evals.py:259-263). */
int vr_gather_rows_multi_f32(int npts, const float* const* X, const int64_t* d, const int64_t* ldx,
                             int nrows, const int32_t* src, const int32_t* dst, float* const* out,
                             const int64_t* ldo, void* stream);
size_t vr_rdm_planes_tiles_workspace(int64_t n, int64_t d, int64_t tile_begin, int64_t tile_end);
int vr_rdm_pearson_tiles_planes(const uint16_t* planes, const float* mean, const float* stdv,
                                int64_t n, int64_t d, float* rdm, int64_t ldr, float correction,
                                int64_t tile_begin, int64_t tile_end, void* ws, size_t ws_bytes,
                                void* stream);
int vr_rdm_tiles_pack(const float* rdm, int64_t ldr, int64_t n, int64_t tile_begin,
                      int64_t tile_end, float* packed, void* stream);
int vr_rdm_tiles_unpack(const float* packed, int64_t n, int64_t tile_begin, int64_t tile_end,
                        float* rdm, int64_t ldr, void* stream);

/* One RDM over stimulus-sharded rows behind the C ABI (SURVEY §8(b),(e)): rank `rank` of an
 * RCCL communicator `comm` (ncclComm_t) holds rows_local <= ceil(n / world) consecutive
 * stimulus rows X_local [dev] fp32 (row stride ldx), the ranks' blocks in rank order make
 * the n rows. Block sizes, the split bf16 hi/lo plane records (+ row statistics) and the
 * packed tile ranges are all-gathered over RCCL; each rank computes one tile range cut at
 * the wide kernel's aligned boundaries (vr_rdm_sharded_range: bit-identical tiles to the
 * one-GPU split-Gram launch), and every rank ends with the full RDM in rdm [dev] (ldr >= n).
 * Collective: every rank calls it with the same n, d, world. RCCL is bound at run time
 * (librccl.so.1, the copy torch loaded if any); vr_rccl_* create a communicator from it for
 * callers without their own RCCL binding. No reference counterpart (single-GPU reference). */
int vr_rccl_available(void);
int vr_rccl_unique_id(void* out /* 128 bytes (ncclUniqueId) */);
int vr_rccl_comm_init(void** comm, int world, const void* unique_id, int rank);
int vr_rccl_comm_destroy(void* comm);
int vr_rdm_sharded_range(int64_t n, int64_t d, int world, int rank, int64_t* tile_begin, int64_t* tile_end);
size_t vr_rdm_sharded_workspace(int64_t n, int64_t d, int world);
int vr_rdm_pearson_sharded(const float* X_local, int64_t rows_local, int64_t n, int64_t d, int64_t ldx, float* rdm,
                           int64_t ldr, float correction, void* comm, int rank, int world, void* ws, size_t ws_bytes,
                           void* stream);

/* The collective behind the sharded entry points, as a table: all_gather(send, recv, bytes,
 * user, stream) must leave rank r's `bytes` of send at recv + r * bytes on every rank, ordered
 * on `stream`, and return 0 (non-zero fails the call with VR_EHIP). vr_comm_rccl fills the table
 * with RCCL's ncclAllGather over `nccl_comm` (what vr_rdm_pearson_sharded uses); a caller with
 * another transport (MPI, a host loopback in tests) fills it itself. */
typedef int (*vr_allgather_fn)(const void* send, void* recv, size_t bytes, void* user, void* stream);
typedef struct vr_comm {
  int world;
  int rank;
  vr_allgather_fn all_gather;
  void* user;
} vr_comm;
int vr_comm_rccl(vr_comm* out, void* nccl_comm, int world, int rank);
int vr_rdm_pearson_sharded_comm(const float* X_local, int64_t rows_local, int64_t n, int64_t d, int64_t ldx,
                                float* rdm, int64_t ldr, float correction, const vr_comm* comm, void* ws,
                                size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Image preprocessing: the eval loaders' get_transform (visreps/dataloaders/obj_cls.py:
 * 27-45) = torchvision Resize(resize, BILINEAR) on a PIL image (Pillow's ImagingResample:
 * antialiased separable bilinear, 22-bit fixed point, uint8 intermediate) ->
 * CenterCrop(crop) -> ToTensor -> Normalize(mean, std), bit-exact.
 * src [device] B x H x W x 3 uint8 (RGB, same size images); out [device] B x 3 x crop x
 * crop float32; mean, std [host] 3 floats each. crop must not exceed the resized image.
 * -------------------------------------------------------------------------- */
size_t vr_transform_workspace(int64_t B, int64_t H, int64_t W, int64_t resize, int64_t crop,
                              int filter);
/* filter: 0 = BILINEAR (get_transform), 1 = BICUBIC (the CLIP and timm DINOv3 loaders,
 * clip_representations.py:27, dino_representations.py:31-32) */
int vr_transform_u8(const uint8_t* src, int64_t B, int64_t H, int64_t W, int64_t resize,
                    int64_t crop, int filter, const float* mean, const float* std, float* out,
                    void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * PCA covariance for the coarse-grained PCA labels: replaces
 * batched_pca's mean and covariance, scripts/coarsegrain/compute_eigenvectors.py:23-36
 *   mean = X.mean(axis=0);  cov = sum_b (X[b].astype(f64) - mean)^T (..) / (n - 1).
 * X [dev] fp32 row-major (n, p), leading dimension ldx >= p.
 * -------------------------------------------------------------------------- */
/* Column sums in numpy's float32 order (rows added in row order, one float32 running sum
 * per column), continued from init [dev] p (nullable: 0). sum [dev] p. Bit-identical to
 * numpy's X.sum(axis=0) on a C-order float32 array; chained over row shards it is the
 * same sum (the multi-GPU form passes the previous shard's sum as init). */
int vr_col_sum_f32(const float* X, int64_t n, int64_t p, int64_t ldx, const float* init,
                   float* sum, void* stream);
/* X.mean(axis=0) as numpy: the column sums / float32(n). mean [dev] p. */
int vr_col_mean_f32(const float* X, int64_t n, int64_t p, int64_t ldx, float* mean, void* stream);
/* mean [dev] p = sum [dev] p / float32(n) (may alias). */
int vr_mean_from_sum_f32(const float* sum, int64_t p, int64_t n, float* mean, void* stream);
/* cov [dev] fp64 (p, p), leading dimension ldc: sum over rows of
 * ((double)x - (double)mean)^T ((double)x - (double)mean) / denom, exactly symmetric, on
 * the fp64 MFMA. mean [dev] fp32 p. denom = n - 1 for the reference's covariance, 1 for a
 * rank's partial sum (multi-GPU: all-reduce, then divide). */
size_t vr_pca_cov_workspace(int64_t n, int64_t p);
int vr_pca_cov_f64(const float* X, int64_t n, int64_t p, int64_t ldx, const float* mean,
                   double denom, double* cov, int64_t ldc, void* ws, size_t ws_bytes,
                   void* stream);

/* Uncentred fp64 Grams of fp32 features on the same fp64 MFMA tiles (the encoding score's
 * ridge): replaces the fp64 X^T X / X X^T that himalaya 0.4.9's
 * RidgeCV(solver="svd") needs, called from visreps/analysis/encoding_score.py:47-62.
 * X [dev] fp32 row-major (n, p), leading dimension ldx >= p. rows = 0: G = X^T X (p x p,
 * the primal form, p < n); rows = 1: G = X X^T (n x n, the kernel form, p >= n). Products
 * of two fp32 values are exact in fp64, sums fp64. G [dev] fp64, leading dimension ldg,
 * exactly symmetric. Workspace: vr_gram64_workspace(n, p, rows). */
size_t vr_gram64_workspace(int64_t n, int64_t p, int rows);
int vr_gram64_f32(const float* X, int64_t n, int64_t p, int64_t ldx, int rows, double* G, int64_t ldg,
                  void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------
 * Host: legacy numpy RandomState (MT19937) index streams, bit-exact.
 * Replaces np.random.RandomState(seed) + .choice(n, k, replace=False) / .permutation(n)
 * (evals.py:260-261,356,362-364; rsa.py:169,176,248-250; evals.py:111-113).
 * -------------------------------------------------------------------------- */
/* Opaque generator state (caller-allocated, vr_rng_state_bytes() bytes). */
size_t vr_rng_state_bytes(void);
int vr_rng_seed(void* state, uint32_t seed);                /* RandomState(seed) */
int vr_rng_permutation(void* state, int64_t n, int32_t* out); /* .permutation(n) */
int vr_rng_choice(void* state, int64_t n, int64_t k, int32_t* out); /* .choice(n,k,replace=False) */
int vr_rng_random_u32(void* state, int64_t count, uint32_t* out);   /* raw MT19937 draws */
/* Convenience: fresh RandomState(seed), then n_draws successive choice(n, k) calls
 * into out (n_draws, k) [host]. */
int vr_legacy_choice(uint32_t seed, int64_t n, int64_t k, int64_t n_draws, int32_t* out);

/* numpy.percentile(x, q) with the default 'linear' method (evals.py:371-372),
 * NaN-propagating. x [host] double (n). Returns the percentile (NaN if n == 0). */
double vr_percentile_linear(const double* x, int64_t n, double q);

#ifdef __cplusplus
}
#endif

#endif /* VISREPS_HIP_H */
