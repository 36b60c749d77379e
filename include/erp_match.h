/*
 * erp_match.h -- C ABI of the MI355X-native ERP matcher + spherical eight-point estimator.
 *
 * This is the drop-in boundary for the reference's hot path (Kitsunetic/ERP_match_eightpoint_test):
 *
 *   erp_match_two_image / erp_match_knn2_ratio
 *       replaces  std::vector<cv::DMatch> feature_matcher::match_two_image(
 *                     const cv::Mat& descriptor1, const cv::Mat& descriptor2)
 *                 /root/reference/src/feature_matcher.hpp:36, body src/feature_matcher.cpp:42-59
 *                 (FLANN knnMatch k=2 + ratio 0.3f; here: EXACT k=2 in flann::L2 order).
 *   erp_eight_point_find
 *       replaces  void eight_point::find(int im_width, int im_height,
 *                     std::vector<cv::KeyPoint>& key_left, std::vector<cv::KeyPoint>& key_right,
 *                     cv::Vec3f& R_vec_out, cv::Vec3f& T_vec_out, int match_size)
 *                 /root/reference/src/eight_point.hpp:11-14, body src/eight_point.cpp:152-192
 *                 (initial_guess :87-150 and the random_array sampler eight_point.hpp:30-59 run
 *                  inside; the iteration count, sample fraction, trim window and validity bound
 *                  are the hard-coded constants of :99,:102,:143,:76 exposed in erp_ransac_cfg).
 *   erp_eight_point_estimation
 *       replaces  void eight_point::eight_point_estimation(int, int, std::vector<cv::Point3d>&,
 *                     std::vector<cv::Point3d>&, cv::Vec3f& R1, cv::Vec3f& R2, cv::Vec3f& T,
 *                     bool& R1_valid, bool& R2_valid, int match_size)
 *                 /root/reference/src/eight_point.hpp:15-19, body src/eight_point.cpp:16-85
 *   erp_pair_batch_run
 *       the fused hot path for many ERP pairs at once: spherical_surf::do_all's
 *       match -> gather (src/spherical_surf.cpp:153-162, 177) -> eight_point::find
 *       (src/automatic.cpp:117-126 calls exactly this sequence per pair).
 *
 * Conventions: plain C types only; `void* stream` is a hipStream_t (NULL = default stream);
 * device-pointer entry points are asynchronous on that stream, host-pointer ones synchronous.
 * A context (erp_ctx) owns grow-only scratch that every call on it reuses, so calls on one
 * context are serialised on the device: a call enqueued on a different stream than the previous
 * call on the same context first waits (hipStreamWaitEvent) for that call's work to finish.
 * Independent work that should overlap needs one context per stream.  Calls are thread-safe
 * (one lock per context; host-pointer calls hold it across upload, run and download).
 * No C++ exception crosses this boundary; every call returns an erp_status.  The reference's
 * undefined behaviour cases are given explicit statuses (see erp_status).
 */
#ifndef ERP_MATCH_H
#define ERP_MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ERP_MATCH_ABI_VERSION 2  /* 2: erp_ctx_set_option replaced the environment knobs (r06) */

typedef enum erp_status {
    ERP_OK = 0,
    ERP_INVALID_ARG = 1,
    ERP_TOO_FEW_POINTS = 2,       /* train set < 2 (knn_matches[i][1] UB, feature_matcher.cpp:52),
                                     or (int)(M*sample_frac) < 1 (A_mat with 0 rows, :18) */
    ERP_NO_VALID_HYPOTHESIS = 3,  /* K == 0: R_vec_arr[min_idx] on an empty vector (:148) */
    ERP_HIP_ERROR = 4,
    ERP_NO_DEVICE = 5,
    ERP_OUT_OF_MEMORY = 6,
    ERP_INTERNAL = 7
} erp_status;

/* cv::DMatch layout */
typedef struct erp_dmatch {
    int32_t queryIdx;
    int32_t trainIdx;
    int32_t imgIdx;
    float distance;
} erp_dmatch;

/* cv::KeyPoint::pt (the only KeyPoint field the hot path reads) */
typedef struct erp_point2f {
    float x;
    float y;
} erp_point2f;

typedef enum erp_sampler {
    ERP_SAMPLER_GLIBC = 0, /* replay of glibc rand() + libstdc++ random_shuffle (the reference) */
    ERP_SAMPLER_PHILOX = 1 /* counter-based, no reference counterpart:
                              iteration h's subset by Floyd's algorithm on Philox4x32-10 draws,
                              h = offset + iteration (offset counts iterations, not rand() calls);
                              the exact definition: oracle/erp_oracle.c erpo_philox_sample.
                              A pair with more than 20480 matches (the per-lane LDS bitmap)
                              gets ERP_INVALID_ARG. */
} erp_sampler;

/* initial_guess parameters; erp_ransac_cfg_default() gives the reference constants. */
typedef struct erp_ransac_cfg {
    int32_t iters;       /* 80   src/eight_point.cpp:99 */
    int32_t sampler;     /* ERP_SAMPLER_GLIBC (the reference) or ERP_SAMPLER_PHILOX */
    double sample_frac;  /* 0.25 :102 */
    double trim_lo;      /* 0.2  :143 */
    double trim_hi;      /* 0.8  :143 */
    double valid_abs;    /* 1.57 :76,81 */
    uint32_t seed;       /* 1: the reference never calls srand() */
    float inlier_thr;    /* 0 (default) = off: nothing below changes.  > 0: every iteration also
                            counts its inliers, the correspondences with |l^T E' r| < inlier_thr
                            (l, r the unit bearings of a match, E' = E_mat_correct of that
                            iteration, src/eight_point.cpp:46-50: the rank-2 correction of the
                            unit-norm solved e), into erp_hypothesis.inliers (the winner's count:
                            the record of the iteration that pushed row min_idx).  No reference
                            counterpart (its loop, :99-127, keeps no score): the opt-in
                            "inlier count" of SURVEY.md F2.  Exact definition (fp64, fixed
                            order): u_k = l_i * r_j (k = 3i + j), res = E'_0 u_0, then
                            res = fma(E'_k, u_k, res) for k = 1..8; inlier iff |res| < thr
                            (oracle/erp_oracle.c erpo_inlier_count). */
    uint64_t offset;     /* rand() calls consumed before initial_guess (e.g. by FLANN) */
} erp_ransac_cfg;

/* one initial_guess iteration (R1, R2, T as Vec3f; E = the solved 9-vector, sign arbitrary) */
typedef struct erp_hypothesis {
    float R1[3];
    float R2[3];
    float T[3];
    int32_t R1_valid;
    int32_t R2_valid;
    int32_t inliers;     /* matches with |l^T E' r| < cfg.inlier_thr (erp_ransac_cfg); 0 when off */
    double E[9];
} erp_hypothesis;

/* per-pair result of find / the batch pipeline */
typedef struct erp_pair_result {
    float R[3];          /* R_vec_out (XYZ Euler, rad) */
    float T[3];          /* T_vec_out (unit) */
    int32_t status;      /* erp_status of this pair */
    int32_t M;           /* matches after the ratio test (match_size) */
    int32_t K;           /* valid rotation hypotheses */
    int32_t min_idx;     /* consensus winner in R_vec_arr order */
    int32_t sample_n;    /* (int)(M * sample_frac) */
    int32_t near_ties;   /* rows re-scored exactly by the near-tie resolver */
    int32_t survivors;   /* rows whose trimmed-mean bounds did not exclude them (a diagnostic:
                            it depends on which pruning references ran, so a row-sharded
                            consensus -- erp_consensus_hyps_shard/finish_dev -- may report a
                            different count than the unsharded one; 1 <= survivors <= K, and
                            <= binned_rows when that is reported) */
    int32_t binned_rows; /* rows whose K-column distance histogram was built (K, or the
                            reference rows + the rows Lipschitz pre-pruning kept; K on the
                            row-sharded path, whose shards do not combine it) */
    double min_dist;     /* trimmed-mean distance of the winner */
} erp_pair_result;

/* device pointers describing a batch of ERP pairs (rows concatenated pair after pair) */
typedef struct erp_pair_batch {
    int32_t n_pairs;
    int32_t dim;                /* descriptor length (64 for SURF; the fast path needs 64) */
    int32_t max_nq;             /* host-known upper bound of rows per pair (queries / left) */
    int32_t max_nt;             /* ... (train / right) */
    const float* desc_l;        /* [sum nq][dim] queries  (descriptor1) */
    const float* desc_r;        /* [sum nt][dim] train    (descriptor2) */
    const erp_point2f* kp_l;    /* [sum nq] keypoints of desc_l rows */
    const erp_point2f* kp_r;    /* [sum nt] */
    const int64_t* off_l;       /* [n_pairs+1] row offsets into desc_l / kp_l */
    const int64_t* off_r;       /* [n_pairs+1] */
    const int32_t* width;       /* [n_pairs] ERP width  (im_width) */
    const int32_t* height;      /* [n_pairs] ERP height (im_height) */
} erp_pair_batch;

/* optional device outputs of the batch pipeline (NULL = not needed) */
typedef struct erp_batch_outputs {
    erp_pair_result* results;   /* [n_pairs] (required) */
    erp_dmatch* matches;        /* [n_pairs][max_nq], queryIdx/trainIdx local to the pair */
    erp_point2f* key_left;      /* [n_pairs][max_nq] gathered matched keypoints (valid_key_left) */
    erp_point2f* key_right;     /* [n_pairs][max_nq] */
    erp_hypothesis* hyps;       /* [n_pairs][iters] */
    int32_t* samples;           /* [n_pairs][iters][max sample_n] sampled match indices (as a set,
                                   order unspecified) */
    float* rvec;                /* [n_pairs][2*iters][3] R_vec_arr */
    float* tvec;                /* [n_pairs][2*iters][3] T_vec_arr */
    double* dist;               /* [n_pairs][2*iters] trimmed means of the rows that survive the
                                   bounds test (exact order statistics, fp64 sum; near ties are
                                   re-scored with the reference's sorted sequential sum); +inf for
                                   rows proven not to be the minimum */
} erp_batch_outputs;

typedef struct erp_ctx erp_ctx;

/* ---- context ---- */
erp_status erp_ctx_create(int32_t device, erp_ctx** out);
erp_status erp_ctx_destroy(erp_ctx* ctx);
const char* erp_status_string(erp_status s);
void erp_ransac_cfg_default(erp_ransac_cfg* cfg);
int32_t erp_abi_version(void);
/* Pre-size device scratch so later calls allocate nothing (graph-capture friendly). */
erp_status erp_ctx_reserve(erp_ctx* ctx, int32_t n_pairs, int32_t max_nq, int32_t max_nt,
                           int32_t iters);

/* ---- stage timing (the reference's START_TIME/STOP_TIME, src/debug_print.h:9-13, applied to
   the hot path): HIP events recorded around every kernel on the pipeline's stream. ---- */
typedef enum erp_stage {
    ERP_STAGE_KNN2_FILTER = 0,  /* bf16 split + the one MFMA pass: bounds + provisional candidates */
    ERP_STAGE_KNN2_MERGE = 1,   /* chunk fold + ratio test + compaction */
    ERP_STAGE_BEARINGS = 2,     /* gather + pixel -> bearing */
    ERP_STAGE_JUMP_PREP = 3,    /* glibc jump-ahead polynomials */
    ERP_STAGE_SAMPLER = 4,      /* random_array replay (glibc, backwards, bitmap) */
    ERP_STAGE_EIGEN = 5,        /* 9x9 Jacobi, rank-2 fix, decomposeEssentialMat, Euler */
    ERP_STAGE_VALID_COMPACT = 6,
    ERP_STAGE_CONSENSUS_ROWS = 7,   /* exact order statistics of the surviving rows */
    ERP_STAGE_CONSENSUS_FINAL = 8,
    ERP_STAGE_CONSENSUS_BOUNDS = 9, /* per-row trimmed-mean bounds (one pass over K^2) */
    ERP_STAGE_CONSENSUS_SELECT = 10,
    ERP_STAGE_WINDOWS = 11,         /* per-iteration glibc end windows (jump-ahead) */
    ERP_STAGE_GRAM = 12,            /* A^T A of every sample (fp64) */
    ERP_STAGE_KNN2_CANDIDATES = 13, /* unused since r02 (the two MFMA passes were fused) */
    ERP_STAGE_KNN2_RESCORE = 14,    /* exact flann::L2 distances of the candidates */
    ERP_STAGE_CONSENSUS_REFINE = 15, /* tighter bounds for the survivors (sub-bins) */
    ERP_STAGE_KNN2_EXACT = 16,      /* exact sweep on packed FP32 VALU (ERP_MATCHER_VALU_EXACT) */
    ERP_STAGE_SAMPLER_GRAM = 17,    /* unused since r06 (the fused sampler + Gram kernel, slower, was removed) */
    ERP_STAGE_INLIERS = 18,         /* opt-in per-iteration inlier count (cfg.inlier_thr > 0) */
    ERP_STAGE_COUNT = 19
} erp_stage;
erp_status erp_ctx_set_profiling(erp_ctx* ctx, int32_t enable);
const char* erp_stage_name(int32_t stage);
/* Waits for the recorded events, writes per-stage total milliseconds and launch counts
   (arrays of ERP_STAGE_COUNT), then clears the record. */
erp_status erp_ctx_stage_times(erp_ctx* ctx, double* total_ms, int64_t* launches);

/* ---- matcher (feature_matcher::match_two_image) ---- */
/* How the exact k=2 is computed (both give the same bit-exact matches):
   MFMA_FILTER: bf16 MFMA upper/lower bounds -> candidates -> exact flann::L2 rescoring (default);
   VALU_EXACT:  every distance exactly, LDS-tiled packed FP32 sweep (configs[3]'s scalar path). */
typedef enum erp_matcher_method {
    ERP_MATCHER_MFMA_FILTER = 0,
    ERP_MATCHER_VALU_EXACT = 1
} erp_matcher_method;
erp_status erp_ctx_set_matcher(erp_ctx* ctx, int32_t method);
/* enable != 0: erp_pair_batch_run captures its launch sequence (every kernel and memset of the
   pipeline, ~60 nodes) into a HIP graph the first time it sees a (batch, cfg, outputs, ratio,
   scratch) combination and replays that graph on later calls with the same one -- one launch
   instead of ~60, for the latency of small batches (configs[1]'s single pair).  Pointers are
   baked into the graph: a call with other buffers, or one that grows the context's scratch,
   captures anew (up to 8 graphs per context, least recently used dropped).  Not used while
   stage timing is on or on the NULL stream.  Default off. */
erp_status erp_ctx_set_graphs(erp_ctx* ctx, int32_t enable);
/* Route options of a context (no reference counterpart).  Each selects between code paths whose
   results are identical -- by construction, and checked by the GPU tests that set it -- and
   whose default is the measured fastest; none changes what is computed.  The library reads no
   environment variable: these setters are the only way to steer a route.  Options are part of
   a captured HIP graph's key (erp_ctx_set_graphs).  -1 = automatic where noted.
   ERP_OPT_SMALL_BATCH    consensus route: -1 auto (n_pairs (2 iters)^2 <= 2e9); n >= 0: batches
                          of <= n pairs bin every row in one pass (0 = never)
   ERP_OPT_SAMPLER_LAT    glibc replay blocks: -1 auto (latency blocks for launches of <= 1024
                          waves); 0 throughput blocks, 1 latency step by step, 2 latency with
                          the block's positions first
   ERP_OPT_SAMPLER_SPLIT  split replay: -1 auto (<= 256 workgroups); 0 off; 1 on (where its
                          bitmaps fit the LDS)
   ERP_OPT_GRAM_TILES     32-iteration row tiles per Gram MFMA wave: 0 auto (2 once the launch
                          has >= 512 wide blocks), 1, 2
   ERP_OPT_ZOOM_LEVELS    the survivors' zoom levels 0 (default) .. 2
   ERP_OPT_SMALL_ZOOM     1: the small-batch route keeps the zoom levels (default 0)
   ERP_OPT_LIP2           second pre-pruning stage 1 / 0
   ERP_OPT_LIPG           convexity-augmented pre-pruning: bit 0 first stage (1), bit 1 second
                          stage too (3), 0 off
   ERP_OPT_REFINE_HINT    hinted refine windows 1 / 0
   ERP_OPT_FLAT_REFS      flat-pair route above this % of rows listed (25); 0 off
                          (these four: -1, the default, = automatic: the values in brackets / 1
                          for launches of >= 8 pairs, 0 below -- a few pairs with a large K, as
                          configs[4]'s one 100k-iteration find, run faster without them)
   ERP_OPT_BOUND_RATIO    the matcher's ratio test decided from the bf16 bounds where they
                          suffice 1 (default) / 0
   ERP_OPT_DEBUG_STAGES   debug: bit mask of the stage groups erp_pair_batch_run enqueues (1
                          matcher + gather, 2 jump polynomials + windows, 4 sampler, 8 Gram, 32
                          eigen + estimate, 16 consensus); -1 (default) all.  A skipped group
                          leaves the previous call's scratch in place.
   ERP_OPT_DEBUG_SNAP     debug: 1 keeps a device copy of lb, ub ([P][2 iters] f64 each), the
                          first-stage list counts ([P] i32) and the first-stage Lipschitz
                          references right after the bounds pass, for erp_debug_snapshot */
typedef enum erp_ctx_option {
    ERP_OPT_SMALL_BATCH = 0,
    ERP_OPT_SAMPLER_LAT = 1,
    ERP_OPT_SAMPLER_SPLIT = 2,
    ERP_OPT_GRAM_TILES = 3,
    ERP_OPT_ZOOM_LEVELS = 4,
    ERP_OPT_SMALL_ZOOM = 5,
    ERP_OPT_LIP2 = 6,
    ERP_OPT_LIPG = 7,
    ERP_OPT_REFINE_HINT = 8,
    ERP_OPT_FLAT_REFS = 9,
    ERP_OPT_BOUND_RATIO = 10,
    ERP_OPT_DEBUG_STAGES = 11,
    ERP_OPT_DEBUG_SNAP = 12,
    ERP_OPT_COUNT = 13
} erp_ctx_option;
/* ERP_INVALID_ARG for an unknown option or a value outside its range */
erp_status erp_ctx_set_option(erp_ctx* ctx, int32_t option, int32_t value);
erp_status erp_ctx_get_option(erp_ctx* ctx, int32_t option, int32_t* value);
/* debugging hooks (no reference counterpart):
   erp_debug_set_alloc_pad(N): device buffers allocated from then on get N canary bytes (0xA5)
   past their end (process-wide; 0 = off, the default); erp_debug_check_pads() returns how
   many canaries a kernel overwrote (reported on stderr).
   erp_debug_snapshot (ERP_OPT_DEBUG_SNAP) copies the snapshot to host (returns its size; host
   NULL: size only). */
void erp_debug_set_alloc_pad(size_t bytes);
int erp_debug_check_pads(void);
long long erp_debug_snapshot(erp_ctx* ctx, void* host, size_t bytes);
/* debug counters of a library built with -DERP_LIP_VERIFY=1 (the Lipschitz pruning pass
   re-checks its LDS operands against their global sources): copies 64 words into out64 and
   resets them; returns 0, -1 for a library built without the check, -2 when the copy failed. */
int erp_debug_lip_counters(uint32_t* out64);

/* device pointers; writes up to nq matches in ascending queryIdx order and *d_count. */
erp_status erp_match_knn2_ratio(erp_ctx* ctx, const float* d_query, int32_t nq,
                                const float* d_train, int32_t nt, int32_t dim, float ratio,
                                erp_dmatch* d_out, int32_t* d_count, void* stream);
/* host pointers, synchronous: the drop-in for match_two_image (ratio 0.3f). */
erp_status erp_match_two_image(erp_ctx* ctx, const float* h_desc1, int32_t n1,
                               const float* h_desc2, int32_t n2, int32_t dim,
                               erp_dmatch* h_out, int32_t* h_count);

/* ---- estimator (eight_point::find / eight_point_estimation) ---- */
/* device pointers: m matched keypoint pairs -> result (R, T, diagnostics). */
erp_status erp_eight_point_find_dev(erp_ctx* ctx, int32_t W, int32_t H, const erp_point2f* d_kl,
                                    const erp_point2f* d_kr, int32_t m, const erp_ransac_cfg* cfg,
                                    erp_pair_result* d_result, erp_hypothesis* d_hyps,
                                    void* stream);
/* device pointers: the initial_guess ITERATIONS only (no consensus) -> cfg->iters records.
   cfg->offset positions the glibc stream, so iteration block [a, b) of a larger find() is
   reproduced exactly with iters = b - a and offset = base + a*(m-1): the hypothesis-block
   sharding of configs[4] (src/eight_point.cpp:99-127). */
erp_status erp_eight_point_hypotheses_dev(erp_ctx* ctx, int32_t W, int32_t H,
                                          const erp_point2f* d_kl, const erp_point2f* d_kr,
                                          int32_t m, const erp_ransac_cfg* cfg,
                                          erp_hypothesis* d_hyps, void* stream);
/* device pointers: the trimmed-mean consensus (src/eight_point.cpp:129-149) on K Euler vectors
   d_rvec [K][3] with their translations d_tvec [K][3] (R_vec_arr / T_vec_arr order). */
erp_status erp_consensus_dev(erp_ctx* ctx, const float* d_rvec, const float* d_tvec, int32_t K,
                             double trim_lo, double trim_hi, erp_pair_result* d_result,
                             void* stream);
/* device pointers: valid-list compaction (R1 then R2 per record, src/eight_point.cpp:113-126)
   + the consensus over n_hyps initial_guess records d_hyps (e.g. the rank-ordered all-gather of
   hypothesis blocks; records with both flags 0 push nothing, so blocks may be zero-padded);
   m = match_size (only reported in the result). */
erp_status erp_consensus_hyps_dev(erp_ctx* ctx, int32_t m, const erp_hypothesis* d_hyps,
                                  int32_t n_hyps, const erp_ransac_cfg* cfg,
                                  erp_pair_result* d_result, void* stream);
/* The same consensus with its K^2 bounds pass split over nshards ranks (configs[4] strong
   scaling): on every rank, with the same merged d_hyps, call _shard_dev (valid-list compaction
   + the bounds of rows [K*shard/nshards, K*(shard+1)/nshards) into d_lb / d_ub / d_bsel, each
   2*n_hyps entries of 8 bytes, zero elsewhere), SUM the three arrays over the ranks (e.g. one
   RCCL all_reduce), then call _finish_dev on the SAME context (select, refine, exact means,
   first-argmin).  The result equals erp_consensus_hyps_dev's. */
erp_status erp_consensus_hyps_shard_dev(erp_ctx* ctx, int32_t m, const erp_hypothesis* d_hyps,
                                        int32_t n_hyps, const erp_ransac_cfg* cfg, int32_t shard,
                                        int32_t nshards, double* d_lb, double* d_ub,
                                        int32_t* d_bsel, void* stream);
erp_status erp_consensus_hyps_finish_dev(erp_ctx* ctx, int32_t m, const erp_hypothesis* d_hyps,
                                         int32_t n_hyps, const erp_ransac_cfg* cfg, double* d_lb,
                                         double* d_ub, int32_t* d_bsel, erp_pair_result* d_result,
                                         void* stream);
/* host pointers, synchronous: the drop-in for eight_point::find. */
erp_status erp_eight_point_find(erp_ctx* ctx, int32_t W, int32_t H, const erp_point2f* h_kl,
                                const erp_point2f* h_kr, int32_t m, const erp_ransac_cfg* cfg,
                                float R_out[3], float T_out[3], erp_pair_result* h_result);
/* host pointers, synchronous: initial_guess on m bearing pairs (m x 3 doubles each), i.e. find
   after the pixel->bearing step (src/eight_point.cpp:87-150). */
erp_status erp_initial_guess(erp_ctx* ctx, const double* h_bl, const double* h_br, int32_t m,
                             const erp_ransac_cfg* cfg, float R_out[3], float T_out[3],
                             erp_pair_result* h_result);
/* host pointers, synchronous: one eight_point_estimation on m bearing pairs (m x 3 doubles). */
erp_status erp_eight_point_estimation(erp_ctx* ctx, const double* h_bl, const double* h_br,
                                      int32_t m, erp_hypothesis* h_out);

/* ---- fused batch: match -> gather -> find for every pair ---- */
erp_status erp_pair_batch_run(erp_ctx* ctx, const erp_pair_batch* batch, float ratio,
                              const erp_ransac_cfg* cfg, const erp_batch_outputs* out,
                              void* stream);

/* ---- ERP remaps around the hot path ----
   Images are 8-bit 3-channel (CV_8UC3, BGR) H x W x 3, row-major, device pointers.  Output
   pixels whose inverse-warped source falls outside the image are NOT written (the reference
   leaves them uninitialised): pre-fill the outputs. */
/* spherical_surf::crop_rotated_image(pitch, im) (src/spherical_surf.cpp:16-48): the central
   H/4 rows of the image rotated by pitch degrees about Y -> d_out (H/4) x W x 3. */
erp_status erp_crop_rotated_image_dev(erp_ctx* ctx, const uint8_t* d_im, int32_t W, int32_t H,
                                      float pitch_deg, uint8_t* d_out, void* stream);
/* the four bands of spherical_surf::do_all (src/spherical_surf.cpp:77-93) for n_images images
   (contiguous, each H x W x 3): d_bands [n][4][H/4][W][3] = crop(45), rows [3H/8, 3H/8 + H/4),
   crop(-45), crop(-90). */
erp_status erp_spherical_bands_dev(erp_ctx* ctx, const uint8_t* d_ims, int32_t n_images,
                                   int32_t W, int32_t H, uint8_t* d_bands, void* stream);
/* spherical_surf::rotate_keypoint(pitch, key, width, height) (src/spherical_surf.cpp:50-63),
   in place on n keypoints (pt.x, pt.y). */
erp_status erp_rotate_keypoints_dev(erp_ctx* ctx, erp_point2f* d_kp, int32_t n, float pitch_deg,
                                    int32_t W, int32_t H, void* stream);
/* do_all's keypoint un-rotation (src/spherical_surf.cpp:120-133) on the band keypoints
   concatenated in band order n0, n1, n2, n3 (counts[4]), in place: the result is the
   left_key_tmp / right_key_tmp index space of the matcher (:136-144). */
erp_status erp_unrotate_band_keypoints_dev(erp_ctx* ctx, erp_point2f* d_kp,
                                           const int32_t counts[4], int32_t W, int32_t H,
                                           void* stream);
/* erp_rotation::rotate_image(im, rot_mat) (src/erp_rotation.cpp:94-122). */
erp_status erp_rotate_image_dev(erp_ctx* ctx, const uint8_t* d_im, int32_t W, int32_t H,
                                const double rot_mat[9], uint8_t* d_out, void* stream);
/* rectify(im_left, im_right, R_vec, T_vec) (src/automatic.cpp:66-79): both rotate_image calls
   in one launch. */
erp_status erp_rectify_dev(erp_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int32_t W,
                           int32_t H, const double rot_vec[3], const double t_vec[3],
                           uint8_t* d_left_out, uint8_t* d_right_out, void* stream);
/* the vertical view of src/automatic.cpp:148-151: rotate_image by eular2rot(RAD(89.999), 0, 0)
   .inv(), then cv::rotate(ROTATE_90_CLOCKWISE), fused -> d_out W x H x 3 (W rows). */
erp_status erp_vertical_rotate_dev(erp_ctx* ctx, const uint8_t* d_im, int32_t W, int32_t H,
                                   uint8_t* d_out, void* stream);
/* ---- SURF: feature_matcher::detect_key_point + comput_descriptor
   (src/feature_matcher.cpp:26-40) with xfeatures2d::SURF::create() defaults ---- */
typedef struct erp_keypoint {   /* cv::KeyPoint layout */
    float x, y;                 /* pt */
    float size, angle, response;
    int32_t octave, class_id;
} erp_keypoint;
typedef struct erp_surf_params {
    double hessian_threshold;   /* 100 */
    int32_t n_octaves;          /* 4 */
    int32_t n_octave_layers;    /* 3 */
    int32_t extended;           /* 0 (64-D; 1 is not supported) */
    int32_t upright;            /* 0 (1 is not supported) */
} erp_surf_params;
void erp_surf_params_default(erp_surf_params* p);
/* n_images images of H x W (channels 1 = gray, 3 = BGR), contiguous, device pointers ->
   per image up to max_kp keypoints [n][max_kp] in OpenCV's KeypointGreater order (descending
   response) and their unit 64-D descriptors [n][max_kp][64]; d_count[n] = keypoints found, or
   -(needed) when max_kp was too small (rerun larger).  Enqueued on `stream`; synchronises
   it once inside (the detected counts size the descriptor pass). */
erp_status erp_surf_detect_compute_dev(erp_ctx* ctx, const uint8_t* d_images, int32_t n_images,
                                       int32_t W, int32_t H, int32_t channels,
                                       const erp_surf_params* params, int32_t max_kp,
                                       erp_keypoint* d_kp, float* d_desc, int32_t* d_count,
                                       void* stream);

/* ---- visual outputs, device images ---- */
/* epipolar_tool (src/epipolar_tool.hpp / .cpp:7-71, constructor + draw_epipole :74-128): n_key
   (<= 7, the reference's color_set) of the m matched pairs (host keypoints, ERP pixels of an
   im_width x im_height image) chosen as the first n_key of std::random_shuffle(iota(m)) on the
   glibc rand() stream at (seed, offset) (the process-global rand() state: 1 / 0 in a fresh
   process); on an out_width x out_height CV_8UC3 canvas d_out (written whole) the pixels p with
   |l^T E p| < 0.002 for a chosen left bearing l get that key's colour and 11 x 11 dots mark the
   chosen right keypoints (resized).  E: row-major 3x3 (test_E_mat).  The reference's OpenMP
   loop races on overlapping writes; here the sequential order of its loop decides: a pixel
   shows the last key whose dot covers it, else the last key whose curve passes, else 0 (the
   corner pixel (H-1, W-1) interleaves curve k and dot k in key order).  A dot pixel lands at
   its linear address like the unchecked Mat::at (past the left/right edge it wraps into the
   neighbouring row); writes that would leave the canvas are dropped.
   h_random_idx (may be NULL): the n_key chosen match indices. */
erp_status erp_epipolar_draw_dev(erp_ctx* ctx, const erp_point2f* h_key_left,
                                 const erp_point2f* h_key_right, int32_t m, int32_t im_width,
                                 int32_t im_height, int32_t out_width, int32_t out_height,
                                 int32_t n_key, uint32_t seed, uint64_t offset, const double E[9],
                                 uint8_t* d_out, int32_t* h_random_idx, void* stream);
/* epipolar_tool's constructor choice (src/epipolar_tool.cpp:13-16), host only: the first n of
   std::random_shuffle(iota(m)) on the glibc rand() stream at (seed, offset) into h_idx (n <= m;
   the shuffle consumes m - 1 rand() calls).  The same indices erp_epipolar_draw_dev draws. */
erp_status erp_random_shuffle_prefix(uint32_t seed, uint64_t offset, int32_t m, int32_t n,
                                     int32_t* h_idx);
/* feature_matcher::draw_match (src/feature_matcher.cpp:61-86): d_out (W x H CV_8UC3) = the
   grey images of d_left / d_right (cvtColor CV_RGB2GRAY, as the reference calls it on its BGR
   images) in channels 0 / 1, 0 in channel 2, with a line of thickness 5 from key_left[i] to
   key_right[i] (device keypoints, rounded like cv::Point(Point2f)) in the colour
   HSV(i 180 / m, 180, 150) -> BGR, later matches on top.  Lines are the pixels within 2.5 of
   the segment (cv::line's thickness-5 rasteriser is not restated: parity with OpenCV is
   unpinned).  m <= 65535; the three image pointers are 4-byte aligned. */
erp_status erp_draw_match_dev(erp_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right,
                              int32_t W, int32_t H, const erp_point2f* d_key_left,
                              const erp_point2f* d_key_right, int32_t m, uint8_t* d_out,
                              void* stream);

/* host 3x3 geometry (row-major doubles) */
void erp_eular2rot(const double theta[3], double R[9]);         /* erp_rotation.cpp:14-40 */
void erp_rot2eular(const double R[9], double e[3]);             /* erp_rotation.cpp:43-63 */
void erp_rot_from_vec(const double v1[3], const double v2[3], double R[9]); /* automatic.cpp:50-64 */
int32_t erp_inv3(const double m[9], double out[9]);            /* cv::Mat::inv() on 3x3 */
/* the two matrices rotate_pixel applies in rectify's rotate_image calls */
erp_status erp_rectify_matrices(const double rot_vec[3], const double t_vec[3], double m_left[9],
                                double m_right[9]);

#ifdef __cplusplus
}
#endif
#endif /* ERP_MATCH_H */
