/*
 * erp_oracle.h -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity CHECKER for the MI355X implementation in
 * erp_match_eightpoint_test_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library never links it and never falls back
 * to it.
 *
 * It restates, in plain C99 (built with -ffp-contract=off, no fast-math):
 *   - feature_matcher::match_two_image      /root/reference/src/feature_matcher.cpp:42-59
 *     (FLANN kNN k=2 replaced by EXACT brute-force k=2 in the flann::L2<float> accumulation
 *      order; ratio test d0 < 0.3f*d1; output in ascending queryIdx order)
 *   - spherical_surf concat+gather          /root/reference/src/spherical_surf.cpp:135-162
 *   - eight_point::find                     /root/reference/src/eight_point.cpp:152-192
 *   - eight_point::initial_guess            /root/reference/src/eight_point.cpp:87-150
 *   - eight_point::eight_point_estimation   /root/reference/src/eight_point.cpp:16-85
 *   - random_array (iota + random_shuffle)  /root/reference/src/eight_point.hpp:30-59
 *   - erp_rotation::eular2rot / rot2eular   /root/reference/src/erp_rotation.cpp:14-63
 *   - erp_rotation::rotate_pixel / rotate_image  /root/reference/src/erp_rotation.cpp:66-122
 *   - spherical_surf::crop_rotated_image / rotate_keypoint + do_all's band steps
 *                                           /root/reference/src/spherical_surf.cpp:16-63,77-133
 *   - rot_from_vec / rectify / vertical view /root/reference/src/automatic.cpp:50-79,148-152
 * plus the third-party arithmetic those call, restated from the published algorithms:
 *   - glibc rand() (TYPE_3 additive feedback generator, srand never called => seed 1)
 *   - libstdc++ (GCC 11) std::random_shuffle
 *   - OpenCV 3.4 cv::SVDecomp (JacobiSVDImpl_, flags=0, thin/full selection of _SVDcompute)
 *   - OpenCV 3.4 cv::decomposeEssentialMat, cv::determinant (3x3), small-matrix gemm,
 *     Mat::inv() on 3x3 doubles (adjugate / determinant), cv::rotate(ROTATE_90_CLOCKWISE)
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   - glibc rand() and std::random_shuffle: PINNED against the real libc / libstdc++ of this
 *     container (tests/golden/gen_glibc_shuffle.cpp -> tests/golden/glibc_shuffle.json).
 *   - OpenCV SVD / decomposeEssentialMat / FLANN: OpenCV is not vendored in the reference and
 *     not installed here, so these are restated from the published algorithm and cross-checked
 *     against LAPACK (numpy) up to sign plus the reference's own known-answer experiments
 *     (one_image_test / two_synthesis_image_test: mean |dEuler| < 1 deg).  OpenCV-internal
 *     rounding order / sign conventions are therefore "parity unpinned".
 */
#ifndef ERP_ORACLE_H
#define ERP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cv::DMatch layout (queryIdx, trainIdx, imgIdx, distance) */
typedef struct {
    int32_t queryIdx;
    int32_t trainIdx;
    int32_t imgIdx;
    float distance;
} erpo_dmatch;

/* glibc random_r TYPE_3 state, restated. */
typedef struct {
    uint32_t r[34];  /* ring of the last 34 words */
    uint32_t pos;    /* number of words generated so far (index of next word) */
} erpo_glibc;

void erpo_glibc_seed(erpo_glibc* g, uint32_t seed);
int32_t erpo_glibc_rand(erpo_glibc* g);                /* == rand() after srand(seed) */
void erpo_glibc_discard(erpo_glibc* g, uint64_t n);
/* the 31-word window (r[n-31..n-1] of the additive recurrence) that precedes draw n=pos */
void erpo_glibc_window(const erpo_glibc* g, uint32_t out[31]);

/* Philox4x32-10 block; iteration h's s-subset of [0, m) in ascending order (erp_oracle.c) */
void erpo_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void erpo_philox_sample(int32_t m, int32_t s, uint64_t h, uint32_t seed, int32_t* out);

/* libstdc++ std::random_shuffle over iota(n) using g (random_array::rand_idx_generate) */
void erpo_random_array(int32_t* a, int32_t n, erpo_glibc* g);

/* ---------------- matcher ---------------- */
/* flann::L2<float> distance in its accumulation order (squared) */
float erpo_l2sq(const float* a, const float* b, int32_t dim);
/* Exact k=2 + ratio test.  Optional per-query outputs (may be NULL): best index, d0^2, d1^2.
 * Returns number of matches written to out (capacity nq), or -1 on invalid arguments,
 * -2 when nt < 2 (reference: knn_matches[i][1] out of range = UB). */
int32_t erpo_match_two_image(const float* q, int32_t nq, const float* t, int32_t nt, int32_t dim,
                             float ratio, erpo_dmatch* out, int32_t* best, float* d0sq, float* d1sq,
                             int32_t nthreads);

/* ---------------- geometry ---------------- */
void erpo_eular2rot(const double e[3], double R[9]);
void erpo_rot2eular(const double R[9], double e[3]);
/* eight_point::find pixel -> bearing (src/eight_point.cpp:163-186) */
void erpo_pixel_to_bearing(int32_t W, int32_t H, float px, float py, double b[3]);

/* ---- ERP remaps.  Images: H x W x 3 bytes.  Unwritten pixels (source
   outside the image) keep the output's prior content, as in the reference. ---- */
void erpo_rotate_pixel(int32_t row, int32_t col, const double m[9], int32_t W, int32_t H,
                       int32_t out[2]);
int32_t erpo_inv3(const double m[9], double out[9]);
void erpo_rotate_pixel_prefix(const int32_t* rows, const int32_t* cols, int32_t n, const double m[9],
                              int32_t W, int32_t H, double* out);
void erpo_rot_from_vec(const double v1[3], const double v2[3], double R[9]);
void erpo_crop_rotated_image(const uint8_t* im, int32_t W, int32_t H, float pitch_deg,
                             uint8_t* out);
void erpo_rotate_keypoint(float* kp_xy, int32_t n, float pitch_deg, int32_t W, int32_t H);
void erpo_unrotate_band_keypoints(float* kp_xy, const int32_t counts[4], int32_t W, int32_t H);
int32_t erpo_rotate_image(const uint8_t* im, int32_t W, int32_t H, const double rot_mat[9],
                          uint8_t* out);
int32_t erpo_rectify(const uint8_t* left, const uint8_t* right, int32_t W, int32_t H,
                     const double rot_vec[3], const double t_vec[3], uint8_t* left_out,
                     uint8_t* right_out);
int32_t erpo_vertical_rotate(const uint8_t* im, int32_t W, int32_t H, uint8_t* out);

/* ---- SURF (erp_surf.c): xfeatures2d::SURF::create() defaults as
   called by src/feature_matcher.cpp:13-15,26-40.  Parity with OpenCV UNPINNED. ---- */
typedef struct erpo_keypoint {  /* cv::KeyPoint layout */
    float x, y, size, angle, response;
    int32_t octave, class_id;
} erpo_keypoint;
typedef struct erpo_surf_params {
    double hessian_threshold;  /* 100 */
    int32_t n_octaves;         /* 4 */
    int32_t n_octave_layers;   /* 3 */
} erpo_surf_params;
void erpo_gray_bgr(const uint8_t* bgr, int32_t W, int32_t H, uint8_t* gray);
void erpo_integral(const uint8_t* img, int32_t W, int32_t H, int32_t* sum);
float erpo_fast_atan2(float y, float x);
int32_t erpo_surf_layer_size(int octave, int layer);
int32_t erpo_surf_detect(const int32_t* sum, int32_t W, int32_t H, const erpo_surf_params* prm,
                         erpo_keypoint* kps, int32_t max_kp);
void erpo_resize_area(const uint8_t* src, int ss, uint8_t* dst, int ds);
void erpo_surf_describe(const uint8_t* img, const int32_t* sum, int32_t W, int32_t H,
                        erpo_keypoint* kp, float* vec);
int32_t erpo_surf(const uint8_t* img, int32_t W, int32_t H, int32_t channels,
                  const erpo_surf_params* prm, erpo_keypoint* kps, float* desc, int32_t max_kp);

/* OpenCV 3.4 SVDecomp(src m x n, flags=0) restated.  w: min(m,n); u: m x min(m,n) row-major;
 * vt: min(m,n) x n row-major.  Returns 0 on success. */
int erpo_svdecomp(const double* src, int32_t m, int32_t n, double* w, double* u, double* vt);

/* ---------------- estimator ---------------- */
typedef struct {
    float R1[3], R2[3], T[3];
    int32_t R1_valid, R2_valid;
    int32_t inliers;    /* erpo_inlier_count of E_corr at cfg->inlier_thr (0 when off) */
    double E[9];        /* e = last row of vt, reshaped row-major */
    double E_corr[9];   /* u * diag(w0,w1,0) * vt */
} erpo_hyp;

/* eight_point_estimation on `m` bearing pairs (bl,br: m x 3 row-major). Returns 0, or
 * -2 when m < 1. */
int erpo_eight_point_estimation(const double* bl, const double* br, int32_t m, erpo_hyp* h);

typedef struct {
    int32_t iters;        /* reference: 80 (src/eight_point.cpp:99) */
    double sample_frac;   /* 0.25 (:102) */
    double trim_lo;       /* 0.2 (:143) */
    double trim_hi;       /* 0.8 (:143) */
    double valid_abs;     /* 1.57 (:76,81) */
    uint32_t seed;        /* 1: srand never called */
    uint64_t offset;      /* rand() calls consumed before initial_guess (e.g. by FLANN);
                             sampler 1: the first iteration's counter */
    int32_t sampler;      /* 0: glibc replay (the reference), 1: Philox4x32-10 + Floyd */
    double inlier_thr;    /* > 0: every iteration's erpo_inlier_count (no reference counterpart) */
} erpo_cfg;

/* E_mat_correct (src/eight_point.cpp:45-50) of a solved 9-vector e: SVDecomp of the 3x3,
 * w_f[2] = 0, u_f * diag(w_f) * vt_f */
void erpo_rank2(const double e[9], double Ec[9]);
/* The opt-in inlier count (erp_ransac_cfg.inlier_thr; no reference counterpart): matches i
 * with |res_i| < thr, res_i = Ec_0 u_0 then fma(Ec_k, u_k, res) for k = 1..8, u_k = l_i*r_j
 * (k = 3i + j) in fp64.  *n_band (optional): matches with ||res_i| - thr| <= band (the ones a
 * differently rounded Ec could flip). */
int32_t erpo_inlier_count(const double* bl, const double* br, int32_t m, const double Ec[9],
                          double thr, double band, int32_t* n_band);

typedef struct {
    int32_t K;            /* valid R vectors */
    int32_t min_idx;      /* consensus winner in R_vec_arr order */
    int32_t sample_n;
    int32_t status;       /* 0 ok, -2 too few points, -3 no valid hypothesis */
    double min_dist;      /* trimmed mean of the winner */
} erpo_diag;

/* consensus on K float Euler vectors (src/eight_point.cpp:129-149).  dist (K) optional. */
int erpo_consensus(const float* rvec, int32_t K, double trim_lo, double trim_hi, int32_t* min_idx,
                   double* dist);

/* initial_guess on bearings.  hyp (cfg->iters entries), samples (iters*sample_n), rvec/tvec
 * (2*iters*3), dist (2*iters) are optional outputs. */
int erpo_initial_guess(const double* bl, const double* br, int32_t m, const erpo_cfg* cfg,
                       float R_out[3], float T_out[3], erpo_diag* diag, erpo_hyp* hyp,
                       int32_t* samples, float* rvec, float* tvec, double* dist);

/* find on pixel keypoints (m x 2 float, x then y).  Optional outputs as initial_guess. */
int erpo_find(int32_t W, int32_t H, const float* kl, const float* kr, int32_t m, const erpo_cfg* cfg,
              float R_out[3], float T_out[3], erpo_diag* diag, erpo_hyp* hyp, int32_t* samples,
              float* rvec, float* tvec, double* dist);

#ifdef __cplusplus
}
#endif
/* ---------------- visual outputs (erp_viz.c) ---------------- */
int32_t erpo_epipolar_draw(const float* key_left, const float* key_right, int32_t m,
                           int32_t im_width, int32_t im_height, int32_t out_w, int32_t out_h,
                           int32_t n_key, uint32_t seed, uint64_t offset, const double E[9],
                           uint8_t* out, int32_t* random_idx, double* min_margin);
double erpo_epipolar_value(const double l[3], const double E[9], int32_t i, int32_t j, int32_t out_w,
                           int32_t out_h);
void erpo_hsv2bgr(int h, int s, int v, uint8_t bgr[3]);
void erpo_draw_match(const uint8_t* left, const uint8_t* right, int32_t W, int32_t H,
                     const float* key_left, const float* key_right, int32_t m, uint8_t* out);

#endif
