/*
 * erp_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY
 * (the parity checker; see erp_oracle.h for scope, citations and pinning status).
 *
 * Build: oracle/Makefile  (gcc -O2 -std=c99 -ffp-contract=off -fno-fast-math -fopenmp)
 * -ffp-contract=off matters: the reference is x86-64 SSE code without FMA contraction, and
 * the flann::L2 order / OpenCV Jacobi rotations must round exactly as written.
 */
#define _POSIX_C_SOURCE 200809L
#include "erp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ======================================================================================
 * glibc rand() restated (stdlib/random_r.c, TYPE_3: degree 31, separation 3).
 * srand(seed): r[0]=seed; r[i]=16807*r[i-1] % 2147483647 (Schrage) for i<31;
 * r[i]=r[i-31] for 31<=i<34; then r[i]=r[i-3]+r[i-31] (mod 2^32); the first 310 outputs
 * are discarded; rand() returns r[i]>>1.  The reference never calls srand, so seed = 1
 * (src/eight_point.hpp:57 -> std::random_shuffle -> rand()).
 * ==================================================================================== */
void erpo_glibc_seed(erpo_glibc* g, uint32_t seed) {
    int32_t r[34];
    int i;
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (i = 1; i < 31; i++) {
        const long hi = r[i - 1] / 127773;
        const long lo = r[i - 1] % 127773;
        long word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    for (i = 31; i < 34; i++) r[i] = r[i - 31];
    for (i = 0; i < 34; i++) g->r[i] = (uint32_t)r[i];
    g->pos = 0; /* ring slot of absolute index 34 */
    for (i = 34; i < 344; i++) {
        const uint32_t s = g->pos;
        g->r[s] = g->r[(s + 34 - 3) % 34] + g->r[(s + 34 - 31) % 34];
        g->pos = (s + 1) % 34;
    }
}

static inline uint32_t glibc_next_word(erpo_glibc* g) {
    const uint32_t s = g->pos;
    const uint32_t v = g->r[(s + 34 - 3) % 34] + g->r[(s + 34 - 31) % 34];
    g->r[s] = v;
    g->pos = (s + 1) % 34;
    return v;
}

int32_t erpo_glibc_rand(erpo_glibc* g) { return (int32_t)(glibc_next_word(g) >> 1); }

void erpo_glibc_discard(erpo_glibc* g, uint64_t n) {
    for (uint64_t k = 0; k < n; k++) (void)glibc_next_word(g);
}

void erpo_glibc_window(const erpo_glibc* g, uint32_t out[31]) {
    for (int j = 0; j < 31; j++) out[j] = g->r[(g->pos + 34 - 31 + j) % 34];
}

/* libstdc++ (GCC 11) std::random_shuffle(first, last):
 *   for (i = first + 1; i != last; ++i) { j = first + rand() % ((i - first) + 1);
 *                                          if (i != j) iter_swap(i, j); }
 * applied to iota(0..n-1): random_array::rand_idx_generate (src/eight_point.hpp:54-58). */
void erpo_random_array(int32_t* a, int32_t n, erpo_glibc* g) {
    for (int32_t i = 0; i < n; i++) a[i] = i;
    for (int32_t i = 1; i < n; i++) {
        const int32_t j = (int32_t)((long)erpo_glibc_rand(g) % ((long)i + 1));
        if (i != j) {
            const int32_t t = a[i];
            a[i] = a[j];
            a[j] = t;
        }
    }
}

/* ======================================================================================
 * Counter-based sampler (ERP_SAMPLER_PHILOX; SURVEY.md section 8b's `sampler = PHILOX`).  No
 * reference counterpart: the reference only has the glibc shuffle above.  Philox4x32-10 as
 * published (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3",
 * SC'11; Random123's constants), checked against Random123's known-answer vectors
 * (tests/test_oracle.py).  Iteration h's s-subset of [0, m): Floyd's algorithm, draw k
 * (k = 0 .. s-1, j = m - s + k) t = floor(u_k (j + 1) / 2^32) with
 *   u_k = philox4x32_10(ctr = (lo32(h), hi32(h), k / 4, 0), key = (seed, 0x243F6A88))[k mod 4],
 * t joins the set unless it is already there, then j does.  (The multiply-shift range map is
 * biased by < (j + 1) / 2^32 <= 2^-16 per draw; h = cfg->offset + iteration.)
 * ==================================================================================== */
void erpo_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

void erpo_philox_sample(int32_t m, int32_t s, uint64_t h, uint32_t seed, int32_t* out) {
    uint8_t* in = (uint8_t*)calloc((size_t)(m > 0 ? m : 1), 1);
    const uint32_t key[2] = {seed, 0x243F6A88u};
    uint32_t u[4] = {0, 0, 0, 0};
    for (int32_t k = 0; k < s; k++) {
        if ((k & 3) == 0) {
            const uint32_t ctr[4] = {(uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(k >> 2), 0u};
            erpo_philox4x32(ctr, key, u);
        }
        const int32_t j = m - s + k;
        const int32_t t = (int32_t)(((uint64_t)u[k & 3] * (uint64_t)(j + 1)) >> 32);
        if (in[t]) in[j] = 1; else in[t] = 1;
    }
    int32_t n = 0;
    for (int32_t i = 0; i < m; i++)
        if (in[i]) out[n++] = i;
    free(in);
}

/* ======================================================================================
 * Matcher: feature_matcher::match_two_image (src/feature_matcher.cpp:42-59).
 * FlannBasedMatcher::knnMatch(k=2) is approximate (randomized KD-trees); the oracle is its
 * exact limit: brute force in flann::L2<float>::operator() accumulation order (groups of 4,
 * result += d0*d0 + d1*d1 + d2*d2 + d3*d3), DMatch.distance = sqrtf(squared) as in
 * FlannBasedMatcher::convertToDMatches, ratio test d0 < 0.3f * d1 (:47,52).
 * Ties on the squared distance keep the lowest train index first.
 * ==================================================================================== */
float erpo_l2sq(const float* a, const float* b, int32_t dim) {
    float result = 0.0f;
    int32_t k = 0;
    for (; k + 3 < dim; k += 4) {
        const float d0 = a[k] - b[k];
        const float d1 = a[k + 1] - b[k + 1];
        const float d2 = a[k + 2] - b[k + 2];
        const float d3 = a[k + 3] - b[k + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    for (; k < dim; k++) {
        const float d0 = a[k] - b[k];
        result += d0 * d0;
    }
    return result;
}

int32_t erpo_match_two_image(const float* q, int32_t nq, const float* t, int32_t nt, int32_t dim,
                             float ratio, erpo_dmatch* out, int32_t* best, float* d0sq, float* d1sq,
                             int32_t nthreads) {
    if (nq < 0 || nt < 0 || dim <= 0) return -1;
    if (nq == 0) return 0;
    if (nt < 2) return -2;
    int32_t* bj = (int32_t*)malloc(sizeof(int32_t) * (size_t)nq);
    float* b0 = (float*)malloc(sizeof(float) * (size_t)nq);
    float* b1 = (float*)malloc(sizeof(float) * (size_t)nq);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int32_t i = 0; i < nq; i++) {
        float s0 = INFINITY, s1 = INFINITY;
        int32_t j0 = -1;
        const float* qi = q + (size_t)i * dim;
        for (int32_t j = 0; j < nt; j++) {
            const float d = erpo_l2sq(qi, t + (size_t)j * dim, dim);
            if (d < s0) {
                s1 = s0;
                s0 = d;
                j0 = j;
            } else if (d < s1) {
                s1 = d;
            }
        }
        bj[i] = j0;
        b0[i] = s0;
        b1[i] = s1;
    }
    (void)nthreads;
    int32_t m = 0;
    for (int32_t i = 0; i < nq; i++) {
        const float d0 = sqrtf(b0[i]);
        const float d1 = sqrtf(b1[i]);
        if (best) best[i] = bj[i];
        if (d0sq) d0sq[i] = b0[i];
        if (d1sq) d1sq[i] = b1[i];
        if (d0 < ratio * d1) {
            if (out) {
                out[m].queryIdx = i;
                out[m].trainIdx = bj[i];
                out[m].imgIdx = 0;
                out[m].distance = d0;
            }
            m++;
        }
    }
    free(bj);
    free(b0);
    free(b1);
    return m;
}

/* ======================================================================================
 * Geometry: erp_rotation (src/erp_rotation.cpp:14-63) and find's pixel->bearing
 * (src/eight_point.cpp:163-186, MPEG OMAF axes).
 * ==================================================================================== */
/* cv::gemm small-matrix path (3x3 double): d[i][j] = a[i][0]b[0][j] + a[i][1]b[1][j] + a[i][2]b[2][j] */
static void gemm33(const double* a, const double* b, double* d) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            t[i * 3 + j] = a[i * 3 + 0] * b[0 * 3 + j] + a[i * 3 + 1] * b[1 * 3 + j] + a[i * 3 + 2] * b[2 * 3 + j];
    memcpy(d, t, sizeof(t));
}

void erpo_eular2rot(const double e[3], double R[9]) {
    const double Rx[9] = {1, 0, 0, 0, cos(e[0]), -sin(e[0]), 0, sin(e[0]), cos(e[0])};
    const double Ry[9] = {cos(e[1]), 0, sin(e[1]), 0, 1, 0, -sin(e[1]), 0, cos(e[1])};
    const double Rz[9] = {cos(e[2]), -sin(e[2]), 0, sin(e[2]), cos(e[2]), 0, 0, 0, 1};
    double t[9];
    gemm33(Rx, Ry, t);
    gemm33(t, Rz, R);
}

void erpo_rot2eular(const double R[9], double e[3]) {
    const double sy = sqrt(R[8] * R[8] + R[5] * R[5]);
    const int singular = sy < 1e-6;
    if (!singular) {
        e[0] = atan2(-R[5], R[8]);
        e[1] = atan2(R[2], sy);
        e[2] = atan2(-R[1], R[0]);
    } else {
        e[0] = 0;
        e[1] = atan2(R[2], sy);
        e[2] = atan2(-R[1], R[0]);
    }
}

void erpo_pixel_to_bearing(int32_t W, int32_t H, float px, float py, double b[3]) {
    /* lon = 2*M_PI*(pt.x / im_width): float/int division in float, then double */
    const float fx = px / (float)W;
    const float fy = py / (float)H;
    const double lon = 2 * M_PI * (double)fx;
    const double lat = M_PI * (double)fy;
    b[0] = -sin(lat) * cos(lon);
    b[1] = sin(lat) * sin(lon);
    b[2] = cos(lat);
}

/* ======================================================================================
 * OpenCV 3.4 SVD (modules/core/src/lapack.cpp), restated:
 *   _SVDcompute(src m x n, flags=0): if m < n work on src itself (at = true) else on src^T;
 *   JacobiSVDImpl_<double>(At, W, Vt, m', n', n1 = n', DBL_MIN, 10*DBL_EPSILON):
 *   one-sided cyclic Jacobi on the n' rows of At (length m'), max_iter = max(m', 30);
 *   singular values sorted descending (rows of At and Vt swapped along);
 *   rows of At normalized by multiplying with 1/sd; zero singular values get a random
 *   vector from cv::RNG(0x12345678) orthogonalized twice against previous rows.
 *   Output: at == false: u = At^T, vt = Vt;  at == true: u = Vt^T, vt = At.
 * The OpenCV SIMD (VBLAS) inner loops may sum in a different order; the restatement uses
 * the scalar template order (rounding-level difference, unpinned).
 * ==================================================================================== */
typedef struct {
    uint64_t state;
} cv_rng;

static uint32_t cv_rng_next(cv_rng* r) {
    r->state = (uint64_t)(uint32_t)r->state * 4164903690U + (uint32_t)(r->state >> 32);
    return (uint32_t)r->state;
}

static void jacobi_svd_impl(double* At, int astep, double* W_out, double* Vt, int vstep, int m, int n,
                            int n1, double minval, double eps) {
    double* W = (double*)malloc(sizeof(double) * (size_t)n);
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    double c, s, sd;

    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) {
            const double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sd;
        if (Vt) {
            for (k = 0; k < n; k++) Vt[i * vstep + k] = 0;
            Vt[i * vstep + i] = 1;
        }
    }

    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                double *Ai = At + i * astep, *Aj = At + j * astep;
                double a = W[i], p = 0, b = W[j];
                for (k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = hypot(p, beta);
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (k = 0; k < m; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (Vt) {
                    double *Vi = Vt + i * vstep, *Vj = Vt + j * vstep;
                    for (k = 0; k < n; k++) {
                        const double t0 = c * Vi[k] + s * Vj[k];
                        const double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }

    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) {
            const double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }

    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            if (Vt) {
                for (k = 0; k < m; k++) {
                    t = At[i * astep + k];
                    At[i * astep + k] = At[j * astep + k];
                    At[j * astep + k] = t;
                }
                for (k = 0; k < n; k++) {
                    t = Vt[i * vstep + k];
                    Vt[i * vstep + k] = Vt[j * vstep + k];
                    Vt[j * vstep + k] = t;
                }
            }
        }
    }

    for (i = 0; i < n; i++) W_out[i] = W[i];

    if (!Vt) {
        free(W);
        return;
    }

    cv_rng rng = {0x12345678};
    for (i = 0; i < n1; i++) {
        sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (k = 0; k < m; k++) {
                const double val = (cv_rng_next(&rng) & 256) != 0 ? val0 : -val0;
                At[i * astep + k] = val;
            }
            for (iter = 0; iter < 2; iter++) {
                for (j = 0; j < i; j++) {
                    sd = 0;
                    for (k = 0; k < m; k++) sd += At[i * astep + k] * At[j * astep + k];
                    double asum = 0;
                    for (k = 0; k < m; k++) {
                        const double t = At[i * astep + k] - sd * At[j * astep + k];
                        At[i * astep + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (k = 0; k < m; k++) At[i * astep + k] *= asum;
                }
            }
            sd = 0;
            for (k = 0; k < m; k++) {
                const double t = At[i * astep + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        s = sd > minval ? 1 / sd : 0.;
        for (k = 0; k < m; k++) At[i * astep + k] *= s;
    }
    free(W);
}

int erpo_svdecomp(const double* src, int32_t m, int32_t n, double* w, double* u, double* vt) {
    if (m <= 0 || n <= 0) return -1;
    int at = 0;
    int mm = m, nn = n;
    if (m < n) {
        mm = n;
        nn = m;
        at = 1;
    }
    /* temp_a: nn rows of length mm */
    double* A = (double*)malloc(sizeof(double) * (size_t)nn * mm);
    double* V = (double*)malloc(sizeof(double) * (size_t)nn * nn);
    double* W = (double*)malloc(sizeof(double) * (size_t)nn);
    if (!at) {
        for (int i = 0; i < nn; i++)
            for (int k = 0; k < mm; k++) A[i * mm + k] = src[(size_t)k * n + i]; /* transpose */
    } else {
        memcpy(A, src, sizeof(double) * (size_t)nn * mm);
    }
    jacobi_svd_impl(A, mm, W, V, nn, mm, nn, nn, DBL_MIN, DBL_EPSILON * 10);
    if (w) memcpy(w, W, sizeof(double) * (size_t)nn);
    if (!at) {
        /* u = transpose(temp_u): m x nn ; vt = temp_v: nn x nn (= n x n) */
        if (u)
            for (int r = 0; r < mm; r++)
                for (int c = 0; c < nn; c++) u[r * nn + c] = A[c * mm + r];
        if (vt) memcpy(vt, V, sizeof(double) * (size_t)nn * nn);
    } else {
        /* u = transpose(temp_v): nn x nn (= m x m); vt = temp_u: nn x mm (= m x n) */
        if (u)
            for (int r = 0; r < nn; r++)
                for (int c = 0; c < nn; c++) u[r * nn + c] = V[c * nn + r];
        if (vt) memcpy(vt, A, sizeof(double) * (size_t)nn * mm);
    }
    free(A);
    free(V);
    free(W);
    return 0;
}

/* cv::determinant for 3x3 double (modules/core/src/lapack.cpp, explicit formula) */
static double det33(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

/* cv::decomposeEssentialMat (modules/calib3d/src/five-point.cpp), restated. */
static void decompose_essential(const double* E, double* R1, double* R2, double* t) {
    double D[3], U[9], Vt[9];
    erpo_svdecomp(E, 3, 3, D, U, Vt);
    if (det33(U) < 0)
        for (int k = 0; k < 9; k++) U[k] *= -1.;
    if (det33(Vt) < 0)
        for (int k = 0; k < 9; k++) Vt[k] *= -1.;
    const double Wm[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    const double Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double tmp[9];
    gemm33(U, Wm, tmp);
    gemm33(tmp, Vt, R1);
    gemm33(U, Wt, tmp);
    gemm33(tmp, Vt, R2);
    t[0] = U[2] * 1.0;
    t[1] = U[5] * 1.0;
    t[2] = U[8] * 1.0;
}

/* eight_point::max_vec (src/eight_point.cpp:6-14) */
static double max_vec(const float* v) {
    if ((v[0] > v[1]) && (v[0] > v[2])) return v[0];
    else if (v[1] > v[2])
        return v[1];
    else
        return v[2];
}

void erpo_rank2(const double e[9], double Ec[9]) {
    double wf[3], uf[9], vtf[9];
    erpo_svdecomp(e, 3, 3, wf, uf, vtf); /* (:46) */
    wf[2] = 0.0;                          /* w_f.at<double>(0,2) = 0 (:47) */
    const double wd[9] = {wf[0], 0, 0, 0, wf[1], 0, 0, 0, wf[2]};
    double tmp[9];
    gemm33(uf, wd, tmp);
    gemm33(tmp, vtf, Ec); /* E_mat_correct = u_f * w_f_diag * vt_f (:50) */
}

/* the opt-in inlier count (no reference counterpart; erp_match.h erp_ransac_cfg.inlier_thr) */
int32_t erpo_inlier_count(const double* bl, const double* br, int32_t m, const double Ec[9],
                          double thr, double band, int32_t* n_band) {
    int32_t n = 0, nb = 0;
    for (int32_t i = 0; i < m; i++) {
        const double* l = bl + (size_t)i * 3;
        const double* r = br + (size_t)i * 3;
        double res = Ec[0] * (l[0] * r[0]);
        for (int k = 1; k < 9; k++) res = fma(Ec[k], l[k / 3] * r[k % 3], res);
        const double a = fabs(res);
        n += a < thr;
        nb += fabs(a - thr) <= band;
    }
    if (n_band) *n_band = nb;
    return n;
}

static int eight_point_estimation_impl(const double* bl, const double* br, int32_t m, double valid_abs,
                                       erpo_hyp* h) {
    if (m < 1) return -2;
    /* A row = [lx*rx, lx*ry, lx*rz, ly*rx, ly*ry, ly*rz, lz*rx, lz*ry, lz*rz] (:22-37) */
    double* A = (double*)malloc(sizeof(double) * (size_t)m * 9);
    for (int32_t i = 0; i < m; i++) {
        const double* l = bl + (size_t)i * 3;
        const double* r = br + (size_t)i * 3;
        double* a = A + (size_t)i * 9;
        a[0] = l[0] * r[0];
        a[1] = l[0] * r[1];
        a[2] = l[0] * r[2];
        a[3] = l[1] * r[0];
        a[4] = l[1] * r[1];
        a[5] = l[1] * r[2];
        a[6] = l[2] * r[0];
        a[7] = l[2] * r[1];
        a[8] = l[2] * r[2];
    }
    const int rows = m < 9 ? m : 9;
    double w[9];
    double* vt = (double*)malloc(sizeof(double) * (size_t)rows * 9);
    double* u = (double*)malloc(sizeof(double) * (size_t)m * rows);
    erpo_svdecomp(A, m, 9, w, u, vt); /* SVDecomp(A_mat, w, u, vt) (:39) */
    double E[9];
    memcpy(E, vt + (size_t)(rows - 1) * 9, sizeof(E)); /* e = vt.row(vt.rows-1) (:42-44) */
    free(A);
    free(vt);
    free(u);

    double Ec[9];
    erpo_rank2(E, Ec);

    double R1[9], R2[9], t[3];
    decompose_essential(Ec, R1, R2, t); /* (:54) */
    double e1[3], e2[3];
    erpo_rot2eular(R1, e1);
    erpo_rot2eular(R2, e2);
    for (int k = 0; k < 3; k++) {
        h->R1[k] = (float)e1[k];
        h->R2[k] = (float)e2[k];
        h->T[k] = (float)t[k];
    }
    const float a1[3] = {fabsf(h->R1[0]), fabsf(h->R1[1]), fabsf(h->R1[2])};
    const float a2[3] = {fabsf(h->R2[0]), fabsf(h->R2[1]), fabsf(h->R2[2])};
    h->R1_valid = max_vec(a1) < valid_abs;
    h->R2_valid = max_vec(a2) < valid_abs;
    memcpy(h->E, E, sizeof(E));
    memcpy(h->E_corr, Ec, sizeof(Ec));
    return 0;
}

int erpo_eight_point_estimation(const double* bl, const double* br, int32_t m, erpo_hyp* h) {
    return eight_point_estimation_impl(bl, br, m, 1.57, h);
}

/* consensus (src/eight_point.cpp:129-149) */
static int cmp_double(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

int erpo_consensus(const float* rvec, int32_t K, double trim_lo, double trim_hi, int32_t* min_idx,
                   double* dist_out) {
    if (K <= 0) return -3;
    double* dist = (double*)malloc(sizeof(double) * (size_t)K);
    const long lo = (long)(K * trim_lo);
    const long hi = (long)(K * trim_hi);
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
        double* arr = (double*)malloc(sizeof(double) * (size_t)K);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int32_t i = 0; i < K; i++) {
            for (int32_t j = 0; j < K; j++) {
                const float dx = rvec[i * 3 + 0] - rvec[j * 3 + 0];
                const float dy = rvec[i * 3 + 1] - rvec[j * 3 + 1];
                const float dz = rvec[i * 3 + 2] - rvec[j * 3 + 2];
                arr[j] = (double)sqrtf(dx * dx + dy * dy + dz * dz);
            }
            qsort(arr, (size_t)K, sizeof(double), cmp_double);
            double acc = 0.0;
            for (long k = lo; k < hi; k++) acc += arr[k];
            dist[i] = acc / ((double)(hi - lo) * 1.0);
        }
        free(arr);
    }
    int32_t best = 0;
    for (int32_t i = 1; i < K; i++)
        if (dist[i] < dist[best]) best = i; /* std::min_element: first minimum */
    *min_idx = best;
    if (dist_out) memcpy(dist_out, dist, sizeof(double) * (size_t)K);
    free(dist);
    return 0;
}

int erpo_initial_guess(const double* bl, const double* br, int32_t m, const erpo_cfg* cfg,
                       float R_out[3], float T_out[3], erpo_diag* diag, erpo_hyp* hyp,
                       int32_t* samples, float* rvec, float* tvec, double* dist) {
    erpo_diag dg;
    memset(&dg, 0, sizeof(dg));
    const int32_t iters = cfg->iters;
    const int32_t sample_n = (int32_t)(m * cfg->sample_frac); /* int sample_n = match_size*0.25 */
    dg.sample_n = sample_n;
    dg.min_idx = -1;
    if (m < 1 || sample_n < 1 || iters < 1) {
        dg.status = -2;
        if (diag) *diag = dg;
        return -2;
    }
    /* draw every subset first (the rand() stream is sequential), then estimate in parallel */
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)iters * sample_n);
    if (cfg->sampler == 1) {  /* ERP_SAMPLER_PHILOX: ascending index sets */
        for (int32_t it = 0; it < iters; it++)
            erpo_philox_sample(m, sample_n, cfg->offset + (uint64_t)it, cfg->seed,
                               idx + (size_t)it * sample_n);
    } else {
        erpo_glibc g;
        erpo_glibc_seed(&g, cfg->seed);
        erpo_glibc_discard(&g, cfg->offset);
        int32_t* a = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
        for (int32_t it = 0; it < iters; it++) {
            erpo_random_array(a, m, &g);
            memcpy(idx + (size_t)it * sample_n, a, sizeof(int32_t) * (size_t)sample_n);
        }
        free(a);
    }
    if (samples) memcpy(samples, idx, sizeof(int32_t) * (size_t)iters * sample_n);
    erpo_hyp* hs = (erpo_hyp*)malloc(sizeof(erpo_hyp) * (size_t)iters);
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
        double* sl = (double*)malloc(sizeof(double) * (size_t)sample_n * 3);
        double* sr = (double*)malloc(sizeof(double) * (size_t)sample_n * 3);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int32_t it = 0; it < iters; it++) {
            for (int32_t k = 0; k < sample_n; k++) {
                const int32_t p = idx[(size_t)it * sample_n + k];
                memcpy(sl + (size_t)k * 3, bl + (size_t)p * 3, 3 * sizeof(double));
                memcpy(sr + (size_t)k * 3, br + (size_t)p * 3, 3 * sizeof(double));
            }
            eight_point_estimation_impl(sl, sr, sample_n, cfg->valid_abs, &hs[it]);
            hs[it].inliers = cfg->inlier_thr > 0
                                 ? erpo_inlier_count(bl, br, m, hs[it].E_corr, cfg->inlier_thr,
                                                     0.0, NULL)
                                 : 0;
        }
        free(sl);
        free(sr);
    }
    free(idx);
    /* push R1 then R2 per iteration (:113-126) */
    float* rv = (float*)malloc(sizeof(float) * (size_t)iters * 6);
    float* tv = (float*)malloc(sizeof(float) * (size_t)iters * 6);
    int32_t K = 0;
    for (int32_t it = 0; it < iters; it++) {
        if (hs[it].R1_valid) {
            memcpy(rv + (size_t)K * 3, hs[it].R1, 3 * sizeof(float));
            memcpy(tv + (size_t)K * 3, hs[it].T, 3 * sizeof(float));
            K++;
        }
        if (hs[it].R2_valid) {
            memcpy(rv + (size_t)K * 3, hs[it].R2, 3 * sizeof(float));
            memcpy(tv + (size_t)K * 3, hs[it].T, 3 * sizeof(float));
            K++;
        }
    }
    if (hyp) memcpy(hyp, hs, sizeof(erpo_hyp) * (size_t)iters);
    free(hs);
    dg.K = K;
    int rc = 0;
    if (K == 0) {
        dg.status = -3; /* reference: R_vec_arr[0] on an empty vector = UB */
        rc = -3;
    } else {
        double* d = (double*)malloc(sizeof(double) * (size_t)K);
        int32_t mi = 0;
        erpo_consensus(rv, K, cfg->trim_lo, cfg->trim_hi, &mi, d);
        dg.min_idx = mi;
        dg.min_dist = d[mi];
        memcpy(R_out, rv + (size_t)mi * 3, 3 * sizeof(float));
        memcpy(T_out, tv + (size_t)mi * 3, 3 * sizeof(float));
        if (dist) memcpy(dist, d, sizeof(double) * (size_t)K);
        free(d);
    }
    if (rvec) memcpy(rvec, rv, sizeof(float) * (size_t)K * 3);
    if (tvec) memcpy(tvec, tv, sizeof(float) * (size_t)K * 3);
    free(rv);
    free(tv);
    if (diag) *diag = dg;
    return rc;
}

int erpo_find(int32_t W, int32_t H, const float* kl, const float* kr, int32_t m, const erpo_cfg* cfg,
              float R_out[3], float T_out[3], erpo_diag* diag, erpo_hyp* hyp, int32_t* samples,
              float* rvec, float* tvec, double* dist) {
    if (m < 0) return -1;
    double* bl = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1) * 3);
    double* br = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1) * 3);
    for (int32_t i = 0; i < m; i++) {
        erpo_pixel_to_bearing(W, H, kl[2 * i], kl[2 * i + 1], bl + (size_t)i * 3);
        erpo_pixel_to_bearing(W, H, kr[2 * i], kr[2 * i + 1], br + (size_t)i * 3);
    }
    const int rc = erpo_initial_guess(bl, br, m, cfg, R_out, T_out, diag, hyp, samples, rvec, tvec, dist);
    free(bl);
    free(br);
    return rc;
}

/* ======================================================================================
 * ERP remaps: src/erp_rotation.cpp:66-122, src/spherical_surf.cpp:16-63,
 * 77-133, src/automatic.cpp:50-79,148-152.
 * ==================================================================================== */
/* x86-64 cvttsd2si / cvttss2si: truncation, INT32_MIN ("integer indefinite") for NaN and
 * out-of-range values -- what the reference's implicit double/float -> int conversions do */
static int32_t cvt_x86_d(double x) {
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int32_t)x;
}
static int32_t cvt_x86_f(float x) {
    if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
    return (int32_t)x;
}

/* erp_rotation::rotate_pixel, src/erp_rotation.cpp:66-92 (in_vec = (row, col)) */
void erpo_rotate_pixel(int32_t row, int32_t col, const double m[9], int32_t W, int32_t H,
                       int32_t out[2]) {
    const double a = M_PI * row / H;                 /* :68 */
    const double b = 2 * M_PI * col / W;
    const double c0 = -sin(a) * cos(b);              /* :71-73 */
    const double c1 = sin(a) * sin(b);
    const double c2 = cos(a);
    const double r0 = m[0] * c0 + m[1] * c1 + m[2] * c2;  /* :77-79 */
    const double r1 = m[3] * c0 + m[4] * c1 + m[5] * c2;
    const double r2 = m[6] * c0 + m[7] * c1 + m[8] * c2;
    const double v0 = acos(r2);                      /* :82-85 */
    double v1 = atan2(r1, -r0);
    if (v1 < 0) v1 += M_PI * 2;
    out[0] = cvt_x86_d(H * v0 / M_PI);               /* :88-89 */
    out[1] = cvt_x86_d(W * v1 / (2 * M_PI));
}

/* rotate_pixel's two values BEFORE the truncating conversion (H*acos/M_PI, W*atan2'/(2*M_PI))
 * for n pixels: the test diagnostic that tells a last-ulp libm decision (value within ~1e-12
 * of an integer) from a real remap error */
void erpo_rotate_pixel_prefix(const int32_t* rows, const int32_t* cols, int32_t n, const double m[9],
                              int32_t W, int32_t H, double* out) {
    int32_t k;
    for (k = 0; k < n; k++) {
        const double a = M_PI * rows[k] / H;
        const double b = 2 * M_PI * cols[k] / W;
        const double c0 = -sin(a) * cos(b);
        const double c1 = sin(a) * sin(b);
        const double c2 = cos(a);
        const double r0 = m[0] * c0 + m[1] * c1 + m[2] * c2;
        const double r1 = m[3] * c0 + m[4] * c1 + m[5] * c2;
        const double r2 = m[6] * c0 + m[7] * c1 + m[8] * c2;
        double v1 = atan2(r1, -r0);
        if (v1 < 0) v1 += M_PI * 2;
        out[2 * k] = H * acos(r2) / M_PI;
        out[2 * k + 1] = W * v1 / (2 * M_PI);
    }
}

/* Mat::inv() (DECOMP_LU) on a 3x3 double matrix: adjugate / determinant [OpenCV, recalled] */
int32_t erpo_inv3(const double m[9], double out[9]) {
    double d = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
               m[2] * (m[3] * m[7] - m[4] * m[6]);
    double t[9];
    if (d == 0.0) return 0;
    d = 1. / d;
    t[0] = (m[4] * m[8] - m[5] * m[7]) * d;
    t[1] = (m[2] * m[7] - m[1] * m[8]) * d;
    t[2] = (m[1] * m[5] - m[2] * m[4]) * d;
    t[3] = (m[5] * m[6] - m[3] * m[8]) * d;
    t[4] = (m[0] * m[8] - m[2] * m[6]) * d;
    t[5] = (m[2] * m[3] - m[0] * m[5]) * d;
    t[6] = (m[3] * m[7] - m[4] * m[6]) * d;
    t[7] = (m[1] * m[6] - m[0] * m[7]) * d;
    t[8] = (m[0] * m[4] - m[1] * m[3]) * d;
    memcpy(out, t, sizeof(t));
    return 1;
}

/* rot_from_vec, src/automatic.cpp:50-64: I + [v]x + [v]x*[v]x*(1/1+c), 1/1 = 1 (int) */
void erpo_rot_from_vec(const double v1[3], const double v2[3], double R[9]) {
    const double v[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                         v1[0] * v2[1] - v1[1] * v2[0]};
    const double c = v1[0] * v2[0] + v1[1] * v2[1] + v1[2] * v2[2];
    const double vx[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
    double sq[9];
    int k;
    gemm33(vx, vx, sq);
    for (k = 0; k < 9; k++) R[k] = ((k % 4 == 0 ? 1.0 : 0.0) + vx[k]) + sq[k] * (1 / 1 + c);
}

/* eular2rot(Vec3f(0, RAD(pitch), 0)): RAD in double, stored into a float Vec3f */
static void pitch_rot(float deg, double R[9]) {
    const double e[3] = {0.0, (double)(float)(M_PI * deg / 180.0), 0.0};
    erpo_eular2rot(e, R);
}

static void copy_px(const uint8_t* s, uint8_t* d) { d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; }

/* crop_rotated_image, src/spherical_surf.cpp:16-48 */
void erpo_crop_rotated_image(const uint8_t* im, int32_t W, int32_t H, float pitch_deg,
                             uint8_t* out) {
    double R[9];
    int i;
    pitch_rot(pitch_deg, R);
#pragma omp parallel for schedule(static)
    for (i = 0; i < H / 4; i++) {
        int j;
        for (j = 0; j < W; j++) {
            int32_t o[2];
            erpo_rotate_pixel(i + H * 3 / 8, j, R, W, H, o);
            if (o[0] >= 0 && o[1] >= 0 && o[0] < H && o[1] < W)
                copy_px(im + ((size_t)o[0] * W + o[1]) * 3, out + ((size_t)i * W + j) * 3);
        }
    }
}

/* rotate_keypoint, src/spherical_surf.cpp:50-63 (kp_xy = n x (pt.x, pt.y) floats) */
void erpo_rotate_keypoint(float* kp_xy, int32_t n, float pitch_deg, int32_t W, int32_t H) {
    double R[9];
    int32_t i;
    pitch_rot(pitch_deg, R);
    for (i = 0; i < n; i++) {
        const int32_t offset_i = cvt_x86_f(kp_xy[2 * i + 1] + (float)(H * 3 / 8));
        int32_t o[2];
        erpo_rotate_pixel(offset_i, cvt_x86_f(kp_xy[2 * i]), R, W, H, o);
        kp_xy[2 * i] = (float)o[1];
        kp_xy[2 * i + 1] = (float)o[0];
    }
}

/* do_all's keypoint step, src/spherical_surf.cpp:120-126 (bands n0, n1, n2, n3 in order) */
void erpo_unrotate_band_keypoints(float* kp_xy, const int32_t counts[4], int32_t W, int32_t H) {
    float* p = kp_xy;
    int32_t i;
    erpo_rotate_keypoint(p, counts[0], 45.f, W, H);
    p += 2 * (size_t)counts[0];
    for (i = 0; i < counts[1]; i++) p[2 * i + 1] = p[2 * i + 1] + (float)(H * 3 / 8);
    p += 2 * (size_t)counts[1];
    erpo_rotate_keypoint(p, counts[2], -45.f, W, H);
    p += 2 * (size_t)counts[2];
    erpo_rotate_keypoint(p, counts[3], -90.f, W, H);
}

/* rotate_image, src/erp_rotation.cpp:94-122 (rot_mat inverted inside, :103) */
int32_t erpo_rotate_image(const uint8_t* im, int32_t W, int32_t H, const double rot_mat[9],
                          uint8_t* out) {
    double Ri[9];
    int i;
    if (!erpo_inv3(rot_mat, Ri)) return 0;
#pragma omp parallel for schedule(static)
    for (i = 0; i < H; i++) {
        int j;
        for (j = 0; j < W; j++) {
            int32_t o[2];
            erpo_rotate_pixel(i, j, Ri, W, H, o);
            if (o[0] >= 0 && o[1] >= 0 && o[0] < H && o[1] < W)
                copy_px(im + ((size_t)o[0] * W + o[1]) * 3, out + ((size_t)i * W + j) * 3);
        }
    }
    return 1;
}

/* rectify, src/automatic.cpp:66-79 */
int32_t erpo_rectify(const uint8_t* left, const uint8_t* right, int32_t W, int32_t H,
                     const double rot_vec[3], const double t_vec[3], uint8_t* left_out,
                     uint8_t* right_out) {
    const double down[3] = {0, -1, 0};
    double Rl[9], Rl_inv[9], E[9], E_inv[9], Rr[9], Rr_inv[9];
    erpo_rot_from_vec(down, t_vec, Rl);
    if (!erpo_inv3(Rl, Rl_inv)) return 0;
    erpo_eular2rot(rot_vec, E);
    if (!erpo_inv3(E, E_inv)) return 0;
    gemm33(Rl, E_inv, Rr);
    if (!erpo_inv3(Rr, Rr_inv)) return 0;
    return erpo_rotate_image(left, W, H, Rl_inv, left_out) &&
           erpo_rotate_image(right, W, H, Rr_inv, right_out);
}

/* src/automatic.cpp:148-151: rotate_image by eular2rot(RAD(89.999),0,0).inv(), then
 * cv::rotate(ROTATE_90_CLOCKWISE): out (W rows x H cols), out[r][c] = tmp[H-1-c][r].  The
 * intermediate starts as a copy of `out`'s prior content transposed back, so unwritten pixels
 * keep it (the kernel writes only mapped pixels). */
int32_t erpo_vertical_rotate(const uint8_t* im, int32_t W, int32_t H, uint8_t* out) {
    const double e[3] = {M_PI * (89.999) / 180.0, 0, 0};
    double R[9], Ri[9];
    uint8_t* tmp = (uint8_t*)malloc((size_t)W * H * 3);
    int i;
    if (!tmp) return 0;
    erpo_eular2rot(e, R);
    if (!erpo_inv3(R, Ri)) { free(tmp); return 0; }
    for (i = 0; i < H; i++) {
        int j;
        for (j = 0; j < W; j++)  /* tmp[i][j] <- out[j][H-1-i] (prior content) */
            copy_px(out + ((size_t)j * H + (H - 1 - i)) * 3, tmp + ((size_t)i * W + j) * 3);
    }
    if (!erpo_rotate_image(im, W, H, Ri, tmp)) { free(tmp); return 0; }
    for (i = 0; i < W; i++) {
        int c;
        for (c = 0; c < H; c++)
            copy_px(tmp + ((size_t)(H - 1 - c) * W + i) * 3, out + ((size_t)i * H + c) * 3);
    }
    free(tmp);
    return 1;
}
