// erp_device.hpp -- per-hypothesis math of the eight-point estimator, written once and compiled
// for gfx950 (inside the HIP kernels) and for the host (tests/host_math harness only, so the
// numerics can be checked against the oracle without a GPU).  No OpenCV.
//
// What each function follows in the reference:
//   gram_jacobi9      SVDecomp(A_mat, w, u, vt); e = vt.row(vt.rows-1)  src/eight_point.cpp:39-44
//                     -- evaluated in Gram space (G = A^T A, 9x9, fp64) with the SAME cyclic
//                        one-sided Jacobi rotation formulas/order OpenCV's JacobiSVDImpl_ applies
//                        to the columns of A, so the right singular vectors agree up to sign.
//   svd3_opencv       SVDecomp on 3x3 (src/eight_point.cpp:46, and inside decomposeEssentialMat)
//                     -- OpenCV JacobiSVDImpl_ restated operation-for-operation, so the sign
//                        conventions that decide T's sign and the R1/R2 order match.
//   decompose_e       cv::decomposeEssentialMat (src/eight_point.cpp:54)
//   rot2eular         src/erp_rotation.cpp:43-63
//   pixel_to_bearing  src/eight_point.cpp:163-186
//   estimate_from_e   src/eight_point.cpp:42-84 (rank-2 fix, decompose, Euler, validity)
//   rotate_pixel      src/erp_rotation.cpp:66-92 (band remap, keypoint un-rotation, rectification)
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ERP_HD __host__ __device__
#define ERP_INLINE __forceinline__
#else
#include <math.h>
#define ERP_HD
#define ERP_INLINE inline
#endif

namespace erp {

constexpr double kPi = 3.14159265358979323846;
constexpr double kDblEps = 2.2204460492503131e-16;
constexpr double kDblMin = 2.2250738585072014e-308;

struct Hyp {            // per-iteration record (parity/debug output and consensus input)
    float R1[3], R2[3], T[3];
    int32_t R1_valid, R2_valid;
    double E[9];        // e = eigen/singular vector reshaped row-major (sign arbitrary)
};

// ---------------------------------------------------------------- small 3x3 helpers ----
// cv::gemm small-matrix path: d[i][j] = a[i][0]*b[0][j] + a[i][1]*b[1][j] + a[i][2]*b[2][j]
ERP_HD ERP_INLINE void gemm33(const double* a, const double* b, double* d) {
    double t[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            t[i * 3 + j] = a[i * 3 + 0] * b[0 * 3 + j] + a[i * 3 + 1] * b[1 * 3 + j] + a[i * 3 + 2] * b[2 * 3 + j];
#pragma unroll
    for (int k = 0; k < 9; k++) d[k] = t[k];
}

ERP_HD ERP_INLINE double det33(const double* m) {
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

ERP_HD ERP_INLINE uint32_t cv_rng_next(uint64_t& state) {
    state = (uint64_t)(uint32_t)state * 4164903690U + (uint32_t)(state >> 32);
    return (uint32_t)state;
}

// OpenCV 3.4 SVDecomp(src 3x3, flags=0): at == false, so At = src^T (rows = columns of src),
// JacobiSVDImpl_<double>(At, W, Vt, m=3, n=3, n1=3, DBL_MIN, 10*DBL_EPSILON);
// u = At^T (normalised), vt = Vt.  Operation order follows the scalar template.
ERP_HD inline void svd3_opencv(const double* src, double* w_out, double* u, double* vt) {
    double At[9], V[9], W[3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) At[i * 3 + k] = src[k * 3 + i];
    const double eps = kDblEps * 10;
    const double minval = kDblMin;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const double t = At[i * 3 + k];
            sd += t * t;
        }
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < 3; k++) V[i * 3 + k] = 0;
        V[i * 3 + i] = 1;
    }
    for (int iter = 0; iter < 30; iter++) {  // max_iter = max(m, 30)
        bool changed = false;
#pragma unroll
        for (int pr = 0; pr < 3; pr++) {
            const int i = pr < 2 ? 0 : 1;
            const int j = pr == 0 ? 1 : 2;
            double a = W[i], p = 0, b = W[j];
#pragma unroll
            for (int k = 0; k < 3; k++) p += At[i * 3 + k] * At[j * 3 + k];
            if (fabs(p) <= eps * sqrt(a * b)) continue;
            p *= 2;
            const double beta = a - b, gamma = hypot(p, beta);
            double c, s;
            if (beta < 0) {
                const double delta = (gamma - beta) * 0.5;
                s = sqrt(delta / gamma);
                c = p / (gamma * s * 2);
            } else {
                c = sqrt((gamma + beta) / (gamma * 2));
                s = p / (gamma * c * 2);
            }
            a = b = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const double t0 = c * At[i * 3 + k] + s * At[j * 3 + k];
                const double t1 = -s * At[i * 3 + k] + c * At[j * 3 + k];
                At[i * 3 + k] = t0;
                At[j * 3 + k] = t1;
                a += t0 * t0;
                b += t1 * t1;
            }
            W[i] = a;
            W[j] = b;
            changed = true;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const double t0 = c * V[i * 3 + k] + s * V[j * 3 + k];
                const double t1 = -s * V[i * 3 + k] + c * V[j * 3 + k];
                V[i * 3 + k] = t0;
                V[j * 3 + k] = t1;
            }
        }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const double t = At[i * 3 + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    // selection sort descending, swapping rows of At and Vt: i = 0 swaps row 0 with the first
    // maximum j, i = 1 rows 1 and 2 if W[1] < W[2].  Written as conditional swaps with fixed
    // indices (the same moves: a per-lane row index j made every access a select chain over
    // all 21 values, ~190 v_cndmask per decomposition)
    auto cswap = [&](bool c, int a, int b) {
        double t = W[a];
        W[a] = c ? W[b] : t;
        W[b] = c ? t : W[b];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            t = At[a * 3 + k];
            At[a * 3 + k] = c ? At[b * 3 + k] : t;
            At[b * 3 + k] = c ? t : At[b * 3 + k];
            t = V[a * 3 + k];
            V[a * 3 + k] = c ? V[b * 3 + k] : t;
            V[b * 3 + k] = c ? t : V[b * 3 + k];
        }
    };
    {
        const bool j1 = W[0] < W[1];              // k = 1
        const bool j2 = (j1 ? W[1] : W[0]) < W[2];  // k = 2 against W[j]
        cswap(j1 && !j2, 0, 1);
        cswap(j2, 0, 2);
        cswap(W[1] < W[2], 1, 2);
    }
    uint64_t rng = 0x12345678;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double sd = W[i];
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / 3;
#pragma unroll
            for (int k = 0; k < 3; k++) At[i * 3 + k] = (cv_rng_next(rng) & 256) != 0 ? val0 : -val0;
            for (int it2 = 0; it2 < 2; it2++) {
#pragma unroll
                for (int j = 0; j < i; j++) {
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < 3; k++) sd += At[i * 3 + k] * At[j * 3 + k];
                    double asum = 0;
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const double t = At[i * 3 + k] - sd * At[j * 3 + k];
                        At[i * 3 + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < 3; k++) At[i * 3 + k] *= asum;
                }
            }
            sd = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const double t = At[i * 3 + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
#pragma unroll
        for (int k = 0; k < 3; k++) At[i * 3 + k] *= s;
    }
#pragma unroll
    for (int i = 0; i < 3; i++) w_out[i] = W[i];
    // u = transpose(temp_u): u[r][c] = At[c][r]
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) u[r * 3 + c] = At[c * 3 + r];
#pragma unroll
    for (int k = 0; k < 9; k++) vt[k] = V[k];
}

// cv::decomposeEssentialMat restated
ERP_HD inline void decompose_e(const double* E, double* R1, double* R2, double* t) {
    double D[3], U[9], Vt[9];
    svd3_opencv(E, D, U, Vt);
    if (det33(U) < 0)
#pragma unroll
        for (int k = 0; k < 9; k++) U[k] *= -1.;
    if (det33(Vt) < 0)
#pragma unroll
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

ERP_HD ERP_INLINE void rot2eular(const double* R, double* e) {
    const double sy = sqrt(R[8] * R[8] + R[5] * R[5]);
    const bool singular = sy < 1e-6;
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

// eight_point::find pixel -> bearing: lon = 2*M_PI*(pt.x / im_width) with the division in
// float, lat likewise; OMAF axes.
ERP_HD ERP_INLINE void pixel_to_bearing(int32_t W, int32_t H, float px, float py, double* b) {
    const float fx = px / (float)W;
    const float fy = py / (float)H;
    const double lon = 2 * kPi * (double)fx;
    const double lat = kPi * (double)fy;
    const double sl = sin(lat);
    b[0] = -sl * cos(lon);
    b[1] = sl * sin(lon);
    b[2] = cos(lat);
}

// ---- ERP remapping (section 8f: band remap and rectification) ---------------------------
// double -> int32 as x86-64's cvttsd2si (the reference's implicit conversions compile to it):
// truncation toward zero, and the "integer indefinite" INT32_MIN for NaN or out-of-range values
// (C leaves those undefined; the GPU's v_cvt_i32_f64 would clamp / give 0 instead).
ERP_HD ERP_INLINE int32_t trunc_i32_x86(double x) {
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int32_t)x;
}
ERP_HD ERP_INLINE int32_t trunc_i32_x86f(float x) {  // cvttss2si
    if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT32_MIN;
    return (int32_t)x;
}

// atan2 / acos as glibc's (correctly rounded in practice) where the device library is not:
// the results that decide a truncated pixel index at the ERP seams are pi - tiny and
// pi/2 - tiny (e.g. column W/2, where sin(2*M_PI*col/W) = 1.2e-16 makes atan2(tiny, x<0));
// the device atan2 returns atan(|y/x|) subtracted from pi without pi's low part and can land
// one ulp below glibc, flipping (int)(W*v/(2*M_PI)) from W/2 to W/2-1.  In those regimes the
// value is rebuilt from pi = PI_HI + PI_LO: pi - z = PI_HI + (PI_LO - z) (one rounding), with
// atan(z) = z (1 - z^2/3 + ...) = z to far below an ulp for z <= 2^-30.
ERP_HD ERP_INLINE double atan2_ref(double y, double x) {
    constexpr double kPiHi = 3.141592653589793116, kPiLo = 1.2246467991473532e-16;
    if (x < 0 && fabs(y) <= 0x1p-30 * -x) {
        const double z = fabs(y) / -x;
        return copysign(kPiHi + (kPiLo - z), y);
    }
    return atan2(y, x);
}
ERP_HD ERP_INLINE double acos_ref(double r) {
    constexpr double kPio2Hi = 1.5707963267948966, kPio2Lo = 6.123233995736766e-17;
    if (fabs(r) <= 0x1p-30) return kPio2Hi + (kPio2Lo - r);  // acos r = pi/2 - r - r^3/6 ...
    return acos(r);
}

// ---- correctly rounded sin / cos / acos / atan2 (double-double), the boundary slow path ----
// rotate_pixel truncates H*acos(.)/M_PI and W*atan2(.)/(2*M_PI); when such a value lies within
// ~1e-8 of an integer the index depends on the LAST ulp of the four transcendentals.  glibc
// (the reference's libm) rounds them correctly but for rare hard cases (<= ~0.52 ulp), the
// device library does not (1-2 ulp), so near a boundary the pixel is recomputed with these
// correctly rounded versions: reduction by pi/2 in three parts, Taylor series in double-double
// (|r| <= pi/4: 14 terms, truncation < 1e-30), and one Newton step in double-double for
// acos / atan2 from the fast value.
struct DD {
    double h, l;
};
ERP_HD ERP_INLINE DD dd_two_sum(double a, double b) {
    const double s = a + b, t = s - a;
    return DD{s, (a - (s - t)) + (b - t)};
}
ERP_HD ERP_INLINE DD dd_quick(double a, double b) {
    const double s = a + b;
    return DD{s, b - (s - a)};
}
ERP_HD ERP_INLINE DD dd_add(DD x, DD y) {
    DD s = dd_two_sum(x.h, y.h);
    const DD t = dd_two_sum(x.l, y.l);
    s.l += t.h;
    s = dd_quick(s.h, s.l);
    s.l += t.l;
    return dd_quick(s.h, s.l);
}
ERP_HD ERP_INLINE DD dd_mul(DD x, DD y) {
    const double p = x.h * y.h;
    double e = fma(x.h, y.h, -p);
    e += x.h * y.l + x.l * y.h;
    return dd_quick(p, e);
}
ERP_HD ERP_INLINE DD dd_mul_d(DD x, double d) {
    const double p = x.h * d;
    double e = fma(x.h, d, -p);
    e += x.l * d;
    return dd_quick(p, e);
}
// 1/n!, n = 2..27, as double-double
ERP_HD ERP_INLINE DD dd_inv_fact(int n) {
    const double t[26][2] = {
        {0.5, 0.0}, {0.16666666666666666, 9.25185853854297e-18},
        {0.041666666666666664, 2.3129646346357427e-18}, {0.008333333333333333, 1.1564823173178714e-19},
        {0.001388888888888889, -5.300543954373577e-20}, {0.0001984126984126984, 1.7209558293420705e-22},
        {2.48015873015873e-05, 2.1511947866775882e-23}, {2.7557319223985893e-06, -1.858393274046472e-22},
        {2.755731922398589e-07, 2.3767714622250297e-23}, {2.505210838544172e-08, -1.448814070935912e-24},
        {2.08767569878681e-09, -1.20734505911326e-25}, {1.6059043836821613e-10, 1.2585294588752098e-26},
        {1.1470745597729725e-11, 2.0655512752830745e-28}, {7.647163731819816e-13, 7.03872877733453e-30},
        {4.779477332387385e-14, 4.399205485834081e-31}, {2.8114572543455206e-15, 1.6508842730861433e-31},
        {1.5619206968586225e-16, 1.1910679660273754e-32}, {8.22063524662433e-18, 2.2141894119604265e-34},
        {4.110317623312165e-19, 1.4412973378659527e-36}, {1.9572941063391263e-20, -1.3643503830087908e-36},
        {8.896791392450574e-22, -7.911402614872376e-38}, {3.868170170630684e-23, -8.843177655482344e-40},
        {1.6117375710961184e-24, -3.6846573564509766e-41}, {6.446950284384474e-26, -1.9330404233703465e-42},
        {2.4795962632247976e-27, -1.2953730964765229e-43}, {9.183689863795546e-29, 1.4303150396787322e-45}};
    return DD{t[n - 2][0], t[n - 2][1]};
}
// sin and cos of a double x (|x| < 16) in double-double
ERP_HD ERP_INLINE void dd_sincos(double x, DD* sn, DD* cs) {
    constexpr double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17,
                     P3 = -1.4973849048591698e-33;
    const double k = rint(x * 0.63661977236758138);
    const double p = k * P1, pe = fma(k, P1, -p);  // k * P1 = p + pe exactly
    DD r = dd_two_sum(x - p, -pe);                  // x - p exact (Sterbenz, or k = 0)
    const double q2 = k * P2;
    r = dd_add(r, DD{-q2, -fma(k, P2, -q2)});
    r = dd_add(r, DD{-k * P3, 0.0});
    const DD z = dd_mul(r, r);
    DD s = dd_inv_fact(27), c = dd_inv_fact(26);
#pragma unroll
    for (int n = 25; n >= 3; n -= 2) {  // (unrolled: the table folds into constants)  // S(z) = 1/1! - z/3! + ..., C(z) = 1 - z/2! + ...
        s = dd_add(dd_inv_fact(n), dd_mul_d(dd_mul(s, z), -1.0));
        c = dd_add(dd_inv_fact(n - 1), dd_mul_d(dd_mul(c, z), -1.0));
    }
    s = dd_add(DD{1.0, 0.0}, dd_mul_d(dd_mul(s, z), -1.0));
    c = dd_add(DD{1.0, 0.0}, dd_mul_d(dd_mul(c, z), -1.0));
    s = dd_mul(s, r);
    const int q = ((int)fmod(k, 4.0) + 4) & 3;
    const DD ns{-s.h, -s.l}, nc{-c.h, -c.l};
    *sn = q == 0 ? s : q == 1 ? c : q == 2 ? ns : nc;
    *cs = q == 0 ? c : q == 1 ? ns : q == 2 ? nc : s;
}
ERP_HD ERP_INLINE void sincos_cr(double x, double* sn, double* cs) {
    if (!(fabs(x) < 16.0)) {
        *sn = sin(x);
        *cs = cos(x);
        return;
    }
    DD s, c;
    dd_sincos(x, &s, &c);
    *sn = s.h;
    *cs = c.h;
}
ERP_HD ERP_INLINE double acos_cr(double x) {
    const double y0 = acos_ref(x);
    if (!(fabs(x) < 1.0) || y0 == 0.0) return y0;
    DD s, c;
    dd_sincos(y0, &s, &c);
    const DD num = dd_add(c, DD{-x, 0.0});  // cos(y0) - x;  acos' = -1/sin
    return y0 + num.h / s.h;
}
ERP_HD ERP_INLINE double atan2_cr(double y, double x) {
    const double t0 = atan2_ref(y, x);
    if (!(fabs(t0) < 4.0) || (x == 0.0 && y == 0.0) || !(fabs(x) < 1e300 && fabs(y) < 1e300))
        return t0;
    DD s, c;
    dd_sincos(t0, &s, &c);
    const DD num = dd_add(dd_mul_d(c, y), dd_mul_d(s, -x));  // y cos t - x sin t
    const double den = x * c.h + y * s.h;                     // x cos t + y sin t (= rho)
    if (!(den > 0.0)) return t0;
    return t0 + num.h / den;
}

// erp_rotation::rotate_pixel (src/erp_rotation.cpp:66-92): pixel (row, col) -> sphere (OMAF
// axes) -> m * v -> pixel, each conversion truncating.  The polar / azimuth angles of the input
// come from their sines and cosines (sa = sin(M_PI*row/height), ca = cos(...), sb, cb of
// 2*M_PI*col/width), so callers can tabulate them per row / per column.  Returns true when a
// truncated value lies within 1e-8 of an integer: the caller then redoes the pixel with
// rotate_pixel_cr (correctly rounded transcendentals, see above).
ERP_HD ERP_INLINE bool near_boundary(double X) { return fabs(X - rint(X)) < 1e-8; }
template <bool CR>
ERP_HD ERP_INLINE bool rotate_pixel_core(double sa, double ca, double sb, double cb,
                                         const double* m, int32_t W, int32_t H, int32_t* out_row,
                                         int32_t* out_col) {
    const double c0 = -sa * cb;
    const double c1 = sa * sb;
    const double c2 = ca;
    const double r0 = m[0] * c0 + m[1] * c1 + m[2] * c2;
    const double r1 = m[3] * c0 + m[4] * c1 + m[5] * c2;
    const double r2 = m[6] * c0 + m[7] * c1 + m[8] * c2;
    const double v0 = CR ? acos_cr(r2) : acos_ref(r2);
    double v1 = CR ? atan2_cr(r1, -r0) : atan2_ref(r1, -r0);
    if (v1 < 0) v1 += kPi * 2;
    const double X0 = (double)H * v0 / kPi, X1 = (double)W * v1 / (2 * kPi);
    *out_row = trunc_i32_x86(X0);
    *out_col = trunc_i32_x86(X1);
    return near_boundary(X0) || near_boundary(X1);
}
ERP_HD ERP_INLINE bool rotate_pixel_sc(double sa, double ca, double sb, double cb,
                                       const double* m, int32_t W, int32_t H, int32_t* out_row,
                                       int32_t* out_col) {
    return rotate_pixel_core<false>(sa, ca, sb, cb, m, W, H, out_row, out_col);
}
// the boundary slow path: every transcendental correctly rounded (a = polar, b = azimuth)
ERP_HD ERP_INLINE void rotate_pixel_cr(double a, double b, const double* m, int32_t W, int32_t H,
                                       int32_t* out_row, int32_t* out_col) {
    double sa, ca, sb, cb;
    sincos_cr(a, &sa, &ca);
    sincos_cr(b, &sb, &cb);
    (void)rotate_pixel_core<true>(sa, ca, sb, cb, m, W, H, out_row, out_col);
}
ERP_HD ERP_INLINE double erp_polar(int32_t row, int32_t H) { return kPi * (double)row / (double)H; }
ERP_HD ERP_INLINE double erp_azimuth(int32_t col, int32_t W) {
    return 2 * kPi * (double)col / (double)W;
}
ERP_HD ERP_INLINE void rotate_pixel(int32_t row, int32_t col, const double* m, int32_t W,
                                    int32_t H, int32_t* out_row, int32_t* out_col) {
    const double a = erp_polar(row, H), b = erp_azimuth(col, W);
    if (rotate_pixel_sc(sin(a), cos(a), sin(b), cos(b), m, W, H, out_row, out_col))
        rotate_pixel_cr(a, b, m, W, H, out_row, out_col);
}

ERP_HD ERP_INLINE double max_vec(const float* v) {
    if ((v[0] > v[1]) && (v[0] > v[2])) return v[0];
    else if (v[1] > v[2])
        return v[1];
    else
        return v[2];
}

// Rank-2 correction, decomposition, Euler conversion and validity
// (src/eight_point.cpp:42-84).  e: 9-vector (E row-major, sign irrelevant: every step below is
// odd in E and decomposeEssentialMat's det fixes cancel the sign exactly).
// E_mat_correct (src/eight_point.cpp:45-50): SVDecomp of the 3x3 E, w_f[2] = 0,
// u_f * diag(w_f) * vt_f
ERP_HD inline void rank2_correct(const double* e, double* Ec) {
    double wf[3], uf[9], vtf[9];
    svd3_opencv(e, wf, uf, vtf);
    wf[2] = 0.0;
    const double wd[9] = {wf[0], 0, 0, 0, wf[1], 0, 0, 0, wf[2]};
    double tmp[9];
    gemm33(uf, wd, tmp);
    gemm33(tmp, vtf, Ec);
}

// The opt-in inlier residual (erp_ransac_cfg.inlier_thr; no reference counterpart):
// res = l^T Ec r in a fixed fp64 order, u_k = l_i r_j (k = 3i + j), res = Ec_0 u_0, then
// res = fma(Ec_k, u_k, res), k = 1..8 (oracle/erp_oracle.c erpo_inlier_count: the same order)
ERP_HD ERP_INLINE double inlier_residual(const double* Ec, const double* l, const double* r) {
    double res = Ec[0] * (l[0] * r[0]);
#pragma unroll
    for (int k = 1; k < 9; k++) res = fma(Ec[k], l[k / 3] * r[k % 3], res);
    return res;
}

ERP_HD inline void estimate_from_e(const double* e, double valid_abs, Hyp& h) {
    double Ec[9];
    rank2_correct(e, Ec);
    double R1[9], R2[9], t[3];
    decompose_e(Ec, R1, R2, t);
    double e1[3], e2[3];
    rot2eular(R1, e1);
    rot2eular(R2, e2);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        h.R1[k] = (float)e1[k];
        h.R2[k] = (float)e2[k];
        h.T[k] = (float)t[k];
    }
    const float a1[3] = {fabsf(h.R1[0]), fabsf(h.R1[1]), fabsf(h.R1[2])};
    const float a2[3] = {fabsf(h.R2[0]), fabsf(h.R2[1]), fabsf(h.R2[2])};
    h.R1_valid = max_vec(a1) < valid_abs;
    h.R2_valid = max_vec(a2) < valid_abs;
#pragma unroll
    for (int k = 0; k < 9; k++) h.E[k] = e[k];
}

// ------------------------------------------------------------ Gram-space Jacobi (9x9) ----
// G index of the 36 distinct Gram values: A column a = 3*i + j holds l_i * r_j, so
//   G[a][b] = sum_p (l_i l_k)(r_j r_l)  with a = (i,j), b = (k,l)
// = LL[u(i,k)] * RR[u(j,l)] summed, u(.,.) the index of the unordered pair in
// {00,01,02,11,12,22}.  gram36[6*u1 + u2] = sum_p LL_p[u1] * RR_p[u2].
ERP_HD ERP_INLINE int sym3(int i, int k) {
    // 00->0 01->1 02->2 11->3 12->4 22->5
    const int a = i < k ? i : k, b = i < k ? k : i;
    return a == 0 ? b : (a == 1 ? 2 + b : 5);
}

ERP_HD ERP_INLINE void gram36_to_full(const double* g36, double* G) {
#pragma unroll
    for (int a = 0; a < 9; a++)
#pragma unroll
        for (int b = 0; b < 9; b++) {
            const int i = a / 3, j = a % 3, k = b / 3, l = b % 3;
            G[a * 9 + b] = g36[6 * sym3(i, k) + sym3(j, l)];
        }
}

// Cyclic Jacobi on the symmetric Gram matrix, mirroring OpenCV's one-sided Jacobi on A's
// columns: pair order (i<j row by row), angle from (a=G_ii, b=G_jj, p=G_ij) with the same
// formulas, Vt rows rotated the same way, then rows sorted by sqrt(G_ii) descending.
// Returns in `e` the Vt row index min(s,9)-1 (thin SVD rule of _SVDcompute for s < 9).
// Convergence: OpenCV's |p| <= 10*eps*sqrt(a*b), plus an absolute floor of
// 4*eps*trace(G) that the Gram formulation needs (rounding noise of size eps*||G|| would
// otherwise keep re-rotating exact null directions).
ERP_HD inline void gram_jacobi9(const double* G_in, int32_t s, double* e) {
    double G[81], V[81];
#pragma unroll
    for (int k = 0; k < 81; k++) {
        G[k] = G_in[k];
        V[k] = (k % 10) == 0 ? 1.0 : 0.0;
    }
    double tr = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) tr += G[i * 10];
    const double eps = kDblEps * 10;
    const double floor_abs = 4 * kDblEps * tr;
    for (int sweep = 0; sweep < 40; sweep++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < 8; i++) {
#pragma unroll
            for (int j = i + 1; j < 9; j++) {
                const double a = G[i * 9 + i], b = G[j * 9 + j], p = G[i * 9 + j];
                const double ap = fabs(p);
                if (ap <= eps * sqrt(fabs(a * b)) || ap <= floor_abs) continue;
                const double p2 = 2 * p;
                const double beta = a - b, gamma = hypot(p2, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p2 / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p2 / (gamma * c * 2);
                }
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    if (k == i || k == j) continue;
                    const double gik = G[i * 9 + k], gjk = G[j * 9 + k];
                    const double ni = c * gik + s * gjk;
                    const double nj = -s * gik + c * gjk;
                    G[i * 9 + k] = ni;
                    G[k * 9 + i] = ni;
                    G[j * 9 + k] = nj;
                    G[k * 9 + j] = nj;
                }
                const double cs2p = 2 * c * s * p;
                G[i * 9 + i] = c * c * a + cs2p + s * s * b;
                G[j * 9 + j] = s * s * a - cs2p + c * c * b;
                G[i * 9 + j] = 0;
                G[j * 9 + i] = 0;
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    const double vi = V[i * 9 + k], vj = V[j * 9 + k];
                    V[i * 9 + k] = c * vi + s * vj;
                    V[j * 9 + k] = -s * vi + c * vj;
                }
                changed = true;
            }
        }
        if (!changed) break;
    }
    // W = sqrt(diag), selection order of JacobiSVDImpl_ (first maximum), keep only the
    // permutation (rows of V are not moved: we track the index instead).
    double W[9];
    int order[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const double d = G[i * 10];
        W[i] = sqrt(d > 0 ? d : 0);
        order[i] = i;
    }
    for (int i = 0; i < 8; i++) {
        int j = i;
        for (int k = i + 1; k < 9; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            const double t = W[i];
            W[i] = W[j];
            W[j] = t;
            const int o = order[i];
            order[i] = order[j];
            order[j] = o;
        }
    }
    const int rows = s < 9 ? s : 9;
    const int sel = order[rows - 1];
    // dynamic row select without dynamic register indexing
#pragma unroll
    for (int k = 0; k < 9; k++) {
        double v = 0;
#pragma unroll
        for (int r = 0; r < 9; r++) v = (r == sel) ? V[r * 9 + k] : v;
        e[k] = v;
    }
}

// ---- s >= 9: the smallest eigenvector without accumulating V ---------------------------
// For s >= 9 the selected Vt row is the eigenvector of G's smallest eigenvalue.  The same
// cyclic Jacobi sweeps run on the upper triangle only (no V: 45 instead of 162 doubles live,
// so the kernel keeps several waves per SIMD), giving lambda_min to ~eps*trace(G); then two
// steps of inverse iteration with (G - mu I), mu = lambda_min - 8 eps trace(G), factored as
// L D L^T (symmetric positive definite by construction; Cholesky-type factorizations of SPD
// matrices are backward stable without pivoting).  The vector agrees with the rotation-
// accumulated one to O(eps * trace / gap) -- the accuracy either has -- and its sign is
// arbitrary, as the reference's is (E and -E decompose to the same R, T).
ERP_HD ERP_INLINE constexpr int ut9(int i, int j) {
    return i <= j ? i * 9 - i * (i - 1) / 2 + (j - i) : j * 9 - j * (j - 1) / 2 + (i - j);
}

// g36[k * stride + h]: the 36 distinct Gram values (base uniform across a wave, h the lane
// part, so the device loads use a scalar base and a 32-bit lane offset)
ERP_HD ERP_INLINE void gram36_to_ut(const double* g36, int stride, int h, double* S) {
#pragma unroll
    for (int a = 0; a < 9; a++)
#pragma unroll
        for (int b = a; b < 9; b++) {
            const int i = a / 3, j = a % 3, k = b / 3, l = b % 3;
            S[ut9(a, b)] = g36[(6 * sym3(i, k) + sym3(j, l)) * stride + h];
        }
}

ERP_HD inline void gram_min_eigvec9_jacobi(const double* g36, int stride, int h, double* e) {
    double S[45];
    gram36_to_ut(g36, stride, h, S);
    double tr = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) tr += S[ut9(i, i)];
    const double eps = kDblEps * 10;
    const double floor_abs = 4 * kDblEps * tr;
    for (int sweep = 0; sweep < 40; sweep++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < 8; i++) {
#pragma unroll
            for (int j = i + 1; j < 9; j++) {
                const double a = S[ut9(i, i)], b = S[ut9(j, j)], p = S[ut9(i, j)];
                const double ap = fabs(p);
                if (ap <= eps * sqrt(fabs(a * b)) || ap <= floor_abs) continue;
                const double p2 = 2 * p;
                const double beta = a - b, gamma = hypot(p2, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p2 / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p2 / (gamma * c * 2);
                }
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    if (k == i || k == j) continue;
                    const double gik = S[ut9(i, k)], gjk = S[ut9(j, k)];
                    S[ut9(i, k)] = c * gik + s * gjk;
                    S[ut9(j, k)] = -s * gik + c * gjk;
                }
                const double cs2p = 2 * c * s * p;
                S[ut9(i, i)] = c * c * a + cs2p + s * s * b;
                S[ut9(j, j)] = s * s * a - cs2p + c * c * b;
                S[ut9(i, j)] = 0;
                changed = true;
            }
        }
        if (!changed) break;
    }
    double lmin = S[0];
#pragma unroll
    for (int i = 1; i < 9; i++) lmin = fmin(lmin, S[ut9(i, i)]);
    const double tiny = kDblEps * (tr > 0 ? tr : 1.0);
    const double mu = lmin - 8 * tiny;
    // L D L^T of B = G - mu I, in place (L below the diagonal, stored at ut9(j, i), D on it).
    // G is read again from memory, not kept live through the sweeps: the barrier stops the
    // compiler from reusing the first loads (72 VGPRs of occupancy).
    __asm__ volatile("" ::: "memory");
    gram36_to_ut(g36, stride, h, S);
#pragma unroll
    for (int i = 0; i < 9; i++) S[ut9(i, i)] -= mu;
#pragma unroll
    for (int j = 0; j < 9; j++) {
        double d = S[ut9(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) d -= S[ut9(k, j)] * S[ut9(k, j)] * S[ut9(k, k)];
        d = d > tiny * 1e-3 ? d : tiny * 1e-3;  // rounding can only touch the last pivots
        S[ut9(j, j)] = d;
        const double inv = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < 9; i++) {
            double v = S[ut9(j, i)];
#pragma unroll
            for (int k = 0; k < j; k++) v -= S[ut9(k, i)] * S[ut9(k, j)] * S[ut9(k, k)];
            S[ut9(j, i)] = v * inv;  // L[i][j]
        }
    }
    double x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) x[i] = 1.0;
#pragma unroll
    for (int it = 0; it < 2; it++) {
#pragma unroll
        for (int i = 0; i < 9; i++)  // L y = x
#pragma unroll
            for (int k = 0; k < i; k++) x[i] -= S[ut9(k, i)] * x[k];
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] /= S[ut9(i, i)];
#pragma unroll
        for (int i = 8; i >= 0; i--)  // L^T x = z
#pragma unroll
            for (int k = i + 1; k < 9; k++) x[i] -= S[ut9(i, k)] * x[k];
        double nrm = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) nrm += x[i] * x[i];
        const double inv = 1.0 / sqrt(nrm);
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] *= inv;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) e[i] = x[i];
}

// L D L^T of B = G - mu I from the 36 Gram values, in place in S (L below the diagonal, stored
// at ut9(j, i); D on the diagonal, clamped at floor_d) and 1/D in dinv (the division the
// factorisation makes anyway: the solves only multiply by it)
ERP_HD ERP_INLINE void gram_ldlt9(const double* g36, int stride, int h, double mu, double floor_d,
                                  double* S, double* dinv) {
    gram36_to_ut(g36, stride, h, S);
#pragma unroll
    for (int i = 0; i < 9; i++) S[ut9(i, i)] -= mu;
#pragma unroll
    for (int j = 0; j < 9; j++) {
        double d = S[ut9(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) d -= S[ut9(k, j)] * S[ut9(k, j)] * S[ut9(k, k)];
        d = d > floor_d ? d : floor_d;
        S[ut9(j, j)] = d;
        const double inv = 1.0 / d;
        dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < 9; i++) {
            double v = S[ut9(j, i)];
#pragma unroll
            for (int k = 0; k < j; k++) v -= S[ut9(k, i)] * S[ut9(k, j)] * S[ut9(k, k)];
            S[ut9(j, i)] = v * inv;  // L[i][j]
        }
    }
}

// s >= 9: the eigenvector of G's smallest eigenvalue by inverse iteration on G itself (shift
// mu = -16 eps tr(G): G - mu I is positive definite, so L D L^T needs no pivoting).  The
// eight-point Grams have lambda_1 / lambda_2 ~ 1e-5 (every sampled correspondence nearly
// satisfies the same epipolar constraint), so each step gains ~5 digits: the loop stops one
// step after the iterate moves by < 1e-12 and the vector is then at rounding level.  A lane
// whose iterate has not settled after kInvIt steps (near-degenerate lambda_1 ~ lambda_2) takes
// the Jacobi path (eigenvalue shift + inverse iteration, gram_min_eigvec9_jacobi).
// The inverse-iteration part alone (the device kernel runs the Jacobi fallback in a second,
// rarely busy kernel so that its registers do not size the common one): false = not settled.
// The solves multiply by 1/D (gram_ldlt9's dinv).
ERP_HD ERP_INLINE bool gram_min_eigvec9_inv(const double* g36, int stride, int h, double* e) {
    constexpr int kInvIt = 10;
    double S[45];
    double tr = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) tr += g36[(6 * sym3(i / 3, i / 3) + sym3(i % 3, i % 3)) * stride + h];
    const double tiny = kDblEps * (tr > 0 ? tr : 1.0);
    double dinv[9];
    gram_ldlt9(g36, stride, h, -16 * tiny, tiny * 1e-3, S, dinv);
    double x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) x[i] = 1.0 / 3.0;
    int settled = -1;  // step at which the iterate stopped moving
    for (int it = 0; it < kInvIt; it++) {
        double y[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {  // L y = x
            double v = x[i];
#pragma unroll
            for (int k = 0; k < i; k++) v -= S[ut9(k, i)] * y[k];
            y[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 9; i++) y[i] *= dinv[i];
#pragma unroll
        for (int i = 8; i >= 0; i--)  // L^T z = y
#pragma unroll
            for (int k = i + 1; k < 9; k++) y[i] -= S[ut9(i, k)] * y[k];
        double nrm = 0, dot = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            nrm += y[i] * y[i];
            dot += y[i] * x[i];
        }
        const double inv = (dot < 0 ? -1.0 : 1.0) / sqrt(nrm);  // keep the sign: no flip-flop
        double dlt = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const double v = y[i] * inv;
            dlt = fmax(dlt, fabs(v - x[i]));
            x[i] = v;
        }
        if (settled >= 0) break;     // one more step after settling
        if (dlt < 1e-12) settled = it;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) e[i] = x[i];
    return settled >= 0;
}

ERP_HD inline void gram_min_eigvec9(const double* g36, int stride, int h, double* e) {
    constexpr int kInvIt = 10;
    double S[45];
    double tr = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) tr += g36[(6 * sym3(i / 3, i / 3) + sym3(i % 3, i % 3)) * stride + h];
    const double tiny = kDblEps * (tr > 0 ? tr : 1.0);
    double dinv[9];
    gram_ldlt9(g36, stride, h, -16 * tiny, tiny * 1e-3, S, dinv);
    double x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) x[i] = 1.0 / 3.0;
    int settled = -1;  // step at which the iterate stopped moving
    for (int it = 0; it < kInvIt; it++) {
        double y[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {  // L y = x
            double v = x[i];
#pragma unroll
            for (int k = 0; k < i; k++) v -= S[ut9(k, i)] * y[k];
            y[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 9; i++) y[i] *= dinv[i];
#pragma unroll
        for (int i = 8; i >= 0; i--)  // L^T z = y
#pragma unroll
            for (int k = i + 1; k < 9; k++) y[i] -= S[ut9(i, k)] * y[k];
        double nrm = 0, dot = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            nrm += y[i] * y[i];
            dot += y[i] * x[i];
        }
        const double inv = (dot < 0 ? -1.0 : 1.0) / sqrt(nrm);  // keep the sign: no flip-flop
        double dlt = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const double v = y[i] * inv;
            dlt = fmax(dlt, fabs(v - x[i]));
            x[i] = v;
        }
        if (settled >= 0) break;     // one more step after settling
        if (dlt < 1e-12) settled = it;
    }
    if (settled < 0) {
        gram_min_eigvec9_jacobi(g36, stride, h, e);
        return;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) e[i] = x[i];
}

// the selected Vt row for any s: rotation-accumulated Jacobi for the thin case (s < 9,
// where the row is not the smallest eigenvector), the V-free path otherwise
ERP_HD inline void gram_select_vec(const double* g36, int32_t s, double* e) {
    if (s >= 9) {
        gram_min_eigvec9(g36, 1, 0, e);
    } else {
        double G[81];
        gram36_to_full(g36, G);
        gram_jacobi9(G, s, e);
    }
}

}  // namespace erp
