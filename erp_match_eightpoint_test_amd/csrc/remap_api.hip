// remap_api.hip -- C ABI of the ERP remaps around the hot path (include/erp_match.h, section
// "ERP remaps"): the band remap + keypoint un-rotation of spherical_surf::do_all and the
// rectification of automatic.cpp, plus the host-side 3x3 geometry they need (eular2rot,
// rot_from_vec, OpenCV's 3x3 inverse), each restating the reference line it cites.
#include <hip/hip_runtime.h>

#include <math.h>
#include <string.h>

#include <algorithm>

#include "../../include/erp_match.h"
#include "erp_device.hpp"
#include "erp_remap.hpp"

int32_t erp_ctx_device_internal(erp_ctx* ctx);  // capi.hip
void* erp_ctx_scratch_internal(erp_ctx* ctx, int which, size_t bytes);  // capi.hip (grow-only)
// capi.hip: the context's call section (lock + stream order after the previous call, whose
// scratch this call reuses; records the end of this call's work on exit)
void* erp_ctx_call_begin_internal(erp_ctx* ctx, hipStream_t st);
void erp_ctx_call_end_internal(void* call);
namespace {
struct CtxCallGuard {
    void* h;
    CtxCallGuard(erp_ctx* c, hipStream_t st) : h(erp_ctx_call_begin_internal(c, st)) {}
    ~CtxCallGuard() { erp_ctx_call_end_internal(h); }
};
}  // namespace

namespace {

// cv::gemm on 3x3 doubles: d[i][j] = (a[i][0] b[0][j] + a[i][1] b[1][j]) + a[i][2] b[2][j]
void gemm33(const double* a, const double* b, double* d) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            t[i * 3 + j] = a[i * 3 + 0] * b[0 * 3 + j] + a[i * 3 + 1] * b[1 * 3 + j] +
                           a[i * 3 + 2] * b[2 * 3 + j];
    memcpy(d, t, sizeof(t));
}

// RAD(pitch) of a float pitch stored into a cv::Vec3f (src/spherical_surf.cpp:26,52):
// M_PI*(x)/180.0 in double, rounded to float, widened back by eular2rot(Vec3d)
double rad_f(float deg) { return (double)(float)(erp::kPi * (double)deg / 180.0); }

void pitch_matrix(float deg, double m[9]) {
    const double th[3] = {0.0, rad_f(deg), 0.0};
    erp_eular2rot(th, m);
}

erp_status set_dev(erp_ctx* ctx) {
    if (!ctx) return ERP_INVALID_ARG;
    return hipSetDevice(erp_ctx_device_internal(ctx)) == hipSuccess ? ERP_OK : ERP_HIP_ERROR;
}

// the boundary list of a launch of up to kMaxRemapJobs jobs of `pixels` output pixels each
bool scratch(erp_ctx* ctx, size_t pixels, erp::RemapScratch* scr) {
    void* p = erp_ctx_scratch_internal(ctx, 0, 16 + pixels * erp::kMaxRemapJobs * 8);
    if (!p) return false;
    scr->count = (uint32_t*)p;
    scr->list = (uint64_t*)((char*)p + 16);
    return true;
}

bool dims_ok(int32_t W, int32_t H) {
    return W > 0 && H > 0 && (int64_t)W * H <= ((int64_t)1 << 31) / 3;
}

}  // namespace

extern "C" {

// src/erp_rotation.cpp:14-40: R = R_x * R_y * R_z (two cv::gemm products)
void erp_eular2rot(const double theta[3], double R[9]) {
    const double Rx[9] = {1, 0, 0, 0, cos(theta[0]), -sin(theta[0]), 0, sin(theta[0]), cos(theta[0])};
    const double Ry[9] = {cos(theta[1]), 0, sin(theta[1]), 0, 1, 0, -sin(theta[1]), 0, cos(theta[1])};
    const double Rz[9] = {cos(theta[2]), -sin(theta[2]), 0, sin(theta[2]), cos(theta[2]), 0, 0, 0, 1};
    double t[9];
    gemm33(Rx, Ry, t);
    gemm33(t, Rz, R);
}

// src/erp_rotation.cpp:43-63
void erp_rot2eular(const double R[9], double e[3]) { erp::rot2eular(R, e); }

// cv::Mat::inv() = invert(DECOMP_LU), whose 3x3 double case is the adjugate over the
// determinant [OpenCV 3.4 lapack.cpp, recalled]:
//   d = m00 (m11 m22 - m12 m21) - m01 (m10 m22 - m12 m20) + m02 (m10 m21 - m11 m20);
//   d = 1/d;  t0 = (m11 m22 - m12 m21) d; t1 = (m02 m21 - m01 m22) d; ...
// Returns 0 (and leaves out untouched) when d == 0.
int32_t erp_inv3(const double m[9], double out[9]) {
#define M(i, j) m[(i) * 3 + (j)]
    double d = M(0, 0) * (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) -
               M(0, 1) * (M(1, 0) * M(2, 2) - M(1, 2) * M(2, 0)) +
               M(0, 2) * (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0));
    if (d == 0.0) return 0;
    d = 1. / d;
    double t[9];
    t[0] = (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d;
    t[1] = (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d;
    t[2] = (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d;
    t[3] = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d;
    t[4] = (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d;
    t[5] = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d;
    t[6] = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d;
    t[7] = (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d;
    t[8] = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d;
#undef M
    memcpy(out, t, sizeof(t));
    return 1;
}

// src/automatic.cpp:50-64: R = I + [v]x + [v]x^2 * (1/1+c), where the integer 1/1 makes the
// factor 1 + c (kept: it is the reference's behaviour); MatExpr evaluates the gemm with its
// scale folded in, then (I + [v]x) + that
void erp_rot_from_vec(const double v1[3], const double v2[3], double R[9]) {
    const double v[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                         v1[0] * v2[1] - v1[1] * v2[0]};
    const double c = v1[0] * v2[0] + v1[1] * v2[1] + v1[2] * v2[2];
    const double vx[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
    double sq[9];
    gemm33(vx, vx, sq);
    const double s = 1 / 1 + c;
    for (int k = 0; k < 9; k++) {
        const double ipv = (k % 4 == 0 ? 1.0 : 0.0) + vx[k];
        R[k] = ipv + sq[k] * s;
    }
}

// src/automatic.cpp:66-79: the matrices rotate_pixel applies inside the two rotate_image
// calls of rectify (each rotate_image inverts its argument again, src/erp_rotation.cpp:103)
erp_status erp_rectify_matrices(const double rot_vec[3], const double t_vec[3], double m_left[9],
                                double m_right[9]) {
    if (!rot_vec || !t_vec || !m_left || !m_right) return ERP_INVALID_ARG;
    const double down[3] = {0, -1, 0};
    double Rl[9], Rl_inv[9], E[9], E_inv[9], Rr[9], Rr_inv[9];
    erp_rot_from_vec(down, t_vec, Rl);
    if (!erp_inv3(Rl, Rl_inv)) return ERP_INVALID_ARG;
    erp_eular2rot(rot_vec, E);
    if (!erp_inv3(E, E_inv)) return ERP_INVALID_ARG;
    gemm33(Rl, E_inv, Rr);
    if (!erp_inv3(Rr, Rr_inv)) return ERP_INVALID_ARG;
    if (!erp_inv3(Rl_inv, m_left) || !erp_inv3(Rr_inv, m_right)) return ERP_INVALID_ARG;
    return ERP_OK;
}

erp_status erp_crop_rotated_image_dev(erp_ctx* ctx, const uint8_t* d_im, int32_t W, int32_t H,
                                      float pitch_deg, uint8_t* d_out, void* stream) {
    if (!d_im || !d_out || !dims_ok(W, H) || H < 4) return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    erp::RemapScratch scr;
    if (!scratch(ctx, (size_t)W * H, &scr)) return ERP_OUT_OF_MEMORY;
    erp::RemapJobs jobs{};
    erp::RemapJob& j = jobs.j[0];
    j.src = d_im;
    j.dst = d_out;
    pitch_matrix(pitch_deg, j.m);
    j.row0 = H * 3 / 8;
    j.rows = H / 4;
    j.mode = erp::kRemapCrop;
    return erp::launch_remap(jobs, 1, H / 4, W, W, H, scr, (hipStream_t)stream) == hipSuccess
               ? ERP_OK : ERP_HIP_ERROR;
}

erp_status erp_spherical_bands_dev(erp_ctx* ctx, const uint8_t* d_ims, int32_t n_images,
                                   int32_t W, int32_t H, uint8_t* d_bands, void* stream) {
    if (n_images < 0 || (n_images > 0 && (!d_ims || !d_bands)) || !dims_ok(W, H) || H < 4)
        return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    erp::RemapScratch scr;
    if (!scratch(ctx, (size_t)W * H, &scr)) return ERP_OUT_OF_MEMORY;
    static const float pitch[4] = {45.f, 0.f, -45.f, -90.f};  // do_all :77-83 (n1 unrotated)
    double pm[4][9];
    for (int b = 0; b < 4; b++)
        if (b != 1) pitch_matrix(pitch[b], pm[b]);
    const size_t img = (size_t)W * H * 3, band = (size_t)(H / 4) * W * 3;
    constexpr int per = erp::kMaxRemapJobs / 4;  // images per launch
    for (int i0 = 0; i0 < n_images; i0 += per) {
        erp::RemapJobs jobs{};
        int n = 0;
        for (int i = i0; i < std::min(n_images, i0 + per); i++)
            for (int b = 0; b < 4; b++, n++) {
                erp::RemapJob& j = jobs.j[n];
                j.src = d_ims + (size_t)i * img;
                j.dst = d_bands + ((size_t)i * 4 + b) * band;
                if (b != 1) memcpy(j.m, pm[b], sizeof(j.m));
                j.row0 = H * 3 / 8;
                j.rows = H / 4;
                j.mode = b == 1 ? erp::kRemapCopy : erp::kRemapCrop;
            }
        if (erp::launch_remap(jobs, n, H / 4, W, W, H, scr, (hipStream_t)stream) != hipSuccess)
            return ERP_HIP_ERROR;
    }
    return ERP_OK;
}

erp_status erp_rotate_keypoints_dev(erp_ctx* ctx, erp_point2f* d_kp, int32_t n, float pitch_deg,
                                    int32_t W, int32_t H, void* stream) {
    if (n < 0 || (n > 0 && !d_kp) || !dims_ok(W, H)) return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    erp::BandKeypointArgs a{};
    for (int b = 0; b < 4; b++) {
        pitch_matrix(pitch_deg, a.m[b]);
        a.end[b] = n;
    }
    a.shift_band = -1;
    a.W = W;
    a.H = H;
    return erp::launch_band_keypoints(d_kp, a, (hipStream_t)stream) == hipSuccess ? ERP_OK
                                                                                   : ERP_HIP_ERROR;
}

erp_status erp_unrotate_band_keypoints_dev(erp_ctx* ctx, erp_point2f* d_kp,
                                           const int32_t counts[4], int32_t W, int32_t H,
                                           void* stream) {
    if (!counts || !dims_ok(W, H)) return ERP_INVALID_ARG;
    int64_t total = 0;
    for (int b = 0; b < 4; b++) {
        if (counts[b] < 0) return ERP_INVALID_ARG;
        total += counts[b];
    }
    if (total > INT32_MAX || (total > 0 && !d_kp)) return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    static const float pitch[4] = {45.f, 0.f, -45.f, -90.f};  // do_all :121-126
    erp::BandKeypointArgs a{};
    int32_t e = 0;
    for (int b = 0; b < 4; b++) {
        if (b != 1) pitch_matrix(pitch[b], a.m[b]);
        e += counts[b];
        a.end[b] = e;
    }
    a.shift_band = 1;
    a.W = W;
    a.H = H;
    return erp::launch_band_keypoints(d_kp, a, (hipStream_t)stream) == hipSuccess ? ERP_OK
                                                                                   : ERP_HIP_ERROR;
}

erp_status erp_rotate_image_dev(erp_ctx* ctx, const uint8_t* d_im, int32_t W, int32_t H,
                                const double rot_mat[9], uint8_t* d_out, void* stream) {
    if (!d_im || !d_out || !rot_mat || !dims_ok(W, H)) return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    erp::RemapScratch scr;
    if (!scratch(ctx, (size_t)W * H, &scr)) return ERP_OUT_OF_MEMORY;
    erp::RemapJobs jobs{};
    erp::RemapJob& j = jobs.j[0];
    if (!erp_inv3(rot_mat, j.m)) return ERP_INVALID_ARG;  // rot_mat.inv(), erp_rotation.cpp:103
    j.src = d_im;
    j.dst = d_out;
    j.row0 = 0;
    j.rows = H;
    j.mode = erp::kRemapFull;
    return erp::launch_remap(jobs, 1, H, W, W, H, scr, (hipStream_t)stream) == hipSuccess
               ? ERP_OK : ERP_HIP_ERROR;
}

erp_status erp_rectify_dev(erp_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int32_t W,
                           int32_t H, const double rot_vec[3], const double t_vec[3],
                           uint8_t* d_left_out, uint8_t* d_right_out, void* stream) {
    if (!d_left || !d_right || !d_left_out || !d_right_out || !dims_ok(W, H))
        return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    erp::RemapScratch scr;
    if (!scratch(ctx, (size_t)W * H, &scr)) return ERP_OUT_OF_MEMORY;
    erp::RemapJobs jobs{};
    s = erp_rectify_matrices(rot_vec, t_vec, jobs.j[0].m, jobs.j[1].m);
    if (s != ERP_OK) return s;
    for (int k = 0; k < 2; k++) {
        erp::RemapJob& j = jobs.j[k];
        j.src = k ? d_right : d_left;
        j.dst = k ? d_right_out : d_left_out;
        j.row0 = 0;
        j.rows = H;
        j.mode = erp::kRemapFull;
    }
    return erp::launch_remap(jobs, 2, H, W, W, H, scr, (hipStream_t)stream) == hipSuccess
               ? ERP_OK : ERP_HIP_ERROR;
}

erp_status erp_vertical_rotate_dev(erp_ctx* ctx, const uint8_t* d_im, int32_t W, int32_t H,
                                   uint8_t* d_out, void* stream) {
    if (!d_im || !d_out || !dims_ok(W, H)) return ERP_INVALID_ARG;
    erp_status s = set_dev(ctx);
    if (s != ERP_OK) return s;
    CtxCallGuard call(ctx, (hipStream_t)stream);
    erp::RemapScratch scr;
    if (!scratch(ctx, (size_t)W * H, &scr)) return ERP_OUT_OF_MEMORY;
    // rot_mat_90deg = eular2rot(Vec3d(RAD(89.999), 0, 0)).inv(); rotate_image inverts it again
    const double th[3] = {erp::kPi * (89.999) / 180.0, 0, 0};
    double R[9], Ri[9];
    erp_eular2rot(th, R);
    erp::RemapJobs jobs{};
    erp::RemapJob& j = jobs.j[0];
    if (!erp_inv3(R, Ri) || !erp_inv3(Ri, j.m)) return ERP_INVALID_ARG;
    j.src = d_im;
    j.dst = d_out;
    j.row0 = 0;
    j.rows = H;
    j.mode = erp::kRemapRot90;
    return erp::launch_remap(jobs, 1, W, H, W, H, scr, (hipStream_t)stream) == hipSuccess
               ? ERP_OK : ERP_HIP_ERROR;
}

}  // extern "C"
