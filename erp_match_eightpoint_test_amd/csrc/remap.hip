// remap.hip -- gfx950 kernels of the ERP pixel remaps around the hot path:
//
//   spherical_surf::crop_rotated_image  src/spherical_surf.cpp:16-48   remap_kernel (mode CROP)
//   band n1 = im(roi)                   src/spherical_surf.cpp:70-79   remap_kernel (mode COPY)
//   spherical_surf::rotate_keypoint     src/spherical_surf.cpp:50-63,  band_keypoints_kernel
//     + band concat (n0, n1, n2, n3)    :120-144
//   erp_rotation::rotate_image          src/erp_rotation.cpp:94-122    remap_kernel (mode FULL)
//   + cv::rotate(ROTATE_90_CLOCKWISE)   src/automatic.cpp:148-152      remap_kernel (mode ROT90)
//
// Every output pixel is an inverse warp through erp::rotate_pixel (erp_device.hpp, the
// reference's double-precision formula with x86 truncation semantics) followed by a 3-byte
// gather; pixels whose source falls outside the image are NOT written (the reference leaves
// them uninitialised), so callers pre-fill the output.  The work per pixel is ~2 fp64
// transcendentals (acos, atan2) + a 3x3 mat-vec: FP64-VALU bound, not HBM (6 B per pixel).
// The polar sines/cosines depend only on the source row and the azimuth ones only on the
// column, so a block computes them once per row / column into LDS (256 columns x 16 rows per
// block) instead of 4 sincos per pixel.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "erp_device.hpp"
#include "erp_remap.hpp"
#include "erp_launch.hpp"

namespace erp {

namespace {

constexpr int kRmCols = 256;  // columns per block (one per thread)
constexpr int kRmRows = 16;   // rows per block

__device__ __forceinline__ void copy_px(const uint8_t* __restrict__ s, uint8_t* __restrict__ d) {
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
}

// the boundary slow path of one output pixel
__device__ __forceinline__ void remap_pixel_cr(const RemapJob& jb, int r, int c, int W, int H,
                                            int out_cols, const double* m) {
    int32_t oi, oj;
    if (jb.mode == kRemapRot90)
        rotate_pixel_cr(erp_polar(H - 1 - c, H), erp_azimuth(r, W), m, W, H, &oi, &oj);
    else
        rotate_pixel_cr(erp_polar(jb.row0 + r, H), erp_azimuth(c, W), m, W, H, &oi, &oj);
    if (oi >= 0 && oj >= 0 && oi < H && oj < W)
        copy_px(jb.src + ((size_t)oi * W + oj) * 3, jb.dst + ((size_t)r * out_cols + c) * 3);
}

__global__ __launch_bounds__(256) void remap_kernel(const RemapJobs jobs, int W, int H,
                                                    RemapScratch scr) {
    __shared__ double rs[kRmRows], rc[kRmRows];
    const RemapJob& jb = jobs.j[blockIdx.z];
    const int mode = jb.mode;
    const int tid = threadIdx.x;
    // output geometry: ROT90 writes a W-row x H-column image, the others `rows` x W
    const int out_rows = mode == kRemapRot90 ? W : jb.rows;
    const int out_cols = mode == kRemapRot90 ? H : W;
    const int r0 = blockIdx.y * kRmRows;
    const int c = blockIdx.x * kRmCols + tid;
    if (r0 >= out_rows || blockIdx.x * kRmCols >= out_cols) return;  // uniform
    const uint8_t* __restrict__ src = jb.src;
    uint8_t* __restrict__ dst = jb.dst;
    if (mode == kRemapCopy) {  // the n1 band: rows [row0, row0 + rows) as they are
        if (c < out_cols)
            for (int r = r0; r < min(r0 + kRmRows, out_rows); r++)
                copy_px(src + ((size_t)(jb.row0 + r) * W + c) * 3, dst + ((size_t)r * W + c) * 3);
        return;
    }
    double m[9];
#pragma unroll
    for (int k = 0; k < 9; k++) m[k] = jb.m[k];
    // per-thread column angle and per-block row angles.  CROP / FULL: output (r, c) is source
    // pixel (row0 + r, c).  ROT90: output (r, c) is rotate_image's pixel (H - 1 - c, r).
    double sa_t = 0, ca_t = 0, sb_t = 0, cb_t = 0;
    if (c < out_cols) {
        if (mode == kRemapRot90) {
            const double a = erp_polar(H - 1 - c, H);
            sa_t = sin(a);
            ca_t = cos(a);
        } else {
            const double b = erp_azimuth(c, W);
            sb_t = sin(b);
            cb_t = cos(b);
        }
    }
    if (tid < kRmRows) {
        const int r = r0 + tid;
        if (mode == kRemapRot90) {
            const double b = erp_azimuth(r, W);
            rs[tid] = sin(b);
            rc[tid] = cos(b);
        } else {
            const double a = erp_polar(jb.row0 + r, H);
            rs[tid] = sin(a);
            rc[tid] = cos(a);
        }
    }
    __syncthreads();
    if (c >= out_cols) return;
    const int r1 = min(r0 + kRmRows, out_rows);
    for (int r = r0; r < r1; r++) {
        int32_t oi, oj;
        bool slow;
        if (mode == kRemapRot90)
            slow = rotate_pixel_sc(sa_t, ca_t, rs[r - r0], rc[r - r0], m, W, H, &oi, &oj);
        else
            slow = rotate_pixel_sc(rs[r - r0], rc[r - r0], sb_t, cb_t, m, W, H, &oi, &oj);
        if (slow) {  // near a truncation boundary: deferred to the fix-up kernel
            const uint32_t k = atomicAdd(scr.count, 1u);  // (cap = every pixel of the launch)
            scr.list[k] = ((uint64_t)blockIdx.z << 32) | ((uint64_t)r * out_cols + c);
            continue;
        }
        if (oi >= 0 && oj >= 0 && oi < H && oj < W)
            copy_px(src + ((size_t)oi * W + oj) * 3, dst + ((size_t)r * out_cols + c) * 3);
    }
}

// the deferred boundary pixels: correctly rounded transcendentals (grid-stride over the list)
__global__ __launch_bounds__(256) void remap_fixup_kernel(const RemapJobs jobs, int W, int H,
                                                          RemapScratch scr) {
    const uint32_t n = *scr.count;
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint64_t e = scr.list[k];
        const RemapJob& jb = jobs.j[e >> 32];
        const int out_cols = jb.mode == kRemapRot90 ? H : W;
        const uint32_t pix = (uint32_t)e;
        double m[9];
#pragma unroll
        for (int q = 0; q < 9; q++) m[q] = jb.m[q];
        remap_pixel_cr(jb, (int)(pix / out_cols), (int)(pix % out_cols), W, H, out_cols, m);
    }
}

// do_all's keypoint step: band b's keypoints (segments of the concatenated list) back to ERP
// pixels.  Bands 0, 2, 3: rotate_keypoint with the band's pitch matrix (offset_i =
// pt.y + height*3/8 in float, truncated; col = (int)pt.x); band 1: pt.y += height*3/8 (float).
__global__ __launch_bounds__(256) void band_keypoints_kernel(erp_point2f* __restrict__ kp,
                                                             BandKeypointArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.end[3]) return;
    const int band = (i >= a.end[0]) + (i >= a.end[1]) + (i >= a.end[2]);
    erp_point2f p = kp[i];
    const float off = (float)(a.H * 3 / 8);
    if (band == a.shift_band) {
        p.y = p.y + off;
    } else {
        const int32_t oi = trunc_i32_x86f(p.y + off);
        const int32_t ci = trunc_i32_x86f(p.x);
        int32_t r, c;
        rotate_pixel(oi, ci, a.m[band], a.W, a.H, &r, &c);
        p.x = (float)c;
        p.y = (float)r;
    }
    kp[i] = p;
}

}  // namespace

hipError_t launch_remap(const RemapJobs& jobs, int n_jobs, int max_out_rows, int max_out_cols,
                        int W, int H, const RemapScratch& scr, hipStream_t st) {
    hipError_t e = hipMemsetAsync(scr.count, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    dim3 grid((max_out_cols + kRmCols - 1) / kRmCols, (max_out_rows + kRmRows - 1) / kRmRows,
              n_jobs);
    ERP_LAUNCH(remap_kernel, grid, dim3(256), 0, st, jobs, W, H, scr);
    ERP_LAUNCH(remap_fixup_kernel, dim3(256), dim3(256), 0, st, jobs, W, H, scr);
    return hipGetLastError();
}

hipError_t launch_band_keypoints(erp_point2f* d_kp, const BandKeypointArgs& a, hipStream_t st) {
    if (a.end[3] <= 0) return hipSuccess;
    ERP_LAUNCH(band_keypoints_kernel, dim3((a.end[3] + 255) / 256), dim3(256), 0, st, d_kp,
                       a);
    return hipGetLastError();
}

}  // namespace erp
