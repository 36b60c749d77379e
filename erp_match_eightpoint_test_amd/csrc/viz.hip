// viz.hip -- the reference's two visual outputs on the device:
//   epipolar_tool (src/epipolar_tool.cpp:7-71 constructor, :74-128 draw_epipole): curves
//     |l^T E p| < 0.002 of up to 7 randomly chosen left keypoints on an ERP canvas, dots at
//     their right keypoints;
//   feature_matcher::draw_match (src/feature_matcher.cpp:61-86): the two grey images overlaid
//     in two channels with a 5-px line per match.
// Both are per-pixel work over an output image: one thread per pixel (the epipolar canvas, the
// composition of the overlay) plus, for the match lines, one block per match rasterising its
// capsule into a per-pixel "last match" buffer with atomicMax of (call epoch << 16 | match)
// stamps (later matches on top, deterministic where the reference's OpenMP loop races; the
// epoch makes the buffer reusable across calls without clearing it).  Compiled with -ffp-contract=off:
// the epipolar value is the reference's double expression in its written order.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/erp_match.h"
#include "erp_launch.hpp"

int32_t erp_ctx_device_internal(erp_ctx* ctx);                          // capi.hip
void* erp_ctx_stamp_buffer_internal(erp_ctx* ctx, size_t bytes, uint32_t* epoch, bool* fresh);
void* erp_ctx_call_begin_internal(erp_ctx* ctx, hipStream_t st);
void erp_ctx_call_end_internal(void* call);
void host_glibc_window(uint32_t seed, uint64_t offset, uint32_t out[31]);  // capi.hip

namespace erp {
namespace {

constexpr int kEpiMaxKeys = 7;        // color_set has 7 entries (src/epipolar_tool.cpp:18-24)
constexpr double kPiD = 3.14159265358979323846;

struct EpiKeys {
    double l[kEpiMaxKeys][3];         // key_point_left_rect (OMAF axes)
    int32_t di[kEpiMaxKeys], dj[kEpiMaxKeys];  // right key dot centres (row, col in [0, W))
    uint8_t color[kEpiMaxKeys][3];
    double e[9];                      // test_E_mat (row-major CV_64F)
    int32_t n;
};

// sequential semantics of the reference's loop (rows, cols, keys) with the per-pixel curve
// write and the per-key 11 x 11 dot write inside: every dot is rewritten at every pixel, so
// the final canvas has the dots on top (last key whose dot covers the pixel), else the last
// key whose curve passes through the pixel, else 0; the last pixel (H-1, W-1) interleaves
// curve k and dot k in key order.  (oracle/erp_viz.c runs the loop literally.)
constexpr int kEpiRows = 8;  // canvas rows per block: the row terms sin / cos(ry) come from LDS

__global__ __launch_bounds__(256) void epipolar_kernel(EpiKeys k, int W, int H,
                                                       uint8_t* __restrict__ out) {
    __shared__ double srow[kEpiRows][2];
    const int j = blockIdx.x * 256 + threadIdx.x, i0 = blockIdx.y * kEpiRows;
    if (threadIdx.x < kEpiRows) {
        const double ry = kPiD * (double(i0 + threadIdx.x) / H);
        srow[threadIdx.x][0] = sin(ry);
        srow[threadIdx.x][1] = cos(ry);
    }
    __syncthreads();
    if (j >= W) return;
    // pixel_rect[i][j] (src/epipolar_tool.cpp:57-68): the column terms once per thread
    const double rx = 2 * kPiD * (double(j) / W);
    const double crx = cos(rx), srx = sin(rx);
    const double* e = k.e;
    for (int r = 0; r < kEpiRows; r++) {
        const int i = i0 + r;
        if (i >= H) break;
        const double sry = srow[r][0];
        const double p0 = -sry * crx, p1 = sry * srx, p2 = srow[r][1];
            // the reference's expression, its three inner sums being the same for every key
        const double s0 = p0 * e[0] + p1 * e[3] + p2 * e[6];
        const double s1 = p0 * e[1] + p1 * e[4] + p2 * e[7];
        const double s2 = p0 * e[2] + p1 * e[5] + p2 * e[8];
        int curve = -1, dot = -1, last = -1;  // last: the final event's key (corner pixel)
        for (int t = 0; t < k.n; t++) {
            const double* l = k.l[t];
            const double result = l[0] * s0 + l[1] * s1 + l[2] * s2;
            if (fabs(result) < 0.002) {
                curve = t;
                last = t;
            }
            // Mat::at<Vec3b>(dot_i, dot_j) addresses data + (dot_i W + dot_j) 3 with no bounds
            // check: a dot past the left/right edge wraps into the neighbouring row, one past
            // the top/bottom leaves the buffer (dropped here).  With the centre normalised to
            // column dj in [0, W) (row di carrying the rest) and W >= 11 the 11 x 11 dot covers
            // (di + dy, dj + dx), wrapping at most one row at either side.
            bool in_dot;
            const int u = j - k.dj[t], v = i - k.di[t];
            if (W >= 11) {
                in_dot = ((unsigned)(v + 5) <= 10u && (unsigned)(u + 5) <= 10u) ||
                         ((unsigned)(v + 4) <= 10u && (unsigned)(u + W + 5) <= 10u) ||
                         ((unsigned)(v + 6) <= 10u && (unsigned)(u - W + 5) <= 10u);
            } else {
                const int64_t d = (int64_t)v * W + u;
                in_dot = false;
                for (int dy = -5; dy <= 5; dy++) {
                    const int64_t dx = d - (int64_t)dy * W;
                    in_dot |= dx >= -5 && dx <= 5;
                }
            }
            if (in_dot) {
                dot = t;
                last = t;
            }
        }
        int c = dot >= 0 ? dot : curve;
        if (i == H - 1 && j == W - 1) c = last;  // the corner: curve k and dot k interleave
        uint8_t* o = out + ((int64_t)i * W + j) * 3;
        o[0] = c >= 0 ? k.color[c][0] : 0;
        o[1] = c >= 0 ? k.color[c][1] : 0;
        o[2] = c >= 0 ? k.color[c][2] : 0;
    }
}

// HSV -> BGR of one 8-bit pixel (cv::cvtColor COLOR_HSV2BGR, hrange 180; OpenCV 3.4
// HSV2RGB_b / HSV2RGB_f [OpenCV, recalled]: float path, saturate_cast<uchar>(x * 255))
__host__ __device__ inline void hsv2bgr(int hh, int ss, int vv, uint8_t bgr[3]) {
    float h = (float)hh, s = ss * (1.f / 255.f), v = vv * (1.f / 255.f);
    float b, g, r;
    if (s == 0) {
        b = g = r = v;
    } else {
        const int sector_data[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        const float hscale = 6.f / 180.f;
        h *= hscale;
        if (h < 0)
            do h += 6; while (h < 0);
        else if (h >= 6)
            do h -= 6; while (h >= 6);
        int sector = (int)floorf(h);
        h -= sector;
        if ((unsigned)sector >= 6u) {
            sector = 0;
            h = 0.f;
        }
        float tab[4];
        tab[0] = v;
        tab[1] = v * (1.f - s);
        tab[2] = v * (1.f - s * h);
        tab[3] = v * (1.f - s * (1.f - h));
        b = tab[sector_data[sector][0]];
        g = tab[sector_data[sector][1]];
        r = tab[sector_data[sector][2]];
    }
    const float f[3] = {b, g, r};
    for (int k = 0; k < 3; k++) {
        const float x = rintf(f[k] * 255.f);  // cvRound: round half to even
        bgr[k] = (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x));
    }
}

// cvRound of a float (lrintf: round half to even)
__device__ inline int round_even(float x) { return (int)rintf(x); }

// one block per match: the capsule of radius 2.5 around the segment between the rounded
// endpoints, walked along its major axis (12 candidate pixels per step cover the capsule's
// cross-section, caps included); a covered pixel takes max(match index)
__global__ __launch_bounds__(256) void match_lines_kernel(const erp_point2f* __restrict__ kl,
                                                          const erp_point2f* __restrict__ kr,
                                                          int m, int W, int H, uint32_t epoch,
                                                          uint32_t* __restrict__ win) {
    const int i = blockIdx.x;
    if (i >= m) return;
    // a non-finite keypoint draws nothing; coordinates are clamped to +-2^20 before the
    // conversion (defined behaviour, no int overflow below), and the walk along the major axis
    // to the canvas (pixels outside it are never written)
    if (!isfinite(kl[i].x) || !isfinite(kl[i].y) || !isfinite(kr[i].x) || !isfinite(kr[i].y))
        return;
    const float kLim = 1048576.f;
    const int ax = round_even(fminf(fmaxf(kl[i].x, -kLim), kLim));
    const int ay = round_even(fminf(fmaxf(kl[i].y, -kLim), kLim));
    const int bx = round_even(fminf(fmaxf(kr[i].x, -kLim), kLim));
    const int by = round_even(fminf(fmaxf(kr[i].y, -kLim), kLim));
    const int dx = bx - ax, dy = by - ay;
    const bool xmaj = abs(dx) >= abs(dy);
    const int ext = xmaj ? W : H;
    const int a0 = max(xmaj ? min(ax, bx) - 3 : min(ay, by) - 3, -3);
    const int a1 = min(xmaj ? max(ax, bx) + 3 : max(ay, by) + 3, ext + 2);
    if (a0 > a1) return;
    const double len2 = (double)dx * dx + (double)dy * dy;
    const int steps = (a1 - a0 + 1) * 12;
    for (int s = threadIdx.x; s < steps; s += 256) {
        const int t = a0 + s / 12, o = s % 12;
        // the line's minor coordinate at major coordinate t (clamped to the segment)
        double c;
        if (xmaj)
            c = dx != 0 ? ay + (double)(min(max(t, min(ax, bx)), max(ax, bx)) - ax) * dy / dx : ay;
        else
            c = dy != 0 ? ax + (double)(min(max(t, min(ay, by)), max(ay, by)) - ay) * dx / dy : ax;
        const int u = (int)floor(c) - 5 + o;
        const int x = xmaj ? t : u, y = xmaj ? u : t;
        if (x < 0 || x >= W || y < 0 || y >= H) continue;
        // distance from the pixel to the segment
        double px = x - ax, py = y - ay;
        double w = len2 > 0 ? (px * dx + py * dy) / len2 : 0.0;
        w = w < 0 ? 0 : (w > 1 ? 1 : w);
        const double ex = px - w * dx, ey = py - w * dy;
        if (ex * ex + ey * ey <= 6.25) atomicMax(&win[(size_t)y * W + x], (epoch << 16) | i);
    }
}

__device__ inline uint8_t grey(uint32_t c0, uint32_t c1, uint32_t c2) {
    return (uint8_t)((c0 * 4899 + c1 * 9617 + c2 * 1868 + (1 << 13)) >> 14);
}

// Scalar(i * (180.0 / match_size), 180, 150) stored into CV_8UC3 (saturate_cast), -> BGR
__device__ inline uint32_t match_colour(uint32_t idx, int m) {
    const double hd = idx * (180.0 / m);
    const int hh = min(255, max(0, (int)rint(hd)));
    uint8_t c[3];
    hsv2bgr(hh, 180, 150, c);
    return c[0] | (uint32_t)c[1] << 8 | (uint32_t)c[2] << 16;
}

// the overlay (cvtColor CV_RGB2GRAY of each BGR input: channel 0 weighted as R; OpenCV's
// fixed point (R 4899 + G 9617 + B 1868 + 2^13) >> 14) with the winning match's colour.  One
// thread per 4 pixels: 12 bytes = 3 aligned dwords of each input and of the output, one dwordx4
// of line stamps (a stamp of an older call's epoch is "no line").
__global__ __launch_bounds__(256) void draw_match_kernel(const uint8_t* __restrict__ left,
                                                         const uint8_t* __restrict__ right,
                                                         const uint32_t* __restrict__ win,
                                                         uint32_t epoch, int m, int64_t npix,
                                                         uint8_t* __restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t q0 = g * 4;
    if (q0 >= npix) return;
    if (q0 + 4 <= npix) {
        const uint32_t* a = (const uint32_t*)(left + q0 * 3);
        const uint32_t* b = (const uint32_t*)(right + q0 * 3);
        const uint32_t av[3] = {a[0], a[1], a[2]}, bv[3] = {b[0], b[1], b[2]};
        const uint4 w = *(const uint4*)(win + q0);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        uint32_t ov[3] = {0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            auto byte = [&](const uint32_t* v, int o) { return (v[o >> 2] >> ((o & 3) * 8)) & 255u; };
            uint32_t px;
            if ((ws[k] >> 16) == epoch) {
                px = match_colour(ws[k] & 0xFFFFu, m);
            } else {
                px = grey(byte(av, 3 * k), byte(av, 3 * k + 1), byte(av, 3 * k + 2)) |
                     (uint32_t)grey(byte(bv, 3 * k), byte(bv, 3 * k + 1), byte(bv, 3 * k + 2)) << 8;
            }
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const int o = 3 * k + c;
                ov[o >> 2] |= ((px >> (8 * c)) & 255u) << ((o & 3) * 8);
            }
        }
        uint32_t* o = (uint32_t*)(out + q0 * 3);
        o[0] = ov[0];
        o[1] = ov[1];
        o[2] = ov[2];
        return;
    }
    for (int64_t q = q0; q < npix; q++) {  // the last < 4 pixels
        const uint32_t w = win[q];
        uint8_t* o = out + q * 3;
        if ((w >> 16) == epoch) {
            const uint32_t c = match_colour(w & 0xFFFFu, m);
            o[0] = c & 255u;
            o[1] = (c >> 8) & 255u;
            o[2] = c >> 16;
        } else {
            const uint8_t* a = left + q * 3;
            const uint8_t* b = right + q * 3;
            o[0] = grey(a[0], a[1], a[2]);
            o[1] = grey(b[0], b[1], b[2]);
            o[2] = 0;
        }
    }
}

struct CallGuard {
    void* h;
    CallGuard(erp_ctx* c, hipStream_t st) : h(erp_ctx_call_begin_internal(c, st)) {}
    ~CallGuard() { erp_ctx_call_end_internal(h); }
};

}  // namespace
}  // namespace erp

extern "C" {

erp_status erp_random_shuffle_prefix(uint32_t seed, uint64_t offset, int32_t m, int32_t n,
                                     int32_t* h_idx) {
    if (m < 1 || n < 0 || n > m || (n > 0 && !h_idx)) return ERP_INVALID_ARG;
    uint32_t ring[31];
    host_glibc_window(seed, offset, ring);
    int pos = 0;  // ring[pos] = r[n-31]
    auto rnd = [&]() {
        const uint32_t v = ring[(pos + 28) % 31] + ring[pos];  // r[n] = r[n-3] + r[n-31]
        ring[pos] = v;
        pos = (pos + 1) % 31;
        return (int32_t)(v >> 1);
    };
    std::vector<int32_t> idx(m);
    for (int32_t i = 0; i < m; i++) idx[i] = i;
    for (int32_t i = 1; i < m; i++) {
        const int32_t j = (int32_t)((long)rnd() % ((long)i + 1));
        if (i != j) std::swap(idx[i], idx[j]);
    }
    for (int32_t t = 0; t < n; t++) h_idx[t] = idx[t];
    return ERP_OK;
}

erp_status erp_epipolar_draw_dev(erp_ctx* ctx, const erp_point2f* h_key_left,
                                 const erp_point2f* h_key_right, int32_t m, int32_t im_width,
                                 int32_t im_height, int32_t out_width, int32_t out_height,
                                 int32_t n_key, uint32_t seed, uint64_t offset, const double E[9],
                                 uint8_t* d_out, int32_t* h_random_idx, void* stream) {
    using namespace erp;
    if (!ctx || !E || !d_out || m < 1 || n_key < 0 || n_key > kEpiMaxKeys || n_key > m ||
        im_width < 1 || im_height < 1 || out_width < 1 || out_height < 1 || !h_key_left ||
        !h_key_right || (int64_t)out_width * out_height > ((int64_t)1 << 30))
        return ERP_INVALID_ARG;
    if (hipSetDevice(erp_ctx_device_internal(ctx)) != hipSuccess) return ERP_HIP_ERROR;
    const hipStream_t st = (hipStream_t)stream;
    CallGuard call(ctx, st);
    // iota + std::random_shuffle on the glibc rand() stream (src/epipolar_tool.cpp:13-16)
    int32_t idx[kEpiMaxKeys];
    if (n_key > 0) (void)erp_random_shuffle_prefix(seed, offset, m, n_key, idx);
    EpiKeys k{};
    k.n = n_key;
    static const uint8_t colors[kEpiMaxKeys][3] = {{0, 0, 255}, {0, 127, 255}, {0, 255, 255},
                                                   {0, 255, 0}, {255, 0, 0}, {135, 0, 75},
                                                   {211, 0, 148}};
    const double rw = double(out_width) / double(im_width);
    const double rh = double(out_height) / double(im_height);
    for (int t = 0; t < n_key; t++) {
        const erp_point2f L = h_key_left[idx[t]], R = h_key_right[idx[t]];
        // radian.x = 2 M_PI (pt.x / im_width): float / int in float, then double
        const double lon = 2 * kPiD * (L.x / im_width);
        const double lat = kPiD * (L.y / im_height);
        k.l[t][0] = -sin(lat) * cos(lon);
        k.l[t][1] = sin(lat) * sin(lon);
        k.l[t][2] = cos(lat);
        const int di = (int)(R.y * rh);  // int i_idx = pt.y * resize_ratio_h (truncation)
        const int dj = (int)(R.x * rw);
        // the same linear address with the column in [0, W) (epipolar_kernel's dot test)
        const int djn = ((dj % out_width) + out_width) % out_width;
        k.di[t] = di + (dj - djn) / out_width;
        k.dj[t] = djn;
        memcpy(k.color[t], colors[t], 3);
        if (h_random_idx) h_random_idx[t] = idx[t];
    }
    memcpy(k.e, E, sizeof(k.e));
    ERP_LAUNCH_S(epipolar_kernel,
                       dim3((out_width + 255) / 256, (out_height + kEpiRows - 1) / kEpiRows),
                       dim3(256), 0, st, k, out_width, out_height, d_out);
    return hipGetLastError() == hipSuccess ? ERP_OK : ERP_HIP_ERROR;
}

erp_status erp_draw_match_dev(erp_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right,
                              int32_t W, int32_t H, const erp_point2f* d_key_left,
                              const erp_point2f* d_key_right, int32_t m, uint8_t* d_out,
                              void* stream) {
    using namespace erp;
    if (!ctx || !d_left || !d_right || !d_out || W < 1 || H < 1 || m < 0 || m > 65535 ||
        (m > 0 && (!d_key_left || !d_key_right)) || (int64_t)W * H > ((int64_t)1 << 30) ||
        (((uintptr_t)d_left | (uintptr_t)d_right | (uintptr_t)d_out) & 3))
        return ERP_INVALID_ARG;
    if (hipSetDevice(erp_ctx_device_internal(ctx)) != hipSuccess) return ERP_HIP_ERROR;
    const hipStream_t st = (hipStream_t)stream;
    CallGuard call(ctx, st);
    const int64_t npix = (int64_t)W * H;
    uint32_t epoch = 0;
    bool fresh = false;
    auto* win = (uint32_t*)erp_ctx_stamp_buffer_internal(ctx, (size_t)(npix + 4) * 4, &epoch,
                                                         &fresh);
    if (!win) return ERP_OUT_OF_MEMORY;
    if (fresh && hipMemsetAsync(win, 0, (size_t)(npix + 4) * 4, st) != hipSuccess)
        return ERP_HIP_ERROR;
    if (m > 0)
        ERP_LAUNCH_S(match_lines_kernel, dim3(m), dim3(256), 0, st, d_key_left, d_key_right,
                           m, W, H, epoch, win);
    const int64_t groups = (npix + 3) / 4;
    ERP_LAUNCH_S(draw_match_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st,
                       d_left, d_right, win, epoch, m, npix, d_out);
    return hipGetLastError() == hipSuccess ? ERP_OK : ERP_HIP_ERROR;
}

}  // extern "C"
