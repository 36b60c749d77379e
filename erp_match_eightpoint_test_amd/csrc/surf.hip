// surf.hip -- SURF detector + 64-D descriptor on gfx950: what the reference
// runs on every band image before the matcher (src/feature_matcher.cpp:13-15,26-40:
// xfeatures2d::SURF::create() defaults, detect() then compute(); 8 calls per pair from
// src/spherical_surf.cpp:96-118).  The algorithm follows OpenCV 3.4's surf.cpp as restated in
// oracle/erp_surf.c (OpenCV itself is absent: parity with it is unpinned); the kernels repeat
// the restatement operation for operation, so detection is bit-exact with the oracle and the
// descriptor differs only where the device sin/cos of the orientation differ in the last ulp.
//
//   surf_gray_kernel        cvtColor(BGR2GRAY), 14-bit fixed point
//   surf_integral_*         integral(CV_32S): row scans, then column scans
//   surf_hessian_kernel     calcLayerDetAndTrace for every (octave, layer): box filters on the
//                           integral image, det = dx dy - 0.81 dxy^2 (fp64 box accumulation)
//   surf_extrema_kernel     findMaximaInLayer: 3x3x3 strict maxima above the threshold,
//                           interpolateKeypoint (Cramer), appended per image
//   surf_sort_kernel        KeypointGreater order by rank counting (deterministic)
//   surf_orient_kernel      one wave per keypoint: orientation (Haar responses on the radius-6s
//                           disc, fastAtan2, 72 sliding 60-degree windows), window row starts
//   surf_window_kernel      per 16-row band of a keypoint's rotated 20s window: pixels generated
//                           on the fly (bilinear), horizontal INTER_AREA pass
//   surf_descriptor_kernel  vertical INTER_AREA pass -> 21 x 21, gradients, 4 x 4 x 4 sums, norm
//   surf_compact_kernel     drop the keypoints marked for deletion, keep the order
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stdint.h>

#include "erp_surf.hpp"
#include "erp_launch.hpp"

namespace erp {

namespace {

__device__ __forceinline__ int cv_roundf(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int cv_roundd(double v) { return (int)__builtin_rint(v); }

__global__ __launch_bounds__(256) void surf_gray_kernel(const uint8_t* __restrict__ src, int ch,
                                                        size_t npix, uint8_t* __restrict__ gray) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += (size_t)gridDim.x * 256) {
        if (ch == 3) {
            const uint32_t b = src[3 * i], g = src[3 * i + 1], r = src[3 * i + 2];
            gray[i] = (uint8_t)((b * 1868u + g * 9617u + r * 4899u + (1u << 13)) >> 14);
        } else {
            gray[i] = src[i];
        }
    }
}

// row prefix sums: sum[img][y+1][x+1] = sum over x' <= x of gray[y][x'] (row 0 / column 0 = 0)
__global__ __launch_bounds__(256) void surf_integral_rows_kernel(const uint8_t* __restrict__ gray,
                                                                 int W, int H,
                                                                 int32_t* __restrict__ sum) {
    __shared__ int32_t ws[4];
    const int y = blockIdx.x, img = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    const uint8_t* g = gray + ((size_t)img * H + y) * W;
    int32_t* out = sum + ((size_t)img * (H + 1) + y + 1) * (W + 1);
    if (tid == 0) out[0] = 0;
    int32_t carry = 0;
    for (int x0 = 0; x0 < W; x0 += 256) {
        const int x = x0 + tid;
        int32_t v = x < W ? (int32_t)g[x] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t t = __shfl_up(v, o, 64);
            if (lane >= o) v += t;
        }
        if (lane == 63) ws[tid >> 6] = v;
        __syncthreads();
        int32_t pre = carry;
        for (int w = 0; w < (tid >> 6); w++) pre += ws[w];
        if (x < W) out[x + 1] = pre + v;
        carry += ws[0] + ws[1] + ws[2] + ws[3];
        __syncthreads();
    }
}

// column prefix sums over the row sums; row 0 = 0.  A block per (64 columns, image) and one wave
// per row segment (kColSeg of them): each lane sums its column's segment, the segment totals are
// scanned in LDS, and each lane rewrites its segment as running sums.  (Until r06 one thread
// walked a whole column: ~700 waves on the chip, each a 672-step chain of dependent
// load -> add -> store round trips, 250 µs per 8 bands of 672 x 5376.)  Integer sums: the
// result does not depend on the order (< 2^31: 255 * 673 * 5377).
constexpr int kColSeg = 16;
__global__ __launch_bounds__(64 * kColSeg) void surf_integral_cols_kernel(
    int W, int H, int32_t* __restrict__ sum) {
    __shared__ int32_t tot[kColSeg][64];
    const int lane = threadIdx.x & 63, seg = threadIdx.x >> 6;
    const int x = blockIdx.x * 64 + lane, img = blockIdx.y;
    const bool live = x <= W;
    int32_t* s = sum + (size_t)img * (H + 1) * (W + 1) + x;
    const int per = (H + kColSeg - 1) / kColSeg;
    const int y0 = 1 + seg * per, y1 = min(H + 1, y0 + per);
    const size_t st = (size_t)(W + 1);
    int32_t t = 0;
    if (live)
#pragma unroll 4
        for (int y = y0; y < y1; y++) t += s[(size_t)y * st];
    tot[seg][lane] = t;
    __syncthreads();
    int32_t acc = 0;
    for (int k = 0; k < seg; k++) acc += tot[k][lane];
    if (!live) return;
    if (seg == 0) s[0] = 0;
    for (int y = y0; y < y1; y++) {
        acc += s[(size_t)y * st];
        s[(size_t)y * st] = acc;
    }
}

// calcHaarPattern: (int box sum) * float weight in float, accumulated in double
__device__ __forceinline__ float haar(const int32_t* __restrict__ o, const SurfHF* f, int n) {
    double d = 0;
    for (int k = 0; k < n; k++) d += (float)(o[f[k].p0] + o[f[k].p3] - o[f[k].p1] - o[f[k].p2]) * f[k].w;
    return (float)d;
}

// octave 0 (step 1, ~80 % of the samples; SurfPlan.n_tiled octaves): one block per
// 64 x (16 / STEP) samples stages the integral image tile they and all nL + 2 filters of the
// octave touch ((16 + max_size) x (64 STEP + max_size) int32, <= 40 KB at step 1) in LDS
// once, one wave per tile row (coalesced).  The tile is stored as STEP x STEP parity planes
// (row % STEP, column % STEP), so the lanes of a wave (consecutive samples) read consecutive
// words of one plane for every box corner: conflict-free at any step.  Same integer / float /
// double operations as calcHaarPattern (surf_hessian_hi_kernel, the oracle).
constexpr int kHTJ = 64;
// A 1-D grid is dealt round-robin over the 8 XCDs; renumber so that XCD x owns the x-th
// contiguous run of tiles (row-major, per image): tiles resident together on one XCD are
// neighbours and re-read each other's halo rows from that XCD's L2, not from HBM.
__device__ __forceinline__ int xcd_tile(int id, int nb) {
    const int xcd = id & 7, local = id >> 3, per = nb >> 3, rem = nb & 7;
    return xcd < rem ? xcd * (per + 1) + local : rem * (per + 1) + (xcd - rem) * per + local;
}
template <int STEP>
__global__ __launch_bounds__(STEP == 1 ? 256 : 512) void surf_hessian_tile_kernel(
    const int32_t* __restrict__ sum, int W, int H, const SurfLayer* __restrict__ layers, int lb,
    int le, int max_size, size_t det_per_img, float* __restrict__ det) {
    extern __shared__ int32_t T[];
    constexpr int IS = 16 / STEP;        // sample rows per block
    constexpr int NW = STEP == 1 ? 4 : 8;  // waves per block
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int TW = kHTJ * STEP + max_size, TH = IS * STEP + max_size;
    const int TWs = (TW + STEP - 1) / STEP, THs = (TH + STEP - 1) / STEP, PL = TWs * THs;
    const int nbx = ((W / STEP) + kHTJ - 1) / kHTJ, nby = ((H / STEP) + IS - 1) / IS;
    const int t = xcd_tile(blockIdx.x, gridDim.x), bx = t % nbx, by = (t / nbx) % nby;
    const int j0 = bx * kHTJ, i0 = by * IS, img = t / (nbx * nby);
    const int32_t* S = sum + (size_t)img * (H + 1) * (W + 1);
    for (int r = wv; r < TH; r += NW) {
        const int gi = i0 * STEP + r;
        int32_t* Tr = T + (r % STEP) * STEP * PL + (r / STEP) * TWs;
        for (int c = lane; c < TW; c += 64) {
            const int gj = j0 * STEP + c;
            Tr[(c % STEP) * PL + c / STEP] = (gi <= H && gj <= W) ? S[(size_t)gi * (W + 1) + gj] : 0;
        }
    }
    __syncthreads();
    const int j = lane, ib = wv;
    float* D = det + (size_t)img * det_per_img;
    for (int l = lb; l < le; l++) {
        const SurfLayer& L = layers[l];
        const int si = L.samples_i, sj = L.samples_j;
        if (si <= 0 || j0 + j >= sj) continue;
        int off[10][4];
        float w[10];
        auto at = [&](int y, int x) { return ((y % STEP) * STEP + x % STEP) * PL + (y / STEP) * TWs + x / STEP; };
#pragma unroll
        for (int b = 0; b < 10; b++) {
            off[b][0] = at(L.box[b][1], L.box[b][0]);  // p0 = (y1, x1)
            off[b][1] = at(L.box[b][3], L.box[b][0]);  // p1 = (y2, x1)
            off[b][2] = at(L.box[b][1], L.box[b][2]);  // p2 = (y1, x2)
            off[b][3] = at(L.box[b][3], L.box[b][2]);  // p3 = (y2, x2)
            w[b] = b < 3 ? L.dx[b].w : b < 6 ? L.dy[b - 3].w : L.dxy[b - 6].w;
        }
#pragma unroll
        for (int q = 0; q < IS / NW; q++) {
            const int ti = ib + NW * q, i = i0 + ti;
            if (i >= si) break;
            const int32_t* o = T + ti * TWs + j;  // sample (ti, j) -> tile (ti STEP, j STEP)
            double hx = 0, hy = 0, hxy = 0;
#pragma unroll
            for (int b = 0; b < 3; b++)
                hx += (float)(o[off[b][0]] + o[off[b][3]] - o[off[b][1]] - o[off[b][2]]) * w[b];
#pragma unroll
            for (int b = 3; b < 6; b++)
                hy += (float)(o[off[b][0]] + o[off[b][3]] - o[off[b][1]] - o[off[b][2]]) * w[b];
#pragma unroll
            for (int b = 6; b < 10; b++)
                hxy += (float)(o[off[b][0]] + o[off[b][3]] - o[off[b][1]] - o[off[b][2]]) * w[b];
            const float dx = (float)hx, dy = (float)hy, dxy = (float)hxy;
            D[L.off + (size_t)(i + L.margin) * L.cols + j0 + j + L.margin] = dx * dy - 0.81f * dxy * dxy;
        }
    }
}

// the remaining octaves: one thread per sample; the layers [l0, nT) own consecutive runs of blocks
// (SurfLayer.sample_pre, in blocks), so the layer is uniform per block and its filter table
// is read by scalar loads (no empty blocks, none of the per-layer grid padding)
__global__ __launch_bounds__(256) void surf_hessian_hi_kernel(const int32_t* __restrict__ sum, int W,
                                                              int H,
                                                              const SurfLayer* __restrict__ layers,
                                                              int l0, int nT,
                                                              size_t det_per_img,
                                                              float* __restrict__ det) {
    const int img = blockIdx.y, b = blockIdx.x;
    int l = l0;
    while (l + 1 < nT && b >= layers[l + 1].sample_pre) l++;
    l = __builtin_amdgcn_readfirstlane(l);
    const SurfLayer& L = layers[l];
    const int r = (b - L.sample_pre) * 256 + (int)threadIdx.x;
    if (r >= L.samples_i * L.samples_j) return;
    const int i = r / L.samples_j, j = r - i * L.samples_j;
    const int32_t* o = sum + (size_t)img * (H + 1) * (W + 1) + (size_t)i * L.step * (W + 1) +
                       (size_t)j * L.step;
    const float dx = haar(o, L.dx, 3);
    const float dy = haar(o, L.dy, 3);
    const float dxy = haar(o, L.dxy, 4);
    det[(size_t)img * det_per_img + L.off + (size_t)(i + L.margin) * L.cols + j + L.margin] =
        dx * dy - 0.81f * dxy * dxy;
}

// interpolateKeypoint (restated in oracle/erp_surf.c)
__device__ bool surf_interpolate(const float (&N9)[3][9], int dx, int dy, int ds, erp_keypoint& kp) {
    const float b0 = -(N9[1][5] - N9[1][3]) / 2, b1 = -(N9[1][7] - N9[1][1]) / 2,
                b2 = -(N9[2][4] - N9[0][4]) / 2;
    const float a00 = N9[1][3] - 2 * N9[1][4] + N9[1][5];
    const float a01 = (N9[1][8] - N9[1][6] - N9[1][2] + N9[1][0]) / 4;
    const float a02 = (N9[2][5] - N9[2][3] - N9[0][5] + N9[0][3]) / 4;
    const float a11 = N9[1][1] - 2 * N9[1][4] + N9[1][7];
    const float a12 = (N9[2][7] - N9[2][1] - N9[0][7] + N9[0][1]) / 4;
    const float a22 = N9[0][4] - 2 * N9[1][4] + N9[2][4];
    const float a10 = a01, a20 = a02, a21 = a12;
    const double dd = (double)a00 * ((double)a11 * a22 - (double)a12 * a21) -
                      (double)a01 * ((double)a10 * a22 - (double)a12 * a20) +
                      (double)a02 * ((double)a10 * a21 - (double)a11 * a20);
    float d = (float)dd;
    if (d == 0) return false;
    d = 1 / d;
    const float x0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) +
                          a02 * (b1 * a21 - a11 * b2));
    const float x1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) +
                          a02 * (a10 * b2 - b1 * a20));
    const float x2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) +
                          b0 * (a10 * a21 - a11 * a20));
    if (!((x0 != 0 || x1 != 0 || x2 != 0) && fabsf(x0) <= 1 && fabsf(x1) <= 1 && fabsf(x2) <= 1))
        return false;
    kp.x += x0 * dx;
    kp.y += x1 * dy;
    kp.size = (float)cv_roundf(kp.size + x2 * ds);
    return true;
}

// findMaximaInLayer over every middle layer: one thread per cell; the middle layers own
// consecutive runs of blocks (SurfLayer.cell_pre, in blocks: layer uniform per block)
__global__ __launch_bounds__(256) void surf_extrema_kernel(
    const int32_t* __restrict__ sum, int W, int H, const SurfLayer* __restrict__ layers,
    const int* __restrict__ mid, int n_mid, size_t det_per_img,
    const float* __restrict__ det, float thr, int max_kp, erp_keypoint* __restrict__ raw,
    int32_t* __restrict__ counts) {
    const int img = blockIdx.y, b = blockIdx.x;
    int m = 0;
    while (m + 1 < n_mid && b >= layers[mid[m + 1]].cell_pre) m++;
    const int li = __builtin_amdgcn_readfirstlane(mid[m]);
    const SurfLayer& L = layers[li];
    const int size = L.size, step = L.step, lc = L.cols;
    const int r = (b - L.cell_pre) * 256 + (int)threadIdx.x;
    if (r >= L.cells) return;
    const int i = L.cell_margin + r / L.cell_cols, j = L.cell_margin + r % L.cell_cols;
    const float* base = det + (size_t)img * det_per_img;
    const size_t c = (size_t)i * lc + j;
    const float v = base[L.off + c];
    if (!(v > thr)) return;
    float N9[3][9];
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int u = 0; u < 9; u++)
            N9[a][u] = base[layers[li - 1 + a].off + c + (size_t)((u / 3 - 1) * lc) + (u % 3 - 1)];
    bool ok = true;
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int u = 0; u < 9; u++)
            if (!(a == 1 && u == 4)) ok = ok && (v > N9[a][u]);
    if (!ok) return;
    const int sum_i = step * (i - (size / 2) / step);
    const int sum_j = step * (j - (size / 2) / step);
    erp_keypoint kp;
    kp.x = sum_j + (size - 1) * 0.5f;
    kp.y = sum_i + (size - 1) * 0.5f;
    kp.size = (float)size;
    kp.angle = -1;
    kp.response = v;
    kp.octave = L.octave;
    {  // trace = dx + dy at the maximum (the layer's sign; recomputed, not stored)
        const int32_t* o = sum + (size_t)img * (H + 1) * (W + 1) + (size_t)(i - L.margin) * step * (W + 1) +
                           (size_t)(j - L.margin) * step;
        const float tr = haar(o, L.dx, 3) + haar(o, L.dy, 3);
        kp.class_id = (tr > 0) - (tr < 0);
    }
    if (!surf_interpolate(N9, step, step, size - layers[li - 1].size, kp)) return;
    const int slot = atomicAdd(&counts[img], 1);
    if (slot < max_kp) raw[(size_t)img * max_kp + slot] = kp;
}

__device__ __forceinline__ bool kp_greater(const erp_keypoint& a, const erp_keypoint& b) {
    if (a.response > b.response) return true;
    if (a.response < b.response) return false;
    if (a.size > b.size) return true;
    if (a.size < b.size) return false;
    if (a.octave > b.octave) return true;
    if (a.octave < b.octave) return false;
    if (a.y < b.y) return false;
    if (a.y > b.y) return true;
    return a.x < b.x;
}

// rank = #keypoints greater + #equal keys earlier in the raw list (those are identical
// keypoints: their relative order changes nothing)
__global__ __launch_bounds__(256) void surf_sort_kernel(const erp_keypoint* __restrict__ raw,
                                                        const int32_t* __restrict__ counts,
                                                        int max_kp, erp_keypoint* __restrict__ out) {
    __shared__ erp_keypoint tile[256];
    const int img = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
    const int n = min(counts[img], max_kp);
    if (blockIdx.x * 256 >= n) return;
    const erp_keypoint* R = raw + (size_t)img * max_kp;
    erp_keypoint me{};
    if (k < n) me = R[k];
    int rank = 0;
    for (int t0 = 0; t0 < n; t0 += 256) {
        __syncthreads();
        if (t0 + threadIdx.x < n) tile[threadIdx.x] = R[t0 + threadIdx.x];
        __syncthreads();
        const int m = min(256, n - t0);
        for (int u = 0; u < m; u++) {
            const erp_keypoint& o = tile[u];
            rank += kp_greater(o, me) || (!kp_greater(me, o) && t0 + u < k);
        }
    }
    if (k < n) out[(size_t)img * max_kp + rank] = me;
}

// ---- descriptor ---------------------------------------------------------------------------
constexpr int kPatch = kSurfPatch, kNOri = kSurfNOri;  // lattice points of the radius-6 disc

__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float s = (float)(180 / M_PI);
    const float p1 = 0.9997878412794807f * s, p3 = -0.3258083974640975f * s;
    const float p5 = 0.1555786518463281f * s, p7 = -0.04432655554792128f * s;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__device__ __forceinline__ void resize_haar4(const int (&src)[2][5], SurfHF* dst, int newSize,
                                             int widthStep) {
    const float ratio = (float)newSize / 4;
    for (int k = 0; k < 2; k++) {
        const int dx1 = cv_roundf(ratio * src[k][0]), dy1 = cv_roundf(ratio * src[k][1]);
        const int dx2 = cv_roundf(ratio * src[k][2]), dy2 = cv_roundf(ratio * src[k][3]);
        dst[k].p0 = dy1 * widthStep + dx1;
        dst[k].p1 = dy2 * widthStep + dx1;
        dst[k].p2 = dy1 * widthStep + dx2;
        dst[k].p3 = dy2 * widthStep + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

// one area-resize table entry range for output index d (computeResizeAreaTab): up to two
// fractional ends and the whole cells between
struct AreaSpan {
    int first, last;        // whole cells [first, last)
    int lo_i, hi_i;         // fractional cells (-1: none)
    float lo_a, hi_a, mid_a;
};
__device__ __forceinline__ AreaSpan area_span(int d, double scale, int ss) {
    const double f1 = d * scale, f2 = f1 + scale;
    const double cw = fmin(scale, ss - f1);
    int s1 = (int)ceil(f1), s2 = (int)floor(f2);
    s2 = min(s2, ss - 1);
    s1 = min(s1, s2);
    AreaSpan a;
    a.lo_i = (s1 - f1 > 1e-3) ? s1 - 1 : -1;
    a.lo_a = (float)((s1 - f1) / cw);
    a.first = s1;
    a.last = s2;
    a.mid_a = (float)(1.0 / cw);
    a.hi_i = (f2 - s2 > 1e-3) ? s2 : -1;
    a.hi_a = (float)(fmin(fmin(f2 - s2, 1.), cw) / cw);
    return a;
}

// The rotated window's sample positions: the reference walks each row with
// px += cos_dir, py -= sin_dir in DOUBLE from a float row start.  When the row starts and
// |cos_dir|, |sin_dir| are 0 or >= 2^-16 and every |coordinate| stays below 2^14, every partial
// sum start + j*c is a multiple of min(ulp(start), ulp(c)) >= 2^-39 below 2^14, i.e. exactly
// representable: the walk never rounds and fma(j, c, start) gives the same double.  Keypoints
// outside that range walk sequentially (rare).
__device__ __forceinline__ bool exact_walk(float v) {
    return v == 0.f || (fabsf(v) >= 0x1p-16f && fabsf(v) < 0x1p13f);
}

// The descriptor in three launches, so that a few large keypoints (window up to ~740^2 pixels)
// do not serialise the whole pass behind one block:
//   surf_orient_kernel   one wave per keypoint: orientation, the window's row starts and its
//                        exact-walk flag into the keypoint's slot, band items (16 window rows)
//                        appended to the work list
//   surf_window_kernel   one block per band item: the horizontal INTER_AREA pass
//                        tmp[dx][sy] = sum over the dx span of win(sy, sx) * alpha, each window
//                        pixel generated on the fly (bilinear, the reference's walk)
//   surf_descriptor_kernel  one block per keypoint: the vertical pass -> the 21 x 21 patch,
//                        gradients, 4 x 4 x 4 sums, norm
// Keypoints are numbered g = 0 .. total-1 over the images (kpre[img] = first g of img); a
// chunk [g0, g0 + n) is described per launch triple; slot g - g0 holds tmp[21][win] then
// stx[win], sty[win] (slot stride = 23 * max_win floats).
constexpr int kBandRows = 16;

__device__ __forceinline__ void kp_of(int g, const int32_t* __restrict__ kpre, int n_images,
                                      int* img, int* k) {
    int i = 0;
    while (i + 1 < n_images && g >= kpre[i + 1]) i++;
    *img = i;
    *k = g - kpre[i];
}

// window pixel (row i, column j): bilinear inside, nearest clamped outside (the reference's
// rotated-window loop); the exact walk = fma(j, c, start) when it never rounds (header above)
__device__ __forceinline__ float win_pixel(const uint8_t* __restrict__ I, int W, int H, float stx,
                                           float sty, int j, float cos_dir, float sin_dir,
                                           bool exact) {
    double px, py;
    if (exact) {
        px = __builtin_fma((double)j, (double)cos_dir, (double)stx);
        py = __builtin_fma(-(double)j, (double)sin_dir, (double)sty);
    } else {
        px = stx;
        py = sty;
        for (int q = 0; q < j; q++) {
            px += cos_dir;
            py -= sin_dir;
        }
    }
    const int nc1 = W - 1, nr1 = H - 1;
    const int ix = (int)floor(px), iy = (int)floor(py);
    if ((unsigned)ix < (unsigned)nc1 && (unsigned)iy < (unsigned)nr1) {
        const float a = (float)(px - ix), b = (float)(py - iy);
        const uint8_t* p = I + (size_t)iy * W + ix;
        return (float)(uint8_t)cv_roundf(p[0] * (1.f - a) * (1.f - b) + p[1] * a * (1.f - b) +
                                         p[W] * (1.f - a) * b + p[W + 1] * a * b);
    }
    int x = cv_roundd(px), y = cv_roundd(py);
    x = x < 0 ? 0 : x > nc1 ? nc1 : x;
    y = y < 0 ? 0 : y > nr1 ? nr1 : y;
    return (float)I[(size_t)y * W + x];
}

__device__ __forceinline__ bool integer_scale(int win, double* scale, int* iscale) {
    *scale = (double)win / (kPatch + 1);
    *iscale = (int)(*scale + 0.5);
    return fabs(*scale - *iscale) < DBL_EPSILON && *iscale >= 1;
}

__global__ __launch_bounds__(64) void surf_orient_kernel(
    const int32_t* __restrict__ sum, int W, int H, int n_images, int max_kp,
    const int32_t* __restrict__ kpre, int g0, int ng, erp_keypoint* __restrict__ kps, SurfConsts K,
    float* __restrict__ pool, size_t slot, int max_win, SurfJob* __restrict__ jobs,
    int2* __restrict__ items, int32_t* __restrict__ nitems) {
    __shared__ float sX[kNOri], sY[kNOri], sA[kNOri];
    __shared__ float sMod[72], sSx[72], sSy[72];
    const int lane = threadIdx.x;
    const int ws = W + 1;
    for (int c = blockIdx.x; c < ng; c += gridDim.x) {
        int img, k;
        kp_of(g0 + c, kpre, n_images, &img, &k);
        erp_keypoint* kpp = kps + (size_t)img * max_kp + k;
        const erp_keypoint kp = *kpp;
        const int32_t* S = sum + (size_t)img * (H + 1) * ws;
        const float s = kp.size * 1.2f / 9.0f;
        const int grad = 2 * cv_roundf(2 * s);
        const int win = (int)((kPatch + 1) * s);
        SurfJob job{0.f, 0.f, 0, 0};
        if (H + 1 < grad || W + 1 < grad || win > max_win) {  // (win > max_win cannot happen)
            if (lane == 0) {
                kpp->size = -1;
                jobs[c] = job;
            }
            continue;
        }
        // orientation samples in disc order, compacted (order kept)
        const int dx_s[2][5] = {{0, 0, 2, 4, -1}, {2, 0, 4, 4, 1}};
        const int dy_s[2][5] = {{0, 0, 4, 2, 1}, {0, 2, 4, 4, -1}};
        SurfHF dxt[2], dyt[2];
        resize_haar4(dx_s, dxt, grad, ws);
        resize_haar4(dy_s, dyt, grad, ws);
        int nangle = 0;
        for (int k0 = 0; k0 < kNOri; k0 += 64) {
            const int kk = k0 + lane;
            bool valid = false;
            float vx = 0, vy = 0;
            if (kk < kNOri) {
                const int x = cv_roundf(kp.x + K.aptx[kk] * s - (float)(grad - 1) / 2);
                const int y = cv_roundf(kp.y + K.apty[kk] * s - (float)(grad - 1) / 2);
                valid = !(y < 0 || y >= H + 1 - grad || x < 0 || x >= W + 1 - grad);
                if (valid) {
                    const int32_t* ptr = S + (size_t)y * ws + x;
                    vx = haar(ptr, dxt, 2) * K.aptw[kk];
                    vy = haar(ptr, dyt, 2) * K.aptw[kk];
                }
            }
            const uint64_t bal = __builtin_amdgcn_ballot_w64(valid);
            if (valid) {
                const int pos = nangle + __builtin_popcountll(bal & ((1ull << lane) - 1ull));
                sX[pos] = vx;
                sY[pos] = vy;
                sA[pos] = fast_atan2(vy, vx);
            }
            nangle += __builtin_popcountll(bal);
        }
        __syncthreads();
        if (nangle == 0) {
            if (lane == 0) {
                kpp->size = -1;
                jobs[c] = job;
            }
            __syncthreads();
            continue;
        }
        // 72 windows of 60 degrees, 5 apart; each summed sequentially over the samples
        for (int w = lane; w < 72; w += 64) {
            const int i = 5 * w;
            float sx = 0, sy = 0;
            for (int j = 0; j < nangle; j++) {
                const int d = abs(cv_roundf(sA[j]) - i);
                if (d < 30 || d > 330) {
                    sx += sX[j];
                    sy += sY[j];
                }
            }
            sMod[w] = sx * sx + sy * sy;
            sSx[w] = sx;
            sSy[w] = sy;
        }
        __syncthreads();
        if (lane == 0) {
            float best = 0, bx = 0, by = 0;  // the first window with a strictly larger modulus
            for (int w = 0; w < 72; w++)
                if (sMod[w] > best) {
                    best = sMod[w];
                    bx = sSx[w];
                    by = sSy[w];
                }
            const float dir_deg = fast_atan2(-by, bx);
            const float dir = dir_deg * (float)(M_PI / 180);
            const float sin_dir = -(float)sin((double)dir), cos_dir = (float)cos((double)dir);
            kpp->angle = dir_deg;
            // row starts: the reference's float recurrence, sequentially
            float* stx = pool + (size_t)c * slot + (size_t)(kPatch + 1) * win;
            float* sty = stx + win;
            const float woff = -(float)(win - 1) / 2;
            float a = kp.x + woff * cos_dir + woff * sin_dir;
            float b = kp.y - woff * sin_dir + woff * cos_dir;
            bool ex = exact_walk(cos_dir) && exact_walk(sin_dir);
            for (int i = 0; i < win; i++, a += sin_dir, b += cos_dir) {
                stx[i] = a;
                sty[i] = b;
                ex = ex && exact_walk(a) && exact_walk(b) &&
                     fabsf(a) + win * fabsf(cos_dir) < 0x1p13f &&
                     fabsf(b) + win * fabsf(sin_dir) < 0x1p13f;
            }
            job.cos_dir = cos_dir;
            job.sin_dir = sin_dir;
            job.win = win;
            job.exact = ex;
            jobs[c] = job;
            const int nb = (win + kBandRows - 1) / kBandRows;
            const int base = atomicAdd(nitems, nb);
            for (int q = 0; q < nb; q++) items[base + q] = make_int2(c, q);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void surf_window_kernel(
    const uint8_t* __restrict__ gray, int W, int H, int n_images, const int32_t* __restrict__ kpre,
    int g0, const float* __restrict__ pool_in, float* __restrict__ pool, size_t slot,
    const SurfJob* __restrict__ jobs, const int2* __restrict__ items,
    const int32_t* __restrict__ nitems) {
    const int tid = threadIdx.x;
    const int n = *nitems;
    for (int it = blockIdx.x; it < n; it += gridDim.x) {
        const int2 item = items[it];
        const int c = item.x, r0 = item.y * kBandRows;
        const SurfJob job = jobs[c];
        const int win = job.win;
        const int rows = min(kBandRows, win - r0);
        int img, k;
        kp_of(g0 + c, kpre, n_images, &img, &k);
        const uint8_t* I = gray + (size_t)img * W * H;
        float* tmp = pool + (size_t)c * slot;
        const float* stx = pool_in + (size_t)c * slot + (size_t)(kPatch + 1) * win;
        const float* sty = stx + win;
        double scale;
        int iscale;
        const bool integ = integer_scale(win, &scale, &iscale);
        for (int o = tid; o < rows * (kPatch + 1); o += 256) {
            const int sy = r0 + o % rows, dx = o / rows;
            const float ax = stx[sy], ay = sty[sy];
            float bsum = 0;
            if (integ) {  // integer sums (exact in float)
                int sacc = 0;
                for (int b = 0; b < iscale; b++)
                    sacc += (int)win_pixel(I, W, H, ax, ay, dx * iscale + b, job.cos_dir, job.sin_dir,
                                           job.exact);
                bsum = (float)sacc;
            } else {
                const AreaSpan xs = area_span(dx, scale, win);
                if (xs.lo_i >= 0)
                    bsum += win_pixel(I, W, H, ax, ay, xs.lo_i, job.cos_dir, job.sin_dir, job.exact) *
                            xs.lo_a;
                for (int sx = xs.first; sx < xs.last; sx++)
                    bsum += win_pixel(I, W, H, ax, ay, sx, job.cos_dir, job.sin_dir, job.exact) *
                            xs.mid_a;
                if (xs.hi_i >= 0)
                    bsum += win_pixel(I, W, H, ax, ay, xs.hi_i, job.cos_dir, job.sin_dir, job.exact) *
                            xs.hi_a;
            }
            tmp[(size_t)dx * win + sy] = bsum;
        }
    }
}

__global__ __launch_bounds__(256) void surf_descriptor_kernel(
    int n_images, int max_kp, const int32_t* __restrict__ kpre, int g0, int ng,
    const float* __restrict__ pool, size_t slot, const SurfJob* __restrict__ jobs,
    float* __restrict__ desc, SurfConsts K) {
    __shared__ uint8_t patch[kPatch + 1][kPatch + 1];
    __shared__ float DX[kPatch][kPatch], DY[kPatch][kPatch];
    __shared__ float vecs[64];
    __shared__ float sNorm;
    const int tid = threadIdx.x;
    for (int c = blockIdx.x; c < ng; c += gridDim.x) {
        const int win = jobs[c].win;
        if (win == 0) continue;  // deleted keypoint (uniform over the block)
        int img, k;
        kp_of(g0 + c, kpre, n_images, &img, &k);
        const float* tmp = pool + (size_t)c * slot;
        double scale;
        int iscale;
        const bool integ = integer_scale(win, &scale, &iscale);
        for (int o = tid; o < (kPatch + 1) * (kPatch + 1); o += 256) {
            const int dy = o / (kPatch + 1), dx = o % (kPatch + 1);
            const float* T = tmp + (size_t)dx * win;
            if (integ) {
                const int area = iscale * iscale;
                int sacc = 0;
                for (int a = 0; a < iscale; a++) sacc += (int)T[dy * iscale + a];
                patch[dy][dx] = (uint8_t)((sacc + area / 2) / area);
            } else {
                const AreaSpan ys = area_span(dy, scale, win);
                float acc = 0;
                if (ys.lo_i >= 0) acc += ys.lo_a * T[ys.lo_i];
                for (int sy = ys.first; sy < ys.last; sy++) acc += ys.mid_a * T[sy];
                if (ys.hi_i >= 0) acc += ys.hi_a * T[ys.hi_i];
                const int v = cv_roundf(acc);
                patch[dy][dx] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
        __syncthreads();
        for (int q = tid; q < kPatch * kPatch; q += 256) {
            const int i = q / kPatch, j = q % kPatch;
            const float dw = K.gdesc[i] * K.gdesc[j];
            DX[i][j] = (patch[i][j + 1] - patch[i][j] + patch[i + 1][j + 1] - patch[i + 1][j]) * dw;
            DY[i][j] = (patch[i + 1][j] - patch[i][j] + patch[i + 1][j + 1] - patch[i][j + 1]) * dw;
        }
        __syncthreads();
        if (tid < 16) {
            const int i = tid >> 2, j = tid & 3;
            float v0 = 0, v1 = 0, v2 = 0, v3 = 0;
            for (int y = i * 5; y < i * 5 + 5; y++)
                for (int x = j * 5; x < j * 5 + 5; x++) {
                    const float tx = DX[y][x], ty = DY[y][x];
                    v0 += tx;
                    v1 += ty;
                    v2 += fabsf(tx);
                    v3 += fabsf(ty);
                }
            vecs[4 * tid] = v0;
            vecs[4 * tid + 1] = v1;
            vecs[4 * tid + 2] = v2;
            vecs[4 * tid + 3] = v3;
        }
        __syncthreads();
        if (tid == 0) {
            double sq = 0;
            for (int q = 0; q < 64; q++) sq += vecs[q] * vecs[q];
            sNorm = (float)(1. / (sqrt(sq) + FLT_EPSILON));
        }
        __syncthreads();
        if (tid < 64) desc[((size_t)img * max_kp + k) * 64 + tid] = vecs[tid] * sNorm;
        __syncthreads();
    }
}

// remove the keypoints marked for deletion (size <= 0), order kept; counts -> final counts
// (or -needed when the raw list overflowed max_kp)
__global__ __launch_bounds__(1024) void surf_compact_kernel(const erp_keypoint* __restrict__ kin,
                                                            const float* __restrict__ din,
                                                            int max_kp, int32_t* __restrict__ counts,
                                                            erp_keypoint* __restrict__ kout,
                                                            float* __restrict__ dout) {
    __shared__ int ws[16];
    const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nraw = counts[img];
    if (nraw > max_kp) {
        __syncthreads();
        if (tid == 0) counts[img] = -nraw;
        return;
    }
    int base = 0;
    for (int k0 = 0; k0 < nraw; k0 += 1024) {
        const int k = k0 + tid;
        const bool keep = k < nraw && kin[(size_t)img * max_kp + k].size > 0;
        int x = keep;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wid] = x;
        __syncthreads();
        int pre = base, tot = 0;
        for (int w = 0; w < 16; w++) {
            if (w < wid) pre += ws[w];
            tot += ws[w];
        }
        if (keep) {
            const int pos = pre + x - 1;
            kout[(size_t)img * max_kp + pos] = kin[(size_t)img * max_kp + k];
            for (int q = 0; q < 64; q++)
                dout[((size_t)img * max_kp + pos) * 64 + q] = din[((size_t)img * max_kp + k) * 64 + q];
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) counts[img] = base;
}

}  // namespace

hipError_t launch_surf_detect(const uint8_t* images, int n_images, int W, int H, int channels,
                              const SurfPlan& plan, const SurfScratch& scr, int max_kp,
                              int32_t* counts, hipStream_t st) {
    const size_t npix = (size_t)n_images * W * H;
    const uint8_t* gray = images;
    if (channels == 3) {
        ERP_LAUNCH(surf_gray_kernel, dim3(2048), dim3(256), 0, st, images, 3, npix, scr.gray);
        gray = scr.gray;
    }
    ERP_LAUNCH(surf_integral_rows_kernel, dim3(H, n_images), dim3(256), 0, st, gray, W, H, scr.sum);
    ERP_LAUNCH(surf_integral_cols_kernel, dim3((W + 1 + 63) / 64, n_images), dim3(64 * kColSeg), 0,
                       st, W, H, scr.sum);
    hipError_t e = hipMemsetAsync(scr.det, 0, plan.det_per_img * n_images * sizeof(float), st);
    if (e != hipSuccess) return e;
    for (int o = 0; o < plan.n_tiled; o++) {
        const int lb = o * plan.n_layers0, le = std::min(lb + plan.n_layers0, plan.n_layers);
        const int ms = plan.max_size0 << o;
        if (o == 0) {
            const size_t lds = sizeof(int32_t) * (kHTJ + ms) * (16 + ms);
            ERP_LAUNCH(surf_hessian_tile_kernel<1>,
                               dim3(((W + kHTJ - 1) / kHTJ) * ((H + 15) / 16) * n_images), dim3(256), lds, st, scr.sum, W, H, plan.d_layers, lb, le, ms, plan.det_per_img,
                               scr.det);
        } else if (W >= 2 && H >= 2) {
            const size_t lds = sizeof(int32_t) * 4 * ((2 * kHTJ + ms + 1) / 2) * ((16 + ms + 1) / 2);
            ERP_LAUNCH(surf_hessian_tile_kernel<2>,
                               dim3(((W / 2 + kHTJ - 1) / kHTJ) * ((H / 2 + 7) / 8) * n_images), dim3(512), lds, st,
                               scr.sum, W, H, plan.d_layers, lb, le, ms, plan.det_per_img, scr.det);
        }
    }
    if (plan.samples_hi > 0)
        ERP_LAUNCH(surf_hessian_hi_kernel, dim3(plan.samples_hi, n_images), dim3(256), 0, st,
                           scr.sum, W, H, plan.d_layers, plan.n_tiled * plan.n_layers0, plan.n_layers,
                           plan.det_per_img, scr.det);
    e = hipMemsetAsync(counts, 0, sizeof(int32_t) * n_images, st);
    if (e != hipSuccess) return e;
    if (plan.mid_cells > 0)
        ERP_LAUNCH(surf_extrema_kernel, dim3(plan.mid_cells, n_images), dim3(256), 0, st,
                           scr.sum, W, H, plan.d_layers, plan.d_mid, plan.n_mid, plan.det_per_img, scr.det, plan.threshold, max_kp, scr.raw, counts);
    ERP_LAUNCH(surf_sort_kernel, dim3((max_kp + 255) / 256, n_images), dim3(256), 0, st, scr.raw,
                       counts, max_kp, scr.sorted);
    return hipGetLastError();
}

hipError_t launch_surf_describe(const uint8_t* images, int n_images, int W, int H, int channels,
                                const SurfPlan& plan, const SurfScratch& scr, int max_kp,
                                const int32_t* d_kpre, int g0, int ng, hipStream_t st) {
    if (ng <= 0) return hipSuccess;
    const uint8_t* gray = channels == 3 ? (const uint8_t*)scr.gray : images;
    hipError_t e = hipMemsetAsync(scr.nitems, 0, sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    ERP_LAUNCH(surf_orient_kernel, dim3(min(ng, 8192)), dim3(64), 0, st, scr.sum, W, H,
                       n_images, max_kp, d_kpre, g0, ng, scr.sorted, plan.consts, scr.pool, scr.slot,
                       scr.max_win, scr.jobs, scr.items, scr.nitems);
    ERP_LAUNCH(surf_window_kernel, dim3(8192), dim3(256), 0, st, gray, W, H, n_images, d_kpre,
                       g0, (const float*)scr.pool, scr.pool, scr.slot, (const SurfJob*)scr.jobs,
                       (const int2*)scr.items, (const int32_t*)scr.nitems);
    ERP_LAUNCH(surf_descriptor_kernel, dim3(min(ng, 4096)), dim3(256), 0, st, n_images, max_kp,
                       d_kpre, g0, ng, (const float*)scr.pool, scr.slot, (const SurfJob*)scr.jobs,
                       scr.desc, plan.consts);
    return hipGetLastError();
}

hipError_t launch_surf_compact(int n_images, const SurfScratch& scr, int max_kp, erp_keypoint* kp_out,
                               float* desc_out, int32_t* counts, hipStream_t st) {
    ERP_LAUNCH(surf_compact_kernel, dim3(n_images), dim3(1024), 0, st, scr.sorted, scr.desc,
                       max_kp, counts, kp_out, desc_out);
    return hipGetLastError();
}

size_t surf_job_bytes() { return sizeof(SurfJob); }
int surf_band_rows() { return kBandRows; }

}  // namespace erp
