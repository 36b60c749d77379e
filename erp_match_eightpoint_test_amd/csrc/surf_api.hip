// surf_api.hip -- C ABI of the SURF detector + descriptor (include/erp_match.h, "SURF"):
// the host side builds the Fast-Hessian layer table (resizeHaarPattern per layer, the
// orientation disc and the Gaussian weights, as oracle/erp_surf.c restates OpenCV 3.4's
// surf.cpp) once per (W, H, params), sizes the context's scratch and launches surf.hip.
#include <hip/hip_runtime.h>

#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/erp_match.h"
#include "erp_surf.hpp"

int32_t erp_ctx_device_internal(erp_ctx* ctx);
void* erp_ctx_scratch_internal(erp_ctx* ctx, int which, size_t bytes);
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
uint64_t* erp_ctx_surf_key_internal(erp_ctx* ctx);

namespace {

const int kDx[3][5] = {{0, 2, 3, 7, 1}, {3, 2, 6, 7, -2}, {6, 2, 9, 7, 1}};
const int kDy[3][5] = {{2, 0, 7, 3, 1}, {2, 3, 7, 6, -2}, {2, 6, 7, 9, 1}};
const int kDxy[4][5] = {{1, 1, 4, 4, 1}, {5, 1, 8, 4, -1}, {1, 5, 4, 8, -1}, {5, 5, 8, 8, 1}};

int cv_round(double v) { return (int)rint(v); }

// resizeHaarPattern (OpenCV surf.cpp, restated in oracle/erp_surf.c)
void resize_haar(const int src[][5], erp::SurfHF* dst, int n, int oldSize, int newSize, int ws,
                 int (*box)[4]) {
    const float ratio = (float)newSize / oldSize;
    for (int k = 0; k < n; k++) {
        const int dx1 = cv_round(ratio * src[k][0]), dy1 = cv_round(ratio * src[k][1]);
        const int dx2 = cv_round(ratio * src[k][2]), dy2 = cv_round(ratio * src[k][3]);
        box[k][0] = dx1;
        box[k][1] = dy1;
        box[k][2] = dx2;
        box[k][3] = dy2;
        dst[k].p0 = dy1 * ws + dx1;
        dst[k].p1 = dy2 * ws + dx1;
        dst[k].p2 = dy1 * ws + dx2;
        dst[k].p3 = dy2 * ws + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

// getGaussianKernel(n, sigma, CV_32F)
void gaussian(int n, double sigma, float* cf) {
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        cf[i] = (float)exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
}

}  // namespace

extern "C" {

void erp_surf_params_default(erp_surf_params* p) {
    if (!p) return;
    p->hessian_threshold = 100;
    p->n_octaves = 4;
    p->n_octave_layers = 3;
    p->extended = 0;
    p->upright = 0;
}

erp_status erp_surf_detect_compute_dev(erp_ctx* ctx, const uint8_t* d_images, int32_t n_images,
                                       int32_t W, int32_t H, int32_t channels,
                                       const erp_surf_params* prm, int32_t max_kp,
                                       erp_keypoint* d_kp, float* d_desc, int32_t* d_count,
                                       void* stream) {
    if (!ctx || !prm || n_images < 0 || W < 1 || H < 1 || (channels != 1 && channels != 3) ||
        max_kp < 1 || prm->extended != 0 || prm->upright != 0 || prm->n_octaves < 1 ||
        prm->n_octaves > 8 || prm->n_octave_layers < 1 || prm->n_octave_layers > 8 ||
        (int64_t)(W + 1) * (H + 1) * 255 >= ((int64_t)1 << 31))  // CV_32S integral image
        return ERP_INVALID_ARG;
    if (n_images == 0) return ERP_OK;
    if (!d_images || !d_kp || !d_desc || !d_count) return ERP_INVALID_ARG;
    if (hipSetDevice(erp_ctx_device_internal(ctx)) != hipSuccess) return ERP_HIP_ERROR;
    hipStream_t st = (hipStream_t)stream;
    CtxCallGuard call(ctx, st);
    const int nO = prm->n_octaves, nL = prm->n_octave_layers, nT = (nL + 2) * nO;
    // layer table (host)
    std::vector<erp::SurfLayer> layers(nT);
    std::vector<int> mid;
    erp::SurfPlan plan{};
    size_t off = 0;
    int max_samples = 0, max_mid = 0;
    for (int o = 0, li = 0; o < nO; o++)
        for (int l = 0; l < nL + 2; l++, li++) {
            erp::SurfLayer& L = layers[li];
            memset(&L, 0, sizeof(L));
            L.size = (9 + 6 * l) << o;
            L.step = 1 << o;
            L.rows = H / L.step;
            L.cols = W / L.step;
            L.octave = o;
            L.off = off;
            off += (size_t)L.rows * L.cols;
            if (L.size <= H && L.size <= W) {
                resize_haar(kDx, L.dx, 3, 9, L.size, W + 1, L.box);
                resize_haar(kDy, L.dy, 3, 9, L.size, W + 1, L.box + 3);
                resize_haar(kDxy, L.dxy, 4, 9, L.size, W + 1, L.box + 6);
                L.samples_i = 1 + (H - L.size) / L.step;
                L.samples_j = 1 + (W - L.size) / L.step;
                L.margin = (L.size / 2) / L.step;
                max_samples = std::max(max_samples, L.samples_i * L.samples_j);
            }
            if (l >= 1 && l <= nL) {
                mid.push_back(li);
                max_mid = std::max(max_mid, L.rows * L.cols);
            }
        }
    // largest rotated window: keypoint sizes of a fitting middle layer grow by < one layer
    // step (6 << o) in interpolateKeypoint; win = (int)(21 * size * 1.2 / 9)
    int max_win = 1;
    for (int li : mid) {
        const erp::SurfLayer& L = layers[li];
        if (L.size > H || L.size > W) continue;
        const float sz = (float)(L.size + (6 << L.octave) + 1);
        max_win = std::max(max_win, (int)(21.0f * (sz * 1.2f / 9.0f)) + 1);
    }
    // block runs (256 threads each): samples of the layers of octaves >= 1, extrema cells of
    // the middle layers (findMaximaInLayer's margin from the layer above)
    // octave 0 takes the LDS-tiled Hessian pass (step 1); octave 1 through the same kernel at
    // step 2 measured slower than the gather kernel (0.79 vs 0.62 ms for 8 bands: one sample
    // row per thread and layer leaves 40 LDS address adds + the per-layer box setup per
    // sample), so octaves >= 1 take surf_hessian_hi_kernel
    plan.n_tiled = 1;
    int spre = 0, cpre = 0;
    for (int li = 0; li < nT; li++) {
        erp::SurfLayer& L = layers[li];
        if (L.octave >= plan.n_tiled) {
            L.sample_pre = spre;
            spre += (std::max(L.samples_i, 0) * std::max(L.samples_j, 0) + 255) / 256;
        }
    }
    for (int li : mid) {
        erp::SurfLayer& L = layers[li];
        const erp::SurfLayer& Lu = layers[li + 1];
        L.cell_pre = cpre;
        L.cells = 0;
        if (Lu.size <= H && Lu.size <= W) {
            L.cell_margin = (Lu.size / 2) / L.step + 1;
            const int nr = L.rows - 2 * L.cell_margin, nc = L.cols - 2 * L.cell_margin;
            if (nr > 0 && nc > 0) {
                L.cells = nr * nc;
                L.cell_cols = nc;
            }
        }
        cpre += (L.cells + 255) / 256;
    }
    plan.n_layers0 = nL + 2;
    plan.max_size0 = 9 + 6 * (nL + 1);
    plan.samples_hi = spre;
    plan.mid_cells = cpre;
    plan.det_per_img = std::max<size_t>(off, 1);
    plan.n_layers = nT;
    plan.n_mid = (int)mid.size();
    plan.max_samples = std::max(max_samples, 1);
    plan.max_mid_cells = std::max(max_mid, 1);
    plan.threshold = (float)prm->hessian_threshold;
    {
        float G_ori[13];
        gaussian(13, 2.5, G_ori);
        int n = 0;
        for (int i = -6; i <= 6; i++)
            for (int j = -6; j <= 6; j++)
                if (i * i + j * j <= 36) {
                    plan.consts.aptx[n] = i;
                    plan.consts.apty[n] = j;
                    plan.consts.aptw[n++] = G_ori[i + 6] * G_ori[j + 6];
                }
        if (n != erp::kSurfNOri) return ERP_INTERNAL;
        gaussian(20, 3.3, plan.consts.gdesc);
    }
    // the table on the device (slot 1), uploaded when (W, H, params) change
    const size_t tbytes = sizeof(erp::SurfLayer) * nT + sizeof(int) * mid.size();
    char* tab = (char*)erp_ctx_scratch_internal(ctx, 1, tbytes);
    if (!tab) return ERP_OUT_OF_MEMORY;
    uint64_t key = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { key = (key ^ v) * 1099511628211ull; };
    mix((uint64_t)W); mix((uint64_t)H); mix((uint64_t)nO); mix((uint64_t)nL);
    mix((uint64_t)(uintptr_t)tab);
    uint64_t* cached = erp_ctx_surf_key_internal(ctx);
    if (*cached != key) {
        std::vector<char> host(tbytes);
        memcpy(host.data(), layers.data(), sizeof(erp::SurfLayer) * nT);
        memcpy(host.data() + sizeof(erp::SurfLayer) * nT, mid.data(), sizeof(int) * mid.size());
        if (hipMemcpyAsync(tab, host.data(), tbytes, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return ERP_HIP_ERROR;
        *cached = key;
    }
    plan.d_layers = (const erp::SurfLayer*)tab;
    plan.d_mid = (const int*)(tab + sizeof(erp::SurfLayer) * nT);
    // scratch
    erp::SurfScratch scr{};
    const size_t n = (size_t)n_images, K = (size_t)max_kp;
    scr.gray = (uint8_t*)erp_ctx_scratch_internal(ctx, 2, channels == 3 ? n * W * H : 16);
    scr.sum = (int32_t*)erp_ctx_scratch_internal(ctx, 3, n * (W + 1) * (H + 1) * 4);
    scr.det = (float*)erp_ctx_scratch_internal(ctx, 4, n * plan.det_per_img * 4);
    scr.raw = (erp_keypoint*)erp_ctx_scratch_internal(ctx, 5, n * K * sizeof(erp_keypoint));
    scr.sorted = (erp_keypoint*)erp_ctx_scratch_internal(ctx, 6, n * K * sizeof(erp_keypoint));
    scr.desc = (float*)erp_ctx_scratch_internal(ctx, 7, n * K * 64 * 4);
    if (!scr.gray || !scr.sum || !scr.det || !scr.raw || !scr.sorted || !scr.desc)
        return ERP_OUT_OF_MEMORY;
    if (erp::launch_surf_detect(d_images, n_images, W, H, channels, plan, scr, max_kp, d_count, st) !=
        hipSuccess)
        return ERP_HIP_ERROR;
    // the raw counts on the host (the descriptor pass is sized by them): one stream sync
    std::vector<int32_t> cnt(n_images);
    if (hipMemcpyAsync(cnt.data(), d_count, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return ERP_HIP_ERROR;
    std::vector<int32_t> kpre(n_images + 1, 0);
    for (int i = 0; i < n_images; i++)  // an overflowed image (count < 0) is not described
        kpre[i + 1] = kpre[i] + std::min(std::max(cnt[i], 0), max_kp);
    const int total = kpre[n_images];
    // chunks of keypoints whose slots fit in 1 GiB
    scr.max_win = max_win;
    scr.slot = (size_t)(erp::kSurfPatch + 3) * max_win;
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(total, 1),
                                                                 ((size_t)1 << 30) / (scr.slot * 4)));
    const int nbands = (max_win + erp::surf_band_rows() - 1) / erp::surf_band_rows();
    scr.pool = (float*)erp_ctx_scratch_internal(ctx, 8, (size_t)chunk * scr.slot * 4);
    scr.jobs = (erp::SurfJob*)erp_ctx_scratch_internal(ctx, 9, (size_t)chunk * erp::surf_job_bytes());
    scr.items = (int2*)erp_ctx_scratch_internal(ctx, 10, (size_t)chunk * nbands * sizeof(int2));
    int32_t* dk = (int32_t*)erp_ctx_scratch_internal(ctx, 11, (n + 1 + 16) * sizeof(int32_t));
    if (!scr.pool || !scr.jobs || !scr.items || !dk) return ERP_OUT_OF_MEMORY;
    scr.nitems = dk + n + 1;
    if (total > 0) {
        if (hipMemcpyAsync(dk, kpre.data(), sizeof(int32_t) * (n + 1), hipMemcpyHostToDevice, st) !=
            hipSuccess)
            return ERP_HIP_ERROR;
        for (int g0 = 0; g0 < total; g0 += chunk)
            if (erp::launch_surf_describe(d_images, n_images, W, H, channels, plan, scr, max_kp, dk, g0,
                                          std::min(chunk, total - g0), st) != hipSuccess)
                return ERP_HIP_ERROR;
    }
    return erp::launch_surf_compact(n_images, scr, max_kp, d_kp, d_desc, d_count, st) == hipSuccess
               ? ERP_OK
               : ERP_HIP_ERROR;
}

}  // extern "C"
