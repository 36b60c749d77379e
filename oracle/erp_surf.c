/*
 * erp_surf.c -- CPU restatement of the SURF detector + descriptor the reference runs on every
 * band (src/feature_matcher.cpp:13-15,26-40: xfeatures2d::SURF::create() defaults,
 * detect() then compute(); called 8x per pair from src/spherical_surf.cpp:96-118).
 * TEST INFRASTRUCTURE ONLY (the parity checker of the HIP SURF in
 * erp_match_eightpoint_test_amd/csrc/surf.hip).
 *
 * OpenCV (3.4 xfeatures2d/src/surf.cpp, imgproc resize INTER_AREA, cvtColor BGR2GRAY,
 * integral, getGaussianKernel, core fastAtan2) is NOT in the container or the reference, so
 * everything below is restated from the published algorithm (Bay et al. 2008) as OpenCV 3.4
 * implements it [OpenCV, recalled]: parity of this oracle with OpenCV is UNPINNED.  The HIP
 * kernels follow this file operation for operation (same integer / float / double order, no
 * FMA contraction), so GPU vs oracle parity is exact for detection and tolerance-level for the
 * descriptor (device sinf/cosf).
 *
 * Defaults: hessianThreshold 100, nOctaves 4, nOctaveLayers 3, extended false (64-D), upright
 * false.
 */
#define _POSIX_C_SOURCE 200809L
#include "erp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ---------------------------------------------------------------- OpenCV helpers */
static int cv_round(double v) { return (int)rint(v); }  /* cvRound: nearest, ties to even */
static int cv_floor(double v) { return (int)floor(v); }
static int cv_ceil(double v) { return (int)ceil(v); }

/* cvtColor(COLOR_BGR2GRAY) on 8-bit: fixed point, 14 bits (0.114, 0.587, 0.299) */
void erpo_gray_bgr(const uint8_t* bgr, int32_t W, int32_t H, uint8_t* gray) {
    size_t i, n = (size_t)W * H;
    for (i = 0; i < n; i++) {
        const uint32_t b = bgr[3 * i], g = bgr[3 * i + 1], r = bgr[3 * i + 2];
        gray[i] = (uint8_t)((b * 1868u + g * 9617u + r * 4899u + (1u << 13)) >> 14);
    }
}

/* integral(img, sum, CV_32S): (H+1) x (W+1), row 0 and column 0 zero */
void erpo_integral(const uint8_t* img, int32_t W, int32_t H, int32_t* sum) {
    const int32_t ws = W + 1;
    int32_t x, y;
    for (x = 0; x <= W; x++) sum[x] = 0;
    for (y = 0; y < H; y++) {
        int32_t s = 0;
        sum[(size_t)(y + 1) * ws] = 0;
        for (x = 0; x < W; x++) {
            s += img[(size_t)y * W + x];
            sum[(size_t)(y + 1) * ws + x + 1] = sum[(size_t)y * ws + x + 1] + s;
        }
    }
}

/* getGaussianKernel(n, sigma, CV_32F) with sigma > 0 */
static void gaussian_kernel(int n, double sigma, float* cf) {
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    int i;
    for (i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        const double t = exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
}

/* fastAtan2 / phase(..., angleInDegrees = true): the 7th-order polynomial of OpenCV 3.4 */
float erpo_fast_atan2(float y, float x) {
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

/* ---------------------------------------------------------------- Haar patterns */
typedef struct { int p0, p1, p2, p3; float w; } surf_hf;

/* resizeHaarPattern: box corners scaled by newSize/oldSize (cvRound), weight / area */
void erpo_surf_resize_haar(const int src[][5], surf_hf* dst, int n, int oldSize, int newSize,
                           int widthStep) {
    const float ratio = (float)newSize / oldSize;
    int k;
    for (k = 0; k < n; k++) {
        const int dx1 = cv_round(ratio * src[k][0]), dy1 = cv_round(ratio * src[k][1]);
        const int dx2 = cv_round(ratio * src[k][2]), dy2 = cv_round(ratio * src[k][3]);
        dst[k].p0 = dy1 * widthStep + dx1;
        dst[k].p1 = dy2 * widthStep + dx1;
        dst[k].p2 = dy1 * widthStep + dx2;
        dst[k].p3 = dy2 * widthStep + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

/* calcHaarPattern: double accumulation of the box sums times their float weights */
static float haar(const int32_t* origin, const surf_hf* f, int n) {
    double d = 0;
    int k;
    for (k = 0; k < n; k++)
        d += (origin[f[k].p0] + origin[f[k].p3] - origin[f[k].p1] - origin[f[k].p2]) * f[k].w;
    return (float)d;
}

static const int kDx[3][5] = {{0, 2, 3, 7, 1}, {3, 2, 6, 7, -2}, {6, 2, 9, 7, 1}};
static const int kDy[3][5] = {{2, 0, 7, 3, 1}, {2, 3, 7, 6, -2}, {2, 6, 7, 9, 1}};
static const int kDxy[4][5] = {{1, 1, 4, 4, 1}, {5, 1, 8, 4, -1}, {1, 5, 4, 8, -1}, {5, 5, 8, 8, 1}};

/* calcLayerDetAndTrace: det = dx*dy - 0.81f*dxy*dxy, trace = dx + dy at every sampleStep-th
 * position whose box fits; stored at (i + margin, j + margin) of the rows/step x cols/step
 * layer (other entries stay 0 here; OpenCV leaves them unset and never reads them) */
static void layer_det_trace(const int32_t* sum, int W, int H, int size, int step, float* det,
                            float* trace) {
    const int ws = W + 1, lc = W / step;
    surf_hf Dx[3], Dy[3], Dxy[4];
    int i, j, samples_i, samples_j, margin;
    if (size > H || size > W) return;
    erpo_surf_resize_haar(kDx, Dx, 3, 9, size, ws);
    erpo_surf_resize_haar(kDy, Dy, 3, 9, size, ws);
    erpo_surf_resize_haar(kDxy, Dxy, 4, 9, size, ws);
    samples_i = 1 + (H - size) / step;
    samples_j = 1 + (W - size) / step;
    margin = (size / 2) / step;
    for (i = 0; i < samples_i; i++) {
        const int32_t* sp = sum + (size_t)i * step * ws;
        for (j = 0; j < samples_j; j++) {
            const float dx = haar(sp + (size_t)j * step, Dx, 3);
            const float dy = haar(sp + (size_t)j * step, Dy, 3);
            const float dxy = haar(sp + (size_t)j * step, Dxy, 4);
            det[(size_t)(i + margin) * lc + j + margin] = dx * dy - 0.81f * dxy * dxy;
            trace[(size_t)(i + margin) * lc + j + margin] = dx + dy;
        }
    }
}

/* interpolateKeypoint: one Newton step on the 3x3x3 det neighbourhood, Matx33f::solve by
 * Cramer's rule with the determinant in double [OpenCV, recalled] */
static int interpolate(const float N9[3][9], int dx, int dy, int ds, erpo_keypoint* kp) {
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
    float d = (float)dd, x0, x1, x2;
    if (d == 0) return 0;
    d = 1 / d;
    x0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) +
              a02 * (b1 * a21 - a11 * b2));
    x1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) +
              a02 * (a10 * b2 - b1 * a20));
    x2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) +
              b0 * (a10 * a21 - a11 * a20));
    if (!((x0 != 0 || x1 != 0 || x2 != 0) && fabsf(x0) <= 1 && fabsf(x1) <= 1 && fabsf(x2) <= 1))
        return 0;
    kp->x += x0 * dx;
    kp->y += x1 * dy;
    kp->size = (float)cv_round(kp->size + x2 * ds);
    return 1;
}

/* KeypointGreater: response, size, octave descending, then y descending?, x ascending */
static int kp_greater(const erpo_keypoint* a, const erpo_keypoint* b) {
    if (a->response > b->response) return 1;
    if (a->response < b->response) return 0;
    if (a->size > b->size) return 1;
    if (a->size < b->size) return 0;
    if (a->octave > b->octave) return 1;
    if (a->octave < b->octave) return 0;
    if (a->y < b->y) return 0;
    if (a->y > b->y) return 1;
    return a->x < b->x;
}
static int kp_cmp(const void* pa, const void* pb) {
    const erpo_keypoint* a = (const erpo_keypoint*)pa;
    const erpo_keypoint* b = (const erpo_keypoint*)pb;
    if (kp_greater(a, b)) return -1;
    if (kp_greater(b, a)) return 1;
    return 0;
}

int32_t erpo_surf_layer_size(int octave, int layer) { return (9 + 6 * layer) << octave; }

/* fastHessianDetector: every middle layer, 3x3x3 strict maxima above the threshold,
 * interpolated; sorted by KeypointGreater (qsort: equal keys unordered, as std::sort) */
int32_t erpo_surf_detect(const int32_t* sum, int32_t W, int32_t H, const erpo_surf_params* prm,
                         erpo_keypoint* kps, int32_t max_kp) {
    const int nO = prm->n_octaves, nL = prm->n_octave_layers, nT = (nL + 2) * nO;
    float** dets = (float**)calloc((size_t)nT, sizeof(float*));
    float** traces = (float**)calloc((size_t)nT, sizeof(float*));
    int* sizes = (int*)calloc((size_t)nT, sizeof(int));
    int* steps = (int*)calloc((size_t)nT, sizeof(int));
    int n = 0, o, l, idx = 0;
    for (o = 0; o < nO; o++) {
        const int step = 1 << o;
        for (l = 0; l < nL + 2; l++, idx++) {
            const size_t cells = (size_t)(H / step) * (W / step);
            dets[idx] = (float*)calloc(cells ? cells : 1, sizeof(float));
            traces[idx] = (float*)calloc(cells ? cells : 1, sizeof(float));
            sizes[idx] = erpo_surf_layer_size(o, l);
            steps[idx] = step;
            layer_det_trace(sum, W, H, sizes[idx], step, dets[idx], traces[idx]);
        }
    }
    for (o = 0; o < nO; o++)
        for (l = 1; l <= nL; l++) {
            const int li = o * (nL + 2) + l, size = sizes[li], step = steps[li];
            const int lr = H / step, lc = W / step;
            const int margin = (sizes[li + 1] / 2) / step + 1;
            const float *d0 = dets[li - 1], *d1 = dets[li], *d2 = dets[li + 1], *tr = traces[li];
            int i, j;
            if (sizes[li + 1] > H || sizes[li + 1] > W) continue;
            for (i = margin; i < lr - margin; i++)
                for (j = margin; j < lc - margin; j++) {
                    const size_t c = (size_t)i * lc + j;
                    const float v = d1[c];
                    float N9[3][9];
                    int a, u, ok = 1;
                    if (!(v > prm->hessian_threshold)) continue;
                    for (a = 0; a < 3; a++) {
                        const float* d = a == 0 ? d0 : a == 1 ? d1 : d2;
                        for (u = 0; u < 9; u++) N9[a][u] = d[c + (size_t)((u / 3 - 1) * lc) + (u % 3 - 1)];
                    }
                    for (a = 0; a < 3 && ok; a++)
                        for (u = 0; u < 9; u++)
                            if (!(a == 1 && u == 4) && !(v > N9[a][u])) { ok = 0; break; }
                    if (!ok) continue;
                    {
                        const int sum_i = step * (i - (size / 2) / step);
                        const int sum_j = step * (j - (size / 2) / step);
                        erpo_keypoint kp;
                        kp.x = sum_j + (size - 1) * 0.5f;
                        kp.y = sum_i + (size - 1) * 0.5f;
                        kp.size = (float)size;
                        kp.angle = -1;
                        kp.response = v;
                        kp.octave = o;
                        kp.class_id = (tr[c] > 0) - (tr[c] < 0);
                        if (interpolate((const float(*)[9])N9, step, step, size - sizes[li - 1], &kp)) {
                            if (n < max_kp) kps[n] = kp;
                            n++;
                        }
                    }
                }
        }
    for (idx = 0; idx < nT; idx++) {
        free(dets[idx]);
        free(traces[idx]);
    }
    free(dets); free(traces); free(sizes); free(steps);
    if (n > max_kp) return -n;
    qsort(kps, (size_t)n, sizeof(erpo_keypoint), kp_cmp);
    return n;
}

/* resize(win, patch 21x21, INTER_AREA) for a square win_size >= 21 window (area weights of
 * computeResizeAreaTab, float accumulation per output row, cvRound) */
void erpo_resize_area(const uint8_t* src, int ss, uint8_t* dst, int ds) {
    const double scale = (double)ss / ds;
    int iscale = (int)(scale + 0.5);  /* saturate_cast<int> */
    int xi[4096], xo[4096], k = 0, dx, dy, sy;
    float xa[4096];
    if (fabs(scale - iscale) < DBL_EPSILON && iscale >= 1) {
        /* integer scale: resizeAreaFast_ -- (sum of the iscale^2 block + area/2) / area */
        const int area = iscale * iscale;
        for (dy = 0; dy < ds; dy++)
            for (dx = 0; dx < ds; dx++) {
                int s = 0, a, b;
                for (a = 0; a < iscale; a++)
                    for (b = 0; b < iscale; b++) s += src[(size_t)(dy * iscale + a) * ss + dx * iscale + b];
                dst[dy * ds + dx] = (uint8_t)((s + area / 2) / area);
            }
        return;
    }
    for (dx = 0; dx < ds; dx++) {  /* computeResizeAreaTab */
        const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
        const double cellWidth = fmin(scale, ss - fsx1);
        int sx1 = cv_ceil(fsx1), sx2 = cv_floor(fsx2), sx;
        sx2 = sx2 < ss - 1 ? sx2 : ss - 1;
        sx1 = sx1 < sx2 ? sx1 : sx2;
        if (sx1 - fsx1 > 1e-3) { xo[k] = dx; xi[k] = sx1 - 1; xa[k++] = (float)((sx1 - fsx1) / cellWidth); }
        for (sx = sx1; sx < sx2; sx++) { xo[k] = dx; xi[k] = sx; xa[k++] = (float)(1.0 / cellWidth); }
        if (fsx2 - sx2 > 1e-3) {
            xo[k] = dx; xi[k] = sx2;
            xa[k++] = (float)(fmin(fmin(fsx2 - sx2, 1.), cellWidth) / cellWidth);
        }
    }
    {
        const int xk = k;
        int yo[4096], yi[4096], yk = 0, j;
        float ya[4096], buf[64], sum[64];
        for (dy = 0; dy < ds; dy++) {  /* the same table for rows */
            const double fsy1 = dy * scale, fsy2 = fsy1 + scale;
            const double cellH = fmin(scale, ss - fsy1);
            int sy1 = cv_ceil(fsy1), sy2 = cv_floor(fsy2);
            sy2 = sy2 < ss - 1 ? sy2 : ss - 1;
            sy1 = sy1 < sy2 ? sy1 : sy2;
            if (sy1 - fsy1 > 1e-3) { yo[yk] = dy; yi[yk] = sy1 - 1; ya[yk++] = (float)((sy1 - fsy1) / cellH); }
            for (sy = sy1; sy < sy2; sy++) { yo[yk] = dy; yi[yk] = sy; ya[yk++] = (float)(1.0 / cellH); }
            if (fsy2 - sy2 > 1e-3) {
                yo[yk] = dy; yi[yk] = sy2;
                ya[yk++] = (float)(fmin(fmin(fsy2 - sy2, 1.), cellH) / cellH);
            }
        }
        /* ResizeArea_Invoker: per source row, buf[dx] = sum alpha * S[sx]; then sum[dx] +=
         * beta * buf[dx]; a finished destination row is written with cvRound */
        for (dx = 0; dx < ds; dx++) sum[dx] = 0;
        {
            int prev_dy = yo[0];
            for (j = 0; j < yk; j++) {
                const int d_y = yo[j];
                const float beta = ya[j];
                const uint8_t* S = src + (size_t)yi[j] * ss;
                for (dx = 0; dx < ds; dx++) buf[dx] = 0;
                for (k = 0; k < xk; k++) buf[xo[k]] += S[xi[k]] * xa[k];
                if (d_y != prev_dy) {
                    for (dx = 0; dx < ds; dx++) {
                        const int v = cv_round(sum[dx]);
                        dst[prev_dy * ds + dx] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
                        sum[dx] = beta * buf[dx];
                    }
                    prev_dy = d_y;
                } else {
                    for (dx = 0; dx < ds; dx++) sum[dx] += beta * buf[dx];
                }
            }
            for (dx = 0; dx < ds; dx++) {
                const int v = cv_round(sum[dx]);
                dst[prev_dy * ds + dx] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
    }
}

/* SURFInvoker: orientation (Haar responses of size 4s on the radius-6s disc, Gaussian 2.5,
 * 60-degree sliding window in 5-degree steps, fastAtan2) and the 64-D descriptor (20s window
 * rotated and bilinearly sampled, INTER_AREA to 21x21, Haar-like gradients of the patch with a
 * 3.3 Gaussian, 4x4 subregions of (sum dx, sum dy, sum |dx|, sum |dy|), unit norm).  Keypoints
 * whose gradient window does not fit get size -1 (deleted by the caller). */
void erpo_surf_describe(const uint8_t* img, const int32_t* sum, int32_t W, int32_t H,
                        erpo_keypoint* kp, float* vec) {
    enum { ORI_RADIUS = 6, ORI_WIN = 60, PATCH_SZ = 20, NOB = (2 * ORI_RADIUS + 1) * (2 * ORI_RADIUS + 1) };
    static const int dx_s[2][5] = {{0, 0, 2, 4, -1}, {2, 0, 4, 4, 1}};
    static const int dy_s[2][5] = {{0, 0, 4, 2, 1}, {0, 2, 4, 4, -1}};
    float G_ori[2 * ORI_RADIUS + 1], G_desc[PATCH_SZ], aptw[NOB], X[NOB], Y[NOB], ang[NOB];
    float DX[PATCH_SZ][PATCH_SZ], DY[PATCH_SZ][PATCH_SZ];
    uint8_t PATCH[PATCH_SZ + 1][PATCH_SZ + 1];
    int aptx[NOB], apty[NOB], nOri = 0, i, j, kk, nangle = 0;
    const int ws = W + 1;
    surf_hf dxt[2], dyt[2];
    const float size = kp->size, cx = kp->x, cy = kp->y;
    const float s = size * 1.2f / 9.0f;
    const int grad = 2 * cv_round(2 * s);
    float descriptor_dir = 360.f - 90.f;
    gaussian_kernel(2 * ORI_RADIUS + 1, 2.5, G_ori);
    gaussian_kernel(PATCH_SZ, 3.3, G_desc);
    for (i = -ORI_RADIUS; i <= ORI_RADIUS; i++)
        for (j = -ORI_RADIUS; j <= ORI_RADIUS; j++)
            if (i * i + j * j <= ORI_RADIUS * ORI_RADIUS) {
                aptx[nOri] = i;  /* apt = Point(i, j): x = i, y = j */
                apty[nOri] = j;
                aptw[nOri++] = G_ori[i + ORI_RADIUS] * G_ori[j + ORI_RADIUS];
            }
    if (H + 1 < grad || W + 1 < grad) { kp->size = -1; return; }
    erpo_surf_resize_haar(dx_s, dxt, 2, 4, grad, ws);
    erpo_surf_resize_haar(dy_s, dyt, 2, 4, grad, ws);
    for (kk = 0; kk < nOri; kk++) {
        const int x = cv_round(cx + aptx[kk] * s - (float)(grad - 1) / 2);
        const int y = cv_round(cy + apty[kk] * s - (float)(grad - 1) / 2);
        const int32_t* ptr;
        if (y < 0 || y >= H + 1 - grad || x < 0 || x >= W + 1 - grad) continue;
        ptr = sum + (size_t)y * ws + x;
        X[nangle] = haar(ptr, dxt, 2) * aptw[kk];
        Y[nangle] = haar(ptr, dyt, 2) * aptw[kk];
        nangle++;
    }
    if (nangle == 0) { kp->size = -1; return; }
    for (j = 0; j < nangle; j++) ang[j] = erpo_fast_atan2(Y[j], X[j]);
    {
        float bestx = 0, besty = 0, dmod = 0;
        for (i = 0; i < 360; i += 5) {
            float sx = 0, sy = 0, m;
            for (j = 0; j < nangle; j++) {
                const int d = abs(cv_round(ang[j]) - i);
                if (d < ORI_WIN / 2 || d > 360 - ORI_WIN / 2) { sx += X[j]; sy += Y[j]; }
            }
            m = sx * sx + sy * sy;
            if (m > dmod) { dmod = m; bestx = sx; besty = sy; }
        }
        descriptor_dir = erpo_fast_atan2(-besty, bestx);
    }
    kp->angle = descriptor_dir;
    if (!vec) return;
    {
        const int win_size = (int)((PATCH_SZ + 1) * s);
        uint8_t* win = (uint8_t*)malloc((size_t)win_size * win_size);
        const float dir = descriptor_dir * (float)(M_PI / 180);
        const float sin_dir = -sinf(dir), cos_dir = cosf(dir);
        const float win_offset = -(float)(win_size - 1) / 2;
        float start_x = cx + win_offset * cos_dir + win_offset * sin_dir;
        float start_y = cy - win_offset * sin_dir + win_offset * cos_dir;
        const int nc1 = W - 1, nr1 = H - 1;
        double square_mag = 0;
        float scale;
        for (i = 0; i < win_size; i++, start_x += sin_dir, start_y += cos_dir) {
            double px = start_x, py = start_y;
            for (j = 0; j < win_size; j++, px += cos_dir, py -= sin_dir) {
                const int ix = cv_floor(px), iy = cv_floor(py);
                if ((unsigned)ix < (unsigned)nc1 && (unsigned)iy < (unsigned)nr1) {
                    const float a = (float)(px - ix), b = (float)(py - iy);
                    const uint8_t* p = img + (size_t)iy * W + ix;
                    win[i * win_size + j] = (uint8_t)cv_round(p[0] * (1.f - a) * (1.f - b) + p[1] * a * (1.f - b) +
                                                              p[W] * (1.f - a) * b + p[W + 1] * a * b);
                } else {
                    int x = cv_round(px), y = cv_round(py);
                    x = x < 0 ? 0 : x > nc1 ? nc1 : x;
                    y = y < 0 ? 0 : y > nr1 ? nr1 : y;
                    win[i * win_size + j] = img[(size_t)y * W + x];
                }
            }
        }
        erpo_resize_area(win, win_size, &PATCH[0][0], PATCH_SZ + 1);
        free(win);
        for (i = 0; i < PATCH_SZ; i++)
            for (j = 0; j < PATCH_SZ; j++) {
                const float dw = G_desc[i] * G_desc[j];
                DX[i][j] = (PATCH[i][j + 1] - PATCH[i][j] + PATCH[i + 1][j + 1] - PATCH[i + 1][j]) * dw;
                DY[i][j] = (PATCH[i + 1][j] - PATCH[i][j] + PATCH[i + 1][j + 1] - PATCH[i][j + 1]) * dw;
            }
        for (kk = 0; kk < 64; kk++) vec[kk] = 0;
        {
            float* v = vec;
            int y, x;
            for (i = 0; i < 4; i++)
                for (j = 0; j < 4; j++) {
                    for (y = i * 5; y < i * 5 + 5; y++)
                        for (x = j * 5; x < j * 5 + 5; x++) {
                            const float tx = DX[y][x], ty = DY[y][x];
                            v[0] += tx; v[1] += ty;
                            v[2] += (float)fabs(tx); v[3] += (float)fabs(ty);
                        }
                    for (kk = 0; kk < 4; kk++) square_mag += v[kk] * v[kk];
                    v += 4;
                }
        }
        scale = (float)(1. / (sqrt(square_mag) + FLT_EPSILON));
        for (kk = 0; kk < 64; kk++) vec[kk] *= scale;
    }
}

/* SURF::detect then SURF::compute on one image (8-bit gray or BGR): keypoints in
 * KeypointGreater order, deleted ones (size <= 0) removed, 64-D descriptors.  Returns the
 * count, or -(needed) when max_kp is too small. */
int32_t erpo_surf(const uint8_t* img, int32_t W, int32_t H, int32_t channels,
                  const erpo_surf_params* prm, erpo_keypoint* kps, float* desc, int32_t max_kp) {
    uint8_t* gray = (uint8_t*)malloc((size_t)W * H);
    int32_t* sum = (int32_t*)malloc((size_t)(W + 1) * (H + 1) * sizeof(int32_t));
    int32_t n, k, j = 0;
    if (channels == 3) erpo_gray_bgr(img, W, H, gray);
    else memcpy(gray, img, (size_t)W * H);
    erpo_integral(gray, W, H, sum);
    n = erpo_surf_detect(sum, W, H, prm, kps, max_kp);
    if (n < 0) { free(gray); free(sum); return n; }
#pragma omp parallel for schedule(dynamic, 16)
    for (k = 0; k < n; k++) erpo_surf_describe(gray, sum, W, H, &kps[k], desc ? desc + (size_t)k * 64 : NULL);
    for (k = 0; k < n; k++)
        if (kps[k].size > 0) {
            if (k > j) {
                kps[j] = kps[k];
                if (desc) memcpy(desc + (size_t)j * 64, desc + (size_t)k * 64, 64 * sizeof(float));
            }
            j++;
        }
    free(gray);
    free(sum);
    return j;
}
