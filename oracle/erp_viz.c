/* erp_viz.c -- CPU oracle (TEST INFRASTRUCTURE ONLY: never linked into the product) of the two
 * visual outputs of SURVEY.md section 8 row f4, restated literally:
 *   epipolar_tool (src/epipolar_tool.cpp:7-71 constructor, :74-128 draw_epipole): the loop over
 *     rows, cols and keys with the curve write and the 11 x 11 dot write inside it, run
 *     sequentially (the reference runs it under OpenMP, where overlapping writes race); a dot
 *     pixel is written at its linear address like the unchecked Mat::at (past the left/right
 *     edge it wraps into the neighbouring row), and dropped when that leaves the buffer;
 *   feature_matcher::draw_match (src/feature_matcher.cpp:61-86): cvtColor(CV_RGB2GRAY) of the two
 *     BGR images into channels 0 / 1, zeros in channel 2, then per match in order the colour of
 *     HSV(i 180 / m, 180, 150) (cvtColor HSV2BGR, OpenCV 3.4's float path [OpenCV, recalled]) on
 *     every pixel within 2.5 of the segment between the rounded keypoints -- the product's
 *     definition of cv::line(thickness 5), whose rasteriser is not restated (parity with OpenCV
 *     unpinned).
 * Built with -ffp-contract=off like the rest of the oracle. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "erp_oracle.h"

static const double kPi = 3.14159265358979323846;

int32_t erpo_epipolar_draw(const float* key_left, const float* key_right, int32_t m,
                           int32_t im_width, int32_t im_height, int32_t out_w, int32_t out_h,
                           int32_t n_key, uint32_t seed, uint64_t offset, const double E[9],
                           uint8_t* out, int32_t* random_idx, double* min_margin) {
    static const uint8_t colors[7][3] = {{0, 0, 255}, {0, 127, 255}, {0, 255, 255}, {0, 255, 0},
                                         {255, 0, 0}, {135, 0, 75}, {211, 0, 148}};
    if (m < 1 || n_key < 0 || n_key > 7 || n_key > m) return -1;
    erpo_glibc g;
    erpo_glibc_seed(&g, seed);
    erpo_glibc_discard(&g, offset);
    int32_t* a = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
    erpo_random_array(a, m, &g); /* iota + std::random_shuffle (src/epipolar_tool.cpp:13-16) */
    double l[7][3];
    int di[7], dj[7];
    const double rw = (double)out_w / (double)im_width, rh = (double)out_h / (double)im_height;
    for (int t = 0; t < n_key; t++) {
        const float* L = key_left + 2 * (size_t)a[t];
        const float* R = key_right + 2 * (size_t)a[t];
        const double lon = 2 * kPi * (L[0] / im_width);  /* float / int, then double */
        const double lat = kPi * (L[1] / im_height);
        l[t][0] = -sin(lat) * cos(lon);
        l[t][1] = sin(lat) * sin(lon);
        l[t][2] = cos(lat);
        di[t] = (int)(R[1] * rh);
        dj[t] = (int)(R[0] * rw);
        if (random_idx) random_idx[t] = a[t];
    }
    free(a);
    memset(out, 0, (size_t)out_w * out_h * 3);
    double mm = INFINITY;
    for (int i = 0; i < out_h; i++)
        for (int j = 0; j < out_w; j++) {
            const double rx = 2 * kPi * ((double)j / out_w), ry = kPi * ((double)i / out_h);
            const double p0 = -sin(ry) * cos(rx), p1 = sin(ry) * sin(rx), p2 = cos(ry);
            for (int t = 0; t < n_key; t++) {
                const double result = l[t][0] * (p0 * E[0] + p1 * E[3] + p2 * E[6]) +
                                      l[t][1] * (p0 * E[1] + p1 * E[4] + p2 * E[7]) +
                                      l[t][2] * (p0 * E[2] + p1 * E[5] + p2 * E[8]);
                const double d = fabs(fabs(result) - 0.002);
                if (d < mm) mm = d;
                if (fabs(result) < 0.002) memcpy(out + ((size_t)i * out_w + j) * 3, colors[t], 3);
                for (int y = di[t] - 5; y < di[t] + 6; y++)
                    for (int x = dj[t] - 5; x < dj[t] + 6; x++) {
                        /* Mat::at(y, x): data + (y W + x) 3, unchecked */
                        const int64_t lin = (int64_t)y * out_w + x;
                        if (lin >= 0 && lin < (int64_t)out_w * out_h)
                            memcpy(out + (size_t)lin * 3, colors[t], 3);
                    }
            }
        }
    if (min_margin) *min_margin = mm;
    return 0;
}

/* the epipolar value |l^T E p| of pixel (i, j) for key t of the chosen set (certification of
 * pixels within a rounding of the 0.002 threshold) */
double erpo_epipolar_value(const double l[3], const double E[9], int32_t i, int32_t j, int32_t out_w,
                           int32_t out_h) {
    const double rx = 2 * kPi * ((double)j / out_w), ry = kPi * ((double)i / out_h);
    const double p0 = -sin(ry) * cos(rx), p1 = sin(ry) * sin(rx), p2 = cos(ry);
    return l[0] * (p0 * E[0] + p1 * E[3] + p2 * E[6]) + l[1] * (p0 * E[1] + p1 * E[4] + p2 * E[7]) +
           l[2] * (p0 * E[2] + p1 * E[5] + p2 * E[8]);
}

void erpo_hsv2bgr(int h_, int s_, int v_, uint8_t bgr[3]) {
    float h = (float)h_, s = s_ * (1.f / 255.f), v = v_ * (1.f / 255.f);
    float b, g, r;
    if (s == 0) {
        b = g = r = v;
    } else {
        static const int sector_data[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1},
                                              {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        const float hscale = 6.f / 180.f;
        float tab[4];
        int sector;
        h *= hscale;
        if (h < 0)
            do h += 6; while (h < 0);
        else if (h >= 6)
            do h -= 6; while (h >= 6);
        sector = (int)floorf(h);
        h -= sector;
        if ((unsigned)sector >= 6u) {
            sector = 0;
            h = 0.f;
        }
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
        const float x = rintf(f[k] * 255.f);
        bgr[k] = (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x));
    }
}

void erpo_draw_match(const uint8_t* left, const uint8_t* right, int32_t W, int32_t H,
                     const float* key_left, const float* key_right, int32_t m, uint8_t* out) {
    for (size_t q = 0; q < (size_t)W * H; q++) {
        const uint8_t* a = left + q * 3;
        const uint8_t* b = right + q * 3;
        out[q * 3] = (uint8_t)((a[0] * 4899 + a[1] * 9617 + a[2] * 1868 + (1 << 13)) >> 14);
        out[q * 3 + 1] = (uint8_t)((b[0] * 4899 + b[1] * 9617 + b[2] * 1868 + (1 << 13)) >> 14);
        out[q * 3 + 2] = 0;
    }
    for (int i = 0; i < m; i++) {
        uint8_t c[3];
        const double hd = i * (180.0 / m);
        const int hh = (int)rint(hd);
        erpo_hsv2bgr(hh < 0 ? 0 : (hh > 255 ? 255 : hh), 180, 150, c);
        const int ax = (int)rintf(key_left[2 * i]), ay = (int)rintf(key_left[2 * i + 1]);
        const int bx = (int)rintf(key_right[2 * i]), by = (int)rintf(key_right[2 * i + 1]);
        const int dx = bx - ax, dy = by - ay;
        const double len2 = (double)dx * dx + (double)dy * dy;
        const int x0 = (ax < bx ? ax : bx) - 3, x1 = (ax > bx ? ax : bx) + 3;
        const int y0 = (ay < by ? ay : by) - 3, y1 = (ay > by ? ay : by) + 3;
        for (int y = y0 < 0 ? 0 : y0; y <= y1 && y < H; y++)
            for (int x = x0 < 0 ? 0 : x0; x <= x1 && x < W; x++) {
                const double px = x - ax, py = y - ay;
                double w = len2 > 0 ? (px * dx + py * dy) / len2 : 0.0;
                w = w < 0 ? 0 : (w > 1 ? 1 : w);
                const double ex = px - w * dx, ey = py - w * dy;
                if (ex * ex + ey * ey <= 6.25) memcpy(out + ((size_t)y * W + x) * 3, c, 3);
            }
    }
}
