// erp_surf.hpp -- launcher of the SURF kernels (surf.hip), SURVEY.md §8f-2.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/erp_match.h"

namespace erp {

struct SurfHF {         // one box of a Haar pattern: integral-image corner offsets, weight
    int p0, p1, p2, p3;
    float w;
};

struct SurfLayer {      // one (octave, layer) of the Fast-Hessian pyramid
    int size, step;     // filter size (9 + 6 layer) << octave, sample step 1 << octave
    int rows, cols;     // layer dims (H / step, W / step)
    int margin;         // (size / 2) / step: det of sample (i, j) sits at (i + margin, j + margin)
    int samples_i, samples_j;
    int octave;
    size_t off;         // float offset of the layer in the image's det buffer
    SurfHF dx[3], dy[3], dxy[4];
};

constexpr int kSurfNOri = 113;
struct SurfConsts {     // orientation disc (Point(i, j) order) + Gaussian weights (host-built)
    int aptx[kSurfNOri], apty[kSurfNOri];
    float aptw[kSurfNOri];
    float gdesc[20];
};

struct SurfPlan {
    const SurfLayer* d_layers;
    const int* d_mid;   // indices of the middle layers
    int n_layers, n_mid;
    int max_samples, max_mid_cells;
    size_t det_per_img;
    float threshold;
    SurfConsts consts;
};

constexpr int kSurfDescBlocks = 2048;  // describe grid (one wave each, grid-stride)
constexpr int kSurfBigWin = 900;       // largest rotated window (s < 43 -> 21 s < 900)

struct SurfScratch {
    uint8_t* gray;          // [n][H][W] (BGR input only)
    int32_t* sum;           // [n][H+1][W+1]
    float* det;             // [n][det_per_img]
    erp_keypoint* raw;      // [n][max_kp]
    erp_keypoint* sorted;   // [n][max_kp]
    float* desc;            // [n][max_kp][64]
    uint8_t* big;           // [kSurfDescBlocks][big_slot]: the horizontal area pass tmp[21][win]
    size_t big_slot;
};

hipError_t launch_surf(const uint8_t* images, int n_images, int W, int H, int channels,
                       const SurfPlan& plan, const SurfScratch& scr, int max_kp,
                       erp_keypoint* kp_out, float* desc_out, int32_t* counts, hipStream_t st);

}  // namespace erp
