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
    int box[10][4];     // the same 10 boxes as (x1, y1, x2, y2) (the LDS-tiled octave-0 pass)
    int sample_pre;     // first block of this layer (the Hessian pass of octaves >= n_tiled)
    int cell_pre;       // first block of this layer's extrema cells (middle layers)
    int cells, cell_margin, cell_cols;
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
    int n_layers0;      // layers per octave (nL + 2)
    int n_tiled;        // octaves of the LDS-tiled Hessian pass (1 or 2), the rest flattened
    int max_size0;      // largest filter of octave 0
    int samples_hi;     // blocks of the Hessian pass of octaves >= n_tiled
    int mid_cells;      // blocks of the extrema pass
    size_t det_per_img;
    float threshold;
    SurfConsts consts;
};

constexpr int kSurfPatch = 20;  // the descriptor's 20 x 20 gradient patch (21 x 21 resampled)

struct SurfJob {        // a keypoint's rotated window (surf_orient_kernel)
    float cos_dir, sin_dir;
    int win, exact;     // win = 0: deleted keypoint
};

struct SurfScratch {
    uint8_t* gray;          // [n][H][W] (BGR input only)
    int32_t* sum;           // [n][H+1][W+1]
    float* det;             // [n][det_per_img]
    erp_keypoint* raw;      // [n][max_kp]
    erp_keypoint* sorted;   // [n][max_kp]
    float* desc;            // [n][max_kp][64]
    // descriptor pass over a chunk of keypoints (surf.hip): per keypoint slot tmp[21][win],
    // stx[win], sty[win] (slot = 23 * max_win floats), a job record, band work items
    float* pool;
    size_t slot;
    int max_win;
    SurfJob* jobs;
    int2* items;
    int32_t* nitems;
};

size_t surf_job_bytes();
int surf_band_rows();
// detection: gray, integral, Fast-Hessian layers, maxima + interpolation, KeypointGreater order
// (raw counts in counts[]; -needed when max_kp overflowed)
hipError_t launch_surf_detect(const uint8_t* images, int n_images, int W, int H, int channels,
                              const SurfPlan& plan, const SurfScratch& scr, int max_kp,
                              int32_t* counts, hipStream_t st);
// orientation + descriptor of keypoints g0 .. g0 + ng - 1 (numbered over the images by the
// device prefix d_kpre[n_images])
hipError_t launch_surf_describe(const uint8_t* images, int n_images, int W, int H, int channels,
                                const SurfPlan& plan, const SurfScratch& scr, int max_kp,
                                const int32_t* d_kpre, int g0, int ng, hipStream_t st);
// drop the deleted keypoints (order kept) into the outputs; final counts
hipError_t launch_surf_compact(int n_images, const SurfScratch& scr, int max_kp, erp_keypoint* kp_out,
                               float* desc_out, int32_t* counts, hipStream_t st);

}  // namespace erp
