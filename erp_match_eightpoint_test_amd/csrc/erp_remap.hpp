// erp_remap.hpp -- launchers of the ERP pixel-remap kernels (remap.hip): the spherical band
// remap of spherical_surf::do_all and the rectification remaps of automatic.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/erp_match.h"

namespace erp {

enum RemapMode : int32_t {
    kRemapCrop = 0,   // crop_rotated_image: output rows r <- source rows row0 + r, rotated
    kRemapCopy = 1,   // the unrotated band: rows [row0, row0 + rows) copied
    kRemapFull = 2,   // rotate_image: every pixel of the H x W image
    kRemapRot90 = 3   // rotate_image, then cv::rotate(ROTATE_90_CLOCKWISE): W x H output
};

struct RemapJob {
    const uint8_t* src;  // H x W x 3 (BGR bytes, row-major)
    uint8_t* dst;
    double m[9];         // the matrix rotate_pixel applies (row-major)
    int32_t row0;        // source row of output row 0 (crop / copy)
    int32_t rows;        // output rows (crop / copy: H/4, full: H)
    int32_t mode;        // RemapMode
    int32_t pad;
};

constexpr int kMaxRemapJobs = 8;
struct RemapJobs {
    RemapJob j[kMaxRemapJobs];
};

// pixels whose truncated values fall within 1e-8 of an integer are deferred to a fix-up kernel
// (correctly rounded transcendentals, erp_device.hpp rotate_pixel_cr): list of
// (job << 32 | output pixel index), sized for every output pixel of the launch
struct RemapScratch {
    uint32_t* count;        // device counter (zeroed by launch_remap)
    uint64_t* list;         // [n_jobs * out_rows * out_cols]
};

// up to kMaxRemapJobs independent remaps of images sharing W x H: the remap launch + the
// boundary fix-up launch
hipError_t launch_remap(const RemapJobs& jobs, int n_jobs, int max_out_rows, int max_out_cols,
                        int W, int H, const RemapScratch& scr, hipStream_t st);

struct BandKeypointArgs {
    double m[4][9];     // per band: rotate_keypoint's matrix (unused for shift_band)
    int32_t end[4];     // exclusive end index of each band's segment in the concatenated list
    int32_t shift_band; // the unrotated band (pt.y += height*3/8), 1 in do_all; -1 = none
    int32_t W, H;
};
hipError_t launch_band_keypoints(erp_point2f* d_kp, const BandKeypointArgs& a, hipStream_t st);

}  // namespace erp
