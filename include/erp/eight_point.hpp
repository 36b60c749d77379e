// erp/eight_point.hpp -- C++ mirror of the reference's eight_point class (and random_array's
// role) without OpenCV.  Reference: /root/reference/src/eight_point.hpp:8-59.
//
// The hard-coded constants of initial_guess (80 iterations, 25 % samples, 20-80 % trimmed
// mean, 1.57 rad validity) live in `cfg` with the reference values as defaults; the sampler
// replays the reference's process-global glibc rand() stream (seed 1, `cfg.offset` draws
// consumed before).  All work runs on the GPU through the C ABI (include/erp_match.h).
#pragma once

#include <vector>

#include "../erp_match.h"
#include "types.hpp"

namespace erp {

class eight_point {
public:
    explicit eight_point(int device = 0);
    ~eight_point();
    eight_point(const eight_point&) = delete;
    eight_point& operator=(const eight_point&) = delete;

    // src/eight_point.hpp:11-14
    void find(int im_width, int im_height, std::vector<KeyPoint>& key_left,
              std::vector<KeyPoint>& key_right, Vec3f& R_vec_out, Vec3f& T_vec_out, int match_size);
    // src/eight_point.hpp:15-19
    void eight_point_estimation(int im_width, int im_height, std::vector<Point3d>& key_point_left_rect,
                                std::vector<Point3d>& key_point_right_rect, Vec3f& R1_vec,
                                Vec3f& R2_vec, Vec3f& T_vec, bool& R1_valid, bool& R2_valid,
                                int match_size);
    // src/eight_point.hpp:20-23
    void initial_guess(int im_width, int im_height, std::vector<Point3d>& key_point_left_rect,
                       std::vector<Point3d>& key_point_right_rect, Vec3f& R_vec_out,
                       Vec3f& T_vec_out, int match_size);

    erp_ransac_cfg cfg;                 // reference constants (erp_ransac_cfg_default)
    const erp_pair_result& last_result() const { return last_; }

private:
    erp_ctx* ctx_ = nullptr;
    erp_pair_result last_{};
};

}  // namespace erp
