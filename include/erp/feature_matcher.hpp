// erp/feature_matcher.hpp -- C++ mirror of the reference's feature_matcher class for the hot
// path (match_two_image), without OpenCV.  Reference: /root/reference/src/feature_matcher.hpp:26-51.
//
// Differences that are deliberate:
//  * descriptors are passed as a plain row-major float view (cv::Mat CV_32FC1 equivalent);
//  * matching is EXACT k=2 (FlannBasedMatcher is an approximate randomized KD-tree search);
//  * SURF detection/description (detect_key_point, comput_descriptor), draw_match and do_all
//    are outside the accelerated path and not provided.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "../erp_match.h"
#include "types.hpp"

namespace erp {

class feature_matcher {
public:
    explicit feature_matcher(int device = 0);
    ~feature_matcher();
    feature_matcher(const feature_matcher&) = delete;
    feature_matcher& operator=(const feature_matcher&) = delete;

    // src/feature_matcher.hpp:36 -- k=2 nearest neighbours of every descriptor1 row among the
    // descriptor2 rows, kept when d0 < 0.3f * d1; ascending queryIdx.
    std::vector<DMatch> match_two_image(const Descriptors& descriptor1, const Descriptors& descriptor2);

    float ratio_thresh = 0.3f;  // src/feature_matcher.cpp:47

private:
    erp_ctx* ctx_ = nullptr;
};

}  // namespace erp
