// erp/types.hpp -- OpenCV-free POD mirrors of the cv:: types the hot path touches.
#pragma once

#include <stddef.h>
#include <stdexcept>
#include <string>

#include "../erp_match.h"

namespace erp {

struct Point2f { float x = 0, y = 0; };
struct Point3d { double x = 0, y = 0, z = 0; };

// cv::KeyPoint layout (pt, size, angle, response, octave, class_id); only pt is read.
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};

// cv::DMatch
struct DMatch {
    int queryIdx = -1, trainIdx = -1, imgIdx = -1;
    float distance = 0;
};

// cv::Vec3f
struct Vec3f {
    float val[3] = {0, 0, 0};
    float& operator[](int i) { return val[i]; }
    float operator[](int i) const { return val[i]; }
};

// a CV_32FC1 descriptor matrix view (rows x cols, row stride in bytes)
struct Descriptors {
    const float* data = nullptr;
    int rows = 0;
    int cols = 64;
    size_t step = 0;  // bytes between rows; 0 = cols * sizeof(float)
};

// thrown where the reference would hit an OpenCV assertion or undefined behaviour
struct error : std::runtime_error {
    erp_status status;
    error(erp_status s, const std::string& what)
        : std::runtime_error(what + ": " + erp_status_string(s)), status(s) {}
};

}  // namespace erp
