// host_api.cpp -- the C++ class API (include/erp/*.hpp) over the C ABI.  Host code only.
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/erp/eight_point.hpp"
#include "../../include/erp/feature_matcher.hpp"

namespace erp {

static void check(erp_status s, const char* where) {
    if (s != ERP_OK) throw error(s, where);
}

feature_matcher::feature_matcher(int device) { check(erp_ctx_create(device, &ctx_), "feature_matcher"); }
feature_matcher::~feature_matcher() {
    if (ctx_) erp_ctx_destroy(ctx_);
}

std::vector<DMatch> feature_matcher::match_two_image(const Descriptors& d1, const Descriptors& d2) {
    if (d1.cols != d2.cols) throw error(ERP_INVALID_ARG, "match_two_image: descriptor size");
    auto pack = [](const Descriptors& d, std::vector<float>& buf) -> const float* {
        const size_t row = (size_t)d.cols * sizeof(float);
        if (d.step == 0 || d.step == row) return d.data;
        buf.resize((size_t)d.rows * d.cols);
        for (int r = 0; r < d.rows; r++)
            memcpy(&buf[(size_t)r * d.cols], (const char*)d.data + (size_t)r * d.step, row);
        return buf.data();
    };
    std::vector<float> b1, b2;
    const float* p1 = pack(d1, b1);
    const float* p2 = pack(d2, b2);
    std::vector<erp_dmatch> out((size_t)std::max(d1.rows, 1));
    int32_t n = 0;
    erp_status s;
    if (ratio_thresh == 0.3f) {
        s = erp_match_two_image(ctx_, p1, d1.rows, p2, d2.rows, d1.cols, out.data(), &n);
    } else {
        s = ERP_INVALID_ARG;  // the host entry point fixes the reference ratio
    }
    check(s, "match_two_image");
    std::vector<DMatch> res((size_t)n);
    for (int32_t i = 0; i < n; i++) {
        res[i].queryIdx = out[i].queryIdx;
        res[i].trainIdx = out[i].trainIdx;
        res[i].imgIdx = out[i].imgIdx;
        res[i].distance = out[i].distance;
    }
    return res;
}

eight_point::eight_point(int device) {
    erp_ransac_cfg_default(&cfg);
    check(erp_ctx_create(device, &ctx_), "eight_point");
}
eight_point::~eight_point() {
    if (ctx_) erp_ctx_destroy(ctx_);
}

void eight_point::find(int W, int H, std::vector<KeyPoint>& kl, std::vector<KeyPoint>& kr,
                       Vec3f& R, Vec3f& T, int match_size) {
    if (match_size < 0 || (size_t)match_size > kl.size() || (size_t)match_size > kr.size())
        throw error(ERP_INVALID_ARG, "find: match_size");
    std::vector<erp_point2f> a((size_t)match_size), b((size_t)match_size);
    for (int i = 0; i < match_size; i++) {
        a[i] = erp_point2f{kl[i].pt.x, kl[i].pt.y};
        b[i] = erp_point2f{kr[i].pt.x, kr[i].pt.y};
    }
    check(erp_eight_point_find(ctx_, W, H, a.data(), b.data(), match_size, &cfg, R.val, T.val, &last_),
          "find");
}

void eight_point::initial_guess(int, int, std::vector<Point3d>& l, std::vector<Point3d>& r, Vec3f& R,
                                Vec3f& T, int match_size) {
    if (match_size < 0 || (size_t)match_size > l.size() || (size_t)match_size > r.size())
        throw error(ERP_INVALID_ARG, "initial_guess: match_size");
    check(erp_initial_guess(ctx_, &l[0].x, &r[0].x, match_size, &cfg, R.val, T.val, &last_),
          "initial_guess");
}

void eight_point::eight_point_estimation(int, int, std::vector<Point3d>& l, std::vector<Point3d>& r,
                                         Vec3f& R1, Vec3f& R2, Vec3f& T, bool& v1, bool& v2,
                                         int match_size) {
    if (match_size < 0 || (size_t)match_size > l.size() || (size_t)match_size > r.size())
        throw error(ERP_INVALID_ARG, "eight_point_estimation: match_size");
    erp_hypothesis h;
    check(erp_eight_point_estimation(ctx_, &l[0].x, &r[0].x, match_size, &h), "eight_point_estimation");
    for (int k = 0; k < 3; k++) {
        R1[k] = h.R1[k];
        R2[k] = h.R2[k];
        T[k] = h.T[k];
    }
    v1 = h.R1_valid != 0;
    v2 = h.R2_valid != 0;
}

}  // namespace erp
