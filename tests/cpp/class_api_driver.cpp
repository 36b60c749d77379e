// A reference-side C++ program that uses ONLY the drop-in class API (include/erp/*.hpp, the
// INTEGRATION.md section 1 snippet): feature_matcher::match_two_image -> gather ->
// eight_point::find, plus eight_point::eight_point_estimation and initial_guess on bearings.
// No OpenCV, no Python: the calls a maintainer of the reference would make
// (src/spherical_surf.cpp:153, src/automatic.cpp:126, src/eight_point.hpp:11-23).
//
//   class_api_driver <in_dir> <out_dir>
// in:  meta.i32 = {N, T, W, H, iters, n_est}; desc_l.f32 [N][64]; desc_r.f32 [T][64];
//      kp_l.f32 [N][2]; kp_r.f32 [T][2]; est_l.f64 / est_r.f64 [n_est][3] (bearings)
// out: matches.bin (erp::DMatch rows), find.bin (R, T as 6 floats + erp_pair_result),
//      est.bin (R1, R2, T as 9 floats + R1_valid, R2_valid as 2 int32),
//      guess.bin (R, T as 6 floats + erp_pair_result)
#include <erp/eight_point.hpp>
#include <erp/feature_matcher.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

template <class T>
static std::vector<T> read_all(const std::string& path, size_t n) {
    std::vector<T> v(n);
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f || std::fread(v.data(), sizeof(T), n, f) != n) {
        std::fprintf(stderr, "read %s failed\n", path.c_str());
        std::exit(2);
    }
    std::fclose(f);
    return v;
}

static void write_all(const std::string& path, const void* p, size_t bytes) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(p, 1, bytes, f) != bytes) {
        std::fprintf(stderr, "write %s failed\n", path.c_str());
        std::exit(2);
    }
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s <in_dir> <out_dir>\n", argv[0]);
        return 2;
    }
    const std::string in = argv[1], out = argv[2];
    const std::vector<int> meta = read_all<int>(in + "/meta.i32", 6);
    const int N = meta[0], T = meta[1], W = meta[2], H = meta[3], iters = meta[4], n_est = meta[5];
    const std::vector<float> dl = read_all<float>(in + "/desc_l.f32", (size_t)N * 64);
    const std::vector<float> dr = read_all<float>(in + "/desc_r.f32", (size_t)T * 64);
    const std::vector<float> pl = read_all<float>(in + "/kp_l.f32", (size_t)N * 2);
    const std::vector<float> pr = read_all<float>(in + "/kp_r.f32", (size_t)T * 2);
    try {
        // src/spherical_surf.cpp:153 -- fm.match_two_image(descriptor_left, descriptor_right)
        erp::feature_matcher fm(0);
        const std::vector<erp::DMatch> m =
            fm.match_two_image(erp::Descriptors{dl.data(), N, 64, 0}, erp::Descriptors{dr.data(), T, 64, 0});
        write_all(out + "/matches.bin", m.data(), m.size() * sizeof(erp::DMatch));
        // :175-179 gather, then src/automatic.cpp:126 -- estimater.find(...)
        std::vector<erp::KeyPoint> kl(m.size()), kr(m.size());
        for (size_t i = 0; i < m.size(); i++) {
            kl[i].pt = {pl[2 * m[i].queryIdx], pl[2 * m[i].queryIdx + 1]};
            kr[i].pt = {pr[2 * m[i].trainIdx], pr[2 * m[i].trainIdx + 1]};
        }
        erp::eight_point ep(0);
        ep.cfg.iters = iters;
        erp::Vec3f R, Tv;
        ep.find(W, H, kl, kr, R, Tv, (int)m.size());
        {
            std::vector<char> buf(6 * sizeof(float) + sizeof(erp_pair_result));
            std::memcpy(buf.data(), R.val, 12);
            std::memcpy(buf.data() + 12, Tv.val, 12);
            std::memcpy(buf.data() + 24, &ep.last_result(), sizeof(erp_pair_result));
            write_all(out + "/find.bin", buf.data(), buf.size());
        }
        if (n_est > 0) {
            const std::vector<double> bl = read_all<double>(in + "/est_l.f64", (size_t)n_est * 3);
            const std::vector<double> br = read_all<double>(in + "/est_r.f64", (size_t)n_est * 3);
            std::vector<erp::Point3d> l(n_est), r(n_est);
            for (int i = 0; i < n_est; i++) {
                l[i] = {bl[3 * i], bl[3 * i + 1], bl[3 * i + 2]};
                r[i] = {br[3 * i], br[3 * i + 1], br[3 * i + 2]};
            }
            // src/eight_point.hpp:15-19
            erp::Vec3f R1, R2, Te;
            bool v1 = false, v2 = false;
            ep.eight_point_estimation(W, H, l, r, R1, R2, Te, v1, v2, n_est);
            float f9[9] = {R1[0], R1[1], R1[2], R2[0], R2[1], R2[2], Te[0], Te[1], Te[2]};
            int vv[2] = {v1 ? 1 : 0, v2 ? 1 : 0};
            std::vector<char> buf(sizeof(f9) + sizeof(vv));
            std::memcpy(buf.data(), f9, sizeof(f9));
            std::memcpy(buf.data() + sizeof(f9), vv, sizeof(vv));
            write_all(out + "/est.bin", buf.data(), buf.size());
            // src/eight_point.hpp:20-23 on the same bearings
            erp::Vec3f Rg, Tg;
            ep.initial_guess(W, H, l, r, Rg, Tg, n_est);
            std::vector<char> gb(6 * sizeof(float) + sizeof(erp_pair_result));
            std::memcpy(gb.data(), Rg.val, 12);
            std::memcpy(gb.data() + 12, Tg.val, 12);
            std::memcpy(gb.data() + 24, &ep.last_result(), sizeof(erp_pair_result));
            write_all(out + "/guess.bin", gb.data(), gb.size());
        }
    } catch (const erp::error& e) {
        std::fprintf(stderr, "erp::error %d: %s\n", (int)e.status, e.what());
        return 3;
    }
    std::printf("ok\n");
    return 0;
}
