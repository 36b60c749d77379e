// Matcher internals probe (dev tool): runs knn2_filter + knn2_rescore on B random unit-vector
// pairs (N x N, 80 % of the queries with a noisy partner) through the library's launchers and
// prints the per-pair max norm, the slot-count histogram, the overflow count and stage times.
//   hipcc -O2 -std=c++17 -I include -I erp_match_eightpoint_test_amd/csrc scripts/dev/matcher_probe.cpp \
//     -L erp_match_eightpoint_test_amd/lib -lerp_match -Wl,-rpath,$PWD/erp_match_eightpoint_test_amd/lib -o scripts/dev/matcher_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "erp_kernels.hpp"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 8, N = argc > 2 ? atoi(argv[2]) : 4096;
    std::mt19937 rng(7);
    std::normal_distribution<float> g(0.f, 1.f);
    std::vector<float> q((size_t)B * N * 64), t((size_t)B * N * 64);
    auto unit = [&](float* v) {
        double s = 0;
        for (int k = 0; k < 64; k++) s += (double)v[k] * v[k];
        for (int k = 0; k < 64; k++) v[k] = (float)(v[k] / std::sqrt(s));
    };
    for (size_t i = 0; i < (size_t)B * N; i++) {
        float* tv = &t[i * 64];
        for (int k = 0; k < 64; k++) tv[k] = g(rng);
        unit(tv);
    }
    std::uniform_int_distribution<int> pick(0, N - 1);
    std::uniform_real_distribution<float> u01(0.f, 1.f);
    for (int p = 0; p < B; p++)
        for (int i = 0; i < N; i++) {
            float* qv = &q[((size_t)p * N + i) * 64];
            if (u01(rng) < 0.8f) {
                const float* tv = &t[((size_t)p * N + pick(rng)) * 64];
                for (int k = 0; k < 64; k++) qv[k] = tv[k] + 0.03f * g(rng);
            } else {
                for (int k = 0; k < 64; k++) qv[k] = g(rng);
            }
            unit(qv);
        }
    std::vector<int64_t> off(B + 1);
    for (int p = 0; p <= B; p++) off[p] = (int64_t)p * N;
    erp::BatchShape sh{};
    sh.n_pairs = B;
    sh.max_nq = sh.max_nt = N;
    const int qblocks = (N + 255) / 256;
    int chunks = (1024 + qblocks * B - 1) / (qblocks * B);
    chunks = std::max(1, std::min(chunks, (N + 255) / 256));
    int chunk_len = ((N + chunks - 1) / chunks + 31) / 32 * 32;
    sh.fchunk_len = chunk_len;
    sh.fchunks = (N + chunk_len - 1) / chunk_len;
    printf("B=%d N=%d chunks=%d chunk_len=%d\n", B, N, sh.fchunks, sh.fchunk_len);
    float *dq, *dt, *dpu;
    int64_t *doff;
    int32_t *dcc, *dovf;
    void *split, *cand;
    erp::Top2* part;
    const size_t PQ = (size_t)B * N;
    CK(hipMalloc(&dq, q.size() * 4));
    CK(hipMalloc(&dt, t.size() * 4));
    CK(hipMalloc(&doff, (B + 1) * 8));
    CK(hipMalloc(&dpu, PQ * sh.fchunks * 8));
    CK(hipMalloc(&dcc, PQ * sh.fchunks * 2 * 4));
    CK(hipMalloc(&dovf, 4 + 12 * PQ * sh.fchunks));
    CK(hipMalloc(&split, erp::knn2_split_bytes(sh)));
    CK(hipMalloc(&cand, erp::knn2_cand_bytes(sh)));
    CK(hipMalloc(&part, PQ * sh.fchunks * sizeof(erp::Top2)));
    CK(hipMemcpy(dq, q.data(), q.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(doff, off.data(), (B + 1) * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0, 0));
        CK(erp::launch_knn2_filter(dq, dt, doff, doff, sh, split, (float2*)dpu, dcc, cand, 0));
        CK(hipEventRecord(e1, 0));
        CK(erp::launch_knn2_rescore(dq, dt, doff, doff, sh, split, (const float2*)dpu, dcc, cand,
                                    part, dovf, -1.f, 0));
        CK(hipEventRecord(e2, 0));
        CK(hipEventSynchronize(e2));
        float a, b;
        CK(hipEventElapsedTime(&a, e0, e1));
        CK(hipEventElapsedTime(&b, e1, e2));
        printf("filter %.3f ms  rescore %.3f ms\n", a, b);
    }
    std::vector<int32_t> cc(PQ * sh.fchunks * 2);
    CK(hipMemcpy(cc.data(), dcc, cc.size() * 4, hipMemcpyDeviceToHost));
    int32_t novf;
    CK(hipMemcpy(&novf, dovf, 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> tmax(B);
    CK(hipMemcpy(tmax.data(), (char*)split + (size_t)B * N * (64 * 2 + 4), B * 4, hipMemcpyDeviceToHost));
    std::vector<float> pu(PQ * sh.fchunks * 2);
    CK(hipMemcpy(pu.data(), dpu, pu.size() * 4, hipMemcpyDeviceToHost));
    float tm;
    std::memcpy(&tm, &tmax[0], 4);
    printf("tmax[0] = %g  overflow entries = %d\n", tm, novf);
    int hist[20] = {};
    double mean = 0;
    for (int v : cc) {
        hist[std::min(v, 19)]++;
        mean += v;
    }
    printf("slot counts per (query, chunk, half): mean %.2f\n", mean / cc.size());
    for (int k = 0; k < 20; k++) printf("%d:%d ", k, hist[k]);
    printf("\npu[0..3] = (%g %g) (%g %g)\n", pu[0], pu[1], pu[2], pu[3]);
    return 0;
}
