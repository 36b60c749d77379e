// Generates tests/golden/glibc_shuffle.json from the REAL glibc rand() and libstdc++
// std::random_shuffle of this container (the third-party code the reference's sampler calls:
// /root/reference/src/eight_point.hpp:54-58).  Pins oracle/erp_oracle.c's restatement.
// Build+run: g++ -O0 -std=c++14 gen_glibc_shuffle.cpp -o /tmp/gen && /tmp/gen > glibc_shuffle.json
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

static void dump_shuffles(const char* key, const int* sizes, int nsizes, int reps) {
    std::printf("  \"%s\": [\n", key);
    for (int s = 0; s < nsizes; s++) {
        for (int r = 0; r < reps; r++) {
            std::vector<int> a(sizes[s]);
            std::iota(a.begin(), a.end(), 0);
            std::random_shuffle(a.begin(), a.end());  // same call as random_array
            std::printf("    {\"n\": %d, \"perm\": [", sizes[s]);
            for (int i = 0; i < sizes[s]; i++) std::printf(i ? ",%d" : "%d", a[i]);
            bool last = (s == nsizes - 1) && (r == reps - 1);
            std::printf("]}%s\n", last ? "" : ",");
        }
    }
    std::printf("  ],\n");
}

int main() {
    std::printf("{\n");
    // 1) unseeded rand(): the reference never calls srand (seed 1)
    std::printf("  \"rand_seed1\": [");
    for (int i = 0; i < 2000; i++) std::printf(i ? ",%d" : "%d", std::rand());
    std::printf("],\n");
    // 2) consecutive random_array shuffles continuing the same global stream
    const int sizes[] = {1, 2, 5, 9, 36, 100, 400};
    dump_shuffles("shuffles_after_2000", sizes, 7, 2);
    // 3) seeded stream (sampler seed parameter)
    std::srand(20200423u);
    std::printf("  \"rand_seed20200423\": [");
    for (int i = 0; i < 500; i++) std::printf(i ? ",%d" : "%d", std::rand());
    std::printf("],\n");
    // 4) the stream after a long discard (jump-ahead check): draws 1e6..1e6+99 of seed 1
    std::srand(1u);
    for (int i = 0; i < 1000000; i++) (void)std::rand();
    std::printf("  \"rand_seed1_from_1e6\": [");
    for (int i = 0; i < 100; i++) std::printf(i ? ",%d" : "%d", std::rand());
    std::printf("]\n}\n");
    return 0;
}
