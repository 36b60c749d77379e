// Developer micro-benchmark (not part of the library): variants of the consensus-bounds
// histogram loop on synthetic clustered rotation vectors, timed with HIP events.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/dev/bench_bounds.hip -o /tmp/bb
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int kNB = 1280;

template <int ROWS, int MODE, int THREADS, int CPI = 1>
__global__ __launch_bounds__(THREADS) void bounds(const float* X, const float* Y, const float* Z, int K, int base, uint32_t* out) {
    constexpr int STRIDE = kNB + 4;
    __shared__ uint32_t hist[ROWS * STRIDE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int r0 = blockIdx.x * ROWS;
    float xi[ROWS], yi[ROWS], zi[ROWS];
    int hoff[ROWS];
#pragma unroll
    for (int t = 0; t < ROWS; t++) {
        const int r = (lane + t) & (ROWS - 1);
        const int row = min(r0 + r, K - 1);
        xi[t] = X[row]; yi[t] = Y[row]; zi[t] = Z[row];
        hoff[t] = r * STRIDE - base;
    }
    for (int k = tid; k < ROWS * STRIDE; k += THREADS) hist[k] = 0u;
    __syncthreads();
    uint32_t chk = 0;
    // prefetched columns: CPI per iteration, next iteration's loaded before this one computes
    float cx[CPI], cy[CPI], cz[CPI];
    int j = tid;
#pragma unroll
    for (int c = 0; c < CPI; c++) {
        const int jj = min(j + c * THREADS, K - 1);
        cx[c] = X[jj]; cy[c] = Y[jj]; cz[c] = Z[jj];
    }
    for (; j < K; j += CPI * THREADS) {
        float nx[CPI], ny[CPI], nz[CPI];
#pragma unroll
        for (int c = 0; c < CPI; c++) {
            const int jj = min(j + (CPI + c) * THREADS, K - 1);
            nx[c] = X[jj]; ny[c] = Y[jj]; nz[c] = Z[jj];
        }
#pragma unroll
        for (int c = 0; c < CPI; c++) {
            const bool ok = j + c * THREADS < K;
#pragma unroll
            for (int t = 0; t < ROWS; t++) {
                const float dx = xi[t] - cx[c], dy = yi[t] - cy[c], dz = zi[t] - cz[c];
                float s;
                if (MODE == 0) s = dx * dx + dy * dy + dz * dz;
                else s = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
                const int key = (int)(__float_as_uint(s) >> 18);
                const int b = min(max(key, base), base + kNB - 1);
                if (MODE == 2) chk += b;
                else if (MODE == 3) hist[hoff[t] + b] = (uint32_t)j;
                else if (ok) atomicAdd(&hist[hoff[t] + b], 1u);
            }
        }
#pragma unroll
        for (int c = 0; c < CPI; c++) { cx[c] = nx[c]; cy[c] = ny[c]; cz[c] = nz[c]; }
    }
    __syncthreads();
    uint32_t acc = chk;
    for (int k = tid; k < ROWS * STRIDE; k += THREADS) acc += hist[k] * (k + 1);
    if (acc == 0x12345u) out[blockIdx.x + gridDim.x * blockIdx.y] = acc;  // keep the work alive
}

template <int ROWS, int MODE, int THREADS, int CPI = 1>
float run(const float* X, const float* Y, const float* Z, int K, int base, uint32_t* out, int pairs) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    dim3 grid((K + ROWS - 1) / ROWS, pairs);
    for (int w = 0; w < 2; w++)
        hipLaunchKernelGGL((bounds<ROWS, MODE, THREADS, CPI>), grid, dim3(THREADS), 0, 0, X, Y, Z, K, base, out);
    CK(hipEventRecord(a, 0));
    const int reps = 5;
    for (int w = 0; w < reps; w++)
        hipLaunchKernelGGL((bounds<ROWS, MODE, THREADS, CPI>), grid, dim3(THREADS), 0, 0, X, Y, Z, K, base, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 10000;
    const float sig = argc > 2 ? atof(argv[2]) : 0.003f;
    const int pairs = 8;
    std::mt19937 g(1);
    std::normal_distribution<float> n(0.f, 1.f);
    std::uniform_real_distribution<float> u(-0.25f, 0.25f);
    std::vector<float> h(3 * K);
    for (int i = 0; i < K; i++) {
        const bool in = (i % 5) != 0;
        for (int c = 0; c < 3; c++) h[c * K + i] = in ? 0.1f * (c + 1) + sig * n(g) : 0.1f * (c + 1) + u(g);
    }
    float* d; uint32_t* out;
    CK(hipMalloc(&d, 3 * K * 4)); CK(hipMalloc(&out, 4 * K * 64));
    CK(hipMemcpy(d, h.data(), 3 * K * 4, hipMemcpyHostToDevice));
    const float* X = d; const float* Y = d + K; const float* Z = d + 2 * K;
    // base: 40 binades of s below (0.87)^2 ~ exponent 126 -> t = 127, elo = 87
    const int base = (127 - 40) << 5;
    printf("K=%d sig=%g pairs=%d (ms per %d launches = one B=%d step)\n", K, sig, pairs, pairs, pairs);
    printf("R8 fma atomic 256t cpi1: %.3f\n", run<8, 1, 256, 1>(X, Y, Z, K, base, out, pairs));
    printf("R8 fma atomic 256t cpi2: %.3f\n", run<8, 1, 256, 2>(X, Y, Z, K, base, out, pairs));
    printf("R8 fma atomic 256t cpi4: %.3f\n", run<8, 1, 256, 4>(X, Y, Z, K, base, out, pairs));
    printf("R8 fma noLDS  256t cpi2: %.3f\n", run<8, 2, 256, 2>(X, Y, Z, K, base, out, pairs));
    printf("R8 exact atomic 256t cpi2: %.3f\n", run<8, 0, 256, 2>(X, Y, Z, K, base, out, pairs));
    printf("R16 fma atomic 256t cpi2: %.3f\n", run<16, 1, 256, 2>(X, Y, Z, K, base, out, pairs));
    printf("R16 fma atomic 512t cpi2: %.3f\n", run<16, 1, 512, 2>(X, Y, Z, K, base, out, pairs));
    printf("R8 fma atomic 128t cpi2: %.3f\n", run<8, 1, 128, 2>(X, Y, Z, K, base, out, pairs));
    printf("R8 fma atomic 128t cpi4: %.3f\n", run<8, 1, 128, 4>(X, Y, Z, K, base, out, pairs));
    printf("R16 fma noLDS 512t cpi2: %.3f\n", run<16, 2, 512, 2>(X, Y, Z, K, base, out, pairs));
    return 0;
}
