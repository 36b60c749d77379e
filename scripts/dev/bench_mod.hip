// Developer micro-benchmark (not part of the library): throughput of exact x mod d variants
// (x < 2^31, 256 <= d <= 65536, d uniform across the wave) as in the sampler's replay.
//   hipcc --offload-arch=gfx950 -O3 scripts/dev/bench_mod.hip -o /tmp/bm
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1;} } while (0)

template <int V>
__global__ __launch_bounds__(256) void kmod(uint32_t seed, int n, const double* rtab, const float* rtabf, const uint32_t* magic, uint32_t* out) {
    uint32_t x = seed * 2654435761u + threadIdx.x * 40503u + blockIdx.x * 7919u;
    uint32_t acc = 0;
    for (int it = 0; it < n; it++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int d = 1000 + ((it * 16 + u) & 1023);  // uniform
            x = x * 1664525u + 1013904223u;
            const uint32_t xv = x >> 1;
            uint32_t j;
            if (V == 0) {        // fp64: cvt, mul, cvt, mad_i24
                const int q = (int)((double)xv * rtab[d]);
                j = (uint32_t)((int)xv - q * d);
            } else if (V == 1) { // f32 estimate + fix-ups
                int q = (int)((float)xv * rtabf[d]);
                int r = (int)xv - q * d;
                r = r < 0 ? r + d : r;
                r = r < 0 ? r + d : r;
                r = r >= d ? r - d : r;
                j = (uint32_t)r;
            } else {             // magic-number mulhi
                const uint32_t m = magic[d];
                const uint32_t q = __umulhi(xv, m) >> 16;
                int r = (int)xv - (int)q * d;
                r = r >= d ? r - d : r;
                j = (uint32_t)r;
            }
            acc += j;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const int N = 65538;
    double* hr = new double[N]; float* hf = new float[N]; uint32_t* hm = new uint32_t[N];
    for (int d = 1; d < N; d++) { hr[d] = 1.0 / d * (1 + 1e-12); hf[d] = 1.0f / d; hm[d] = (uint32_t)((65536.0 * 4294967296.0) / d) + 1; }
    double* dr; float* df; uint32_t* dm; uint32_t* o;
    CK(hipMalloc(&dr, N * 8)); CK(hipMalloc(&df, N * 4)); CK(hipMalloc(&dm, N * 4)); CK(hipMalloc(&o, 4096 * 256 * 4));
    CK(hipMemcpy(dr, hr, N * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(df, hf, N * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(dm, hm, N * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int blocks = 4096, n = 256;
    for (int v = 0; v < 3; v++) {
        for (int rep = 0; rep < 2; rep++) {
            CK(hipEventRecord(a, 0));
            if (v == 0) hipLaunchKernelGGL(kmod<0>, dim3(blocks), dim3(256), 0, 0, 1u, n, dr, df, dm, o);
            if (v == 1) hipLaunchKernelGGL(kmod<1>, dim3(blocks), dim3(256), 0, 0, 1u, n, dr, df, dm, o);
            if (v == 2) hipLaunchKernelGGL(kmod<2>, dim3(blocks), dim3(256), 0, 0, 1u, n, dr, df, dm, o);
            CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("variant %d: %.3f ms  %.1f Gmod/s\n", v, ms, (double)blocks * 256 * n * 16 / ms / 1e6);
        }
    }
    return 0;
}
