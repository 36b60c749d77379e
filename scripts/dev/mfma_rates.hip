// MFMA issue-rate probe on gfx950 (dev): v_mfma_f32_32x32x16_bf16 with NCH independent
// accumulation chains per wave, WPS waves per SIMD (blocks of 256 threads, WPS blocks per CU),
// VGPR or AGPR accumulators as compiled.  Prints cycles per MFMA per SIMD at 2.4 GHz nominal
// (wall time; the chip clocks lower under MFMA load, so the floor reads ~36-40 at 2.0-2.1 GHz).
//   hipcc -O3 --offload-arch=gfx950 [-mllvm -amdgpu-mfma-vgpr-form] scripts/dev/mfma_rates.hip -o scripts/dev/mfma_rates
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kIters = 4096;

template <int NCH>
__global__ __launch_bounds__(256) void probe(float* out, float seed) {
    bf16x8 a, b;
    for (int k = 0; k < 8; k++) {
        a[k] = (__bf16)(seed * (threadIdx.x + k));
        b[k] = (__bf16)(seed * (threadIdx.x - k));
    }
    f32x16 acc[NCH];
    for (int c = 0; c < NCH; c++)
        for (int k = 0; k < 16; k++) acc[c][k] = 0.f;
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int c = 0; c < NCH; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    }
    float s = 0.f;
    for (int c = 0; c < NCH; c++)
        for (int k = 0; k < 16; k++) s += acc[c][k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NCH>
void run(int wps, float* out) {
    const int blocks = 256 * wps;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    probe<NCH><<<blocks, 256>>>(out, 1e-3f);
    (void)hipEventRecord(e0);
    probe<NCH><<<blocks, 256>>>(out, 2e-3f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double mfma_per_simd = (double)wps * kIters * NCH;
    printf("chains %d waves/SIMD %d: %.3f ms  %.1f cyc/MFMA/SIMD (2.4 GHz)  %.0f TF/s\n", NCH, wps, ms,
           ms * 1e-3 * 2.4e9 / mfma_per_simd, 1024.0 * mfma_per_simd * 32768.0 / (ms * 1e-3) / 1e12);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 8 * 256 * 4);
    for (int wps : {1, 2, 3, 4}) {
        run<1>(wps, out);
        run<2>(wps, out);
        run<4>(wps, out);
    }
    return 0;
}
