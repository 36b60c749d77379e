// VALU issue-rate probe on gfx950: cycles per wave64 instruction per SIMD for the op mix the
// sampler uses (int add / shift / lshl_add / mad_i32_i24 / bfe, fp64 fma, cvt_f64_u32, fp32 fma).
// 8 independent chains per lane, a long unrolled loop, many waves per SIMD; wall time by HIP
// events, clock from the kernel's own s_memtime delta.
//   hipcc -O3 --offload-arch=gfx950 scripts/dev/valu_rates.hip -o scripts/dev/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 32768;

#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t a[CHAINS];
    double f[CHAINS];
    float g[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; k++) {
        a[k] = seed + threadIdx.x * 7 + k;
        f[k] = (double)a[k];
        g[k] = (float)a[k];
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int k = 0; k < CHAINS; k++) {
            if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 1) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 2) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(a[k]));
            if constexpr (OP == 3) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 4) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 5) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 6) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 7) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 8) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 9) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 10) asm volatile("v_mad_i32_i24 %0, %0, %1, %0" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 11) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 12) asm volatile("v_bfe_u32 %0, %0, %1, 1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 13) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 14) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(f[k]) : "v"(f[(k + 1) % CHAINS]));
            if constexpr (OP == 15) asm volatile("v_add_f64 %0, %0, %1" : "+v"(f[k]) : "v"(f[(k + 1) % CHAINS]));
            if constexpr (OP == 16) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(f[k]) : "v"(a[k]));
            if constexpr (OP == 17) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(g[k]) : "v"(g[(k + 1) % CHAINS]));
            if constexpr (OP == 18) asm volatile("v_add_f32 %0, %0, %1" : "+v"(g[k]) : "v"(g[(k + 1) % CHAINS]));
            if constexpr (OP == 19) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(g[k]) : "v"(g[(k + 1) % CHAINS]));
            if constexpr (OP == 20) asm volatile("v_min_f32 %0, %0, %1" : "+v"(g[k]) : "v"(g[(k + 1) % CHAINS]));
            if constexpr (OP == 21) asm volatile("v_min3_f32 %0, %0, %1, %1" : "+v"(g[k]) : "v"(g[(k + 1) % CHAINS]));
            if constexpr (OP == 22) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(f[k]) : "v"(f[(k + 1) % CHAINS]));
            if constexpr (OP == 23) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(f[k]) : "v"(f[(k + 1) % CHAINS]));
            if constexpr (OP == 24) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) % CHAINS]));
            if constexpr (OP == 25) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(g[k]) : "v"(a[k]));
            if constexpr (OP == 26) asm volatile("v_cmp_lt_f32 vcc, %0, %1" :: "v"(g[k]), "v"(g[(k + 1) % CHAINS]) : "vcc");
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < CHAINS; k++) s += a[k] + (uint32_t)f[k] + (uint32_t)g[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, int blocks_per_cu, uint32_t* out, uint64_t* clk) {
    const int blocks = 256 * blocks_per_cu;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<OP><<<blocks, 256>>>(out, clk, 1);
    hipEventRecord(e0);
    probe<OP><<<blocks, 256>>>(out, clk, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t c[1];
    hipMemcpy(c, clk, 8, hipMemcpyDeviceToHost);
    // wave-instructions per SIMD: blocks * 4 waves * iters * chains / (256 CUs * 4 SIMDs)
    const double winst = (double)blocks * 4 * kIters * CHAINS / 1024.0;
    const double ghz_wall = 0;  (void)ghz_wall;
    // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH.md)
    const double cyc_wall_2p4 = ms * 1e-3 * 2.4e9;
    printf("%-16s waves/SIMD %d: %.3f ms, %.2f cyc/inst/SIMD at 2.4 GHz wall, block0 memtime %.2f cyc/inst/SIMD-share\n",
           name, blocks_per_cu, ms, cyc_wall_2p4 / winst,
           (double)c[0] / ((double)kIters * CHAINS * blocks_per_cu));
}

int main() {
    uint32_t* out;
    uint64_t* clk;
    hipMalloc(&out, 256 * 16 * 256 * 4);
    hipMalloc(&clk, 256 * 16 * 8);
    for (int bpc : {2, 4}) {
        run<0>("v_add_u32", bpc, out, clk);
        run<1>("v_sub_u32", bpc, out, clk);
        run<2>("v_lshrrev_b32", bpc, out, clk);
        run<3>("v_lshlrev_b32", bpc, out, clk);
        run<4>("v_and_b32", bpc, out, clk);
        run<5>("v_or_b32", bpc, out, clk);
        run<6>("v_min_u32", bpc, out, clk);
        run<7>("v_lshl_add_u32", bpc, out, clk);
        run<8>("v_lshl_or_b32", bpc, out, clk);
        run<9>("v_add3_u32", bpc, out, clk);
        run<10>("v_mad_i32_i24", bpc, out, clk);
        run<11>("v_mul_u32_u24", bpc, out, clk);
        run<12>("v_bfe_u32", bpc, out, clk);
        run<13>("v_cndmask_b32", bpc, out, clk);
        run<14>("v_fma_f64", bpc, out, clk);
        run<15>("v_add_f64", bpc, out, clk);
        run<16>("v_cvt_f64_u32", bpc, out, clk);
        run<17>("v_fma_f32", bpc, out, clk);
        run<18>("v_add_f32", bpc, out, clk);
        run<19>("v_mul_f32", bpc, out, clk);
        run<20>("v_min_f32", bpc, out, clk);
        run<21>("v_min3_f32", bpc, out, clk);
        run<22>("v_pk_fma_f32", bpc, out, clk);
        run<23>("v_pk_add_f32", bpc, out, clk);
        run<24>("v_mul_hi_u32", bpc, out, clk);
        run<25>("v_cvt_f32_u32", bpc, out, clk);
        run<26>("v_cmp_lt_f32", bpc, out, clk);
    }
    return 0;
}
