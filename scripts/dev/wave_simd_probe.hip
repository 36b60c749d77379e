// Which SIMD does each wave of a 768-thread (12-wave) workgroup land on, and how fast do VALU
// chains run when only some waves work?  (Design input for the fused sampler_gram_kernel:
// its waves 0-3 replay the sampler, waves 4-11 run MFMAs.)
//   hipcc -O3 --offload-arch=gfx950 scripts/dev/wave_simd_probe.hip -o /tmp/wsp && /tmp/wsp
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdint.h>

// HW_REG_HW_ID fields (gfx9): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13
__global__ __launch_bounds__(768, 1) void probe(uint32_t* out, int busy_mask, int iters,
                                                uint64_t* cyc) {
    extern __shared__ uint32_t lds[];
    const int wv = threadIdx.x >> 6;
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 12 + wv] = id;
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint64_t t0 = __builtin_readcyclecounter();
    float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f, d = 0.25f;
    if ((busy_mask >> wv) & 1) {
        for (int k = 0; k < iters; k++) {
            a = __builtin_fmaf(a, b, c);
            c = __builtin_fmaf(c, b, d);
            d = __builtin_fmaf(d, b, a);
            b = __builtin_fmaf(b, 0.9999f, 1e-4f);
        }
    }
    uint64_t t1 = __builtin_readcyclecounter();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 12 + wv] = t1 - t0;
    if (a == 12345.f) out[0] = 0;  // keep the chain
}

int main() {
    const int nb = 256;
    uint32_t* out;
    uint64_t* cyc;
    hipMalloc(&out, nb * 12 * 4);
    hipMalloc(&cyc, nb * 12 * 8);
    uint32_t h[nb * 12];
    uint64_t hc[nb * 12];
    for (int mask : {0x00f, 0x111, 0xfff, 0x001, 0x00f0}) {
        hipLaunchKernelGGL(probe, dim3(nb), dim3(768), 80 * 1024, 0, out, mask, 20000, cyc);
        hipDeviceSynchronize();
        hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
        hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
        printf("busy mask 0x%03x: block 0 waves -> simd:", mask);
        for (int w = 0; w < 12; w++) printf(" %u", (h[w] >> 4) & 3);
        printf("   (block 1:");
        for (int w = 0; w < 12; w++) printf(" %u", (h[12 + w] >> 4) & 3);
        printf(")\n   cycles per busy wave (block 0):");
        for (int w = 0; w < 12; w++)
            if ((mask >> w) & 1) printf(" w%d=%llu", w, (unsigned long long)hc[w]);
        printf("\n");
    }
    return 0;
}
