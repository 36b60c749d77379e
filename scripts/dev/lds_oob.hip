// Probe: what an LDS masked-OR-with-return does at addresses beyond the workgroup's LDS
// allocation on gfx950 (the sampler's clamp-free MODE 0 relies on: returns 0, no write).
// hipcc -O2 --offload-arch=gfx950 scripts/dev/lds_oob.hip -o scripts/dev/lds_oob
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__global__ __launch_bounds__(64) void probe(int nwords, int kmax, uint32_t* out, uint32_t* after) {
    extern __shared__ uint32_t bm[];
    const int lane = threadIdx.x;
    for (int k = 0; k < nwords; k++) bm[k * 64 + lane] = 0xA5A5A5A5u ^ (k * 64 + lane);
    __syncthreads();
    for (int k = 0; k < kmax; k++) {
        const uint32_t a = (uint32_t)(k * 256 + lane * 4);
        uint32_t old;
        asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(old) : "v"(a), "v"(0x1u), "v"(0u) : "memory");
        out[k * 64 + lane] = old;
    }
    __syncthreads();
    for (int k = 0; k < nwords; k++) after[k * 64 + lane] = bm[k * 64 + lane];
}

int main(int argc, char** argv) {
    const int nwords = argc > 1 ? atoi(argv[1]) : 4, kmax = 2048;  // probe up to 512 KB
    uint32_t *out, *after;
    hipMalloc(&out, kmax * 64 * 4);
    hipMalloc(&after, nwords * 64 * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), nwords * 256, 0, nwords, kmax, out, after);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 1; }
    static uint32_t h[2048 * 64], ha[64 * 64];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(ha, after, sizeof(ha), hipMemcpyDeviceToHost);
    int bad_in = 0, bad_after = 0;
    long nonzero_oob = 0;
    int first_nz = -1;
    for (int k = 0; k < kmax; k++)
        for (int l = 0; l < 64; l++) {
            const uint32_t v = h[k * 64 + l];
            if (k < nwords) bad_in += v != (0xA5A5A5A5u ^ (k * 64 + l));
            else if (v) { nonzero_oob++; if (first_nz < 0) first_nz = k; }
        }
    for (int k = 0; k < nwords; k++)
        for (int l = 0; l < 64; l++)
            bad_after += ha[k * 64 + l] != ((0xA5A5A5A5u ^ (k * 64 + l)) & ~1u);
    int last_nz = -1;
    for (int k = nwords; k < kmax; k++)
        for (int l = 0; l < 64; l++) if (h[k * 64 + l]) last_nz = k;
    printf("nwords %d: last nonzero word %d; ", nwords, last_nz);
    printf("in-range old mismatches %d, in-range final mismatches %d, out-of-range nonzero %ld "
           "(first word %d)\n", bad_in, bad_after, nonzero_oob, first_nz);
    return 0;
}
