// What bounds consensus_bounds' K-column loop on gfx950: the distance VALU work, the LDS
// histogram atomics, or neither.  Standalone copy of the loop's shape (16 rows per 256-thread
// block, [bin][16 rows] histogram, packed f32 distances of two rows, 4-column batches) with
// variants:
//   0  as in kernels.hip (distance + key + ds_add_u32)
//   1  distance + key, no LDS (keys xor-folded into a register)
//   2  ds_add_u32 only, addresses from a cheap hash (1 VALU per add)
//   3  as 0 with scalar v_fma_f32 / v_sub_f32 instead of packed f32
//   5  ds_add_u32 only, each lane its own bank (conflict-free); 6: exactly 2-way conflicts
//   4  32 rows per block, distances of 32 stream columns x 32 rows by ONE
//      v_mfma_f32_32x32x16_f16 (hi/lo split operands; timing only, values synthetic), then
//      key + ds_add_u32 into a [bin][32 rows] histogram (a lane's row = lane & 31: the 32
//      lanes of a bank group hit 32 distinct rows, conflict-free)
// Prints ms and cycles per wave-distance per SIMD (at the clock measured by s_memtime).
//   hipcc -O3 --offload-arch=gfx950 scripts/dev/bounds_probe.hip -o scripts/dev/bounds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

constexpr int R = 16, kNB = 576, kGuard = 64, kBinShift = 19;

__device__ __forceinline__ uint32_t lshl6_add(uint32_t key, uint32_t base) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 6, %2" : "=v"(r) : "v"(key), "v"(base));
    return r;
}
__device__ __forceinline__ void lds_inc(uint32_t a) {
    __hip_atomic_fetch_add((lds_u32*)(size_t)a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int V>
__global__ __launch_bounds__(256) void probe(const float* __restrict__ X, const float* __restrict__ Y,
                                             const float* __restrict__ Z, int K, int base,
                                             uint32_t* __restrict__ out, uint64_t* clk) {
    __shared__ __align__(16) uint32_t hist[(kGuard + kNB) * R];
    const int tid = threadIdx.x, lane = tid & 63;
    const int l0 = blockIdx.x * R;
    f32x2 xi[R / 2], yi[R / 2], zi[R / 2];
    uint32_t hoff[R];
    const uint32_t ha = (uint32_t)(size_t)(lds_u32*)hist;
#pragma unroll
    for (int t = 0; t < R; t++) {
        const int r = (lane + t) & (R - 1);
        xi[t >> 1][t & 1] = X[l0 + r];
        yi[t >> 1][t & 1] = Y[l0 + r];
        zi[t >> 1][t & 1] = Z[l0 + r];
        hoff[t] = ha + 4u * (uint32_t)r - 64u * (uint32_t)(base - kGuard);
    }
    for (int k = tid; k < (kGuard + kNB) * R; k += 256) hist[k] = 0;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const f32x2 bias = {1e-12f, 1e-12f};
    uint32_t acc = 0;
    for (int j = tid; j < K; j += 256) {
        const float xj = X[j], yj = Y[j], zj = Z[j];
#pragma unroll
        for (int t = 0; t < R / 2; t++) {
            if constexpr (V == 3) {  // scalar f32 instead of packed
                float s0 = __builtin_fmaf(xi[t][0] - xj, xi[t][0] - xj, 1e-12f);
                float s1 = __builtin_fmaf(xi[t][1] - xj, xi[t][1] - xj, 1e-12f);
                s0 = __builtin_fmaf(yi[t][0] - yj, yi[t][0] - yj, s0);
                s1 = __builtin_fmaf(yi[t][1] - yj, yi[t][1] - yj, s1);
                s0 = __builtin_fmaf(zi[t][0] - zj, zi[t][0] - zj, s0);
                s1 = __builtin_fmaf(zi[t][1] - zj, zi[t][1] - zj, s1);
                lds_inc(lshl6_add(__float_as_uint(s0) >> kBinShift, hoff[2 * t]));
                lds_inc(lshl6_add(__float_as_uint(s1) >> kBinShift, hoff[2 * t + 1]));
            } else if constexpr (V == 5 || V == 6) {  // LDS-only, conflict-free / 2-way
                const uint32_t h = ((uint32_t)j * 2654435761u + 40503u * t) >> 25;  // 0..127
                const uint32_t w = V == 5 ? (uint32_t)lane
                                          : (uint32_t)((lane & 15) + 32 * ((lane >> 4) & 1) + 16 * (lane >> 5));
                lds_inc(ha + 4u * (w + 64u * h));
                lds_inc(ha + 4u * (w + 64u * (h ^ 1u)));
            } else if constexpr (V == 2) {
                const uint32_t h = ((uint32_t)j * 2654435761u) >> 23;  // 0..511
                lds_inc(lshl6_add(h + (uint32_t)base + (uint32_t)t, hoff[2 * t]));
                lds_inc(lshl6_add(h + (uint32_t)base + 7u * t, hoff[2 * t + 1]));
            } else {
                const f32x2 dx = xi[t] - xj, dy = yi[t] - yj, dz = zi[t] - zj;
                f32x2 s = __builtin_elementwise_fma(dx, dx, bias);
                s = __builtin_elementwise_fma(dy, dy, s);
                s = __builtin_elementwise_fma(dz, dz, s);
                const uint32_t a0 = lshl6_add(__float_as_uint(s[0]) >> kBinShift, hoff[2 * t]);
                const uint32_t a1 = lshl6_add(__float_as_uint(s[1]) >> kBinShift, hoff[2 * t + 1]);
                if constexpr (V == 1) {
                    acc ^= a0 + a1;
                } else {
                    lds_inc(a0);
                    lds_inc(a1);
                }
            }
        }
    }
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0 && blockIdx.x == 0) *clk = t1 - t0;
    uint32_t c = acc;
    for (int k = tid; k < (kGuard + kNB) * R; k += 256) c += hist[k] * (uint32_t)k;
    out[blockIdx.x * 256 + tid] = c;
}


typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));
constexpr int R32 = 32;
__global__ __launch_bounds__(256) void probe_mfma(const half8* __restrict__ A, int K, int base,
                                                  uint32_t* __restrict__ out, uint64_t* clk) {
    extern __shared__ __align__(16) uint32_t hist32[];  // [(guard + bin)][32 rows]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t ha = (uint32_t)(size_t)(lds_u32*)hist32;
    const uint32_t hoff = ha + 4u * (uint32_t)(lane & 31) - 128u * (uint32_t)(base - kGuard);
    for (int k = tid; k < (kGuard + kNB) * R32; k += 256) hist32[k] = 0;
    // B operand: the block's 32 rows (lane & 31), k = 8 (lane >> 5) .. + 7
    half8 b = A[(size_t)(blockIdx.x * 32 + (lane & 31)) * 2 + (lane >> 5)];
    float16v c;
    for (int q = 0; q < 16; q++) c[q] = 1e-9f + 1e-12f * (float)(lane & 31);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const int ntiles = (K + 31) / 32;
    half8 a = A[(size_t)((w * 32 + (lane & 31)) % K) * 2 + (lane >> 5)];
    for (int t = w; t < ntiles; t += 4) {
        const int tn = t + 4 < ntiles ? t + 4 : t;
        const half8 an = A[(size_t)(tn * 32 + (lane & 31)) * 2 + (lane >> 5)];
        const float16v d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 16; q++) {
            uint32_t r;
            asm("v_lshl_add_u32 %0, %1, 7, %2" : "=v"(r) : "v"(__float_as_uint(d[q]) >> kBinShift), "v"(hoff));
            lds_inc(r);
        }
        a = an;
    }
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0 && blockIdx.x == 0) *clk = t1 - t0;
    uint32_t s = 0;
    for (int k = tid; k < (kGuard + kNB) * R32; k += 256) s += hist32[k] * (uint32_t)k;
    out[blockIdx.x * 256 + tid] = s;
}

// variant 7: 16 rows per block (the B operand: row = lane & 15), 16 stream columns per
// v_mfma_f32_16x16x4_f32 (A = column i = lane & 15, component lane >> 4), D = n_i + n_j - 2 u.v
// with C = n_j (per lane); 4 distances per lane per MFMA -> key, address, ds_add_u32 into the
// [bin][16 rows] histogram of the VALU kernel (41 KB, 3 blocks per CU)
typedef float float4v __attribute__((ext_vector_type(4)));
template <int UNR>
__global__ __launch_bounds__(256) void probe_mfma16(const float4* __restrict__ col, int K, int base,
                                                    uint32_t* __restrict__ out, uint64_t* clk) {
    __shared__ __align__(16) uint32_t hist[(kGuard + kNB) * R];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t ha = (uint32_t)(size_t)(lds_u32*)hist;
    const int j = lane & 15, k = lane >> 4;
    const uint32_t hoff = ha + 4u * (uint32_t)j - 64u * (uint32_t)(base - kGuard);
    for (int q = tid; q < (kGuard + kNB) * R; q += 256) hist[q] = 0;
    const float4 rj = col[blockIdx.x * 16 + j];
    const float b = k == 0 ? rj.x : k == 1 ? rj.y : k == 2 ? rj.z : 1.0f;
    const float nj = rj.x * rj.x + rj.y * rj.y + rj.z * rj.z + 1e-12f;
    const float4v c = {nj, nj, nj, nj};
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const int ntiles = (K + 15) / 16;
    const float* cf = reinterpret_cast<const float*>(col);
    float a = cf[(size_t)((w * 16 + j) % K) * 4 + k];
    if (UNR == 1) {
        for (int t = w; t < ntiles; t += 4) {
            const int tn = t + 4 < ntiles ? t + 4 : t;
            const float an = cf[(size_t)(tn * 16 + j) * 4 + k];
            const float4v d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; q++) lds_inc(lshl6_add(__float_as_uint(d[q]) >> kBinShift, hoff));
            a = an;
        }
    } else {
        // UNR tiles per step: their MFMAs issued together, the next step's operands loaded ahead
        float av[UNR], an[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) av[u] = cf[(size_t)(((w * UNR + u) * 16 + j) % K) * 4 + k];
        for (int t = w * UNR; t < ntiles; t += 4 * UNR) {
#pragma unroll
            for (int u = 0; u < UNR; u++) {
                const int tn = min(t + 4 * UNR + u, ntiles - 1);
                an[u] = cf[(size_t)(tn * 16 + j) * 4 + k];
            }
            float4v d[UNR];
#pragma unroll
            for (int u = 0; u < UNR; u++) d[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b, c, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < UNR; u++)
#pragma unroll
                for (int q = 0; q < 4; q++) lds_inc(lshl6_add(__float_as_uint(d[u][q]) >> kBinShift, hoff));
#pragma unroll
            for (int u = 0; u < UNR; u++) av[u] = an[u];
        }
    }
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0 && blockIdx.x == 0) *clk = t1 - t0;
    uint32_t s = 0;
    for (int q = tid; q < (kGuard + kNB) * R; q += 256) s += hist[q] * (uint32_t)q;
    out[blockIdx.x * 256 + tid] = s;
}

template <int V>
float run(const float* X, const float* Y, const float* Z, int K, int rows, int base, uint32_t* out,
          uint64_t* clk, uint64_t* hclk) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    probe<V><<<rows / R, 256>>>(X, Y, Z, K, base, out, clk);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) probe<V><<<rows / R, 256>>>(X, Y, Z, K, base, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(hclk, clk, 8, hipMemcpyDeviceToHost);
    return ms / reps;
}

int main() {
    const int K = 10000, rows = 131072;
    std::mt19937 g(1);
    std::normal_distribution<float> n(0.f, 3e-5f);
    std::vector<float> h(3 * K);
    for (int i = 0; i < K; i++) {
        h[i] = 0.1f + n(g);
        h[K + i] = 0.2f + n(g);
        h[2 * K + i] = 0.3f + n(g);
    }
    float* d;
    hipMalloc(&d, 4 * 3 * K);
    hipMemcpy(d, h.data(), 4 * 3 * K, hipMemcpyHostToDevice);
    uint32_t* out;
    hipMalloc(&out, 4 * rows / R * 256);
    uint64_t* clk;
    hipMalloc(&clk, 8);
    // bins: s ~ 1e-9 .. 1e-8: exponent of 1e-12 (bias) minus a few binades -> base
    const float sref = 1e-12f * 0.5f;
    const int base = (int)(__builtin_bit_cast(uint32_t, sref) >> kBinShift) - 8;
    const double wd = (double)rows * K / 64.0;  // wave-distance instructions
    int dev;
    hipGetDevice(&dev);
    int mhz = 0;
    hipDeviceGetAttribute(&mhz, hipDeviceAttributeClockRate, dev);
    for (int v = 0; v < 7; v++) {
        if (v == 4) continue;
        uint64_t hc = 0;
        float ms = v == 0 ? run<0>(d, d + K, d + 2 * K, K, rows, base, out, clk, &hc)
                 : v == 1 ? run<1>(d, d + K, d + 2 * K, K, rows, base, out, clk, &hc)
                 : v == 2 ? run<2>(d, d + K, d + 2 * K, K, rows, base, out, clk, &hc)
                 : v == 3 ? run<3>(d, d + K, d + 2 * K, K, rows, base, out, clk, &hc)
                 : v == 5 ? run<5>(d, d + K, d + 2 * K, K, rows, base, out, clk, &hc)
                          : run<6>(d, d + K, d + 2 * K, K, rows, base, out, clk, &hc);
        const double cyc = ms * 1e-3 * 2.4e9 * 1024.0 / wd;
        printf("variant %d: %.3f ms  %.1f cycles (2.4 GHz) per wave-distance per SIMD  block0 memtime %llu\n",
               v, ms, cyc, (unsigned long long)hc);
    }
    {
        // variant 4: f16 operands, 2 x 8 halfs per column (rows use the same array)
        std::vector<_Float16> hv((size_t)rows * 16);
        for (size_t q = 0; q < hv.size(); q++) hv[q] = (_Float16)(__builtin_fabsf(0.5f + 0.25f * n(g) / 3e-5f) * 0.125f);
        _Float16* dA;
        hipMalloc(&dA, hv.size() * 2);
        hipMemcpy(dA, hv.data(), hv.size() * 2, hipMemcpyHostToDevice);
        const size_t shm = (size_t)(kGuard + kNB) * R32 * 4;
        hipFuncSetAttribute((const void*)probe_mfma, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        const int b32 = (int)(__builtin_bit_cast(uint32_t, 1e-9f) >> kBinShift) - 16;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        probe_mfma<<<rows / R32, 256, shm>>>((const half8*)dA, K, b32, out, clk);
        hipEventRecord(e0);
        for (int r = 0; r < 5; r++) probe_mfma<<<rows / R32, 256, shm>>>((const half8*)dA, K, b32, out, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        uint64_t hc;
        hipMemcpy(&hc, clk, 8, hipMemcpyDeviceToHost);
        printf("variant 4 (mfma, 32 rows/block, %zu B LDS): %.3f ms  %.1f cycles per wave-distance per SIMD  memtime %llu  err %s\n",
               shm, ms, ms * 1e-3 * 2.4e9 * 1024.0 / wd, (unsigned long long)hc, hipGetErrorString(hipGetLastError()));
    }
    {
        // variant 7: columns as float4 (x', y', z', |x'|^2 as -2x' ... timing only): centered,
        // A = -2 u, n; B = u, 1
        std::vector<float4> hc(rows);
        for (int i = 0; i < rows; i++) {
            const float x = h[i % K] - 0.1f, y = h[K + i % K] - 0.2f, z = h[2 * K + i % K] - 0.3f;
            hc[i] = make_float4(-2.f * x, -2.f * y, -2.f * z, x * x + y * y + z * z);
        }
        float4* dc;
        hipMalloc(&dc, rows * 16);
        hipMemcpy(dc, hc.data(), rows * 16, hipMemcpyHostToDevice);
        const int b16 = (int)(__builtin_bit_cast(uint32_t, 1e-12f) >> kBinShift) - 16;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        auto go = [&](auto kern, const char* name) {
            kern<<<rows / 16, 256>>>(dc, K, b16, out, clk);
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++) kern<<<rows / 16, 256>>>(dc, K, b16, out, clk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 5;
            printf("variant 7 (%s): %.3f ms  %.1f cycles per wave-distance per SIMD  err %s\n",
                   name, ms, ms * 1e-3 * 2.4e9 * 1024.0 / wd, hipGetErrorString(hipGetLastError()));
        };
        go(probe_mfma16<1>, "mfma 16x16x4 f32, 16 rows/block");
        go(probe_mfma16<2>, "same, 2 tiles per step");
        go(probe_mfma16<4>, "same, 4 tiles per step");
    }
    return 0;
}
