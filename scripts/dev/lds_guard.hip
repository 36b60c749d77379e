// Probe: does any kernel of the pipeline write into ANOTHER workgroup's LDS?
// A guard kernel (256 threads, nw words per thread of dynamic LDS) fills its allocation with a
// known pattern, then re-reads it until `spin` ticks of the 100 MHz real-time counter have
// passed, recording every word that changed (and repairing it).  Launched on a stream of its
// own beside the pipeline's streams, its workgroups share CUs with the pipeline's kernels; a
// word that changes under it was written by someone else.
// hipcc -O3 -ffp-contract=off -fno-slp-vectorize -fPIC -shared --offload-arch=gfx950 scripts/dev/lds_guard.hip -o scripts/dev/liblds_guard.so
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ uint32_t pat(uint32_t seed, uint32_t blk, uint32_t idx) {
    uint32_t x = seed ^ (blk * 0x9E3779B9u) ^ (idx * 0x85EBCA6Bu);
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

// out[0] = mismatches, out[1] = records written, out[2] = guard workgroups that finished,
// out[3] = check rounds (sum), records from out[16]: 8 words each
__global__ __launch_bounds__(256) void guard_kernel(int nw, long long spin, uint32_t seed,
                                                    uint32_t* __restrict__ out, int max_rec) {
    extern __shared__ uint32_t g[];
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    for (int k = 0; k < nw; k++) g[k * 256 + tid] = pat(seed, blk, k * 256 + tid);
    __syncthreads();
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    uint32_t rounds = 0;
    long long now = t0;
    do {
        for (int k = 0; k < nw; k++) {
            const uint32_t e = pat(seed, blk, k * 256 + tid);
            const uint32_t v = g[k * 256 + tid];
            if (v != e) {
                atomicAdd(&out[0], 1u);
                const uint32_t r = atomicAdd(&out[1], 1u);
                uint32_t hw, xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                if ((int)r < max_rec) {
                    uint32_t* o = out + 16 + 8 * r;
                    o[0] = blk;
                    o[1] = k * 256 + tid;
                    o[2] = v;
                    o[3] = e;
                    o[4] = hw;
                    o[5] = xcc;
                    o[6] = (uint32_t)(now - t0);
                    o[7] = (uint32_t)((unsigned long long)now & 0xffffffffu);
                }
                g[k * 256 + tid] = e;
            }
        }
        rounds++;
        now = (long long)__builtin_amdgcn_s_memrealtime();
    } while (now - t0 < spin);
    __syncthreads();
    if (tid == 0) {
        atomicAdd(&out[2], 1u);
        atomicAdd(&out[3], rounds);
    }
}

// Probe 2: the pruning pass's packed-f32 test (lip_prune_rows: two rows per thread share
// v_pk_add / v_pk_mul / v_pk_fma) against the same arithmetic in scalar f32, on deterministic
// inputs staged in LDS like the kernel's; every (thread, reference) whose packed result differs
// from the scalar one is counted.  Run beside the pipeline's kernels on other streams.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void pk_probe_kernel(long long spin, uint32_t seed,
                                                       uint32_t* __restrict__ out, int max_rec) {
    __shared__ float4 refs[512];
    __shared__ float4 act[512];
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    auto u01 = [&](uint32_t i) { return (float)(pat(seed, blk, i) >> 8) * 0x1p-24f - 0.5f; };
    for (int c = tid; c < 512; c += 256) {
        refs[c] = make_float4(u01(4 * c), u01(4 * c + 1), u01(4 * c + 2), 0.25f * u01(4 * c + 3) + 0.125f);
        act[c] = make_float4(u01(9000 + 4 * c), u01(9001 + 4 * c), u01(9002 + 4 * c), 0.f);
    }
    __syncthreads();
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    long long now = t0;
    uint32_t rounds = 0;
    do {
        const float4 a0 = act[2 * tid], a1 = act[2 * tid + 1];
        const f32x2 xi = {a0.x, a1.x}, yi = {a0.y, a1.y}, zi = {a0.z, a1.z};
        for (int q = 0; q < 512; q += 8) {
            float4 r[8];
#pragma unroll
            for (int u = 0; u < 8; u++) r[u] = refs[q + u];
            uint32_t bad = 0;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const f32x2 dx = xi - r[u].x, dy = yi - r[u].y, dz = zi - r[u].z;
                f32x2 s2 = dx * dx;
                s2 = __builtin_elementwise_fma(dy, dy, s2);
                s2 = __builtin_elementwise_fma(dz, dz, s2);
                const f32x2 d = s2 - r[u].w;
                // scalar reference of the lo and hi halves
                // (operands laundered through empty asm: no sharing with the packed path)
                float sx0 = a0.x, sy0 = a0.y, sz0 = a0.z, sx1 = a1.x, sy1 = a1.y, sz1 = a1.z;
                float rx = r[u].x, ry = r[u].y, rz = r[u].z, rw = r[u].w;
                asm volatile("" : "+v"(sx0), "+v"(sy0), "+v"(sz0), "+v"(sx1), "+v"(sy1), "+v"(sz1));
                asm volatile("" : "+v"(rx), "+v"(ry), "+v"(rz), "+v"(rw));
                const float ex0 = sx0 - rx, ey0 = sy0 - ry, ez0 = sz0 - rz;
                const float ex1 = sx1 - rx, ey1 = sy1 - ry, ez1 = sz1 - rz;
                const float t0s = __builtin_fmaf(ez0, ez0, __builtin_fmaf(ey0, ey0, ex0 * ex0)) - rw;
                const float t1s = __builtin_fmaf(ez1, ez1, __builtin_fmaf(ey1, ey1, ex1 * ex1)) - rw;
                const bool b0 = __float_as_uint(d[0]) != __float_as_uint(t0s);
                const bool b1 = __float_as_uint(d[1]) != __float_as_uint(t1s);
                if (b0 | b1) {
                    bad++;
                    const uint32_t k = atomicAdd(&out[1], 1u);
                    if ((int)k < max_rec) {
                        uint32_t* o = out + 16 + 8 * k;
                        o[0] = blk;
                        o[1] = tid;
                        o[2] = q + u;
                        o[3] = __float_as_uint(d[0]);
                        o[4] = __float_as_uint(t0s);
                        o[5] = __float_as_uint(d[1]);
                        o[6] = __float_as_uint(t1s);
                        o[7] = (uint32_t)(now - t0);
                    }
                }
            }
            if (bad) atomicAdd(&out[0], bad);
        }
        rounds++;
        now = (long long)__builtin_amdgcn_s_memrealtime();
    } while (now - t0 < spin);
    __syncthreads();
    if (tid == 0) {
        atomicAdd(&out[2], 1u);
        atomicAdd(&out[3], rounds);
    }
}

extern "C" int pk_probe_launch(void* stream, int nblocks, long long spin, uint32_t seed,
                               uint32_t* out, int max_rec) {
    hipLaunchKernelGGL(pk_probe_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, spin,
                       seed, out, max_rec);
    return (int)hipGetLastError();
}

// Synthetic aggressors: one instruction class in a loop until `spin` ticks have passed
// (kind 0: v_mfma_i32_32x32x32_i8, 1: v_mfma_f32_32x32x16_bf16, 2: v_fma_f64 chains,
//  3: v_mfma_i32_16x16x64_i8, 4: v_mfma_f64_16x16x4f64)
typedef int i32x4v __attribute__((ext_vector_type(4)));
typedef int i32x16v __attribute__((ext_vector_type(16)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef double f64x4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void aggressor_kernel(int kind, long long spin, uint32_t* out) {
    const uint32_t tid = threadIdx.x;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    uint32_t acc_out = 0;
    if (kind == 0 || kind == 3) {
        i32x4v a = {(int)tid, 3, 5, 7}, b = {11, (int)tid, 13, 17};
        i32x16v c = {};
        i32x4v c4 = {};
        do {
            for (int k = 0; k < 64; k++) {
                if (kind == 0) c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
                else c4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c4, 0, 0, 0);
            }
        } while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < spin);
        for (int k = 0; k < 16; k++) acc_out += (uint32_t)c[k];
        for (int k = 0; k < 4; k++) acc_out += (uint32_t)c4[k];
    } else if (kind == 1) {
        bf16x8v a, b;
        for (int k = 0; k < 8; k++) {
            a[k] = (__bf16)(float)(tid + k);
            b[k] = (__bf16)(float)(k);
        }
        f32x16v c = {};
        do {
            for (int k = 0; k < 64; k++) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
        } while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < spin);
        for (int k = 0; k < 16; k++) acc_out += __float_as_uint(c[k]);
    } else if (kind == 2) {
        double x[8];
        for (int k = 0; k < 8; k++) x[k] = 1.0 + tid * 1e-3 + k;
        do {
            for (int k = 0; k < 64; k++)
#pragma unroll
                for (int u = 0; u < 8; u++) x[u] = __builtin_fma(x[u], 0.999999, 1e-9);
        } while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < spin);
        for (int k = 0; k < 8; k++) acc_out += (uint32_t)__double_as_longlong(x[k]);
    } else if (kind == 4) {
        double a = 1.0 + tid, b = 2.0;
        f64x4v c = {};
        do {
            for (int k = 0; k < 64; k++) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
        } while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < spin);
        for (int k = 0; k < 4; k++) acc_out += (uint32_t)__double_as_longlong(c[k]);
    }
    if (acc_out == 0x12345678u) out[0] = acc_out;  // (keeps the loop)
}

// Probe 3: one instruction class per mode, a per-thread checksum of its results over 512
// LDS-staged operands per round, against a golden checksum the same launch shape wrote alone
// (write = 1): mode 0 packed f32 (lo / hi halves apart), 1 scalar f32, 2 fp64, 3 int32
// (mad24 / mul_lo / shifts), 4 packed f16.  out[0] = rounds whose lo checksum differed, out[1] =
// hi, out[2] = workgroups, out[3] = rounds
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void valu_gold_kernel(int mode, int write, long long spin,
                                                        uint32_t* __restrict__ gold,
                                                        uint32_t* __restrict__ out) {
    __shared__ float4 refs[512];
    __shared__ float4 act[512];
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    auto u01 = [&](uint32_t i) { return (float)(pat(0x5151u, blk, i) >> 8) * 0x1p-24f - 0.5f; };
    for (int c = tid; c < 512; c += 256) {
        refs[c] = make_float4(u01(4 * c), u01(4 * c + 1), u01(4 * c + 2), 0.25f * u01(4 * c + 3) + 0.125f);
        act[c] = make_float4(u01(9000 + 4 * c), u01(9001 + 4 * c), u01(9002 + 4 * c), 0.f);
    }
    __syncthreads();
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    uint32_t rounds = 0, bad_lo = 0, bad_hi = 0;
    do {
        const float4 a0 = act[2 * tid], a1 = act[2 * tid + 1];
        uint32_t ck0 = 0, ck1 = 0;
        for (int q = 0; q < 512; q += 8) {
            float4 r[8];
#pragma unroll
            for (int u = 0; u < 8; u++) r[u] = refs[q + u];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                uint32_t v0 = 0, v1 = 0;
                if (mode == 0) {
                    const f32x2 xi = {a0.x, a1.x}, yi = {a0.y, a1.y}, zi = {a0.z, a1.z};
                    const f32x2 dx = xi - r[u].x, dy = yi - r[u].y, dz = zi - r[u].z;
                    f32x2 s2 = dx * dx;
                    s2 = __builtin_elementwise_fma(dy, dy, s2);
                    s2 = __builtin_elementwise_fma(dz, dz, s2);
                    const f32x2 d = s2 - r[u].w;
                    v0 = __float_as_uint(d[0]);
                    v1 = __float_as_uint(d[1]);
                } else if (mode == 1) {
                    const float ex0 = a0.x - r[u].x, ey0 = a0.y - r[u].y, ez0 = a0.z - r[u].z;
                    const float ex1 = a1.x - r[u].x, ey1 = a1.y - r[u].y, ez1 = a1.z - r[u].z;
                    v0 = __float_as_uint(__builtin_fmaf(ez0, ez0, __builtin_fmaf(ey0, ey0, ex0 * ex0)) - r[u].w);
                    v1 = __float_as_uint(__builtin_fmaf(ez1, ez1, __builtin_fmaf(ey1, ey1, ex1 * ex1)) - r[u].w);
                } else if (mode == 2) {
                    const double ex = (double)a0.x - r[u].x, ey = (double)a0.y - r[u].y, ez = (double)a1.z - r[u].z;
                    const double d = __builtin_fma(ez, ez, __builtin_fma(ey, ey, ex * ex)) - r[u].w;
                    const uint64_t b = (uint64_t)__double_as_longlong(d);
                    v0 = (uint32_t)b;
                    v1 = (uint32_t)(b >> 32);
                } else if (mode == 3) {
                    const uint32_t x = __float_as_uint(a0.x), y = __float_as_uint(r[u].y);
                    v0 = __umul24(x, y) + (x >> (y & 15)) + x * y;
                    v1 = (x ^ y) + __umulhi(x, y);
                } else {
                    const f16x2 xi = {(_Float16)a0.x, (_Float16)a1.x}, yi = {(_Float16)a0.y, (_Float16)a1.y};
                    const f16x2 rx = {(_Float16)r[u].x, (_Float16)r[u].x}, ry = {(_Float16)r[u].y, (_Float16)r[u].y};
                    const f16x2 dx = xi - rx, dy = yi - ry;
                    const f16x2 d = __builtin_elementwise_fma(dy, dy, dx * dx);
                    v0 = (uint32_t)__builtin_bit_cast(uint16_t, d[0]);
                    v1 = (uint32_t)__builtin_bit_cast(uint16_t, d[1]);
                }
                ck0 = ((ck0 << 5) | (ck0 >> 27)) ^ v0;
                ck1 = ((ck1 << 5) | (ck1 >> 27)) ^ v1;
            }
        }
        uint32_t* g = gold + ((size_t)blk * 256 + tid) * 2;
        if (write) {
            g[0] = ck0;
            g[1] = ck1;
        } else {
            bad_lo += g[0] != ck0;
            bad_hi += g[1] != ck1;
        }
        rounds++;
    } while (!write && (long long)__builtin_amdgcn_s_memrealtime() - t0 < spin);
    if (bad_lo) atomicAdd(&out[0], bad_lo);
    if (bad_hi) atomicAdd(&out[1], bad_hi);
    __syncthreads();
    if (tid == 0) {
        atomicAdd(&out[2], 1u);
        atomicAdd(&out[3], rounds);
    }
}

extern "C" int valu_gold_launch(void* stream, int nblocks, int mode, int write, long long spin,
                                uint32_t* gold, uint32_t* out) {
    hipLaunchKernelGGL(valu_gold_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, mode,
                       write, spin, gold, out);
    return (int)hipGetLastError();
}

extern "C" int aggressor_launch(void* stream, int nblocks, int kind, long long spin, uint32_t* out) {
    hipLaunchKernelGGL(aggressor_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, kind,
                       spin, out);
    return (int)hipGetLastError();
}

extern "C" int lds_guard_launch(void* stream, int nblocks, int nw, long long spin, uint32_t seed,
                                uint32_t* out, int max_rec) {
    const size_t shmem = (size_t)nw * 256 * 4;
    if (shmem > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)guard_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)shmem);
        if (e != hipSuccess) return (int)e;
    }
    hipLaunchKernelGGL(guard_kernel, dim3(nblocks), dim3(256), shmem, (hipStream_t)stream, nw, spin,
                       seed, out, max_rec);
    return (int)hipGetLastError();
}
