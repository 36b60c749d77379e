// Speed-of-light probe for the glibc-replay sampler (VERDICT r05 "next" 1).
//
// The same per-lane backwards ring (r[n-31] = r[n] - r[n-3], the glibc TYPE_3 recurrence run in
// reverse), the same Granlund-Montgomery magic quotient + v_mad_i32_i24 remainder, the same launch
// shape as sampler_kernel<0> (one 64-lane wave per 64 iterations, grid (waves, pairs), the pair's
// draws i = M-1 .. 1 in blocks of 31 with the block's divisor constants by scalar loads) -- with
// the bookkeeping cut away stage by stage:
//   V0  generator only:                 ring subtract, >> 1, xor into an accumulator
//   V1  generator + modulo (the floor):  + mulhi, shift, mad_i24 remainder
//   V2  + the i >= s bookkeeping on every step: clamp, LDS masked OR with return, bit extract
//       and placement, one coalesced selection-word store per block (no prefix / mixed blocks)
//   V3  V2 with the magic shift as a compile-time constant per power-of-two range of d
//   V4  V3 with the selection bit accumulated through the carry (v_and + v_add_co + v_addc)
// The real kernel (prefix and mixed blocks included) is timed beside it by sampler_sol.py through
// the library's own stage timer.  Results are not the sampler's (the windows are random words):
// this measures instruction cost, not parity.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC scripts/dev/sampler_sol.hip \
//         -o devlibs/libsampler_sol.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __forceinline__ uint32_t mskor_rtn(uint32_t addr, uint32_t mask, uint32_t data) {
    uint32_t old;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(old) : "v"(addr), "v"(mask), "v"(data)
                 : "memory");
    return old;
}
__device__ __forceinline__ void wait_lag(uint32_t& o, int v) {
    if (30 - v >= 8) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(o) : : "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(o) : : "memory");
}
__device__ __forceinline__ uint32_t mad24(uint32_t q, int negd, uint32_t x) {
    int j;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(j) : "v"(q), "s"(negd), "v"(x));
    return (uint32_t)j;
}

constexpr int kLag = 8;

// one block of 31 steps i0 .. i0-30 (all >= 1 when FULL); SH >= 0: the magic shift as a constant
template <int V, int SH, bool I24>
__device__ __forceinline__ uint32_t sol_block(uint32_t (&ring)[31], uint32_t bm_lane, int i0, int s,
                                              const uint64_t* __restrict__ mtab, uint32_t& acc) {
    uint64_t mt[31];
#pragma unroll
    for (int u = 0; u < 31; u++) mt[u] = mtab[i0 - u + 1];
    uint32_t olds[31], pos[31], bits[31];
    uint32_t nw = 0;
#pragma unroll
    for (int u = 0; u < 31 + kLag; u++) {
        if (u < 31) {
            const int d = i0 - u + 1;
            const int slot = 30 - u;
            const uint32_t rv = ring[slot];
            ring[slot] = rv - ring[(slot + 28) % 31];
            const uint32_t x = rv >> 1;
            if (V == 0) { acc ^= x; continue; }
            const uint32_t hi = __umulhi(x, (uint32_t)mt[u]);
            const uint32_t q = SH >= 0 ? hi >> SH : hi >> (uint32_t)(mt[u] >> 32);
            uint32_t j = I24 ? mad24(q, -d, x) : x - q * (uint32_t)d;
            if (V == 1) { acc ^= j; continue; }
            j = min(j, (uint32_t)s);
            uint32_t a;
            asm("v_lshl_add_u32 %0, %1, 8, %2" : "=v"(a) : "v"(j >> 5), "v"(bm_lane));
            bits[u] = 1u << (j & 31);
            olds[u] = mskor_rtn(a, bits[u], 0u);
            pos[u] = j;
        }
        const int v = u - kLag;
        if (V >= 2 && v >= 0) {
            wait_lag(olds[v], v);
            if (V == 4) {
                // carry = (old & bit) != 0, shifted in from the bottom (bit order reversed)
                const uint32_t t = olds[v] & bits[v];
                uint32_t c;
                asm volatile("v_add_co_u32 %0, vcc, -1, %1\n\tv_addc_co_u32 %2, vcc, %2, %2, vcc"
                             : "=&v"(c), "+v"(nw) : "v"(t) : "vcc");
                (void)c;
            } else {
                nw |= __builtin_amdgcn_ubfe(olds[v], pos[v], 1) << v;
            }
        }
    }
    return V == 4 ? __builtin_bitreverse32(nw) >> 1 : nw;
}

template <int V>
__global__ __launch_bounds__(64) void sol_kernel(const int32_t* __restrict__ counts, int nwaves,
                                                 double frac, const uint64_t* __restrict__ mtab,
                                                 uint32_t* __restrict__ out, int nbw, int nalloc) {
    extern __shared__ uint32_t bm[];
    const int p = blockIdx.y, w = blockIdx.x, lane = threadIdx.x;
    const int M = counts[p];
    const int s = (int)(M * frac);
    if (V >= 2)
        for (int k = 0; k < nalloc; k++)
            bm[k * 64 + lane] = k < (s >> 5) ? ~0u : k == (s >> 5) ? (1u << (s & 31)) - 1u : 0u;
    uint32_t ring[31];
    uint32_t h = (uint32_t)(p * 7919 + w * 104729 + lane * 31337) | 1u;
#pragma unroll
    for (int t = 0; t < 31; t++) {
        h ^= h << 13; h ^= h >> 17; h ^= h << 5;
        ring[t] = h;
    }
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    uint32_t* o = out + ((size_t)p * nwaves + w) * (size_t)nbw * 64 + lane;
    uint32_t acc = 0;
    int i = M - 1, b = 0;
    while (i - 30 >= 1) {
        uint32_t word;
        if (V == 3 || V == 4) {
            // the shift is constant when the block's 31 divisors share ceil(log2 d)
            // ceil(log2 d) = bit length of d - 1: d = i + 1 .. i - 29
            const int lhi = 32 - __builtin_clz((uint32_t)i);
            const int llo = 32 - __builtin_clz((uint32_t)(i - 30));
            const int l = lhi == llo ? lhi : -1;
            switch (l) {
#define SOL_CASE(L) case L: word = sol_block<V, L - 1, true>(ring, bm_lane, i, s, mtab, acc); break;
                SOL_CASE(9) SOL_CASE(10) SOL_CASE(11) SOL_CASE(12) SOL_CASE(13)
#undef SOL_CASE
                default: word = i - 30 >= 256 ? sol_block<V, -1, true>(ring, bm_lane, i, s, mtab, acc)
                                              : sol_block<V, -1, false>(ring, bm_lane, i, s, mtab, acc);
                         break;
            }
        } else {
            word = i - 30 >= 256 ? sol_block<V, -1, true>(ring, bm_lane, i, s, mtab, acc)
                                 : sol_block<V, -1, false>(ring, bm_lane, i, s, mtab, acc);
        }
        if (V >= 2) o[(size_t)b * 64] = word;
        i -= 31;
        b++;
    }
    o[(size_t)b * 64] = acc ^ (uint32_t)i;
}

}  // namespace

extern "C" {
// n_pairs pairs with counts[p] matches (device), iterations -> grid; mtab = the magic table
// (device, d = 0 .. 65538: m_d | (l_d - 1) << 32); out = nbw words per lane (device).
// Returns the kernel time in ms (hipEvent), or -1 on an error.
float sol_run(int variant, const int32_t* counts, int n_pairs, int iters, double frac,
              const uint64_t* mtab, uint32_t* out, int nbw, int nalloc, int reps) {
    const int nwaves = (iters + 63) / 64;
    const size_t shmem = (size_t)nalloc * 64 * 4;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; r++) {
        switch (variant) {
#define SOL_L(V) case V: hipLaunchKernelGGL(sol_kernel<V>, dim3(nwaves, n_pairs), dim3(64), shmem, 0, \
                                             counts, nwaves, frac, mtab, out, nbw, nalloc); break;
            SOL_L(0) SOL_L(1) SOL_L(2) SOL_L(3) SOL_L(4)
#undef SOL_L
            default: return -1.f;
        }
    }
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return hipGetLastError() == hipSuccess ? ms / reps : -1.f;
}
}
