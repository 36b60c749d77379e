// matcher.hip -- gfx950 kernels of the exact k=2 + ratio-0.3 matcher
// (src/feature_matcher.cpp:42-59, FlannBasedMatcher::knnMatch(k = 2) + the ratio test; the
// exact brute-force limit of FLANN's randomized KD-tree, distances in flann::L2<float>'s order).
//
// Compiled with -ffp-contract=off (the flann::L2 accumulation, the ratio test and sqrtf must
// round like the reference's x86-64 code), -mllvm -amdgpu-mfma-vgpr-form (the filter's MFMA
// accumulators live in VGPRs: no v_accvgpr_read per element before the bounds epilogue) and
// -fno-honor-nans (descriptors are finite: no NaN-quieting ops in the filter's min trees).
//
// Kernels: knn2_split (train rows -> bf16(-2 t), |t|^2), knn2_filter (ONE bf16 MFMA pass:
// per-query upper bounds + provisional candidates), knn2_rescore (exact distances of the
// candidates that survive the final bound), knn2_sweep (exact sweep for overflowed lists),
// knn2_exact (the packed-FP32 sweep: the non-MFMA matcher), knn2_fold / knn2_merge (chunk fold,
// ratio test, order-preserving compaction).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "erp_device.hpp"
#include "erp_kernels.hpp"
#include "erp_launch.hpp"

namespace erp {

namespace {

constexpr float kInf = __builtin_huge_valf();

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int wave_lane() { return threadIdx.x & 63; }

// exclusive scan over a block of BLOCK threads (BLOCK multiple of 64, <= 1024)
template <int BLOCK>
__device__ int block_exclusive_scan(int v, int* ws, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) ws[wid] = x;
    __syncthreads();
    if (wid == 0) {
        int t = lane < BLOCK / 64 ? ws[lane] : 0;
#pragma unroll
        for (int o = 1; o < BLOCK / 64; o <<= 1) {
            const int y = __shfl_up(t, o, 64);
            if (lane >= o) t += y;
        }
        if (lane < BLOCK / 64) ws[lane] = t;
    }
    __syncthreads();
    const int base = wid ? ws[wid - 1] : 0;
    *total = ws[BLOCK / 64 - 1];
    __syncthreads();
    return base + x - v;
}

// ===================================================================== matcher =========
// Exact k=2 in two steps (the result is identical to a brute-force sweep in the flann::L2
// order, lowest train index winning ties):
//  1. knn2_filter: ONE bf16 MFMA product per (query, train) pair gives u' = tu - 2 qh.th with
//     qh = bf16(q), th = bf16(t) (|q_i - qh_i| <= 2^-8 |q_i|) and tu = |t|^2 (1 + eps) loaded
//     as the MFMA's C operand (the B operand holds bf16(-2 t), exact scaling), so the element
//     needs no epilogue arithmetic.  With S = |q|^2 + |t|^2 and a = |q|^2 + |t|^2 - 2 qh.th,
//       |q.t - qh.th| <= 2^-7 (1 + 2^-9) |q||t| <= 2^-8 (1 + 2^-9) S,
//     and the f32 accumulation of the 64 exact bf16 products, the f32 norms, e's own rounding
//     (64 f32 squares summed: <= 2^-16.9 S) and the few f32 roundings of u' and the bounds
//     (each <= 2^-24 3 S) add < 2e-5 S, so |a - e| <= 0.0078444 S for the reference's exact
//     f32 value e, against eps = 0x1.08p-7 = 0.0080566: u = a + eps S >= e + 2.1e-4 S and
//     l = a - eps S <= e - 2.1e-4 S.  QB = |q|^2 (1 + eps) + tiny turns u' into u = u' + QB.
//     Running bound: every lane keeps the two smallest of its tile minima of u' (the lane's
//     16 rows of a tile; since r06w -- r05 kept (tile, 8-row group) minima, and before it the
//     groups were fixed, all tiles' elements 0-7 and all 8-15, looser whenever both smallest
//     rows fell in one of them: rescore 1.21 -> 0.89 ms per step), two minima of disjoint row
//     sets, so the second smallest of a query's four kept minima (both lane halves) G bounds
//     the chunk's second smallest u' from above, and G + QB >= e_(2) (the
//     true second-neighbour distance).  A row t with e_t <= e_(2) (both neighbours and all
//     their ties) has l_t <= e_(2) - 2.1e-4 S_t <= G + QB, i.e.
//       u'_t <= G + (QB - QL) + 2 eps |t|^2 <= thr := G + (QB - QL) + teM,
//     QL = |q|^2 (1 - eps) - tiny, teM = 2 eps max_t |t|^2 (per pair, rounded up): every such
//     row is stored as a provisional candidate with the lower bound l* = u'_t + QL - teM <= l_t.
//     G only falls as the chunk proceeds, so the set stored is a superset of the rows with
//     l_t <= the chunk's final bound.  The first stage of the chunk runs bounds-only (with no
//     bound yet every row would qualify) and is recomputed for candidates after the last.
//  2. knn2_rescore: U2 = the second smallest bound over all chunks (>= e_(2)); candidates with
//     l* <= U2 are re-scored exactly in the flann order, one lane per (query, chunk); a list
//     that overflowed kCandSlots gets an exact sweep of its chunk.
// Matrix layout for v_mfma_f32_32x32x16_bf16: A = 32 train rows x 16 dims (LDS), B = 16 dims x
// 32 queries (registers, rounded once), C/D = 32 x 32 with the query on the lane (col = lane &
// 31) and 16 train rows in the registers (row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)).  A wave
// owns 64 queries (two B operands share every A fragment and the C operand), a block 4 waves x
// 64 queries x one train chunk.  Per 32-row tile a wave issues 8 MFMAs (256 cycles) against
// 8 ds_read_b128 and ~24 VALU (the two group-minimum trees and the candidate test).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef const __attribute__((address_space(1))) void* glb_vptr;
constexpr int kFW = 64;             // queries per wave
constexpr int kFQ = 4 * kFW;        // queries per block
constexpr int kFT = 32;             // train rows per tile
constexpr int kFST = 4;             // 32-row tiles per LDS stage (one barrier per stage)
constexpr float kFEps = 0x1.08p-7f;
constexpr float kFTiny = 0x1p-100f; // absolute floor (flushed denormals)
constexpr float kFMargin = 0x1p-20f;

// LDS stage (one of two): 128 train rows x 128 B (64 bf16), filled by LDS-DMA
// (global_load_lds: lane l of a 1-KB wave piece lands at piece + 16 l, so a piece holds 8 rows
// unpadded).  The 16-B pieces of row r are XOR-swizzled, position c' = c ^ ((r >> 1) & 7), on
// the global (source) side: the b128 A-fragment reads of a wave (16 rows of one lane group,
// one piece each) then fall on 16 distinct 4-dword bank slots (rows of either parity take all 8
// positions).  Then the stage's tu = |t|^2 (1 + eps) (+inf past the chunk).
constexpr int kFRowB = 128;
constexpr int kFHiB = kFST * kFT * kFRowB;        // 16384
constexpr int kFStageB = kFHiB + kFST * kFT * 4;  // + 512
// Tile schedule (profiles/r03g_filter_chains_ab.txt, same-box A/B per 768-pair step): 0 = the
// two query blocks' MFMA chains interleaved, both min trees after the last MFMA (2.68 ms);
// 1 = chain 0 whole, then chain 1 with chain 0's min tree between its MFMAs (2.57 ms);
// 2 = as 1, and chain 1's min tree deferred past the next tile's MFMAs (2.55 ms, 158 VGPRs).
#ifndef ERP_FILTER_CHAINS
#define ERP_FILTER_CHAINS 2
#endif
// bounds-only stages at the start of a chunk (recomputed for candidates after its last stage):
// the running bound G the candidate test compares with only falls as rows are seen, so tiles
// tested early against a loose G are stored and re-scored for nothing.  Same-box A/Bs per
// 768-pair step (profiles/r04c_ab_filter_warm.txt): 1 (until r04) filter + rescore 2.78 + 1.57
// ms; 4: 2.78 + 1.35; 8: 2.87-2.92 + 1.23 (kept, +1.5-2 % pairs/s); 12: 3.03 + 1.17; 16: 3.16 +
// 1.13 (the recomputed quarter of the chunk's MFMAs starts to cost more than it saves)
#ifndef ERP_FILTER_WARM
#define ERP_FILTER_WARM 8
#endif
constexpr int kFWarm = ERP_FILTER_WARM;
// timing ablations only (wrong results): 1 = no candidate slot stores, 2 = no staging DMAs after
// the first stage (every stage reuses the first stage's rows)
#ifndef ERP_FILTER_ABLATE
#define ERP_FILTER_ABLATE 0
#endif

__device__ __forceinline__ bf16x8 round8(const float4 a, const float4 b, float s) {
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    bf16x8 h;
#pragma unroll
    for (int k = 0; k < 8; k++) h[k] = (__bf16)(v[k] * s);
    return h;
}

__device__ __forceinline__ float sq8(const float4 a, const float4 b) {
    return a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z +
           b.w * b.w;
}

// train rows -> thi [pair][max_nt][64] = bf16(-2 t) (round to nearest; exact scaling of
// bf16(t)), tu [pair][max_nt] = |t|^2 (1 + eps) (the filter's C operand), tmaxb[pair][block] =
// the block's max |t|^2 (float bits; knn2_filter reduces a pair's blocks); four threads per row
// (16 dims each).  Block (0, p) also resets the per-call state of pair p (flags) and block (0, 0)
// the batch's (the rescore's overflow counter, the filter's sentinel row): the kernels that read
// them run after this one on the stream -- no memset launches (single-pair latency)
__global__ __launch_bounds__(256) void knn2_split_kernel(const float* __restrict__ dt,
                                                         const int64_t* __restrict__ off_t,
                                                         int max_nt, bf16x8* __restrict__ thi,
                                                         float* __restrict__ tn,
                                                         uint32_t* __restrict__ tmaxb,
                                                         int32_t* __restrict__ ovf,
                                                         uint32_t* __restrict__ sent,
                                                         int32_t* __restrict__ flags) {
    const int p = blockIdx.y, tid = threadIdx.x;
    if (blockIdx.x == 0) {
        if (flags && tid == 0) flags[p] = 0;
        if (p == 0 && tid < 33) sent[tid] = tid < 32 ? 0u : 0x7f800000u;  // 64 bf16 zeros, tu = inf
        if (ovf && p == 0 && tid == 0) ovf[0] = 0;
    }
    const int j = blockIdx.x * 64 + (tid >> 2), part = tid & 3;
    const int64_t tbase = off_t[p];
    const int nt = (int)(off_t[p + 1] - tbase);
    if (blockIdx.x * 64 >= nt) return;  // uniform
    float ss = 0.f;
    const size_t o = ((size_t)p * max_nt + j) * 8 + 2 * part;  // in bf16x8 units
    if (j < nt) {
        const float4* tp = reinterpret_cast<const float4*>(dt + (tbase + j) * kDim + 16 * part);
        const float4 a = tp[0], b = tp[1], c = tp[2], d = tp[3];
        thi[o] = round8(a, b, -2.f);
        thi[o + 1] = round8(c, d, -2.f);
        ss = sq8(a, b) + sq8(c, d);
    }
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    if (part == 0 && j < nt) tn[(size_t)p * max_nt + j] = __builtin_fmaf(ss, kFEps, ss);
    __shared__ float wmax[4];
    float m = (j < nt) ? ss : 0.f;
#pragma unroll
    for (int s = 4; s < 64; s <<= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
    if ((tid & 63) == 0) wmax[tid >> 6] = m;
    __syncthreads();
    if (tid == 0)  // |t|^2 >= 0: the float bits order like the values
        tmaxb[(size_t)p * gridDim.x + blockIdx.x] =
            __float_as_uint(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])));
}

// max |t|^2 of pair p over its split blocks' maxima (every wave of the calling block; the
// blocks past the pair's rows wrote nothing)
__device__ __forceinline__ uint32_t pair_tmax(const uint32_t* __restrict__ tmaxb, int p, int nt,
                                              int max_nt) {
    const int nbx = (max_nt + 63) / 64, nb = (nt + 63) / 64, lane = threadIdx.x & 63;
    uint32_t m = 0;
    for (int b = lane; b < nb; b += 64) m = max(m, tmaxb[(size_t)p * nbx + b]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    return m;
}

// min trees of the filter (v_min3_f32 / v_min_f32: the file is built with -fno-honor-nans, so
// the compiler drops the sNaN-quieting v_max_f32 it would put in front of every operand; the
// bounds of finite descriptors are never NaN).  Not inline asm: the hazard recognizer must see
// these reads of MFMA results (an asm v_min3 read them before the MFMA had written them).
__device__ __forceinline__ float min3f(float a, float b, float c) { return fminf(fminf(a, b), c); }
__device__ __forceinline__ float min2f(float a, float b) { return fminf(a, b); }

// second smallest of {a0, a1, b0, b1} given a0/a1 and b0/b1 in any order
__device__ __forceinline__ float second4(float a0, float a1, float b0, float b1) {
    const float m1 = fminf(a0, a1), m2 = fmaxf(a0, a1);
    const float o1 = fminf(b0, b1), o2 = fmaxf(b0, b1);
    return fminf(fmaxf(m1, o1), fminf(m2, o2));
}

// A candidate slot is one 32-B record: the tile's 16 bounds as bf16, with the tile's index
// (tile0 / 32 < 2048: rows < 65536, chunk lengths are multiples of 32) in the 16 mantissa LSBs:
// bit d of the index in dword d's low half, bit d + 8 in its high half (d < 8).  The
// knn2_rescore side widens each value by 2^-6 |v| instead of 2^-8 |v| (round to nearest: 1/2
// ulp, the replaced LSB: 1 ulp, so |v - u'| <= 3 2^-8 |v|).  Before round 3 the tile index went
// to a separate int32 array: a scattered 4-B store per slot that HBM wrote as a whole sector
// (the filter's slot writes 0.72 GB per 192-pair launch against 0.35 GB of bounds;
// ERP_CAND_TILE_ARRAY=1 keeps that layout for A/B; with the interleaved slots of
// ERP_CAND_INTERLEAVE=1 its stores coalesce, profiles/r05q_ab_slots.txt).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// v_bfi_b32: (m & b) | (~m & w) with the mask in a VGPR and the wave-uniform bits in an SGPR
// (one VALU op per dword; the compiler's AND + OR took two: a VOP3 on gfx950 reads one SGPR and
// no literal).  w is a v_cvt_pk_bf16_f32 result, not an MFMA result: no MFMA read hazard.
__device__ __forceinline__ uint32_t bfi_lsb(uint32_t m, uint32_t b, uint32_t w) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "s"(b), "v"(w));
    return r;
}
// T = the tile index spread for the embedding: bits 0-7 at 0-7, bits 8-15 at 16-23, so that
// dword d takes (T >> d) under the mask 0x00010001 (one scalar shift per dword)
__device__ __forceinline__ uint32_t cand_spread(int tile0) {
    const uint32_t ti = (uint32_t)tile0 >> 5;
    return (ti & 0xffu) | ((ti >> 8) << 16);
}
__device__ __forceinline__ bf16x8 cand_embed_tile(bf16x8 b, int g, uint32_t T) {
    u32x4 w = __builtin_bit_cast(u32x4, b);
    const uint32_t m = 0x00010001u;
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = bfi_lsb(m, T >> (4 * g + k), w[k]);
    return __builtin_bit_cast(bf16x8, w);
}
__device__ __forceinline__ int cand_tile(bf16x8 v0, bf16x8 v1) {
    const u32x4 a = __builtin_bit_cast(u32x4, v0), b = __builtin_bit_cast(u32x4, v1);
    uint32_t ti = 0;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const uint32_t w = d < 4 ? a[d] : b[d - 4];
        ti |= ((w & 1u) << d) | (((w >> 16) & 1u) << (d + 8));
    }
    return (int)(ti << 5);
}

// ERP_FILTER_MIN_WAVES = n > 0: amdgpu_waves_per_eu(n) (A/B knob; 3 for the CHAINS == 3 form)
#ifndef ERP_FILTER_MIN_WAVES
#define ERP_FILTER_MIN_WAVES (ERP_FILTER_CHAINS == 3 ? 3 : 0)
#endif
#if ERP_FILTER_MIN_WAVES > 0
#define ERP_FILTER_WAVES __attribute__((amdgpu_waves_per_eu(ERP_FILTER_MIN_WAVES)))
#else
#define ERP_FILTER_WAVES
#endif
// Slot record index of list (pair p, chunk ch, query q, lane half h), slot sl.  Default: the
// list's slots contiguous, [pair][query][chunk][half][slot] (query space padded to 32): a lane's
// successive records fill whole lines.  ERP_CAND_INTERLEAVE=1 (an A/B knob, round 5) interleaves
// the lists of 32 consecutive queries x 2 halves slot by slot, [pair][chunk][query / 32][slot]
// [half][query % 32], so that a filter chain's 64 lanes store one slot index to one 2-KB run:
// filter 2.96 -> 2.89 ms per step, but lanes that stop extracting leave holes in their lines --
// filter writes 124 -> 194 MB and rescore reads 200 -> 217 MB per 128-pair launch
// (profiles/r05q_ab_slots.txt), so the contiguous lists stay.
// ERP_CAND_TILE_ARRAY=1 (development build only): the tile index of a candidate slot in its own
// int32 array (the layout before round 3; the inline index won the A/B)
#ifndef ERP_CAND_TILE_ARRAY
#define ERP_CAND_TILE_ARRAY 0
#endif
constexpr int kCandTileArray = ERP_CAND_TILE_ARRAY;
#ifndef ERP_CAND_INTERLEAVE
#define ERP_CAND_INTERLEAVE 0
#endif
__device__ __forceinline__ size_t cand_slot(int p, int ch, int chunks, int nqb, int q, int h, int sl) {
#if ERP_CAND_INTERLEAVE
    return ((((size_t)p * chunks + ch) * nqb + (q >> 5)) * kCandSlots + sl) * 64 + h * 32 + (q & 31);
#else  // [list][slot], list = ((pair, query, chunk), half) in the padded query space
    return ((((size_t)p * (nqb * 32) + q) * chunks + ch) * 2 + h) * kCandSlots + sl;
#endif
}

__global__ __launch_bounds__(256) ERP_FILTER_WAVES void knn2_filter_kernel(const float* __restrict__ dq,
                                                          const bf16x8* __restrict__ thi,
                                                          const float* __restrict__ tn,
                                                          const uint32_t* __restrict__ tmaxb,
                                                          uint32_t* __restrict__ tmax,
                                                          const int64_t* __restrict__ off_q,
                                                          const int64_t* __restrict__ off_t,
                                                          int chunk_len, int chunks, int max_nq,
                                                          int max_nt, int qblocks,
                                                          float2* __restrict__ pu,
                                                          int32_t* __restrict__ ccount,
                                                          int32_t* __restrict__ ctile,
                                                          bf16x8* __restrict__ cval,
                                                          const bf16x8* __restrict__ sent_hi,
                                                          const float* __restrict__ sent_tu,
                                                          float* __restrict__ qn) {
    constexpr int tile_array = kCandTileArray;
    __shared__ __align__(16) char sm[2 * kFStageB];
    // XCD-aware block order: workgroups are dealt to the 8 XCDs round-robin by linear id, so
    // XCD x gets the contiguous logical range [x NB/8, (x+1) NB/8) (query blocks fastest, then
    // chunks, then pairs): all blocks of a pair share one XCD's L2, which holds the pair's bf16
    // train rows (512 KB at 4096 rows) for every query block instead of refetching them from
    // HBM per XCD.  (Identity when NB is not a multiple of 8.)
    const int NB = gridDim.x;
    const int lb = (NB & 7) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (NB >> 3) + (blockIdx.x >> 3));
    const int qb = lb % qblocks, ch = (lb / qblocks) % chunks, p = lb / (qblocks * chunks);
    const int64_t qbase = off_q[p];
    const int nq = (int)(off_q[p + 1] - qbase);
    const int nt = (int)(off_t[p + 1] - off_t[p]);
    const int q0 = qb * kFQ;
    const int t0 = ch * chunk_len;
    if (q0 >= nq || t0 >= nt) return;  // uniform over the block
    const int t1 = min(t0 + chunk_len, nt);
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
    // teM >= 2 eps |t|^2 for every row of the pair (the pair's max for knn2_rescore from the
    // pair's first block)
    const uint32_t tmx = pair_tmax(tmaxb, p, nt, max_nt);
    if (qb == 0 && ch == 0 && tid == 0) tmax[p] = tmx;
    const float teM = __uint_as_float(tmx) * (2.f * kFEps) * (1.f + kFMargin) + kFTiny;
    // the wave's two 32-query column blocks: fragments dims 16c + 8h .. +7, rounded once
    bf16x8 qh[2][4];
    float QB[2], cq[2];
    bool qv[2];
    int qi[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int q = q0 + (tid >> 6) * kFW + 32 * j + r;
        qv[j] = q < nq;
        qi[j] = qv[j] ? q : 0;
        const float* qp = dq + (qbase + qi[j]) * kDim + 8 * h;
        float qq = 0.f;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const float4 a = *reinterpret_cast<const float4*>(qp + 16 * c);
            const float4 b = *reinterpret_cast<const float4*>(qp + 16 * c + 4);
            qq += sq8(a, b);
            qh[j][c] = round8(a, b, 1.f);
        }
        qq += __shfl_xor(qq, 32, 64);
        // |q|^2 for knn2_rescore (its bound offsets; the f32 rounding of either summation order
        // is far inside the 2.1e-4 S slack), so that it reads the query row only when an exact
        // distance is needed (queries the bounds reject never do)
        if (ch == 0 && h == 0 && qv[j]) qn[(size_t)p * max_nq + qi[j]] = qq;
        QB[j] = __builtin_fmaf(qq, kFEps, qq) + kFTiny;
        const float QL = __builtin_fmaf(qq, -kFEps, qq) - kFTiny;
        cq[j] = QB[j] - (QL - teM);       // thr = G + cq (rounded up below)
    }
    float gm[2][2] = {{kInf, kInf}, {kInf, kInf}};
    float thr[2] = {-kInf, -kInf};
    int ncand[2] = {0, 0};
    uint32_t cl[2];  // (pair, query, chunk, lane half) list index (< 2^31: the launcher checks)
    // the lists' first slot records, computed once (the 64-bit slot arithmetic inside the
    // extraction branch cost ~20 VALU per taken branch)
    bf16x8* clist[2];
    int32_t* ctl[2];
    constexpr int kSlotStride = ERP_CAND_INTERLEAVE ? 64 : 1;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        cl[j] = (((uint32_t)p * (uint32_t)max_nq + (uint32_t)qi[j]) * (uint32_t)chunks + ch) * 2u + h;
        const size_t s0 = cand_slot(p, ch, chunks, (max_nq + 31) >> 5, qi[j], h, 0);
        clist[j] = cval + s0 * 2;
        ctl[j] = tile_array ? ctile + s0 : nullptr;
    }
    // staging by LDS-DMA: wave w moves the stage's 1-KB pieces 4 w .. 4 w + 3 (8 rows each;
    // lane -> row 8 k + (lane >> 3), swizzled source piece) and, waves 0 and 1, 64 tu each;
    // rows past the chunk read the sentinel row (bf16 zeros, tu = +inf)
    const int wv = tid >> 6;
    const bf16x8* thp = thi + (size_t)p * max_nt * 8;
    const float* tup = tn + (size_t)p * max_nt;
    const int drow = lane >> 3;
    auto dma = [&](char* sb, int st) {
        const int rb = t0 + st * kFST * kFT;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int m = 4 * wv + k;  // piece: rows 8 m .. 8 m + 7 of the stage
            const int row = 8 * m + drow;
            const int dpc = (lane & 7) ^ ((row >> 1) & 7);  // source piece of LDS position lane & 7
            const bf16x8* src = rb + row < t1 ? thp + (size_t)(rb + row) * 8 + dpc : sent_hi + dpc;
            __builtin_amdgcn_global_load_lds((glb_vptr)src,
                                             (lds_vptr)(sb + (4 * wv + k) * 1024), 16, 0, 0);
        }
        if (wv < 2) {
            const int row = 64 * wv + lane;
            const float* src = rb + row < t1 ? tup + rb + row : sent_tu;
            __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(sb + kFHiB + 256 * wv), 4,
                                             0, 0);
        }
    };
    const int nstages = (t1 - t0 + kFST * kFT - 1) / (kFST * kFT);  // rows past t1: +inf
    // LDS byte addresses: A fragment (row r, piece 2 c + h = dims 16 c + 8 h, swizzled) and the
    // C operand rows 8 g + 4 h
    int rd_hi[4];
#pragma unroll
    for (int c = 0; c < 4; c++) rd_hi[c] = r * kFRowB + (((2 * c + h) ^ ((r >> 1) & 7)) << 4);
    const int rd_tu = kFHiB + 16 * h;
    // one tile: the A fragments and C operand from LDS, two 4-MFMA chains (the wave's two query
    // blocks); then the epilogue of each chain (group minima; with `extract`, the candidate test
    // and slot stores)
    struct Acc2 {
        f32x16 a0, a1;
    };
    struct Frag {
        bf16x8 ah[4];
        f32x16 ci;
    };
    auto tile_frags = [&](const char* sb, int u) __attribute__((always_inline)) -> Frag {
        Frag f;
#pragma unroll
        for (int c = 0; c < 4; c++)
            f.ah[c] = *reinterpret_cast<const bf16x8*>(sb + rd_hi[c] + u * kFT * kFRowB);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const float4 t4 = *reinterpret_cast<const float4*>(sb + rd_tu + 4 * (u * kFT + 8 * g));
            f.ci[4 * g] = t4.x;
            f.ci[4 * g + 1] = t4.y;
            f.ci[4 * g + 2] = t4.z;
            f.ci[4 * g + 3] = t4.w;
        }
        return f;
    };
    auto tile_mma_f = [&](const Frag& f) __attribute__((always_inline)) -> Acc2 {
        const bf16x8(&ah)[4] = f.ah;
        const f32x16& ci = f.ci;
        Acc2 r;
        r.a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[0], qh[0][0], ci, 0, 0, 0);
#pragma unroll
        for (int c = 1; c < 4; c++)
            r.a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], qh[0][c], r.a0, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        r.a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[0], qh[1][0], ci, 0, 0, 0);
#pragma unroll
        for (int c = 1; c < 4; c++)
            r.a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], qh[1][c], r.a1, 0, 0, 0);
        return r;
    };
    auto tile_mma = [&](const char* sb, int u) __attribute__((always_inline)) -> Acc2 {
        (void)tile_mma_f;
        (void)tile_frags;
        bf16x8 ah[4];
#pragma unroll
        for (int c = 0; c < 4; c++)
            ah[c] = *reinterpret_cast<const bf16x8*>(sb + rd_hi[c] + u * kFT * kFRowB);
        f32x16 ci;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const float4 t4 = *reinterpret_cast<const float4*>(sb + rd_tu + 4 * (u * kFT + 8 * g));
            ci[4 * g] = t4.x;
            ci[4 * g + 1] = t4.y;
            ci[4 * g + 2] = t4.z;
            ci[4 * g + 3] = t4.w;
        }
        Acc2 r;
        r.a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[0], qh[0][0], ci, 0, 0, 0);
#pragma unroll
        for (int c = 1; c < 4; c++)
            r.a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], qh[0][c], r.a0, 0, 0, 0);
#if ERP_FILTER_CHAINS
        // chain 0 whole before chain 1: its min tree then issues between chain 1's MFMAs instead
        // of after both (the interleaved order exposes the last MFMA's drain)
        __builtin_amdgcn_sched_barrier(0);
#endif
        r.a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[0], qh[1][0], ci, 0, 0, 0);
#pragma unroll
        for (int c = 1; c < 4; c++)
            r.a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[c], qh[1][c], r.a1, 0, 0, 0);
        return r;
    };
    // updc: std::integral_constant<bool, false> in the final recompute of the warm stages
    auto tile_epi = [&](int j, f32x16 e, int tile0, bool extract, auto updc) __attribute__((always_inline)) {
        // the running bound: the lane's two smallest TILE minima (16 rows each), minima of
        // disjoint row sets, so 2 rows have u' <= gm[j][1].  Round 5's (tile, 8-row group)
        // minima were tighter only when both smallest rows of the lane's ~2k share one tile
        // (~1 %), for two trees of 8 and a 6-op update against one tree of 16 and 3 ops here
        // (filter -3 %, rescore unchanged, profiles/r06w_ab_filter_top2.txt); before r05 the
        // minima of two fixed row groups were looser still (rescore 1.21 -> 0.89 ms).  Not in the
        // final recompute of the warm stages: a tile seen twice could fill both places
        float t = min3f(e[0], e[1], e[2]);
#pragma unroll
        for (int k = 3; k < 15; k += 2) t = min3f(t, e[k], e[k + 1]);
        t = min2f(t, e[15]);
        if (decltype(updc)::value) {
            gm[j][1] = min2f(fmaxf(gm[j][0], t), gm[j][1]);
            gm[j][0] = min2f(gm[j][0], t);
        }
        const float tmin = t;
        // a lane whose 16 rows of the tile may hold a candidate stores them whole (16 bounds
        // as bf16 carrying the tile index: two 16-B stores); knn2_rescore picks the rows under
        // the final bound (widening each stored value by its bf16 rounding and the replaced LSB)
        if (extract && tmin <= thr[j]) {
            const int sl = ncand[j]++;
            if (sl < kCandSlots && ERP_FILTER_ABLATE != 1) {
                if (tile_array) ctl[j][sl * kSlotStride] = tile0;
#pragma unroll
                for (int g = 0; g < 2; g++) {
                    bf16x8 b;
#pragma unroll
                    for (int i = 0; i < 8; i++) b[i] = (__bf16)e[8 * g + i];
                    clist[j][sl * (2 * kSlotStride) + g] =
                        tile_array ? b : cand_embed_tile(b, g, cand_spread(tile0));
                }
            }
        }
    };
    // the stage's 4 tiles.  ERP_FILTER_CHAINS == 2: software-pipelined by one chain -- tile u's
    // second chain is reduced after tile u + 1's MFMAs are issued, so neither chain's drain is
    // waited on (+16 live VGPRs)
    auto tiles = [&](const char* sb, int tb0, bool extract, auto updc) __attribute__((always_inline)) {
#if ERP_FILTER_CHAINS == 3
        // as 2, and tile u + 1's fragment reads issued right after tile u's MFMAs (in flight
        // during them and the epilogues) instead of in front of tile u + 1's MFMAs, where each
        // tile waited lgkmcnt(0) on its own reads
        f32x16 prev;
        (void)tile_mma;
        Frag f = tile_frags(sb, 0);
#pragma unroll
        for (int u = 0; u < kFST; u++) {
            const Acc2 acc = tile_mma_f(f);
            __builtin_amdgcn_sched_barrier(0);
            if (u + 1 < kFST) f = tile_frags(sb, u + 1);
            tile_epi(0, acc.a0, tb0 + u * kFT, extract, updc);
            if (u > 0) tile_epi(1, prev, tb0 + (u - 1) * kFT, extract, updc);
            prev = acc.a1;
        }
        tile_epi(1, prev, tb0 + (kFST - 1) * kFT, extract, updc);
#elif ERP_FILTER_CHAINS == 2
        f32x16 prev;
#pragma unroll
        for (int u = 0; u < kFST; u++) {
            const Acc2 acc = tile_mma(sb, u);
            tile_epi(0, acc.a0, tb0 + u * kFT, extract, updc);
            if (u > 0) tile_epi(1, prev, tb0 + (u - 1) * kFT, extract, updc);
            prev = acc.a1;
        }
        tile_epi(1, prev, tb0 + (kFST - 1) * kFT, extract, updc);
#else
#pragma unroll
        for (int u = 0; u < kFST; u++) {
            const Acc2 acc = tile_mma(sb, u);
            tile_epi(0, acc.a0, tb0 + u * kFT, extract, updc);
            tile_epi(1, acc.a1, tb0 + u * kFT, extract, updc);
        }
#endif
    };
    // one stage: wait for its DMAs (issued during the previous stage), barrier, the next
    // stage's DMAs into the other buffer (whose reads finished before this barrier), 4 tiles,
    // then (except in the final recompute) the query's running bound and candidate threshold
    // (the first `warm` stages run bounds-only -- kFWarm, at most a quarter of the chunk's, at
    // least one -- and are recomputed for candidates after the last)
    const int warm = max(1, min(kFWarm, nstages / 4));
    const int last = nstages + warm - 1;  // iterations 0 .. last
    auto stage = [&](auto bufc, auto updc, int it) {
        constexpr int BUF = decltype(bufc)::value;
        char* sb = sm + BUF * kFStageB;
        const int st = it < nstages ? it : it - nstages;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (it < last && ERP_FILTER_ABLATE != 2) {
            const int nx = it + 1 < nstages ? it + 1 : it + 1 - nstages;
            dma(sm + (1 - BUF) * kFStageB, nx);
        }
        tiles(sb, t0 + st * kFST * kFT, it >= warm, updc);
        if (it < nstages) {
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const float G = second4(gm[j][0], gm[j][1], __shfl_xor(gm[j][0], 32, 64),
                                        __shfl_xor(gm[j][1], 32, 64));
                thr[j] = qv[j] ? (G + cq[j]) + (fabsf(G) + cq[j]) * kFMargin : -kInf;
            }
        }
    };
    // stage sequence: 0 .. warm - 1 (bounds only), warm .. nstages - 1, then 0 .. warm - 1 again
    // (candidates only, against the chunk's final bound); LDS buffers alternate
    dma(sm, 0);
    {
        const std::integral_constant<int, 0> b0{};
        const std::integral_constant<int, 1> b1{};
        const std::integral_constant<bool, true> u1{};
        const std::integral_constant<bool, false> u0{};
        int it = 0;
        for (; it + 1 < nstages; it += 2) {
            stage(b0, u1, it);
            stage(b1, u1, it + 1);
        }
        if (it < nstages) stage(b0, u1, it++);
        for (; it <= last; it++) {  // the recompute (buffer = iteration parity)
            if (it & 1) stage(b1, u0, it);
            else stage(b0, u0, it);
        }
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const float m1 = fminf(gm[j][0], gm[j][1]), m2 = fmaxf(gm[j][0], gm[j][1]);
        const float o1 = __shfl_xor(m1, 32, 64), o2 = __shfl_xor(m2, 32, 64);
        const float n2 = fminf(fmaxf(m1, o1), fminf(m2, o2));
        const float n1 = fminf(m1, o1);
        if (h == 0 && qv[j])
            pu[((size_t)p * chunks + ch) * max_nq + qi[j]] =
                make_float2(n1 + QB[j], n2 + QB[j]);
        if (qv[j]) ccount[cl[j]] = ncand[j];
    }
}

// exact squared distance in the flann::L2<float> order: per group of 4,
// acc += d0*d0 + d1*d1 + d2*d2 + d3*d3 (no FMA)
__device__ __forceinline__ float exact_l2(const float4* qr, const float4* __restrict__ tp) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 16; c++) {
        const float4 tv = tp[c];
        const float d0 = qr[c].x - tv.x;
        const float d1 = qr[c].y - tv.y;
        const float d2 = qr[c].z - tv.z;
        const float d3 = qr[c].w - tv.w;
        acc += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    return acc;
}

// k=2 update with the sweep's tie rule (lowest train index first among equal distances)
__device__ __forceinline__ void top2_consider(float acc, int j, float& b0, int& j0, float& b1) {
    if (acc < b0 || (acc == b0 && j < j0)) {
        b1 = b0;
        b0 = acc;
        j0 = j;
    } else if (acc < b1) {
        b1 = acc;
    }
}

constexpr int kPassList = 24;  // rows under the final bound per (query, chunk) (more: sweep)

// k=2 fold with the lowest-index tie rule (chunks / lanes / waves in any order)
__device__ __forceinline__ void top2_fold(float& b0, int& j0, float& b1, float ob0, int oj, float ob1) {
    if (ob0 < b0 || (ob0 == b0 && oj < j0)) {
        b1 = fminf(b0, ob1);
        b0 = ob0;
        j0 = oj;
    } else {
        b1 = fminf(b1, ob0);
    }
}

// one lane per (query, train chunk): U2 = the second smallest bound over all chunks, then the
// stored rows with l* = u' + QL - teM <= U2 (u' widened by its bf16 rounding) into the lane's
// LDS list, then their exact distances in increasing l*: once l* > b1 (the exact second
// smallest so far) the row's e > b1 >= b0 cannot change (j0, d0, d1), nor can any later row
// -> the chunk's exact k=2 in part[pair][chunk][query].  A (query, chunk) whose slot list
// overflowed in knn2_filter (or with more than kPassList rows) goes to the overflow list
// (exact sweep of that chunk, knn2_sweep_kernel).  Chunks with no candidates write an empty
// Top2.
__global__ __launch_bounds__(256) void knn2_rescore_kernel(const float* __restrict__ dq,
                                                           const float* __restrict__ dt,
                                                           const int64_t* __restrict__ off_q,
                                                           const int64_t* __restrict__ off_t,
                                                           int max_nq, int chunk_len, int chunks,
                                                           const uint32_t* __restrict__ tmax,
                                                           const float2* __restrict__ pu,
                                                           const int32_t* __restrict__ ccount,
                                                           const int32_t* __restrict__ ctile,
                                                           const bf16x8* __restrict__ cval,
                                                           Top2* __restrict__ part,
                                                           int32_t* __restrict__ ovf, int qblocks,
                                                           float ratio,
                                                           const float* __restrict__ qn) {
    constexpr int tile_array = kCandTileArray;
    __shared__ int32_t plist[kPassList * 256];
    __shared__ float plb[kPassList * 256];
    // XCD-aware block order as in knn2_filter (a pair's blocks on one XCD: its f32 train rows,
    // gathered by the exact distances, stay in that XCD's L2)
    const int NB = gridDim.x;
    const int lb = (NB & 7) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (NB >> 3) + (blockIdx.x >> 3));
    const int c = (lb / qblocks) % chunks, p = lb / (qblocks * chunks);
    const int q = (lb % qblocks) * 256 + threadIdx.x;
    const int64_t qbase = off_q[p];
    const int nq = (int)(off_q[p + 1] - qbase);
    const int64_t tbase = off_t[p];
    const int nt = (int)(off_t[p + 1] - tbase);
    if (q >= nq || c * chunk_len >= nt) return;
    const size_t l0 = (((size_t)p * max_nq + q) * chunks + c) * 2;
    const int n0 = ccount[l0], n1 = ccount[l0 + 1];
    Top2* out = part + ((size_t)p * chunks + c) * max_nq + q;
    auto overflow = [&]() {
        const int slot = atomicAdd(&ovf[0], 1);
        ovf[1 + 3 * slot] = p;
        ovf[2 + 3 * slot] = q;
        ovf[3 + 3 * slot] = c;
    };
    if (n0 > kCandSlots || n1 > kCandSlots) {
        overflow();
        return;
    }
    float b0 = kInf, b1 = kInf;
    int j0 = 0x7fffffff;
    if (n0 + n1 > 0) {
        const int nch = (nt + chunk_len - 1) / chunk_len;
        float m1 = kInf, m2 = kInf;
        for (int cc = 0; cc < nch; cc++) {
            const float2 v = pu[((size_t)p * chunks + cc) * max_nq + q];
            m2 = fminf(fmaxf(m1, v.x), fminf(m2, v.y));
            m1 = fminf(m1, v.x);
        }
        const float U2 = m2;
        // the query row only once an exact distance is needed (since r05; |q|^2 from the filter)
        float4 qr[16];
        bool have_q = false;
        const float4* qp = reinterpret_cast<const float4*>(dq + (qbase + q) * kDim);
        auto load_q = [&]() {
            if (have_q) return;
#pragma unroll
            for (int k = 0; k < 16; k++) qr[k] = qp[k];
            have_q = true;
        };
        const float qq = qn[(size_t)p * max_nq + q];
        // l* = u' + lq <= the row's l (knn2_filter header; lq's rounding is inside the slack)
        const float teM = __uint_as_float(tmax[p]) * (2.f * kFEps) * (1.f + kFMargin) + kFTiny;
        const float lq = (__builtin_fmaf(qq, -kFEps, qq) - kFTiny) - teM;
        // u* = v + 2^-8 |v| + |q|^2 (1 + eps) >= u' + |q|^2 (1 + eps) = u >= e (the filter's
        // upper bound; the f32 roundings here are far inside its 2.1e-4 S slack)
        const float uq = __builtin_fmaf(qq, kFEps, qq) + kFTiny;
        // the stored value's widening: round to nearest (2^-8 |v|), +1 ulp with the tile index
        // in the LSB (3 2^-8 |v|, taken as 2^-6)
        const float wv = tile_array ? 0x1p-8f : 0x1p-6f;
        int npass = 0;
        float l1 = kInf, l2 = kInf, umin = kInf;  // two smallest l*, smallest u*
        int r1 = -1, ra = -1;                     // their rows
        for (int h = 0; h < 2; h++) {
            const int n = h ? n1 : n0;
            for (int k = 0; k < n; k++) {
                const size_t slot = cand_slot(p, c, chunks, (max_nq + 31) >> 5, q, h, k);
                const bf16x8 v0 = cval[slot * 2], v1 = cval[slot * 2 + 1];
                const int tile0 = tile_array ? ctile[slot] : cand_tile(v0, v1);
#pragma unroll
                for (int e = 0; e < 16; e++) {
                    // bf16 round to nearest: |v - u'| <= 2^-9 |u'|, so v - 2^-8 |v| <= u'
                    const float x = (float)(e < 8 ? v0[e] : v1[e - 8]);
                    const float lo = __builtin_fmaf(-wv, fabsf(x), x) + lq;
                    const int row = tile0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (lo <= U2 && row < nt) {
                        if (npass < kPassList) {
                            plist[npass * 256 + threadIdx.x] = row;
                            plb[npass * 256 + threadIdx.x] = lo;
                        }
                        npass++;
                        const float hi = __builtin_fmaf(wv, fabsf(x), x) + uq;
                        if (lo < l1) {
                            l2 = l1;
                            l1 = lo;
                            r1 = row;
                        } else {
                            l2 = fminf(l2, lo);
                        }
                        if (hi < umin) {
                            umin = hi;
                            ra = row;
                        }
                    }
                }
            }
        }
        if (npass > kPassList) {  // (never seen on SURF-like data) exact sweep of the chunk
            overflow();
            return;
        }
        // The ratio test decided by the bounds (single-chunk launches only: the merge then sees
        // this lane's record alone).  Every row with e <= e_(2) is listed (unlisted rows have
        // e >= l* > U2 >= e_(2)), so e_(1) >= l1, e_(2) >= the smallest l* of the rows other than
        // the one holding e_(1), and e_(2) <= U2.  sqrtf and fl(ratio * x) are monotone, so
        //  reject: sqrtf(l1) >= fl(ratio sqrtf(U2)) gives d0 >= ratio d1 -- record {inf, -1, inf}
        //    (the merge's d0 < ratio d1 is false for it, as for the exact values);
        //  accept: when one row's u* is below every other row's l*, it is the unique nearest;
        //    its exact e gives d0, and d0 < fl(ratio sqrtf(L_other)) <= fl(ratio d1) -- record
        //    {e, row, L_other}, on which the merge's test passes just as on {e, row, e_(2)}.
        if (ratio >= 0.f && npass > 0) {
            if (__builtin_sqrtf(fmaxf(l1, 0.f)) >= ratio * __builtin_sqrtf(U2)) {
                *out = Top2{kInf, -1, kInf};
                return;
            }
            const float lother = r1 == ra ? l2 : l1;
            if (umin < lother) {
                load_q();
                const float e = exact_l2(qr, reinterpret_cast<const float4*>(dt + (tbase + ra) * kDim));
                const float lb2 = fmaxf(lother, 0.f);
                if (__builtin_sqrtf(e) < ratio * __builtin_sqrtf(lb2)) {
                    *out = Top2{e, ra, lb2};
                    return;
                }
            }
        }
        for (int k = 0; k < npass; k++) {
            int kb = k;
            float lbest = plb[k * 256 + threadIdx.x];
            for (int m = k + 1; m < npass; m++) {
                const float v = plb[m * 256 + threadIdx.x];
                if (v < lbest) {
                    lbest = v;
                    kb = m;
                }
            }
            if (lbest > b1) break;
            const int row = plist[kb * 256 + threadIdx.x];
            if (kb != k) {  // swap the chosen entry into position k
                plist[kb * 256 + threadIdx.x] = plist[k * 256 + threadIdx.x];
                plb[kb * 256 + threadIdx.x] = plb[k * 256 + threadIdx.x];
            }
            load_q();
            top2_consider(exact_l2(qr, reinterpret_cast<const float4*>(dt + (tbase + row) * kDim)),
                          row, b0, j0, b1);
        }
    }
    *out = Top2{b0, j0 == 0x7fffffff ? -1 : j0, b1};
}

// exact sweep over the train rows of one chunk for the overflowed (query, chunk) entries: one
// 256-thread block per entry (rows strided over the threads, two rows in flight per thread),
// a fixed grid striding over the list

__global__ __launch_bounds__(256) void knn2_sweep_kernel(const float* __restrict__ dq,
                                                         const float* __restrict__ dt,
                                                         const int64_t* __restrict__ off_q,
                                                         const int64_t* __restrict__ off_t,
                                                         int max_nq, int chunk_len, int chunks,
                                                         const int32_t* __restrict__ ovf,
                                                         Top2* __restrict__ part) {
    __shared__ Top2 red[4];
    const int lane = wave_lane(), wid = threadIdx.x >> 6;
    const int nov = ovf[0];
    for (int w = blockIdx.x; w < nov; w += gridDim.x) {
        const int p = ovf[1 + 3 * w], q = ovf[2 + 3 * w], c = ovf[3 + 3 * w];
        const int64_t qbase = off_q[p], tbase = off_t[p];
        const int nt = (int)(off_t[p + 1] - tbase);
        const int ja = c * chunk_len, jb = min(nt, ja + chunk_len);
        float4 qr[16];
        const float4* qp = reinterpret_cast<const float4*>(dq + (qbase + q) * kDim);
#pragma unroll
        for (int k = 0; k < 16; k++) qr[k] = qp[k];
        float b0 = kInf, b1 = kInf;
        int j0 = 0x7fffffff;
        for (int j = ja + (int)threadIdx.x; j < jb; j += 512) {
            const float da = exact_l2(qr, reinterpret_cast<const float4*>(dt + (tbase + j) * kDim));
            const int j2 = j + 256;
            const float db = j2 < jb
                                 ? exact_l2(qr, reinterpret_cast<const float4*>(dt + (tbase + j2) * kDim))
                                 : kInf;
            top2_consider(da, j, b0, j0, b1);
            if (j2 < jb) top2_consider(db, j2, b0, j0, b1);
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1)
            top2_fold(b0, j0, b1, __shfl_xor(b0, o, 64), __shfl_xor(j0, o, 64), __shfl_xor(b1, o, 64));
        if (lane == 0) red[wid] = Top2{b0, j0, b1};
        __syncthreads();
        if (threadIdx.x == 0) {
            Top2 r = red[0];
            for (int k = 1; k < 4; k++) top2_fold(r.d0, r.j0, r.d1, red[k].d0, red[k].j0, red[k].d1);
            part[((size_t)p * chunks + c) * max_nq + q] = Top2{r.d0, r.j0 == 0x7fffffff ? -1 : r.j0, r.d1};
        }
        __syncthreads();
    }
}

// ---- LDS-tiled exact sweep on packed FP32 VALU (the non-MFMA matcher, configs[3]) ----------
// Every (query, train) distance in the flann::L2<float> order, no filter: per group of 4 dims
// acc += ((d0*d0 + d1*d1) + d2*d2) + d3*d3, each operation rounded (no FMA).  Two train rows
// share every instruction (v_pk_add_f32 / v_pk_mul_f32 with the query value broadcast), so an
// element costs 1.5 VALU instructions: sub, mul, add.
// Block = 256 threads = 16 (tq) x 16 (tt); tile = 128 queries (resident in LDS for the whole
// chunk) x 128 train rows per step.  Thread (tq, tt) owns queries tq + 16 k (k < 8) and the
// train row pairs tt + 16 k (k < 4): 64 accumulators.  Train rows sit in LDS as row pairs,
// dims interleaved ([pair][dim][2]), so one ds_read_b128 yields 2 dims x 2 rows = two packed
// operands; query rows are [row][68] (the 16 rows a wave reads per instruction fall on 64
// distinct banks).  The next tile is prefetched into registers during the current one.
// Output: per (pair, chunk, query) the chunk's exact k=2 (Top2, lowest index among ties);
// knn2_merge folds chunks in train order.
constexpr int kXQ = 128, kXT = 128;
constexpr int kXQRow = 68;             // floats per query row in LDS
constexpr int kXPair = 2 * kDim + 4;   // floats per train row pair in LDS

struct ExactLds {
    float q[kXQ * kXQRow];
    float t[kXT / 2 * kXPair];
    Top2 red[4][kXQ];                  // cross-wave fold of the k=2 partials
};

__global__ __launch_bounds__(256) void knn2_exact_kernel(const float* __restrict__ dq,
                                                         const float* __restrict__ dt,
                                                         const int64_t* __restrict__ off_q,
                                                         const int64_t* __restrict__ off_t,
                                                         int chunk_len, int chunks, int max_nq,
                                                         Top2* __restrict__ xpart) {
    __shared__ ExactLds sm;
    const int p = blockIdx.z;
    const int64_t qbase = off_q[p], tbase = off_t[p];
    const int nq = (int)(off_q[p + 1] - qbase);
    const int nt = (int)(off_t[p + 1] - tbase);
    const int q0 = blockIdx.x * kXQ;
    const int t0 = blockIdx.y * chunk_len;
    if (q0 >= nq || t0 >= nt) return;  // uniform over the block
    const int t1 = min(t0 + chunk_len, nt);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int tq = lane & 15, tt = (lane >> 4) + 4 * wid;
    // query tile: 128 rows x 16 float4, 8 float4 per thread (rows beyond nq read as 0)
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int e = tid + 256 * u, row = e >> 4, c = e & 15;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q0 + row < nq) v = reinterpret_cast<const float4*>(dq + (qbase + q0 + row) * kDim)[c];
        *reinterpret_cast<float4*>(&sm.q[row * kXQRow + 4 * c]) = v;
    }
    // train staging: thread -> row pair (tid >> 2) of the tile, dims 16 (tid & 3) .. +15
    const int spair = tid >> 2, sdim = 16 * (tid & 3);
    float4 ga[4], gb[4];
    auto gload = [&](int tile0) {
        const int ra = tile0 + 2 * spair, rb = ra + 1;
        const float4* pa = reinterpret_cast<const float4*>(dt + (tbase + min(ra, t1 - 1)) * kDim + sdim);
        const float4* pb = reinterpret_cast<const float4*>(dt + (tbase + min(rb, t1 - 1)) * kDim + sdim);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            ga[c] = pa[c];
            gb[c] = pb[c];
        }
    };
    float b0[8], b1[8];
    int j0[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        b0[k] = kInf;
        b1[k] = kInf;
        j0[k] = 0x7fffffff;
    }
    const int ntiles = (t1 - t0 + kXT - 1) / kXT;
    gload(t0);
    for (int s = 0; s < ntiles; s++) {
        const int tile0 = t0 + s * kXT;
        __syncthreads();  // previous tile's reads are done
#pragma unroll
        for (int c = 0; c < 4; c++) {
            float* w = &sm.t[spair * kXPair + 2 * (sdim + 4 * c)];
            *reinterpret_cast<float4*>(w) = make_float4(ga[c].x, gb[c].x, ga[c].y, gb[c].y);
            *reinterpret_cast<float4*>(w + 4) = make_float4(ga[c].z, gb[c].z, ga[c].w, gb[c].w);
        }
        __syncthreads();
        if (s + 1 < ntiles) gload(tile0 + kXT);
        f32x2 acc[8][4];
#pragma unroll
        for (int k = 0; k < 8; k++)
#pragma unroll
            for (int kk = 0; kk < 4; kk++) acc[k][kk] = f32x2{0.f, 0.f};
#pragma unroll 2
        for (int g = 0; g < 16; g++) {
            float4 tv[4][2];
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const float* tp = &sm.t[(tt + 16 * kk) * kXPair + 8 * g];
                tv[kk][0] = *reinterpret_cast<const float4*>(tp);
                tv[kk][1] = *reinterpret_cast<const float4*>(tp + 4);
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const float4 qv = *reinterpret_cast<const float4*>(&sm.q[(tq + 16 * k) * kXQRow + 4 * g]);
                const f32x2 qx = {qv.x, qv.x}, qy = {qv.y, qv.y}, qz = {qv.z, qv.z},
                            qw = {qv.w, qv.w};
#pragma unroll
                for (int kk = 0; kk < 4; kk++) {
                    const f32x2 e0 = qx - f32x2{tv[kk][0].x, tv[kk][0].y};
                    const f32x2 e1 = qy - f32x2{tv[kk][0].z, tv[kk][0].w};
                    const f32x2 e2 = qz - f32x2{tv[kk][1].x, tv[kk][1].y};
                    const f32x2 e3 = qw - f32x2{tv[kk][1].z, tv[kk][1].w};
                    acc[k][kk] = acc[k][kk] + (((e0 * e0 + e1 * e1) + e2 * e2) + e3 * e3);
                }
            }
        }
        // k=2 update, branch-free: a thread sees its rows in increasing train index, so a later
        // row never wins a tie (strict <); second = med3(b0, b1, d).  Rows >= t1 count as +inf.
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
            const int ja = tile0 + 2 * (tt + 16 * kk);
            const bool va = ja < t1, vb = ja + 1 < t1;
#pragma unroll
            for (int k = 0; k < 8; k++) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const float d = (h ? vb : va) ? acc[k][kk][h] : kInf;
                    b1[k] = __builtin_amdgcn_fmed3f(b0[k], b1[k], d);
                    j0[k] = d < b0[k] ? ja + h : j0[k];
                    b0[k] = fminf(b0[k], d);
                }
            }
        }
    }
    // fold the 16 threads of a query: lanes tq + 16 m of a wave (xor 16, 32), then 4 waves
#pragma unroll
    for (int k = 0; k < 8; k++) {
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
            const float ob0 = __shfl_xor(b0[k], o, 64), ob1 = __shfl_xor(b1[k], o, 64);
            const int oj = __shfl_xor(j0[k], o, 64);
            if (ob0 < b0[k] || (ob0 == b0[k] && oj < j0[k])) {
                b1[k] = fminf(b0[k], ob1);
                b0[k] = ob0;
                j0[k] = oj;
            } else {
                b1[k] = fminf(b1[k], ob0);
            }
        }
        if (lane < 16) sm.red[wid][tq + 16 * k] = Top2{b0[k], j0[k], b1[k]};
    }
    __syncthreads();
    if (tid < kXQ && q0 + tid < nq) {
        Top2 r = sm.red[0][tid];
#pragma unroll
        for (int w = 1; w < 4; w++) {
            const Top2 o = sm.red[w][tid];
            if (o.d0 < r.d0 || (o.d0 == r.d0 && o.j0 < r.j0)) {
                r.d1 = fminf(r.d0, o.d1);
                r.d0 = o.d0;
                r.j0 = o.j0;
            } else {
                r.d1 = fminf(r.d1, o.d0);
            }
        }
        if (r.j0 == 0x7fffffff) r.j0 = -1;
        xpart[((size_t)p * chunks + blockIdx.y) * max_nq + q0 + tid] = r;
    }
}

// Fold of per-chunk partials part[pair][chunk][query] into one exact k=2 per query
// (out[pair][query]), chunks in train order (an earlier chunk wins ties): one lane per query,
// so a single large pair uses the whole chip (the merge below is one block per pair).
__device__ __forceinline__ void merge_query(const Top2* part, size_t stride, int nch, int q,
                                            float& B0, int& J, float& B1);

__global__ __launch_bounds__(256) void knn2_fold_kernel(const Top2* __restrict__ part,
                                                        const int64_t* __restrict__ off_q,
                                                        const int64_t* __restrict__ off_t,
                                                        int chunk_len, int chunks, int max_nq,
                                                        Top2* __restrict__ out) {
    const int p = blockIdx.y;
    const int q = blockIdx.x * 256 + threadIdx.x;
    const int nq = (int)(off_q[p + 1] - off_q[p]);
    const int nt = (int)(off_t[p + 1] - off_t[p]);
    if (q >= nq) return;
    float B0, B1;
    int J;
    merge_query(part + (size_t)p * chunks * max_nq, (size_t)max_nq,
                max(1, (nt + chunk_len - 1) / chunk_len), q, B0, J, B1);
    out[(size_t)p * max_nq + q] = Top2{B0, J, B1};
}

// Fold chunk partials in train order (lowest index wins ties), apply the ratio test
// d0 < ratio * d1 on the sqrt'd distances (convertToDMatches + feature_matcher.cpp:52), and
// compact the survivors in ascending queryIdx order (knn2_merge_count / knn2_merge below).
__device__ __forceinline__ void merge_query(const Top2* part, size_t stride, int nch, int q,
                                            float& B0, int& J, float& B1) {
    B0 = kInf;
    B1 = kInf;
    J = -1;
    for (int c = 0; c < nch; c++) {
        const Top2 t = part[(size_t)c * stride + q];
        if (t.d0 < B0) {
            B1 = fminf(B0, t.d1);
            B0 = t.d0;
            J = t.j0;
        } else {
            B1 = fminf(B1, t.d0);
        }
    }
}

// Two passes over (pair, block of 1024 queries): the survivors of each block counted, then
// each block places its survivors at (the counts of the pair's earlier blocks) + (its own
// exclusive scan) -- ascending queryIdx, one query per thread, coalesced partial reads, and
// the whole grid busy for a single large pair (configs[3]: 16 blocks for 16384 queries).
constexpr int kMergeBlock = 1024;

__device__ __forceinline__ bool merge_one(const Top2* pp, int max_nq, int nch, int q, int nq,
                                          float ratio, int& J, float& d0) {
    if (q >= nq) return false;
    float B0, B1;
    merge_query(pp, (size_t)max_nq, nch, q, B0, J, B1);
    d0 = __builtin_sqrtf(B0);
    const float d1 = __builtin_sqrtf(B1);
    return d0 < ratio * d1;
}

__global__ __launch_bounds__(kMergeBlock) void knn2_merge_count_kernel(
    const Top2* __restrict__ part, const int64_t* __restrict__ off_q,
    const int64_t* __restrict__ off_t, int chunk_len, int chunks, int max_nq, float ratio,
    int32_t* __restrict__ bcount) {
    __shared__ int ws[16];
    const int p = blockIdx.y, b = blockIdx.x;
    const int nq = (int)(off_q[p + 1] - off_q[p]);
    const int nt = (int)(off_t[p + 1] - off_t[p]);
    if (nt < 2 || b * kMergeBlock >= nq) return;  // uniform over the block
    const int nch = (nt + chunk_len - 1) / chunk_len;
    int J;
    float d0;
    const bool keep = merge_one(part + (size_t)p * chunks * max_nq, max_nq, nch,
                                b * kMergeBlock + (int)threadIdx.x, nq, ratio, J, d0);
    int total;
    (void)block_exclusive_scan<kMergeBlock>(keep ? 1 : 0, ws, &total);
    if (threadIdx.x == 0) bcount[(size_t)p * gridDim.x + b] = total;
}

__global__ __launch_bounds__(kMergeBlock) void knn2_merge_kernel(
    const Top2* __restrict__ part, const int64_t* __restrict__ off_q,
    const int64_t* __restrict__ off_t, int chunk_len, int chunks, int max_nq, float ratio,
    const int32_t* __restrict__ bcount, erp_dmatch* __restrict__ out,
    int32_t* __restrict__ counts, int32_t* __restrict__ flags, BearingOut bo) {
    __shared__ int ws[16];
    __shared__ int base_s;
    const int p = blockIdx.y, b = blockIdx.x, nb = gridDim.x;
    if (bo.pts && b == 0 && threadIdx.x == 0) {  // zero sentinel row (pads the Gram batches)
        double* z = bo.pts + ((size_t)p * (max_nq + 1) + max_nq) * 6;
        for (int k = 0; k < 6; k++) z[k] = 0.0;
    }
    const int nq = (int)(off_q[p + 1] - off_q[p]);
    const int nt = (int)(off_t[p + 1] - off_t[p]);
    if (nt < 2 || nq <= 0) {
        if (b == 0 && threadIdx.x == 0) {
            counts[p] = 0;
            if (nq > 0) flags[p] |= 1;  // knn_matches[i][1] would not exist (UB in the reference)
        }
        return;
    }
    const int nqb = (nq + kMergeBlock - 1) / kMergeBlock;  // this pair's live blocks
    if (b >= nqb) return;
    if (threadIdx.x < 64) {  // the pair's earlier blocks (and, for the last one, all of them)
        const int32_t* bc = bcount + (size_t)p * nb;
        int pre = 0, all = 0;
        for (int k = threadIdx.x; k < nqb; k += 64) {
            const int c = bc[k];
            pre += k < b ? c : 0;
            all += c;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            pre += __shfl_xor(pre, o, 64);
            all += __shfl_xor(all, o, 64);
        }
        if (threadIdx.x == 0) {
            base_s = pre;
            if (b == nqb - 1) counts[p] = all;
        }
    }
    const int nch = (nt + chunk_len - 1) / chunk_len;
    const int q = b * kMergeBlock + (int)threadIdx.x;
    int J = 0;
    float d0 = 0.f;
    const bool keep = merge_one(part + (size_t)p * chunks * max_nq, max_nq, nch, q, nq, ratio, J, d0);
    int total;
    const int pos = block_exclusive_scan<kMergeBlock>(keep ? 1 : 0, ws, &total);  // syncs base_s
    if (!keep) return;
    const int m = base_s + pos;
    out[(size_t)p * max_nq + m] = erp_dmatch{q, J, 0, d0};
    if (bo.pts) {
        const erp_point2f kl = bo.kp_l[off_q[p] + q];
        const erp_point2f kr = bo.kp_r[off_t[p] + J];
        double* o = bo.pts + ((size_t)p * (max_nq + 1) + m) * 6;
        pixel_to_bearing(bo.width[p], bo.height[p], kl.x, kl.y, o);
        pixel_to_bearing(bo.width[p], bo.height[p], kr.x, kr.y, o + 3);
        if (bo.key_l) bo.key_l[(size_t)p * max_nq + m] = kl;
        if (bo.key_r) bo.key_r[(size_t)p * max_nq + m] = kr;
    }
}


}  // namespace

// ====================================================================== launchers =======
size_t knn2_cand_bytes(const BatchShape& sh) {
    return (size_t)sh.n_pairs * ((sh.max_nq + 31) / 32 * 32) * sh.fchunks * 2 * kCandSlots *
           (2 * sizeof(bf16x8) + 4);
}

size_t knn2_split_bytes(const BatchShape& sh) {  // rows, tu, tmax, sentinel row, block maxima
    return (size_t)sh.n_pairs * sh.max_nt * (kDim * sizeof(__bf16) + sizeof(float)) +
           (size_t)sh.n_pairs * sizeof(uint32_t) + 16 + 128 + 16 +
           (size_t)sh.n_pairs * ((sh.max_nt + 63) / 64) * sizeof(uint32_t);
}

static void cand_split(const BatchShape& sh, void* cand, int32_t** ctile, bf16x8** cval) {
    const size_t lists = (size_t)sh.n_pairs * ((sh.max_nq + 31) / 32 * 32) * sh.fchunks * 2 * kCandSlots;
    *cval = (bf16x8*)cand;
    *ctile = (int32_t*)(*cval + lists * 2);
}

static uint32_t* split_tmax(const BatchShape& sh, void* split) {
    return (uint32_t*)((char*)split + (size_t)sh.n_pairs * sh.max_nt * (kDim * sizeof(__bf16) + sizeof(float)));
}
// the sentinel row after tmax (16-B aligned): 64 bf16 zeros, then tu = +inf
static char* split_sentinel(const BatchShape& sh, void* split) {
    const size_t o = (size_t)((char*)(split_tmax(sh, split) + sh.n_pairs) - (char*)split);
    return (char*)split + ((o + 15) & ~(size_t)15);
}

hipError_t launch_knn2_filter(const float* desc_q, const float* desc_t, const int64_t* off_q,
                              const int64_t* off_t, const BatchShape& sh, void* split,
                              float2* pu, int32_t* ccount, void* cand, hipStream_t st,
                              int32_t* ovf, int32_t* flags) {
    bf16x8* thi = (bf16x8*)split;
    float* tn = (float*)(thi + (size_t)sh.n_pairs * sh.max_nt * 8);
    uint32_t* tmax = split_tmax(sh, split);
    char* sent = split_sentinel(sh, split);
    uint32_t* tmaxb = (uint32_t*)(sent + 144);  // (after the sentinel row and its tu, 16-B aligned)
    ERP_LAUNCH(knn2_split_kernel, dim3((sh.max_nt + 63) / 64, sh.n_pairs), dim3(256), 0,
                       st, desc_t, off_t, sh.max_nt, thi, tn, tmaxb, ovf, (uint32_t*)sent, flags);
    int32_t* ctile;
    bf16x8* cval;
    cand_split(sh, cand, &ctile, &cval);
    const int qblocks = (sh.max_nq + kFQ - 1) / kFQ;
    if ((size_t)sh.n_pairs * sh.max_nq * sh.fchunks * 2 >= (1ull << 31)) return hipErrorInvalidValue;
    float* qn = (float*)(pu + (size_t)sh.n_pairs * sh.max_nq * sh.fchunks);  // (after pu)
    ERP_LAUNCH(knn2_filter_kernel, dim3(qblocks * sh.fchunks * sh.n_pairs), dim3(256), 0,
                       st, desc_q, thi, tn, (const uint32_t*)tmaxb, tmax, off_q, off_t,
                       sh.fchunk_len, sh.fchunks,
                       sh.max_nq, sh.max_nt, qblocks, pu, ccount, ctile, cval,
                       (const bf16x8*)sent, (const float*)(sent + 128), qn);
    return hipGetLastError();
}

hipError_t launch_knn2_rescore(const float* desc_q, const float* desc_t, const int64_t* off_q,
                               const int64_t* off_t, const BatchShape& sh, void* split,
                               const float2* pu, const int32_t* ccount, void* cand, Top2* part,
                               int32_t* ovf, float ratio, hipStream_t st) {
    int32_t* ctile;
    bf16x8* cval;
    cand_split(sh, cand, &ctile, &cval);
    // (ovf[0] was zeroed by knn2_split_kernel, launch_knn2_filter)
    const int qblocks = (sh.max_nq + 255) / 256;
    ERP_LAUNCH(knn2_rescore_kernel, dim3(qblocks * sh.fchunks * sh.n_pairs), dim3(256), 0,
                       st, desc_q, desc_t, off_q, off_t, sh.max_nq, sh.fchunk_len, sh.fchunks,
                       split_tmax(sh, split), pu, ccount, ctile, cval, part, ovf, qblocks,
                       sh.fchunks == 1 ? ratio : -1.f,  // (bound decisions need one chunk)
                       (const float*)(pu + (size_t)sh.n_pairs * sh.max_nq * sh.fchunks));
    ERP_LAUNCH(knn2_sweep_kernel, dim3(256), dim3(256), 0, st, desc_q, desc_t, off_q, off_t,
                       sh.max_nq, sh.fchunk_len, sh.fchunks, ovf, part);
    return hipGetLastError();
}

hipError_t launch_knn2_exact(const float* desc_q, const float* desc_t, const int64_t* off_q,
                             const int64_t* off_t, const BatchShape& sh, Top2* xpart,
                             hipStream_t st) {
    dim3 grid((sh.max_nq + kXQ - 1) / kXQ, sh.xchunks, sh.n_pairs);
    ERP_LAUNCH(knn2_exact_kernel, grid, dim3(256), 0, st, desc_q, desc_t, off_q, off_t,
                       sh.xchunk_len, sh.xchunks, sh.max_nq, xpart);
    return hipGetLastError();
}

hipError_t launch_knn2_fold(const Top2* part, const int64_t* off_q, const int64_t* off_t,
                            const BatchShape& sh, int chunk_len, int chunks, Top2* out,
                            hipStream_t st) {
    ERP_LAUNCH(knn2_fold_kernel, dim3((sh.max_nq + 255) / 256, sh.n_pairs), dim3(256), 0,
                       st, part, off_q, off_t, chunk_len, chunks, sh.max_nq, out);
    return hipGetLastError();
}

size_t knn2_merge_scratch_bytes(const BatchShape& sh) {
    return (size_t)sh.n_pairs * ((sh.max_nq + kMergeBlock - 1) / kMergeBlock) * sizeof(int32_t) + 4;
}

hipError_t launch_knn2_merge(const Top2* part, const int64_t* off_q, const int64_t* off_t,
                             const BatchShape& sh, int chunk_len, int chunks, float ratio,
                             erp_dmatch* matches, int32_t* counts, int32_t* flags,
                             int32_t* bcount, hipStream_t st, const BearingOut* bo) {
    const dim3 grid(std::max(1, (sh.max_nq + kMergeBlock - 1) / kMergeBlock), sh.n_pairs);
    const BearingOut none{};
    ERP_LAUNCH(knn2_merge_count_kernel, grid, dim3(kMergeBlock), 0, st, part, off_q, off_t,
                       chunk_len, chunks, sh.max_nq, ratio, bcount);
    ERP_LAUNCH(knn2_merge_kernel, grid, dim3(kMergeBlock), 0, st, part, off_q, off_t,
                       chunk_len, chunks, sh.max_nq, ratio, (const int32_t*)bcount, matches, counts,
                       flags, bo ? *bo : none);
    return hipGetLastError();
}

}  // namespace erp
