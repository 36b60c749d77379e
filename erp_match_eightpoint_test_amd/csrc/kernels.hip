// kernels.hip -- gfx950 kernels of the ERP matcher + spherical eight-point hot path.
//
// Compiled with -ffp-contract=off: every f32 expression that must round like the reference
// (flann::L2 accumulation, ratio test, consensus distances) is written in the reference's
// order and must not be fused; FMA is used only where written explicitly (__builtin_fma in
// the fp64 Gram accumulation, which is parity-checked by tolerance).
//
// Stage                    reference                                   kernel
// exact k=2 + ratio        src/feature_matcher.cpp:42-59               knn2_filter/_rescore/_merge
// gather + pixel->bearing  src/spherical_surf.cpp:155-162,
//                          src/eight_point.cpp:163-186                 bearings_*
// random_array sampler     src/eight_point.hpp:30-59 (glibc replay)    jump_prep / sampler_window /
//                                                                      sampler
// A^T A of the sample      src/eight_point.cpp:22-39                   gram_limbs / gram_mfma
// SVD, rank 2, decompose   src/eight_point.cpp:39-84                   eigen / estimate
// push valid R1/R2         src/eight_point.cpp:113-126                 valid_compact
// trimmed-mean consensus   src/eight_point.cpp:129-149                 consensus_bounds / _select /
//                                                                      _refine / _rows / _final
#include <hip/hip_runtime.h>
#include <atomic>

#include <math.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "erp_device.hpp"
#include "erp_kernels.hpp"
#include "erp_launch.hpp"

namespace erp {

namespace {

constexpr float kInf = __builtin_huge_valf();

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// x^(31+d) mod (x^31 - x^28 - 1), d = 0..29: reduction of a 61-coefficient product
__constant__ uint32_t c_red[30][31];

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

// (the batch pipeline's gather + bearings: knn2_merge_kernel since r05, matcher.hip)

__global__ void bearings_direct_kernel(const erp_point2f* __restrict__ kl,
                                       const erp_point2f* __restrict__ kr, int m, int W, int H,
                                       double* __restrict__ pts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0)
        for (int k = 0; k < 6; k++) pts[(size_t)m * 6 + k] = 0.0;  // zero sentinel row
    if (i >= m) return;
    pixel_to_bearing(W, H, kl[i].x, kl[i].y, pts + (size_t)i * 6);
    pixel_to_bearing(W, H, kr[i].x, kr[i].y, pts + (size_t)i * 6 + 3);
}

// ============================================================ glibc jump-ahead ==========
// glibc TYPE_3: r[n+31] = r[n+28] + r[n] (mod 2^32), so x^d mod P(x) = x^31 - x^28 - 1 maps a
// 31-word window r[n..n+30] to r[n+d..n+d+30].  One wave per pair computes
//   R_l = x^(l(M-1)) (l = 0..64) and Q_k = x^(64(M-1) 2^k),
// the hops from a wave's first hypothesis to each lane's hypothesis and between waves.
// One wave: out = a * b mod P (31 coefficients each, in LDS).  Lane n < 61 forms the
// convolution coefficient c_n; lanes t < 31 then fold c_31..c_60 with the reduction table
// column they hold in registers (cred[d] = c_red[d][t]).  out may alias neither a nor b.
__device__ __forceinline__ void pmul_wave(const uint32_t* a, const uint32_t* b, uint32_t* out,
                                          const uint32_t (&cred)[30]) {
    const int lane = wave_lane();
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 31; i++) {
        const int j = lane - i;
        const uint32_t bj = (j >= 0 && j <= 30) ? b[j < 0 ? 0 : (j > 30 ? 30 : j)] : 0u;
        c += a[i] * bj;
    }
    uint32_t r = c;
#pragma unroll
    for (int d = 0; d < 30; d++) r += (uint32_t)__builtin_amdgcn_readlane((int)c, 31 + d) * cred[d];
    if (lane < 31) out[lane] = r;
}

// x^(2^j) mod P, j < kPow2: the host builds it once (init_constants)
constexpr int kPow2 = 48;  // bits of M - 1 (< 2^16) + 6 + kMaxQ (24) fit
__constant__ uint32_t c_pow2[kPow2][31];

// glibc jump-ahead polynomials of one pair (one block of 16 waves):
//   R_l = x^(l(M-1)) mod P (l = 0..64) and Q_k = x^(64(M-1) 2^k) (k < nq_needed).
// R_1 and every Q_k are products of table powers: x^((M-1) 2^sh) = prod over the set bits b of
// M-1 of x^(2^(b + sh)) (sh = 0 for R_1, 6 + k for Q_k), each on a wave of its own, all at once;
// then R_2..R_64 in six doubling levels (R_{h+j} = R_h R_j, the level's products spread over
// the waves).  popcount(M-1) - 1 + 6 dependent products (11 at M = 2700) instead of the ~26
// of square-and-shift plus repeated squaring (single-pair latency: 28 -> ~12 us).
__global__ __launch_bounds__(1024) void jump_prep_kernel(const int32_t* __restrict__ counts,
                                                         double sample_frac, int nq_needed,
                                                         uint32_t* __restrict__ polyR,
                                                         uint32_t* __restrict__ polyQ) {
    __shared__ uint32_t Rl[65][32];
    __shared__ uint32_t tq[16][2][32];
    __shared__ uint32_t fac[16][16][32];  // each wave's table factors, staged once
    const int p = blockIdx.x, lane = wave_lane(), wid = threadIdx.x >> 6;
    const int M = counts[p];
    if ((int)(M * sample_frac) < 1 || M < 2) return;
    uint32_t cred[30];
#pragma unroll
    for (int d = 0; d < 30; d++) cred[d] = lane < 31 ? c_red[d][lane] : 0u;
    const uint32_t e = (uint32_t)(M - 1);  // >= 1
    uint32_t* Q = polyQ + (size_t)p * kMaxQ * 31;
    // products: item 0 = R_1 (shift 0), item 1 + k = Q_k (shift 6 + k)
    for (int item = wid; item <= nq_needed; item += 16) {
        const int sh = item == 0 ? 0 : 6 + (item - 1);
        // the factors x^(2^(b + sh)) into LDS, all loads in flight at once (pmul_wave reads its
        // second operand per lane: from constant memory that is a dependent load per term)
        int nf = 0;
        for (uint32_t rest = e; rest; rest &= rest - 1u, nf++)  // (uniform)
            if (lane < 31) fac[wid][nf][lane] = c_pow2[__builtin_ctz(rest) + sh][lane];
        int cur = 0;
        if (lane < 31) tq[wid][0][lane] = fac[wid][0][lane];
        for (int f = 1; f < nf; f++) {
            pmul_wave(tq[wid][cur], fac[wid][f], tq[wid][cur ^ 1], cred);
            cur ^= 1;
        }
        if (lane < 31) {
            if (item == 0) {
                Rl[0][lane] = lane == 0 ? 1u : 0u;
                Rl[1][lane] = tq[wid][cur][lane];
            } else {
                Q[(item - 1) * 31 + lane] = tq[wid][cur][lane];
            }
        }
    }
    __syncthreads();
    for (int have = 1; have < 64; have *= 2) {  // R_{have+1 .. 2 have}
        for (int j = wid; j < have; j += 16) pmul_wave(Rl[have], Rl[j + 1], Rl[have + 1 + j], cred);
        __syncthreads();
    }
    uint32_t* R = polyR + (size_t)p * 65 * 31;
    for (int t = threadIdx.x; t < 65 * 31; t += 1024) R[t] = Rl[t / 31][t % 31];
}

// window (31 words in win[]) -> apply polynomial c: win <- x^d window.  ext: 61 words scratch.
__device__ void apply_coop(const uint32_t* __restrict__ c, uint32_t* win, uint32_t* ext) {
    const int lane = wave_lane();
    if (lane < 31) ext[lane] = win[lane];
    __syncthreads();
    if (lane == 0) {
        uint32_t t[61];
#pragma unroll
        for (int k = 0; k < 31; k++) t[k] = ext[k];
#pragma unroll
        for (int d = 31; d < 61; d++) {
            t[d] = t[d - 3] + t[d - 31];
            ext[d] = t[d];
        }
    }
    __syncthreads();
    uint32_t acc = 0;
    if (lane < 31) {
#pragma unroll
        for (int j = 0; j < 31; j++) acc += c[j] * ext[lane + j];
    }
    __syncthreads();
    if (lane < 31) win[lane] = acc;
    __syncthreads();
}

// ====================================================== sampler + Gram accumulation =====
// One lane = one initial_guess iteration h (src/eight_point.cpp:99-112).  The reference
// shuffles iota(M) with M-1 rand() calls (libstdc++ random_shuffle) and keeps the first
// sample_n entries.  Here the same draws are replayed BACKWARDS from the hypothesis's end
// window (glibc's recurrence runs backwards just as cheaply: r[n-31] = r[n] - r[n-3]), which
// lets the final prefix SET be decided with an s-bit bitmap per lane instead of an M-entry
// array:
//   steps i >= s: i stays in the prefix iff it is the LAST hit on position j_i < s;
//   steps i <  s: track the set T of prefix positions whose value is still unresolved
//                 (initially the positions never hit by a step >= s); reverse step i emits i
//                 iff j_i is in T, and then T[j_i] := T[i].
// Three kernels: windows (jump-ahead to each lane's end window), sampler (the replay, writing
// exactly s indices per lane), gram (36 distinct Gram values of the sampled rows, fp64).

// lane end windows: win[p][w][t][lane] = r[base + (64w + lane + 1)(M-1) + t]
__global__ __launch_bounds__(64) void sampler_window_kernel(
    const int32_t* __restrict__ counts, const uint32_t* __restrict__ polyR,
    const uint32_t* __restrict__ polyQ, const uint32_t* __restrict__ w0, int nwaves,
    double sample_frac, uint32_t* __restrict__ wins) {
    __shared__ uint32_t win[32], ext[64];
    const int p = blockIdx.y, w = blockIdx.x, lane = wave_lane();
    const int M = counts[p];
    if ((int)(M * sample_frac) < 1 || M < 2) return;
    if (lane < 31) win[lane] = w0[lane];
    __syncthreads();
    const uint32_t* Q = polyQ + (size_t)p * kMaxQ * 31;
    for (int k = 0; k < kMaxQ && (w >> k); k++)
        if ((w >> k) & 1) apply_coop(Q + k * 31, win, ext);
    if (lane < 31) ext[lane] = win[lane];
    __syncthreads();
    if (lane == 0) {
        uint32_t t[61];
#pragma unroll
        for (int k = 0; k < 31; k++) t[k] = ext[k];
#pragma unroll
        for (int d = 31; d < 61; d++) {
            t[d] = t[d - 3] + t[d - 31];
            ext[d] = t[d];
        }
    }
    __syncthreads();
    uint32_t e[61];
#pragma unroll
    for (int k = 0; k < 61; k++) e[k] = ext[k];
    const uint32_t* R = polyR + ((size_t)p * 65 + (lane + 1)) * 31;
    uint32_t c[31];
#pragma unroll
    for (int j = 0; j < 31; j++) c[j] = R[j];
    uint32_t* o = wins + ((size_t)p * nwaves + w) * 31 * 64 + lane;
#pragma unroll
    for (int t = 0; t < 31; t++) {
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < 31; j++) acc += c[j] * e[t + j];
        o[t * 64] = acc;
    }
}

// exact j = x mod d for x < 2^31, 2 <= d <= 65536, from r = 1/d rounded UP to within
// 2^-32 relative (rup_recip; both conditions are checked exactly with an fma residual when the
// table is built, recip_table_kernel).  Then x*r >= x/d, and x*r - x/d < 2^-1/d, so
// trunc(fl(x*r)) = floor(x/d): for an exact multiple k*d, fl(x*r) >= k (rounding is monotone
// and k is representable); otherwise x/d <= k + 1 - 1/d leaves a margin far above the error.
// The remainder x - q*d is then exact: fma(-q, d, x) in fp64, or for d >= 256 (q < 2^23) one
// v_mad_i32_i24.  The reciprocals come from a table indexed by the step (uniform across the
// wave): scalar loads, issued one block ahead, whose lgkmcnt wait coincides with the block's
// own wait for its LDS atomics.
__device__ __forceinline__ double rup_recip(double dd, bool* bad) {
    const double r0 = __builtin_amdgcn_rcp(dd);
    double r = __builtin_fma(r0, __builtin_fma(-dd, r0, 1.0), r0);
    r = __builtin_fma(r, 0x1p-40, r);                  // one-sided: NR error is ~2^-52
    const double e = __builtin_fma(-dd, r, 1.0);       // exact residual 1 - d*r
    *bad = !(e <= 0.0 && e > -0x1p-32);
    return r;
}

// rtab[d] = rup_recip(d), d = 0 .. n-1 (entries 0, 1 unused: 1.0); *bad counts violations
__global__ __launch_bounds__(256) void recip_table_kernel(int n, double* __restrict__ rtab,
                                                          int32_t* __restrict__ bad) {
    const int d = blockIdx.x * 256 + threadIdx.x;
    if (d >= n) return;
    bool b = false;
    rtab[d] = d >= 2 ? rup_recip((double)d, &b) : 1.0;
    if (b) atomicAdd(bad, 1);
}

__device__ __forceinline__ uint32_t mod_rup(uint32_t x, double r, double dd) {
    const double xd = (double)x;
    const double q = __builtin_trunc(xd * r);
    return (uint32_t)(int32_t)__builtin_fma(-q, dd, xd);
}
// d >= 256: q = floor(x/d) < 2^23, so x - q*d is one 24-bit multiply-add.  The sampler runs
// with the fp64 rounding mode set to round-toward-zero (sampler_kernel's prologue), so
// t = fma(x, r, 2^52) = 2^52 + floor(x r) EXACTLY (x r < 2^31: the sum lies in [2^52, 2^53),
// where the fp64 grid is the integers, and one truncating rounding of the exact x r + 2^52 is
// its floor) and q is t's low word: the fma does the multiply, the truncation and the
// conversion (3 VALU per draw for the modulo instead of 4).
__device__ __forceinline__ uint32_t mod_rup_i24(uint32_t x, double r, int d) {
    const double t = __builtin_fma((double)x, r, 0x1p52);
    const int q = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);
    int j;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(j) : "v"(q), "s"(-d), "v"(x));
    return (uint32_t)j;
}


// ERP_SAMPLER_MAGIC (round 4): the d >= 256 steps' quotient by a 32-bit multiply-high instead of
// the fp64 reciprocal: floor(x / d) = mulhi(x, m_d) >> (l_d - 1) for every x < 2^31 with
// l_d = ceil(log2 d) and m_d = ceil(2^(31 + l_d) / d) < 2^32 (Granlund & Montgomery,
// "Division by invariant integers using multiplication", PLDI 1994, Thm 4.2: 2^(31+l) <= m d <=
// 2^(31+l) + 2^l; checked exactly for every d when the host builds the table).  v_mul_hi_u32 +
// one shift by a scalar (2 VALU, 6 cycles) replaces v_cvt_f64_u32 + v_fma_f64 (8 cycles); the
// remainder stays one v_mad_i32_i24.  The table mtab[d] = m_d | (l_d - 1) << 32 sits right after
// the reciprocal table (rtab + kRecipTable), read by scalar loads like it.
// (default since r04: sampler 6.66 / 6.63 -> 6.43 / 6.42 ms per 768-pair step in a same-box A/B,
// profiles/r04c_ab_sampler_magic.txt; every sampler / full-size fixture test green on it)
#ifndef ERP_SAMPLER_MAGIC
#define ERP_SAMPLER_MAGIC 1
#endif
__device__ __forceinline__ uint32_t mod_magic_i24(uint32_t x, uint64_t mt, int d) {
    const uint32_t q = __umulhi(x, (uint32_t)mt) >> (uint32_t)(mt >> 32);
    int j;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(j) : "v"(q), "s"(-d), "v"(x));
    return (uint32_t)j;
}
// the per-step divisor constant of a d >= 256 step: the magic pair or the reciprocal
#if ERP_SAMPLER_MAGIC
typedef uint64_t StepDiv;
__device__ __forceinline__ StepDiv step_div(const double* rtab, int d) {
    return reinterpret_cast<const uint64_t*>(rtab + kRecipTable)[d];
}
__device__ __forceinline__ uint32_t mod_i24(uint32_t x, StepDiv c, int d) { return mod_magic_i24(x, c, d); }
#else
typedef double StepDiv;
__device__ __forceinline__ StepDiv step_div(const double* rtab, int d) { return rtab[d]; }
__device__ __forceinline__ uint32_t mod_i24(uint32_t x, StepDiv c, int d) { return mod_rup_i24(x, c, d); }
#endif
// the d < 256 steps (round 5): the same magic quotient (the table and its exactness check cover
// every d >= 2, x < 2^31) with the remainder by a full 32-bit multiply (the quotient exceeds
// mad_i24's 24 bits) -- 4 integer ops instead of the fp64 reciprocal's conversions, multiply,
// truncation and residual FMA.  ERP_SAMPLER_MAGIC=0 keeps the fp64 path everywhere.
__device__ __forceinline__ uint32_t mod_small(uint32_t x, uint64_t mt, double r, int d) {
#if ERP_SAMPLER_MAGIC
    (void)r;
    const uint32_t q = __umulhi(x, (uint32_t)mt) >> (uint32_t)(mt >> 32);
    return x - q * (uint32_t)d;
#else
    (void)mt;
    return mod_rup(x, r, (double)d);
#endif
}

// One block of 31 reverse steps i0, i0-1, ..., i0-30 of one lane's replay (ring = the 31-word
// glibc window, advanced backwards in place).  Returns the block's selection word: bit u set
// iff step i0-u's index ends in the sample.  bm = the lane's s-bit LDS bitmap, [word][lane],
// bit SET = position still unresolved (available):
//   steps i >= s (replay_block_draws):   sel = bm[j];  bm[j] := 0
//   steps 1 <= i < s (replay_block_prefix): sel = bm[j];  bm[j] := bm[i]
//   the block straddling s / running below step 1 (replay_block_mixed): per step
// A position j >= s is clamped to s (ERP_SAMPLER_CLAMP, default since r05): bit s is 0 (the
// prologue clears every word of the allocation past the positions < s) and its word is
// allocated, so no LDS access leaves the workgroup's allocation.  Until r05 the clamp was left
// out (one v_min_u32 per draw, sampler ~5 % slower), relying on gfx950 dropping writes and
// returning 0 beyond the allocation (scripts/dev/lds_oob.hip; and an LDS guard kernel beside
// the sampler saw no foreign write, profiles/r05a_lds_guard_stage_bisect.txt) -- undocumented
// behaviour a drop-in exact path should not rest on.  The LDS ops' results are consumed
// kReplayLag steps after issue, so the traffic streams without waits.
// (bm_lane = LDS byte address of the lane's word 0; words are 2^RS B apart -- 256 B for the
// standalone sampler's [word][lane], 1 KB for the fused kernel's [word][wave][lane]: the address
// is one v_lshl_add_u32 of j >> 5)
template <int RS>
__device__ __forceinline__ uint32_t lds_word_addr(uint32_t bm_lane, uint32_t j) {
    uint32_t a;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(a) : "v"(j >> 5), "i"(RS), "v"(bm_lane));
    return a;
}
// uint32 index of word w of the lane's bitmap column
template <int RS>
__device__ __forceinline__ int bm_index(int w, int lane) { return (w << (RS - 2)) + lane; }

// replay blocks consume a step's LDS return `kReplayLag` steps after issuing it (fewer live
// registers than consuming all 31 after the block: occupancy)
constexpr int kReplayLag = 8;

// LDS masked OR with return: old = bm[a]; bm[a] = (old & ~mask) | data (one DS op: the bit
// clear of the i >= s steps with data = 0, the "T[j] := T[i]" bit copy of the prefix steps).
// The compiler does not track the asm's result, so every use goes through an explicit
// lgkmcnt wait that carries the result as an operand.
__device__ __forceinline__ uint32_t lds_mskor_rtn(uint32_t addr, uint32_t mask, uint32_t data) {
    uint32_t old;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(old) : "v"(addr), "v"(mask), "v"(data)
                 : "memory");
    return old;
}

// consume step v of a replay block whose steps 0 .. 30 were issued in order (v + lag issued so
// far): at most `lag` masked ORs may still be in flight after it (LDS returns in order; SMEM in
// the count only makes the wait stricter)
__device__ __forceinline__ void lds_wait_step(uint32_t& o, int v) {
    if (min(30 - v, kReplayLag) >= 8)
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(o) : : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(o) : : "memory");
}

// ERP_SAMPLER_CLAMP=0 (A/B only): the r04 clamp-free draws (positions j >= s address words
// past the allocation)
#ifndef ERP_SAMPLER_CLAMP
#define ERP_SAMPLER_CLAMP 1
#endif
// steps i >= s: one LDS op per draw, positions clamped to s, no validity select
template <bool I24, int RS = 8>
__device__ __forceinline__ uint32_t replay_block_draws(uint32_t (&ring)[31], uint32_t* bm,
                                                       int lane, int i0, int s,
                                                       const double* __restrict__ rtab) {
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    double rt[31];  // 1/(i+1) of the block's steps: scalar loads (uniform index)
    StepDiv mt[31];  // (I24: the d >= 256 divisor constants)
#pragma unroll
    for (int u = 0; u < 31; u++) {
        if (I24 || ERP_SAMPLER_MAGIC) mt[u] = step_div(rtab, i0 - u + 1);
        else rt[u] = rtab[i0 - u + 1];
    }
    const uint32_t zero = 0;
    uint32_t olds[31], pos[31];
    uint32_t nw = 0;
#pragma unroll
    for (int u = 0; u < 31 + kReplayLag; u++) {
        if (u < 31) {
            const int ii = i0 - u;  // uniform, >= s >= 1
            const int slot = 30 - u;
            const uint32_t rv = ring[slot];
            ring[slot] = rv - ring[(slot + 28) % 31];
            uint32_t j = I24 ? mod_i24(rv >> 1, mt[u], ii + 1)
                             : mod_small(rv >> 1, (uint64_t)mt[u], ERP_SAMPLER_MAGIC ? 0.0 : rt[u], ii + 1);
            if (ERP_SAMPLER_CLAMP) j = min(j, (uint32_t)s);  // (bit s: clear and allocated)
            olds[u] = lds_mskor_rtn(lds_word_addr<RS>(bm_lane, j), 1u << (j & 31), zero);
            pos[u] = j;
        }
        const int v = u - kReplayLag;
        if (v >= 0) {
            lds_wait_step(olds[v], v);
            nw |= __builtin_amdgcn_ubfe(olds[v], pos[v], 1) << v;
        }
    }
    return nw;
}

// steps 1 <= i < s with the block's own 31 bits bm[i0-30 .. i0] in one register: bm[i] is a
// constant-position bit extract, the bit copy bm[j] := bm[i] is one masked OR (returning old
// bm[j]), and a step that writes inside the window updates it with one bfi (out-of-window j
// lands on the unused bit 31).  ~17 VALU + 1 DS per step.
template <bool I24, int RS = 8>
__device__ __forceinline__ uint32_t replay_block_prefix(uint32_t (&ring)[31], uint32_t* bm,
                                                        int lane, int i0,
                                                        const double* __restrict__ rtab) {
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    double rt[31];
#pragma unroll
    for (int u = 0; u < 31; u++) rt[u] = rtab[i0 - u + 1];
    const int base = i0 - 30;  // >= 1
    const int wA = i0 >> 5, wB = base >> 5;
    const uint32_t hi = bm[bm_index<RS>(wA, lane)], lo = bm[bm_index<RS>(wB, lane)];
    uint32_t win = wA == wB ? (lo >> (base & 31)) : __builtin_amdgcn_alignbit(hi, lo, base & 31);
    uint32_t olds[31], pos[31];
    uint32_t nw = 0;
#pragma unroll
    for (int u = 0; u < 31 + kReplayLag; u++) {
        if (u < 31) {
            const int ii = i0 - u;
            const int slot = 30 - u;
            const uint32_t rv = ring[slot];
            ring[slot] = rv - ring[(slot + 28) % 31];
            const uint32_t j = I24 ? mod_rup_i24(rv >> 1, rt[u], ii + 1)
                                   : mod_rup(rv >> 1, rt[u], (double)(ii + 1));
            const uint32_t bsp = (uint32_t)__builtin_amdgcn_sbfe((int)win, 30 - u, 1);  // bm[i]
            const uint32_t bit = 1u << (j & 31);
            olds[u] = lds_mskor_rtn(lds_word_addr<RS>(bm_lane, j), bit, bsp & bit);
            pos[u] = j;
            const uint32_t t = min(j - (uint32_t)base, 31u);
            const uint32_t m = 1u << t;
            win = (win & ~m) | (bsp & m);
        }
        const int v = u - kReplayLag;
        if (v >= 0) {
            lds_wait_step(olds[v], v);
            nw |= __builtin_amdgcn_ubfe(olds[v], pos[v], 1) << v;
        }
    }
    return nw;
}

// The same steps with bm[i] read back from LDS per step instead of a register window (no
// window bookkeeping: ~13.5 instead of ~16.5 VALU per step).  A wave's LDS ops complete in
// order, so the read of bm[i] issued after the previous step's masked OR sees it; the read is
// issued before the step's modulo, whose VALU work (and the other waves') covers its latency.
#ifndef ERP_PREFIX_READ
#define ERP_PREFIX_READ 1
#endif
template <bool I24, int RS = 8>
__device__ __forceinline__ uint32_t replay_block_prefix_rd(uint32_t (&ring)[31], uint32_t* bm,
                                                           int lane, int i0,
                                                           const double* __restrict__ rtab) {
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    // the reads are volatile asm, ordered against the masked ORs as volatile asm; only the
    // first carries a memory clobber (every earlier bitmap access is emitted before it, and the
    // block's reciprocal loads above it, where they merge into wide scalar loads -- sunk into
    // the steps one by one, their 31 addresses spill)
    double rt[31];
    StepDiv mt[31];
    uint32_t nw = 0, prev = 0, ppos = 0;
#pragma unroll
    for (int u = 0; u < 31; u++) {
        const int ii = i0 - u;  // uniform, >= 1
        if (u == 0 || u == 16)  // the reciprocals in two halves (SGPR pressure)
#pragma unroll
            for (int k = u; k < (u == 0 ? 16 : 31); k++) {
                if (I24 || ERP_SAMPLER_MAGIC) mt[k] = step_div(rtab, i0 - k + 1);
                else rt[k] = rtab[i0 - k + 1];
            }
        uint32_t rd;
        const uint32_t ra = bm_lane + ((uint32_t)(ii >> 5) << RS);
        if (u == 0 || u == 16)  // the memory clobber holds the half's loads (merged) above it
            asm volatile("ds_read_b32 %0, %1" : "=v"(rd) : "v"(ra) : "memory");
        else
            asm volatile("ds_read_b32 %0, %1" : "=v"(rd) : "v"(ra));
        const int slot = 30 - u;
        const uint32_t rv = ring[slot];
        ring[slot] = rv - ring[(slot + 28) % 31];
        const uint32_t j = I24 ? mod_i24(rv >> 1, mt[u], ii + 1)
                               : mod_small(rv >> 1, (uint64_t)mt[u], ERP_SAMPLER_MAGIC ? 0.0 : rt[u], ii + 1);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rd), "+v"(prev));
        if (u > 0) nw |= __builtin_amdgcn_ubfe(prev, ppos, 1) << (u - 1);
        const uint32_t bsp = (uint32_t)__builtin_amdgcn_sbfe((int)rd, ii & 31, 1);  // bm[i]
        const uint32_t bit = 1u << (j & 31);
        prev = lds_mskor_rtn(lds_word_addr<RS>(bm_lane, j), bit, bsp & bit);
        ppos = j;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(prev) : : "memory");
    return nw | (__builtin_amdgcn_ubfe(prev, ppos, 1) << 30);
}

// the block that straddles s, and the last block that runs below step 1: at most two per
// iteration, so each step is done on its own (compiler-tracked atomics; keeps the kernel's
// register budget at the other blocks' level).  Steps below 1 do nothing.
template <int RS = 8>
__device__ __forceinline__ uint32_t replay_block_mixed(uint32_t (&ring)[31], uint32_t* bm,
                                                       int lane, int i0, int s,
                                                       const double* __restrict__ rtab) {
    uint32_t word = 0;
#pragma unroll
    for (int u = 0; u < 31; u++) {
        const int ii = i0 - u;  // uniform
        const int slot = 30 - u;
        const uint32_t rv = ring[slot];
        ring[slot] = rv - ring[(slot + 28) % 31];
        if (ii < 1) continue;
#if ERP_SAMPLER_MAGIC
        uint32_t j = mod_small(rv >> 1, (uint64_t)step_div(rtab, ii + 1), 0.0, ii + 1);
#else
        uint32_t j = mod_rup(rv >> 1, rtab[ii + 1], (double)(ii + 1));
#endif
        if (ERP_SAMPLER_CLAMP) j = min(j, (uint32_t)s);
        // bm[i] (read before the clear: j = i keeps the bit)
        const uint32_t bi = ii < s ? (bm[bm_index<RS>(ii >> 5, lane)] >> (ii & 31)) & 1u : 0u;
        uint32_t* wp = &bm[bm_index<RS>((int)(j >> 5), lane)];  // j >= s: a cleared or out-of-allocation word
        const uint32_t old = atomicAnd(wp, ~(1u << (j & 31)));
        if (ii < s) atomicOr(wp, bi << (j & 31));
        word |= __builtin_amdgcn_ubfe(old, j, 1) << u;
    }
    return word;
}

// wait until at most n LDS ops are in flight, carrying o as an operand (n is a constant after
// unrolling: the switch folds to one s_waitcnt)
template <int N>
__device__ __forceinline__ void lds_wait_imm(uint32_t& o) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(o) : "n"(N) : "memory");
}
__device__ __forceinline__ void lds_wait_n(uint32_t& o, int n) {
    switch (n) {
#define ERP_W(k) case k: lds_wait_imm<k>(o); break;
        ERP_W(0) ERP_W(1) ERP_W(2) ERP_W(3) ERP_W(4) ERP_W(5) ERP_W(6) ERP_W(7)
        ERP_W(8) ERP_W(9) ERP_W(10) ERP_W(11) ERP_W(12) ERP_W(13) ERP_W(14)
#undef ERP_W
        default: lds_wait_imm<15>(o); break;
    }
}
// a wave alone on its SIMD has nothing else to cover the masked-OR latency: the ILP variants keep
// up to 15 in flight (the lgkmcnt limit) instead of kReplayLag
constexpr int kIlpLag = 15;
// the latency blocks' default (1: step by step, 2: positions first; the context option
// ERP_OPT_SAMPLER_LAT overrides)
constexpr int kSamplerLatMode = 2;

// ---- latency variant (sampler_kernel<2>: waves alone on their SIMDs) -----------------------
// SQ counters of the single-pair path (profiles/r05n_sq_latency.txt): the standalone sampler's
// lone waves sat at s_waitcnt ~40 % of their cycles.  Each block's 31 divisor constants come
// by scalar loads issued at the block's start, and SMEM returns out of order, so their first use
// waits lgkmcnt(0): an L2 round trip per block that also drains the block's in-flight masked
// ORs.  Four waves per SIMD hide that; one does not.  Here the constants of the NEXT block are
// fetched by vector loads (counted by vmcnt, apart from the LDS ops) one block ahead, and the
// prefix blocks keep bm[i] in a register window (no per-step LDS round trip).  Raw 64-bit
// words: the magic pair for d >= 256 blocks (ERP_SAMPLER_MAGIC), else the fp64 reciprocal.
template <bool I24>
__device__ __forceinline__ uint32_t lat_mod(uint32_t x, uint64_t c, int d) {
    if (I24) return mod_i24(x, __builtin_bit_cast(StepDiv, c), d);
    return mod_small(x, c, __builtin_bit_cast(double, c), d);
}

// block kinds: 0 draws (d >= 256), 1 draws, 2 prefix (d >= 256), 3 prefix, 4 mixed / ending
__device__ __forceinline__ int lat_kind(int i, int s) {
    if (i - 30 >= s) return i - 30 >= 255 ? 0 : 1;
    if (i < s && i - 30 >= 1) return i - 30 >= 255 ? 2 : 3;
    return 4;
}

// the constants of block i0 (kinds 0-3: every d = i0 - u + 1 >= 2) by vector loads
__device__ __forceinline__ void lat_fetch(const double* __restrict__ rtab, int i0, int kind,
                                          uint64_t (&c)[31]) {
    const uint64_t* t = reinterpret_cast<const uint64_t*>(rtab) + (ERP_SAMPLER_MAGIC ? kRecipTable : 0);
    (void)kind;
    int d0 = i0 + 1;
    asm volatile("" : "+v"(d0));  // a VGPR index: global (vmcnt) loads, not scalar ones
#pragma unroll
    for (int u = 0; u < 31; u++) c[u] = t[d0 - u];
}
// a use of every constant of a set before the next set's loads are issued: the compiler's wait
// for this set (vmcnt) then cannot count the next set's loads in (at a loop head it would wait
// vmcnt(0), i.e. for the loads just issued)
__device__ __forceinline__ void lat_ready(uint64_t (&c)[31]) {
#pragma unroll
    for (int u = 0; u < 28; u += 4)
        asm volatile("" : "+v"(c[u]), "+v"(c[u + 1]), "+v"(c[u + 2]), "+v"(c[u + 3]));
    asm volatile("" : "+v"(c[28]), "+v"(c[29]), "+v"(c[30]));
}

// PF: the block's 31 positions first (31 independent modulo chains for the scheduler to
// interleave: a lone wave has no other wave to cover a chain's dependent-issue latency), then the
// masked ORs with up to kIlpLag in flight; else each step's chain in turn (lag kReplayLag)
template <bool I24, bool PF>
__device__ __forceinline__ void lat_positions(uint32_t (&ring)[31], int i0, const uint64_t (&c)[31],
                                              uint32_t (&jj)[31]) {
#pragma unroll
    for (int u = 0; u < 31; u++) {
        const int slot = 30 - u;
        const uint32_t rv = ring[slot];
        ring[slot] = rv - ring[(slot + 28) % 31];
        jj[u] = lat_mod<I24>(rv >> 1, c[u], i0 - u + 1);
    }
}

template <bool I24, bool PF, int RS = 8>
__device__ __forceinline__ uint32_t replay_block_draws_lat(uint32_t (&ring)[31], uint32_t* bm,
                                                           int lane, int i0, int s,
                                                           const uint64_t (&c)[31]) {
    constexpr int LAG = PF ? kIlpLag : kReplayLag;
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    const uint32_t zero = 0;
    uint32_t olds[31], jj[31];
    if (PF) lat_positions<I24, PF>(ring, i0, c, jj);
    uint32_t nw[2] = {0, 0};
#pragma unroll
    for (int u = 0; u < 31 + LAG; u++) {
        if (u < 31) {
            if (!PF) {
                const int slot = 30 - u;
                const uint32_t rv = ring[slot];
                ring[slot] = rv - ring[(slot + 28) % 31];
                jj[u] = lat_mod<I24>(rv >> 1, c[u], i0 - u + 1);
            }
            if (ERP_SAMPLER_CLAMP) jj[u] = min(jj[u], (uint32_t)s);
            olds[u] = lds_mskor_rtn(lds_word_addr<RS>(bm_lane, jj[u]), 1u << (jj[u] & 31), zero);
        }
        const int v = u - LAG;
        if (v >= 0) {
            lds_wait_n(olds[v], min(30 - v, LAG));
            nw[v & 1] |= __builtin_amdgcn_ubfe(olds[v], jj[v], 1) << v;
        }
    }
    return nw[0] | nw[1];
}

template <bool I24, bool PF, int RS = 8>
__device__ __forceinline__ uint32_t replay_block_prefix_lat(uint32_t (&ring)[31], uint32_t* bm,
                                                            int lane, int i0,
                                                            const uint64_t (&c)[31]) {
    constexpr int LAG = PF ? kIlpLag : kReplayLag;
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    const int base = i0 - 30;  // >= 1
    const int wA = i0 >> 5, wB = base >> 5;
    // (compiler-tracked reads: its wait for them is at least as strict as needed, since the
    // masked ORs issued after them only add to the count)
    const uint32_t hi = bm[bm_index<RS>(wA, lane)], lo = bm[bm_index<RS>(wB, lane)];
    uint32_t win = wA == wB ? (lo >> (base & 31)) : __builtin_amdgcn_alignbit(hi, lo, base & 31);
    uint32_t olds[31], jj[31];
    if (PF) lat_positions<I24, PF>(ring, i0, c, jj);
    uint32_t nw[2] = {0, 0};
#pragma unroll
    for (int u = 0; u < 31 + LAG; u++) {
        if (u < 31) {
            if (!PF) {
                const int slot = 30 - u;
                const uint32_t rv = ring[slot];
                ring[slot] = rv - ring[(slot + 28) % 31];
                jj[u] = lat_mod<I24>(rv >> 1, c[u], i0 - u + 1);
            }
            const uint32_t j = jj[u];
            const uint32_t bsp = (uint32_t)__builtin_amdgcn_sbfe((int)win, 30 - u, 1);  // bm[i]
            const uint32_t bit = 1u << (j & 31);
            olds[u] = lds_mskor_rtn(lds_word_addr<RS>(bm_lane, j), bit, bsp & bit);
            const uint32_t t = min(j - (uint32_t)base, 31u);
            const uint32_t m = 1u << t;
            win = (win & ~m) | (bsp & m);
        }
        const int v = u - LAG;
        if (v >= 0) {
            lds_wait_n(olds[v], min(30 - v, LAG));
            nw[v & 1] |= __builtin_amdgcn_ubfe(olds[v], jj[v], 1) << v;
        }
    }
    return nw[0] | nw[1];
}

template <bool PF, int RS>
__device__ __forceinline__ uint32_t replay_block_lat(uint32_t (&ring)[31], uint32_t* bm, int lane,
                                                     int i, int s, int kind,
                                                     const double* __restrict__ rtab,
                                                     const uint64_t (&c)[31]) {
    switch (kind) {
        case 0: return replay_block_draws_lat<true, PF, RS>(ring, bm, lane, i, s, c);
        case 1: return replay_block_draws_lat<false, PF, RS>(ring, bm, lane, i, s, c);
        case 2: return replay_block_prefix_lat<true, PF, RS>(ring, bm, lane, i, c);
        case 3: return replay_block_prefix_lat<false, PF, RS>(ring, bm, lane, i, c);
        default: return replay_block_mixed<RS>(ring, bm, lane, i, s, rtab);
    }
}

// the 31 reverse steps i .. i-30 of one lane's replay, by block kind (uniform: i and s are)
template <int RS>
__device__ __forceinline__ uint32_t replay_block(uint32_t (&ring)[31], uint32_t* bm, int lane,
                                                 int i, int s, const double* __restrict__ rtab) {
    if (i - 30 >= s && i - 30 >= 255) return replay_block_draws<true, RS>(ring, bm, lane, i, s, rtab);
    if (i - 30 >= s) return replay_block_draws<false, RS>(ring, bm, lane, i, s, rtab);
    if (i < s && i - 30 >= 255)
        return ERP_PREFIX_READ ? replay_block_prefix_rd<true, RS>(ring, bm, lane, i, rtab)
                               : replay_block_prefix<true, RS>(ring, bm, lane, i, rtab);
    if (i < s && i - 30 >= 1)
        return ERP_PREFIX_READ ? replay_block_prefix_rd<false, RS>(ring, bm, lane, i, rtab)
                               : replay_block_prefix<false, RS>(ring, bm, lane, i, rtab);
    return replay_block_mixed<RS>(ring, bm, lane, i, s, rtab);
}

// One lane = one iteration; writes the iteration's selection bitmap in block space:
// sel[p][w][b][lane] bit u <-> index i = M-1-31b-u (b = 0 .. (M-1)/31), exactly s bits set.
// MODE 0: the throughput blocks; 2 / 3: the latency blocks, step by step / positions first
// (constants prefetched one block ahead by vector loads, two blocks per loop trip so that the two
// constant sets alternate without register copies)
template <int MODE>
__global__ __launch_bounds__(64) void sampler_kernel(
    const int32_t* __restrict__ counts, const uint32_t* __restrict__ wins, int nwaves, int nbw,
    double sample_frac, const double* __restrict__ rtab, uint32_t* __restrict__ selw,
    int32_t* __restrict__ flags, int nalloc) {
    extern __shared__ uint32_t bm[];  // [nwords][64]
    const int p = blockIdx.y, w = blockIdx.x, lane = wave_lane();
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || M < 2) return;
    // fp64 round-toward-zero for the rest of the wave (mod_rup_i24's fma; mod_rup stays exact
    // under it: trunc of a one-sided product, then an exact fma residual)
    // (inline asm: the compiler's mode-register pass would otherwise put the default mode back
    // in front of every fp64 instruction; nothing else in this kernel depends on fp64 rounding)
    asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3\n\ts_nop 3" ::: "memory");
    // positions < s available, every other bitmap word of the allocation (nalloc words: the
    // batch's largest s, rounded up to the allocation granule) clear
    for (int k = 0; k < nalloc; k++)
        bm[k * 64 + lane] = k < (s >> 5) ? ~0u : k == (s >> 5) ? (1u << (s & 31)) - 1u : 0u;
    uint32_t ring[31];
    {
        const uint32_t* wi = wins + ((size_t)p * nwaves + w) * 31 * 64 + lane;
#pragma unroll
        for (int t = 0; t < 31; t++) ring[t] = wi[t * 64];
    }
    uint32_t* out = selw + ((size_t)p * nwaves + w) * (size_t)nbw * 64 + lane;
    const int b0 = (M - 1) / 31, u0 = (M - 1) % 31;  // slot of position 0
    int i = M - 1, b = 0, emitted = 0;
    uint32_t lastw = 0;
    auto emit = [&](uint32_t word) {
        emitted += __builtin_popcount(word);
        if (b == b0) lastw = word;
        else out[(size_t)b * 64] = word;
        i -= 31;
        b++;
    };
    if (MODE >= 2) {
        uint64_t ca[31] = {}, cb[31] = {};
        int ka = lat_kind(i, s);
        if (ka < 4) lat_fetch(rtab, i, ka, ca);
        while (i >= 1) {
            const int kb = i - 31 >= 1 ? lat_kind(i - 31, s) : 4;
            lat_ready(ca);
            if (kb < 4) lat_fetch(rtab, i - 31, kb, cb);
            emit(replay_block_lat<MODE == 3, 8>(ring, bm, lane, i, s, ka, rtab, ca));
            if (i < 1) break;
            ka = i - 31 >= 1 ? lat_kind(i - 31, s) : 4;
            lat_ready(cb);
            if (ka < 4) lat_fetch(rtab, i - 31, ka, ca);
            emit(replay_block_lat<MODE == 3, 8>(ring, bm, lane, i, s, kb, rtab, cb));
        }
    } else {
        while (i >= 1) emit(replay_block<8>(ring, bm, lane, i, s, rtab));
    }
    if (bm[lane] & 1u) {  // position 0 still unresolved: its value 0 stays in the prefix
        lastw |= 1u << u0;
        emitted++;
    }
    out[(size_t)b0 * 64] = lastw;
    if (emitted != s) atomicOr(&flags[p], 2);  // internal consistency check
}

// ---- split replay (round 5; launches of <= 256 workgroups, e.g. one pair) -------------------
// A lone wave replays an iteration's M - 1 steps one after the other (~125 us at M ~ 3.4k).  The
// steps i >= s only ever CLEAR bits of the bitmap (a step keeps i iff it is the last hit on its
// position j < s, i.e. the first in the reverse order), so they split into segments: segment g
// (blocks [nbd g / G, nbd (g + 1) / G) of the nbd all-draw blocks) is replayed exactly once its
// start bitmap is known -- the positions < s that no earlier segment hit.  So kSplitG waves per
// workgroup (64 iterations, one wave per segment) first collect their segment's hit set H_g
// (one LDS OR per draw, no return, no wait), then, after one barrier, replay their segment with
// the bitmap avail & ~(H_0 | ... | H_{g-1}); a last wave replays the prefix / mixed blocks that
// follow with avail & ~(H_0 | ... | H_{G-1}) -- exactly the state the serial replay reaches there.
// Each wave first walks the glibc window back to its segment (31 subtractions per block, ~0.1 of
// a draw).  The selection words are the serial kernel's, word for word.
#ifndef ERP_SPLIT_G
#define ERP_SPLIT_G 3
#endif
#ifndef ERP_SPLIT_STAMPS
#define ERP_SPLIT_STAMPS 0
#endif
constexpr int kSplitG = ERP_SPLIT_G;  // draw segments (+ 1 prefix wave: 4 waves, one per SIMD)

template <bool I24, int RS = 8>
__device__ __forceinline__ void split_hits_block(uint32_t (&ring)[31], uint32_t* bm, int lane,
                                                 int i0, int s, const uint64_t (&c)[31]) {
    const uint32_t bm_lane = (uint32_t)(size_t)(lds_u32*)bm + 4u * (uint32_t)lane;
    uint32_t jj[31];
    lat_positions<I24, true>(ring, i0, c, jj);
#pragma unroll
    for (int u = 0; u < 31; u++) {
        const uint32_t j = min(jj[u], (uint32_t)s);  // (bit s: allocated, cleared below)
        asm volatile("ds_or_b32 %0, %1" : : "v"(lds_word_addr<RS>(bm_lane, j)), "v"(1u << (j & 31))
                     : "memory");
    }
}

// the window walked back over one block without draws
__device__ __forceinline__ void ring_skip_block(uint32_t (&ring)[31]) {
#pragma unroll
    for (int u = 0; u < 31; u++) {
        const int slot = 30 - u;
        ring[slot] = ring[slot] - ring[(slot + 28) % 31];
    }
}

// blocks [b0, b1) of the replay (block b: steps M-1-31b .. M-31-31b; those below step 1 ignored),
// each block's divisor constants fetched one block ahead as in sampler_kernel<2/3>
template <typename F>
__device__ __forceinline__ void lat_blocks(int M, int s, int b0, int b1,
                                           const double* __restrict__ rtab, F&& fn) {
    uint64_t ca[31] = {}, cb[31] = {};
    auto live = [&](int b) { return b < b1 && M - 1 - 31 * b >= 1; };
    auto kind = [&](int b) { return live(b) ? lat_kind(M - 1 - 31 * b, s) : 4; };
    int b = b0;
    int ka = kind(b);
    if (live(b) && ka < 4) lat_fetch(rtab, M - 1 - 31 * b, ka, ca);
    while (live(b)) {
        const int kb = kind(b + 1);
        lat_ready(ca);
        if (live(b + 1) && kb < 4) lat_fetch(rtab, M - 1 - 31 * (b + 1), kb, cb);
        fn(b, ka, ca);
        b++;
        if (!live(b)) break;
        ka = kind(b + 1);
        lat_ready(cb);
        if (live(b + 1) && ka < 4) lat_fetch(rtab, M - 1 - 31 * (b + 1), ka, ca);
        fn(b, kb, cb);
        b++;
    }
}

__global__ __launch_bounds__(64 * (kSplitG + 1)) void sampler_split_kernel(
    const int32_t* __restrict__ counts, const uint32_t* __restrict__ wins, int nwaves, int nbw,
    double sample_frac, const double* __restrict__ rtab, uint32_t* __restrict__ selw,
    int32_t* __restrict__ flags, int nalloc) {
    extern __shared__ uint32_t sm[];  // H[G][nalloc][64], then B[G + 1][nalloc][64]
    __shared__ int esum[64];
    const int p = blockIdx.y, w = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || M < 2) return;  // (uniform over the workgroup)
    asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3\n\ts_nop 3" ::: "memory");
#if ERP_SPLIT_STAMPS
    uint64_t ts[8];
    ts[0] = __builtin_amdgcn_s_memtime();
#endif
    const size_t reg = (size_t)nalloc * 64;
    uint32_t* H = sm + (size_t)wv * reg;                    // (segment waves)
    uint32_t* Bm = sm + (size_t)(kSplitG + wv) * reg;        // this wave's replay bitmap
    auto avail = [&](int k) -> uint32_t {
        return k < (s >> 5) ? ~0u : k == (s >> 5) ? (1u << (s & 31)) - 1u : 0u;
    };
    if (wv < kSplitG)
        for (int k = 0; k < nalloc; k++) H[k * 64 + lane] = 0u;
    if (wv == 0) esum[lane] = 0;
    const int nbd = M - 31 - s >= 0 ? (M - 31 - s) / 31 + 1 : 0;  // all-draw blocks
    const int bb = wv < kSplitG ? nbd * wv / kSplitG : nbd;
    const int be = wv < kSplitG ? nbd * (wv + 1) / kSplitG : 0x7fffffff;
    uint32_t ring[31];
    {
        const uint32_t* wi = wins + ((size_t)p * nwaves + w) * 31 * 64 + lane;
#pragma unroll
        for (int t = 0; t < 31; t++) ring[t] = wi[t * 64];
    }
    for (int b = 0; b < bb; b++) ring_skip_block(ring);
#if ERP_SPLIT_STAMPS
    ts[1] = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();  // (H and esum cleared)
    // pass 1 (segment waves): the segment's hit set (positions clamped to s like the replay's)
    uint32_t ring0[31];
#pragma unroll
    for (int t = 0; t < 31; t++) ring0[t] = ring[t];
    if (wv < kSplitG)
        lat_blocks(M, s, bb, be, rtab, [&](int b, int kind, const uint64_t(&c)[31]) {
            const int i0 = M - 1 - 31 * b;
            if (kind == 0) split_hits_block<true>(ring, H, lane, i0, s, c);
            else split_hits_block<false>(ring, H, lane, i0, s, c);
        });
    // (the asm ORs are not in the compiler's count: drain them before the barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if ERP_SPLIT_STAMPS
    ts[2] = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();  // (every segment's hits in H)
#if ERP_SPLIT_STAMPS
    ts[3] = __builtin_amdgcn_s_memtime();
#endif
    // this wave's start bitmap: avail minus the hits of the segments before it (all of them for
    // the prefix wave); bit s and the words past it stay clear
    // (words 8 at a time, every region's read of them issued before the first use: one LDS
    // round trip per 8 words instead of one per read -- 15-18k cycles -> a few thousand)
    const int lim = wv < kSplitG ? wv : kSplitG;
    for (int k0 = 0; k0 < nalloc; k0 += 8) {
        uint32_t e[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
        for (int x = 0; x < kSplitG; x++) {
            if (x < lim) {
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (k0 + q < nalloc) e[q] |= sm[(size_t)x * reg + (k0 + q) * 64 + lane];
            }
        }
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (k0 + q < nalloc) Bm[(k0 + q) * 64 + lane] = avail(k0 + q) & ~e[q];
    }
#if ERP_SPLIT_STAMPS
    ts[4] = __builtin_amdgcn_s_memtime();
#endif
    // pass 2: the exact replay of this wave's blocks (the words are the serial kernel's)
#pragma unroll
    for (int t = 0; t < 31; t++) ring[t] = ring0[t];
    uint32_t* out = selw + ((size_t)p * nwaves + w) * (size_t)nbw * 64 + lane;
    const int b0 = (M - 1) / 31, u0 = (M - 1) % 31;  // slot of position 0 (a prefix-wave block)
    int emitted = 0;
    uint32_t lastw = 0;
    lat_blocks(M, s, bb, be, rtab, [&](int b, int kind, const uint64_t(&c)[31]) {
        const uint32_t word = replay_block_lat<true, 8>(ring, Bm, lane, M - 1 - 31 * b, s, kind, rtab, c);
        emitted += __builtin_popcount(word);
        if (b == b0) lastw = word;
        else out[(size_t)b * 64] = word;
    });
#if ERP_SPLIT_STAMPS
    ts[5] = __builtin_amdgcn_s_memtime();
#endif
    if (wv == kSplitG) {
        if (Bm[lane] & 1u) {  // position 0 still unresolved: its value 0 stays in the prefix
            lastw |= 1u << u0;
            emitted++;
        }
        out[(size_t)b0 * 64] = lastw;
    }
    atomicAdd(&esum[lane], emitted);
    __syncthreads();
    if (wv == kSplitG && esum[lane] != s) atomicOr(&flags[p], 2);  // internal consistency check
#if ERP_SPLIT_STAMPS  // (diagnostic builds only: one workgroup's phase times, in shader cycles)
    if (blockIdx.x == 0 && blockIdx.y == 0 && lane == 0)
        printf("split wave %d: skip %d pass1 %d barrier %d init %d pass2 %d (blocks %d..%d, M %d s %d)\n",
               wv, (int)(ts[1] - ts[0]), (int)(ts[2] - ts[1]), (int)(ts[3] - ts[2]),
               (int)(ts[4] - ts[3]), (int)(ts[5] - ts[4]), bb, be, M, s);
#endif
}

// the estimate of one iteration from its selected vector e (rank-2 fix, decomposition, Euler
// angles, validity) into its hypothesis record
// ---- counter-based sampler (ERP_SAMPLER_PHILOX) ------------------------------------------
// No reference counterpart (the reference replays glibc rand(): sampler_kernel above); SURVEY.md
// section 8b's `sampler = PHILOX`: iteration h's s-subset of [0, M) by Floyd's algorithm on
// Philox4x32-10 draws, exactly as oracle/erp_oracle.c erpo_philox_sample defines it:
//   draw k (j = M - s + k): u_k = philox(ctr = (lo32(h), hi32(h), k / 4, 0), key = (seed,
//   0x243F6A88))[k mod 4], t = mulhi(u_k, j + 1); t joins the set unless it is there, then j.
// h = offset + iteration.  s draws per iteration instead of the replay's M - 1 (a quarter at
// the reference's sample_frac), each a Philox quarter-block (~20 VALU) and an LDS bit test-and-
// set; no serial dependence between iterations, so no jump polynomials or windows.  One lane =
// one iteration, an M-bit LDS bitmap per lane ([word][lane]: the 32 lanes of a bank group on 32
// banks); the set is then written in the replay's selection-word format (bit u of word b <->
// index M-1-31b-u), which the Gram kernel reads unchanged.
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        // one 32x32->64 product each (v_mad_u64_u32) instead of a mul_hi + mul_lo pair
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0, n2;  // three-input xors (gfx950 v_bitop3, LUT 0x96 = a ^ b ^ c)
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c[1]), "s"(k0));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c[3]), "s"(k1));
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

__global__ __launch_bounds__(64) void philox_sampler_kernel(
    const int32_t* __restrict__ counts, int iters, int nwaves, int nbw, double sample_frac,
    uint32_t seed, uint64_t offset, int nwords, uint32_t* __restrict__ selw,
    int32_t* __restrict__ flags) {
    extern __shared__ uint32_t bm[];  // [nwords][64]
    const int p = blockIdx.y, w = blockIdx.x, lane = wave_lane();
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || M < 2) return;
    uint32_t* out = selw + ((size_t)p * nwaves + w) * (size_t)nbw * 64 + lane;
    const int nb = (M - 1) / 31 + 1;
    if ((M + 31) / 32 > nwords) {  // M beyond the per-lane LDS bitmap (> 20 480): loud status
        if (lane == 0) atomicOr(&flags[p], 8);  // ERP_INVALID_ARG; empty sets for the Gram pass
        for (int b = 0; b < nb; b++) out[(size_t)b * 64] = 0u;
        return;
    }
    const int mw = (M + 31) / 32;
    for (int k = 0; k < mw; k++) bm[k * 64 + lane] = 0u;
    const uint64_t h = offset + (uint64_t)(w * 64 + lane);
    uint32_t u[4];
    for (int k0 = 0; k0 < s; k0 += 4) {
        u[0] = (uint32_t)h;
        u[1] = (uint32_t)(h >> 32);
        u[2] = (uint32_t)(k0 >> 2);
        u[3] = 0u;
        philox4x32_10(u, seed, 0x243F6A88u);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int k = k0 + q;
            if (k < s) {  // (uniform)
                const uint32_t j = (uint32_t)(M - s + k);
                const uint32_t t = __umulhi(u[q], j + 1u);
                const uint32_t old = atomicOr(&bm[(t >> 5) * 64 + lane], 1u << (t & 31));
                if (old & (1u << (t & 31))) atomicOr(&bm[(j >> 5) * 64 + lane], 1u << (j & 31));
            }
        }
    }
    // the set as selection words: block b holds indices hi = M-1-31b down to hi - 30
    int emitted = 0;
    for (int b = 0; b < nb; b++) {
        const int hi = M - 1 - 31 * b, lo = hi - 30;  // lo may be negative (the last block)
        const int l0 = lo < 0 ? 0 : lo;
        const uint32_t a = bm[(l0 >> 5) * 64 + lane];
        const uint32_t c = ((l0 >> 5) + 1) < mw ? bm[((l0 >> 5) + 1) * 64 + lane] : 0u;
        uint32_t win = __builtin_amdgcn_alignbit(c, a, (uint32_t)(l0 & 31));  // bits l0 ..
        if (lo < 0) win = (win << (-lo));  // position v of the window <-> index lo + v
        win &= 0x7fffffffu;                // the block's 31 indices lo .. hi
        const uint32_t word = __builtin_bitreverse32(win) >> 1;  // bit u <-> index hi - u
        emitted += __builtin_popcount(word);
        out[(size_t)b * 64] = word;
    }
    if (emitted != s) atomicOr(&flags[p], 2);  // internal consistency check
}

__device__ __forceinline__ void estimate_store(const double* e, double valid_abs,
                                               erp_hypothesis* __restrict__ o,
                                               bool with_e = true) {
    Hyp hy;
    estimate_from_e(e, valid_abs, hy);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        o->R1[k] = hy.R1[k];
        o->R2[k] = hy.R2[k];
        o->T[k] = hy.T[k];
    }
    o->R1_valid = hy.R1_valid;
    o->R2_valid = hy.R2_valid;
    o->inliers = 0;  // (the opt-in inlier_count_kernel overwrites it)
    if (!with_e) return;  // E is only read when the caller asked for the records
#pragma unroll
    for (int k = 0; k < 9; k++) o->E[k] = hy.E[k];
}

// ---- Gram on int8 MFMA: exact fixed-point sums -------------------------------------------
// G_h = sum over the sampled rows i of P_i, P_i = (l l^T) x (r r^T) (36 distinct values), is a
// product of the 0/1 selection matrix (iterations x rows) with P (rows x 36).  Each P_i value
// (|P| <= 1) is rounded ONCE to the fixed point q = rint(P 2^44) and split into 6 balanced
// base-256 digits (int8), so G_h 2^44 = sum_limb 256^limb * (selection x digits_limb) is
// computed EXACTLY by v_mfma_i32_32x32x32_i8 (the int32 sums stay below 65536 * 128 < 2^31)
// and recombined in int64; the only roundings are the per-row quantisation (<= 2^-45 per
// value, <= s 2^-45 per Gram entry: below the fp64 FMA chain's own s-step accumulation error)
// and the final conversion to double.  Sums are order-independent and deterministic.
// K order = the sampler's selection words: k = 32 b + u <-> row M-1-31b-u (u < 31; u = 31 is
// a zero pad), so the A operand is the selection word itself, expanded 4 bits -> 4 bytes by
// one 24-bit multiply and a mask.  Columns: tile t < 6 holds limb t of entries c = 0..31 (one
// entry per lane: its 6 limbs recombine in registers), tile 6 holds the 6 limbs of entries
// 32..35 (column 4 limb + c - 32; recombined by lane shuffles).
constexpr int kGramLimbs = 6;
constexpr int kGramTiles = 7;                 // 32-column MFMA tiles
constexpr int kGramN = kGramTiles * 32;
constexpr double kGramScale = 0x1p44;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// G 2^44 = sum_t a_t 256^t from the six limb sums, times 2^-44, in fp64 without the int64
// recombination (|a_t| <= 65537 * 128 < 2^24): the partial sums of limbs 0-2 and 3-5 are
// integers below 2^41 (exact in fp64, the power-of-two scalings too), and the last FMA rounds
// their exact sum once -- the same correctly rounded value as (double)(int64 sum) * 2^-44, for
// 6 conversions and 5 FMAs instead of the int64 shifts, adds and int64 -> fp64 conversions
__device__ __forceinline__ double gram_join(int a0, int a1, int a2, int a3, int a4, int a5) {
    const double lo = __builtin_fma((double)a2, 0x1p-28,
                                    __builtin_fma((double)a1, 0x1p-36, (double)a0 * 0x1p-44));
    const double hi = __builtin_fma((double)a5, 0x1p16, __builtin_fma((double)a4, 0x1p8, (double)a3));
    return __builtin_fma(hi, 0x1p-20, lo);
}

__device__ __forceinline__ int gram_col(int limb, int c) {
    return c < 32 ? limb * 32 + c : 192 + limb * 4 + (c - 32);
}

// Byte u of column n in a word's 7 KB limb image: 32 B per column, the two 16-B halves swapped
// on columns with bit 3 set, so the ds_read_b128 of 16 consecutive columns (half hh) covers all
// 64 banks once.  The image is copied into LDS unchanged (lane-linear LDS-DMA).
__device__ __forceinline__ int gram_swz(int n, int u) {
    return n * 32 + ((((u >> 4) ^ (n >> 3)) & 1) << 4) + (u & 15);
}

// limbs[p][b][7 KB image]: byte u of column n = gram_col(limb, c) = digit of row M-1-31b-u
__global__ __launch_bounds__(256) void gram_limbs_kernel(const int32_t* __restrict__ counts,
                                                         const double* __restrict__ pts,
                                                         int max_nq, int nbw,
                                                         int8_t* __restrict__ limbs) {
    __shared__ __align__(16) int8_t tile[kGramN * 32];
    const int p = blockIdx.y, b = blockIdx.x, tid = threadIdx.x;
    const int M = counts[p];
    if (M < 2 || b > (M - 1) / 31) return;
    for (int k = tid; k < kGramN * 32 / 16; k += 256)
        reinterpret_cast<uint4*>(tile)[k] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const double* P = pts + (size_t)p * (max_nq + 1) * 6;
    for (int item = tid; item < 31 * 36; item += 256) {
        const int u = item / 36, c = item - 36 * (item / 36);
        const int i = M - 1 - 31 * b - u;
        if (i < 0) continue;
        const double* pr = P + (size_t)i * 6;
        const int a = c / 6, e = c - 6 * (c / 6);
        // (l l^T) and (r r^T) index pairs 00 01 02 11 12 22 (entry c = 6 a + e)
        const int ai = a < 3 ? 0 : (a < 5 ? 1 : 2), aj = a < 3 ? a : (a < 5 ? a - 2 : 2);
        const int ei = e < 3 ? 0 : (e < 5 ? 1 : 2), ej = e < 3 ? e : (e < 5 ? e - 2 : 2);
        const double LL = pr[ai] * pr[aj], RR = pr[3 + ei] * pr[3 + ej];
        long long q = __double2ll_rn((LL * RR) * kGramScale);
#pragma unroll
        for (int k = 0; k < kGramLimbs; k++) {
            const int d = (int)(int8_t)(q & 0xff);
            tile[gram_swz(gram_col(k, c), u)] = (int8_t)d;
            q = (q - d) >> 8;
        }
    }
    __syncthreads();
    uint4* o = reinterpret_cast<uint4*>(limbs + ((size_t)p * nbw + b) * kGramN * 32);
    for (int k = tid; k < kGramN * 32 / 16; k += 256) o[k] = reinterpret_cast<const uint4*>(tile)[k];
}

// Block = kGramWaves waves x 32 WT iterations (WT MFMA row tiles each); K loop over the pair's
// selection words, two words (64 rows, 14 WT MFMAs per wave) per step.  Operands reach LDS only by
// LDS-DMA (global_load_lds: the 14 KB limb images of the step's two words and the block's
// 2 x 32 WT kGramWaves selection words) into a ring of GramCfg::kRing slots, issued kRing - 1
// steps ahead: the selection words stream from HBM once, and their latency is covered by the ring, not
// by occupancy.  The limb images are read once per block and step, so the block's iteration
// count sets the L2 -> LDS traffic per MFMA.  One raw
// barrier per step after a counted vmcnt (never 0 in the loop); all LDS in one __shared__ array.
// All 14 B fragments of a step are read before the first MFMA.  gram[p][36][iters] (SoA, the
// eigen layout).
// (measured r02h, per 384-pair step: 4 waves / 3 blocks per CU 2.42 ms; 8 waves -- half the
// L2 -> LDS image traffic -- 2.44; 6 waves 2.91 (a 6-wave block loads the SIMDs 2/2/1/1); all
// 14 fragment reads issued before the first MFMA (ERP_GRAM_SCHED, 194 VGPRs) 2.55-2.63)
#ifndef ERP_GRAM_WAVES
#define ERP_GRAM_WAVES 4
#endif
#ifndef ERP_GRAM_SCHED
#define ERP_GRAM_SCHED 0
#endif
constexpr int kGramWaves = ERP_GRAM_WAVES;                      // waves per block
constexpr int kGramWords = 2;                                   // selection words per K step
constexpr int kGramWordBytes = kGramN * 32;                     // one word's limb image (7 KB)
constexpr int kGramSelOff = kGramWords * kGramWordBytes;        // selection words in a slot
#ifndef ERP_GRAM_RING
#define ERP_GRAM_RING 3
#endif
#ifndef ERP_GRAM_MINBLOCKS
#define ERP_GRAM_MINBLOCKS 3
#endif
constexpr int kGramPieces = kGramSelOff / 1024;                 // 1-KB limb pieces per step
static_assert(kGramPieces == 14, "14 limb pieces of 1 KB per step");
// WT = 32-iteration row tiles per wave (round 5).  WT = 2: every B fragment read from LDS feeds
// two MFMAs (14 accumulator tiles, 256 registers, 2 waves per SIMD), 256 iterations per block, a
// 5-slot ring (80 KB: the epilogue's 256 Grams fit) and 2 blocks per CU -- gram 5.12 -> 4.72 ms
// per step (profiles/r05f_ab_gram_wt.txt).  WT = 1 (32 iterations per wave, 3 blocks per CU)
// keeps small launches (one pair: 79 blocks of 128 iterations, not 40 of 256) spread over the
// CUs.  ERP_GRAM_WT = 1 / 2 forces one (default 0: by launch size, launch_gram_mfma).
template <int WT>
struct GramCfg {
    static constexpr int kIters = 32 * kGramWaves * WT;         // iterations per block
    static constexpr int kChunks = kIters / 64;                 // 64-iteration sampler waves
    static constexpr int kSelPW = kGramWords * kChunks / kGramWaves;  // selection-word DMAs per wave
    static constexpr int kRing = WT == 1 ? ERP_GRAM_RING : 5;   // slots: DMAs kRing - 1 steps ahead
    static constexpr int kSlotBytes = kGramSelOff + kGramWords * kIters * 4;
    static constexpr int kMinBlocks = WT == 1 ? ERP_GRAM_MINBLOCKS : 2;
    static_assert(kRing >= 3, "ring");
    static_assert(kIters % 64 == 0 && kGramWords * kChunks % kGramWaves == 0 && kGramWaves <= 14,
                  "whole selection-word DMAs per wave");
};
// limb pieces moved by wave w: the first (14 % W) waves move one more
constexpr int gram_pieces_of(int w) {
    return kGramPieces / kGramWaves + (w < kGramPieces % kGramWaves ? 1 : 0);
}
constexpr int gram_piece0(int w) {
    return w * (kGramPieces / kGramWaves) + (w < kGramPieces % kGramWaves ? w : kGramPieces % kGramWaves);
}

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef const __attribute__((address_space(1))) void* glb_vptr;

template <int WT>
__global__ __launch_bounds__(64 * kGramWaves, GramCfg<WT>::kMinBlocks) void gram_mfma_kernel(
    const int32_t* __restrict__ counts, const int8_t* __restrict__ limbs,
    const uint32_t* __restrict__ selw, int iters, int nwaves, int nbw, double sample_frac,
    double* __restrict__ gram, int nhb, double* __restrict__ evec,
    erp_hypothesis* __restrict__ hyps, double valid_abs) {
    using C = GramCfg<WT>;
    __shared__ __align__(16) int8_t lds[C::kRing * C::kSlotBytes];
    // XCD-aware block order (1-D grid of nhb iteration blocks x pairs): workgroups go to the 8
    // XCDs round-robin by linear id, so XCD x takes the contiguous logical range
    // [x NB/8, (x+1) NB/8) -- all iteration blocks of a pair on one XCD, whose L2 then holds the
    // pair's limb images (7 KB per selection word) for every block instead of each XCD
    // fetching them from HBM (identity when NB is not a multiple of 8)
    const int NB = gridDim.x;
    const int lbk = (NB & 7) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (NB >> 3) + (blockIdx.x >> 3));
    const int p = lbk / nhb, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || M < 2) return;
    const int hb = (lbk % nhb) * C::kIters;
    if (hb >= iters) return;  // uniform over the block
    const int nb = (M - 1) / 31 + 1;
    const int nsteps = (nb + kGramWords - 1) / kGramWords;  // words read: <= 2 nsteps - 1 <= nb < nbw
    const int h0 = hb + wv * 32 * WT;
    const int r = lane & 31, hh = lane >> 5;
    const int8_t* lg = limbs + (size_t)p * nbw * kGramWordBytes + lane * 16;
    // wave wv moves limb pieces gram_piece0(wv) .. + gram_pieces_of(wv) - 1 and the selection
    // words d = wv C::kSelPW + e: word d / C::kChunks of 64-iteration chunk d % C::kChunks
    // (chunks past the last iteration are clamped: their rows are never stored)
    const int lp0 = [&] {
        int v = 0;
#pragma unroll
        for (int w = 0; w < kGramWaves; w++) v = (w == wv) ? gram_piece0(w) : v;
        return v;
    }();
    const bool extra = wv < kGramPieces % kGramWaves;  // moves kGramPieces / W + 1 pieces
    const uint32_t* sg[C::kSelPW];
#pragma unroll
    for (int e = 0; e < C::kSelPW; e++) {
        const int d = wv * C::kSelPW + e;
        const int chunk = min((hb >> 6) + d % C::kChunks, nwaves - 1);
        sg[e] = selw + ((size_t)p * nwaves + chunk) * (size_t)nbw * 64 + lane +
                (size_t)(d / C::kChunks) * 64;
    }
    const int soff = kGramSelOff + wv * C::kSelPW * 256;
    auto issue = [&](int step) {
        const int sx = min(step, nsteps - 1);  // past the end: a harmless reload, never read
        int8_t* slot = lds + (step % C::kRing) * C::kSlotBytes;
        const int8_t* src = lg + (size_t)sx * kGramSelOff;
#pragma unroll
        for (int k = 0; k < kGramPieces / kGramWaves; k++)
            __builtin_amdgcn_global_load_lds((glb_vptr)(src + (lp0 + k) * 1024),
                                             (lds_vptr)(slot + (lp0 + k) * 1024), 16, 0, 0);
        if (extra)
            __builtin_amdgcn_global_load_lds(
                (glb_vptr)(src + (lp0 + kGramPieces / kGramWaves) * 1024),
                (lds_vptr)(slot + (lp0 + kGramPieces / kGramWaves) * 1024), 16, 0, 0);
#pragma unroll
        for (int e = 0; e < C::kSelPW; e++)
            __builtin_amdgcn_global_load_lds((glb_vptr)(sg[e] + (size_t)(sx * kGramWords) * 64),
                                             (lds_vptr)(slot + soff + e * 256), 4, 0, 0);
    };
    i32x16 acc[WT][kGramTiles];
#pragma unroll
    for (int w = 0; w < WT; w++)
#pragma unroll
        for (int t = 0; t < kGramTiles; t++)
#pragma unroll
            for (int k = 0; k < 16; k++) acc[w][t][k] = 0;
#pragma unroll
    for (int k = 0; k < C::kRing - 1; k++) issue(k);
    const int boff = r * 32 + (((hh ^ (r >> 3)) & 1) << 4);
    for (int st = 0; st < nsteps; st++) {
        // step st's DMAs retired: the C::kRing - 2 later steps may fly (pieces + 1 each)
        constexpr int kBase = kGramPieces / kGramWaves + C::kSelPW;
        static_assert((kBase + 1) * (C::kRing - 2) <= 63, "vmcnt range");
        if (extra) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kBase + 1) * (C::kRing - 2)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kBase * (C::kRing - 2)) : "memory");
        __builtin_amdgcn_s_barrier();
        issue(st + C::kRing - 1);  // into the slot every wave finished reading in step st - 1
        const int8_t* slot = lds + (st % C::kRing) * C::kSlotBytes;
        // every B fragment of the step in flight at once (the MFMAs then wait on counted
        // lgkmcnts): the step's LDS latency is exposed once, not once per fragment pair
        i32x4 bf[kGramWords][kGramTiles];
#pragma unroll
        for (int i = 0; i < kGramWords; i++)
#pragma unroll
            for (int t = 0; t < kGramTiles; t++)
                bf[i][t] = *reinterpret_cast<const i32x4*>(slot + i * kGramWordBytes +
                                                           t * 32 * 32 + boff);
        uint32_t wsel[WT][kGramWords];  // read after the fragments: one wait covers the step
#pragma unroll
        for (int w = 0; w < WT; w++)
#pragma unroll
            for (int i = 0; i < kGramWords; i++)
                wsel[w][i] = reinterpret_cast<const uint32_t*>(slot + kGramSelOff)[
                    i * C::kIters + (wv * WT + w) * 32 + r];
        i32x4 a[WT][kGramWords];
#pragma unroll
        for (int w = 0; w < WT; w++)
#pragma unroll
            for (int i = 0; i < kGramWords; i++) {
                const uint32_t wm = (st * kGramWords + i < nb) ? 0xffffu : 0u;  // words past nb
                const uint32_t bits = (wsel[w][i] >> (16 * hh)) & wm;
#pragma unroll
                for (int v = 0; v < 4; v++)
                    a[w][i][v] = (int)((((bits >> (4 * v)) & 0xfu) * 0x00204081u) & 0x01010101u);
            }
#if ERP_GRAM_SCHED
        __builtin_amdgcn_sched_group_barrier(0x100, kGramWords * (kGramTiles + 1), 0);  // LDS reads
        __builtin_amdgcn_sched_group_barrier(0x002, 4 * kGramWords * 4, 0);            // VALU
        __builtin_amdgcn_sched_group_barrier(0x008, kGramWords * kGramTiles, 0);       // MFMAs
#endif
#pragma unroll
        for (int i = 0; i < kGramWords; i++)
#pragma unroll
            for (int t = 0; t < kGramTiles; t++)
#pragma unroll
                for (int w = 0; w < WT; w++)
                    acc[w][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[w][i], bf[i][t], acc[w][t], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's tail DMAs
    // recombine: row = (k & 3) + 8 (k >> 2) + 4 hh; entry r from tiles 0..5 of this lane,
    // entries 32..35 from tile 6 (lane 4 limb + e)
    double* go = gram + (size_t)p * 36 * iters;
    if (evec && s >= 9) {  // uniform over the block
        // fused eigen stage: the block's 128 Grams go through LDS (the ring, now idle) instead
        // of an HBM round trip; waves 0 and 1 then run the inverse iteration of eigen_kernel
        // on one iteration per lane.  Only the lanes that do not settle write their Gram to HBM
        // (for eigen_fallback_kernel, which finds them by the NaN in evec).  hyps != NULL: the
        // settled lanes also run the estimate (estimate_kernel's work) here.
        constexpr int kStg = C::kIters + 1;  // [36][kStg] doubles: odd stride, no bank conflicts
        static_assert(36 * kStg * 8 <= C::kRing * C::kSlotBytes, "Gram stage fits the ring");
        double* stg = reinterpret_cast<double*>(lds);
        __syncthreads();  // every wave's last fragment reads have returned
#pragma unroll
        for (int w = 0; w < WT; w++)
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int row = (wv * WT + w) * 32 + (k & 3) + 8 * (k >> 2) + 4 * hh;
            static_assert(kGramLimbs == 6, "gram_join takes six limbs");
            const int x = acc[w][kGramLimbs][k];
            int y[kGramLimbs];
#pragma unroll
            for (int t = 0; t < kGramLimbs; t++) y[t] = __shfl(x, (lane & 32) + 4 * t + (r & 3), 64);
            stg[r * kStg + row] = gram_join(acc[w][0][k], acc[w][1][k], acc[w][2][k], acc[w][3][k],
                                            acc[w][4][k], acc[w][5][k]);
            if (r < 4) stg[(32 + r) * kStg + row] = gram_join(y[0], y[1], y[2], y[3], y[4], y[5]);
        }
        __syncthreads();
        if (wv >= C::kIters / 64) return;
        const int hl = wv * 64 + lane, h = hb + hl;
        double e[9];
        const bool ok = gram_min_eigvec9_inv(stg, kStg, hl, e);
        if (h >= iters) return;
        if (!ok) {
            e[0] = __builtin_nan("");
#pragma unroll 4
            for (int k = 0; k < 36; k++) go[(size_t)k * iters + h] = stg[k * kStg + hl];
        } else if (hyps) {
            estimate_store(e, valid_abs, hyps + (size_t)p * iters + h);
            evec[(size_t)p * 9 * iters + h] = 0.0;  // settled (eigen_fallback_kernel skips it)
            return;
        }
        double* eo = evec + (size_t)p * 9 * iters + h;
#pragma unroll
        for (int k = 0; k < 9; k++) eo[(size_t)k * iters] = e[k];
        return;
    }
#pragma unroll
    for (int w = 0; w < WT; w++)
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int row = w * 32 + (k & 3) + 8 * (k >> 2) + 4 * hh;
        const int x = acc[w][kGramLimbs][k];
        int y[kGramLimbs];
#pragma unroll
        for (int t = 0; t < kGramLimbs; t++) y[t] = __shfl(x, (lane & 32) + 4 * t + (r & 3), 64);
        if (h0 + row < iters) {
            go[(size_t)r * iters + h0 + row] = gram_join(acc[w][0][k], acc[w][1][k], acc[w][2][k],
                                                         acc[w][3][k], acc[w][4][k], acc[w][5][k]);
            if (r < 4)
                go[(size_t)(32 + r) * iters + h0 + row] = gram_join(y[0], y[1], y[2], y[3], y[4], y[5]);
        }
    }
}

// debug output: the sampled match indices of every iteration (as a set, descending), from the
// selection words
__global__ __launch_bounds__(64) void samples_kernel(const int32_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ selw, int iters,
                                                     int nwaves, int nbw, int idx_stride,
                                                     double sample_frac,
                                                     int32_t* __restrict__ samples) {
    const int p = blockIdx.y, lane = wave_lane();
    const int h = blockIdx.x * 64 + lane;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || M < 2 || h >= iters) return;
    const uint32_t* sp = selw + ((size_t)p * nwaves + blockIdx.x) * (size_t)nbw * 64 + lane;
    int32_t* o = samples + ((size_t)p * iters + h) * idx_stride;
    int n = 0;
    for (int b = 0; b <= (M - 1) / 31; b++) {
        uint32_t w = sp[(size_t)b * 64];
        while (w) {
            const int u = __builtin_ctz(w);
            w &= w - 1u;
            if (n < idx_stride) o[n] = M - 1 - 31 * b - u;
            n++;
        }
    }
}

// Gram of ALL m rows (eight_point_estimation called directly, src/manual.cpp:152)
__global__ __launch_bounds__(256) void gram_all_kernel(const double* __restrict__ pts, int m,
                                                       double* __restrict__ gram) {
    __shared__ double red[36][256];
    const int tid = threadIdx.x;
    double g[36];
#pragma unroll
    for (int k = 0; k < 36; k++) g[k] = 0.0;
    for (int v = tid; v < m; v += 256) {
        const double* pt = pts + (size_t)v * 6;
        const double l0 = pt[0], l1 = pt[1], l2 = pt[2], r0 = pt[3], r1 = pt[4], r2 = pt[5];
        const double LL[6] = {l0 * l0, l0 * l1, l0 * l2, l1 * l1, l1 * l2, l2 * l2};
        const double RR[6] = {r0 * r0, r0 * r1, r0 * r2, r1 * r1, r1 * r2, r2 * r2};
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int b = 0; b < 6; b++) g[6 * a + b] = __builtin_fma(LL[a], RR[b], g[6 * a + b]);
    }
#pragma unroll
    for (int k = 0; k < 36; k++) red[k][tid] = g[k];
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o)
#pragma unroll
            for (int k = 0; k < 36; k++) red[k][tid] += red[k][tid + o];
        __syncthreads();
    }
    if (tid < 36) gram[tid] = red[tid][0];
}

// ========================================================= per-hypothesis solve ==========
// THIN = false: pairs with s >= 9 (V-free eigenvector); THIN = true: pairs with s < 9
// (rotation-accumulated Jacobi).  Two instantiations so the common case is not sized by the
// thin path's 162 live doubles; each returns at once for the other class of pairs.  The
// selected vector overwrites the first 9 doubles of the iteration's Gram record; the
// estimate (rank-2 fix, decomposition, Euler angles) runs in estimate_kernel.
template <bool THIN>
__global__ __launch_bounds__(64) void eigen_kernel(const int32_t* __restrict__ counts,
                                                   const double* __restrict__ gram, int iters,
                                                   double sample_frac,
                                                   double* __restrict__ evec,
                                                   erp_hypothesis* __restrict__ hyps,
                                                   double valid_abs) {
    const int p = blockIdx.y;
    const int h = blockIdx.x * 64 + threadIdx.x;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || h >= iters || (s < 9) != THIN) return;
    // gram[p][36][iters] (SoA): the solve reads the 36 values with stride iters, the vector
    // goes to evec[p][9][iters]
    const double* gi = gram + (size_t)p * 36 * iters + h;
    double e[9];
    if (THIN) {
        double g36[36], G[81];
#pragma unroll
        for (int k = 0; k < 36; k++) g36[k] = gi[(size_t)k * iters];
        gram36_to_full(g36, G);
        gram_jacobi9(G, s, e);
    } else if (!gram_min_eigvec9_inv(gi, iters, 0, e)) {
        e[0] = __builtin_nan("");  // not settled: eigen_fallback_kernel takes the Jacobi path
    }
    if (THIN && hyps) {  // the fused pipeline has no estimate_kernel
        estimate_store(e, valid_abs, hyps + (size_t)p * iters + h);
        return;
    }
    double* eo = evec + (size_t)p * 9 * iters + h;
#pragma unroll
    for (int k = 0; k < 9; k++) eo[(size_t)k * iters] = e[k];
}

// the lanes whose inverse iteration did not settle (near-degenerate lambda_1 ~ lambda_2; rare):
// eigenvalue shift by cyclic Jacobi, then inverse iteration (gram_min_eigvec9_jacobi)
__global__ __launch_bounds__(64) void eigen_fallback_kernel(const int32_t* __restrict__ counts,
                                                            const double* __restrict__ gram,
                                                            int iters, double sample_frac,
                                                            double* __restrict__ evec,
                                                            erp_hypothesis* __restrict__ hyps,
                                                            double valid_abs) {
    const int p = blockIdx.y;
    const int h = blockIdx.x * 64 + threadIdx.x;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 9 || h >= iters) return;
    double* eo = evec + (size_t)p * 9 * iters + h;
    if (!__builtin_isnan(eo[0])) return;
    double e[9];
    gram_min_eigvec9_jacobi(gram + (size_t)p * 36 * iters + h, iters, 0, e);
    if (hyps) {  // the fused pipeline has no estimate_kernel
        estimate_store(e, valid_abs, hyps + (size_t)p * iters + h);
        return;
    }
#pragma unroll
    for (int k = 0; k < 9; k++) eo[(size_t)k * iters] = e[k];
}

// the fused pipeline's leftovers in ONE launch (single-pair latency: one dispatch fewer): pairs
// with s < 9 take eigen_kernel<true>'s thin path, the others eigen_fallback_kernel's (only the
// lanes the Gram kernel's inverse iteration left NaN)
__global__ __launch_bounds__(64) void eigen_rest_kernel(const int32_t* __restrict__ counts,
                                                        const double* __restrict__ gram, int iters,
                                                        double sample_frac,
                                                        double* __restrict__ evec,
                                                        erp_hypothesis* __restrict__ hyps,
                                                        double valid_abs) {
    const int p = blockIdx.y;
    const int h = blockIdx.x * 64 + threadIdx.x;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || h >= iters) return;
    double* eo = evec + (size_t)p * 9 * iters + h;
    const double* gi = gram + (size_t)p * 36 * iters + h;
    double e[9];
    if (s < 9) {
        double g36[36], G[81];
#pragma unroll
        for (int k = 0; k < 36; k++) g36[k] = gi[(size_t)k * iters];
        gram36_to_full(g36, G);
        gram_jacobi9(G, s, e);
    } else {
        if (!__builtin_isnan(eo[0])) return;
        gram_min_eigvec9_jacobi(gi, iters, 0, e);
    }
    if (hyps) {
        estimate_store(e, valid_abs, hyps + (size_t)p * iters + h);
        return;
    }
#pragma unroll
    for (int k = 0; k < 9; k++) eo[(size_t)k * iters] = e[k];
}

#ifdef ERP_EST_WAVES
#define ERP_EST_ATTR __attribute__((amdgpu_waves_per_eu(ERP_EST_WAVES)))
#else
#define ERP_EST_ATTR
#endif
__global__ __launch_bounds__(64) ERP_EST_ATTR void estimate_kernel(const int32_t* __restrict__ counts,
                                                      const double* __restrict__ evec, int iters,
                                                      double sample_frac, double valid_abs,
                                                      erp_hypothesis* __restrict__ hyps,
                                                      int with_e) {
    const int p = blockIdx.y;
    const int h = blockIdx.x * 64 + threadIdx.x;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1 || h >= iters) return;
    const double* ei = evec + (size_t)p * 9 * iters + h;
    double e[9];
#pragma unroll
    for (int k = 0; k < 9; k++) e[k] = ei[(size_t)k * iters];
    estimate_store(e, valid_abs, hyps + (size_t)p * iters + h, with_e != 0);
}

// The batch pipeline's estimate when nothing asks for the hypothesis records (round 5): instead
// of 120-B records that valid_count / valid_scatter read back twice (~3.1 GB per 768-pair
// step), each iteration's R1, R2, T go to hl[p][9][iters] as f32 SoA (36 B, coalesced; an
// invalid rotation's x is NaN: valid implies max |euler| < 1.57, so a valid x is finite), and
// each 64-iteration wave writes its valid-rotation count and their bounding box to
// wsum[p][wave][8] -- what valid_place_kernel needs to place R1-then-R2 in iteration order
// (src/eight_point.cpp:117-126) without re-reading the iterations twice.
// REST (batches with fewer waves than the chip has SIMDs, e.g. one pair): eigen_rest_kernel's
// work -- the thin path of s < 9 pairs, the Jacobi fallback of lanes the Gram kernel left NaN --
// in this launch too (one dependent launch fewer; the wider register budget costs nothing when
// the chip is mostly idle)
template <bool REST>
__global__ __launch_bounds__(64) ERP_EST_ATTR void estimate_lite_kernel(
    const int32_t* __restrict__ counts, const double* __restrict__ evec, int iters,
    double sample_frac, double valid_abs, float* __restrict__ hl, int32_t* __restrict__ wsum,
    const double* __restrict__ gram) {
    const int p = blockIdx.y, w = blockIdx.x, lane = threadIdx.x;
    const int h = w * 64 + lane;
    const int M = counts[p];
    const int s = (int)(M * sample_frac);
    if (s < 1) return;  // (uniform: valid_place_kernel reports K = 0 for the pair)
    Hyp hy;
    hy.R1_valid = hy.R2_valid = 0;
    if (h < iters) {
        const double* ei = evec + (size_t)p * 9 * iters + h;
        double e[9];
#pragma unroll
        for (int k = 0; k < 9; k++) e[k] = ei[(size_t)k * iters];
        if (REST) {
            const double* gi = gram + (size_t)p * 36 * iters + h;
            if (s < 9) {
                double g36[36], G[81];
#pragma unroll
                for (int k = 0; k < 36; k++) g36[k] = gi[(size_t)k * iters];
                gram36_to_full(g36, G);
                gram_jacobi9(G, s, e);
            } else if (__builtin_isnan(e[0])) {
                gram_min_eigvec9_jacobi(gi, iters, 0, e);
            }
        }
        estimate_from_e(e, valid_abs, hy);
        float* o = hl + (size_t)p * 9 * iters + h;
        const float qnan = __builtin_nanf("");
        o[0] = hy.R1_valid ? hy.R1[0] : qnan;
        o[(size_t)1 * iters] = hy.R1[1];
        o[(size_t)2 * iters] = hy.R1[2];
        o[(size_t)3 * iters] = hy.R2_valid ? hy.R2[0] : qnan;
        o[(size_t)4 * iters] = hy.R2[1];
        o[(size_t)5 * iters] = hy.R2[2];
#pragma unroll
        for (int k = 0; k < 3; k++) o[(size_t)(6 + k) * iters] = hy.T[k];
    }
    int cnt = (hy.R1_valid != 0) + (hy.R2_valid != 0);
    float mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (hy.R1_valid) {
            mn[k] = fminf(mn[k], hy.R1[k]);
            mx[k] = fmaxf(mx[k], hy.R1[k]);
        }
        if (hy.R2_valid) {
            mn[k] = fminf(mn[k], hy.R2[k]);
            mx[k] = fmaxf(mx[k], hy.R2[k]);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], o, 64));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], o, 64));
        }
    }
    if (lane < 8) {
        const int32_t v = lane == 0 ? cnt : lane < 4 ? __float_as_int(mn[lane - 1])
                          : lane < 7 ? __float_as_int(mx[lane - 4]) : 0;
        wsum[((size_t)p * gridDim.x + w) * 8 + lane] = v;
    }
}

// push R1 (if valid) then R2 (if valid) per iteration, in iteration order
// Two launches over (chunk of 1024 iterations, pair): valid_count_kernel writes each chunk's
// number of valid rotations and its bounding box; valid_scatter_kernel adds the totals of the
// chunks before it (at most ~200 values) and block-scans its chunk, keeping the reference's
// push order (iteration, then R1, R2).  Chunk 0 also writes K and the bounding-box diagonal
// of the valid R set (>= every pairwise distance: the scale of the consensus histograms).
// vchunk[p][c] = {count, min x, min y, min z, max x, max y, max z, pad}
__device__ __forceinline__ int hyp_valid_count(const erp_hypothesis& hy) {
    return (hy.R1_valid != 0) + (hy.R2_valid != 0);
}

__global__ __launch_bounds__(1024) void valid_count_kernel(const int32_t* __restrict__ counts,
                                                           const erp_hypothesis* __restrict__ hyps,
                                                           int iters, double sample_frac,
                                                           int32_t* __restrict__ vchunk) {
    __shared__ int ws[16];
    __shared__ float red6[6][16];
    const int p = blockIdx.y, c = blockIdx.x, tid = threadIdx.x;
    const int M = counts[p];
    if ((int)(M * sample_frac) < 1) return;
    const int h = c * 1024 + tid;
    erp_hypothesis hy;
    hy.R1_valid = 0;
    hy.R2_valid = 0;
    if (h < iters) hy = hyps[(size_t)p * iters + h];
    float mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
#pragma unroll
    for (int which = 0; which < 2; which++) {
        if (!(which ? hy.R2_valid : hy.R1_valid)) continue;
        const float* R = which ? hy.R2 : hy.R1;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], R[k]);
            mx[k] = fmaxf(mx[k], R[k]);
        }
    }
    int total;
    (void)block_exclusive_scan<1024>(hyp_valid_count(hy), ws, &total);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float a = mn[k], b = mx[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a = fminf(a, __shfl_xor(a, o, 64));
            b = fmaxf(b, __shfl_xor(b, o, 64));
        }
        if ((tid & 63) == 0) {
            red6[k][tid >> 6] = a;
            red6[3 + k][tid >> 6] = b;
        }
    }
    __syncthreads();
    int32_t* o = vchunk + ((size_t)p * gridDim.x + c) * 8;
    if (tid == 0) o[0] = total;
    if (tid >= 1 && tid <= 6) {
        const int k = tid - 1;
        float v = k < 3 ? kInf : -kInf;
        for (int w = 0; w < 16; w++) v = k < 3 ? fminf(v, red6[k][w]) : fmaxf(v, red6[k][w]);
        o[tid] = __float_as_int(v);
    }
}

__global__ __launch_bounds__(1024) void valid_scatter_kernel(const int32_t* __restrict__ counts,
                                                             const erp_hypothesis* __restrict__ hyps,
                                                             int iters, double sample_frac,
                                                             const int32_t* __restrict__ vchunk,
                                                             float* __restrict__ rv,
                                                             float* __restrict__ tv,
                                                             int32_t* __restrict__ kcount,
                                                             float* __restrict__ rv_aos,
                                                             float* __restrict__ dscale) {
    __shared__ int ws[16];
    __shared__ int sbase[16];
    const int p = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, nch = gridDim.x;
    const int M = counts[p];
    if ((int)(M * sample_frac) < 1) {
        if (c == 0 && tid == 0) kcount[p] = 0;
        return;
    }
    const int32_t* vc = vchunk + (size_t)p * nch * 8;
    // chunks before this one (and, for chunk 0, all of them: K and the bounding box)
    const int upto = c == 0 ? nch : c;
    int part = 0;
    for (int q = tid; q < upto; q += 1024) part += vc[q * 8];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if ((tid & 63) == 0) sbase[tid >> 6] = part;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < 16; w++) base += sbase[w];
    if (c == 0) {
        if (tid == 0) {
            kcount[p] = base;
            double d2 = 0;
            for (int k = 0; k < 3; k++) {
                float a = kInf, b = -kInf;
                for (int q = 0; q < nch; q++) {
                    a = fminf(a, __int_as_float(vc[q * 8 + 1 + k]));
                    b = fmaxf(b, __int_as_float(vc[q * 8 + 4 + k]));
                }
                const double e = base > 0 ? (double)b - (double)a : 0.0;
                d2 += e * e;
            }
            dscale[p] = (float)(sqrt(d2) * (1.0 + 1e-6));
        }
        base = 0;
    }
    const int h = c * 1024 + tid;
    erp_hypothesis hy;
    hy.R1_valid = 0;
    hy.R2_valid = 0;
    if (h < iters) hy = hyps[(size_t)p * iters + h];
    int total;
    int pos = base + block_exclusive_scan<1024>(hyp_valid_count(hy), ws, &total);
    const int stride = 2 * iters;
    float* X = rv + (size_t)p * 3 * stride;
    float* T = tv + (size_t)p * 3 * stride;
    float* A = rv_aos ? rv_aos + (size_t)p * 3 * stride : nullptr;
#pragma unroll
    for (int which = 0; which < 2; which++) {
        if (!(which ? hy.R2_valid : hy.R1_valid)) continue;
        const float* R = which ? hy.R2 : hy.R1;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            X[k * stride + pos] = R[k];
            T[3 * pos + k] = hy.T[k];
            if (A) A[3 * pos + k] = R[k];
        }
        pos++;
    }
}

// ============================================== opt-in inlier count (cfg.inlier_thr > 0) ===
// No reference counterpart (src/eight_point.cpp:99-127 keeps no score): for every
// iteration, the matches among ALL M with |l^T E' r| < thr, E' = E_mat_correct of that
// iteration (:45-50), fp64 in the fixed order of inlier_residual (erp_device.hpp).  Work per
// pair: M x iters residuals (~2.7e7 at configs[1]), so the count runs in f32 and only the band
// the f32 evaluation cannot decide is redone exactly:
//   |res32 - res64| <= (9 + 4 + 1) 2^-24 sum_k |E'_k| |u_k| <= 14 2^-24 ||E'||_F |l| |r|
//                   ~= 8.4e-7   (9 roundings of the FMA chain, 3 of u = fl(fl(l) fl(r)), 1 of
//                                fl(E'); ||E'||_F <= ||e|| = 1 and |l| = |r| = 1 up to ulps),
// so with d = 2^-19 (~1.9e-6, twice that plus the rounding of thr -+ d to f32) |res32| < thr - d
// is an inlier, |res32| >= thr + d is not, and the rest is recomputed in fp64.
constexpr float kInlierBand = 0x1p-19f;
constexpr int kInlierChunk = 256;  // matches per pass of a wave (4 per lane)

// E' of every iteration from its record's e (rank2_correct: the estimate's own operations) ->
// ec64 [p][iters][9] (the exact path) and its f32 image ec32 [p][iters][16]
__global__ __launch_bounds__(64) void inlier_prep_kernel(const int32_t* __restrict__ counts,
                                                         const erp_hypothesis* __restrict__ hyps,
                                                         int iters, double sample_frac,
                                                         double* __restrict__ ec64,
                                                         float* __restrict__ ec32) {
    const int p = blockIdx.y, h = blockIdx.x * 64 + threadIdx.x;
    if ((int)(counts[p] * sample_frac) < 1 || h >= iters) return;
    const erp_hypothesis* hy = hyps + (size_t)p * iters + h;
    double e[9], Ec[9];
#pragma unroll
    for (int k = 0; k < 9; k++) e[k] = hy->E[k];
    rank2_correct(e, Ec);
    double* o = ec64 + ((size_t)p * iters + h) * 9;
    float* f = ec32 + ((size_t)p * iters + h) * 16;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        o[k] = Ec[k];
        f[k] = (float)Ec[k];
    }
}

// u = fl(l) (x) fl(r) per match as f32, SoA [p][9][mpad]; rows >= M are NaN (never counted)
__global__ __launch_bounds__(256) void inlier_points_kernel(const int32_t* __restrict__ counts,
                                                            const double* __restrict__ pts,
                                                            int max_nq, int mpad,
                                                            float* __restrict__ u32) {
    const int p = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= mpad) return;
    float* o = u32 + (size_t)p * 9 * mpad + i;
    if (i >= counts[p]) {
#pragma unroll
        for (int k = 0; k < 9; k++) o[(size_t)k * mpad] = __builtin_nanf("");
        return;
    }
    const double* q = pts + ((size_t)p * (max_nq + 1) + i) * 6;
    const float l[3] = {(float)q[0], (float)q[1], (float)q[2]};
    const float r[3] = {(float)q[3], (float)q[4], (float)q[5]};
#pragma unroll
    for (int k = 0; k < 9; k++) o[(size_t)k * mpad] = l[k / 3] * r[k % 3];
}

// One wave per 64 iterations of a pair.  The wave holds 256 matches in VGPRs (u: 4 per lane)
// and runs its iterations over them with E' wave-uniform (scalar loads): 9 f32 FMAs per
// (match, iteration), the wave-reduced count popcount(ballot(|res| < thr - d)) on the SALU, the
// band [thr - d, thr + d) recomputed in fp64 by its lanes.  Iteration h's count accumulates in
// lane h of `acc`, written into the record once at the end.
__global__ __launch_bounds__(64) void inlier_count_kernel(
    const int32_t* __restrict__ counts, const float* __restrict__ u32,
    const float* __restrict__ ec32, const double* __restrict__ ec64,
    const double* __restrict__ pts, int max_nq, int mpad, int iters, double sample_frac,
    float thr_lo, float thr_hi, double thr, erp_hypothesis* __restrict__ hyps) {
    const int p = blockIdx.y, lane = threadIdx.x, h0 = blockIdx.x * 64;
    const int M = counts[p];
    if ((int)(M * sample_frac) < 1) return;
    const int nh = min(64, iters - h0);
    const float* U = u32 + (size_t)p * 9 * mpad;
    const float* E32 = ec32 + ((size_t)p * iters + h0) * 16;
    int acc = 0;
    for (int c0 = 0; c0 < M; c0 += kInlierChunk) {
        float u[4][9];
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int k = 0; k < 9; k++) u[q][k] = U[(size_t)k * mpad + c0 + q * 64 + lane];
        for (int h = 0; h < nh; h++) {
            const float* e = E32 + h * 16;
            float ev[9];
#pragma unroll
            for (int k = 0; k < 9; k++) ev[k] = e[k];
            int cnt = 0;
            uint64_t amb_any = 0;
            bool amb[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float res = ev[0] * u[q][0];
#pragma unroll
                for (int k = 1; k < 9; k++) res = fmaf(ev[k], u[q][k], res);
                const float a = fabsf(res);
                const uint64_t in = __ballot(a < thr_lo);
                const uint64_t below_hi = __ballot(a < thr_hi);
                cnt += __popcll(in);
                amb[q] = ((below_hi & ~in) >> lane) & 1;
                amb_any |= below_hi & ~in;
            }
            if (amb_any) {  // rare: the matches the f32 value cannot decide, exactly
                const double* E64 = ec64 + ((size_t)p * iters + h0 + h) * 9;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    bool ex = false;
                    if (amb[q]) {
                        const double* b =
                            pts + ((size_t)p * (max_nq + 1) + c0 + q * 64 + lane) * 6;
                        ex = fabs(inlier_residual(E64, b, b + 3)) < thr;
                    }
                    cnt += __popcll(__ballot(ex));
                }
            }
            acc = lane == h ? acc + cnt : acc;
        }
    }
    if (lane < nh) hyps[(size_t)p * iters + h0 + lane].inliers = acc;
}

// ================================================================= consensus ============
// dist_ij = (double) sqrtf(dx*dx + dy*dy + dz*dz) on Vec3f differences (src/eight_point.cpp:138-139)
__device__ __forceinline__ float rdist(float xi, float yi, float zi, float xj, float yj, float zj) {
    const float dx = xi - xj;
    const float dy = yi - yj;
    const float dz = zi - zj;
    return __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
}

// its square (same operations; sqrtf of it is the distance)
__device__ __forceinline__ float rdist2(float xi, float yi, float zi, float xj, float yj, float zj) {
    const float dx = xi - xj;
    const float dy = yi - yj;
    const float dz = zi - zj;
    return dx * dx + dy * dy + dz * dz;
}

// find the bin holding `rank` in hist[0..N-1] (block of 256); returns bin, writes #before
template <int N>
__device__ int find_bin(const uint32_t* hist, long rank, long* before, int* ws, int* res) {
    constexpr int PER = N / 256;
    const int tid = threadIdx.x;
    uint32_t loc = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) loc += hist[tid * PER + k];
    int total;
    const int ex = block_exclusive_scan<256>((int)loc, ws, &total);
    if (tid == 0) {
        res[0] = -1;
        res[1] = 0;
    }
    __syncthreads();
    if ((long)ex <= rank && rank < (long)ex + (long)loc) {
        long c = ex;
        for (int k = 0; k < PER; k++) {
            const long nc = c + hist[tid * PER + k];
            if (rank < nc) {
                res[0] = tid * PER + k;
                res[1] = (int)c;
                break;
            }
            c = nc;
        }
    }
    __syncthreads();
    const int bin = res[0];
    *before = res[1];
    __syncthreads();
    return bin;
}

__device__ double block_sum_f64(double v, double* red) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    const double s = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return s;
}

__device__ long block_sum_i64(long v, double* red) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    long* r = reinterpret_cast<long*>(red);
    __syncthreads();
    if ((tid & 63) == 0) r[tid >> 6] = v;
    __syncthreads();
    const long s = r[0] + r[1] + r[2] + r[3];
    __syncthreads();
    return s;
}

struct RankKeys {
    uint32_t va, vb;  // the keys at ranks lo and hi-1
    long lt_a, le_a;  // #keys < va, #keys <= va
    long lt_b;        // #keys < vb
};
// the f32 keys of ranks ra and rb of row i by a 3-level radix select (three passes)
__device__ RankKeys radix_rank_keys(const float* X, const float* Y, const float* Z, int K,
                                    float xi, float yi, float zi, long ra, long rb,
                                    uint32_t* histA, uint32_t* histB, int* ws, int* res) {
    const int tid = threadIdx.x;
    for (int k = tid; k < 2048; k += 256) histA[k] = 0;
    __syncthreads();
    for (int j = tid; j < K; j += 256) {
        const uint32_t key = __float_as_uint(rdist2(xi, yi, zi, X[j], Y[j], Z[j]));
        atomicAdd(&histA[key >> 21], 1u);
    }
    __syncthreads();
    long ca, cb;
    const int ba = find_bin<2048>(histA, ra, &ca, ws, res);
    const int bb = find_bin<2048>(histA, rb, &cb, ws, res);
    for (int k = tid; k < 2048; k += 256) {
        histA[k] = 0;
        histB[k] = 0;
    }
    __syncthreads();
    for (int j = tid; j < K; j += 256) {
        const uint32_t key = __float_as_uint(rdist2(xi, yi, zi, X[j], Y[j], Z[j]));
        const uint32_t top = key >> 21;
        if (top == (uint32_t)ba) atomicAdd(&histA[(key >> 10) & 2047], 1u);
        if (top == (uint32_t)bb) atomicAdd(&histB[(key >> 10) & 2047], 1u);
    }
    __syncthreads();
    long ca1, cb1;
    const int ba1 = find_bin<2048>(histA, ra - ca, &ca1, ws, res);
    const int bb1 = find_bin<2048>(histB, rb - cb, &cb1, ws, res);
    const uint32_t pa = ((uint32_t)ba << 11) | (uint32_t)ba1;  // key >> 10
    const uint32_t pb = ((uint32_t)bb << 11) | (uint32_t)bb1;
    for (int k = tid; k < 2048; k += 256) {
        histA[k] = 0;
        histB[k] = 0;
    }
    __syncthreads();
    for (int j = tid; j < K; j += 256) {
        const uint32_t key = __float_as_uint(rdist2(xi, yi, zi, X[j], Y[j], Z[j]));
        const uint32_t top = key >> 10;
        if (top == pa) atomicAdd(&histA[key & 1023], 1u);
        if (top == pb) atomicAdd(&histB[key & 1023], 1u);
    }
    __syncthreads();
    long ca2, cb2;
    const int ba2 = find_bin<2048>(histA, ra - ca - ca1, &ca2, ws, res);
    const int bb2 = find_bin<2048>(histB, rb - cb - cb1, &cb2, ws, res);
    RankKeys r;
    r.va = (pa << 10) | (uint32_t)ba2;  // key at rank ra
    r.vb = (pb << 10) | (uint32_t)bb2;  // key at rank rb
    r.lt_a = ca + ca1 + ca2;
    r.le_a = r.lt_a + histA[ba2];
    r.lt_b = cb + cb1 + cb2;
    __syncthreads();  // the histograms' readers are done before the caller reuses them
    return r;
}

// Window sum of row i (ranks [lo, hi)) by a 3-level radix select (11+11+10 bits) on the f32
// bit patterns of the squared distances s (sqrtf is monotone, so the sorted distances are
// sqrtf of the sorted s), then the sum of sqrtf(s) in fp64.  Four passes over the row; the
// general fallback of consensus_rows.  Returns the sum on every thread.
__device__ double radix_window_sum(const float* X, const float* Y, const float* Z, int K,
                                   float xi, float yi, float zi, long lo, long hi,
                                   uint32_t* histA, uint32_t* histB, int* ws, int* res,
                                   double* red, RankKeys* keys_out = nullptr) {
    const int tid = threadIdx.x;
    const RankKeys rk = radix_rank_keys(X, Y, Z, K, xi, yi, zi, lo, hi - 1, histA, histB, ws, res);
    if (keys_out) *keys_out = rk;
    const uint32_t va = rk.va, vb = rk.vb;
    const long le_a = rk.le_a, lt_b = rk.lt_b;
    double acc = 0.0;
    for (int j = tid; j < K; j += 256) {
        const uint32_t key = __float_as_uint(rdist2(xi, yi, zi, X[j], Y[j], Z[j]));
        if (key > va && key < vb) acc += (double)__builtin_sqrtf(__uint_as_float(key));
    }
    const double inner = block_sum_f64(acc, red);
    if (va == vb) return (double)(hi - lo) * (double)__builtin_sqrtf(__uint_as_float(va));
    return inner + (double)(le_a - lo) * (double)__builtin_sqrtf(__uint_as_float(va)) +
           (double)(hi - lt_b) * (double)__builtin_sqrtf(__uint_as_float(vb));
}

// consensus-only entry: AoS R/T lists -> SoA rv, tv, kcount, dscale (one block)
__global__ __launch_bounds__(1024) void consensus_input_kernel(const float* __restrict__ rvec,
                                                               const float* __restrict__ tvec,
                                                               int K, int stride,
                                                               float* __restrict__ rv,
                                                               float* __restrict__ tv,
                                                               int32_t* __restrict__ kcount,
                                                               float* __restrict__ dscale,
                                                               int32_t* __restrict__ flags) {
    __shared__ float red6[6][16];
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    float mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
    bool fin = true;
    for (int k = threadIdx.x; k < K; k += 1024) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float v = rvec[3 * (size_t)k + c];
            rv[c * (size_t)stride + k] = v;
            tv[3 * (size_t)k + c] = tvec[3 * (size_t)k + c];
            fin = fin && __builtin_isfinite(v);
            mn[c] = fminf(mn[c], v);
            mx[c] = fmaxf(mx[c], v);
        }
    }
    // a non-finite rotation vector has no place in the binned distance space (the pipeline's
    // valid hypotheses are finite by construction: |Euler| < valid_abs): ERP_INVALID_ARG
    if (!fin) bad = 1;
    __syncthreads();
    if (bad) {
        if (threadIdx.x == 0) {
            kcount[0] = 0;
            dscale[0] = 1.f;
            flags[0] = 8;
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
        float a = mn[c], b = mx[c];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a = fminf(a, __shfl_xor(a, o, 64));
            b = fmaxf(b, __shfl_xor(b, o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            red6[c][threadIdx.x >> 6] = a;
            red6[3 + c][threadIdx.x >> 6] = b;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double d2 = 0;
        for (int c = 0; c < 3; c++) {
            float a = kInf, b = -kInf;
            for (int w = 0; w < 16; w++) {
                a = fminf(a, red6[c][w]);
                b = fmaxf(b, red6[3 + c][w]);
            }
            const double e = K > 0 ? (double)b - (double)a : 0.0;
            d2 += e * e;
        }
        dscale[0] = (float)(sqrt(d2) * (1.0 + 1e-6));
        kcount[0] = K;
        flags[0] = 0;
    }
}

// ---- pruning by rigorous bounds -------------------------------------------------------
// Every row's K squared distances are binned into NB geometric bins: 16 per binade of s = d^2
// (= 32 per binade of the distance d) over the 36 binades of s below the squared diameter of
// the set, underflow in bin 0.  The binned value is the biased s' = fma(dz, dz, fma(dy, dy,
// fma(dx, dx, E0g))) (E0g: bounds_bias below): with S = dx^2 + dy^2 + dz^2 exactly (the
// reference's dx = fl(x_i - x_j), identical here), s' is within (1 +- 3.0001 u) of S + E0g
// (three correctly rounded operations on non-negative terms, u = 2^-24) and so is the
// reference's s = dx*dx + dy*dy + dz*dz of S, so s' in bin [E_b, E_b+1) puts the reference's
// d = sqrtf(s) in
//   [sqrt(E_b (1 - 2^-20) - E0g) (1 - 2^-20), sqrt(E_b+1 (1 + 2^-20)) (1 + 2^-20)]
// (the 2^-20 factors absorb the 6u of both roundings and sqrtf).  From the exact bin counts
// the trimmed sum over ranks [lo, hi) is bracketed by
//   LB = sum_b n_b(window) * lower_b,  UB = sum_b n_b(window) * upper_b
// (relative width <= 2^-5; valid because the bins are ordered: the order statistics of the
// per-element lower bounds lower_bin(e) <= d_e are <= those of d).  A row whose LB exceeds the
// smallest UB cannot be the argmin; only the survivors get the exact order statistics.  No
// square root in the K^2 loop.
// Block = 16 rows x 256 columns at a time.  The histograms are laid out [bin][row] (one 4-B
// word per (bin, row)), so row r's bins all live in LDS banks r and r + 16; at step t lane l
// takes row (l + t) & 15, so the 32 lanes of an LDS lane group hit each row twice and collide
// at most 2-way (a random scatter of 32 lanes over 32 banks, the [row][bin] layout, costs ~3.5x:
// that was 2/3 of the kernel's LDS time).  Rows t, t+1 share packed f32 instructions
// (v_pk_add_f32 / v_pk_fma_f32 with the column broadcast), the bias keeps every key >= the
// first guard bin, and the LDS byte address is one v_lshl_add_u32 of the key: five VALU
// instructions and one ds_add_u32 per distance.  Four
// blocks (39 KB of histograms each) per CU.  The d-space bin edges are per pair
// (consensus_edges_kernel); the epilogue holds its slice's edges in registers.
constexpr int kBoundRows = 16;       // rows per bounds block
constexpr int kBinShift = 19;         // bin = key >> 19: 16 bins per binade of s = d^2
constexpr int kMantBits = 23 - kBinShift;
constexpr int kBinsPerBinade = 1 << kMantBits;  // (= 32 per binade of the distance)
constexpr int kBinades = 36;          // of s (576 bins: 4 blocks of 39 KB per CU)
constexpr int kNB = kBinsPerBinade * kBinades;  // 576
constexpr int kSubBits = 10;          // 1024 sub-bins per bin (refine / exact pass) ...
constexpr int kNS = 1 << kSubBits;
constexpr int kLowBits = kBinShift - kSubBits;  // ... and below them the exact values
constexpr int kRefineRows = 4;        // rows per refine block
#ifndef ERP_REFINE_MIN
#define ERP_REFINE_MIN 8
#endif
constexpr int kRefineMin = ERP_REFINE_MIN;  // survivors per pair below which refining does not pay

// first s-binade of the bins: the 40 binades ending with the one holding D^2 (D = dscale is
// the bounding-box diagonal rounded up, >= every distance, so every s <= D^2)
__device__ __forceinline__ int bounds_elo(float D) {
    const float D2 = D * D * (1.0f + 0x1p-18f);
    const int t = (int)(__float_as_uint(D2) >> 23) + 1;
    const int e = t - kBinades;
    return e < 1 ? 1 : e;
}
// d-space edge e of the bins (e = 1 .. NB-1: lower edge of bin e = upper edge of bin e-1)
__device__ __forceinline__ float bin_edge_s(int elo, int e) {
    return __uint_as_float((uint32_t)((elo << kMantBits) + e) << kBinShift);
}


// (key << 2) + base as ONE v_lshl_add_u32 (the compiler otherwise rewrites (x >> 19) << 2 as
// (x >> 17) & ~3 and adds: three instructions in the K^2 loop)
__device__ __forceinline__ uint32_t lshl2_add(uint32_t key, uint32_t base) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(r) : "v"(key), "v"(base));
    return r;
}
__device__ __forceinline__ void lds_inc(uint32_t byte_addr) {
    __hip_atomic_fetch_add((lds_u32*)(size_t)byte_addr, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The bias: s' = fma(dz, dz, fma(dy, dy, fma(dx, dx, E0g))) with E0g = the lower edge of the
// bin kGuard bins (4 binades) below bin 0: every key is >= base - kGuard, so the histogram
// address needs no clamp -- keys in the kGuard guard bins below bin 0 (distances below the
// range) are added to bin 0 by the epilogue.  The bias shifts s by E0g = E_0 / 16, i.e. by
// 2^-(4 + binades above the floor) relative: negligible in the bins that hold the window's ranks.
constexpr int kGuard = 64;
__device__ __forceinline__ float bounds_bias(int elo) {
    return bin_edge_s(elo > 4 ? elo - 4 : 1, 0);
}
// d-space bounds of the reference's d for a biased key in bin b (header comment above), in f32:
// s' in [E_b, E_b+1) puts S in [E_b (1 - 3.0001u) - E0g, E_b+1 (1 + 3.0001u) - E0g] and the
// reference's d within (1 +- 2u) of sqrt(S) (E0g <= E_b / 16: no cancellation); E_b (1 -+ 2^-20)
// - E0g, sqrtf and the final product round by <= u each, so the (1 -+ 2^-19) factors keep the
// bounds outward.  Bin 0 also holds every s below E_1 (the guard bins).
__device__ __forceinline__ float bin_lower_d(int elo, int b) {
    if (b == 0) return 0.f;
    const float v = bin_edge_s(elo, b) * (1.0f - 0x1p-20f) - bounds_bias(elo);
    return __builtin_sqrtf(fmaxf(v, 0.f)) * (1.0f - 0x1p-19f);
}
__device__ __forceinline__ float bin_upper_d(int elo, int b) {
    if (b == kNB - 1) return kInf;
    return __builtin_sqrtf(bin_edge_s(elo, b + 1) * (1.0f + 0x1p-20f)) * (1.0f + 0x1p-19f);
}

// lshl_add with shift 6: the [bin][16 rows] histogram address (bin * 64 + row * 4 + base)
__device__ __forceinline__ uint32_t lshl6_add(uint32_t key, uint32_t base) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 6, %2" : "=v"(r) : "v"(key), "v"(base));
    return r;
}

// d-space bounds of the bins of pair p (the same for every block of the pair):
// edges[p][0][b] = lower bound, edges[p][1][b] = upper bound of the reference's d in bin b
__global__ __launch_bounds__(256) void consensus_edges_kernel(const float* __restrict__ dscale,
                                                              float* __restrict__ edges) {
    const int p = blockIdx.x;
    const int elo = bounds_elo(dscale[p]);
    float* ed = edges + (size_t)p * 2 * kNB;
    for (int b = threadIdx.x; b < kNB; b += 256) {
        ed[b] = bin_lower_d(elo, b);
        ed[kNB + b] = bin_upper_d(elo, b);
    }
}

// valid_count + valid_scatter for the lite estimates: a block per (chunk of 1024 iterations,
// pair) adds the valid counts of the 64-iteration waves before its chunk (wsum, <= ~160 values),
// block-scans its chunk and writes the valid rotations in push order (iteration, R1, R2);
// chunk 0 also writes K and the bounding-box scale (the same min / max values valid_count
// reduces, so dscale is bit-identical to the record path's)
__global__ __launch_bounds__(1024) void valid_place_kernel(
    const int32_t* __restrict__ counts, const float* __restrict__ hl, int iters,
    double sample_frac, const int32_t* __restrict__ wsum, int nwaves, float* __restrict__ rv,
    float* __restrict__ tv, int32_t* __restrict__ kcount, float* __restrict__ rv_aos,
    float* __restrict__ dscale, float* __restrict__ edges) {
    __shared__ int ws[16];
    __shared__ int sbase[16];
    __shared__ float ds_s;
    const int p = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int M = counts[p];
    if ((int)(M * sample_frac) < 1) {
        if (c == 0 && tid == 0) kcount[p] = 0;
        return;
    }
    const int32_t* vw = wsum + (size_t)p * nwaves * 8;
    const int upto = c == 0 ? nwaves : min(16 * c, nwaves);  // waves before this chunk (all for 0)
    int part = 0;
    for (int q = tid; q < upto; q += 1024) part += vw[q * 8];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) sbase[tid >> 6] = part;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < 16; w++) base += sbase[w];
    if (c == 0) {
        // the bounding box over every wave's: six block-wide min / max reductions (one serial
        // thread walking ~160 waves' boxes cost ~25 us of a single pair's latency)
        __shared__ float box[6][16];
        float mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
        for (int q = tid; q < nwaves; q += 1024) {
#pragma unroll
            for (int k = 0; k < 3; k++) {
                mn[k] = fminf(mn[k], __int_as_float(vw[q * 8 + 1 + k]));
                mx[k] = fmaxf(mx[k], __int_as_float(vw[q * 8 + 4 + k]));
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                mn[k] = fminf(mn[k], __shfl_xor(mn[k], o, 64));
                mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], o, 64));
            }
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                box[k][tid >> 6] = mn[k];
                box[3 + k][tid >> 6] = mx[k];
            }
        __syncthreads();
        if (tid == 0) {
            kcount[p] = base;
            double d2 = 0;
            for (int k = 0; k < 3; k++) {
                float a = kInf, b = -kInf;
                for (int w = 0; w < 16; w++) {
                    a = fminf(a, box[k][w]);
                    b = fmaxf(b, box[3 + k][w]);
                }
                const double e = base > 0 ? (double)b - (double)a : 0.0;
                d2 += e * e;
            }
            dscale[p] = (float)(sqrt(d2) * (1.0 + 1e-6));
            ds_s = dscale[p];
        }
        if (edges) {  // consensus_edges_kernel's table (one launch fewer)
            __syncthreads();
            const int elo = bounds_elo(ds_s);
            float* ed = edges + (size_t)p * 2 * kNB;
            for (int b = tid; b < kNB; b += 1024) {
                ed[b] = bin_lower_d(elo, b);
                ed[kNB + b] = bin_upper_d(elo, b);
            }
        }
        base = 0;
    }
    const int h = c * 1024 + tid;
    float r[9];
    bool v1 = false, v2 = false;
    if (h < iters) {
        const float* x = hl + (size_t)p * 9 * iters + h;
#pragma unroll
        for (int k = 0; k < 9; k++) r[k] = x[(size_t)k * iters];
        v1 = !__builtin_isnan(r[0]);
        v2 = !__builtin_isnan(r[3]);
    }
    int total;
    int pos = base + block_exclusive_scan<1024>((int)v1 + (int)v2, ws, &total);
    const int stride = 2 * iters;
    float* X = rv + (size_t)p * 3 * stride;
    float* T = tv + (size_t)p * 3 * stride;
    float* A = rv_aos ? rv_aos + (size_t)p * 3 * stride : nullptr;
#pragma unroll
    for (int which = 0; which < 2; which++) {
        if (!(which ? v2 : v1)) continue;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            X[k * stride + pos] = r[3 * which + k];
            T[3 * pos + k] = r[6 + k];
            if (A) A[3 * pos + k] = r[3 * which + k];
        }
        pos++;
    }
}

__device__ __forceinline__ void consensus_bounds_unit(const int32_t* __restrict__ kcount,
                                                               const float* __restrict__ rv,
                                                               const float* __restrict__ dscale,
                                                               const float* __restrict__ edges,
                                                               int stride, double trim_lo,
                                                               double trim_hi,
                                                               double* __restrict__ lb,
                                                               double* __restrict__ ub,
                                                               int32_t* __restrict__ bsel,
                                                               int shard, int nshards, int rstep,
                                                               const int32_t* __restrict__ rlist,
                                                               const int32_t* __restrict__ rcount, int p, int bx) {
    constexpr int R = kBoundRows;
    constexpr int NS = 256 / R;        // epilogue slices per row
    constexpr int per = kNB / NS;      // bins per slice
    static_assert(kNB % NS == 0, "slices");
    __shared__ __align__(16) uint32_t hist[(kGuard + kNB) * R];  // [guard + bin][row]
    // epilogue partials alias the histogram (read into registers first)
    int (*part)[R] = reinterpret_cast<int (*)[R]>(hist);
    float (*partL)[R] = reinterpret_cast<float (*)[R]>(hist + NS * R);
    float (*partU)[R] = reinterpret_cast<float (*)[R]>(hist + 2 * NS * R);
    const int tid = threadIdx.x, lane = wave_lane();
    const int K = kcount[p];
    // rows [ra, rb) of this shard (hypothesis-block sharding of one find over ranks; 0 / 1
    // otherwise), every rstep-th of them (the reference rows of the Lipschitz pre-pruning), or
    // the rows of a per-pair list (the rows that pre-pruning kept); every column
    const int ra = (int)((int64_t)K * shard / nshards);
    const int rb = (int)((int64_t)K * (shard + 1) / nshards);
    const int nloc = rlist ? rcount[p] : (rb > ra ? (rb - ra + rstep - 1) / rstep : 0);
    const int l0 = bx * R;
    if (l0 >= nloc) return;
    const int32_t* RL = rlist ? rlist + (size_t)p * stride : nullptr;
    auto rowof = [&](int l) { return RL ? (int)RL[l] : ra + l * rstep; };
    const float* X = rv + (size_t)p * 3 * stride;
    const float* Y = X + stride;
    const float* Z = Y + stride;
    const int elo = bounds_elo(dscale[p]);
    const int base = elo << kMantBits;
    constexpr int kPairs = R / 2;
    f32x2 xi[kPairs], yi[kPairs], zi[kPairs];
    uint32_t hoff[R];  // LDS byte address of (bin 0 - base, row)
    const uint32_t hist_addr = (uint32_t)(size_t)(lds_u32*)hist;
#pragma unroll
    for (int t = 0; t < R; t++) {
        const int r = (lane + t) & (R - 1);
        const int row = rowof(min(l0 + r, nloc - 1));
        xi[t >> 1][t & 1] = X[row];
        yi[t >> 1][t & 1] = Y[row];
        zi[t >> 1][t & 1] = Z[row];
        hoff[t] = hist_addr + 4u * (uint32_t)r - 64u * (uint32_t)(base - kGuard);
    }
    for (int k = tid; k < (kGuard + kNB) * R / 4; k += 256)
        reinterpret_cast<uint4*>(hist)[k] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const float e0 = bounds_bias(elo);
    const f32x2 bias = {e0, e0};
    // columns in batches of 4 per lane (j0 + 256 c + tid, c < 4: every load coalesced), the next
    // batch loaded while this one is binned (4 x 32 distances of VALU work hide the L2 latency)
    constexpr int CB = 4;
    float cx[CB], cy[CB], cz[CB], nx[CB], ny[CB], nz[CB];
    // (unsigned 32-bit offsets from uniform bases: global_load with an SGPR base, no 64-bit
    // address arithmetic per load)
    const uint32_t kmax4 = 4u * (uint32_t)(K - 1);  // byte offsets (K < 2^30)
    auto ld = [](const float* base, uint32_t off) {
        return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + off);
    };
#pragma unroll
    for (int c = 0; c < CB; c++) {
        const uint32_t o = min(4u * (uint32_t)(c * 256 + tid), kmax4);
        cx[c] = ld(X, o);
        cy[c] = ld(Y, o);
        cz[c] = ld(Z, o);
    }
    for (int j0 = 0; j0 < K; j0 += CB * 256) {
#pragma unroll
        for (int c = 0; c < CB; c++) {
            const uint32_t o = min(4u * (uint32_t)(j0 + CB * 256 + c * 256 + tid), kmax4);
            nx[c] = ld(X, o);
            ny[c] = ld(Y, o);
            nz[c] = ld(Z, o);
        }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            if (j0 + c * 256 + tid < K) {
                const float xj = cx[c], yj = cy[c], zj = cz[c];
#pragma unroll
                for (int t = 0; t < kPairs; t++) {
                    const f32x2 dx = xi[t] - xj, dy = yi[t] - yj, dz = zi[t] - zj;
                    f32x2 s = __builtin_elementwise_fma(dx, dx, bias);
                    s = __builtin_elementwise_fma(dy, dy, s);
                    s = __builtin_elementwise_fma(dz, dz, s);
                    lds_inc(lshl6_add(__float_as_uint(s[0]) >> kBinShift, hoff[2 * t]));
                    lds_inc(lshl6_add(__float_as_uint(s[1]) >> kBinShift, hoff[2 * t + 1]));
                }
            }
        }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            cx[c] = nx[c];
            cy[c] = ny[c];
            cz[c] = nz[c];
        }
    }
    __syncthreads();
    // per row: NS slices of `per` consecutive bins, thread = slice * R + row; the slice's bin
    // counts and edges in registers.  Window-clipped counts w_b = clip(cum_b + n_b) -
    // clip(cum_b) (clip to [lo, hi]); L, U accumulate w_b * edge in f32 (<= kNB non-negative
    // terms: relative error < kNB * 2^-24, covered by the 2e-4 margins below).
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    const int r = tid & (R - 1), sl = tid / R;
    const float* ed = edges + (size_t)p * 2 * kNB + sl * per;
    float el[per], eu[per];
    int n[per];
    int c = 0;
#pragma unroll
    for (int q = 0; q < per; q++) {
        el[q] = ed[q];
        eu[q] = ed[kNB + q];
        n[q] = (int)hist[(kGuard + sl * per + q) * R + r];
    }
    if (sl == 0)  // distances below the range (guard bins) count as bin 0
        for (int g = 0; g < kGuard; g++) n[0] += (int)hist[g * R + r];
#pragma unroll
    for (int q = 0; q < per; q++) c += n[q];
    __syncthreads();  // every count is in registers: the partials may overwrite the histogram
    part[sl][r] = c;
    __syncthreads();
    int cum = 0;
    for (int q = 0; q < sl; q++) cum += part[q][r];
    const bool rvalid = l0 + r < nloc;
    const int row = rvalid ? rowof(l0 + r) : 0;
    float L = 0.f, U = 0.f;
    int sel_a = -1, sel_b = -1;  // bins holding ranks lo and hi-1 (for the exact pass)
    if (cum < hi && cum + c > lo) {
        int c0 = min(max(cum, lo), hi);
#pragma unroll
        for (int q = 0; q < per; q++) {
            const int nc = cum + n[q];
            const int c1 = min(max(nc, lo), hi);
            const float w = (float)(c1 - c0);
            L = __builtin_fmaf(w, el[q], L);
            // (0 * inf: the last bin's upper edge is +inf, and until r04 every row whose rank
            // window reached the top slice -- a two-cluster set's rank hi-1 in bin ~571 --
            // got UB = NaN, so its pair's U was NaN and the pre-pruning never ran)
            U = w > 0.f ? __builtin_fmaf(w, eu[q], U) : U;
            sel_a = (cum <= lo && lo < nc) ? sl * per + q : sel_a;
            sel_b = (cum <= hi - 1 && hi - 1 < nc) ? sl * per + q : sel_b;
            cum = nc;
            c0 = c1;
        }
    }
    if (rvalid) {
        if (sel_a >= 0) bsel[((size_t)p * stride + row) * 2] = sel_a;
        if (sel_b >= 0) bsel[((size_t)p * stride + row) * 2 + 1] = sel_b;
    }
    partL[sl][r] = L;
    partU[sl][r] = U;
    __syncthreads();
    if (sl == 0 && rvalid) {
        for (int q = 1; q < NS; q++) {
            L += partL[q][r];
            U += partU[q][r];
        }
        const double w = (double)(hi - lo);
        // margins: the f32 accumulation above and the reference's own rounding of its sorted
        // sequential sum
        lb[(size_t)p * stride + row] = hi > lo ? ((double)L / w) * (1.0 - 2e-4) : 0.0;
        ub[(size_t)p * stride + row] = hi > lo ? ((double)U / w) * (1.0 + 2e-4) : 0.0;
    }
}

// one unit (R rows) per block: every row of a shard, or every rstep-th row
__global__ __launch_bounds__(256) void consensus_bounds_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ dscale, const float* __restrict__ edges, int stride, double trim_lo,
    double trim_hi, double* __restrict__ lb, double* __restrict__ ub, int32_t* __restrict__ bsel,
    int shard, int nshards, int rstep) {
    consensus_bounds_unit(kcount, rv, dscale, edges, stride, trim_lo, trim_hi, lb, ub, bsel, shard,
                          nshards, rstep, nullptr, nullptr, blockIdx.y, blockIdx.x);
}

// Lipschitz pre-pruning (before the full bounds pass).  The trimmed mean T(x) of the distances
// from x to the set is 1-Lipschitz in x (every distance is, so are the order statistics and
// their mean): T(i) >= T(c) - d(i, c).  The bounds kernel first runs on the reference rows
// c = 0, kLipStep, 2 kLipStep, ... (1/48 of the rows); with U = their smallest UB, a row i with
// d(i, c) < LB(c) - U for some reference c has T(i) > U >= the final min UB, so it cannot be the
// argmin and skips the K-column histogram pass.  The test runs in squared f32 distances against
// per-reference thresholds thr_c = (LB_c (1 - M) - U (1 + M))^2 (1 - M): the margins M (kLipM,
// 1e-6) cover the f32 rounding of s (<= 5u), the reference's own f32 distances and fp64 sum
// and the rounding of thr, so a pruned row's LB = U (1 + M / 2) is rigorous and strictly above
// every UB that select compares against.  Pruned rows get [LB, +inf) and no
// boundary bins (select drops them); the others are appended (any order) to the per-pair list
// that the second bounds pass reads.  Synthetic configs[1] pairs (one cluster of ~1e4 valid
// rotations): ~80 % of the rows are pruned for ~1/16 + ~1/20 of the full pass's distances.
// every 32nd row was a reference row from r04 to r06 (16 until r04: with the 1e-6 margins of kLipM fewer
// references prune as much; same-box A/Bs per 768-pair step, profiles/r04c_ab_lip_step.txt:
// consensus 6.60 / 6.62 ms at 16, 6.95 / 7.09 at 12, 6.00 / 6.04 at 24, 5.96 / 5.91 at 32,
// 5.83 / 5.82 at 48, 6.08 / 6.07 at 64; pairs/s +3-4 % at 24-48).  Every 48th since r06aj:
// re-measured at the round-6 tree (second stage, convexity pruning, refine hints), 48 took the
// consensus 5.51-5.58 -> 5.35-5.45 ms per step and +1.5-2 % pairs/s on two boxes, worst case
// unchanged; 40 and 64 were no better than 32 (profiles/r06aj_ab_lip_step.txt)
#ifndef ERP_LIP_STEP
#define ERP_LIP_STEP 48
#endif
constexpr int kLipStep = ERP_LIP_STEP;
static_assert(kLipStep % 4 == 0, "a reference row is never a second-stage reference (is_ref2)");
// every 8th survivor is refined first (refine pass; 16th until r06am: the worst-case batch
// 17.1 -> 18.2k pairs/s on two boxes, the headline unchanged, profiles/r06am_ab_ref_step.txt)
#ifndef ERP_REF_STEP
#define ERP_REF_STEP 8
#endif
constexpr int kRefStep = ERP_REF_STEP;
constexpr int kLipMinK = 1024;  // smaller sets: no pre-pruning (every non-reference row listed)
// the convexity-augmented pruning's central references: UB_c <= U kLipGFac (consensus_grad_select;
// r04 A/B, profiles/r04c_ab_consensus_knobs.txt: 1.03 cost +0.2 ms of consensus per step)
#ifndef ERP_LIP_GFAC
#define ERP_LIP_GFAC 1.1f
#endif
constexpr float kLipGFac = ERP_LIP_GFAC;
constexpr int kGradBlocks = 2048;  // consensus_grad_kernel's grid (grid-stride over the references)
#ifndef ERP_LIP2_STEP
#define ERP_LIP2_STEP 4
#endif
constexpr int kLip2Step = ERP_LIP2_STEP;  // 1 in 4 L1 rows is a second-stage reference
static_assert((kLip2Step & (kLip2Step - 1)) == 0, "power of two (is_ref2)");

// The references of a pruning pass, staged ONCE per pair (consensus_lip_refs_kernel) into
// lref[p][0 .. lcnt[p]) as (x, y, z, squared pruning radius), with U = their smallest UB in
// lU[p] (+inf: no pruning for the pair).  Every pruning block then reads them with coalesced
// loads: when each block gathered its references' LB and coordinates itself (dependent
// gathers, ~20 per block of 512 rows) the kernels spent ~80 % of their wave cycles waiting
// (SQ_WAIT_ANY, profiles/r03_sq_lipschitz.txt).
constexpr int kLipChunk2 = 512;  // references per LDS chunk
// The Lipschitz tests' relative margin M (round 4: 1e-6; 1e-5 until r04, ERP_LIP_MARGIN for A/B).
// The reference's T is computed from f32 distances: d_ref = d (1 +- 2.5u) per element (dx, the
// square, two adds), so its order statistics and T_ref = T (1 +- 2.5u) (+ the fp64 sum's
// w 2^-53), and T_ref(i) >= LB_c (1 - 5u) - d(i, c).  The test s_f32(i, c) < thr_c with
// thr_c = (LB_c (1 - M) - U (1 + M))^2 (1 - M) (s_f32 = d^2 (1 +- 4u), thr rounded to f32: u)
// gives d(i, c) < LB_c (1 - M) - U (1 + M), so T_ref(i) > LB_c (M - 5u) + U (1 + M) >= U (1 + M)
// for M >= 6u = 3.6e-7: a pruned row's LB = U (1 + M / 2) is rigorous and strictly above every
// UB that select compares against.  The margin matters where T is flat: on a two-cluster set
// (every T within ~6e-5 of min T ~ 1.3) M = 1e-5 alone removes ~2.6e-5 of every pruning radius.
#ifndef ERP_LIP_MARGIN
#define ERP_LIP_MARGIN 1e-6
#endif
constexpr double kLipM = ERP_LIP_MARGIN;
constexpr double kLipPrunedLB = 1.0 + 0.5 * kLipM;
int lipref_cap(int stride) { return stride / kLip2Step + 64; }  // >= refs of any mode

// one block per pair.  Modes: stage 1 (slist == nullptr, zb == nullptr): rows ra + c lstep of
// the shard (pairs with K >= kLipMinK); list mode (slist, zb == nullptr): survivor-list
// positions c lstep (pairs with > kRefineMin survivors, before the refine pass); stage 2 (slist =
// L1, zb): L1 positions c lstep of the pairs with a second stage, U also <= the stage-1 U
// already in lU[p].  Only references with LB_c > U (1 + M) can prune; their radius is
// thr_c = (LB_c (1 - M) - U (1 + M))^2 (1 - M) in squared f32 distance (kLipM has the margins).
__global__ __launch_bounds__(256) void consensus_lip_refs_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv, int stride, double trim_lo,
    double trim_hi, const double* __restrict__ lb, const double* __restrict__ ub,
    const int32_t* __restrict__ slist, const int32_t* __restrict__ scount, int lstep, int shard,
    int nshards, const int32_t* __restrict__ zb, float4* __restrict__ lref,
    double* __restrict__ lU, int32_t* __restrict__ lcnt, int cap,
    const int32_t* __restrict__ gate = nullptr, int32_t* __restrict__ z0 = nullptr,
    int32_t* __restrict__ z1 = nullptr) {
    __shared__ double red[4];
    __shared__ int nlive;
    const int p = blockIdx.x, tid = threadIdx.x, lane = wave_lane();
    // z0 / z1: per-pair list counters the next kernel appends to, reset here (no memset launch)
    if (tid == 0) {
        if (z0) z0[p] = 0;
        if (z1) z1[p] = 0;
    }
    if (gate && gate[p] <= 0) return;  // (the flat-pair re-run: other pairs keep their refs)
    const int K = kcount[p];
    const int ra = slist ? 0 : (int)((int64_t)K * shard / nshards);
    const int n = slist ? scount[p] : (int)((int64_t)K * (shard + 1) / nshards) - ra;
    const int32_t* SL = slist ? slist + (size_t)p * stride : nullptr;
    auto rowpos = [&](int k) { return SL ? (int)SL[k] : ra + k; };
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    const int nref = n > 0 ? (n + lstep - 1) / lstep : 0;
    bool on = hi > lo && (zb ? zb[p] >= 0 : (SL ? n > kRefineMin : K >= kLipMinK));
    const double Uprev = zb ? lU[p] : __builtin_huge_val();
    double U = __builtin_huge_val();
    if (on) {  // (uniform)
        for (int c = tid; c < nref; c += 256) U = fmin(U, ub[(size_t)p * stride + rowpos(c * lstep)]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) U = fmin(U, __shfl_xor(U, o, 64));
        if (lane == 0) red[tid >> 6] = U;
        if (tid == 0) nlive = 0;
        __syncthreads();
        U = fmin(fmin(fmin(red[0], red[1]), fmin(red[2], red[3])), Uprev);
        on = U > 0.0 && U < __builtin_huge_val();
    }
    if (!on) {
        if (tid == 0) {
            lU[p] = __builtin_huge_val();
            lcnt[p] = 0;
        }
        return;
    }
    const double Um = U * (1.0 + kLipM);
    const float* X = rv + (size_t)p * 3 * stride;
    float4* R = lref + (size_t)p * cap;
    for (int c = tid; c < nref; c += 256) {
        const int row = rowpos(c * lstep);
        const double a = lb[(size_t)p * stride + row] * (1.0 - kLipM) - Um;
        if (a > 0.0) {
            const float thr = (float)(a * a * (1.0 - kLipM));
            R[atomicAdd(&nlive, 1)] = make_float4(X[row], X[stride + row], X[2 * stride + row], thr);
        }
    }
    __syncthreads();
    if (tid == 0) {
        lU[p] = U;
        lcnt[p] = nlive;
    }
}

// The candidate rows of a pruning block (up to 512; x, y, z and the row index as bits in act)
// against the pair's staged references R[0 .. m), kLipChunk2 at a time through LDS.  After
// every kLipBatch references the rows still unpruned are compacted (in place, densely; thread t
// takes slots 2t, 2t + 1 as one packed pair), so the live rows fill the first ceil(na / 128)
// waves and the others skip: on a configs[1] pair ~84 % of the rows are pruned, most by one
// of the first ~100 references in any order (a numpy model of the fixture pair: ~2.5x fewer
// tests than every row against every reference).  prune(row) is called once per pruned row;
// the survivors are left in act[0 .. return value).  Counters cnt[t & 3] of batch t are reset
// two batches ahead, between barriers.
#ifndef ERP_LIP_BATCH
#define ERP_LIP_BATCH 64
#endif
constexpr int kLipBatch = ERP_LIP_BATCH;
struct LipShared {
    float4 act[512];
    float4 refs[kLipChunk2];
    double red[4];
    int cnt[4];
};
#ifndef ERP_LIP_VERIFY
#define ERP_LIP_VERIFY 0
#endif
#if ERP_LIP_VERIFY
// debug (ERP_LIP_VERIFY=1 builds): lip_prune_rows re-checks its LDS operands against their
// global sources after every batch's tests -- [0] staged references that differ, [1] candidate
// rows whose coordinates differ from the rotation vectors, [8..] the first mismatches
__device__ uint32_t g_lip_dbg[64];
__device__ void lip_dbg_note(int kind, uint32_t a, uint32_t b, uint32_t c) {
    atomicAdd(&g_lip_dbg[kind], 1u);
    const uint32_t k = atomicAdd(&g_lip_dbg[2], 1u);
    if (k < 14) {
        g_lip_dbg[8 + 4 * k] = (uint32_t)kind;
        g_lip_dbg[9 + 4 * k] = a;
        g_lip_dbg[10 + 4 * k] = b;
        g_lip_dbg[11 + 4 * k] = c;
    }
}
#endif
template <class Prune>
__device__ int lip_prune_rows(LipShared& sh, int na, const float4* __restrict__ R, int m,
                              Prune prune, const float* __restrict__ Xv = nullptr, int xstride = 0) {
    const int tid = threadIdx.x, lane = wave_lane();
    int t = 0;
    for (int c0 = 0; c0 < m && na > 0; c0 += kLipChunk2) {
        const int nc = min(kLipChunk2, m - c0);
        __syncthreads();  // the previous chunk's readers are done
        // (padded to whole batches with references that prune nothing: radius^2 = -1)
        const int ncp = (nc + kLipBatch - 1) / kLipBatch * kLipBatch;
        for (int c = tid; c < ncp; c += 256)
            sh.refs[c] = c < nc ? R[c0 + c] : make_float4(0.f, 0.f, 0.f, -1.f);
        __syncthreads();
        for (int q0 = 0; q0 < nc && na > 0; q0 += kLipBatch, t++) {
            const bool v0 = 2 * tid < na, v1 = 2 * tid + 1 < na;
            const float4 a0 = sh.act[v0 ? 2 * tid : 0];
            const float4 a1 = sh.act[v1 ? 2 * tid + 1 : 0];
            const f32x2 xi = {a0.x, a1.x}, yi = {a0.y, a1.y}, zi = {a0.z, a1.z};
            uint32_t neg0 = 0u, neg1 = 0u;
            if (v0) {  // (a wave whose slots are all empty skips the tests)
                // eight references' LDS reads ahead of their tests: one LDS latency per eight
                // (one per reference measured the kernel latency-bound, SQ_WAIT_ANY 73 %)
                for (int q = q0; q < q0 + kLipBatch; q += 8) {
                    float4 r[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) r[u] = sh.refs[q + u];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const f32x2 dx = xi - r[u].x, dy = yi - r[u].y, dz = zi - r[u].z;
                        f32x2 s2 = dx * dx;
                        s2 = __builtin_elementwise_fma(dy, dy, s2);
                        s2 = __builtin_elementwise_fma(dz, dz, s2);
                        const f32x2 d = s2 - r[u].w;
                        neg0 |= __float_as_uint(d[0]);
                        neg1 |= __float_as_uint(d[1]);
                    }
                }
            }
            const bool p0 = v0 && (neg0 >> 31), p1 = v1 && (neg1 >> 31);
#if ERP_LIP_VERIFY
            if (tid < kLipBatch) {
                const int c = q0 + tid;
                const float4 g = c < nc ? R[c0 + c] : make_float4(0.f, 0.f, 0.f, -1.f);
                const float4 l = sh.refs[c];
                if (__float_as_uint(g.x) != __float_as_uint(l.x) || __float_as_uint(g.y) != __float_as_uint(l.y) ||
                    __float_as_uint(g.z) != __float_as_uint(l.z) || __float_as_uint(g.w) != __float_as_uint(l.w))
                    lip_dbg_note(0, (uint32_t)c, __float_as_uint(l.w), __float_as_uint(g.w));
            }
            if (Xv) {
                const float4 aa[2] = {a0, a1};
                const bool vv[2] = {v0, v1};
                for (int u = 0; u < 2; u++) {
                    if (!vv[u]) continue;
                    const int row = __float_as_int(aa[u].w);
                    if (row < 0 || row >= xstride || __float_as_uint(Xv[row]) != __float_as_uint(aa[u].x) ||
                        __float_as_uint(Xv[xstride + row]) != __float_as_uint(aa[u].y) ||
                        __float_as_uint(Xv[2 * xstride + row]) != __float_as_uint(aa[u].z))
                        lip_dbg_note(1, (uint32_t)row, __float_as_uint(aa[u].x), (uint32_t)(2 * tid + u));
                }
            }
#endif
            if (p0) prune(__float_as_int(a0.w));
            if (p1) prune(__float_as_int(a1.w));
            const bool k0 = v0 && !p0, k1 = v1 && !p1;
            const uint64_t b0 = __builtin_amdgcn_ballot_w64(k0), b1 = __builtin_amdgcn_ballot_w64(k1);
            int base = 0;
            if (lane == 0 && (b0 | b1))
                base = atomicAdd(&sh.cnt[t & 3], __builtin_popcountll(b0) + __builtin_popcountll(b1));
            base = __shfl(base, 0, 64);
            __syncthreads();  // every slot of this batch is read: compact in place
            const uint64_t below = (1ull << lane) - 1ull;
            if (k0) sh.act[base + __builtin_popcountll(b0 & below)] = a0;
            if (k1) sh.act[base + __builtin_popcountll(b0) + __builtin_popcountll(b1 & below)] = a1;
            __syncthreads();
            na = sh.cnt[t & 3];
            if (tid == 0) sh.cnt[(t + 2) & 3] = 0;
        }
    }
    return na;
}

// the rows act[0 .. na) against the gradient references GR[0 .. m) (two float4 each, staged
// through LDS 256 at a time); same compaction as lip_prune_rows
template <class Prune>
__device__ int lip_prune_grad(LipShared& sh, int na, const float4* __restrict__ GR, int m,
                              double U, Prune prune) {
    constexpr int kChunk = kLipChunk2 / 2, kBatch = 32;
    const int tid = threadIdx.x, lane = wave_lane();
    const float Um = (float)(U * (1.0 + 1.1e-5));  // >= U (1 + 1e-5) after rounding
    // the batch counters restart at zero (lip_prune_rows leaves its last two batches' counts)
    __syncthreads();
    if (tid < 4) sh.cnt[tid] = 0;
    int t = 0;
    for (int c0 = 0; c0 < m && na > 0; c0 += kChunk) {
        const int nc = min(kChunk, m - c0);
        __syncthreads();
        const int ncp = (nc + kBatch - 1) / kBatch * kBatch;  // padding prunes nothing
        for (int c = tid; c < 2 * ncp; c += 256)
            sh.refs[c] = c < 2 * nc ? GR[2 * c0 + c]
                                    : make_float4(0.f, 0.f, 0.f, (c & 1) ? 0.f : -kInf);
        __syncthreads();
        for (int q0 = 0; q0 < nc && na > 0; q0 += kBatch, t++) {
            const bool v0 = 2 * tid < na, v1 = 2 * tid + 1 < na;
            const float4 a0 = sh.act[v0 ? 2 * tid : 0];
            const float4 a1 = sh.act[v1 ? 2 * tid + 1 : 0];
            bool p0 = false, p1 = false;
            if (v0) {
                for (int q = q0; q < q0 + kBatch; q++) {
                    const float4 A = sh.refs[2 * q], B = sh.refs[2 * q + 1];
                    const float dx0 = a0.x - A.x, dy0 = a0.y - A.y, dz0 = a0.z - A.z;
                    const float dx1 = a1.x - A.x, dy1 = a1.y - A.y, dz1 = a1.z - A.z;
                    const float n0 = __builtin_amdgcn_sqrtf(
                        __builtin_fmaf(dz0, dz0, __builtin_fmaf(dy0, dy0, dx0 * dx0)));
                    const float n1 = __builtin_amdgcn_sqrtf(
                        __builtin_fmaf(dz1, dz1, __builtin_fmaf(dy1, dy1, dx1 * dx1)));
                    const float g0 = __builtin_fmaf(B.z, dz0, __builtin_fmaf(B.y, dy0, B.x * dx0));
                    const float g1 = __builtin_fmaf(B.z, dz1, __builtin_fmaf(B.y, dy1, B.x * dx1));
                    p0 |= __builtin_fmaf(-B.w, n0, A.w + g0) > Um;
                    p1 |= __builtin_fmaf(-B.w, n1, A.w + g1) > Um;
                }
            }
            p0 = v0 && p0;
            p1 = v1 && p1;
            if (p0) prune(__float_as_int(a0.w));
            if (p1) prune(__float_as_int(a1.w));
            const bool k0 = v0 && !p0, k1 = v1 && !p1;
            const uint64_t b0 = __builtin_amdgcn_ballot_w64(k0), b1 = __builtin_amdgcn_ballot_w64(k1);
            int base = 0;
            if (lane == 0 && (b0 | b1))
                base = atomicAdd(&sh.cnt[t & 3], __builtin_popcountll(b0) + __builtin_popcountll(b1));
            base = __shfl(base, 0, 64);
            __syncthreads();
            const uint64_t below = (1ull << lane) - 1ull;
            if (k0) sh.act[base + __builtin_popcountll(b0 & below)] = a0;
            if (k1) sh.act[base + __builtin_popcountll(b0) + __builtin_popcountll(b1 & below)] = a1;
            __syncthreads();
            na = sh.cnt[t & 3];
            if (tid == 0) sh.cnt[(t + 2) & 3] = 0;
        }
    }
    return na;
}

// append act[0 .. na) (the rows left) to a per-pair list
// (and, when list2 is given, the rows that are second-stage references, is_ref2, to list2 too)
__device__ __forceinline__ bool is_ref2(int row) { return (row & (kLip2Step - 1)) == 1; }
__device__ void lip_append(const LipShared& sh, int na, int32_t* __restrict__ list,
                           int32_t* __restrict__ count, int32_t* __restrict__ list2 = nullptr,
                           int32_t* __restrict__ count2 = nullptr) {
    const int tid = threadIdx.x, lane = wave_lane();
    const uint64_t below = (1ull << lane) - 1ull;
    for (int a = tid; a - tid < na; a += 256) {
        const bool keep = a < na;
        const int i = keep ? __float_as_int(sh.act[a].w) : 0;
        const uint64_t bal = __builtin_amdgcn_ballot_w64(keep);
        int base = 0;
        if (lane == 0 && bal) base = atomicAdd(count, __builtin_popcountll(bal));
        base = __shfl(base, 0, 64);
        if (keep) list[base + __builtin_popcountll(bal & below)] = i;
        if (list2) {
            const bool k2 = keep && is_ref2(i);
            const uint64_t b2 = __builtin_amdgcn_ballot_w64(k2);
            int base2 = 0;
            if (lane == 0 && b2) base2 = atomicAdd(count2, __builtin_popcountll(b2));
            base2 = __shfl(base2, 0, 64);
            if (k2) list2[base2 + __builtin_popcountll(b2 & below)] = i;
        }
    }
}

// Lipschitz pre-pruning (before the full bounds pass).  The trimmed mean T(x) of the distances
// from x to the set is 1-Lipschitz in x (every distance is, so are the order statistics and
// their mean): T(i) >= T(c) - d(i, c).  The bounds kernel first runs on the reference rows
// c = 0, kLipStep, 2 kLipStep, ... (1/48 of the rows); with U = their smallest UB, a row i with
// d(i, c) < LB(c) - U for some reference c has T(i) > U >= the final min UB, so it cannot be the
// argmin and skips the K-column histogram pass.  The test runs in squared f32 distances against
// per-reference thresholds thr_c = (LB_c (1 - M) - U (1 + M))^2 (1 - M): the margins M (kLipM,
// 1e-6) cover the f32 rounding of s (<= 5u), the reference's own f32 distances and fp64 sum
// and the rounding of thr, so a pruned row's LB = U (1 + M / 2) is rigorous and strictly above
// every UB that select compares against.  Pruned rows get [LB, +inf) and no
// boundary bins (select drops them); the others are appended (any order) to the per-pair list
// that the second bounds pass reads.  Synthetic configs[1] pairs (one cluster of ~1e4 valid
// rotations): ~84 % of the rows are pruned.
//   slist == nullptr: the rows [ra, rb) of row shard `shard` of `nshards` (all K rows when
// unsharded), against that shard's own reference rows ra, ra + 16, ... (configs[4]'s
// row-sharded consensus: U is then the shard's smallest reference UB, still >= the global
// minimum of T, so every pruning stays rigorous); else the per-pair survivor list
// slist[p][0 .. scount[p]) after the first select (before the refine pass, whose reference
// survivors, every kRefStep-th, are already refined).  The references: consensus_lip_refs_kernel.
__global__ __launch_bounds__(256) void consensus_lipschitz_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv, int stride,
    double* __restrict__ lb, double* __restrict__ ub, const int32_t* __restrict__ slist,
    const int32_t* __restrict__ scount, int32_t* __restrict__ rlist, int olstride,
    int32_t* __restrict__ rcount, int shard, int nshards, int lstep,
    const float4* __restrict__ lref, const double* __restrict__ lU,
    const int32_t* __restrict__ lcnt, int cap, int32_t* __restrict__ r2list,
    int32_t* __restrict__ r2cnt, const float4* __restrict__ gref, const int32_t* __restrict__ gcnt,
    int gcap, const int32_t* __restrict__ gate = nullptr) {
    __shared__ LipShared sh;
    const int p = blockIdx.y, tid = threadIdx.x, lane = wave_lane();
    if (gate && gate[p] <= 0) return;  // (the flat-pair re-run: other pairs keep their lists)
    const int K = kcount[p];
    const int ra = slist ? 0 : (int)((int64_t)K * shard / nshards);
    const int n = slist ? scount[p] : (int)((int64_t)K * (shard + 1) / nshards) - ra;
    const int i0 = blockIdx.x * 512;  // positions i0 .. i0 + 511
    if (i0 >= n) return;
    if (slist && n <= kRefineMin) return;  // few survivors: no refine pass, nothing to list
    const int32_t* SL = slist ? slist + (size_t)p * stride : nullptr;
    const float* X = rv + (size_t)p * 3 * stride;
    double* LBp = lb + (size_t)p * stride;
    double* UBp = ub + (size_t)p * stride;
    const double U = lU[p];
    const int m = lcnt[p];
    const bool prune_on = U < __builtin_huge_val();
    // the block's candidate rows, compacted into act; in list mode a survivor whose own
    // (first-pass) LB already exceeds the refined U cannot be the argmin either (T_i >= LB_i >
    // U >= min T: not even a tie): pruned at once, no refine needed
    if (tid < 4) sh.cnt[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int k = i0 + 256 * h + tid;
        bool act = k < n && (k % lstep) != 0;
        const int i = act ? (SL ? (int)SL[k] : ra + k) : 0;
        if (act && SL && prune_on && LBp[i] > U * (1.0 + kLipM)) {
            LBp[i] = fmax(LBp[i], U * kLipPrunedLB);
            UBp[i] = __builtin_huge_val();
            act = false;
        }
        const uint64_t bal = __builtin_amdgcn_ballot_w64(act);
        int base = 0;
        if (lane == 0 && bal) base = atomicAdd(&sh.cnt[3], __builtin_popcountll(bal));
        base = __shfl(base, 0, 64);
        if (act)
            sh.act[base + __builtin_popcountll(bal & ((1ull << lane) - 1ull))] =
                make_float4(X[i], X[stride + i], X[2 * stride + i], __int_as_float(i));
    }
    __syncthreads();
    int na = sh.cnt[3];
    __syncthreads();
    if (tid == 3) sh.cnt[3] = 0;  // (batch counters 0 .. 3 start at zero)
    if (prune_on && m > 0) {
        auto prune = [&](int i) {
            LBp[i] = SL ? fmax(LBp[i], U * kLipPrunedLB) : U * kLipPrunedLB;
            UBp[i] = __builtin_huge_val();
        };
        na = lip_prune_rows(sh, na, lref + (size_t)p * cap, m, prune, X, stride);
    }
    if (prune_on && gref && gcnt[p] > 0) {  // the rows left against the central references' G
        auto prune = [&](int i) {
            LBp[i] = U * (1.0 + 5e-6);
            UBp[i] = __builtin_huge_val();
        };
        na = lip_prune_grad(sh, na, gref + (size_t)p * gcap * 2, gcnt[p], U, prune);
    }
    lip_append(sh, na, rlist + (size_t)p * olstride, &rcount[p],
               r2list ? r2list + (size_t)p * stride : nullptr, r2list ? &r2cnt[p] : nullptr);
}

// f(x_j, y_j, z_j) for the columns j = tid, tid + 256, ... of a block of 256: batches of
// kRowsCB columns per thread with the next batch loaded before this one is processed
constexpr int kRowsCB = 8;
template <class F>
__device__ __forceinline__ void for_columns(const float* __restrict__ X, const float* __restrict__ Y,
                                            const float* __restrict__ Z, int K, F f) {
    const int tid = threadIdx.x;
    float cx[kRowsCB], cy[kRowsCB], cz[kRowsCB], nx[kRowsCB], ny[kRowsCB], nz[kRowsCB];
    const int kmax = K - 1;
#pragma unroll
    for (int c = 0; c < kRowsCB; c++) {
        const int j = min(c * 256 + tid, kmax);
        cx[c] = X[j];
        cy[c] = Y[j];
        cz[c] = Z[j];
    }
    for (int j0 = 0; j0 < K; j0 += kRowsCB * 256) {
#pragma unroll
        for (int c = 0; c < kRowsCB; c++) {
            const int j = min(j0 + kRowsCB * 256 + c * 256 + tid, kmax);
            nx[c] = X[j];
            ny[c] = Y[j];
            nz[c] = Z[j];
        }
#pragma unroll
        for (int c = 0; c < kRowsCB; c++)
            if (j0 + c * 256 + tid < K) f(cx[c], cy[c], cz[c]);
#pragma unroll
        for (int c = 0; c < kRowsCB; c++) {
            cx[c] = nx[c];
            cy[c] = ny[c];
            cz[c] = nz[c];
        }
    }
}

// Rank-key windows of the refine pass (round 4).  Default: the boundary bins b_a, b_b of the
// bounds pass, 1024 sub-bins of 2^kLowBits keys each.  With a hint (consensus_hint_kernel: the
// exact keys va, vb at ranks lo and hi-1 of one survivor h of the pair), the order statistics'
// 1-Lipschitz property puts row i's rank-lo distance within d(i, h) of sqrtf(va) (and likewise
// for hi-1), so the 1024 sub-bins go on that key interval instead, 2^w keys each with the
// smallest w that covers it -- kept only when finer than the bin's own sub-bins.  A two-cluster
// set (R1 and R2 valid in every iteration) is why: all of the far cluster's distances fall in
// ONE bin, so the window's ~6 000 elements there were bracketed at 2^9 keys each (a relative
// bound width ~2e-5, ~1 700 survivors per pair into the exact pass); on the interval they are
// bracketed at 2^2-2^3 keys.  The window placement is only a heuristic: a rank that falls
// outside its window fails the `ok` test below and the row keeps its old bounds.
constexpr int kHintCands = 4;
constexpr int kHintManyRows = 256;
struct HintCand {
    double T;
    int32_t row;  // -1: none
    uint32_t va, vb, pad;
};
struct RefineWin {
    uint32_t a0, a1, b0, b1;  // key windows [a0, a1) (rank lo), [b0, b1) (rank hi-1)
    int wa, wb;               // sub-bin k of a window covers keys [x0 + (k << w), + 2^w)
};
__device__ __forceinline__ bool refine_interval(float dc, float delta, uint32_t* k0, int* w) {
    const float hw = delta * 1.0001f + dc * 0x1p-17f + 0x1p-100f;
    const float dl = fmaxf(dc - hw, 0.f), dh = dc + hw;
    const uint32_t klo = __float_as_uint(dl * dl * (1.f - 0x1p-20f));
    const uint32_t khi = __float_as_uint(dh * dh * (1.f + 0x1p-20f)) + 1u;
    const uint32_t span = khi - klo;
    const int ww = span <= (uint32_t)kNS ? 0 : 32 - __builtin_clz(span - 1u) - kSubBits;
    *k0 = klo;
    *w = ww;
    return ww < kLowBits && khi < 0x7f800000u;
}
// the hint of pair p (the candidate with the smallest exact mean; consensus_hint_kernel):
// h.w = 0 when there is none, else (x_h, y_h, z_h, 1) and the rank keys in *va, *vb
__device__ __forceinline__ float4 pick_hint(const HintCand* __restrict__ cand, const float* __restrict__ X,
                                            int stride, int p, uint32_t* va, uint32_t* vb) {
    int best = -1;
    double bT = 0.0;
#pragma unroll
    for (int q = 0; q < kHintCands; q++) {
        const HintCand c = cand[(size_t)p * kHintCands + q];
        if (c.row >= 0 && (best < 0 || c.T < bT || (c.T == bT && c.row < best))) {
            best = c.row;
            bT = c.T;
            *va = c.va;
            *vb = c.vb;
        }
    }
    if (best < 0) return make_float4(0.f, 0.f, 0.f, 0.f);
    return make_float4(X[best], X[stride + best], X[2 * stride + best], 1.f);
}
__device__ __forceinline__ RefineWin refine_windows(int ba, int bb, float xi, float yi, float zi,
                                                    const HintCand* __restrict__ hint,
                                                    const float* __restrict__ X, int stride,
                                                    int p) {
    RefineWin W;
    W.a0 = (uint32_t)ba << kBinShift;
    W.a1 = (uint32_t)(ba + 1) << kBinShift;
    W.b0 = (uint32_t)bb << kBinShift;
    W.b1 = (uint32_t)(bb + 1) << kBinShift;
    W.wa = W.wb = kLowBits;
    if (!hint) return W;
    uint32_t va = 0, vb = 0;
    const float4 h = pick_hint(hint, X, stride, p, &va, &vb);
    if (!(h.w > 0.f)) return W;
    const float delta = __builtin_sqrtf(rdist2(xi, yi, zi, h.x, h.y, h.z));
    RefineWin A = W;
    uint32_t k0;
    int w;
    if (refine_interval(__builtin_sqrtf(__uint_as_float(va)), delta, &k0, &w)) {
        A.a0 = k0;
        A.a1 = k0 + ((uint32_t)kNS << w);
        A.wa = w;
    }
    if (refine_interval(__builtin_sqrtf(__uint_as_float(vb)), delta, &k0, &w)) {
        A.b0 = k0;
        A.b1 = k0 + ((uint32_t)kNS << w);
        A.wb = w;
    }
    // disjoint and in order, or identical (the default windows of one bin): else the default
    if ((A.a0 == A.b0 && A.wa == A.wb) || A.a1 <= A.b0) return A;
    return W;
}

// Tighter bounds for the surviving rows (4 per block, lanes rotating over the rows as in the
// bounds kernel).  For each row: the exact s of every column (the reference's expression),
// an fp64 sum of sqrt(s) (raw v_sqrt_f32, bracketed by its 2^-22 error bound) over the keys
// strictly between the two rank windows (refine_windows: by default the bins b_a, b_b of ranks
// lo and hi-1 from the bounds kernel), exact counts below them, and 1024-way sub-histograms of
// the two windows.  The window's part inside them is bracketed with sub-bin resolution (2^-15
// relative instead of 2^-5 with the default windows; 2^-20..2^-21 on hinted intervals), so the
// bounds tighten by ~1000x and the next selection keeps only genuine near-ties -- this is what
// makes a two-cluster row set (every row's mean within 1 % of the minimum) cheap.
// A row whose ranks do not fall into its windows under the exact binning keeps its old bounds.
__device__ void consensus_refine_block(const int32_t* __restrict__ kcount,
                                       const float* __restrict__ rv,
                                       const float* __restrict__ dscale, int stride,
                                       double trim_lo, double trim_hi,
                                       const int32_t* __restrict__ surv,
                                       const int32_t* __restrict__ nsurv,
                                       const int32_t* __restrict__ bsel, double* __restrict__ lb,
                                       double* __restrict__ ub, const int32_t* __restrict__ list,
                                       int lstride, const int32_t* __restrict__ lcount, int step,
                                       const HintCand* __restrict__ hint, int p, int vb) {
    __shared__ uint32_t sub[kRefineRows][2][kNS];
    __shared__ double inner_w[4][kRefineRows];  // [wave][row]
    __shared__ int below[kRefineRows][2];
    const int tid = threadIdx.x, lane = wave_lane();
    const int K = kcount[p];
    const int ns = nsurv[p];
    if (ns <= kRefineMin) return;  // few survivors: the exact pass is cheaper
    // the rows refined here: every step-th survivor (step > 1: the Lipschitz references) or the
    // per-pair list of the survivors the references did not prune (lcount)
    const int nl = lcount ? lcount[p] : (ns + step - 1) / step;
    const int s0 = vb * kRefineRows;
    if (s0 >= nl) return;
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    if (hi <= lo) return;
    const float* X = rv + (size_t)p * 3 * stride;
    const float* Y = X + stride;
    const float* Z = Y + stride;
    const int base = bounds_elo(dscale[p]) << kMantBits;
    // (list == nullptr: the rows 0, step, 2 step, ... themselves -- the first-stage references
    // of a flat pair, launch_consensus_bounds)
    const int32_t* S = list ? list + (size_t)p * lstride : nullptr;
    auto srow = [&](int k) { return S ? (int)S[(size_t)k * step] : k * step; };
    float xi[kRefineRows], yi[kRefineRows], zi[kRefineRows];
    uint32_t a0[kRefineRows], b0[kRefineRows];  // the windows (a1 = a0 + (kNS << wa), ...)
    int wa[kRefineRows], wb[kRefineRows];
    float acc[kRefineRows];  // per-thread partial sums (<= ceil(K/256) terms; bracketed below)
    int bel_a[kRefineRows], bel_b[kRefineRows];
#pragma unroll
    for (int t = 0; t < kRefineRows; t++) {
        const int r = (lane + t) & (kRefineRows - 1);
        const int row = srow(min(s0 + r, nl - 1));
        xi[t] = X[row];
        yi[t] = Y[row];
        zi[t] = Z[row];
        const RefineWin W = refine_windows(bsel[((size_t)p * stride + row) * 2] + base,
                                           bsel[((size_t)p * stride + row) * 2 + 1] + base,
                                           xi[t], yi[t], zi[t], hint, X, stride, p);
        a0[t] = W.a0;
        b0[t] = W.b0;
        wa[t] = W.wa;
        wb[t] = W.wb;
        acc[t] = 0.f;
        bel_a[t] = 0;
        bel_b[t] = 0;
    }
    for (int q = tid; q < kRefineRows * 2 * kNS; q += 256) (&sub[0][0][0])[q] = 0u;
    if (tid < kRefineRows) {
        below[tid][0] = 0;
        below[tid][1] = 0;
    }
    __syncthreads();
    for_columns(X, Y, Z, K, [&](float xj, float yj, float zj) {
#pragma unroll
        for (int t = 0; t < kRefineRows; t++) {
            const float s = rdist2(xi[t], yi[t], zi[t], xj, yj, zj);
            const uint32_t key = __float_as_uint(s);
            const bool ba_ = key < a0[t], bb_ = key < b0[t];
            bel_a[t] += ba_;
            bel_b[t] += bb_;
            // sub-bin indices (a key below a window wraps to a huge index)
            const uint32_t ia = (key - a0[t]) >> wa[t], ib = (key - b0[t]) >> wb[t];
            const bool ina = ia < (uint32_t)kNS;
            // branch-free inner sum (raw v_sqrt_f32, <= 1 ulp; f32 accumulation) over the keys
            // in [a1, b0) -- only the window counts take a (short, divergent) branch
            acc[t] += (!ba_ && !ina && bb_) ? __builtin_amdgcn_sqrtf(s) : 0.f;
            if (ina || ib < (uint32_t)kNS) {
                const int r = (lane + t) & (kRefineRows - 1);
                atomicAdd(&sub[r][ina ? 0 : 1][ina ? ia : ib], 1u);
            }
        }
    });
    // the inner sums in a fixed order (a wave tree, then the waves in order): fp64 LDS atomics
    // made the last bits -- and with them a borderline pruning decision of the flat-pair route,
    // whose references' refined bounds set U -- depend on the arrival order
#pragma unroll
    for (int r = 0; r < kRefineRows; r++) {
        float v = 0.f;
#pragma unroll
        for (int t = 0; t < kRefineRows; t++)
            if (((lane + t) & (kRefineRows - 1)) == r) v = acc[t];
        double d = (double)v;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
        if (lane == 0) inner_w[tid >> 6][r] = d;
    }
#pragma unroll
    for (int t = 0; t < kRefineRows; t++) {
        const int r = (lane + t) & (kRefineRows - 1);
        atomicAdd(&below[r][0], bel_a[t]);
        atomicAdd(&below[r][1], bel_b[t]);
    }
    __syncthreads();
    // per row (one wave): bracket the window's part inside the two key windows
    const int r = tid >> 6, sl = tid & 63;
    if (s0 + r >= nl) return;
    const int row = srow(s0 + r);
    const RefineWin W = refine_windows(bsel[((size_t)p * stride + row) * 2] + base,
                                       bsel[((size_t)p * stride + row) * 2 + 1] + base, X[row],
                                       Y[row], Z[row], hint, X, stride, p);
    const int cA = below[r][0], cB = below[r][1];
    // sub-bin k of a window [x0, ...) covers keys [x0 + (k << w), x0 + ((k + 1) << w)); every d
    // in it is <= the lower edge of sub-bin k + 1 (sqrtf is monotone)
    auto sub_lo = [&](uint32_t x0, int w, int k) {
        return (double)__builtin_sqrtf(__uint_as_float(x0 + ((uint32_t)k << w)));
    };
    // the window's ranks inside window A: [max(lo, cA), min(hi, cA + nA)); inside window B
    // (when distinct): [cB, hi).  Count per sub-bin, clipped to those rank ranges, times the
    // sub-bin's d-range gives the bounds.
    double L = 0.0, U = 0.0;
    int nA = 0, nB = 0;
    for (int k = sl; k < kNS; k += 64) {
        nA += (int)sub[r][0][k];
        nB += (int)sub[r][1][k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        nA += __shfl_xor(nA, o, 64);
        nB += __shfl_xor(nB, o, 64);
    }
    const bool same = W.a0 == W.b0;
    bool ok = cA <= lo && lo < cA + nA && (same ? (hi - 1 < cA + nA) : (cB <= hi - 1 && hi - 1 < cB + nB));
    if (ok) {
        // sub-bins in ascending order: thread sl owns k = 16 sl .. 16 sl + 15
        for (int part = 0; part < (same ? 1 : 2); part++) {
            const uint32_t* hh = sub[r][part];
            const uint32_t x0 = part ? W.b0 : W.a0;
            const int w = part ? W.wb : W.wa;
            const int c0 = part ? cB : cA;
            int cnt = 0;
            for (int q = 0; q < 16; q++) cnt += (int)hh[16 * sl + q];
            int x = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (sl >= o) x += y;
            }
            int cum = c0 + x - cnt;
            for (int q = 0; q < 16; q++) {
                const int k = 16 * sl + q;
                const int n = (int)hh[k];
                const int a0_ = max(cum, lo), a1_ = min(cum + n, hi);
                if (a1_ > a0_) {  // (only the sub-bins the rank window overlaps)
                    L += (double)(a1_ - a0_) * sub_lo(x0, w, k);
                    U += (double)(a1_ - a0_) * sub_lo(x0, w, k + 1);
                }
                cum += n;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        L += __shfl_xor(L, o, 64);
        U += __shfl_xor(U, o, 64);
    }
    if (sl == 0 && ok) {
        const double w = (double)(hi - lo);
        const double in = ((inner_w[0][r] + inner_w[1][r]) + inner_w[2][r]) + inner_w[3][r];
        // the inner sum used the raw v_sqrt_f32 (<= 2^-23 relative, flushes below 2^-126) and
        // per-thread f32 sums of n <= ceil(K/256) non-negative terms (relative error <= n 2^-24,
        // then exact enough in fp64): bracket it by 2^-22 + (n + 1) 2^-24 relative plus 2^-63
        // per term (the inner count is at most K)
        const double rel = 0x1p-22 + (double)((K + 255) / 256 + 1) * 0x1p-24;
        const double inl = in * (1.0 - rel), inu = in * (1.0 + rel) + (double)K * 0x1p-63;
        const double nl = ((inl + L) / w) * (1.0 - 1e-9), nu = ((inu + U) / w) * (1.0 + 1e-9);
        double* lp = lb + (size_t)p * stride + row;
        double* up = ub + (size_t)p * stride + row;
        *lp = fmax(*lp, nl);
        *up = fmin(*up, nu);
    }
}

// The refine pass's rank-key hint (refine_windows): per pair with > kRefineMin survivors, a
// survivor h near the minimum and the exact keys va, vb at its ranks lo and hi-1; pairs with
// <= min_nc candidates get none.  h = the candidate with the smallest exact trimmed mean among
// the kHintCands survivors with the smallest UB (lowest row on ties): on a two-cluster set the
// UBs of both clusters' rows lie within the coarse bounds' 2^-5 of each other, and a hint from
// the far cluster leaves every near-cluster row its default windows.  Block (p, q) takes
// candidate q (radix_window_sum: four passes over the pair's K columns) into cand[p][q], and
// the refine pass picks the best per pair (pick_hint).  surv == nullptr: the candidates are the rows 0, step,
// 2 step, ... < nsurv[p] (a flat pair's first-stage references) instead of the survivor list.
__global__ __launch_bounds__(256) void consensus_hint_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv, int stride, double trim_lo,
    double trim_hi, const int32_t* __restrict__ surv, const int32_t* __restrict__ nsurv, int step,
    int min_nc, const double* __restrict__ ub, HintCand* __restrict__ cand) {
    __shared__ uint32_t histA[2048], histB[2048];
    __shared__ int ws[8];
    __shared__ int res[2];
    __shared__ double red[8];
    __shared__ double rb_u[4];
    __shared__ int rb_r[4];
    const int p = blockIdx.x, q = blockIdx.y, tid = threadIdx.x;
    const int K = kcount[p], ns = nsurv[p];
    const long lo = (long)(K * trim_lo), hi = (long)(K * trim_hi);
    const int32_t* S = surv ? surv + (size_t)p * stride : nullptr;
    const int nc = S ? ns : (ns + step - 1) / step;
    HintCand* out = cand + (size_t)p * kHintCands + q;
    if (ns <= kRefineMin || hi <= lo || nc <= min_nc || q >= nc) {
        if (tid == 0) out->row = -1;
        return;
    }
    // the (q+1)-th smallest (UB, row): q + 1 rounds of a block argmin excluding the rows taken
    int taken[kHintCands];
    int br = 0x7fffffff;
    for (int e = 0; e <= q; e++) {
        double bu = __builtin_inf();
        br = 0x7fffffff;
        for (int k = tid; k < nc; k += 256) {
            const int row = S ? (int)S[k] : k * step;
            bool t = false;
            for (int f = 0; f < e; f++) t |= taken[f] == row;
            const double u = ub[(size_t)p * stride + row];
            if (!t && (u < bu || (u == bu && row < br))) {
                bu = u;
                br = row;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double u = __shfl_xor(bu, o, 64);
            const int r = __shfl_xor(br, o, 64);
            if (u < bu || (u == bu && r < br)) {
                bu = u;
                br = r;
            }
        }
        __syncthreads();  // (the previous round's readers of rb_u / rb_r are done)
        if ((tid & 63) == 0) {
            rb_u[tid >> 6] = bu;
            rb_r[tid >> 6] = br;
        }
        __syncthreads();
        bu = rb_u[0];
        br = rb_r[0];
        for (int w = 1; w < 4; w++)
            if (rb_u[w] < bu || (rb_u[w] == bu && rb_r[w] < br)) {
                bu = rb_u[w];
                br = rb_r[w];
            }
        taken[e] = br;
    }
    if (br == 0x7fffffff) {  // (no finite UB left)
        if (tid == 0) out->row = -1;
        return;
    }
    const float* X = rv + (size_t)p * 3 * stride;
    const float* Y = X + stride;
    const float* Z = Y + stride;
    RankKeys rk;
    const double T = radix_window_sum(X, Y, Z, K, X[br], Y[br], Z[br], lo, hi, histA, histB, ws,
                                      res, red, &rk);
    if (tid == 0) {
        out->T = T;
        out->row = br;
        out->va = rk.va;
        out->vb = rk.vb;
    }
}

// Work items of all pairs flattened: item g of the batch = (pair p, unit u); the per-pair unit
// counts are only known on the device, so list_prefix_kernel writes their exclusive prefix uoff
// and the item kernels stride over a fixed grid (no empty blocks, pairs balanced), finding
// each item's pair by one binary search (a walk over the pairs' counts per item costs up to
// n_pairs dependent scalar loads)
__device__ __forceinline__ void pair_of_item(const int32_t* __restrict__ uoff, int n_pairs, int g,
                                             int* p_out, int* u_out) {
    int a = 0, b = n_pairs;  // largest p with uoff[p] <= g
    while (b - a > 1) {
        const int m = (a + b) >> 1;
        if (uoff[m] <= g) a = m; else b = m;
    }
    *p_out = a;
    *u_out = g - uoff[a];
}

// the rows of the per-pair lists (Lipschitz survivors): (pair, unit) items of all pairs
// flattened, so the live units are the first blocks of the grid (the list lengths are only
// known on the device; a [unit][pair] grid sized for full lists would interleave ~80 % empty
// blocks with the live ones).  uoff = exclusive prefix of the per-pair unit counts
// (list_prefix_kernel); item g belongs to the pair p with uoff[p] <= g < uoff[p + 1].
__global__ __launch_bounds__(1024) void list_prefix_kernel(const int32_t* __restrict__ rcount,
                                                           int n_pairs, int div, int minc,
                                                           int32_t* __restrict__ uoff) {
    __shared__ int ws[16];
    __shared__ int carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int q0 = 0; q0 < n_pairs; q0 += 1024) {
        const int q = q0 + tid;
        const int c = q < n_pairs ? rcount[q] : 0;  // units: ceil(c / div), none if c <= minc
        const int u = c > minc ? (c + div - 1) / div : 0;
        int x = u;  // inclusive wave scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[w] = x;
        __syncthreads();
        int before = carry;
        for (int k = 0; k < w; k++) before += ws[k];
        if (q < n_pairs) uoff[q] = before + x - u;
        __syncthreads();
        if (tid == 1023) carry = before + x;
        __syncthreads();
    }
    if (tid == 0) uoff[n_pairs] = carry;
}

// ---- convexity-augmented pruning (round 4; ctx knob ERP_LIPG, default on) ----------------
// Beyond 1-Lipschitz, every distance is CONVEX in x: d(x, x_j) >= a_j + <u_j, x - c> with
// a_j = d(c, x_j) and u_j = (c - x_j) / a_j (u_j = 0 when a_j = 0: d(x, x_j) = |x - c| >= 0).
// With delta = x - c, b_j = <u_j, delta> (|b_j| <= |delta|) and W(v) = the sum of the order
// statistics lo .. hi-1 of v (monotone in every element), F_m(v) = the sum of its m smallest:
//   W(d(x, .)) >= W(a + b) = F_hi(a + b) - F_lo(a + b)
//              >= [F_hi(a) + F_hi(b)] - [F_lo(a) + sum_{S_lo(a)} b]
//              >= W(a) + sum_j b_j - (K - hi) |delta| - <g_S', delta> - (lo - |S'|) |delta|
// (F_hi(a + b) >= F_hi(a) + F_hi(b) over its minimising set; F_lo(a + b) <= the sum over S_lo(a);
// F_hi(b) = sum_j b_j minus its K - hi largest, each <= |delta|; S' = the columns whose key lies
// two or more bins below the bin of rank lo -- strictly below every column from that bin on,
// so inside S_lo(a) whatever the rounding -- and the lo - |S'| other members of S_lo(a) add
// <= |delta| each).  Hence
//   T(x) >= T(c) + <G, delta> - pen |delta|,  G = (g_all - g_S') / w,
//   pen = ((K - hi) + (lo - |S'|)) / w  (~1/3 at the reference's 0.2 / 0.8 trim, against the
// Lipschitz bound's 1).  Near the minimum, where T is flat and Lipschitz pruning stops, this
// prunes ~half of the rows the first stage leaves (a numpy model of the configs[1] fixture
// pair: L1 1631 -> 853 rows with G on the 77 central references of 625).  G costs one more
// K-column pass per reference (unit vectors: one rsq), so only the central references get it:
// those that can prune (LB_c > U) with UB_c <= U gfac.
// Rigor: G is summed in f32 per thread (<= ceil(K/256) unit vectors of norm <= 1 + 2^-21 each)
// and in fp64 over the block, so |G~ - G| w <= K 2^-20 + 256 n^2 2^-23 (n = ceil(K/256)); that
// and the f32 evaluation of the test (delta, the dot product, |delta| by v_sqrt_f32: each
// <= ~1e-6 of (|G| + pen) |delta|) are covered by pen += eps_G + 1e-5 (|G| + pen + 1); the
// reference's own f32 distances and fp64 sum (T_ref = T (1 +- 4u)) by LB_c (1 - 1e-5) and
// U (1 + 1.1e-5), as in the Lipschitz test: a pruned row's LB = U (1 + 5e-6) stays rigorous.

// the references of pair p that get G (stage-1 reference rows ra + c lstep of the shard): can
// prune (LB_c (1 - 1e-5) > U (1 + 1e-5)), central (UB_c <= U gfac), window bin of rank lo >= 2
// (slist != nullptr: the second stage's references, slist[p][0 .. scount[p]), against its U)
__global__ __launch_bounds__(256) void consensus_grad_select_kernel(
    const int32_t* __restrict__ kcount, int stride, const double* __restrict__ lb,
    const double* __restrict__ ub, const int32_t* __restrict__ bsel, int lstep, int shard,
    int nshards, const int32_t* __restrict__ slist, const int32_t* __restrict__ scount,
    const double* __restrict__ lU, float gfac, int32_t* __restrict__ gsel,
    int32_t* __restrict__ gcnt, int gcap) {
    __shared__ int n;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int K = kcount[p];
    const double U = lU[p];
    if (tid == 0) n = 0;
    __syncthreads();
    if (U < __builtin_huge_val()) {
        const int ra = slist ? 0 : (int)((int64_t)K * shard / nshards);
        const int nr = slist ? scount[p] : (int)((int64_t)K * (shard + 1) / nshards) - ra;
        const int nref = nr > 0 ? (nr + lstep - 1) / lstep : 0;
        const int32_t* SL = slist ? slist + (size_t)p * stride : nullptr;
        const double Um = U * (1.0 + 1e-5), Uc = U * (double)gfac;
        for (int c = tid; c < nref; c += 256) {
            const int row = SL ? (int)SL[c * lstep] : ra + c * lstep;
            const size_t o = (size_t)p * stride + row;
            if (lb[o] * (1.0 - 1e-5) > Um && ub[o] <= Uc && bsel[o * 2] >= 2) {
                const int k = atomicAdd(&n, 1);
                if (k < gcap) gsel[(size_t)p * gcap + k] = row;
            }
        }
    }
    __syncthreads();
    if (tid == 0) gcnt[p] = min(n, gcap);
}

// G and pen of every selected reference (items = (pair, reference) flattened by goff): one block
// per item, the K columns in the bounds pass's own key computation (S' membership) -> gref
// [p][k][2] = {(c, LB_c (1 - 1e-5)), (G, pen)}
__global__ __launch_bounds__(256) void consensus_grad_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ dscale, int stride, double trim_lo, double trim_hi,
    const double* __restrict__ lb, const int32_t* __restrict__ bsel,
    const int32_t* __restrict__ gsel, const int32_t* __restrict__ goff, int n_pairs, int gcap,
    float4* __restrict__ gref) {
    __shared__ double red[7][4];
    const int tid = threadIdx.x, lane = wave_lane(), wv = tid >> 6;
    const int total = goff[n_pairs];
    for (int g = blockIdx.x; g < total; g += gridDim.x) {
        int p, k;
        pair_of_item(goff, n_pairs, g, &p, &k);
        const int c = gsel[(size_t)p * gcap + k];
        const int K = kcount[p];
        const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
        const float* X = rv + (size_t)p * 3 * stride;
        const float* Y = X + stride;
        const float* Z = Y + stride;
        const int elo = bounds_elo(dscale[p]);
        const uint32_t kmax = (uint32_t)((elo << kMantBits) + bsel[((size_t)p * stride + c) * 2] - 2);
        const float e0 = bounds_bias(elo);
        const float xc = X[c], yc = Y[c], zc = Z[c];
        float ga[3] = {0.f, 0.f, 0.f}, gs[3] = {0.f, 0.f, 0.f};
        int ns = 0;
        for (int j = tid; j < K; j += 256) {
            const float dx = xc - X[j], dy = yc - Y[j], dz = zc - Z[j];
            // the bounds pass's biased key (rows minus columns there: the squares are equal)
            const float sb = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __builtin_fmaf(dx, dx, e0)));
            const float s = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
            const float r = s > 0.f ? __builtin_amdgcn_rsqf(s) : 0.f;
            const float ux = dx * r, uy = dy * r, uz = dz * r;
            ga[0] += ux;
            ga[1] += uy;
            ga[2] += uz;
            if ((__float_as_uint(sb) >> kBinShift) <= kmax) {
                gs[0] += ux;
                gs[1] += uy;
                gs[2] += uz;
                ns++;
            }
        }
        double v[7] = {ga[0], ga[1], ga[2], gs[0], gs[1], gs[2], (double)ns};
#pragma unroll
        for (int q = 0; q < 7; q++) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
            if (lane == 0) red[q][wv] = v[q];
        }
        __syncthreads();
        if (tid == 0) {
            double t[7];
#pragma unroll
            for (int q = 0; q < 7; q++) t[q] = (red[q][0] + red[q][1]) + (red[q][2] + red[q][3]);
            const double w = (double)(hi - lo);
            const double G0 = (t[0] - t[3]) / w, G1 = (t[1] - t[4]) / w, G2 = (t[2] - t[5]) / w;
            const double nth = (double)((K + 255) / 256);
            const double epsG = ((double)K * 0x1p-20 + 256.0 * nth * nth * 0x1p-23) / w;
            double pen = ((double)(K - hi) + (double)(lo - (int)t[6])) / w + epsG;
            const double gn = sqrt(G0 * G0 + G1 * G1 + G2 * G2);
            pen += 1e-5 * (gn + pen + 1.0);
            float4* o = gref + ((size_t)p * gcap + k) * 2;
            o[0] = make_float4(xc, yc, zc, (float)(lb[(size_t)p * stride + c] * (1.0 - 1e-5)));
            // (G rounded to f32: its error, 2^-24 |G| |delta|, is inside the 1e-5 |G| term)
            o[1] = make_float4((float)G0, (float)G1, (float)G2, (float)(pen * (1.0 + 1e-6)));
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void consensus_bounds_list_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ dscale, const float* __restrict__ edges, int stride, double trim_lo,
    double trim_hi, double* __restrict__ lb, double* __restrict__ ub, int32_t* __restrict__ bsel,
    const int32_t* __restrict__ rlist, const int32_t* __restrict__ rcount,
    const int32_t* __restrict__ uoff, int n_pairs) {
    const int g = blockIdx.x;  // one unit per block (a loop over units doubles the VGPRs)
    if (g >= uoff[n_pairs]) return;
    int a = 0, b = n_pairs;  // largest p with uoff[p] <= g
    while (b - a > 1) {
        const int m = (a + b) >> 1;
        if (uoff[m] <= g) a = m; else b = m;
    }
    consensus_bounds_unit(kcount, rv, dscale, edges, stride, trim_lo, trim_hi, lb, ub, bsel, 0, 1,
                          1, rlist, rcount, a, g - uoff[a]);
}

// ---- zoom: the first selection's survivors re-binned on a 4x finer grid -------------------
// The first bounds pass bins s = d^2 at 16 bins per binade over 36 binades (any distance range);
// its bounds are ~2 % wide in d, so ~150 rows per pair survive the first selection.  The
// survivors' rank windows (bsel: the bins of ranks lo and hi-1) span a few binades, so a second
// histogram pass over the survivors only, at 64 bins per binade over 9 binades placed on those
// windows (per pair: consensus_zoom_prep), tightens LB / UB ~4x; the re-selection then keeps ~8x
// fewer rows (T grows quadratically near its minimum) for refine / the exact pass.  The zoom
// bins the reference's own s (rdist2: same operations, no bias), so the d-range of a bin is
// [sqrtf(s_b), sqrtf(s_b+1)] exactly (sqrtf is monotone); keys below / above the 9 binades are
// clamped into bins 0 / kNB-1, whose edges are 0 / +inf.  Bounds only ever tighten (LB = max,
// UB = min with the first pass); bsel (the coarse bins refine and the exact pass use) stays.
// Two levels: 64 bins per binade over 9 binades placed on the coarse windows (bsel), then
// 256 bins per binade over 2.25 binades placed on the level-1 windows (zsel, written by the
// level-1 pass), each followed by a re-selection.
#ifndef ERP_ZOOM_MIN
#define ERP_ZOOM_MIN 8
#endif
constexpr int kZoomMin = ERP_ZOOM_MIN;         // survivors per pair below which no zoom pass
#ifndef ERP_ZOOM_MAX
#define ERP_ZOOM_MAX 2048
#endif
constexpr int kZoomMax = ERP_ZOOM_MAX;         // ... and above which none either

// d-space edges of the zoom grid whose first bin is z (absolute, in units of key >> (23 - MANT)):
// bin b holds the keys of [z + b, z + b + 1) << (23 - MANT), so the reference's d = sqrtf(s)
// lies in [sqrtf(lower key), sqrtf(upper key)]; the edge bins also hold the clamped keys
// The zoom bins s' = fma(dz, dz, fma(dy, dy, dx dx)) (two roundings fewer than the reference's
// s = dx dx + dy dy + dz dz; both within 2^-22.4 of the exact sum of the exact squares of the
// same dx, dy, dz), so the reference's s of a key in [E_b, E_b+1) lies in [E_b (1 - 2^-21),
// E_b+1 (1 + 2^-21)] and its d = sqrtf(s) in [sqrtf(E_b) (1 - 2^-20), sqrtf(E_b+1) (1 + 2^-20)]
// (the factors also cover sqrtf's own rounding and the f32 products).
template <int MANT>
__device__ __forceinline__ void zoom_grid_edges(int z, float* __restrict__ ed) {
    constexpr int kShift = 23 - MANT;
    for (int b = threadIdx.x; b < kNB; b += blockDim.x) {
        const uint32_t key = (uint32_t)(z + b) << kShift;
        ed[b] = b == 0 ? 0.f : __builtin_sqrtf(__uint_as_float(key)) * (1.0f - 0x1p-20f);
        ed[kNB + b] = b == kNB - 1
                          ? kInf
                          : __builtin_sqrtf(__uint_as_float(key + (1u << kShift))) * (1.0f + 0x1p-20f);
    }
}

// per pair: the zoom grid's first bin zbase[p] (absolute, in units of key >> (23 - MANT); -1:
// no zoom) from the span of the survivors' rank-window bins of the previous grid (SRC_MANT bins
// per binade, absolute), and its d-space edges
template <int MANT, int SRC_MANT>
__global__ __launch_bounds__(256) void consensus_zoom_prep_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ dscale,
    const int32_t* __restrict__ surv, const int32_t* __restrict__ nsurv,
    const int32_t* __restrict__ wsel, int wsel_base_coarse, int stride, double trim_lo,
    double trim_hi, int32_t* __restrict__ zbase, float* __restrict__ edz) {
    static_assert(MANT >= SRC_MANT, "finer grid");
    __shared__ int red[2][4];
    const int p = blockIdx.x, tid = threadIdx.x, lane = wave_lane();
    const int K = kcount[p], n = nsurv[p];
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    // (a pair whose means all lie within ~1 % of each other -- two clusters -- keeps most of its
    // rows through any grid: the refine pass's Lipschitz stage handles it)
    if (n <= kZoomMin || n > kZoomMax || hi <= lo) {
        if (tid == 0) zbase[p] = -1;
        return;
    }
    int amin = 1 << 30, bmax = -1;
    for (int k = tid; k < n; k += 256) {
        const int row = surv[(size_t)p * stride + k];
        const int a = wsel[((size_t)p * stride + row) * 2];
        const int b = wsel[((size_t)p * stride + row) * 2 + 1];
        if (a >= 0 && b >= 0) {  // (-1: a second-stage reference whose window left the fine grid)
            amin = min(amin, a);
            bmax = max(bmax, b);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        amin = min(amin, __shfl_xor(amin, o, 64));
        bmax = max(bmax, __shfl_xor(bmax, o, 64));
    }
    if (lane == 0) {
        red[0][tid >> 6] = amin;
        red[1][tid >> 6] = bmax;
    }
    __syncthreads();
    amin = min(min(red[0][0], red[0][1]), min(red[0][2], red[0][3]));
    bmax = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
    if (bmax < 0) {
        if (tid == 0) zbase[p] = -1;
        return;
    }
    // the first pass's bins are relative to the pair's grid (bsel + (elo << kMantBits));
    // the zoom passes write absolute bins
    const int off = wsel_base_coarse ? (bounds_elo(dscale[p]) << kMantBits) : 0;
    constexpr int up = MANT - SRC_MANT;
    const int ulo = (amin + off) << up, uhi = ((bmax + off + 1) << up) - 1;  // in this grid's bins
    const int z = max(max(ulo, uhi - (kNB - 1)), 1 << MANT);                 // top-aligned
    if (tid == 0) zbase[p] = z;
    zoom_grid_edges<MANT>(z, edz + (size_t)p * 2 * kNB);
}

// one unit (kBoundRows survivors of one pair) per block; items flattened over the pairs; writes
// the tightened bounds and the survivors' rank-window bins on this grid (zsel, absolute)
template <int MANT>
__device__ __forceinline__ void consensus_zoom_unit(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ edz, const int32_t* __restrict__ zbase_p, int stride, double trim_lo,
    double trim_hi, double* __restrict__ lb, double* __restrict__ ub,
    const int32_t* __restrict__ surv, const int32_t* __restrict__ nsurv,
    const int32_t* __restrict__ uoff, int n_pairs, int32_t* __restrict__ zsel, int g,
    uint32_t* hist, int step, const float* __restrict__ dscale, int32_t* __restrict__ bsel_out) {
    constexpr int kShift = 23 - MANT;
    constexpr int R = kBoundRows;
    constexpr int NS = 256 / R;
    constexpr int per = kNB / NS;
    int (*part)[R] = reinterpret_cast<int (*)[R]>(hist);
    float (*partL)[R] = reinterpret_cast<float (*)[R]>(hist + NS * R);
    float (*partU)[R] = reinterpret_cast<float (*)[R]>(hist + 2 * NS * R);
    int p = 0, b = n_pairs;  // largest p with uoff[p] <= g
    while (b - p > 1) {
        const int m = (p + b) >> 1;
        if (uoff[m] <= g) p = m; else b = m;
    }
    const int tid = threadIdx.x, lane = wave_lane();
    const int K = kcount[p], nloc = (nsurv[p] + step - 1) / step, zbase = zbase_p[p];
    const int l0 = (g - uoff[p]) * R;
    if (zbase < 0 || l0 >= nloc) return;  // (uniform)
    const int32_t* RL = surv + (size_t)p * stride;
    auto rowat = [&](int l) { return (int)RL[(size_t)l * step]; };
    const float* X = rv + (size_t)p * 3 * stride;
    const float* Y = X + stride;
    const float* Z = Y + stride;
    constexpr int kPairs = R / 2;
    f32x2 xi[kPairs], yi[kPairs], zi[kPairs];
    uint32_t hoff[R];
    const uint32_t hist_addr = (uint32_t)(size_t)(lds_u32*)hist;
#pragma unroll
    for (int t = 0; t < R; t++) {
        const int r = (lane + t) & (R - 1);
        const int row = rowat(min(l0 + r, nloc - 1));
        xi[t >> 1][t & 1] = X[row];
        yi[t >> 1][t & 1] = Y[row];
        zi[t >> 1][t & 1] = Z[row];
        // (absolute keys: bin 0 of the grid is key zbase)
        hoff[t] = hist_addr + 4u * (uint32_t)r - 64u * (uint32_t)zbase;
    }
    const uint32_t zlo = (uint32_t)zbase, zhi = (uint32_t)zbase + (uint32_t)(kNB - 1);
    for (int k = tid; k < kNB * R / 4; k += 256)
        reinterpret_cast<uint4*>(hist)[k] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    constexpr int CB = 4;
    float cx[CB], cy[CB], cz[CB], nx[CB], ny[CB], nz[CB];
    const uint32_t kmax4 = 4u * (uint32_t)(K - 1);
    auto ld = [](const float* base, uint32_t off) {
        return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + off);
    };
#pragma unroll
    for (int c = 0; c < CB; c++) {
        const uint32_t o = min(4u * (uint32_t)(c * 256 + tid), kmax4);
        cx[c] = ld(X, o);
        cy[c] = ld(Y, o);
        cz[c] = ld(Z, o);
    }
    for (int j0 = 0; j0 < K; j0 += CB * 256) {
#pragma unroll
        for (int c = 0; c < CB; c++) {
            const uint32_t o = min(4u * (uint32_t)(j0 + CB * 256 + c * 256 + tid), kmax4);
            nx[c] = ld(X, o);
            ny[c] = ld(Y, o);
            nz[c] = ld(Z, o);
        }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            if (j0 + c * 256 + tid < K) {
                const float xj = cx[c], yj = cy[c], zj = cz[c];
#pragma unroll
                for (int t = 0; t < kPairs; t++) {
                    // s' (zoom_grid_edges), two rows per packed instruction
                    const f32x2 dx = xi[t] - xj, dy = yi[t] - yj, dz = zi[t] - zj;
                    f32x2 s = dx * dx;
                    s = __builtin_elementwise_fma(dy, dy, s);
                    s = __builtin_elementwise_fma(dz, dz, s);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        // keys outside the grid clamp into its edge bins (one v_med3_u32)
                        uint32_t key;
                        asm("v_med3_u32 %0, %1, %2, %3"
                            : "=v"(key) : "v"(__float_as_uint(s[h]) >> kShift), "s"(zlo), "v"(zhi));
                        lds_inc(lshl6_add(key, hoff[2 * t + h]));
                    }
                }
            }
        }
#pragma unroll
        for (int c = 0; c < CB; c++) {
            cx[c] = nx[c];
            cy[c] = ny[c];
            cz[c] = nz[c];
        }
    }
    __syncthreads();
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    const int r = tid & (R - 1), sl = tid / R;
    const float* ed = edz + (size_t)p * 2 * kNB + sl * per;
    float el[per], eu[per];
    int n[per];
    int c = 0;
#pragma unroll
    for (int q = 0; q < per; q++) {
        el[q] = ed[q];
        eu[q] = ed[kNB + q];
        n[q] = (int)hist[(sl * per + q) * R + r];
        c += n[q];
    }
    __syncthreads();
    part[sl][r] = c;
    __syncthreads();
    int cum = 0;
    for (int q = 0; q < sl; q++) cum += part[q][r];
    const bool rvalid = l0 + r < nloc;
    const int row = rvalid ? rowat(l0 + r) : 0;
    float L = 0.f, U = 0.f;
    int sel_a = -1, sel_b = -1;  // bins of ranks lo and hi-1 on this grid
    if (cum < hi && cum + c > lo) {
        int c0 = min(max(cum, lo), hi);
#pragma unroll
        for (int q = 0; q < per; q++) {
            const int nc = cum + n[q];
            const int c1 = min(max(nc, lo), hi);
            const float w = (float)(c1 - c0);
            L = __builtin_fmaf(w, el[q], L);
            U = w > 0.f ? __builtin_fmaf(w, eu[q], U) : U;  // (0 * inf)
            sel_a = (cum <= lo && lo < nc) ? sl * per + q : sel_a;
            sel_b = (cum <= hi - 1 && hi - 1 < nc) ? sl * per + q : sel_b;
            cum = nc;
            c0 = c1;
        }
    }
    if (rvalid) {
        if (sel_a >= 0) zsel[((size_t)p * stride + row) * 2] = zbase + sel_a;
        if (sel_b >= 0) zsel[((size_t)p * stride + row) * 2 + 1] = zbase + sel_b;
        if (bsel_out) {
            // rows with no first-pass histogram (the second-stage references of the
            // pre-pruning): their rank-window bins on the coarse grid, which refine and the
            // exact pass start from, are the fine bins' coarse parents -- except in a clamped
            // edge bin, where they are unknown (-1: those passes then keep the old bounds /
            // take the radix path)
            static_assert(MANT >= kMantBits, "fine grid");
            const int cb = bounds_elo(dscale[p]) << kMantBits;
            auto coarse = [&](int sel) {
                if (sel <= 0 || sel >= kNB - 1) return -1;
                const int c = ((zbase + sel) >> (MANT - kMantBits)) - cb;
                return (c > 0 && c < kNB - 1) ? c : -1;
            };
            // (written by the slice that holds the rank: exactly one per rank when hi > lo)
            if (sel_a >= 0) bsel_out[((size_t)p * stride + row) * 2] = coarse(sel_a);
            if (sel_b >= 0) bsel_out[((size_t)p * stride + row) * 2 + 1] = coarse(sel_b);
        }
    }
    partL[sl][r] = L;
    partU[sl][r] = U;
    __syncthreads();
    if (sl == 0 && rvalid) {
        for (int q = 1; q < NS; q++) {
            L += partL[q][r];
            U += partU[q][r];
        }
        const double w = (double)(hi - lo);
        // margins: the f32 accumulation and the reference's own rounding of its sorted
        // sequential sum (as in the first pass)
        double* lp = lb + (size_t)p * stride + row;
        double* up = ub + (size_t)p * stride + row;
        const double nl = hi > lo ? ((double)L / w) * (1.0 - 2e-4) : 0.0;
        const double nu = hi > lo ? ((double)U / w) * (1.0 + 2e-4) : 0.0;
        if (bsel_out) {  // no earlier bounds for these rows: overwrite
            *lp = nl;
            *up = nu;
        } else {
            *lp = fmax(*lp, nl);
            *up = fmin(*up, nu);
        }
    }
}

// one unit per block (a loop over units doubles the VGPRs: 122 -> 248), the live units first
template <int MANT>
__global__ __launch_bounds__(256) void consensus_zoom_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ edz, const int32_t* __restrict__ zbase_p, int stride, double trim_lo,
    double trim_hi, double* __restrict__ lb, double* __restrict__ ub,
    const int32_t* __restrict__ surv, const int32_t* __restrict__ nsurv,
    const int32_t* __restrict__ uoff, int n_pairs, int32_t* __restrict__ zsel, int step,
    const float* __restrict__ dscale, int32_t* __restrict__ bsel_out) {
    __shared__ __align__(16) uint32_t hist[kNB * kBoundRows];  // [bin][row]
    if ((int)blockIdx.x >= uoff[n_pairs]) return;
    consensus_zoom_unit<MANT>(kcount, rv, edz, zbase_p, stride, trim_lo, trim_hi, lb, ub, surv,
                              nsurv, uoff, n_pairs, zsel, blockIdx.x, hist, step, dscale,
                              bsel_out);
}

// ---- flat pairs (round 4, ERP_OPT_FLAT_REFS) -------------------------------------------------
// A pair whose first-stage pruning kept more than flat_pct % of its rows is flat: every
// trimmed mean lies within the coarse bounds' 2^-5 of the minimum (the two-cluster sets of R1
// and R2 both valid in every iteration: K = 2 iters, every T within ~1e-3 of min T), so the
// references prune nothing and the list pass bins almost every row.  For such a pair the
// first-stage references themselves are refined (consensus_hint_kernel on the best of them +
// consensus_refine_kernel with the hinted key windows: bounds ~1e-7 wide instead of 2^-5) and
// the first stage re-runs against them: with U and the references' LB exact to ~1e-7 the
// pruning radius LB(c) - U is the true T(c) - min T, and a numpy model of a worst-case pair
// (K = 20 000) keeps ~700 rows instead of ~19 000.  Every pruning stays rigorous (the same
// Lipschitz test, tighter bounds).  Sets the per-pair gate nflat[p] = K (flat) or 0 and resets
// the flat pairs' list counts for the re-run.
__global__ void consensus_flat_gate_kernel(const int32_t* __restrict__ kcount,
                                           int32_t* __restrict__ rcount,
                                           int32_t* __restrict__ r2cnt, int n_pairs, int flat_pct,
                                           double trim_lo, double trim_hi,
                                           int32_t* __restrict__ nflat) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pairs) return;
    const int K = kcount[p];
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    const bool flat = K >= kLipMinK && hi > lo && (int64_t)rcount[p] * 100 > (int64_t)flat_pct * K;
    nflat[p] = flat ? K : 0;
    if (flat) {
        rcount[p] = 0;
        if (r2cnt) r2cnt[p] = 0;
    }
}

// ---- second pre-pruning stage (ERP_LIP2, default on) ------------------------------------
// After the first stage a configs[1] pair still lists ~16 % of its rows (L1): the rows near
// the minimum, where T is flat and the references every kLipStep-th row, with bounds 2^-5 wide, stop
// pruning.  Every m-th L1 row (the second-stage references) is bounded on the fine zoom grid
// (64 bins per binade of s, ~2^-7 wide, consensus_zoom_unit with a list step), and the other
// L1 rows are tested against them exactly as against the first-stage references (T is
// 1-Lipschitz): with U2 = min(U1, min UB over the second-stage references), any UB >= min T, a
// row with d(i, c) < LB(c) - U2 has T(i) > U2, so its LB = U2 (1 + M / 2) is rigorous.  Only
// the rows that survive (L2) get the coarse K-column histogram.  On the fixture pair of
// configs[1] (tests/golden/find_4096_it10k.npz) this bins 408 fine + ~620 coarse rows instead
// of ~1630 coarse rows after the 625 first-stage references (a numpy model of the two tests).
constexpr int kLip2Min = 64;              // smaller L1 lists: no second stage

// per pair: whether the second stage runs (zb[p] = the fine grid's first bin, else -1) and the
// fine grid's edges, placed on the rank windows (first-pass bsel) of the central first-stage
// references (UB within 1/16 of the smallest): the L1 rows lie near them, and T's order
// statistics are 1-Lipschitz too, so their windows lie near those
__global__ __launch_bounds__(256) void consensus_ref2_prep_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ dscale,
    const double* __restrict__ ub, const int32_t* __restrict__ bsel,
    const int32_t* __restrict__ n1c, int stride, double trim_lo, double trim_hi, int shard,
    int nshards, int32_t* __restrict__ zb, float* __restrict__ edz) {
    constexpr int MANT = 6;
    __shared__ double redd[4];
    __shared__ int red[2][4];
    const int p = blockIdx.x, tid = threadIdx.x, lane = wave_lane();
    const int K = kcount[p], n1 = n1c[p];
    const int lo = (int)(K * trim_lo), hi = (int)(K * trim_hi);
    if (n1 < kLip2Min || K < kLipMinK || hi <= lo) {
        if (tid == 0) zb[p] = -1;
        return;
    }
    const int ra = (int)((int64_t)K * shard / nshards), rb = (int)((int64_t)K * (shard + 1) / nshards);
    const int nref = rb > ra ? (rb - ra + kLipStep - 1) / kLipStep : 0;
    const double* U = ub + (size_t)p * stride;
    double m = __builtin_huge_val();
    for (int c = tid; c < nref; c += 256) m = fmin(m, U[ra + c * kLipStep]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
    if (lane == 0) redd[tid >> 6] = m;
    __syncthreads();
    m = fmin(fmin(redd[0], redd[1]), fmin(redd[2], redd[3]));
    const double lim = m * (1.0 + 0.0625);
    int amin = 1 << 30, bmax = -1;
    for (int c = tid; c < nref && m < __builtin_huge_val(); c += 256) {
        const int row = ra + c * kLipStep;
        if (U[row] <= lim) {
            amin = min(amin, bsel[((size_t)p * stride + row) * 2]);
            bmax = max(bmax, bsel[((size_t)p * stride + row) * 2 + 1]);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        amin = min(amin, __shfl_xor(amin, o, 64));
        bmax = max(bmax, __shfl_xor(bmax, o, 64));
    }
    if (lane == 0) {
        red[0][tid >> 6] = amin;
        red[1][tid >> 6] = bmax;
    }
    __syncthreads();
    amin = min(min(red[0][0], red[0][1]), min(red[0][2], red[0][3]));
    bmax = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
    if (bmax < 0 || amin > bmax) {
        if (tid == 0) zb[p] = -1;
        return;
    }
    const int off = bounds_elo(dscale[p]) << kMantBits;
    constexpr int up = MANT - kMantBits;
    const int ulo = (amin + off) << up, uhi = ((bmax + off + 1) << up) - 1;
    // margins: an L1 row's window reaches below the central references' (its rank-lo distance
    // is >= theirs - d(i, c) only) by more than it reaches above: 2 binades of s below ulo, 1
    // above uhi when the span allows, else the top kept
    const int z = max(max(ulo - 2 * (1 << MANT), uhi + (1 << MANT) - (kNB - 1)), 1 << MANT);
    if (tid == 0) zb[p] = z;
    zoom_grid_edges<MANT>(z, edz + (size_t)p * 2 * kNB);
}

// the test itself: the rows of L1 (l1[p][0 .. n1c[p])); those with is_ref2(row) are the
// references (bounded by the zoom pass; a function of the row index, not of the list position,
// so the reference set does not depend on the order the first stage appended L1 in: every
// record, binned_rows included, is the same on every run); the rows that survive are appended to
// l2 / n2c.  A pair without a second stage (zb < 0) passes every L1 row through.
__global__ __launch_bounds__(256) void consensus_lipschitz2_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv, int stride,
    double* __restrict__ lb, double* __restrict__ ub, const int32_t* __restrict__ l1,
    const int32_t* __restrict__ n1c, const int32_t* __restrict__ zb,
    const int32_t* __restrict__ bsel, int32_t* __restrict__ l2, int32_t* __restrict__ n2c,
    int32_t* __restrict__ nfb, const float4* __restrict__ lref, const double* __restrict__ lU,
    const int32_t* __restrict__ lcnt, int cap, const float4* __restrict__ gref,
    const int32_t* __restrict__ gcnt, int gcap) {
    __shared__ LipShared sh;
    const int p = blockIdx.y, tid = threadIdx.x, lane = wave_lane();
    const int n = n1c[p];
    const int i0 = blockIdx.x * 512;  // positions i0 .. i0 + 511 of L1
    if (i0 >= n) return;
    const bool on = zb[p] >= 0;  // (uniform)
    const int32_t* L = l1 + (size_t)p * stride;
    const float* X = rv + (size_t)p * 3 * stride;
    double* LBp = lb + (size_t)p * stride;
    double* UBp = ub + (size_t)p * stride;
    const double U = on ? lU[p] : __builtin_huge_val();  // min(U1, the references' UBs)
    const int nref = on ? lcnt[p] : 0;
    // candidates: the L1 rows that are not second-stage references, and the references whose
    // rank window left the fine grid (coarse window bins unknown, fine bounds loose: the coarse
    // pass re-bins them, overwriting their bounds and window bins)
    if (tid < 4) sh.cnt[tid] = 0;
    __syncthreads();
    int fb = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int k = i0 + 256 * h + tid;
        bool act = k < n;
        const int i = act ? (int)L[k] : 0;
        if (act && on && is_ref2(i)) {
            act = bsel[((size_t)p * stride + i) * 2] < 0 || bsel[((size_t)p * stride + i) * 2 + 1] < 0;
            fb += act;
        }
        const uint64_t bal = __builtin_amdgcn_ballot_w64(act);
        int base = 0;
        if (lane == 0 && bal) base = atomicAdd(&sh.cnt[3], __builtin_popcountll(bal));
        base = __shfl(base, 0, 64);
        if (act)
            sh.act[base + __builtin_popcountll(bal & ((1ull << lane) - 1ull))] =
                make_float4(X[i], X[stride + i], X[2 * stride + i], __int_as_float(i));
    }
    if (fb) atomicAdd(&nfb[p], fb);  // (rare: binned twice, counted once)
    __syncthreads();
    int na = sh.cnt[3];
    __syncthreads();
    if (tid == 3) sh.cnt[3] = 0;
    if (U < __builtin_huge_val() && nref > 0) {
        // (a pruned row's LB = U (1 + M / 2) is rigorous for a reference row too)
        auto prune = [&](int i) {
            LBp[i] = U * kLipPrunedLB;
            UBp[i] = __builtin_huge_val();
        };
        na = lip_prune_rows(sh, na, lref + (size_t)p * cap, nref, prune);
    }
    if (U < __builtin_huge_val() && gref && gcnt[p] > 0) {
        auto prune = [&](int i) {
            LBp[i] = U * (1.0 + 5e-6);
            UBp[i] = __builtin_huge_val();
        };
        na = lip_prune_grad(sh, na, gref + (size_t)p * gcap * 2, gcnt[p], U, prune);
    }
    lip_append(sh, na, l2 + (size_t)p * stride, &n2c[p]);
}

// binned rows beyond the first-stage references (erp_pair_result.binned_rows): the second-stage
// references plus L2
__global__ void consensus_ref2_count_kernel(int n_pairs, const int32_t* __restrict__ zb,
                                            const int32_t* __restrict__ r2c,
                                            const int32_t* __restrict__ n2c,
                                            const int32_t* __restrict__ nfb,
                                            int32_t* __restrict__ n1c) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pairs) return;
    n1c[p] = (zb[p] >= 0 ? r2c[p] : 0) + n2c[p] - nfb[p];
}

// ERP_REFINE_MINB (r03k): 4 blocks per CU bound the kernel to 128 VGPRs (153 unbounded, no
// spills either way; its 32 KB of LDS already allows 4): 4 waves per SIMD instead of 3
// (profiles/r03k_ab.txt: refine 0.626 -> 0.605 ms per 768-pair step)
#ifndef ERP_REFINE_MINB
#define ERP_REFINE_MINB 4
#endif
__global__ __launch_bounds__(256, ERP_REFINE_MINB) void consensus_refine_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ dscale, int stride, double trim_lo, double trim_hi,
    const int32_t* __restrict__ surv, const int32_t* __restrict__ nsurv,
    const int32_t* __restrict__ bsel, double* __restrict__ lb, double* __restrict__ ub,
    const int32_t* __restrict__ list, int lstride, const int32_t* __restrict__ lcount, int step,
    const HintCand* __restrict__ hint, const int32_t* __restrict__ uoff, int n_pairs) {
    const int total = uoff[n_pairs];  // units of kRefineRows listed rows, pairs with > kRefineMin
    for (int g = blockIdx.x; g < total; g += gridDim.x) {
        int p, u;
        pair_of_item(uoff, n_pairs, g, &p, &u);
        __syncthreads();  // the previous item's LDS readers are done
        consensus_refine_block(kcount, rv, dscale, stride, trim_lo, trim_hi, surv, nsurv, bsel,
                               lb, ub, list, lstride, lcount, step, hint, p, u);
    }
}

// Trimmed mean of a surviving row i, ranks [lo, hi), lo = (long)(K*0.2), hi = (long)(K*0.8).
// The bounds kernel already located the (s'-)bins b_a, b_b holding ranks lo and hi-1; here
//   pass 1: exact s = dx*dx + dy*dy + dz*dz for every column; exact counts below b_a and b_b
//           and 1024-way sub-histograms (key bits 18..9) of the two bins -> the sub-bins holding
//           the ranks;
//   pass 2: the fp64 sum of sqrtf(s) over every key strictly between those two sub-bins (a
//           register sum per thread), and 512-way histograms of the two sub-bins (key bits
//           8..0, i.e. exact values) -> the exact keys va, vb at ranks lo and hi-1 and their
//           multiplicities.
// Sum = the pass-2 sum + the exact values inside the rank sub-bins + the boundary
// multiplicities.  (The sort order of the distances is the order of s: sqrtf is monotone.)
// No fp64 LDS atomics (the sub-bins' sums used to be LDS fp64 atomics in pass 1), and the
// columns stream with kRowsCB loads in flight per thread (for_columns): one row per block reads
// all K columns twice, and with 4 loads in flight it waited on L2 for most of its time (on the
// worst-case batch, 1 700 survivors per two-cluster pair: 116 -> 75 ms per step; a
// wave-combined form of the sub-bin counts measured slower: its ballots run on every column).
// When a bin edge moved an element between the s' and s binnings across a rank, or a rank
// sits in the under/overflow bin, the row takes the 4-pass radix path instead.  The sum is
// not the reference's sorted sequential one in the last bits; consensus_final re-scores near
// ties exactly.
__device__ void consensus_rows_block(const int32_t* __restrict__ kcount,
                                     const float* __restrict__ rv,
                                     const float* __restrict__ dscale, int stride, double trim_lo,
                                     double trim_hi, const int32_t* __restrict__ surv,
                                     const int32_t* __restrict__ nsurv,
                                     const int32_t* __restrict__ bsel,
                                     double* __restrict__ tmean, int p, int vb) {
    __shared__ uint32_t histA[2048], histB[2048];  // radix fallback; level counts alias it
    __shared__ int ws[8];
    __shared__ int res[2];
    __shared__ double red[8];
    const int tid = threadIdx.x;
    const int K = kcount[p];
    if (vb >= nsurv[p]) return;
    const int i = surv[(size_t)p * stride + vb];
    const float* X = rv + (size_t)p * 3 * stride;
    const float* Y = X + stride;
    const float* Z = Y + stride;
    const float xi = X[i], yi = Y[i], zi = Z[i];
    const long lo = (long)(K * trim_lo);
    const long hi = (long)(K * trim_hi);
    if (hi <= lo) {
        if (tid == 0) tmean[(size_t)p * stride + i] = __builtin_nan("");
        return;
    }
    const int base = bounds_elo(dscale[p]) << kMantBits;
    const int ba = bsel[((size_t)p * stride + i) * 2], bb = bsel[((size_t)p * stride + i) * 2 + 1];
    bool fast = ba > 0 && bb < kNB - 1 && ba <= bb;
    double sum = 0.0;
    constexpr int NL = 1 << kLowBits;  // exact values per sub-bin
    uint32_t* cA = histA;        // level-2 counts of bin b_a
    uint32_t* cB = histA + kNS;  // of bin b_b (unused when b_a == b_b)
    uint32_t* tA = histB;        // level-3 counts of the sub-bin holding rank lo
    uint32_t* tB = histB + NL;   //                           and rank hi-1
    if (fast) {
        for (int k = tid; k < kNS; k += 256) {
            cA[k] = 0;
            cB[k] = 0;
        }
        for (int k = tid; k < NL; k += 256) {
            tA[k] = 0;
            tB[k] = 0;
        }
        __syncthreads();
        long belowA = 0, belowB = 0;
        // columns in batches of kRowsCB per thread, the next batch's loads in flight while this
        // one is binned (one row per block streams all K columns twice: with 4 loads in flight
        // the kernel waited on L2 for most of its time)
        for_columns(X, Y, Z, K, [&](float xj, float yj, float zj) {
            const float s = rdist2(xi, yi, zi, xj, yj, zj);
            const uint32_t key = __float_as_uint(s);
            const int e = min(max((int)(key >> kBinShift) - base, 0), kNB - 1);
            belowA += e < ba;
            belowB += e < bb;
            if (e == ba || e == bb)
                atomicAdd(&histA[(e == ba ? 0 : kNS) + (int)((key >> kLowBits) & (kNS - 1u))], 1u);
        });
        const long cumA = block_sum_i64(belowA, red);
        const long cumB = block_sum_i64(belowB, red);
        const uint32_t* cX = (ba == bb) ? cA : cB;
        long befA, befB;
        const int sa = find_bin<kNS>(cA, lo - cumA, &befA, ws, res);
        const int sb = find_bin<kNS>(cX, hi - 1 - cumB, &befB, ws, res);
        fast = lo >= cumA && hi - 1 >= cumB && sa >= 0 && sb >= 0;  // uniform
        if (fast) {
            const uint32_t prefA = ((uint32_t)(base + ba) << kSubBits) | (uint32_t)sa;  // key >> kLowBits
            const uint32_t prefB = ((uint32_t)(base + bb) << kSubBits) | (uint32_t)sb;
            double between = 0.0;  // keys in sub-bins strictly between prefA and prefB
            for_columns(X, Y, Z, K, [&](float xj, float yj, float zj) {
                const float s = rdist2(xi, yi, zi, xj, yj, zj);
                const uint32_t key = __float_as_uint(s);
                const uint32_t kp = key >> kLowBits;
                if (kp > prefA && kp < prefB) between += (double)__builtin_sqrtf(s);
                if (kp == prefA) atomicAdd(&tA[key & (NL - 1u)], 1u);
                else if (kp == prefB) atomicAdd(&tB[key & (NL - 1u)], 1u);
            });
            __syncthreads();
            // (prefA == prefB: both ranks in one sub-bin, counted in tA)
            const uint32_t* tX = prefA == prefB ? tA : tB;
            long befA3, befB3;
            const int ta = find_bin<NL>(tA, lo - cumA - befA, &befA3, ws, res);
            const int tb = find_bin<NL>(tX, hi - 1 - cumB - befB, &befB3, ws, res);
            const uint32_t va = (prefA << kLowBits) | (uint32_t)ta;
            const uint32_t vb = (prefB << kLowBits) | (uint32_t)tb;
            const long le_a = cumA + befA + befA3 + tA[ta];  // #keys <= va
            const long lt_b = cumB + befB + befB3;           // #keys <  vb
            double part = between;
            for (int k = tid; k < NL; k += 256) {  // exact values inside the rank sub-bins
                const double dA = (double)__builtin_sqrtf(__uint_as_float((prefA << kLowBits) | k));
                const double dB = (double)__builtin_sqrtf(__uint_as_float((prefB << kLowBits) | k));
                if (prefA != prefB) {
                    if (k > ta) part += (double)tA[k] * dA;
                    if (k < tb) part += (double)tB[k] * dB;
                } else {
                    if (k > ta && k < tb) part += (double)tA[k] * dA;
                }
            }
            const double mid = block_sum_f64(part, red);
            if (va == vb)
                sum = (double)(hi - lo) * (double)__builtin_sqrtf(__uint_as_float(va));
            else
                sum = mid + (double)(le_a - lo) * (double)__builtin_sqrtf(__uint_as_float(va)) +
                      (double)(hi - lt_b) * (double)__builtin_sqrtf(__uint_as_float(vb));
        }
        __syncthreads();
    }
    if (!fast) sum = radix_window_sum(X, Y, Z, K, xi, yi, zi, lo, hi, histA, histB, ws, res, red);
    if (tid == 0) tmean[(size_t)p * stride + i] = sum / ((double)(hi - lo) * 1.0);
}

__global__ __launch_bounds__(256) void consensus_rows_kernel(
    const int32_t* __restrict__ kcount, const float* __restrict__ rv,
    const float* __restrict__ dscale, int stride, double trim_lo, double trim_hi,
    const int32_t* __restrict__ surv, const int32_t* __restrict__ nsurv,
    const int32_t* __restrict__ bsel, double* __restrict__ tmean, const int32_t* __restrict__ uoff,
    int n_pairs) {
    // one unit per survivor; uoff == nullptr (batches of <= 16 pairs): the pairs' survivor
    // counts are walked here instead of a list_prefix_kernel launch
    int total = 0;
    if (uoff) total = uoff[n_pairs];
    else
        for (int q = 0; q < n_pairs; q++) total += nsurv[q];
    for (int g = blockIdx.x; g < total; g += gridDim.x) {
        int p = 0, u = g;
        if (uoff) pair_of_item(uoff, n_pairs, g, &p, &u);
        else
            while (u >= nsurv[p]) u -= nsurv[p++];
        __syncthreads();  // the previous row's LDS readers are done
        consensus_rows_block(kcount, rv, dscale, stride, trim_lo, trim_hi, surv, nsurv, bsel,
                             tmean, p, u);
    }
}

// survivors: rows with LB <= min UB, in row order; pruned rows get tmean = +inf
__global__ __launch_bounds__(1024) void consensus_select_kernel(const int32_t* __restrict__ kcount,
                                                                const double* __restrict__ lb,
                                                                const double* __restrict__ ub,
                                                                int stride, double trim_lo,
                                                                double trim_hi,
                                                                int32_t* __restrict__ surv,
                                                                int32_t* __restrict__ nsurv,
                                                                double* __restrict__ tmean,
                                                                int again) {
    __shared__ double sm[16];
    __shared__ int ws[16];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int K = kcount[p];
    if (again && nsurv[p] <= kRefineMin) return;  // not refined: the list stands
    const double* L = lb + (size_t)p * stride;
    const double* U = ub + (size_t)p * stride;
    double* Tm = tmean + (size_t)p * stride;
    int32_t* S = surv + (size_t)p * stride;
    const long lo = (long)(K * trim_lo), hi = (long)(K * trim_hi);
    if (K <= 0) {
        if (tid == 0) nsurv[p] = 0;
        return;
    }
    if (hi <= lo) {  // empty window: every mean is 0/0 = NaN, std::min_element -> index 0
        for (int k = tid; k < K; k += 1024) Tm[k] = __builtin_nan("");
        if (tid == 0) nsurv[p] = 0;
        return;
    }
    // 4 independent loads in flight per thread (one block per pair: at configs[4]'s K ~ 89k
    // the loops are load-latency bound)
    double m = __builtin_huge_val();
    for (int k0 = 0; k0 < K; k0 += 4096) {
        double u[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = k0 + j * 1024 + tid;
            u[j] = k < K ? U[k] : __builtin_huge_val();
        }
        m = fmin(m, fmin(fmin(u[0], u[1]), fmin(u[2], u[3])));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
    if ((tid & 63) == 0) sm[tid >> 6] = m;
    __syncthreads();
    double minub = sm[0];
    for (int w = 1; w < 16; w++) minub = fmin(minub, sm[w]);
    // compaction in row order: the refine pass takes every kRefStep-th survivor by list position as
    // its references, so an arrival-order list (one LDS atomic per wave, until r04) made the
    // reference set -- and, once the refined references prune well, the survivor count --
    // differ run to run.  Wave w owns the rows [w C, (w + 1) C): pass 1 counts its survivors
    // (ballots), one prefix over the 16 wave counts, pass 2 writes them in order (the L re-read
    // hits L2); two barriers instead of a block scan per 1024 rows
    const int lane = tid & 63, wv = tid >> 6;
    const int C = ((K + 15) / 16 + 63) & ~63;
    const int r0 = wv * C, r1 = min(K, r0 + C);
    int cnt = 0;
    for (int k0 = r0; k0 < r1; k0 += 256) {
        double l[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = k0 + j * 64 + lane;
            l[j] = k < r1 ? L[k] : __builtin_huge_val();
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = k0 + j * 64 + lane;
            const bool keep = k < r1 && l[j] <= minub;
            if (k < r1 && !keep) Tm[k] = __builtin_huge_val();
            cnt += __builtin_popcountll(__builtin_amdgcn_ballot_w64(keep));
        }
    }
    if (lane == 0) ws[wv] = cnt;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; w++) base += ws[w];
    const uint64_t below = (1ull << lane) - 1ull;
    for (int k0 = r0; k0 < r1; k0 += 256) {
        double l[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = k0 + j * 64 + lane;
            l[j] = k < r1 ? L[k] : __builtin_huge_val();
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = k0 + j * 64 + lane;
            const bool keep = k < r1 && l[j] <= minub;
            const uint64_t bal = __builtin_amdgcn_ballot_w64(keep);
            if (keep) S[base + __builtin_popcountll(bal & below)] = k;
            base += __builtin_popcountll(bal);
        }
    }
    if (tid == 1023) nsurv[p] = base;  // (the last wave's end = the total)
}

// exact sorted-sequential trimmed mean of one row (std::sort + std::accumulate semantics)
__device__ double exact_row_mean(const float* X, const float* Y, const float* Z, int K, int i,
                                 long lo, long hi, float* buf, int npow2, double* sres) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const float xi = X[i], yi = Y[i], zi = Z[i];
    for (int j = tid; j < npow2; j += nt) buf[j] = j < K ? rdist(xi, yi, zi, X[j], Y[j], Z[j]) : kInf;
    __syncthreads();
    for (int k = 2; k <= npow2; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int t = tid; t < npow2; t += nt) {
                const int ixj = t ^ jj;
                if (ixj > t) {
                    const float a = buf[t], b = buf[ixj];
                    const bool up = (t & k) == 0;
                    if ((a > b) == up) {
                        buf[t] = b;
                        buf[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    if (tid == 0) {
        double acc = 0.0;
        for (long k = lo; k < hi; k++) acc += (double)buf[k];
        sres[0] = acc / ((double)(hi - lo) * 1.0);
    }
    __syncthreads();
    const double r = sres[0];
    __syncthreads();
    return r;
}

// argmin (std::min_element: first minimum, NaN never wins unless at index 0), exact re-score
// of rows within a relative 1e-9 band of the minimum, and the per-pair result record.
__global__ __launch_bounds__(1024) void consensus_final_kernel(
    const int32_t* __restrict__ counts, const int32_t* __restrict__ kcount,
    const float* __restrict__ rv, const float* __restrict__ tv, const double* __restrict__ tmean,
    const int32_t* __restrict__ flags, const int32_t* __restrict__ nsurv,
    const int32_t* __restrict__ nbin, int stride, int npow2, double sample_frac, double trim_lo,
    double trim_hi, float* __restrict__ sortbuf, erp_pair_result* __restrict__ results) {
    __shared__ double sv[1024];
    __shared__ int si[1024];
    __shared__ int cand[64];
    __shared__ int ws[16];
    __shared__ double sres[1];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int K = kcount[p];
    const int M = counts ? counts[p] : K;
    const int s = counts ? (int)(M * sample_frac) : 1;
    erp_pair_result r;
    for (int k = 0; k < 3; k++) {
        r.R[k] = 0.f;
        r.T[k] = 0.f;
    }
    r.M = M;
    r.K = K;
    r.sample_n = s;
    r.min_idx = -1;
    r.near_ties = 0;
    r.survivors = nsurv[p];
    r.binned_rows = !nbin || nbin[p] < 0 ? K : (K + kLipStep - 1) / kLipStep + nbin[p];
    r.min_dist = 0.0;
    const int fl = flags ? flags[p] : 0;
    if (fl & 1) r.status = ERP_TOO_FEW_POINTS;
    else if (fl & 8)
        r.status = ERP_INVALID_ARG;
    else if (fl & 6)
        r.status = ERP_INTERNAL;
    else if (s < 1)
        r.status = ERP_TOO_FEW_POINTS;
    else if (K == 0)
        r.status = ERP_NO_VALID_HYPOTHESIS;
    else
        r.status = ERP_OK;
    if (r.status != ERP_OK) {
        if (tid == 0) results[p] = r;
        return;
    }
    const double* Tm = tmean + (size_t)p * stride;
    const float* X = rv + (size_t)p * 3 * stride;
    const float* Y = X + stride;
    const float* Z = Y + stride;
    int best;
    double bv;
    if (__builtin_isnan(Tm[0])) {
        best = 0;
        bv = Tm[0];
    } else {
        double v = __builtin_huge_val();
        int bi = 0x7fffffff;
        for (int k0 = 0; k0 < K; k0 += 4096) {  // 4 loads in flight per thread
            double t[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = k0 + j * 1024 + tid;
                t[j] = k < K ? Tm[k] : __builtin_huge_val();
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (t[j] < v) {  // NaN never compares less; increasing k keeps the first index
                    v = t[j];
                    bi = k0 + j * 1024 + tid;
                }
        }
        sv[tid] = v;
        si[tid] = bi;
        __syncthreads();
        for (int o = 512; o > 0; o >>= 1) {
            if (tid < o) {
                const double a = sv[tid], b = sv[tid + o];
                const int ia = si[tid], ib = si[tid + o];
                if (b < a || (b == a && ib < ia)) {
                    sv[tid] = b;
                    si[tid] = ib;
                }
            }
            __syncthreads();
        }
        best = si[0];
        bv = sv[0];
        __syncthreads();
        // near ties: rows within 1e-9 (relative) of the approximate minimum; the first 64 of
        // them in row order (contiguous row ranges per thread + an ordered scan: deterministic,
        // and the lowest index of a run of identical rows is always kept)
        const double tol = 1e-9 * fabs(bv) + 1e-300;
        // count (coalesced); at most 64 candidates (the usual case: 1) are gathered in any order
        // and ranked by row index; more take the ordered contiguous-range scan
        int cnt = 0;
        for (int k0 = 0; k0 < K; k0 += 4096) {
            double t[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = k0 + j * 1024 + tid;
                t[j] = k < K ? Tm[k] : __builtin_huge_val();
            }
#pragma unroll
            for (int j = 0; j < 4; j++) cnt += t[j] <= bv + tol;
        }
        int nc;
        block_exclusive_scan<1024>(cnt, ws, &nc);
        if (nc <= 64) {
            __shared__ int gat[64];
            __shared__ int ng;
            if (tid == 0) ng = 0;
            __syncthreads();
            for (int k = tid; k < K; k += 1024)
                if (Tm[k] <= bv + tol) gat[atomicAdd(&ng, 1)] = k;
            __syncthreads();
            if (tid < nc) {
                const int me = gat[tid];
                int rank = 0;
                for (int d = 0; d < nc; d++) rank += gat[d] < me;
                cand[rank] = me;
            }
        } else {
            const int per = (K + 1023) / 1024;
            const int ka = min(K, tid * per), kb = min(K, ka + per);
            int c2 = 0;
            for (int k = ka; k < kb; k++) c2 += Tm[k] <= bv + tol;
            int nc2;
            int pos = block_exclusive_scan<1024>(c2, ws, &nc2);
            for (int k = ka; k < kb && pos < 64; k++)
                if (Tm[k] <= bv + tol) cand[pos++] = k;
        }
        __syncthreads();
        if (nc > 1) {
            const int n = nc < 64 ? nc : 64;
            const long lo = (long)(K * trim_lo), hi = (long)(K * trim_hi);
            float* buf = sortbuf + (size_t)p * npow2;
            double ev = __builtin_huge_val();
            int eb = -1;
            for (int c = 0; c < n; c++) {
                const int row = cand[c];
                bool dup = false;  // identical R vector as an earlier candidate => identical T
                for (int d = 0; d < c; d++) {
                    const int o = cand[d];
                    if (X[o] == X[row] && Y[o] == Y[row] && Z[o] == Z[row]) dup = true;
                }
                if (dup) continue;
                const double t = exact_row_mean(X, Y, Z, K, row, lo, hi, buf, npow2, sres);
                if (eb < 0 || t < ev) {
                    ev = t;
                    eb = row;
                }
            }
            if (nc > 64) r.near_ties = -nc;  // more candidates than re-scored: flagged
            else
                r.near_ties = n;
            if (eb >= 0) {
                best = eb;
                bv = ev;
            }
        }
    }
    if (tid == 0) {
        r.min_idx = best;
        r.min_dist = bv;
        r.R[0] = X[best];
        r.R[1] = Y[best];
        r.R[2] = Z[best];
        const float* T = tv + (size_t)p * 3 * stride + 3 * (size_t)best;
        r.T[0] = T[0];
        r.T[1] = T[1];
        r.T[2] = T[2];
        results[p] = r;
    }
}

__global__ void set_i32_kernel(int32_t* p, int32_t v) { *p = v; }
__global__ void set_i64x4_kernel(int64_t* p, int64_t a, int64_t b, int64_t c, int64_t d) {
    p[0] = a;
    p[1] = b;
    p[2] = c;
    p[3] = d;
}

}  // namespace

// ====================================================================== launchers =======
hipError_t launch_set_i32(int32_t* p, int32_t v, hipStream_t st) {
    ERP_LAUNCH(set_i32_kernel, dim3(1), dim3(1), 0, st, p, v);
    return hipGetLastError();
}

hipError_t launch_set_i64x4(int64_t* p, int64_t a, int64_t b, int64_t c, int64_t d,
                            hipStream_t st) {
    ERP_LAUNCH(set_i64x4_kernel, dim3(1), dim3(1), 0, st, p, a, b, c, d);
    return hipGetLastError();
}
void init_constants() {
    uint32_t red[30][31] = {};
    uint32_t v[31] = {};
    v[28] = 1;
    v[0] = 1;
    for (int d = 0; d < 30; d++) {
        for (int k = 0; k < 31; k++) red[d][k] = v[k];
        uint32_t nv[31];
        const uint32_t top = v[30];
        nv[0] = 0;
        for (int k = 1; k < 31; k++) nv[k] = v[k - 1];
        nv[28] += top;
        nv[0] += top;
        for (int k = 0; k < 31; k++) v[k] = nv[k];
    }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_red), red, sizeof(red));
    // x^(2^j) mod P by repeated squaring (x^d = x^(d-3) + x^(d-31) folds the product's top)
    uint32_t pw[kPow2][31] = {};
    pw[0][1] = 1;
    for (int j = 1; j < kPow2; j++) {
        uint32_t c[61] = {};
        for (int a = 0; a < 31; a++)
            for (int b = 0; b < 31; b++) c[a + b] += pw[j - 1][a] * pw[j - 1][b];
        for (int d = 60; d >= 31; d--) {
            c[d - 3] += c[d];
            c[d - 31] += c[d];
        }
        for (int k = 0; k < 31; k++) pw[j][k] = c[k];
    }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_pow2), pw, sizeof(pw));
}


hipError_t launch_bearings_direct(const erp_point2f* kl, const erp_point2f* kr, int32_t m,
                                  int32_t W, int32_t H, double* pts, hipStream_t st) {
    ERP_LAUNCH(bearings_direct_kernel, dim3((m + 255) / 256 + (m == 0)), dim3(256), 0, st, kl,
                       kr, m, W, H, pts);
    return hipGetLastError();
}

static int q_needed(int iters) {
    const int nwaves = (iters + 63) / 64;
    int kq = 0;
    while ((1 << kq) < nwaves) kq++;
    return kq;
}

// dynamic LDS above 64 KB is requested from the runtime first (hipFuncAttribute-
// MaxDynamicSharedMemorySize) -- at every such launch: the attribute is per device, contexts may
// live on any device of the process, and the call is cheap next to these launches
static hipError_t ensure_dyn_lds(const void* fn, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

hipError_t launch_jump_prep(const int32_t* counts, const BatchShape& sh, uint32_t* polyR,
                            uint32_t* polyQ, hipStream_t st) {
    // sample_frac is only used to skip pairs with sample_n < 1; pass a tiny positive value so
    // every pair with M >= 2 gets polynomials (the sampler decides on its own)
    ERP_LAUNCH(jump_prep_kernel, dim3(sh.n_pairs), dim3(1024), 0, st, counts, 1.0,
                       q_needed(sh.iters), polyR, polyQ);
    return hipGetLastError();
}

hipError_t launch_sampler(const int32_t* counts, const uint32_t* polyR, const uint32_t* polyQ,
                          const uint32_t* w0, const BatchShape& sh, double sample_frac,
                          const double* rtab, uint32_t* wins, uint32_t* selw, int32_t* flags,
                          hipStream_t st, int part) {
    const int nwaves = (sh.iters + 63) / 64;
    if (part == 0) {
        ERP_LAUNCH(sampler_window_kernel, dim3(nwaves, sh.n_pairs), dim3(64), 0, st, counts,
                           polyR, polyQ, w0, nwaves, sample_frac, wins);
    } else {
        // positions 0 .. max_s, rounded up to the LDS allocation granule (1280 B = 5 words on
        // gfx950, scripts/dev/lds_oob.hip) so that no word of the allocation goes uncleared
        const int nwords = (sh.max_s / 32 + 1 + 4) / 5 * 5;
        const size_t shmem = (size_t)nwords * 64 * sizeof(uint32_t);
        // The latency blocks (modes 2 / 3) where the launch leaves most SIMDs with at most one
        // wave (<= 1024 waves); sh.sampler_lat (ERP_OPT_SAMPLER_LAT) = 0 / 1 / 2 forces mode
        // 0 / 2 / 3
        const int lat = sh.sampler_lat >= 0 ? sh.sampler_lat
                                            : (long)nwaves * sh.n_pairs <= 1024 ? kSamplerLatMode : 0;
        const int mode = lat == 1 ? 2 : lat == 2 ? 3 : 0;
        // (s up to 16 383 at the 65 535-keypoint cap: 515 words x 256 B = 129 KB)
        const void* fns[4] = {(const void*)sampler_kernel<0>, nullptr,
                              (const void*)sampler_kernel<2>, (const void*)sampler_kernel<3>};
        const hipError_t le = ensure_dyn_lds(fns[mode], shmem);
        if (le != hipSuccess) return le;
#define ERP_SAMPLER_LAUNCH(M)                                                                  \
    ERP_LAUNCH(sampler_kernel<M>, dim3(nwaves, sh.n_pairs), dim3(64), shmem, st, counts, wins, \
               nwaves, sh.sel_words, sample_frac, rtab, selw, flags, nwords)
        // the split replay (sampler_split_kernel) where the launch has <= 256 workgroups of
        // 64 iterations (one pair at <= 16k iterations) and its 7 bitmaps fit the CU's LDS;
        // sh.sampler_split (ERP_OPT_SAMPLER_SPLIT) = 0 / 1 forces it off / on (when the LDS fits)
        const size_t split_lds = (size_t)(2 * kSplitG + 1) * nwords * 64 * sizeof(uint32_t);
        const bool split = sh.sampler_split != 0 && split_lds <= 150 * 1024 &&
                           (sh.sampler_split > 0 || (long)nwaves * sh.n_pairs <= 256);
        if (split) {
            const hipError_t se = ensure_dyn_lds((const void*)sampler_split_kernel, split_lds);
            if (se != hipSuccess) return se;
            ERP_LAUNCH(sampler_split_kernel, dim3(nwaves, sh.n_pairs), dim3(64 * (kSplitG + 1)),
                       split_lds, st, counts, wins, nwaves, sh.sel_words, sample_frac, rtab, selw,
                       flags, nwords);
            return hipGetLastError();
        }
        switch (mode) {
            case 2: ERP_SAMPLER_LAUNCH(2); break;
            case 3: ERP_SAMPLER_LAUNCH(3); break;
            default: ERP_SAMPLER_LAUNCH(0); break;
        }
#undef ERP_SAMPLER_LAUNCH
    }
    return hipGetLastError();
}

hipError_t launch_philox_sampler(const int32_t* counts, const BatchShape& sh, double sample_frac,
                                 uint32_t seed, uint64_t offset, int max_m, uint32_t* selw,
                                 int32_t* flags, hipStream_t st) {
    const int nwaves = (sh.iters + 63) / 64;
    // the bitmap is sized for the batch's largest possible M (max_m = max queries), capped at
    // one CU's LDS: 640 words = M <= 20 480; a pair with more matches gets ERP_INVALID_ARG
    const int nwords = std::min((max_m + 31) / 32, 640);
    const size_t shmem = (size_t)nwords * 64 * sizeof(uint32_t);
    const hipError_t le = ensure_dyn_lds((const void*)philox_sampler_kernel, shmem);
    if (le != hipSuccess) return le;
    ERP_LAUNCH(philox_sampler_kernel, dim3(nwaves, sh.n_pairs), dim3(64), shmem, st, counts,
                       sh.iters, nwaves, sh.sel_words, sample_frac, seed, offset, nwords, selw,
                       flags);
    return hipGetLastError();
}

bool build_magic_table(uint64_t* mtab, int n) {
    bool ok = true;
    for (int d = 0; d < n; d++) {
        if (d < 2) {
            mtab[d] = 0;
            continue;
        }
        int l = 0;
        while ((1 << l) < d) l++;  // ceil(log2 d), >= 1
        const uint64_t P = 1ull << (31 + l);
        const uint64_t m = (P + (uint64_t)d - 1) / (uint64_t)d;
        ok = ok && m < (1ull << 32) && m * (uint64_t)d >= P && m * (uint64_t)d - P <= (1ull << l);
        mtab[d] = m | ((uint64_t)(l - 1) << 32);
    }
    return ok;
}

// debug counters of ERP_LIP_VERIFY builds (0 = copied and reset; -1 = not a verify build;
// -2 = the copy failed)
int debug_lip_counters(uint32_t* out64) {
#if ERP_LIP_VERIFY
    if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_lip_dbg), 64 * 4) != hipSuccess) return -2;
    static const uint32_t zero[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lip_dbg), zero, 64 * 4) != hipSuccess) return -2;
    return 0;
#else
    (void)out64;
    return -1;
#endif
}

hipError_t launch_recip_table(int n, double* rtab, int32_t* bad, hipStream_t st) {
    ERP_LAUNCH(recip_table_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, rtab, bad);
    return hipGetLastError();
}

size_t gram_limbs_bytes(const BatchShape& sh) {
    return (size_t)sh.n_pairs * sh.sel_words * kGramN * 32;
}

hipError_t launch_gram_mfma(const int32_t* counts, const double* pts, const uint32_t* selw,
                            const BatchShape& sh, double sample_frac, int8_t* limbs,
                            double* gram, int32_t* samples, double* evec,
                            erp_hypothesis* hyps, double valid_abs, hipStream_t st) {
    const int nwaves = (sh.iters + 63) / 64;
    ERP_LAUNCH(gram_limbs_kernel, dim3(sh.sel_words, sh.n_pairs), dim3(256), 0, st, counts,
                       pts, sh.max_nq, sh.sel_words, limbs);
    // row tiles per wave: 2 once the wide blocks give every CU two of them (GramCfg);
    // sh.gram_tiles (ERP_OPT_GRAM_TILES) = 1 / 2 forces one
    const int wt_force = sh.gram_tiles;
    const int nhb2 = (sh.iters + GramCfg<2>::kIters - 1) / GramCfg<2>::kIters;
    const bool wide = wt_force == 2 || (wt_force != 1 && (long long)nhb2 * sh.n_pairs >= 2 * 256);
    if (wide) {
        ERP_LAUNCH(gram_mfma_kernel<2>, dim3(nhb2 * sh.n_pairs), dim3(64 * kGramWaves), 0, st, counts,
                   limbs, selw, sh.iters, nwaves, sh.sel_words, sample_frac, gram, nhb2, evec, hyps,
                   valid_abs);
    } else {
        const int nhb = (sh.iters + GramCfg<1>::kIters - 1) / GramCfg<1>::kIters;
        ERP_LAUNCH(gram_mfma_kernel<1>, dim3(nhb * sh.n_pairs), dim3(64 * kGramWaves), 0, st, counts,
                   limbs, selw, sh.iters, nwaves, sh.sel_words, sample_frac, gram, nhb, evec, hyps,
                   valid_abs);
    }
    if (samples)
        ERP_LAUNCH(samples_kernel, dim3(nwaves, sh.n_pairs), dim3(64), 0, st, counts, selw,
                           sh.iters, nwaves, sh.sel_words, sh.idx_stride, sample_frac, samples);
    return hipGetLastError();
}

hipError_t launch_gram_all(const double* pts, int32_t m, double* gram, hipStream_t st) {
    ERP_LAUNCH(gram_all_kernel, dim3(1), dim3(256), 0, st, pts, m, gram);
    return hipGetLastError();
}

hipError_t launch_eigen(const int32_t* counts, const double* gram, const BatchShape& sh,
                        double sample_frac, double valid_abs, double* evec, erp_hypothesis* hyps,
                        hipStream_t st, int fused, bool want_e, float* hl, int32_t* wsum) {
    dim3 grid((sh.iters + 63) / 64, sh.n_pairs);
    // small batches with lite estimates: the leftovers inside the estimate launch
    const bool rest_inline = fused == 1 && hl && (size_t)grid.x * grid.y <= 1024;
    // fused >= 1: gram_mfma_kernel ran the inverse iteration (s >= 9) already; fused == 2: and
    // the estimate of its settled lanes, the fallback / thin kernels estimate their own lanes
    erp_hypothesis* own = fused == 2 ? hyps : nullptr;
    if (!fused) {
        ERP_LAUNCH(eigen_kernel<false>, grid, dim3(64), 0, st, counts, gram, sh.iters,
                           sample_frac, evec, nullptr, valid_abs);
        ERP_LAUNCH(eigen_fallback_kernel, grid, dim3(64), 0, st, counts, gram, sh.iters,
                           sample_frac, evec, own, valid_abs);
        // (M is only known on the device: the thin instantiation returns at once for s >= 9)
        ERP_LAUNCH(eigen_kernel<true>, grid, dim3(64), 0, st, counts, gram, sh.iters,
                           sample_frac, evec, own, valid_abs);
    } else if (!rest_inline) {  // the Gram kernel ran the common inverse iteration: fallback
        // + thin in one launch
        ERP_LAUNCH(eigen_rest_kernel, grid, dim3(64), 0, st, counts, gram, sh.iters,
                           sample_frac, evec, own, valid_abs);
    }
    if (fused != 2 && hl && rest_inline)
        ERP_LAUNCH(estimate_lite_kernel<true>, grid, dim3(64), 0, st, counts, evec, sh.iters,
                           sample_frac, valid_abs, hl, wsum, gram);
    else if (fused != 2 && hl)
        ERP_LAUNCH(estimate_lite_kernel<false>, grid, dim3(64), 0, st, counts, evec, sh.iters,
                           sample_frac, valid_abs, hl, wsum, gram);
    else if (fused != 2)
        ERP_LAUNCH(estimate_kernel, grid, dim3(64), 0, st, counts, evec, sh.iters,
                           sample_frac, valid_abs, hyps, (int)want_e);
    return hipGetLastError();
}

size_t hyp_lite_bytes(const BatchShape& sh) {
    const size_t P = sh.n_pairs, nw = (sh.iters + 63) / 64;
    return P * 9 * sh.iters * sizeof(float) + P * nw * 8 * sizeof(int32_t);
}

hipError_t launch_valid_place(const int32_t* counts, const float* hl, const int32_t* wsum,
                              const BatchShape& sh, double sample_frac, float* rv, float* tv,
                              int32_t* kcount, float* rv_aos, float* dscale, float* edges,
                              hipStream_t st) {
    dim3 grid((sh.iters + 1023) / 1024, sh.n_pairs);
    ERP_LAUNCH(valid_place_kernel, grid, dim3(1024), 0, st, counts, hl, sh.iters,
                       sample_frac, wsum, (sh.iters + 63) / 64, rv, tv, kcount, rv_aos, dscale,
                       edges);
    return hipGetLastError();
}

size_t inlier_scratch_bytes(const BatchShape& sh) {
    const size_t P = sh.n_pairs, I = sh.iters;
    const size_t mpad = (size_t)(sh.max_nq + kInlierChunk - 1) / kInlierChunk * kInlierChunk;
    return P * I * 9 * 8 + P * I * 16 * 4 + P * 9 * mpad * 4;
}

hipError_t launch_inliers(const int32_t* counts, const double* pts, const BatchShape& sh,
                          double sample_frac, float thr, void* scratch, erp_hypothesis* hyps,
                          hipStream_t st) {
    const size_t P = sh.n_pairs, I = sh.iters;
    const int mpad = (sh.max_nq + kInlierChunk - 1) / kInlierChunk * kInlierChunk;
    double* ec64 = (double*)scratch;
    float* ec32 = (float*)(ec64 + P * I * 9);
    float* u32 = ec32 + P * I * 16;
    const double t = (double)thr, d = (double)kInlierBand;
    const float lo = t > d ? (float)(t - d) : 0.0f;  // (|res32| < 0 never holds)
    const float hi = (float)(t + d);
    const dim3 g((sh.iters + 63) / 64, sh.n_pairs);
    ERP_LAUNCH(inlier_prep_kernel, g, dim3(64), 0, st, counts, (const erp_hypothesis*)hyps,
                       sh.iters, sample_frac, ec64, ec32);
    ERP_LAUNCH(inlier_points_kernel, dim3(mpad / 256, sh.n_pairs), dim3(256), 0, st, counts,
                       pts, sh.max_nq, mpad, u32);
    ERP_LAUNCH(inlier_count_kernel, g, dim3(64), 0, st, counts, (const float*)u32,
                       (const float*)ec32, (const double*)ec64, pts, sh.max_nq, mpad, sh.iters,
                       sample_frac, lo, hi, t, hyps);
    return hipGetLastError();
}

size_t valid_chunk_bytes(const BatchShape& sh) {
    return (size_t)sh.n_pairs * ((sh.iters + 1023) / 1024) * 8 * sizeof(int32_t);
}

hipError_t launch_valid_compact(const int32_t* counts, const erp_hypothesis* hyps,
                                const BatchShape& sh, double sample_frac, int32_t* vchunk,
                                float* rv, float* tv, int32_t* kcount, float* rv_aos,
                                float* dscale, hipStream_t st) {
    dim3 grid((sh.iters + 1023) / 1024, sh.n_pairs);
    ERP_LAUNCH(valid_count_kernel, grid, dim3(1024), 0, st, counts, hyps, sh.iters,
                       sample_frac, vchunk);
    ERP_LAUNCH(valid_scatter_kernel, grid, dim3(1024), 0, st, counts, hyps, sh.iters,
                       sample_frac, vchunk, rv, tv, kcount, rv_aos, dscale);
    return hipGetLastError();
}

hipError_t launch_consensus_input(const float* rvec, const float* tvec, int K, int stride, float* rv,
                                  float* tv, int32_t* kcount, float* dscale, int32_t* flags,
                                  hipStream_t st) {
    ERP_LAUNCH(consensus_input_kernel, dim3(1), dim3(1024), 0, st, rvec, tvec, K, stride, rv,
                       tv, kcount, dscale, flags);
    return hipGetLastError();
}

// [P][2][kNB] first-pass edges, [P][2][kNB] zoom edges, [P] zoom grids
size_t consensus_edges_bytes(int n_pairs) {
    return (size_t)n_pairs * 4 * kNB * sizeof(float) + (size_t)n_pairs * sizeof(int32_t);
}

hipError_t launch_consensus_zoom(const int32_t* kcount, const float* rv, const float* dscale,
                                 float* edges, const BatchShape& sh, double trim_lo,
                                 double trim_hi, double* lb, double* ub, const int32_t* bsel,
                                 const int32_t* surv, int32_t* nsurv, int32_t* zsel, int level,
                                 hipStream_t st) {
    const int P = sh.n_pairs, stride = 2 * sh.iters;
    float* edz = edges + (size_t)P * 2 * kNB;
    int32_t* zb = reinterpret_cast<int32_t*>(edges + (size_t)P * 4 * kNB);
    int32_t* uoff = nsurv + 2 * P;  // free until the refine pass (launch_consensus_refine)
    if (level == 1)
        ERP_LAUNCH((consensus_zoom_prep_kernel<6, kMantBits>), dim3(P), dim3(256), 0, st,
                           kcount, dscale, surv, (const int32_t*)nsurv, bsel, 1, stride, trim_lo,
                           trim_hi, zb, edz);
    else  // the level-1 windows (zsel) -> the 256-per-binade grid
        ERP_LAUNCH((consensus_zoom_prep_kernel<8, 6>), dim3(P), dim3(256), 0, st, kcount,
                           dscale, surv, (const int32_t*)nsurv, (const int32_t*)zsel, 0, stride,
                           trim_lo, trim_hi, zb, edz);
    ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, (const int32_t*)nsurv, P,
                       kBoundRows, kZoomMin, uoff);
    const int max_units = P * ((stride + kBoundRows - 1) / kBoundRows);
    if (level == 1)
        ERP_LAUNCH(consensus_zoom_kernel<6>, dim3(max_units), dim3(256), 0, st, kcount, rv,
                           (const float*)edz, (const int32_t*)zb, stride, trim_lo, trim_hi, lb,
                           ub, surv, (const int32_t*)nsurv, (const int32_t*)uoff, P, zsel, 1,
                           dscale, (int32_t*)nullptr);
    else
        ERP_LAUNCH(consensus_zoom_kernel<8>, dim3(max_units), dim3(256), 0, st, kcount, rv,
                           (const float*)edz, (const int32_t*)zb, stride, trim_lo, trim_hi, lb,
                           ub, surv, (const int32_t*)nsurv, (const int32_t*)uoff, P, zsel, 1,
                           dscale, (int32_t*)nullptr);
    return hipGetLastError();
}

// the pruning references' scratch: [P][cap] float4, lU [P] doubles, lcnt [P] ints, then the
// second-stage reference list [P][stride] ints and its counts [P]
// then the gradient references: gref [P][gcap][2] float4, gsel [P][gcap], gcnt [P], goff [P + 1]
// (>= the stage-1 references; the second stage's -- a quarter of L1 -- are capped at it)
// then the flat gate [P] ints (consensus_flat_gate_kernel) and the refine pass's rank-key hint
// candidates [P][kHintCands] (consensus_hint_kernel)
static int grad_cap(int stride) { return stride / 4 + 64; }
size_t lipref_bytes(int n_pairs, int stride) {
    const size_t gcap = grad_cap(stride);
    return (size_t)n_pairs * lipref_cap(stride) * sizeof(float4) + (size_t)n_pairs * 16 +
           (size_t)n_pairs * stride * 4 + 64 + (size_t)n_pairs * gcap * 2 * sizeof(float4) +
           (size_t)n_pairs * gcap * 4 + (size_t)n_pairs * 8 + 128 +
           (size_t)n_pairs * 4 + 16 + (size_t)n_pairs * kHintCands * sizeof(HintCand);
}
struct LipRefViews {
    float4* ref;
    double* U;
    int32_t* cnt;
    int32_t* r2cnt;
    int32_t* r2list;
    int cap;
    float4* gref;
    int32_t* gsel;
    int32_t* gcnt;
    int32_t* goff;
    int gcap;
    int32_t* nflat;
    HintCand* hcand;
};
static LipRefViews lipref_views(void* base, int n_pairs, int stride) {
    LipRefViews v;
    v.cap = lipref_cap(stride);
    v.ref = reinterpret_cast<float4*>(base);
    v.U = reinterpret_cast<double*>(v.ref + (size_t)n_pairs * v.cap);
    v.cnt = reinterpret_cast<int32_t*>(v.U + n_pairs);
    v.r2cnt = v.cnt + n_pairs;
    v.r2list = v.r2cnt + n_pairs;
    v.gcap = grad_cap(stride);
    uintptr_t gb = reinterpret_cast<uintptr_t>(v.r2list + (size_t)n_pairs * stride) + 64;
    gb = (gb + 15) & ~(uintptr_t)15;
    v.gref = reinterpret_cast<float4*>(gb);
    v.gsel = reinterpret_cast<int32_t*>(v.gref + (size_t)n_pairs * v.gcap * 2);
    v.gcnt = v.gsel + (size_t)n_pairs * v.gcap;
    v.goff = v.gcnt + n_pairs;
    v.nflat = v.goff + n_pairs + 1;
    uintptr_t cb = reinterpret_cast<uintptr_t>(v.nflat + n_pairs);
    v.hcand = reinterpret_cast<HintCand*>((cb + 15) & ~(uintptr_t)15);
    return v;
}

hipError_t launch_consensus_bounds(const int32_t* kcount, const float* rv, const float* dscale,
                                   float* edges, const BatchShape& sh, double trim_lo,
                                   double trim_hi, double* lb, double* ub, int32_t* bsel,
                                   int shard, int nshards, int32_t* rlist, int32_t* rcount,
                                   int32_t* zsel, int lip2, int32_t* list2, void* lipref,
                                   int lipg, int flat_pct, int use_hint, hipStream_t st,
                                   bool edges_ready) {
    const float gfac = kLipGFac;
    if (!edges_ready)
        ERP_LAUNCH(consensus_edges_kernel, dim3(sh.n_pairs), dim3(256), 0, st, dscale, edges);
    const int stride = 2 * sh.iters;
    if (!rlist) {  // every row of the shard (rcount = -1: no pre-pruning)
        if (rcount) {
            const hipError_t me = hipMemsetAsync(rcount, 0xFF, sizeof(int32_t) * sh.n_pairs, st);
            if (me != hipSuccess) return me;
        }
        const int rows = (stride + nshards - 1) / nshards + 1;  // >= any shard's rows
        dim3 grid((rows + kBoundRows - 1) / kBoundRows, sh.n_pairs);
        ERP_LAUNCH(consensus_bounds_kernel, grid, dim3(256), 0, st, kcount, rv, dscale,
                           edges, stride, trim_lo, trim_hi, lb, ub, bsel, shard, nshards, 1);
        return hipGetLastError();
    }
    // reference rows, Lipschitz pre-pruning, then the rows it kept -- within the row shard
    // (nshards > 1: configs[4]'s consensus split over ranks; each rank's rows only)
    const int srows = (stride + nshards - 1) / nshards + 1;  // >= any shard's rows
    const int nref = (srows + kLipStep - 1) / kLipStep;
    dim3 g1((nref + kBoundRows - 1) / kBoundRows, sh.n_pairs);
    ERP_LAUNCH(consensus_bounds_kernel, g1, dim3(256), 0, st, kcount, rv, dscale, edges,
                       stride, trim_lo, trim_hi, lb, ub, bsel, shard, nshards, kLipStep);
    const int P = sh.n_pairs;
    const LipRefViews lr = lipref_views(lipref, P, stride);
    const bool two = lip2 && list2;  // second pre-pruning stage
    // (the list counters rcount and r2cnt are reset by the references kernel)
    ERP_LAUNCH(consensus_lip_refs_kernel, dim3(P), dim3(256), 0, st, kcount, rv, stride,
                       trim_lo, trim_hi, (const double*)lb, (const double*)ub,
                       (const int32_t*)nullptr, (const int32_t*)nullptr, kLipStep, shard, nshards,
                       (const int32_t*)nullptr, lr.ref, lr.U, lr.cnt, lr.cap,
                       (const int32_t*)nullptr, rcount, two ? lr.r2cnt : (int32_t*)nullptr);
    if (lipg & 1) {  // the central references' G (convexity-augmented pruning)
        ERP_LAUNCH(consensus_grad_select_kernel, dim3(P), dim3(256), 0, st, kcount, stride,
                           (const double*)lb, (const double*)ub, (const int32_t*)bsel, kLipStep,
                           shard, nshards, (const int32_t*)nullptr, (const int32_t*)nullptr,
                           (const double*)lr.U, gfac, lr.gsel, lr.gcnt, lr.gcap);
        ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, (const int32_t*)lr.gcnt,
                           P, 1, 0, lr.goff);
        // (2048 blocks whatever the batch: one pair of configs[4] has ~1000 central references
        // of K ~ 89k columns each; the former min(64 P, 2048) gave it 64 blocks)
        ERP_LAUNCH(consensus_grad_kernel, dim3(kGradBlocks), dim3(256), 0, st,
                           kcount, rv, dscale, stride, trim_lo, trim_hi, (const double*)lb,
                           (const int32_t*)bsel, (const int32_t*)lr.gsel, (const int32_t*)lr.goff,
                           P, lr.gcap, lr.gref);
    }
    ERP_LAUNCH(consensus_lipschitz_kernel, dim3((srows + 511) / 512, P), dim3(256), 0,
                       st, kcount, rv, stride, lb, ub, (const int32_t*)nullptr,
                       (const int32_t*)nullptr, rlist, stride, rcount, shard, nshards, kLipStep,
                       (const float4*)lr.ref, (const double*)lr.U, (const int32_t*)lr.cnt,
                       lr.cap, two ? lr.r2list : nullptr, two ? lr.r2cnt : nullptr,
                       (lipg & 1) ? (const float4*)lr.gref : nullptr, (const int32_t*)lr.gcnt,
                       lr.gcap);
    int32_t* uoff = rcount + P;  // [n_pairs + 1] after the counts
    if (flat_pct > 0 && nshards == 1) {
        // flat pairs: refine the first-stage references, then re-run the first stage
        ERP_LAUNCH(consensus_flat_gate_kernel, dim3((P + 255) / 256), dim3(256), 0, st,
                           kcount, rcount, two ? lr.r2cnt : nullptr, P, flat_pct, trim_lo,
                           trim_hi, lr.nflat);
        const HintCand* hint = nullptr;
        if (use_hint) {
            ERP_LAUNCH(consensus_hint_kernel, dim3(P, kHintCands), dim3(256), 0, st,
                               kcount, rv, stride, trim_lo, trim_hi, (const int32_t*)nullptr,
                               (const int32_t*)lr.nflat, kLipStep, 0, (const double*)ub, lr.hcand);
            hint = lr.hcand;
        }
        ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, (const int32_t*)lr.nflat,
                           P, kRefineRows * kLipStep, kRefineMin, uoff);
        ERP_LAUNCH(consensus_refine_kernel, dim3(2048), dim3(256), 0, st, kcount, rv,
                           dscale, stride, trim_lo, trim_hi, (const int32_t*)nullptr,
                           (const int32_t*)lr.nflat, (const int32_t*)bsel, lb, ub,
                           (const int32_t*)nullptr, stride, (const int32_t*)nullptr, kLipStep,
                           hint, (const int32_t*)uoff, P);
        ERP_LAUNCH(consensus_lip_refs_kernel, dim3(P), dim3(256), 0, st, kcount, rv, stride,
                           trim_lo, trim_hi, (const double*)lb, (const double*)ub,
                           (const int32_t*)nullptr, (const int32_t*)nullptr, kLipStep, 0, 1,
                           (const int32_t*)nullptr, lr.ref, lr.U, lr.cnt, lr.cap,
                           (const int32_t*)lr.nflat);
        ERP_LAUNCH(consensus_lipschitz_kernel, dim3((srows + 511) / 512, P), dim3(256), 0,
                           st, kcount, rv, stride, lb, ub, (const int32_t*)nullptr,
                           (const int32_t*)nullptr, rlist, stride, rcount, 0, 1, kLipStep,
                           (const float4*)lr.ref, (const double*)lr.U, (const int32_t*)lr.cnt,
                           lr.cap, two ? lr.r2list : nullptr, two ? lr.r2cnt : nullptr,
                           (const float4*)nullptr, (const int32_t*)lr.gcnt, lr.gcap,
                           (const int32_t*)lr.nflat);
    }
    const int32_t* blist = rlist;
    const int32_t* bcount = rcount;
    if (two) {
        // second stage: the L1 rows with is_ref2 (listed apart by the first stage) on the fine
        // grid, the other L1 rows tested against them; the survivors (list2, counts after the
        // unit prefix) get the coarse pass
        float* edz = edges + (size_t)P * 2 * kNB;
        int32_t* zb = reinterpret_cast<int32_t*>(edges + (size_t)P * 4 * kNB);
        int32_t* n2 = uoff + P + 1;
        ERP_LAUNCH(consensus_ref2_prep_kernel, dim3(P), dim3(256), 0, st, kcount, dscale,
                           (const double*)ub, (const int32_t*)bsel, (const int32_t*)rcount, stride,
                           trim_lo, trim_hi, shard, nshards, zb, edz);
        ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st,
                           (const int32_t*)lr.r2cnt, P, kBoundRows, 0, uoff);
        const int units2 = P * ((stride / kLip2Step + 1 + kBoundRows - 1) / kBoundRows);
        ERP_LAUNCH(consensus_zoom_kernel<6>, dim3(units2), dim3(256), 0, st, kcount, rv,
                           (const float*)edz, (const int32_t*)zb, stride, trim_lo, trim_hi, lb, ub,
                           (const int32_t*)lr.r2list, (const int32_t*)lr.r2cnt,
                           (const int32_t*)uoff, P, zsel, 1, dscale, bsel);
        // (n2 and nfb = n2 + P reset by the references kernel)
        ERP_LAUNCH(consensus_lip_refs_kernel, dim3(P), dim3(256), 0, st, kcount, rv,
                           stride, trim_lo, trim_hi, (const double*)lb, (const double*)ub,
                           (const int32_t*)lr.r2list, (const int32_t*)lr.r2cnt, 1, shard,
                           nshards, (const int32_t*)zb, lr.ref, lr.U, lr.cnt, lr.cap,
                           (const int32_t*)nullptr, n2, n2 + P);
        if (lipg & 2) {  // G of the central second-stage references (fine bounds)
            ERP_LAUNCH(consensus_grad_select_kernel, dim3(P), dim3(256), 0, st, kcount,
                               stride, (const double*)lb, (const double*)ub, (const int32_t*)bsel,
                               1, 0, 1, (const int32_t*)lr.r2list, (const int32_t*)lr.r2cnt,
                               (const double*)lr.U, gfac, lr.gsel, lr.gcnt, lr.gcap);
            ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st,
                               (const int32_t*)lr.gcnt, P, 1, 0, lr.goff);
            ERP_LAUNCH(consensus_grad_kernel, dim3(kGradBlocks), dim3(256), 0,
                               st, kcount, rv, dscale, stride, trim_lo, trim_hi, (const double*)lb,
                               (const int32_t*)bsel, (const int32_t*)lr.gsel,
                               (const int32_t*)lr.goff, P, lr.gcap, lr.gref);
        }
        ERP_LAUNCH(consensus_lipschitz2_kernel, dim3((srows + 511) / 512, P), dim3(256), 0,
                           st, kcount, rv, stride, lb, ub, (const int32_t*)rlist,
                           (const int32_t*)rcount, (const int32_t*)zb, (const int32_t*)bsel, list2,
                           n2, n2 + P, (const float4*)lr.ref, (const double*)lr.U,
                           (const int32_t*)lr.cnt, lr.cap,
                           (lipg & 2) ? (const float4*)lr.gref : nullptr, (const int32_t*)lr.gcnt,
                           lr.gcap);
        ERP_LAUNCH(consensus_ref2_count_kernel, dim3((P + 255) / 256), dim3(256), 0, st, P,
                           (const int32_t*)zb, (const int32_t*)lr.r2cnt, (const int32_t*)n2,
                           (const int32_t*)(n2 + P), rcount);
        blist = list2;
        bcount = n2;
    }
    ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, bcount, P, kBoundRows, 0,
                       uoff);
    // one block per unit of the longest possible lists: the live units come first in dispatch
    // order, the trailing blocks exit after one load
    const int max_units = P * ((stride + kBoundRows - 1) / kBoundRows);
    ERP_LAUNCH(consensus_bounds_list_kernel, dim3(max_units), dim3(256), 0, st,
                       kcount, rv, dscale, edges, stride, trim_lo, trim_hi, lb, ub, bsel, blist,
                       bcount, (const int32_t*)uoff, P);
    return hipGetLastError();
}

hipError_t launch_consensus_select(const int32_t* kcount, const double* lb, const double* ub,
                                   const BatchShape& sh, double trim_lo, double trim_hi,
                                   int32_t* surv, int32_t* nsurv, double* tmean, int again,
                                   hipStream_t st) {
    ERP_LAUNCH(consensus_select_kernel, dim3(sh.n_pairs), dim3(1024), 0, st, kcount, lb, ub,
                       2 * sh.iters, trim_lo, trim_hi, surv, nsurv, tmean, again);
    return hipGetLastError();
}

hipError_t launch_consensus_refine(const int32_t* kcount, const float* rv, const float* dscale,
                                   const BatchShape& sh, double trim_lo, double trim_hi,
                                   const int32_t* surv, const int32_t* nsurv, const int32_t* bsel,
                                   double* lb, double* ub, int32_t* list2, void* lipref,
                                   int use_hint, hipStream_t st) {
    // scratch after nsurv[n_pairs] and the bounds-list counts[n_pairs]: the unit prefix
    // [n_pairs + 1], then the counts of list2 [n_pairs]
    const int P = sh.n_pairs, stride = 2 * sh.iters, l2stride = sortbuf_len(sh.iters);
    int32_t* uoff = const_cast<int32_t*>(nsurv) + 2 * P;
    int32_t* n2 = uoff + P + 1;
    const LipRefViews lr = lipref_views(lipref, P, stride);
    // (0) the rank-key hint of pairs with > kRefineMin survivors (use_hint = 0: none)
    const HintCand* hint = nullptr;
    if (use_hint) {
        // (pairs with <= kHintManyRows survivors -- a one-cluster pair after the zoom has ~20 --
        // keep the default windows: the hint's K-column passes would cost more than they save)
        ERP_LAUNCH(consensus_hint_kernel, dim3(P, kHintCands), dim3(256), 0, st, kcount,
                           rv, stride, trim_lo, trim_hi, surv, nsurv, 1, kHintManyRows,
                           (const double*)ub, lr.hcand);
        hint = lr.hcand;
    }
    // (A) the reference survivors (every kRefStep-th) of pairs with > kRefineMin survivors
    ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, nsurv, P,
                       kRefineRows * kRefStep, kRefineMin, uoff);
    ERP_LAUNCH(consensus_refine_kernel, dim3(2048), dim3(256), 0, st, kcount, rv, dscale,
                       stride, trim_lo, trim_hi, surv, nsurv, bsel, lb, ub, surv, stride,
                       (const int32_t*)nullptr, kRefStep, hint, (const int32_t*)uoff, P);
    // (B) Lipschitz pruning of the other survivors against the refined references
    // (n2 reset by the references kernel)
    ERP_LAUNCH(consensus_lip_refs_kernel, dim3(P), dim3(256), 0, st, kcount, rv, stride,
                       trim_lo, trim_hi, (const double*)lb, (const double*)ub, surv, nsurv,
                       kRefStep, 0, 1, (const int32_t*)nullptr, lr.ref, lr.U, lr.cnt, lr.cap,
                       (const int32_t*)nullptr, n2);
    ERP_LAUNCH(consensus_lipschitz_kernel, dim3((stride + 511) / 512, P), dim3(256), 0, st,
                       kcount, rv, stride, lb, ub, surv, nsurv, list2, l2stride, n2, 0, 1,
                       kRefStep, (const float4*)lr.ref, (const double*)lr.U,
                       (const int32_t*)lr.cnt, lr.cap, (int32_t*)nullptr, (int32_t*)nullptr,
                       (const float4*)nullptr, (const int32_t*)nullptr, 0);
    // (C) the survivors the references did not prune
    ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, (const int32_t*)n2, P,
                       kRefineRows, 0, uoff);
    ERP_LAUNCH(consensus_refine_kernel, dim3(2048), dim3(256), 0, st, kcount, rv, dscale,
                       stride, trim_lo, trim_hi, surv, nsurv, bsel, lb, ub, (const int32_t*)list2,
                       l2stride, (const int32_t*)n2, 1, hint, (const int32_t*)uoff, P);
    return hipGetLastError();
}

hipError_t launch_consensus_rows(const int32_t* kcount, const float* rv, const float* dscale,
                                 const BatchShape& sh, double trim_lo, double trim_hi,
                                 const int32_t* surv, const int32_t* nsurv, const int32_t* bsel,
                                 double* tmean, hipStream_t st) {
    int32_t* uoff = const_cast<int32_t*>(nsurv) + 2 * sh.n_pairs;  // as in launch_consensus_refine
    if (sh.n_pairs <= 16)
        uoff = nullptr;  // (consensus_rows_kernel walks the counts itself: one launch fewer)
    else
        ERP_LAUNCH(list_prefix_kernel, dim3(1), dim3(1024), 0, st, nsurv, sh.n_pairs, 1, 0,
                           uoff);
    ERP_LAUNCH(consensus_rows_kernel, dim3(2048), dim3(256), 0, st, kcount, rv, dscale,
                       2 * sh.iters, trim_lo, trim_hi, surv, nsurv, bsel, tmean,
                       (const int32_t*)uoff, sh.n_pairs);
    return hipGetLastError();
}

int sortbuf_len(int iters) {
    int p = 1;
    while (p < 2 * iters) p <<= 1;
    return p;
}

hipError_t launch_consensus_final(const int32_t* counts, const int32_t* kcount, const float* rv,
                                  const float* tv, const double* tmean, const int32_t* flags,
                                  const int32_t* nsurv, const int32_t* nbin, const BatchShape& sh,
                                  double sample_frac, double trim_lo, double trim_hi,
                                  float* sortbuf, erp_pair_result* results, hipStream_t st) {
    ERP_LAUNCH(consensus_final_kernel, dim3(sh.n_pairs), dim3(1024), 0, st, counts, kcount,
                       rv, tv, tmean, flags, nsurv, nbin, 2 * sh.iters, sortbuf_len(sh.iters), sample_frac,
                       trim_lo, trim_hi, sortbuf, results);
    return hipGetLastError();
}

}  // namespace erp
