// erp_kernels.hpp -- launchers of the gfx950 kernels (matcher.hip: the matcher; kernels.hip:
// the rest of the hot path).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/erp_match.h"

namespace erp {

constexpr int kDim = 64;          // SURF descriptor length (extended=false)
constexpr int kMaxQ = 24;         // jump polynomials x^(64(M-1)2^k): waves per pair < 2^24
constexpr int kPolyWords = 31;    // glibc TYPE_3 degree
#ifndef ERP_CAND_SLOTS
#define ERP_CAND_SLOTS 28
#endif
constexpr int kCandSlots = ERP_CAND_SLOTS;    // matcher: tiles with candidate rows kept per (query, train
                                  // chunk, lane half) (more: exact sweep of the chunk)

// the batch pipeline's gather + bearings (bearings_from_matches_kernel's work), done by
// knn2_merge_kernel as it places each match (src/spherical_surf.cpp:155-162 +
// src/eight_point.cpp:163-186): pts[p][max_nq + 1][6] (the last row the zero pad of the Gram
// batches), optional valid_key_left / right
struct BearingOut {
    const erp_point2f* kp_l;
    const erp_point2f* kp_r;
    const int32_t* width;
    const int32_t* height;
    double* pts;
    erp_point2f* key_l;
    erp_point2f* key_r;
};
struct Top2 {                     // partial k=2 result of one train chunk for one query
    float d0;                     // best squared distance
    int32_t j0;                   // its train index (lowest index among ties)
    float d1;                     // second squared distance
};

// scratch the pipeline needs for one batch (all device pointers, sized by the context)
struct Workspace {
    Top2* part;                   // [pairs][max_nq] exact k=2 per query
    erp_dmatch* matches;          // [pairs][max_nq]
    int32_t* counts;              // [pairs] M
    double* pts;                  // [pairs][max_nq + 1][6] bearings (l, r); last row = 0
    uint32_t* polyR;              // [pairs][65][31]  x^(l(M-1)) mod P
    uint32_t* polyQ;              // [pairs][kMaxQ][31]
    uint32_t* sel;                // [pairs][waves][sel_words][64] sample selection bitmaps
    double* gram;                 // [pairs][iters][36]
    erp_hypothesis* hyps;         // [pairs][iters]
    float* rv;                    // [pairs][3][2*iters] valid R (SoA)
    float* tv;                    // [pairs][2*iters][3] their T
    int32_t* kcount;              // [pairs]
    double* tmean;                // [pairs][2*iters]
    float* sortbuf;               // [pairs][2*iters] exact tie resolution scratch
    int32_t* flags;               // [pairs] internal error flags
};

struct BatchShape {
    int n_pairs;
    int max_nq, max_nt;
    int fchunks, fchunk_len;      // train chunks of the matcher's MFMA filter
    int xchunks, xchunk_len;      // train chunks of the exact VALU sweep (multiples of 128)
    int iters;
    int max_s;                    // (int)(max_nq * sample_frac)
    int idx_stride;               // entries of one hypothesis in the debug samples output
    int sel_words;                // 31-step selection words per hypothesis (>= (M-1)/31 + 1)
    // route options (erp_ctx_set_option; -1 / 0 = automatic): the sampler's block kind and split
    // replay, the Gram kernel's row tiles per wave
    int sampler_lat = -1, sampler_split = -1, gram_tiles = 0;
};

hipError_t launch_set_i32(int32_t* p, int32_t v, hipStream_t st);  // (values via kernel args:
hipError_t launch_set_i64x4(int64_t* p, int64_t a, int64_t b, int64_t c, int64_t d,  // no host
                            hipStream_t st);                                       // lifetime)
void init_constants();            // reduction table for the jump polynomials (once per device)

// matcher: knn2_filter (train rows split to bf16, then ONE MFMA pass: per-(query, chunk) top-2
// upper bounds pu, and per (query, chunk, lane half) up to kCandSlots tiles that may hold
// candidates: the tile and its 16 bounds of the lane's rows; counts in ccount), rescore (exact
// Top2 per (query, chunk) of the stored rows under the final bound into
// part[pairs][fchunks][max_nq]), merge (ratio + compaction).  split = scratch of
// knn2_split_bytes(sh) (bf16 rows, norms, per-pair max norm); cand = knn2_cand_bytes(sh).
size_t knn2_split_bytes(const BatchShape& sh);
size_t knn2_cand_bytes(const BatchShape& sh);
// (ovf: the rescore's overflow scratch below; its counter ovf[0] is zeroed here)
hipError_t launch_knn2_filter(const float* desc_q, const float* desc_t, const int64_t* off_q,
                              const int64_t* off_t, const BatchShape& sh, void* split,
                              float2* pu, int32_t* ccount, void* cand, hipStream_t st,
                              int32_t* ovf, int32_t* flags);  // flags [n_pairs] zeroed (may be null)
// ovf = scratch of 4 + 12 * n_pairs * max_nq * fchunks bytes: overflowed (pair, query, chunk)
// for the exact sweep (counter zeroed by the launch_knn2_filter before it)
hipError_t launch_knn2_rescore(const float* desc_q, const float* desc_t, const int64_t* off_q,
                               const int64_t* off_t, const BatchShape& sh, void* split,
                               const float2* pu, const int32_t* ccount, void* cand, Top2* part,
                               int32_t* ovf, float ratio, hipStream_t st);
// exact sweep on packed FP32 VALU (no MFMA filter): per-(chunk, query) exact k=2 into
// xpart[pairs][xchunks][max_nq]
hipError_t launch_knn2_exact(const float* desc_q, const float* desc_t, const int64_t* off_q,
                             const int64_t* off_t, const BatchShape& sh, Top2* xpart,
                             hipStream_t st);
// per-chunk partials part[pairs][chunks][max_nq] -> one Top2 per query out[pairs][max_nq]
hipError_t launch_knn2_fold(const Top2* part, const int64_t* off_q, const int64_t* off_t,
                            const BatchShape& sh, int chunk_len, int chunks, Top2* out,
                            hipStream_t st);
// fold of per-chunk partials part[pairs][chunks][max_nq] (chunk c = train rows
// [c*chunk_len, (c+1)*chunk_len)), ratio test, compaction
size_t knn2_merge_scratch_bytes(const BatchShape& sh);
hipError_t launch_knn2_merge(const Top2* part, const int64_t* off_q, const int64_t* off_t,
                             const BatchShape& sh, int chunk_len, int chunks, float ratio,
                             erp_dmatch* matches, int32_t* counts, int32_t* flags,
                             int32_t* bcount, hipStream_t st,
                             const BearingOut* bo = nullptr);
hipError_t launch_bearings_direct(const erp_point2f* kl, const erp_point2f* kr, int32_t m,
                                  int32_t W, int32_t H, double* pts, hipStream_t st);
hipError_t launch_jump_prep(const int32_t* counts, const BatchShape& sh, uint32_t* polyR,
                            uint32_t* polyQ, hipStream_t st);
// part 0: lane end windows (jump-ahead); part 1: the backwards replay -> selection bitmaps
hipError_t launch_sampler(const int32_t* counts, const uint32_t* polyR, const uint32_t* polyQ,
                          const uint32_t* w0, const BatchShape& sh, double sample_frac,
                          const double* rtab, uint32_t* wins, uint32_t* selw, int32_t* flags,
                          hipStream_t st, int part);
// rtab[d] = 1/d rounded up, d < kRecipTable (the sampler's exact modulo); *bad counts entries
// whose one-sided error bound fails (never, by construction; checked once per context)
constexpr int kRecipTable = 65538;
// the sampler's table allocation: rtab [kRecipTable] doubles, then the magic-number table
// [kRecipTable] uint64 (ERP_SAMPLER_MAGIC), then the check counter
constexpr size_t kRecipTableBytes = (size_t)kRecipTable * 16 + 8;
// host: mtab[d] = m_d | (l_d - 1) << 32 (kernels.hip mod_magic_i24); false if a divisor fails
// the exact Granlund-Montgomery condition (never, by construction)
bool build_magic_table(uint64_t* mtab, int n);
// the counter-based sampler (ERP_SAMPLER_PHILOX): selection words in the replay's format,
// max_m = the batch's largest M (<= max_nq); hipErrorInvalidValue when M's bitmap exceeds LDS
hipError_t launch_philox_sampler(const int32_t* counts, const BatchShape& sh, double sample_frac,
                                 uint32_t seed, uint64_t offset, int max_m, uint32_t* selw,
                                 int32_t* flags, hipStream_t st);
hipError_t launch_recip_table(int n, double* rtab, int32_t* bad, hipStream_t st);
int debug_lip_counters(uint32_t* out64);
// Gram of every iteration's sample on int8 MFMA (exact fixed-point sums) -> gram[p][36][iters];
// limbs = scratch of gram_limbs_bytes(sh); samples (debug, may be NULL) = the sampled indices.
// evec != NULL fuses the eigen stage's inverse iteration (pairs with s >= 9) into the Gram
// kernel: evec[p][9][iters] written there, and the Gram written to HBM only for pairs with
// s < 9 and for the iterations whose inverse iteration did not settle (evec NaN); then call
// launch_eigen with fused = 1.  hyps != NULL as well: the settled lanes' estimates too (fused = 2:
// the fallback and thin eigen kernels then write their own lanes' records, no estimate_kernel)
size_t gram_limbs_bytes(const BatchShape& sh);
hipError_t launch_gram_mfma(const int32_t* counts, const double* pts, const uint32_t* selw,
                            const BatchShape& sh, double sample_frac, int8_t* limbs,
                            double* gram, int32_t* samples, double* evec,
                            erp_hypothesis* hyps, double valid_abs, hipStream_t st);

// selected singular vector per iteration from the Grams gram[p][36][iters] -> evec[p][9][iters],
// then the estimate (rank-2 fix, decomposition, Euler angles, validity) -> hyps
hipError_t launch_eigen(const int32_t* counts, const double* gram, const BatchShape& sh,
                        double sample_frac, double valid_abs, double* evec, erp_hypothesis* hyps,
                        hipStream_t st, int fused = 0, bool want_e = true,
                        float* hl = nullptr, int32_t* wsum = nullptr);
// (hl != NULL, round 5: the estimates go to the lite layout -- hl[p][9][iters] f32 R1, R2, T,
// an invalid rotation's x NaN, plus per-64-iteration-wave counts / bounding boxes wsum -- in
// hyp_lite_bytes(sh) (hl, then wsum), for launch_valid_place instead of records)
size_t hyp_lite_bytes(const BatchShape& sh);
hipError_t launch_valid_place(const int32_t* counts, const float* hl, const int32_t* wsum,
                              const BatchShape& sh, double sample_frac, float* rv, float* tv,
                              int32_t* kcount, float* rv_aos, float* dscale, float* edges,
                              hipStream_t st);
// (want_e = false: estimate_kernel leaves the records' E unwritten -- the batch pipeline when the
// caller did not ask for the hypothesis records; nothing downstream reads E)
// the opt-in inlier count (cfg.inlier_thr > 0): every iteration's matches with
// |l^T E' r| < thr into hyps[p][iters].inliers (the records' E must be written); scratch of
// inlier_scratch_bytes(sh)
size_t inlier_scratch_bytes(const BatchShape& sh);
hipError_t launch_inliers(const int32_t* counts, const double* pts, const BatchShape& sh,
                          double sample_frac, float thr, void* scratch, erp_hypothesis* hyps,
                          hipStream_t st);
// R_vec_arr / T_vec_arr in push order + K + bounding-box scale; vchunk = scratch of
// valid_chunk_bytes(sh) (per 1024-iteration chunk: count and bounding box)
size_t valid_chunk_bytes(const BatchShape& sh);
hipError_t launch_valid_compact(const int32_t* counts, const erp_hypothesis* hyps,
                                const BatchShape& sh, double sample_frac, int32_t* vchunk,
                                float* rv, float* tv, int32_t* kcount, float* rv_aos,
                                float* dscale, hipStream_t st);
hipError_t launch_gram_all(const double* pts, int32_t m, double* gram, hipStream_t st);
hipError_t launch_consensus_input(const float* rvec, const float* tvec, int K, int stride, float* rv,
                                  float* tv, int32_t* kcount, float* dscale, int32_t* flags,
                                  hipStream_t st);
// per-row [LB, UB] of the trimmed mean and the bins holding ranks lo / hi-1 (bsel[row][2])
size_t consensus_edges_bytes(int n_pairs);
hipError_t launch_consensus_zoom(const int32_t* kcount, const float* rv, const float* dscale,
                                 float* edges, const BatchShape& sh, double trim_lo,
                                 double trim_hi, double* lb, double* ub, const int32_t* bsel,
                                 const int32_t* surv, int32_t* nsurv, int32_t* zsel, int level,
                                 hipStream_t st);
hipError_t launch_consensus_bounds(const int32_t* kcount, const float* rv, const float* dscale,
                                   float* edges, const BatchShape& sh, double trim_lo,
                                   double trim_hi, double* lb, double* ub, int32_t* bsel,
                                   int shard, int nshards, int32_t* rlist, int32_t* rcount,
                                   int32_t* zsel, int lip2, int32_t* list2, void* lipref,
                                   int lipg, int flat_pct, int use_hint, hipStream_t st,
                                   bool edges_ready = false);
size_t lipref_bytes(int n_pairs, int stride);
// survivors = rows with LB <= min UB (again = 1: only pairs the refine pass touched)
hipError_t launch_consensus_select(const int32_t* kcount, const double* lb, const double* ub,
                                   const BatchShape& sh, double trim_lo, double trim_hi,
                                   int32_t* surv, int32_t* nsurv, double* tmean, int again,
                                   hipStream_t st);
// tighter [LB, UB] for the current survivors (exact inner sums + sub-bins of the boundary bins)
hipError_t launch_consensus_refine(const int32_t* kcount, const float* rv, const float* dscale,
                                   const BatchShape& sh, double trim_lo, double trim_hi,
                                   const int32_t* surv, const int32_t* nsurv, const int32_t* bsel,
                                   double* lb, double* ub, int32_t* list2, void* lipref,
                                   int use_hint, hipStream_t st);
hipError_t launch_consensus_rows(const int32_t* kcount, const float* rv, const float* dscale,
                                 const BatchShape& sh, double trim_lo, double trim_hi,
                                 const int32_t* surv, const int32_t* nsurv, const int32_t* bsel,
                                 double* tmean, hipStream_t st);
hipError_t launch_consensus_final(const int32_t* counts, const int32_t* kcount, const float* rv,
                                  const float* tv, const double* tmean, const int32_t* flags,
                                  const int32_t* nsurv, const int32_t* nbin, const BatchShape& sh,
                                  double sample_frac, double trim_lo, double trim_hi,
                                  float* sortbuf, erp_pair_result* results, hipStream_t st);
int sortbuf_len(int iters);        // power of two >= 2*iters (exact tie re-scoring scratch)

}  // namespace erp
