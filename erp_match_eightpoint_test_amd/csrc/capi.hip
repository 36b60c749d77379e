// capi.hip -- the C ABI declared in include/erp_match.h: context, device scratch and the
// orchestration of the hot-path kernels on one HIP stream.  No host round trip inside a
// pipeline run (match counts, sample sizes and hypothesis counts stay on the device).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/erp_match.h"
#include "erp_kernels.hpp"

// eigen stage fused into the Gram kernel (kernels.hip gram_mfma_kernel: no Gram round trip
// through HBM for the common s >= 9 pairs): 1 = the inverse iteration, 2 = and the estimate;
// 0 = the separate eigen_kernel / estimate_kernel, for A/B
#ifndef ERP_FUSE_EIGEN
#define ERP_FUSE_EIGEN 1
#endif
// hypothesis records' E written only when the caller asked for the records (out->hyps)
#ifndef ERP_SKIP_E
#define ERP_SKIP_E 1
#endif

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

// Debug: erp_debug_set_alloc_pad(N) gives every buffer allocated afterwards N canary bytes
// (0xA5) past its end; erp_debug_check_pads() reports buffers whose canary a kernel overwrote.
std::atomic<size_t> g_alloc_pad{0};
size_t alloc_pad() { return g_alloc_pad.load(std::memory_order_relaxed); }
std::mutex g_pad_mu;
std::vector<std::pair<void*, size_t>> g_padded;

// frees b (and forgets its canary record)
void free_buf(DevBuf& b) {
    if (!b.p) return;
    if (alloc_pad()) {
        std::lock_guard<std::mutex> g(g_pad_mu);
        const auto it = std::find_if(g_padded.begin(), g_padded.end(),
                                     [&](const std::pair<void*, size_t>& e) { return e.first == b.p; });
        if (it != g_padded.end()) g_padded.erase(it);
    }
    (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
}

// grow-only device buffer; returns false on allocation failure
bool ensure(DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.n >= bytes) return true;
    const size_t pad = alloc_pad();
    if (b.p) free_buf(b);
    b.p = nullptr;
    b.n = 0;
    if (hipMalloc(&b.p, bytes + pad) != hipSuccess) return false;
    if (pad) {
        if (hipMemset((char*)b.p + bytes, 0xA5, pad) != hipSuccess) return false;
        std::lock_guard<std::mutex> g(g_pad_mu);
        g_padded.emplace_back(b.p, bytes);
    }
    b.n = bytes;
    return true;
}


}  // namespace

// (global linkage: viz.hip shuffles on the same stream)
// glibc rand() window before draw `offset` of a stream seeded with `seed` (host, sequential;
// same recurrence the kernels jump along).  31 words r[n-31..n-1].
void host_glibc_window(uint32_t seed, uint64_t offset, uint32_t out[31]) {
    int32_t r0[34];
    if (seed == 0) seed = 1;
    r0[0] = (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        const long hi = r0[i - 1] / 127773, lo = r0[i - 1] % 127773;
        long word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r0[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; i++) r0[i] = r0[i - 31];
    uint32_t ring[34];
    for (int i = 0; i < 34; i++) ring[i] = (uint32_t)r0[i];
    uint64_t pos = 34;                    // absolute index of the next word
    const uint64_t end = 344 + offset;    // draw k uses word k + 344
    for (; pos < end; pos++) {
        const uint32_t s = (uint32_t)(pos % 34);
        ring[s] = ring[(pos - 3) % 34] + ring[(pos - 31) % 34];
    }
    for (int j = 0; j < 31; j++) out[j] = ring[(end - 31 + j) % 34];
}

struct erp_ctx {
    int device = 0;
    // one lock per context; recursive so the host-pointer entry points hold it across their
    // copies AND the device entry point they call
    std::recursive_mutex mu;
    // stream ordering between calls (the scratch below is shared by every call): the end of
    // the last call's work, and the stream it was enqueued on
    hipEvent_t done = nullptr;
    hipStream_t last = nullptr;
    bool pending = false;
    // stage timing
    bool profiling = false;
    int32_t matcher = ERP_MATCHER_MFMA_FILTER;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<std::pair<int, size_t>> ev_rec;  // (stage, index of start event; end = +1)
    DevBuf mblk;              // knn2_merge's per-block survivor counts
    DevBuf zsel;              // consensus zoom: the survivors' rank-window bins (level 1 grid)
    DevBuf part, part1, pu, ccount, cand, bsel, edges, gfin, matches, counts, flags, pts, polyR, polyQ, idx, gram, hyps, rv, tv, kcount, tmean,
        sortbuf, w0, off, wh, results, in_a, in_b, in_c, in_d, dscale, lb, ub, surv, nsurv, wins,
        rtab, limbs, tsplit, ovf, remap_scr, vchunk, lipref, inl, hlite;
    DevBuf extra[13];         // erp_ctx_scratch_internal slots (1-11 SURF, 12 viz)
    // route options (erp_ctx_set_option; include/erp_match.h documents each, defaults below)
    int32_t opt[ERP_OPT_COUNT] = {
        -1,  // SMALL_BATCH: auto
        -1,  // SAMPLER_LAT: auto
        -1,  // SAMPLER_SPLIT: auto
        0,   // GRAM_TILES: auto
        // ZOOM_LEVELS: 0 since r05 -- with the hinted refine windows (r04) the survivors' zoom
        // no longer pays for itself; same-box A/B per 768-pair step (profiles/r05w_ab_zoom.txt):
        // consensus 5.81 / 5.87 -> 5.67 / 5.67 ms, worst-case batch 16.2 / 16.1k -> 16.6 /
        // 16.5k pairs/s.  (The second pre-pruning stage's fine pass uses the zoom kernel either way.)
        0,
        0,   // SMALL_ZOOM: the small-batch route skips the zoom (single pair 0.487 -> 0.437 ms)
        // LIP2 / LIPG / REFINE_HINT / FLAT_REFS: -1 = automatic (pruning_opts): on for batches of
        // >= kFewPairs pairs, off below
        -1,  // LIP2: the second pre-pruning stage (kernels.hip consensus_lipschitz2_kernel)
        -1,  // LIPG: the central references' distance gradient (consensus_grad_kernel)
        -1,  // REFINE_HINT: sub-bins on each row's Lipschitz interval (consensus_hint_kernel)
        -1,  // FLAT_REFS: pairs whose first stage kept > 25 % of the rows take the flat route
        1,   // BOUND_RATIO: the matcher's ratio test from the bf16 bounds where they suffice
        -1,  // DEBUG_STAGES: every stage group
        0};  // DEBUG_SNAP
    // debug (ERP_OPT_DEBUG_SNAP): lb, ub and the first-stage list counts right after the bounds
    // pass, fetched with erp_debug_snapshot
    DevBuf snap;
    size_t snap_bytes = 0;
    uint64_t surf_key = 0;    // (W, H, params) of the SURF layer table in extra[1]
    uint32_t viz_epoch = 0;   // stamp epoch of the draw_match line buffer (extra[12])
    // HIP-graph replay of erp_pair_batch_run (erp_ctx_set_graphs): key bytes -> executable graph
    bool use_graphs = false;
    struct Graph {
        std::vector<uint8_t> key;
        hipGraphExec_t exec = nullptr;
        uint64_t used = 0;
    };
    std::vector<Graph> graphs;
    uint64_t graph_clock = 0;
    bool rtab_valid = false;  // rtab[d] = 1/d rounded up (the sampler's exact modulo)
    bool w0_valid = false;
    uint32_t w0_seed = 0;
    uint64_t w0_offset = 0;
};

#define ERP_CK(x)                                         \
    do {                                                  \
        if ((x) != hipSuccess) return ERP_HIP_ERROR;      \
    } while (0)

namespace {

// records an event pair around one launch when profiling is on
struct StageTimer {
    erp_ctx* c;
    int stage;
    hipStream_t st;
    size_t idx = (size_t)-1;
    StageTimer(erp_ctx* c_, int stage_, hipStream_t st_) : c(c_), stage(stage_), st(st_) {
        if (!c->profiling) return;
        while (c->ev_pool.size() < c->ev_used + 2) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;
            c->ev_pool.push_back(e);
        }
        idx = c->ev_used;
        c->ev_used += 2;
        (void)hipEventRecord(c->ev_pool[idx], st);
    }
    ~StageTimer() {
        if (idx == (size_t)-1) return;
        (void)hipEventRecord(c->ev_pool[idx + 1], st);
        c->ev_rec.emplace_back(stage, idx);
    }
};

// A call's enqueue section on a context: holds the context lock, makes this call's stream wait
// for the previous call's work when that went to another stream (every call shares the
// context's scratch, so two calls on different streams would otherwise race on it), and on
// exit records the end of this call's work.  Calls on one stream stay in stream order for free.
struct CtxCall {
    erp_ctx* c;
    hipStream_t st;
    CtxCall(erp_ctx* c_, hipStream_t st_) : c(c_), st(st_) {
        c->mu.lock();
        if (c->pending && st != c->last) (void)hipStreamWaitEvent(st, c->done, 0);
    }
    ~CtxCall() {
        if (!c->done) (void)hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
        if (c->done && hipEventRecord(c->done, st) == hipSuccess) {
            c->last = st;
            c->pending = true;
        }
        c->mu.unlock();
    }
    CtxCall(const CtxCall&) = delete;
    CtxCall& operator=(const CtxCall&) = delete;
};

// The host-pointer entry points that write the shared scratch with blocking copies (null
// stream): join the context's call order and wait on the host for the previous call's device
// work first -- the null stream does not synchronise with non-blocking streams, so an earlier
// *_dev call on such a stream may still be reading the buffers about to be overwritten.
struct HostCtxCall : CtxCall {
    explicit HostCtxCall(erp_ctx* c_) : CtxCall(c_, nullptr) {
        if (c->pending) (void)hipEventSynchronize(c->done);
    }
};

}  // namespace

extern "C" {

int32_t erp_abi_version(void) { return ERP_MATCH_ABI_VERSION; }

}  // extern "C"

int32_t erp_ctx_device_internal(erp_ctx* ctx) { return ctx->device; }  // remap_api.hip

// CtxCall for the entry points of remap_api.hip / surf_api.hip
void* erp_ctx_call_begin_internal(erp_ctx* ctx, hipStream_t st) { return new CtxCall(ctx, st); }
void erp_ctx_call_end_internal(void* call) { delete (CtxCall*)call; }
uint64_t* erp_ctx_surf_key_internal(erp_ctx* ctx) { return &ctx->surf_key; }  // surf_api.hip

// grow-only scratch slots for remap_api.hip / surf_api.hip (slot 0: remap boundary list;
// 1..: SURF buffers)
void* erp_ctx_scratch_internal(erp_ctx* ctx, int which, size_t bytes) {
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    if (which < 0 || which >= (int)(sizeof(ctx->extra) / sizeof(ctx->extra[0]))) return nullptr;
    DevBuf& b = which == 0 ? ctx->remap_scr : ctx->extra[which];
    return ensure(b, bytes) ? b.p : nullptr;
}

// the draw_match line buffer: grown like the other slots, with a per-call epoch for its stamps
// (epoch << 16 | match index); *fresh = the buffer must be zeroed first (new memory, or the
// 16-bit epoch wrapped)
void* erp_ctx_stamp_buffer_internal(erp_ctx* ctx, size_t bytes, uint32_t* epoch, bool* fresh) {
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DevBuf& b = ctx->extra[12];
    // growth is detected by the size: hipMalloc may hand the freed address back for the larger
    // block, whose tail then holds stale stamps
    const size_t n_before = b.n;
    if (!ensure(b, bytes)) return nullptr;
    *fresh = b.n != n_before || ctx->viz_epoch == 0 || ctx->viz_epoch >= 0xFFFFu;
    ctx->viz_epoch = *fresh ? 1u : ctx->viz_epoch + 1u;
    *epoch = ctx->viz_epoch;
    return b.p;
}

extern "C" {

const char* erp_status_string(erp_status s) {
    switch (s) {
        case ERP_OK: return "ok";
        case ERP_INVALID_ARG: return "invalid argument";
        case ERP_TOO_FEW_POINTS: return "too few points";
        case ERP_NO_VALID_HYPOTHESIS: return "no valid rotation hypothesis";
        case ERP_HIP_ERROR: return "HIP error";
        case ERP_NO_DEVICE: return "no HIP device";
        case ERP_OUT_OF_MEMORY: return "out of device memory";
        case ERP_INTERNAL: return "internal consistency check failed";
    }
    return "unknown";
}

void erp_ransac_cfg_default(erp_ransac_cfg* cfg) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->iters = 80;
    cfg->sampler = ERP_SAMPLER_GLIBC;
    cfg->sample_frac = 0.25;
    cfg->trim_lo = 0.2;
    cfg->trim_hi = 0.8;
    cfg->valid_abs = 1.57;
    cfg->seed = 1;
    cfg->offset = 0;
}

erp_status erp_ctx_create(int32_t device, erp_ctx** out) {
    if (!out) return ERP_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ERP_NO_DEVICE;
    if (device < 0 || device >= n) return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(device));
    erp_ctx* c = new (std::nothrow) erp_ctx();
    if (!c) return ERP_OUT_OF_MEMORY;
    c->device = device;
    erp::init_constants();
    *out = c;
    return ERP_OK;
}

erp_status erp_ctx_destroy(erp_ctx* ctx) {
    if (!ctx) return ERP_INVALID_ARG;
    (void)hipSetDevice(ctx->device);
    DevBuf* all[] = {&ctx->mblk, &ctx->zsel, &ctx->part, &ctx->part1, &ctx->pu, &ctx->ccount, &ctx->cand, &ctx->bsel, &ctx->edges, &ctx->gfin,
                     &ctx->matches,
                     &ctx->counts, &ctx->flags, &ctx->pts, &ctx->polyR,
                     &ctx->polyQ, &ctx->idx, &ctx->gram, &ctx->hyps, &ctx->rv, &ctx->tv,
                     &ctx->kcount, &ctx->tmean, &ctx->sortbuf, &ctx->w0, &ctx->off, &ctx->wh,
                     &ctx->results, &ctx->in_a, &ctx->in_b, &ctx->in_c, &ctx->in_d,
                     &ctx->dscale, &ctx->lb, &ctx->ub, &ctx->surv, &ctx->nsurv, &ctx->wins,
                     &ctx->rtab, &ctx->limbs, &ctx->tsplit, &ctx->ovf, &ctx->remap_scr, &ctx->vchunk,
                     &ctx->lipref, &ctx->inl, &ctx->hlite};
    for (DevBuf* b : all) free_buf(*b);
    for (DevBuf& b : ctx->extra) free_buf(b);
    free_buf(ctx->snap);
    for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->done) (void)hipEventDestroy(ctx->done);
    for (auto& g : ctx->graphs) (void)hipGraphExecDestroy(g.exec);
    delete ctx;
    return ERP_OK;
}

}  // extern "C"

namespace {

erp::BatchShape make_shape(int n_pairs, int max_nq, int max_nt, int iters, double frac) {
    erp::BatchShape sh{};
    sh.n_pairs = n_pairs;
    sh.max_nq = std::max(max_nq, 1);
    sh.max_nt = std::max(max_nt, 1);
    // matcher filter grid: 256 queries x one train chunk per block, >= ~1024 blocks, chunks of
    // >= 256 rows (the filter's first stage of every chunk runs twice, bounds then candidates)
    const int qblocks = (sh.max_nq + 255) / 256;
    const int tmax = std::max(1, (sh.max_nt + 255) / 256);
    int chunks = (1024 + qblocks * n_pairs - 1) / (qblocks * n_pairs);
    chunks = std::max(1, std::min(chunks, tmax));
    int chunk_len = (sh.max_nt + chunks - 1) / chunks;
    chunk_len = (chunk_len + 31) / 32 * 32;
    sh.fchunk_len = chunk_len;
    sh.fchunks = (sh.max_nt + chunk_len - 1) / chunk_len;
    // exact VALU sweep: 128 queries x one chunk (multiple of 128 train rows) per block
    const int xqblocks = (sh.max_nq + 127) / 128;
    int xch = (2048 + xqblocks * n_pairs - 1) / (xqblocks * n_pairs);
    xch = std::max(1, std::min(xch, (sh.max_nt + 127) / 128));
    sh.xchunk_len = ((sh.max_nt + xch - 1) / xch + 127) / 128 * 128;
    sh.xchunks = (sh.max_nt + sh.xchunk_len - 1) / sh.xchunk_len;
    sh.iters = std::max(iters, 1);
    sh.max_s = std::max((int)(sh.max_nq * frac), 1);
    sh.idx_stride = sh.max_s;
    sh.sel_words = (sh.max_nq + 30) / 31 + 1;
    return sh;
}

bool ensure_matcher(erp_ctx* c, const erp::BatchShape& sh) {
    const size_t PQ = (size_t)sh.n_pairs * sh.max_nq;
    const size_t fold = PQ * sizeof(erp::Top2);
    if (!ensure(c->mblk, erp::knn2_merge_scratch_bytes(sh))) return false;
    if (c->matcher == ERP_MATCHER_VALU_EXACT)
        return ensure(c->part, PQ * sh.xchunks * sizeof(erp::Top2)) && ensure(c->part1, fold);
    return ensure(c->part, PQ * sh.fchunks * sizeof(erp::Top2)) && ensure(c->part1, fold) &&
           ensure(c->pu, PQ * sh.fchunks * sizeof(float2) + PQ * sizeof(float)) &&  // + |q|^2
           ensure(c->ccount, PQ * sh.fchunks * 2 * 4) &&
           ensure(c->cand, erp::knn2_cand_bytes(sh)) &&
           ensure(c->tsplit, erp::knn2_split_bytes(sh)) &&
           ensure(c->ovf, 4 + 12 * PQ * sh.fchunks);
}

// per-chunk partials -> (fold when there are several chunks) -> ratio test + compaction
// bo != nullptr: the merge also gathers the matched keypoints and writes their bearings
// (bearings_from_matches_kernel's work, one launch fewer)
erp_status fold_and_merge(erp_ctx* ctx, const int64_t* oq, const int64_t* ot,
                          const erp::BatchShape& sh, int chunk_len, int chunks, float ratio,
                          erp_dmatch* matches, int32_t* counts, int32_t* flags, hipStream_t st,
                          const erp::BearingOut* bo = nullptr) {
    StageTimer _t(ctx, ERP_STAGE_KNN2_MERGE, st);
    const erp::Top2* part = (const erp::Top2*)ctx->part.p;
    if (chunks > 1) {
        ERP_CK(erp::launch_knn2_fold(part, oq, ot, sh, chunk_len, chunks, (erp::Top2*)ctx->part1.p,
                                     st));
        part = (const erp::Top2*)ctx->part1.p;
    }
    // a single chunk spanning the whole train set
    ERP_CK(erp::launch_knn2_merge(part, oq, ot, sh, sh.max_nt, 1, ratio, matches, counts, flags,
                                  (int32_t*)ctx->mblk.p, st, bo));
    return ERP_OK;
}

// exact k=2 + ratio test: MFMA filter (bounds + provisional candidates), exact rescoring, merge -- or
// the exact packed-FP32 sweep, merge
erp_status run_matcher(erp_ctx* ctx, const float* dq, const float* dt, const int64_t* oq,
                       const int64_t* ot, const erp::BatchShape& sh, float ratio,
                       erp_dmatch* matches, int32_t* counts, int32_t* flags, hipStream_t st,
                       const erp::BearingOut* bo = nullptr) {
    if (ctx->matcher == ERP_MATCHER_VALU_EXACT) {
        {
            StageTimer _t(ctx, ERP_STAGE_KNN2_EXACT, st);
            ERP_CK(erp::launch_knn2_exact(dq, dt, oq, ot, sh, (erp::Top2*)ctx->part.p, st));
        }
        return fold_and_merge(ctx, oq, ot, sh, sh.xchunk_len, sh.xchunks, ratio, matches, counts,
                              flags, st, bo);
    }
    auto* pu = (float2*)ctx->pu.p;
    auto* cc = (int32_t*)ctx->ccount.p;
    void* cand = ctx->cand.p;
    {
        StageTimer _t(ctx, ERP_STAGE_KNN2_FILTER, st);
        ERP_CK(erp::launch_knn2_filter(dq, dt, oq, ot, sh, ctx->tsplit.p, pu, cc, cand, st,
                                       (int32_t*)ctx->ovf.p, flags));
    }
    {
        StageTimer _t(ctx, ERP_STAGE_KNN2_RESCORE, st);
        ERP_CK(erp::launch_knn2_rescore(dq, dt, oq, ot, sh, ctx->tsplit.p, pu, cc, cand,
                                        (erp::Top2*)ctx->part.p, (int32_t*)ctx->ovf.p,
                                        ctx->opt[ERP_OPT_BOUND_RATIO] ? ratio : -1.f, st));
    }
    return fold_and_merge(ctx, oq, ot, sh, sh.fchunk_len, sh.fchunks, ratio, matches, counts,
                          flags, st, bo);
}

erp_status ensure_estimator(erp_ctx* c, const erp::BatchShape& sh, const erp_batch_outputs* out) {
    const size_t P = (size_t)sh.n_pairs;
    const size_t nwaves = (size_t)(sh.iters + 63) / 64;
    bool ok = ensure(c->counts, P * 4) && ensure(c->flags, P * 4) &&
              ensure(c->pts, P * (sh.max_nq + 1) * 48) &&
              ensure(c->wins, P * nwaves * 31 * 64 * 4) && ensure(c->polyR, P * 65 * 31 * 4) &&
              ensure(c->polyQ, P * erp::kMaxQ * 31 * 4) &&
              ensure(c->idx, P * nwaves * (size_t)sh.sel_words * 64 * 4) &&
              ensure(c->gram, P * sh.iters * 36 * 8) && ensure(c->limbs, erp::gram_limbs_bytes(sh)) &&
              ensure(c->gfin, P * sh.iters * 9 * 8) && ensure(c->rv, P * 6 * sh.iters * 4) &&
              ensure(c->kcount, P * 4) && ensure(c->sortbuf, P * (size_t)erp::sortbuf_len(sh.iters) * 4) &&
              ensure(c->w0, 31 * 4) && ensure(c->results, P * sizeof(erp_pair_result)) &&
              ensure(c->dscale, P * 4) && ensure(c->lb, P * 2 * sh.iters * 8) &&
              ensure(c->ub, P * 2 * sh.iters * 8) && ensure(c->surv, P * 2 * sh.iters * 4) &&
              ensure(c->bsel, P * 2 * sh.iters * 8) && ensure(c->zsel, P * 2 * sh.iters * 8) &&
              ensure(c->lipref, erp::lipref_bytes((int)P, 2 * sh.iters)) && ensure(c->edges, erp::consensus_edges_bytes((int)P)) &&
              ensure(c->nsurv, P * 20 + 8) && ensure(c->vchunk, erp::valid_chunk_bytes(sh));
    if (ok && !(out && out->hyps)) ok = ensure(c->hyps, P * sh.iters * sizeof(erp_hypothesis));
    if (ok) ok = ensure(c->hlite, erp::hyp_lite_bytes(sh));
    if (ok && !(out && out->tvec)) ok = ensure(c->tv, P * 6 * sh.iters * 4);
    if (ok && !(out && out->dist)) ok = ensure(c->tmean, P * 2 * sh.iters * 8);
    if (!ok) return ERP_OUT_OF_MEMORY;
    if (!c->rtab_valid) {  // once per context: the reciprocal table, verified exactly
        constexpr int n = erp::kRecipTable;
        if (!ensure(c->rtab, erp::kRecipTableBytes)) return ERP_OUT_OF_MEMORY;
        {  // the magic-number table after it (the sampler's d >= 256 quotients)
            std::vector<uint64_t> mt(n);
            if (!erp::build_magic_table(mt.data(), n)) return ERP_INTERNAL;
            ERP_CK(hipMemcpy((double*)c->rtab.p + n, mt.data(), (size_t)n * 8,
                             hipMemcpyHostToDevice));
        }
        int32_t* d_bad = (int32_t*)((char*)c->rtab.p + (size_t)n * 16);
        ERP_CK(hipMemset(d_bad, 0, 4));
        ERP_CK(erp::launch_recip_table(n, (double*)c->rtab.p, d_bad, nullptr));
        int32_t bad = 0;
        ERP_CK(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
        if (bad) return ERP_INTERNAL;
        c->rtab_valid = true;
    }
    return ERP_OK;
}

erp_status upload_w0(erp_ctx* c, const erp_ransac_cfg* cfg, hipStream_t st) {
    if (!c->w0_valid || c->w0_seed != cfg->seed || c->w0_offset != cfg->offset) {
        uint32_t w[31];
        host_glibc_window(cfg->seed, cfg->offset, w);
        ERP_CK(hipMemcpyAsync(c->w0.p, w, sizeof(w), hipMemcpyHostToDevice, st));
        ERP_CK(hipStreamSynchronize(st));
        c->w0_valid = true;
        c->w0_seed = cfg->seed;
        c->w0_offset = cfg->offset;
    }
    return ERP_OK;
}

bool cfg_ok(const erp_ransac_cfg* cfg) {
    return cfg && cfg->iters >= 1 &&
           (cfg->sampler == ERP_SAMPLER_GLIBC || cfg->sampler == ERP_SAMPLER_PHILOX) &&
           cfg->sample_frac > 0 &&
           cfg->sample_frac <= 1.0 && cfg->trim_lo >= 0 && cfg->trim_hi <= 1.0 &&
           cfg->trim_lo <= cfg->trim_hi && cfg->inlier_thr >= 0.0f && cfg->inlier_thr < 1e30f;
}

// the Philox sampler's per-lane LDS bitmap holds M <= 20480 positions (kernels.hip
// launch_philox_sampler); entry points that know m on the host refuse larger pairs up front (the
// batch pipeline, where M is only known on the device, flags the pair instead)
constexpr int32_t kPhiloxMaxM = 20480;
bool sampler_m_ok(const erp_ransac_cfg* cfg, int32_t m) {
    return cfg->sampler != ERP_SAMPLER_PHILOX || m <= kPhiloxMaxM;
}

// the records' E: written when the caller asked for the records or the inlier count reads it
bool want_e(const erp_ransac_cfg* cfg, const erp_batch_outputs* out) {
    return !ERP_SKIP_E || (out && out->hyps) || cfg->inlier_thr > 0.0f;
}

// the opt-in inlier count after the estimate (cfg->inlier_thr > 0; nothing runs otherwise)
erp_status run_inliers(erp_ctx* c, const erp::BatchShape& sh, const erp_ransac_cfg* cfg,
                       erp_hypothesis* hyps, hipStream_t st) {
    if (!(cfg->inlier_thr > 0.0f)) return ERP_OK;
    if (!ensure(c->inl, erp::inlier_scratch_bytes(sh))) return ERP_OUT_OF_MEMORY;
    StageTimer _t(c, ERP_STAGE_INLIERS, st);
    ERP_CK(erp::launch_inliers((int32_t*)c->counts.p, (double*)c->pts.p, sh, cfg->sample_frac,
                               cfg->inlier_thr, c->inl.p, hyps, st));
    return ERP_OK;
}

// the lite estimates (launch_eigen's hl: R1, R2, T as f32 SoA + per-wave counts, no records)
// when nothing reads the records: the caller did not ask for them, the opt-in inlier count is
// off (it adds into the records) and the estimate is not fused into the Gram kernel
bool use_lite(const erp_ransac_cfg* cfg, const erp_batch_outputs* out) {
    return !(out && out->hyps) && !(cfg->inlier_thr > 0.0f) && ERP_FUSE_EIGEN != 2;
}
float* lite_hl(erp_ctx* c) { return (float*)c->hlite.p; }
int32_t* lite_wsum(erp_ctx* c, const erp::BatchShape& sh) {
    return (int32_t*)(lite_hl(c) + (size_t)sh.n_pairs * 9 * sh.iters);
}

// estimator stages after counts/pts are in place (lite: the estimates in the lite layout)
erp_status run_hypotheses(erp_ctx* c, const erp::BatchShape& sh_in, const erp_ransac_cfg* cfg,
                          const erp_batch_outputs* out, hipStream_t st, bool lite = false) {
    erp_ctx* ctx = c;
    erp::BatchShape sh = sh_in;  // + the sampler / Gram route options
    sh.sampler_lat = c->opt[ERP_OPT_SAMPLER_LAT];
    sh.sampler_split = c->opt[ERP_OPT_SAMPLER_SPLIT];
    sh.gram_tiles = c->opt[ERP_OPT_GRAM_TILES];
    auto* counts = (int32_t*)c->counts.p;
    auto* flags = (int32_t*)c->flags.p;
    auto* hyps = (out && out->hyps) ? out->hyps : (erp_hypothesis*)c->hyps.p;
    if (cfg->sampler == ERP_SAMPLER_PHILOX) {  // counter-based: no jump polynomials / windows
        if (c->opt[ERP_OPT_DEBUG_STAGES] & 4) {
            StageTimer _t(ctx, ERP_STAGE_SAMPLER, st);
            ERP_CK(erp::launch_philox_sampler(counts, sh, cfg->sample_frac, cfg->seed, cfg->offset,
                                              sh.max_nq, (uint32_t*)c->idx.p, flags, st));
        }
        if (c->opt[ERP_OPT_DEBUG_STAGES] & 8) {
            StageTimer _t(ctx, ERP_STAGE_GRAM, st);
            ERP_CK(erp::launch_gram_mfma(counts, (double*)c->pts.p, (uint32_t*)c->idx.p, sh,
                                         cfg->sample_frac, (int8_t*)c->limbs.p, (double*)c->gram.p,
                                         out ? out->samples : nullptr,
                                         ERP_FUSE_EIGEN ? (double*)c->gfin.p : nullptr,
                                         ERP_FUSE_EIGEN == 2 ? hyps : nullptr, cfg->valid_abs, st));
        }
        if (c->opt[ERP_OPT_DEBUG_STAGES] & 32) {
            StageTimer _t(ctx, ERP_STAGE_EIGEN, st);
            ERP_CK(erp::launch_eigen(counts, (double*)c->gram.p, sh, cfg->sample_frac,
                                     cfg->valid_abs, (double*)c->gfin.p, hyps, st, ERP_FUSE_EIGEN,
                                     want_e(cfg, out), lite ? lite_hl(c) : nullptr,
                                     lite ? lite_wsum(c, sh) : nullptr));
        }
        return run_inliers(c, sh, cfg, hyps, st);
    }
    if (c->opt[ERP_OPT_DEBUG_STAGES] & 2) {
        StageTimer _t(ctx, ERP_STAGE_JUMP_PREP, st);
        ERP_CK(erp::launch_jump_prep(counts, sh, (uint32_t*)c->polyR.p, (uint32_t*)c->polyQ.p, st));
    }
    if (c->opt[ERP_OPT_DEBUG_STAGES] & 2) {
        StageTimer _t(ctx, ERP_STAGE_WINDOWS, st);
        ERP_CK(erp::launch_sampler(counts, (uint32_t*)c->polyR.p, (uint32_t*)c->polyQ.p,
                                   (uint32_t*)c->w0.p, sh, cfg->sample_frac, (double*)c->rtab.p,
                                   (uint32_t*)c->wins.p, (uint32_t*)c->idx.p, flags, st, 0));
    }
    if (c->opt[ERP_OPT_DEBUG_STAGES] & 4) {
        StageTimer _t(ctx, ERP_STAGE_SAMPLER, st);
        ERP_CK(erp::launch_sampler(counts, (uint32_t*)c->polyR.p, (uint32_t*)c->polyQ.p,
                                   (uint32_t*)c->w0.p, sh, cfg->sample_frac, (double*)c->rtab.p,
                                   (uint32_t*)c->wins.p, (uint32_t*)c->idx.p, flags, st, 1));
    }
    if (c->opt[ERP_OPT_DEBUG_STAGES] & 8) {
        StageTimer _t(ctx, ERP_STAGE_GRAM, st);
        ERP_CK(erp::launch_gram_mfma(counts, (double*)c->pts.p, (uint32_t*)c->idx.p, sh,
                                     cfg->sample_frac, (int8_t*)c->limbs.p, (double*)c->gram.p,
                                     out ? out->samples : nullptr,
                                     ERP_FUSE_EIGEN ? (double*)c->gfin.p : nullptr,
                                     ERP_FUSE_EIGEN == 2 ? hyps : nullptr, cfg->valid_abs, st));
    }
    if (c->opt[ERP_OPT_DEBUG_STAGES] & 32) {
        StageTimer _t(ctx, ERP_STAGE_EIGEN, st);
        ERP_CK(erp::launch_eigen(counts, (double*)c->gram.p, sh, cfg->sample_frac,
                                 cfg->valid_abs, (double*)c->gfin.p, hyps, st, ERP_FUSE_EIGEN,
                                 want_e(cfg, out), lite ? lite_hl(c) : nullptr,
                                 lite ? lite_wsum(c, sh) : nullptr));
    }
    return run_inliers(c, sh, cfg, hyps, st);
}

// The pruning refinements of rounds 3-4 (second stage, gradient references, flat route, hinted
// refine windows) were tuned on 128-pair launches.  A launch of a few pairs with a large K
// (configs[4]: one find of 100k iterations, K ~ 89k) runs their per-pair passes on a handful of
// blocks each: there they cost more than they save -- bench.py --workload manual, one box
// (profiles/r06h_manual_opts.txt): 2.11 ms per find with all four, 1.53 ms without.  So their
// automatic setting (-1) is on for launches of >= kFewPairs pairs and off below; an explicit
// option value always wins.  (Results are identical either way: tests/test_gpu_parity.py.)
constexpr int kFewPairs = 8;
struct PruningOpts {
    int lip2, lipg, flat_pct, hint;
};
PruningOpts pruning_opts(const erp_ctx* c, const erp::BatchShape& sh) {
    const bool few = sh.n_pairs < kFewPairs;
    auto pick = [&](int v, int on) { return v >= 0 ? v : (few ? 0 : on); };
    return PruningOpts{pick(c->opt[ERP_OPT_LIP2], 1), pick(c->opt[ERP_OPT_LIPG], 1),
                       pick(c->opt[ERP_OPT_FLAT_REFS], 25), pick(c->opt[ERP_OPT_REFINE_HINT], 1)};
}

// consensus stages after the hypothesis records are in place (counts may be null when the
// valid list is given directly: erp_consensus_dev)
// phase: 0 = everything; 1 = compaction + bounds of rows shard / nshards only (into lb_/ub_/
// bsel_); 2 = the rest (select onward) after a phase-1 call on this context, with the bounds
// of every row in lb_/ub_/bsel_ (combined over the shards by the caller)
erp_status run_consensus(erp_ctx* c, const erp::BatchShape& sh, const erp_ransac_cfg* cfg,
                         const erp_batch_outputs* out, erp_pair_result* results, hipStream_t st,
                         bool from_hyps, int phase = 0, int shard = 0, int nshards = 1,
                         double* lb_ = nullptr, double* ub_ = nullptr, int32_t* bsel_ = nullptr,
                         bool lite = false) {
    erp_ctx* ctx = c;
    double* lbp = lb_ ? lb_ : (double*)c->lb.p;
    double* ubp = ub_ ? ub_ : (double*)c->ub.p;
    int32_t* bselp = bsel_ ? bsel_ : (int32_t*)c->bsel.p;
    auto* counts = from_hyps ? (int32_t*)c->counts.p : nullptr;
    auto* flags = (int32_t*)c->flags.p;  // consensus-only: set by consensus_input (non-finite)
    auto* hyps = (out && out->hyps) ? out->hyps : (erp_hypothesis*)c->hyps.p;
    auto* tv = (out && out->tvec) ? out->tvec : (float*)c->tv.p;
    auto* tmean = (out && out->dist) ? out->dist : (double*)c->tmean.p;
    if (from_hyps && phase != 2 && lite) {
        StageTimer _t(ctx, ERP_STAGE_VALID_COMPACT, st);
        ERP_CK(erp::launch_valid_place(counts, lite_hl(c), lite_wsum(c, sh), sh, cfg->sample_frac,
                                       (float*)c->rv.p, tv, (int32_t*)c->kcount.p,
                                       out ? out->rvec : nullptr, (float*)c->dscale.p,
                                       (float*)c->edges.p, st));
    } else if (from_hyps && phase != 2) {
        StageTimer _t(ctx, ERP_STAGE_VALID_COMPACT, st);
        ERP_CK(erp::launch_valid_compact(counts, hyps, sh, cfg->sample_frac,
                                         (int32_t*)c->vchunk.p, (float*)c->rv.p, tv,
                                         (int32_t*)c->kcount.p, out ? out->rvec : nullptr,
                                         (float*)c->dscale.p, st));
    }
    // small batches (the single-pair call of src/automatic.cpp:117-126): every row gets its
    // K-column histogram, no Lipschitz pre-pruning, no zoom or refine stage.  For one pair at
    // 10k iterations that pass is ~25-35 us of the whole GPU, against ~20 dependent small
    // launches (~0.2 ms) of the pruning stages, which only pay when many pairs share the chip
    // or K is large: the route is taken when n_pairs (2 iters)^2 <= 2e9 (one pair up to ~22k
    // iterations, five at 10k; configs[4]'s 100k-iteration find keeps the pruning), and never
    // for the row-sharded phases.  ERP_OPT_SMALL_BATCH = n >= 0 overrides: batches of <= n pairs
    // take it (0 = never)
    const int sb = c->opt[ERP_OPT_SMALL_BATCH];
    const double kk = 2.0 * sh.iters;
    const bool small = phase == 0 && nshards == 1 &&
                       (sb >= 0 ? sh.n_pairs <= sb : sh.n_pairs * kk * kk <= 2e9);
    const bool prune = !small;
    const PruningOpts po = pruning_opts(c, sh);
    if (phase != 2) {
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_BOUNDS, st);
        ERP_CK(erp::launch_consensus_bounds((int32_t*)c->kcount.p, (float*)c->rv.p,
                                            (float*)c->dscale.p, (float*)c->edges.p, sh,
                                            cfg->trim_lo, cfg->trim_hi, lbp, ubp, bselp, shard,
                                            nshards, prune ? (int32_t*)c->surv.p : nullptr,
                                            prune ? (int32_t*)c->nsurv.p + sh.n_pairs : nullptr,
                                            (int32_t*)c->zsel.p, po.lip2,
                                            (int32_t*)c->sortbuf.p, c->lipref.p, po.lipg,
                                            po.flat_pct, po.hint, st,
                                            from_hyps && lite));  // (valid_place wrote the edges)
    }
    if (c->opt[ERP_OPT_DEBUG_SNAP] && phase == 0) {
        const size_t nrow = (size_t)sh.n_pairs * 2 * sh.iters;
        // (kernels.hip lipref_cap at the default second-stage step 4)
        const size_t lrb = (size_t)sh.n_pairs * (2 * sh.iters / 4 + 64) * 16 + (size_t)sh.n_pairs * 12;
        c->snap_bytes = nrow * 16 + (size_t)sh.n_pairs * 4 + lrb;
        if (!ensure(c->snap, c->snap_bytes)) return ERP_OUT_OF_MEMORY;
        ERP_CK(hipMemcpyAsync(c->snap.p, lbp, nrow * 8, hipMemcpyDeviceToDevice, st));
        ERP_CK(hipMemcpyAsync((char*)c->snap.p + nrow * 8, ubp, nrow * 8, hipMemcpyDeviceToDevice, st));
        if (prune)
            ERP_CK(hipMemcpyAsync((char*)c->snap.p + nrow * 16, (int32_t*)c->nsurv.p + sh.n_pairs,
                                  (size_t)sh.n_pairs * 4, hipMemcpyDeviceToDevice, st));
        else  // (the small-batch route lists nothing: -1 = every row binned)
            ERP_CK(hipMemsetAsync((char*)c->snap.p + nrow * 16, 0xFF, (size_t)sh.n_pairs * 4, st));
        // + the first-stage references (float4 [P][cap]), their U [P] f64 and counts [P] i32
        ERP_CK(hipMemcpyAsync((char*)c->snap.p + nrow * 16 + (size_t)sh.n_pairs * 4, c->lipref.p, lrb,
                              hipMemcpyDeviceToDevice, st));
    }
    if (phase == 1) return ERP_OK;
    if (phase == 2)  // the bounds ran per shard (binned rows not combined): report -1
        ERP_CK(hipMemsetAsync((int32_t*)c->nsurv.p + sh.n_pairs, 0xFF, sizeof(int32_t) * sh.n_pairs, st));
    {
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_SELECT, st);
        ERP_CK(erp::launch_consensus_select((int32_t*)c->kcount.p, lbp,
                                            ubp, sh, cfg->trim_lo, cfg->trim_hi,
                                            (int32_t*)c->surv.p, (int32_t*)c->nsurv.p, tmean, 0,
                                            st));
    }
    // small batches skip the zoom too: the exact pass takes the first selection's survivors
    // (~150 for a typical pair, one grid-wide launch); single pair 0.487 -> 0.437 ms
    // (profiles/r05g_latency_ab.txt; ERP_OPT_SMALL_ZOOM = 1 keeps it)
    const int zoom_levels = prune || c->opt[ERP_OPT_SMALL_ZOOM] ? c->opt[ERP_OPT_ZOOM_LEVELS] : 0;
    for (int level = 1; level <= zoom_levels; level++) {
        {
            StageTimer _t(ctx, ERP_STAGE_CONSENSUS_BOUNDS, st);
            ERP_CK(erp::launch_consensus_zoom((int32_t*)c->kcount.p, (float*)c->rv.p,
                                              (float*)c->dscale.p, (float*)c->edges.p, sh,
                                              cfg->trim_lo, cfg->trim_hi, lbp, ubp, bselp,
                                              (int32_t*)c->surv.p, (int32_t*)c->nsurv.p,
                                              (int32_t*)c->zsel.p, level, st));
        }
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_SELECT, st);
        ERP_CK(erp::launch_consensus_select((int32_t*)c->kcount.p, lbp,
                                            ubp, sh, cfg->trim_lo, cfg->trim_hi,
                                            (int32_t*)c->surv.p, (int32_t*)c->nsurv.p, tmean, 0,
                                            st));
    }
    // (small batches: no refine stage either -- the exact pass takes the survivors in one
    // grid-wide launch; the refine stage's ~8 dependent launches cost a single pair more)
    if (prune) {
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_REFINE, st);
        ERP_CK(erp::launch_consensus_refine((int32_t*)c->kcount.p, (float*)c->rv.p,
                                            (float*)c->dscale.p, sh, cfg->trim_lo, cfg->trim_hi,
                                            (int32_t*)c->surv.p, (int32_t*)c->nsurv.p,
                                            bselp, lbp,
                                            ubp, (int32_t*)c->sortbuf.p, c->lipref.p,
                                            po.hint, st));
    }
    if (prune) {
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_SELECT, st);
        ERP_CK(erp::launch_consensus_select((int32_t*)c->kcount.p, lbp,
                                            ubp, sh, cfg->trim_lo, cfg->trim_hi,
                                            (int32_t*)c->surv.p, (int32_t*)c->nsurv.p, tmean, 1,
                                            st));
    }
    {
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_ROWS, st);
        ERP_CK(erp::launch_consensus_rows((int32_t*)c->kcount.p, (float*)c->rv.p,
                                          (float*)c->dscale.p, sh, cfg->trim_lo, cfg->trim_hi,
                                          (int32_t*)c->surv.p, (int32_t*)c->nsurv.p,
                                          bselp, tmean, st));
    }
    {
        StageTimer _t(ctx, ERP_STAGE_CONSENSUS_FINAL, st);
        ERP_CK(erp::launch_consensus_final(counts, (int32_t*)c->kcount.p, (float*)c->rv.p, tv, tmean,
                                           flags, (int32_t*)c->nsurv.p,
                                           prune ? (int32_t*)c->nsurv.p + sh.n_pairs : nullptr, sh,
                                           cfg->sample_frac, cfg->trim_lo, cfg->trim_hi,
                                           (float*)c->sortbuf.p, results, st));
    }
    if (c->opt[ERP_OPT_DEBUG_SNAP] && phase == 0 && c->snap_bytes) {
        // + the consensus's rotation vectors (SoA [P][3][2 iters] f32) as they are at its end
        const size_t rvb = (size_t)sh.n_pairs * 6 * sh.iters * 4;
        const size_t head = c->snap_bytes;
        DevBuf keep = c->snap;
        if (c->snap.n < head + rvb) {
            c->snap = DevBuf();
            if (!ensure(c->snap, head + rvb)) return ERP_OUT_OF_MEMORY;
            ERP_CK(hipMemcpyAsync(c->snap.p, keep.p, head, hipMemcpyDeviceToDevice, st));
            ERP_CK(hipStreamSynchronize(st));
            free_buf(keep);
        }
        ERP_CK(hipMemcpyAsync((char*)c->snap.p + head, c->rv.p, rvb, hipMemcpyDeviceToDevice, st));
        c->snap_bytes = head + rvb;
    }
    return ERP_OK;
}


erp_status run_estimator(erp_ctx* c, const erp::BatchShape& sh, const erp_ransac_cfg* cfg,
                         const erp_batch_outputs* out, erp_pair_result* results, hipStream_t st) {
    const bool lite = use_lite(cfg, out);
    erp_status es = run_hypotheses(c, sh, cfg, out, st, lite);
    if (es != ERP_OK) return es;
    if (!(c->opt[ERP_OPT_DEBUG_STAGES] & 16)) return ERP_OK;
    return run_consensus(c, sh, cfg, out, results, st, true, 0, 0, 1, nullptr, nullptr, nullptr,
                         lite);
}

}  // namespace

extern "C" {

erp_status erp_ctx_set_profiling(erp_ctx* ctx, int32_t enable) {
    if (!ctx) return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->profiling = enable != 0;
    return ERP_OK;
}

erp_status erp_ctx_set_matcher(erp_ctx* ctx, int32_t method) {
    if (!ctx) return ERP_INVALID_ARG;
    if (method != ERP_MATCHER_MFMA_FILTER && method != ERP_MATCHER_VALU_EXACT)
        return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->matcher = method;
    return ERP_OK;
}

const char* erp_stage_name(int32_t stage) {
    static const char* names[ERP_STAGE_COUNT] = {
        "knn2_filter", "knn2_merge", "bearings", "jump_prep", "sampler",
        "eigen", "valid_compact", "consensus_rows", "consensus_final", "consensus_bounds",
        "consensus_select", "windows", "gram", "knn2_candidates", "knn2_rescore",
        "consensus_refine", "knn2_exact", "sampler_gram", "inliers"};
    return (stage >= 0 && stage < ERP_STAGE_COUNT) ? names[stage] : "unknown";
}

erp_status erp_ctx_stage_times(erp_ctx* ctx, double* total_ms, int64_t* launches) {
    if (!ctx || !total_ms || !launches) return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ERP_CK(hipSetDevice(ctx->device));
    for (int k = 0; k < ERP_STAGE_COUNT; k++) {
        total_ms[k] = 0;
        launches[k] = 0;
    }
    for (const auto& r : ctx->ev_rec) {
        ERP_CK(hipEventSynchronize(ctx->ev_pool[r.second + 1]));
        float ms = 0;
        ERP_CK(hipEventElapsedTime(&ms, ctx->ev_pool[r.second], ctx->ev_pool[r.second + 1]));
        total_ms[r.first] += ms;
        launches[r.first] += 1;
    }
    ctx->ev_rec.clear();
    ctx->ev_used = 0;
    return ERP_OK;
}

erp_status erp_ctx_reserve(erp_ctx* ctx, int32_t n_pairs, int32_t max_nq, int32_t max_nt,
                           int32_t iters) {
    if (!ctx || n_pairs < 1 || max_nq < 0 || max_nt < 0 || iters < 1) return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ERP_CK(hipSetDevice(ctx->device));
    const erp::BatchShape sh = make_shape(n_pairs, max_nq, max_nt, iters, 0.25);
    if (!ensure_matcher(ctx, sh) ||
        !ensure(ctx->matches, (size_t)n_pairs * sh.max_nq * sizeof(erp_dmatch)))
        return ERP_OUT_OF_MEMORY;
    return ensure_estimator(ctx, sh, nullptr);
}

}  // extern "C"

namespace {

// the enqueue part of erp_pair_batch_run (every allocation and host upload done before it)
erp_status batch_enqueue(erp_ctx* ctx, const erp_pair_batch* b, float ratio,
                         const erp_ransac_cfg* cfg, const erp_batch_outputs* out,
                         const erp::BatchShape& sh, erp_dmatch* matches, hipStream_t st) {
    if (!(ctx->opt[ERP_OPT_DEBUG_STAGES] & 1)) return run_estimator(ctx, sh, cfg, out, out->results, st);
    // the optional outputs read zero past each pair's M / K / s, call after call (a HIP-graph
    // replay or a reused buffer would otherwise keep an earlier call's entries there)
    const size_t P = (size_t)sh.n_pairs, I = (size_t)sh.iters, Q = (size_t)b->max_nq;
    const size_t smax = (size_t)std::max((int)(Q * cfg->sample_frac), 1);
    const struct {
        void* p;
        size_t bytes;
    } opt[] = {{out->matches, P * Q * sizeof(erp_dmatch)}, {out->key_left, P * Q * 8},
               {out->key_right, P * Q * 8}, {out->hyps, P * I * sizeof(erp_hypothesis)},
               {out->samples, P * I * smax * 4}, {out->rvec, P * 2 * I * 12},
               {out->tvec, P * 2 * I * 12}, {out->dist, P * 2 * I * 8}};
    for (const auto& o : opt)
        if (o.p) ERP_CK(hipMemsetAsync(o.p, 0, o.bytes, st));
    if (ctx->matcher == ERP_MATCHER_VALU_EXACT)  // (knn2_split_kernel resets them on the MFMA path)
        ERP_CK(hipMemsetAsync(ctx->flags.p, 0, (size_t)sh.n_pairs * 4, st));
    // the merge writes the gather + bearings as it places each match (src/spherical_surf.cpp:
    // 155-162, src/eight_point.cpp:163-186; bearings_from_matches_kernel's work)
    const erp::BearingOut bo{b->kp_l, b->kp_r, b->width, b->height, (double*)ctx->pts.p,
                             out->key_left, out->key_right};
    erp_status es = run_matcher(ctx, b->desc_l, b->desc_r, b->off_l, b->off_r, sh, ratio, matches,
                                (int32_t*)ctx->counts.p, (int32_t*)ctx->flags.p, st, &bo);
    if (es != ERP_OK) return es;
    return run_estimator(ctx, sh, cfg, out, out->results, st);
}

template <class T>
void key_put(std::vector<uint8_t>& k, const T& v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    k.insert(k.end(), p, p + sizeof(T));
}

// everything a captured pipeline bakes in: the call's structs and the context's scratch pointers
// and route options
std::vector<uint8_t> graph_key(const erp_ctx* c, const erp_pair_batch* b, float ratio,
                               const erp_ransac_cfg* cfg, const erp_batch_outputs* out) {
    std::vector<uint8_t> k;
    key_put(k, *b);
    key_put(k, *cfg);
    key_put(k, *out);
    key_put(k, ratio);
    key_put(k, c->matcher);
    key_put(k, c->opt);
    const DevBuf* all[] = {&c->mblk, &c->zsel, &c->part, &c->part1, &c->pu, &c->ccount, &c->cand,
                           &c->bsel, &c->edges, &c->gfin, &c->matches, &c->counts, &c->flags,
                           &c->pts, &c->polyR, &c->polyQ, &c->idx, &c->gram, &c->hyps, &c->rv,
                           &c->tv, &c->kcount, &c->tmean, &c->sortbuf, &c->w0, &c->results,
                           &c->dscale, &c->lb, &c->ub, &c->surv, &c->nsurv, &c->wins, &c->rtab,
                           &c->limbs, &c->tsplit, &c->ovf, &c->vchunk, &c->lipref, &c->inl,
                           &c->hlite};
    for (const DevBuf* d : all) key_put(k, d->p);
    return k;
}

}  // namespace

extern "C" {

erp_status erp_ctx_set_graphs(erp_ctx* ctx, int32_t enable) {
    if (!ctx) return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->use_graphs = enable != 0;
    return ERP_OK;
}

erp_status erp_ctx_set_option(erp_ctx* ctx, int32_t option, int32_t value) {
    if (!ctx || option < 0 || option >= ERP_OPT_COUNT) return ERP_INVALID_ARG;
    int lo = 0, hi = 1;  // the on / off options
    switch (option) {
        case ERP_OPT_SMALL_BATCH: lo = -1; hi = INT32_MAX; break;
        case ERP_OPT_SAMPLER_LAT: lo = -1; hi = 2; break;
        case ERP_OPT_SAMPLER_SPLIT: lo = -1; hi = 1; break;
        case ERP_OPT_GRAM_TILES: lo = 0; hi = 2; break;
        case ERP_OPT_ZOOM_LEVELS: lo = 0; hi = 2; break;
        case ERP_OPT_FLAT_REFS: lo = -1; hi = 100; break;
        case ERP_OPT_LIPG: lo = -1; hi = 3; break;  // bit 0: first stage, bit 1: second stage
        case ERP_OPT_LIP2: lo = -1; hi = 1; break;
        case ERP_OPT_REFINE_HINT: lo = -1; hi = 1; break;
        case ERP_OPT_DEBUG_STAGES: lo = -1; hi = 63; break;
        default: break;
    }
    if (value < lo || value > hi) return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->opt[option] = value;
    return ERP_OK;
}

erp_status erp_ctx_get_option(erp_ctx* ctx, int32_t option, int32_t* value) {
    if (!ctx || !value || option < 0 || option >= ERP_OPT_COUNT) return ERP_INVALID_ARG;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    *value = ctx->opt[option];
    return ERP_OK;
}

void erp_debug_set_alloc_pad(size_t bytes) { g_alloc_pad.store(bytes, std::memory_order_relaxed); }

erp_status erp_pair_batch_run(erp_ctx* ctx, const erp_pair_batch* b, float ratio,
                              const erp_ransac_cfg* cfg, const erp_batch_outputs* out,
                              void* stream) {
    if (!ctx || !b || !out || !out->results || !cfg_ok(cfg)) return ERP_INVALID_ARG;
    if (b->n_pairs < 1 || b->dim != erp::kDim || b->max_nq < 0 || b->max_nt < 0 ||
        b->max_nq > 65535 || !b->desc_l || !b->desc_r || !b->kp_l || !b->kp_r || !b->off_l ||
        !b->off_r || !b->width || !b->height)
        return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    const erp::BatchShape sh = make_shape(b->n_pairs, b->max_nq, b->max_nt, cfg->iters,
                                          cfg->sample_frac);
    if (!ensure_matcher(ctx, sh)) return ERP_OUT_OF_MEMORY;
    erp_dmatch* matches = out->matches;
    if (!matches) {
        if (!ensure(ctx->matches, (size_t)sh.n_pairs * sh.max_nq * sizeof(erp_dmatch)))
            return ERP_OUT_OF_MEMORY;
        matches = (erp_dmatch*)ctx->matches.p;
    }
    erp_status es = ensure_estimator(ctx, sh, out);
    if (es != ERP_OK) return es;
    es = upload_w0(ctx, cfg, st);
    if (es != ERP_OK) return es;
    if (cfg->inlier_thr > 0.0f && !ensure(ctx->inl, erp::inlier_scratch_bytes(sh)))
        return ERP_OUT_OF_MEMORY;
    // plain enqueue: graphs off, stage timing on, the NULL stream, the debug snapshot (its
    // buffer growth synchronises), or a stream the caller is capturing already (the enqueue
    // then becomes part of the caller's graph)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (st != nullptr) ERP_CK(hipStreamIsCapturing(st, &cap));
    if (!ctx->use_graphs || ctx->profiling || st == nullptr || ctx->opt[ERP_OPT_DEBUG_SNAP] ||
        cap != hipStreamCaptureStatusNone)
        return batch_enqueue(ctx, b, ratio, cfg, out, sh, matches, st);
    // graph replay: the same call (structs, buffers, scratch) as a captured one -> one launch
    std::vector<uint8_t> key = graph_key(ctx, b, ratio, cfg, out);
    for (auto& g : ctx->graphs)
        if (g.key == key) {
            g.used = ++ctx->graph_clock;
            ERP_CK(hipGraphLaunch(g.exec, st));
            return ERP_OK;
        }
    ERP_CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    es = batch_enqueue(ctx, b, ratio, cfg, out, sh, matches, st);
    hipGraph_t graph = nullptr;
    const hipError_t ce = hipStreamEndCapture(st, &graph);
    if (es != ERP_OK || ce != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return es != ERP_OK ? es : ERP_HIP_ERROR;
    }
    hipGraphExec_t exec = nullptr;
    const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ie != hipSuccess) return ERP_HIP_ERROR;
    if (ctx->graphs.size() >= 8) {  // drop the least recently used
        auto lru = std::min_element(ctx->graphs.begin(), ctx->graphs.end(),
                                    [](const auto& x, const auto& y) { return x.used < y.used; });
        (void)hipGraphExecDestroy(lru->exec);
        ctx->graphs.erase(lru);
    }
    ctx->graphs.push_back({std::move(key), exec, ++ctx->graph_clock});
    ERP_CK(hipGraphLaunch(exec, st));
    return ERP_OK;
}

erp_status erp_match_knn2_ratio(erp_ctx* ctx, const float* d_query, int32_t nq,
                                const float* d_train, int32_t nt, int32_t dim, float ratio,
                                erp_dmatch* d_out, int32_t* d_count, void* stream) {
    if (!ctx || nq < 0 || nt < 0 || dim != erp::kDim || !d_out || !d_count) return ERP_INVALID_ARG;
    if (nq > 0 && (!d_query || !d_train)) return ERP_INVALID_ARG;
    if (nq > 0 && nt < 2) return ERP_TOO_FEW_POINTS;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    if (nq == 0) {
        ERP_CK(hipMemsetAsync(d_count, 0, 4, st));
        return ERP_OK;
    }
    const erp::BatchShape sh = make_shape(1, nq, nt, 1, 0.25);
    if (!ensure_matcher(ctx, sh) || !ensure(ctx->off, 4 * sizeof(int64_t)) ||
        !ensure(ctx->flags, 16))
        return ERP_OUT_OF_MEMORY;
    ERP_CK(erp::launch_set_i64x4((int64_t*)ctx->off.p, 0, nq, 0, nt, st));
    const int64_t* oq = (const int64_t*)ctx->off.p;
    return run_matcher(ctx, d_query, d_train, oq, oq + 2, sh, ratio, d_out, d_count,
                       (int32_t*)ctx->flags.p, st);
}

erp_status erp_match_two_image(erp_ctx* ctx, const float* h_desc1, int32_t n1, const float* h_desc2,
                               int32_t n2, int32_t dim, erp_dmatch* h_out, int32_t* h_count) {
    if (!ctx || n1 < 0 || n2 < 0 || dim != erp::kDim || !h_out || !h_count) return ERP_INVALID_ARG;
    if (n1 > 0 && (!h_desc1 || !h_desc2)) return ERP_INVALID_ARG;
    if (n1 > 0 && n2 < 2) return ERP_TOO_FEW_POINTS;
    *h_count = 0;
    if (n1 == 0) return ERP_OK;
    // one lock across upload, match and download: the staging buffers are the context's
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ERP_CK(hipSetDevice(ctx->device));
    if (!ensure(ctx->in_a, (size_t)n1 * dim * 4) || !ensure(ctx->in_b, (size_t)n2 * dim * 4) ||
        !ensure(ctx->in_c, (size_t)n1 * sizeof(erp_dmatch) + 16))
        return ERP_OUT_OF_MEMORY;
    ERP_CK(hipMemcpy(ctx->in_a.p, h_desc1, (size_t)n1 * dim * 4, hipMemcpyHostToDevice));
    ERP_CK(hipMemcpy(ctx->in_b.p, h_desc2, (size_t)n2 * dim * 4, hipMemcpyHostToDevice));
    int32_t* d_count = (int32_t*)((char*)ctx->in_c.p + (size_t)n1 * sizeof(erp_dmatch));
    erp_status s = erp_match_knn2_ratio(ctx, (const float*)ctx->in_a.p, n1, (const float*)ctx->in_b.p,
                                        n2, dim, 0.3f, (erp_dmatch*)ctx->in_c.p, d_count, nullptr);
    if (s != ERP_OK) return s;
    ERP_CK(hipDeviceSynchronize());
    int32_t m = 0;
    ERP_CK(hipMemcpy(&m, d_count, 4, hipMemcpyDeviceToHost));
    if (m > 0) ERP_CK(hipMemcpy(h_out, ctx->in_c.p, (size_t)m * sizeof(erp_dmatch), hipMemcpyDeviceToHost));
    *h_count = m;
    return ERP_OK;
}

erp_status erp_eight_point_find_dev(erp_ctx* ctx, int32_t W, int32_t H, const erp_point2f* d_kl,
                                    const erp_point2f* d_kr, int32_t m, const erp_ransac_cfg* cfg,
                                    erp_pair_result* d_result, erp_hypothesis* d_hyps,
                                    void* stream) {
    if (!ctx || W <= 0 || H <= 0 || m < 0 || m > 65535 || !d_result || !cfg_ok(cfg) ||
        !sampler_m_ok(cfg, m))
        return ERP_INVALID_ARG;
    if (m > 0 && (!d_kl || !d_kr)) return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    const erp::BatchShape sh = make_shape(1, m, m, cfg->iters, cfg->sample_frac);
    erp_batch_outputs out{};
    out.results = d_result;
    out.hyps = d_hyps;
    erp_status es = ensure_estimator(ctx, sh, &out);
    if (es != ERP_OK) return es;
    es = upload_w0(ctx, cfg, st);
    if (es != ERP_OK) return es;
    ERP_CK(hipMemsetAsync(ctx->flags.p, 0, 4, st));
    ERP_CK(erp::launch_set_i32((int32_t*)ctx->counts.p, m, st));
    {
        StageTimer _t(ctx, ERP_STAGE_BEARINGS, st);
        ERP_CK(erp::launch_bearings_direct(d_kl, d_kr, m, W, H, (double*)ctx->pts.p, st));
    }
    return run_estimator(ctx, sh, cfg, &out, d_result, st);
}

erp_status erp_eight_point_hypotheses_dev(erp_ctx* ctx, int32_t W, int32_t H,
                                          const erp_point2f* d_kl, const erp_point2f* d_kr,
                                          int32_t m, const erp_ransac_cfg* cfg,
                                          erp_hypothesis* d_hyps, void* stream) {
    if (!ctx || W <= 0 || H <= 0 || m < 0 || m > 65535 || !d_hyps || !cfg_ok(cfg) ||
        !sampler_m_ok(cfg, m))
        return ERP_INVALID_ARG;
    if (m > 0 && (!d_kl || !d_kr)) return ERP_INVALID_ARG;
    if ((int32_t)(m * cfg->sample_frac) < 1) return ERP_TOO_FEW_POINTS;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    const erp::BatchShape sh = make_shape(1, m, m, cfg->iters, cfg->sample_frac);
    erp_batch_outputs out{};
    out.hyps = d_hyps;
    erp_status es = ensure_estimator(ctx, sh, &out);
    if (es != ERP_OK) return es;
    es = upload_w0(ctx, cfg, st);
    if (es != ERP_OK) return es;
    ERP_CK(hipMemsetAsync(ctx->flags.p, 0, 4, st));
    ERP_CK(erp::launch_set_i32((int32_t*)ctx->counts.p, m, st));
    {
        StageTimer _t(ctx, ERP_STAGE_BEARINGS, st);
        ERP_CK(erp::launch_bearings_direct(d_kl, d_kr, m, W, H, (double*)ctx->pts.p, st));
    }
    return run_hypotheses(ctx, sh, cfg, &out, st);
}

erp_status erp_consensus_dev(erp_ctx* ctx, const float* d_rvec, const float* d_tvec, int32_t K,
                             double trim_lo, double trim_hi, erp_pair_result* d_result,
                             void* stream) {
    if (!ctx || K < 0 || !d_result || (K > 0 && (!d_rvec || !d_tvec)) || trim_lo < 0 ||
        trim_hi > 1 || trim_lo > trim_hi)
        return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    erp_ransac_cfg cfg;
    erp_ransac_cfg_default(&cfg);
    cfg.trim_lo = trim_lo;
    cfg.trim_hi = trim_hi;
    cfg.iters = std::max((K + 1) / 2, 1);
    const erp::BatchShape sh = make_shape(1, 1, 1, cfg.iters, cfg.sample_frac);
    erp_status es = ensure_estimator(ctx, sh, nullptr);
    if (es != ERP_OK) return es;
    ERP_CK(erp::launch_consensus_input(d_rvec, d_tvec, K, 2 * sh.iters, (float*)ctx->rv.p,
                                       (float*)ctx->tv.p, (int32_t*)ctx->kcount.p,
                                       (float*)ctx->dscale.p, (int32_t*)ctx->flags.p, st));
    return run_consensus(ctx, sh, &cfg, nullptr, d_result, st, false);
}

erp_status erp_consensus_hyps_dev(erp_ctx* ctx, int32_t m, const erp_hypothesis* d_hyps,
                                  int32_t n_hyps, const erp_ransac_cfg* cfg,
                                  erp_pair_result* d_result, void* stream) {
    if (!ctx || m < 0 || m > 65535 || n_hyps < 1 || !d_hyps || !d_result || !cfg_ok(cfg))
        return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    const erp::BatchShape sh = make_shape(1, std::max(m, 1), std::max(m, 1), n_hyps,
                                          cfg->sample_frac);
    erp_batch_outputs out{};
    out.hyps = const_cast<erp_hypothesis*>(d_hyps);  // read only by the consensus stages
    erp_status es = ensure_estimator(ctx, sh, &out);
    if (es != ERP_OK) return es;
    ERP_CK(hipMemsetAsync(ctx->flags.p, 0, 4, st));
    ERP_CK(erp::launch_set_i32((int32_t*)ctx->counts.p, m, st));
    return run_consensus(ctx, sh, cfg, &out, d_result, st, true);
}

erp_status erp_consensus_hyps_shard_dev(erp_ctx* ctx, int32_t m, const erp_hypothesis* d_hyps,
                                        int32_t n_hyps, const erp_ransac_cfg* cfg, int32_t shard,
                                        int32_t nshards, double* d_lb, double* d_ub,
                                        int32_t* d_bsel, void* stream) {
    if (!ctx || m < 0 || m > 65535 || n_hyps < 1 || !d_hyps || !cfg_ok(cfg) || nshards < 1 ||
        shard < 0 || shard >= nshards || !d_lb || !d_ub || !d_bsel)
        return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    const erp::BatchShape sh = make_shape(1, std::max(m, 1), std::max(m, 1), n_hyps,
                                          cfg->sample_frac);
    erp_batch_outputs out{};
    out.hyps = const_cast<erp_hypothesis*>(d_hyps);
    erp_status es = ensure_estimator(ctx, sh, &out);
    if (es != ERP_OK) return es;
    const size_t rows = 2 * (size_t)n_hyps;
    ERP_CK(hipMemsetAsync(d_lb, 0, rows * 8, st));
    ERP_CK(hipMemsetAsync(d_ub, 0, rows * 8, st));
    ERP_CK(hipMemsetAsync(d_bsel, 0, rows * 8, st));
    ERP_CK(hipMemsetAsync(ctx->flags.p, 0, 4, st));
    ERP_CK(erp::launch_set_i32((int32_t*)ctx->counts.p, m, st));
    return run_consensus(ctx, sh, cfg, &out, nullptr, st, true, 1, shard, nshards, d_lb, d_ub,
                         d_bsel);
}

erp_status erp_consensus_hyps_finish_dev(erp_ctx* ctx, int32_t m, const erp_hypothesis* d_hyps,
                                         int32_t n_hyps, const erp_ransac_cfg* cfg, double* d_lb,
                                         double* d_ub, int32_t* d_bsel, erp_pair_result* d_result,
                                         void* stream) {
    if (!ctx || m < 0 || m > 65535 || n_hyps < 1 || !d_hyps || !cfg_ok(cfg) || !d_lb || !d_ub ||
        !d_bsel || !d_result)
        return ERP_INVALID_ARG;
    ERP_CK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    CtxCall call(ctx, st);
    const erp::BatchShape sh = make_shape(1, std::max(m, 1), std::max(m, 1), n_hyps,
                                          cfg->sample_frac);
    erp_batch_outputs out{};
    out.hyps = const_cast<erp_hypothesis*>(d_hyps);
    erp_status es = ensure_estimator(ctx, sh, &out);
    if (es != ERP_OK) return es;
    return run_consensus(ctx, sh, cfg, &out, d_result, st, true, 2, 0, 1, d_lb, d_ub, d_bsel);
}

erp_status erp_eight_point_find(erp_ctx* ctx, int32_t W, int32_t H, const erp_point2f* h_kl,
                                const erp_point2f* h_kr, int32_t m, const erp_ransac_cfg* cfg,
                                float R_out[3], float T_out[3], erp_pair_result* h_result) {
    if (!ctx || m < 0 || (m > 0 && (!h_kl || !h_kr))) return ERP_INVALID_ARG;
    // one lock across upload, find and download: the staging buffers are the context's
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ERP_CK(hipSetDevice(ctx->device));
    if (!ensure(ctx->in_a, (size_t)m * 8 + 8) || !ensure(ctx->in_b, (size_t)m * 8 + 8) ||
        !ensure(ctx->in_c, sizeof(erp_pair_result)))
        return ERP_OUT_OF_MEMORY;
    if (m > 0) {
        ERP_CK(hipMemcpy(ctx->in_a.p, h_kl, (size_t)m * 8, hipMemcpyHostToDevice));
        ERP_CK(hipMemcpy(ctx->in_b.p, h_kr, (size_t)m * 8, hipMemcpyHostToDevice));
    }
    erp_status s = erp_eight_point_find_dev(ctx, W, H, (const erp_point2f*)ctx->in_a.p,
                                            (const erp_point2f*)ctx->in_b.p, m, cfg,
                                            (erp_pair_result*)ctx->in_c.p, nullptr, nullptr);
    if (s != ERP_OK) return s;
    erp_pair_result r;
    ERP_CK(hipMemcpy(&r, ctx->in_c.p, sizeof(r), hipMemcpyDeviceToHost));
    if (h_result) *h_result = r;
    if (R_out)
        for (int k = 0; k < 3; k++) R_out[k] = r.R[k];
    if (T_out)
        for (int k = 0; k < 3; k++) T_out[k] = r.T[k];
    return (erp_status)r.status;
}

erp_status erp_initial_guess(erp_ctx* ctx, const double* h_bl, const double* h_br, int32_t m,
                             const erp_ransac_cfg* cfg, float R_out[3], float T_out[3],
                             erp_pair_result* h_result) {
    if (!ctx || m < 0 || m > 65535 || (m > 0 && (!h_bl || !h_br)) || !cfg_ok(cfg) ||
        !sampler_m_ok(cfg, m))
        return ERP_INVALID_ARG;
    erp_pair_result r;
    {
        ERP_CK(hipSetDevice(ctx->device));
        HostCtxCall call(ctx);
        const erp::BatchShape sh = make_shape(1, m, m, cfg->iters, cfg->sample_frac);
        erp_status es = ensure_estimator(ctx, sh, nullptr);
        if (es != ERP_OK) return es;
        if (!ensure(ctx->in_c, sizeof(erp_pair_result))) return ERP_OUT_OF_MEMORY;
        es = upload_w0(ctx, cfg, nullptr);
        if (es != ERP_OK) return es;
        std::vector<double> pts((size_t)(m + 1) * 6, 0.0);
        for (int32_t i = 0; i < m; i++)
            for (int k = 0; k < 3; k++) {
                pts[(size_t)i * 6 + k] = h_bl[(size_t)i * 3 + k];
                pts[(size_t)i * 6 + 3 + k] = h_br[(size_t)i * 3 + k];
            }
        ERP_CK(hipMemcpy(ctx->pts.p, pts.data(), (size_t)(m + 1) * 48, hipMemcpyHostToDevice));
        ERP_CK(hipMemcpy(ctx->counts.p, &m, 4, hipMemcpyHostToDevice));
        ERP_CK(hipMemset(ctx->flags.p, 0, 4));
        es = run_estimator(ctx, sh, cfg, nullptr, (erp_pair_result*)ctx->in_c.p, nullptr);
        if (es != ERP_OK) return es;
        ERP_CK(hipMemcpy(&r, ctx->in_c.p, sizeof(r), hipMemcpyDeviceToHost));
    }
    if (h_result) *h_result = r;
    if (R_out)
        for (int k = 0; k < 3; k++) R_out[k] = r.R[k];
    if (T_out)
        for (int k = 0; k < 3; k++) T_out[k] = r.T[k];
    return (erp_status)r.status;
}

erp_status erp_eight_point_estimation(erp_ctx* ctx, const double* h_bl, const double* h_br,
                                      int32_t m, erp_hypothesis* h_out) {
    if (!ctx || m < 0 || !h_out || (m > 0 && (!h_bl || !h_br))) return ERP_INVALID_ARG;
    if (m < 1) return ERP_TOO_FEW_POINTS;
    ERP_CK(hipSetDevice(ctx->device));
    HostCtxCall call(ctx);
    if (!ensure(ctx->in_d, (size_t)m * 48 + 36 * 8 * 2 + sizeof(erp_hypothesis) + 64))
        return ERP_OUT_OF_MEMORY;
    std::vector<double> pts((size_t)m * 6);
    for (int32_t i = 0; i < m; i++)
        for (int k = 0; k < 3; k++) {
            pts[(size_t)i * 6 + k] = h_bl[(size_t)i * 3 + k];
            pts[(size_t)i * 6 + 3 + k] = h_br[(size_t)i * 3 + k];
        }
    char* base = (char*)ctx->in_d.p;
    double* d_pts = (double*)base;
    double* d_gram = (double*)(base + (size_t)m * 48);
    double* d_gfin = (double*)(base + (size_t)m * 48 + 36 * 8);
    int32_t* d_cnt = (int32_t*)(base + (size_t)m * 48 + 36 * 8 * 2);
    erp_hypothesis* d_h = (erp_hypothesis*)(base + (size_t)m * 48 + 36 * 8 * 2 + 16);
    ERP_CK(hipMemcpy(d_pts, pts.data(), pts.size() * 8, hipMemcpyHostToDevice));
    ERP_CK(hipMemcpy(d_cnt, &m, 4, hipMemcpyHostToDevice));
    ERP_CK(erp::launch_gram_all(d_pts, m, d_gram, nullptr));
    erp::BatchShape sh = make_shape(1, m, m, 1, 1.0);
    ERP_CK(erp::launch_eigen(d_cnt, d_gram, sh, 1.0, 1.57, d_gfin, d_h, nullptr));
    ERP_CK(hipMemcpy(h_out, d_h, sizeof(erp_hypothesis), hipMemcpyDeviceToHost));
    return ERP_OK;
}

}  // extern "C"

// debug (ERP_ALLOC_PAD): buffers whose canary bytes were overwritten, reported on stderr;
// returns their number (0 without ERP_ALLOC_PAD)
extern "C" int erp_debug_lip_counters(uint32_t* out64) { return erp::debug_lip_counters(out64); }

extern "C" int erp_debug_check_pads(void) {
    const size_t pad = alloc_pad();
    if (!pad) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    std::lock_guard<std::mutex> g(g_pad_mu);
    std::vector<unsigned char> h(pad);
    int bad = 0;
    for (auto& e : g_padded) {
        if (hipMemcpy(h.data(), (char*)e.first + e.second, pad, hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        size_t first = pad, last = 0;
        for (size_t i = 0; i < pad; i++)
            if (h[i] != 0xA5) first = std::min(first, i), last = i;
        if (first < pad) {
            bad++;
            fprintf(stderr, "erp_debug_check_pads: buffer of %zu bytes at %p: canary bytes %zu .. %zu overwritten\n",
                    e.second, e.first, first, last);
        }
    }
    return bad;
}

// debug (context option ERP_OPT_DEBUG_SNAP = 1): the last run's snapshot (lb [P][2 iters] f64,
// ub, first-stage counts [P] i32) into host memory; returns the snapshot's size in bytes (0: none)
extern "C" long long erp_debug_snapshot(erp_ctx* ctx, void* host, size_t bytes) {
    if (!ctx || !ctx->snap_bytes) return 0;
    if (host && bytes >= ctx->snap_bytes) {
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        if (hipMemcpy(host, ctx->snap.p, ctx->snap_bytes, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    }
    return (long long)ctx->snap_bytes;
}
