// specdec_kernels.hip — fused speculative verify/accept/resample for MI355X (gfx950).
//
// One verify step (sd_verify) is a short chain of memory-bound kernels on one stream,
// with no host sync and no allocation.
//
// PHILOX (perf) mode — two launches:
//   k_stats<TAIL>   grid (span, row): per-span max / Σexp of the processed row -> partials.
//                   The last workgroup of each sequence (agent-scope counter) then decides it:
//                   row stats, p(x_i)/q(x_i), the accept walk -> Decision, prune lengths.
//   k_sample        grid (chunk, B): per-chunk Σ weight of the row to sample — (p_n - q_n)+
//                   (residual) or p (bonus / p-row) — then the last workgroup of each sequence
//                   draws the token by inverse CDF (fp64 scan inside one chunk), writes the
//                   outputs and applies the engine state.  Greedy rows take an exact argmax.
//
// STREAM (parity) mode keeps the reference's serial noise order:
//   k_stats -> k_decide (grid B) -> k_walk (serial over rows) -> k_resample (exponential race
//   with exact candidates, torch's own words) -> k_finalize.
//
// k_threshold (top-k / nucleus rows only) runs first in both modes.  Every logit row is read
// once by k_stats (the algorithmic bytes); the sampling pass re-reads at most two rows per
// sequence (served from the 256 MiB Infinity Cache).  See DESIGN.md.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <map>
#include <tuple>
#include <atomic>
#include <mutex>
#include <type_traits>

#include "sd_device.h"

namespace sd {

constexpr int kMaxCand = 8;
// The decide tails' register-held slot loops are sized for γ <= 16 (kFastSlots target rows, 2γ + 1
// rows per sequence); larger γ (<= SD_MAX_GAMMA) loops over groups of that size or takes the general
// path (decide_seq's seq_stats branch).
constexpr int kFastSlots = 17;

struct Decision {
    int32_t n;          // accepted drafts
    int32_t mode;       // kModeNone / Bonus / Resid / PRow
    int32_t slot;       // target slot sampled from (bonus: gamma, resid/prow: n)
    int32_t status;     // SD_ROW_* bits
    int64_t noise_off;  // STREAM: word offset of the Exp noise; PHILOX: unused
    int32_t stop_index;
    int32_t pad;
    float2 mst, msd;    // PHILOX: (max, Σexp) of the target / drafter row sampled from (k_sample)
};
enum { kModeNone = 0, kModeBonus = 1, kModeResid = 2, kModePRow = 3 };

struct ResPart {
    float sum;                 // Σ residual over the chunk
    float wmax;                // max residual / E
    int32_t ncand;             // candidates kept (> kMaxCand => overflow)
    float pval;                // argmax value (bonus / p-row / engine p fallback); perf: Σ p
    int32_t pidx;              // its index; perf stochastic: the chunk's own inverse-CDF pick
    float cres[kMaxCand];      // candidate residual value
    float ce[kMaxCand];        // candidate noise value
    int32_t cidx[kMaxCand];
};

struct Plan {
    int32_t B, gamma, V, rule;
    int32_t n_tslots, n_dslots, slots, n_chunks, chunk;
    int32_t rn_chunks, rchunk;   // chunking of the resample / sample passes
    int32_t tdt, ddt, draft_is_probs, skip_adj;
    int32_t t_keep, d_keep, t_stoch, n_stop;
    float tT, dT;
    const void* trow[SD_MAX_GAMMA + 1];
    int64_t tstride;
    const void* drow[SD_MAX_GAMMA];
    int64_t dstride;
    const int64_t* draft_tokens;
    int64_t tok_stride;
    const int64_t* stops;
    const uint8_t* active;
    sd_noise noise;
    // outputs
    int32_t* n_accepted;
    int64_t* next_token;
    int64_t next_token_stride;
    float* resample_mass;
    int32_t* prune_drafter;
    int32_t* prune_target;
    int32_t* stop_index;
    int32_t* row_status;
    int64_t* words_used;
    float* token_prob;
    float2* row_stats;          // sd_sample: (max, Σexp) of each processed row (nullable)
    const float2* dstats;       // sd_verify: drafter row stats from sd_sample (nullable)
    int64_t dstats_stride;      // element (d, b) at dstats[d * dstats_stride + b]
    int32_t stat_slots;         // slots whose stats k_stats computes (the rest come from dstats)
    const RowKeep* dkeep;       // sd_verify: drafter keep predicates from sd_sample, at dstats' layout (nullable)
    RowKeep* keep_out;          // sd_sample: each row's keep predicate out (nullable)
    int64_t* generated;
    int64_t gen_stride;
    int32_t step;
    uint8_t* finished;
    int64_t* accepted_count;
    // workspace
    float2* part;
    float2* rowstat;
    RowKeep* keep;
    float* rp;
    float* rq;
    Decision* dec;
    ResPart* rpart;
    uint4* srec;          // k_stats' poll-mode records: rpart, or past the sampler's records (k_verify_lean)
    uint4* sprec;         // sampling-chunk records {Σw, Σp, candidate, tag} (sample_chunk): rpart, or past srec (fused)
    uint4* drec;          // fused verify: per sequence two tagged decision records for its samplers
    uint4* crec;          // fused verify, split records: the chunks' candidates, apart from their totals
    int32_t n_samp;       // fused verify (k_stats<.., SAMP>): sampling workgroups per sequence
    int32_t samp_cps;     //   chunks (of rchunk elements) each sampling workgroup draws: 2, 4 or 8
    int32_t ticket;       // fused verify, any batch: work items by arrival ticket (fused_role), not block id
    int32_t lag;          //   ticket mode: a sequence's samplers come after the spans of the label's lag-th next
    int32_t labels;       //   ticket mode: label = block id % labels, one ticket counter and one sequence set each
    uint32_t* ticket_ctr; //   ticket mode: the labels' ticket counters (kCntStride apart; zero between launches)
    int32_t* keep_hist;   // threshold scratch
    uint32_t* thr_part;   // 16-bit thresholds (sd_threshold.inc): per (row, slice) max key | NaN-inf flag
    float* thr_tail;      //   per (row, slice) Σexp below the window / tie counts
    int32_t* thr_hist;    //   per-row key histogram (global atomics)
    int32_t* thr_shist;   //   poll mode: every (row, slice)'s own histogram window (the decider's tie counts)
    struct ThrRow* thr;   //   per-row tie request
    uint32_t* cnt;        // per-sequence arrival counters (seq_counter): set 0 k_stats, set 1 k_sample
    uint64_t* ts;         // SD_PHASE_TIMING builds only: per-workgroup phase timestamps
    int32_t coh;          // partials may come from the same launch: read them agent-coherently
    int32_t xcd_affine;   // B % 8 == 0: all workgroups of sequence b share XCD group b % 8
    int32_t spoll;       // k_sample (stochastic tails): poll-mode finish (tagged chunk records, no counter)
    int32_t kpoll;        // k_stats (decide tail): poll-mode partials (tagged records, no counter)
    int32_t thr_poll;     // k_thr_hist: slice maxima exchanged in-launch (no k_thr_max launch)
    uint32_t call_nonce;  // sd_verify: per-call value mixed into the sequence epoch (seq_epoch)
    int32_t spin_limit;   // poll modes: re-reads before a record counts as lost (sd_set_poll_policy)
    int32_t* status_or;   // caller's sticky error word (nullable): every row's SD_ROW_ERROR_MASK bits
    int64_t* row_counts;  // sd_verify (nullable): per row += (accepted n, tokens emitted)
    // sd_ngram_verify (sd_ngram.inc)
    struct NgPart* ngpart;
    int64_t* filler_ids;
    int64_t filler_stride;
    int32_t filler_k;
    int32_t filler_pass;    // filler top-K in passes of kNgMaxK: this launch's pass (> 0: filler only)
    int32_t filler_kp;      //   ids this pass selects, <= kNgMaxK
    float2* ng_thr;         //   per row: the last id the previous pass took (value, index bits)
};

// Phase timestamps (diagnostic builds, -DSD_PHASE_TIMING): thread 0 of workgroup `wg` records
// s_memrealtime (100 MHz) at phase `ph`; k_stats workgroups at [0, 8192), k_sample at 8192+.
#ifdef SD_PHASE_TIMING
#define SD_TS(wg, ph)                                                                          \
    do {                                                                                       \
        if (threadIdx.x == 0 && P.ts) {                                                        \
            P.ts[(size_t)(wg) * 16 + (ph)] = __builtin_amdgcn_s_memrealtime();                 \
            if ((wg) >= 8192 && ((ph) == 4 || (ph) == 10)) P.ts[(size_t)(wg) * 16 + 12 + ((ph) == 10)] = __builtin_amdgcn_s_memtime(); \
            if ((wg) >= 8192 && ((ph) == 1 || (ph) == 2)) P.ts[(size_t)(wg) * 16 + 14 + ((ph) == 2)] = __builtin_amdgcn_s_memtime(); \
        }                                                                                      \
    } while (0)
// ticket mode: the work item a workgroup drew, one int64 per block id after the stamp table
#define SD_TS_ROLE(wg, v)                                                                      \
    do {                                                                                       \
        if (threadIdx.x == 0 && P.ts && (wg) < 32768) P.ts[(size_t)32768 * 16 + (wg)] = (v);   \
    } while (0)
#else
#define SD_TS(wg, ph) \
    do {              \
        (void)(wg);   \
    } while (0)
#define SD_TS_ROLE(wg, v) \
    do {                  \
        (void)(wg);       \
    } while (0)
#endif

// Arrival counters live in a fixed block at the front of every workspace layout, so calls with
// different shapes sharing one workspace never overwrite them.  They are zero between calls
// (the last arriving workgroup resets its counter); the workspace must be zero-filled once.
// One counter per 128-byte line: device-scope atomics execute beyond the per-XCD L2, and
// counters sharing a line would serialise every sequence's arrivals on it.
constexpr int kCntMax = 16384;
constexpr int kTailChunks = 1024;   // perf-mode sampling: chunk partials staged in LDS (V <= 2 Mi)
constexpr int32_t kLostDecision = -2;   // fused verify: a sampler's record when the decision never arrived
constexpr int kCntStride = 32;   // uint32 words per counter (128 B)
__device__ __forceinline__ uint32_t* seq_counter(const uint32_t* base, int set, int b) {
    return const_cast<uint32_t*>(base) + ((size_t)set * kCntMax + b) * kCntStride;
}
// This call's epoch of sequence b (counter set 3), mixed with the call's nonce: a workgroup of an
// earlier call dispatched only after that call's waits gave up (and its epoch moved on) tags its
// records with the earlier nonce, so the next call never takes them as its own.  The counter itself
// only counts up (seq_advance unmixes before the +1), so the replays of a captured graph, which
// share one nonce, never see an epoch again.
__device__ __forceinline__ uint32_t seq_epoch(const Plan& P, int b) {
    return __hip_atomic_load(seq_counter(P.cnt, 3, b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ^ P.call_nonce;
}
__device__ __forceinline__ void seq_advance(const Plan& P, int b, uint32_t epoch) {
    __hip_atomic_store(seq_counter(P.cnt, 3, b), (epoch ^ P.call_nonce) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ const void* row_ptr(const Plan& P, int r, int* dt, float* T, bool* keep) {
    const int b = r / P.slots, s = r - b * P.slots;
    if (s < P.n_tslots) {
        *dt = P.tdt; *T = P.tT; *keep = P.t_keep;
        return static_cast<const char*>(P.trow[s]) + b * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
    }
    *dt = P.ddt; *T = P.dT; *keep = P.d_keep;
    return static_cast<const char*>(P.drow[s - P.n_tslots]) + b * P.dstride * (P.ddt == SD_F32 ? 4 : 2);
}

// row r's keep predicate: the threshold search's, or for a drafter row whose draw returned it
// (sd_verify_args.draft_row_keep) the draw's
__device__ __forceinline__ RowKeep keep_of(const Plan& P, int r) {
    if (P.dkeep) {
        const int b = r / P.slots, s = r - b * P.slots;
        if (s >= P.n_tslots) return P.dkeep[(int64_t)(s - P.n_tslots) * P.dstats_stride + b];
    }
    return P.keep[r];
}

__device__ __forceinline__ bool is_stop(const Plan& P, int64_t tok) {
    for (int k = 0; k < P.n_stop; ++k)
        if (P.stops[k] == tok) return true;
    return false;
}

// The loops' stop scan over the accepted drafts (sampling/speculative_decoding.py:150-152,
// ngram_assisted/ngram_assisted.py:124-126) is nonzero(eq(drafts[1, n], stop_tokens[S, 1]))[0, 1]:
// row-major over [S, n], so the stop token LISTED FIRST that occurs wins, at its first position —
// not the earliest stop position when several listed stops occur.  A draft's stop rank is its
// token's first position in the list (INT_MAX: not a stop); the 8-bit form is rank + 1 (0: not a
// stop), saturating at 255 — then the exact rank is recomputed from the list.
__device__ __forceinline__ int stop_rank(const Plan& P, int64_t tok) {
    for (int k = 0; k < P.n_stop; ++k)
        if (P.stops[k] == tok) return k;
    return INT_MAX;
}
__device__ __forceinline__ uint8_t stop_rank8(const Plan& P, int64_t tok) {
    uint32_t r = 0;
    for (int k = P.n_stop - 1; k >= 0; --k)   // no early exit: the last hit is the first occurrence
        if (P.stops[k] == tok) r = k < 254 ? (uint32_t)k + 1u : 255u;
    return (uint8_t)r;
}
// the rank of draft j from its 8-bit form (the list re-read only for saturated ranks)
__device__ __forceinline__ int stop_rank_of(const Plan& P, uint8_t r8, int64_t tok) {
    return r8 == 0 ? INT_MAX : r8 < 255 ? (int)r8 - 1 : stop_rank(P, tok);
}

// stop list staged in LDS by a tail (nullptr / too many stops: the global list)
constexpr int kLdsStops = 64;
__device__ __forceinline__ bool is_stop_l(const Plan& P, int64_t tok, const int64_t* lstops) {
    if (!lstops || P.n_stop > kLdsStops) return is_stop(P, tok);
    for (int k = 0; k < P.n_stop; ++k)
        if (lstops[k] == tok) return true;
    return false;
}

// SGPR budget of the streaming kernels: <= 80 keeps 8 workgroups of 256 threads resident per CU.
// Overridable for tuning (-DSD_SGPR_CAP_N=n; 0 = the compiler's choice).
#ifndef SD_SGPR_CAP_N
#define SD_SGPR_CAP_N 80
#endif
#if SD_SGPR_CAP_N > 0
#define SD_SGPR_CAP __attribute__((amdgpu_num_sgpr(SD_SGPR_CAP_N)))
#else
#define SD_SGPR_CAP
#endif

// ------------------------------------------------------------------ block helpers
struct FMax {
    static constexpr float kId = -INFINITY;
    __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
struct FSum {
    static constexpr float kId = 0.f;
    __device__ float operator()(float a, float b) const { return a + b; }
};

// Block reductions over the workgroup's waves: nw > 0 names the waves that take part (the
// sampling bodies run in k_verify_lean's four data waves after its helper wave has exited, so
// blockDim would count one wave too many), else every wave of the launch.
template <typename F>
__device__ __forceinline__ float block_reduce(float v, F op, float* lds, int nw = 0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wave_reduce(v, F::kId, op);
    __syncthreads();
    if (lane == 0) lds[w] = v;
    __syncthreads();
    float r = lds[0];
    const int n = nw > 0 ? nw : (int)(blockDim.x >> 6);
    for (int k = 1; k < n; ++k) r = op(r, lds[k]);
    return r;
}

// two sums at once (fixed order)
__device__ __forceinline__ float2 block_reduce2(float2 v, float* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v.x = wave_sum(v.x);
    v.y = wave_sum(v.y);
    __syncthreads();
    if (lane == 0) { lds[2 * w] = v.x; lds[2 * w + 1] = v.y; }
    __syncthreads();
    float2 r = make_float2(lds[0], lds[1]);
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) { r.x += lds[2 * k]; r.y += lds[2 * k + 1]; }
    return r;
}

__device__ __forceinline__ void block_argmax(float& v, int32_t& i, float* ldsv, int32_t* ldsi, int nw = 0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    wave_argmax(v, i);
    __syncthreads();
    if (lane == 0) { ldsv[w] = v; ldsi[w] = i; }
    __syncthreads();
    v = ldsv[0]; i = ldsi[0];
    const int n = nw > 0 ? nw : (int)(blockDim.x >> 6);
    for (int k = 1; k < n; ++k)
        if (arg_better(ldsv[k], ldsi[k], v, i)) { v = ldsv[k]; i = ldsi[k]; }
}


// ------------------------------------------------------------------ k_stats
// grid (span, row-of-group): running max / Σexp of y = round_dt(_process(x)/T) over one span of a
// row, streamed through a 4-deep register pipeline (16 B per lane per stage, 16 KiB per
// workgroup in flight) with an online rescaled sum, so loads stay in flight while exp() runs.
#ifndef SD_STATS_PIPE
#define SD_STATS_PIPE 4
#endif
constexpr int kPipe = SD_STATS_PIPE;
#ifndef SD_TICKET_PIPE
#define SD_TICKET_PIPE 4
#endif
constexpr int kTicketPipe = SD_TICKET_PIPE;   // the ticket-order fused verify's spans
constexpr float kLog2e = 1.44269502162933349609375f;

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    const float mn = fmaxf(m, m2);
    if (mn == -INFINITY) return;
    s = (m > -INFINITY ? s * sd_exp(m - mn) : 0.f) + (m2 > -INFINITY ? s2 * sd_exp(m2 - mn) : 0.f);
    m = mn;
}

// one DPP step of the (max, rescaled sum) wave merge; rows outside ROWS merge the identity
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ void merge_step(float& m, float& s) {
    const float m2 = dpp_f<CTRL, ROWS>(-INFINITY, m), s2 = dpp_f<CTRL, ROWS>(0.f, s);
    online_merge(m, s, m2, s2);
}

__device__ __forceinline__ const void* slot_row(const Plan& P, int b, int s) {
    if (s < P.n_tslots)
        return static_cast<const char*>(P.trow[s]) + b * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
    return static_cast<const char*>(P.drow[s - P.n_tslots]) + b * P.dstride * (P.ddt == SD_F32 ? 4 : 2);
}

__device__ __forceinline__ void fetch_drafted(const Plan& P, int b, int i, int64_t tok, float* xt, float* xd);
__device__ __forceinline__ float draw_uniform(const Plan& P, int b, int i, int64_t woff, bool* overrun);

// What the perf-mode decision needs of draft i, gathered by one thread while the row statistics
// stream: the drafted id and its accept uniform (prologue), its raw target / drafter logits, the
// drafter row's (m, S) when they came with the draws, and its stop flag (after the stream).  Draft
// i belongs to thread (i % nw) * 64 + i / nw — lane k of the wave that reduces target slot i in
// seq_stats — so that wave can test draft i as soon as the slot's statistics are reduced.
struct DraftPf {
    int64_t tok = -1;
    float xt = 0.f, xd = 0.f, u = 0.f;
    float2 ds = make_float2(-INFINITY, 0.f);
    uint8_t stop = 0;   // stop_rank8 of the drafted token
    bool act = true;   // engine rule: the sequence is active (draft 0's thread only)
};
__device__ __forceinline__ int pf_draft(const Plan& P) {
    constexpr int nw = kThreads / kWave;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = lane * nw + w;
    return lane < (P.gamma + nw - 1) / nw && i < P.gamma ? i : -1;
}
__device__ __forceinline__ void pf_early(const Plan& P, int b, int i, DraftPf& pf) {
    if (i >= 0) pf.tok = P.draft_tokens[b * P.tok_stride + i];
}
// after the stream: the loads go out together and the Philox ALU work runs while they (and the
// workgroup's arrival) are in flight
__device__ __forceinline__ void pf_late(const Plan& P, int b, int i, DraftPf& pf) {
    if (i < 0) return;
    fetch_drafted(P, b, i, pf.tok, &pf.xt, &pf.xd);
    if (P.dstats) pf.ds = P.dstats[(int64_t)i * P.dstats_stride + b];
    pf.stop = stop_rank8(P, pf.tok);
    if (i == 0 && P.active) pf.act = P.active[b] != 0;
    bool ovr = false;
    pf.u = draw_uniform(P, b, i, 0, &ovr);   // perf mode: Philox, no stream words
}
template <int DT = -1, bool FAST = false>
__device__ __forceinline__ void decide_seq(const Plan& P, int b, const DraftPf& pf, int wg_id, Decision* out = nullptr,
                           bool publish = true, bool coh = true, const uint32_t* poll_epoch = nullptr);

// Poll-mode tag of k_stats' partial record (slot s, chunk c) of sequence b (k_draw_lean's protocol,
// its own salt; the sequence's epoch lives in counter set 3, shared with k_sample's finish)
__device__ __forceinline__ uint32_t stats_tag(uint32_t epoch, int b, int s, int c) {
    uint32_t h = epoch * 0x9E3779B1u + (uint32_t)b * 0x85EBCA77u + (uint32_t)(s * 4096 + c) * 0xC2B2AE3Du + 0x3C6EF372u;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;   // murmur3 fmix32
    return h | 1u;
}
__device__ __forceinline__ uint4* stats_rec(const Plan& P, int b, int s, int c) {
    return P.srec + ((int64_t)b * P.stat_slots + s) * P.n_chunks + c;
}

// Arrival at a per-sequence counter (thread 0, after storing its partials with st_coh): true for
// the last of `total` arrivals, which also re-arms the counter.  coh_wait() completes the
// coherent stores before the increment; the last arrival reads every partial with ld_coh.
__device__ __forceinline__ bool arrive_last(uint32_t* ctr, uint32_t total) {
    coh_wait();
    const uint32_t prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1u != total) return false;
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// arrive_last for <= 65535 arrivals that each carry a flag (high half of the counter): *any says
// whether some arrival set its flag (written for the last arrival only)
__device__ __forceinline__ bool arrive_last_f(uint32_t* ctr, uint32_t total, bool flag, bool* any) {
    coh_wait();
    const uint32_t add = 1u + (flag ? 0x10000u : 0u);
    const uint32_t now = __hip_atomic_fetch_add(ctr, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
    if ((now & 0xffffu) != total) return false;
    *any = (now >> 16) != 0u;
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// XCD-affine workgroup placement.  Workgroups are dealt round-robin over the 8 XCDs by linear
// block id, so id % 8 labels an XCD group (MI355X_MICROARCH.md, dispatch).  When B % 8 == 0 the
// (sequence, item) of block id is chosen with sequence % 8 == id % 8: every workgroup of a
// sequence — its row-statistics spans, its decision tail, its sampling chunks and their tail —
// runs on one XCD, so the sampler re-reads the rows (and the tails their partials) from that
// XCD's L2.  Placement only affects speed: the exchange protocol never assumes it.
__device__ __forceinline__ void affine_split(int id, int per_seq, int& b, int& item) {
    const int w = id & 7, k = id >> 3;
    b = (k / per_seq) * 8 + w;
    item = k % per_seq;
}

// Ticket mode's schedule within one label (stats_body) over its nb sequences j = 0 .. nb-1: units
// u = 0 .. nb + D - 1; unit u holds sequence u's per_seq items (its spans, then its decider) when
// u < nb, then sequence (u - D)'s ns samplers when u >= D.  Ticket t -> (sequence j, item) or
// (sequence j, sampler samp).
__device__ __forceinline__ void fused_role(int t, int nb, int D, int per_seq, int ns, int& j, int& item, int& samp) {
    const int full = per_seq + ns;
    samp = -1;
    item = 0;
    if (t < D * per_seq) {                       // units 0 .. D-1: spans and deciders only
        j = t / per_seq;
        item = t - j * per_seq;
        return;
    }
    t -= D * per_seq;
    if (t < (nb - D) * full) {                   // units D .. nb-1: both
        const int u = t / full, k = t - u * full;
        if (k < per_seq) { j = D + u; item = k; }
        else { j = u; samp = k - per_seq; }
        return;
    }
    t -= (nb - D) * full;                        // units nb .. nb+D-1: samplers only
    const int u = t / ns;
    j = nb - D + u;
    samp = t - u * ns;
}

#ifndef SD_TAIL_PRIO
#define SD_TAIL_PRIO 1   // s_setprio for the draws' tail wave and the fused verify's decider (B = 32 step -0.35 us)
#endif
constexpr int kMaxSampPairs = 4;   // chunk pairs per fused sampler in ticket order: samp_cps <= 8
#ifndef SD_SAMP_PREFETCH
#define SD_SAMP_PREFETCH 0            // 1: ticket-order samplers load the next chunk pair ahead (93 VGPRs: slower at B = 512)
#endif
template <int DT, bool FAST, int MAXP>
__device__ __forceinline__ void fused_sampler(const Plan& P, int b, int c, int wg_id);
template <int DT, bool FAST>
__device__ __forceinline__ void fused_finish(const Plan& P, int b, const Decision& d, uint32_t epoch, int wg_id);

// <= 80 SGPRs keeps 8 workgroups of 256 threads resident per CU (MI355X_MICROARCH.md, residency)
// TAIL (perf mode): the last workgroup to finish a sequence's rows runs its decision (decide_seq).
// SAMP (perf mode, poll, stochastic target rows): the whole verify in this launch — per sequence
// P.n_samp sampling workgroups poll the decider's decision records, draw their chunk's candidate of
// the decided row and publish it; the decider then polls those records and finishes (the token, the
// outputs, the engine state): no k_sample launch, no kernel boundary, no decision reload.
template <int DT, bool FAST, bool TAIL, bool SAMP, bool TICKET = false>
__device__ __forceinline__ void stats_body(const Plan& P, int slot_lo, int slot_cnt) {
    __shared__ float lm[4], ls[4];
    constexpr int VEC = Elem<DT>::kVec;
    constexpr int STEP = kThreads * VEC;                      // elements per workgroup stage
    const int wg_id = blockIdx.y * gridDim.x + blockIdx.x;
    SD_TS(wg_id, 0);
    // The kernel-argument fields the first row loads depend on, read in one straight-line block (no
    // branch between them, both row tables indexed unconditionally): the scalar loads then go out
    // together with one wait, instead of a chain of ~10 dependent waits that put the first row
    // load ~3 us after the start at batch 1.
    const int gx = P.n_chunks;
    const int xa = P.xcd_affine, nt = P.n_tslots;
    const int64_t tstr = P.tstride, dstr = P.dstride;
    // poll mode (TAIL): a 1-D grid of B x (slot_cnt x n_chunks + 1) workgroups — per sequence its
    // streaming spans and one DECIDER, which streams nothing: it prefetches the drafts' inputs while
    // the spans stream, polls their records and decides.  Counter mode: (n_chunks, B x slot_cnt), the
    // last arrival decides.
    const bool poll = TAIL && P.kpoll;
    const int n_span = slot_cnt * gx;
    const int per_seq = n_span + (poll ? 1 : 0);
    int b, s, chunk;
    bool decider = false;
    int samp = -1;
    if constexpr (SAMP && TICKET) {
        // Ticket mode (any batch; the grid need not be resident): a workgroup's work item is the
        // arrival ticket it takes, not its block id.  The sequences are dealt to `labels` labels
        // (b % labels), and a workgroup serves the label of its block id (id % labels: with labels a
        // multiple of 8 every workgroup of a label — so every item of a sequence — shares one XCD,
        // whose L2 then serves the samplers' re-read of the decided rows), taking the next ticket of
        // that label's own counter (one counter for the whole grid serialised its ~B*49 atomics: 92
        // vs 49 us at B = 128).  Every wait points at an EARLIER ticket of the same label — a decider
        // at its spans, a sampler at its decider — whose holder is already running, so the launch
        // always progresses whatever else holds the CUs; the one wait on later tickets (a decider for
        // its samplers, `lag` sequences on) holds at most lag + 1 workgroups per label.  A label's
        // items run sequence by sequence — spans, decider — with a sequence's samplers after the
        // spans of the label's lag-th next sequence (fused_role), so they rarely sit in slots waiting.
        // Each label has the same workgroup count (ceil(B / labels) sequences' worth); a ticket past
        // the label's real work exits.
        const int NL = P.labels, L = (int)(blockIdx.x % (uint32_t)NL);
        const int nbl = (P.B + NL - 1) / NL, nb = (P.B - L + NL - 1) / NL;
        __shared__ uint32_t s_tk;
        if (threadIdx.x == 0) {
            uint32_t* ctr = P.ticket_ctr + (size_t)L * kCntStride;
            const uint32_t t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the label's last ticket: every other has been taken, re-arm the counter
            if (t + 1u == (uint32_t)nbl * (uint32_t)(per_seq + P.n_samp))
                __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_tk = t;
        }
        __syncthreads();
        if ((int)s_tk >= nb * (per_seq + P.n_samp)) return;   // padding: this label has fewer sequences
        int item, j;
        fused_role((int)s_tk, nb, P.lag < nb ? P.lag : nb, per_seq, P.n_samp, j, item, samp);
        b = L + j * NL;
        decider = samp < 0 && item == n_span;
        s = slot_lo + (samp < 0 && item < n_span ? item / gx : 0);
        chunk = samp < 0 && item < n_span ? item % gx : 0;
        SD_TS_ROLE(wg_id, ((int64_t)s_tk << 32) | ((int64_t)b << 12) |
                              (samp >= 0 ? 0x800 | samp : (decider ? 0x400 : item)));
    } else if (SAMP && !TICKET && wg_id >= P.B * per_seq) {
        // the samplers come after every span and decider in dispatch order (block id): they only wait
        // for a decision, so the spans, which wait for nothing, always get their slots first, and a
        // sampler frees its slot once it has published.  Sequence b = id % B: with B % 8 == 0 every
        // workgroup of a sequence sits on one XCD group (affine_split's rule)
        const int t = wg_id - P.B * per_seq;
        b = t % P.B;
        samp = t / P.B;
        s = slot_lo;
        chunk = 0;
    } else {
        int item;
        if (xa) affine_split(wg_id, per_seq, b, item);
        else { b = wg_id / per_seq; item = wg_id - b * per_seq; }
        decider = poll && item == n_span;
        s = slot_lo + (item < n_span ? item / gx : 0);
        chunk = item < n_span ? item % gx : 0;
    }
    if constexpr (SAMP) {
        if (samp >= 0) {
            fused_sampler<DT, FAST, TICKET ? kMaxSampPairs : 1>(P, b, samp, wg_id);
            return;
        }
    }
    __shared__ uint32_t s_epoch;
    if (TAIL && decider) {
        if (SD_TAIL_PRIO) __builtin_amdgcn_s_setprio(2);   // the sequence's critical path (see k_draw_lean's tail)
        // the drafts' ids, logits, drafter stats, stop flags and accept uniforms while the spans stream
        DraftPf pf;
        const int pi = pf_draft(P);
        pf_early(P, b, pi, pf);
        if (threadIdx.x == 0) s_epoch = seq_epoch(P, b);
        pf_late(P, b, pi, pf);
        __syncthreads();
        SD_TS(wg_id, 7);
        if constexpr (SAMP) {
            __shared__ Decision s_dec;
            const double u_row = uniform_d(cdf_uniform(P.noise, (uint32_t)b));   // the chunk pick's, ahead of the records
            decide_seq<DT, FAST>(P, b, pf, wg_id, &s_dec, true, true, &s_epoch);
            __syncthreads();
            SD_TS(wg_id, 3);
            fused_finish<DT, FAST>(P, b, s_dec, s_epoch, wg_id, u_row);
        } else {
            decide_seq(P, b, pf, wg_id, nullptr, true, true, &s_epoch);
            SD_TS(wg_id, 3);
        }
        if (threadIdx.x == 0)   // every span has read the epoch (its record carries it): advance it
            seq_advance(P, b, s_epoch);
        return;
    }
    const bool is_t = s < nt;
    const char* tp = static_cast<const char*>(P.trow[is_t ? s : 0]);
    const char* dp = static_cast<const char*>(P.drow[is_t ? 0 : s - nt]);
    const int r = b * P.slots + s;
    const void* row = is_t ? tp + b * tstr * (P.tdt == SD_F32 ? 4 : 2) : dp + b * dstr * (P.ddt == SD_F32 ? 4 : 2);
    // poll mode: this call's epoch of sequence b (thread 0), issued AFTER the first row loads and
    // kept in a register until the record: loads complete in order, so an atomic issued first
    // held back the wave's first stage (batch 1: stream done 3.2 vs ~1.4 us after the start)
    const bool ep_thread = poll && threadIdx.x == 0;
    uint32_t ep_reg = 0u;
    bool ep_read = false;
    auto read_epoch = [&]() {
        if (ep_thread && !ep_read) ep_reg = seq_epoch(P, b);
        ep_read = true;
    };
    // TAIL, counter mode: drafted ids now (consumed after the loop), their logits right after it,
    // so a workgroup that turns out to be its sequence's last arrival has them in registers.  Poll
    // mode: the decider prefetches them; the spans only stream
    DraftPf pf;
    const bool pf_here = TAIL && !poll;
    const int pf_i = pf_here ? pf_draft(P) : -1;
    if (TAIL) pf_early(P, b, pf_i, pf);
    const float T = is_t ? P.tT : P.dT;
    const bool has_keep = !FAST && (is_t ? P.t_keep : P.d_keep);
    const RowKeep kp = has_keep ? keep_of(P, r) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    // This workgroup's stages (STEP elements each) of the row: one contiguous span.
    const int nst = (P.V + STEP - 1) / STEP;
    const int spw = P.chunk / STEP;
    const int cnt = chunk * spw < nst ? min(spw, nst - chunk * spw) : 0;
    auto stage_of = [&](int i) -> int64_t { return (int64_t)chunk * spw + i; };
    const int64_t hi = P.V;
    const bool aligned = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
    // the row's last stage is partial when STEP does not divide V: it is this workgroup's last, if any
    const bool last_partial = cnt > 0 && (stage_of(cnt - 1) + 1) * STEP > P.V;
    float m = -INFINITY, acc = 0.f;

    // Terms are exp(y - m) = exp2((y - m) * log2e): subtract, multiply, v_exp_f32.  y - m is exact
    // for bf16/fp16 values (and for fp32 ones within 2^24 of each other); the multiply's rounding
    // gives each term an independent ~|y-m|*6e-8 relative error that averages down in the sum, and
    // no rounded product is shared by all terms, so S carries no common bias.  Consumers compute
    // numerators with the compensated sd_exp and use (m, S) as a pair.
    // The reference m is NOT kept at the running max (a per-element max and a per-vector branch
    // on it cost ~25% of this pass): a vector is summed against the current m, and only when its
    // sum is not below 2^64 — a term more than 44 e-folds above m, the first vector (m = -inf),
    // or an inf / NaN — m is raised to the vector's max, the running sum rescaled and the vector
    // re-summed.  So m may trail the true max by up to 44 and S stays far below fp32 overflow
    // (at most 2^64 per element).  NaN propagates; vectors of -inf only add nothing.
    // CHECKED: the vector may run past the span (ragged tail); full stages skip the bound checks
    auto consume = [&](const float* x, int64_t e0, auto checked) {
        float y[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) y[k] = x[k];
        if constexpr (!FAST) process_vec<DT, VEC>(y, e0, T, has_keep, kp);
        if constexpr (decltype(checked)::value) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) y[k] = e0 + k < hi ? y[k] : -INFINITY;
        }
        float sv = 0.f;
#pragma unroll
        for (int k = 0; k < VEC; ++k) sv += __builtin_amdgcn_exp2f((y[k] - m) * kLog2e);
        if (!(sv < 1.8446744e19f)) {   // 2^64 (rare)
            float vm = -INFINITY;
            bool nan = false;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                vm = fmaxf(vm, y[k]);
                nan |= y[k] != y[k];
            }
            if (vm > m) {
                acc = m > -INFINITY ? acc * sd_exp(m - vm) : 0.f;
                m = vm;
            }
            sv = 0.f;
            if (m > -INFINITY) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) sv += __builtin_amdgcn_exp2f((y[k] - m) * kLog2e);
            }
            if (nan) {   // softmax of a row with a NaN is NaN: make it stick through every merge
                sv = NAN;
                if (!(m > -INFINITY)) m = 0.f;
            }
        }
        acc += sv;
    };
    // steady state: stages where every lane's 16-byte vector is in range.  Loads are issued
    // unconditionally (the prefetch index is clamped), so the compiler keeps kPipe of them in
    // flight with counted vmcnt waits instead of draining to vmcnt(0) each stage.
    const int nfull = aligned ? cnt - (last_partial ? 1 : 0) : 0;
    // the row's ragged last stage (aligned rows): one clamped vector per lane, loaded up front
    const bool vtail = aligned && last_partial && P.V >= VEC;
    const int64_t tail_e0 = vtail ? stage_of(cnt - 1) * STEP + threadIdx.x * VEC : 0;
    uint4 tailv = make_uint4(0u, 0u, 0u, 0u);
    if (vtail) tailv = ld16_clamped<DT>(row, tail_e0, last_whole_vec<DT>(P.V));
    if (nfull > 0) {
        // ticket order (large batches): more vectors in flight per span (SD_TICKET_PIPE)
        constexpr int PIPE = TICKET ? kTicketPipe : kPipe;
        const uint4* vb = reinterpret_cast<const uint4*>(row) + threadIdx.x;   // stage k at vb[k * kThreads]
        uint4 buf[PIPE];
#pragma unroll
        for (int d = 0; d < PIPE; ++d) buf[d] = vb[stage_of(d < nfull ? d : nfull - 1) * kThreads];
        read_epoch();
        int it = 0;
        for (; it + PIPE <= nfull; it += PIPE) {
#pragma unroll
            for (int d = 0; d < PIPE; ++d) {
                const uint4 v = buf[d];
                const int nx = it + d + PIPE;
                buf[d] = vb[stage_of(nx < nfull ? nx : nfull - 1) * kThreads];
                float x[VEC];
                unpack16<DT>(v, x);
                consume(x, stage_of(it + d) * STEP + threadIdx.x * VEC, std::false_type{});
            }
        }
#pragma unroll
        for (int d = 0; d < PIPE; ++d) {
            if (it + d < nfull) {
                float x[VEC];
                unpack16<DT>(buf[d], x);
                consume(x, stage_of(it + d) * STEP + threadIdx.x * VEC, std::false_type{});
            }
        }
    }
    if (vtail) {
        float x[VEC];
        finish16<DT>(tailv, row, tail_e0, P.V, x);
        consume(x, tail_e0, std::true_type{});
    }
    // misaligned rows: guarded element loads
    for (int it = vtail ? cnt : nfull; it < cnt; ++it) {
        const int64_t e0 = stage_of(it) * STEP + threadIdx.x * VEC;
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = (e0 + k < hi) ? load_one<DT>(row, e0 + k) : 0.f;
        consume(x, e0, std::true_type{});
    }
    read_epoch();
    if (ep_thread) s_epoch = ep_reg;
    SD_TS(wg_id, 6);
    if (TAIL) pf_late(P, b, pf_i, pf);
    SD_TS(wg_id, 7);
    // workgroup combine (fixed order): the wave's max, every lane's sum rescaled to it, one wave sum;
    // then the 4 waves through LDS.  A NaN sum stays NaN; lanes of only -inf add nothing.
    {
        const float mw = wave_max(m);
        const float sc = m > -INFINITY ? acc * sd_exp(m - mw) : (acc != acc ? acc : 0.f);
        acc = wave_sum(sc);
        m = mw;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { lm[w] = m; ls[w] = acc; }
    __syncthreads();
    SD_TS(wg_id, 1);
    // poll mode (TAIL): one tagged 16-byte record per (slot, span), polled by the sequence's decider
    // — no counter.  Counter mode: the (m, S) partial and an arrival; the last arrival decides.
    if (threadIdx.x == 0) {
        constexpr int NW = kThreads / kWave;
        float M = lm[0];
#pragma unroll
        for (int k = 1; k < NW; ++k) M = fmaxf(M, lm[k]);
        float S = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) S += lm[k] > -INFINITY ? ls[k] * sd_exp(lm[k] - M) : (ls[k] != ls[k] ? ls[k] : 0.f);
        if (poll)
            st_coh16(stats_rec(P, b, s, chunk), make_uint4(__float_as_uint(M), __float_as_uint(S),
                                                           stats_tag(s_epoch, b, s, chunk), 0u));
        else
            st_coh(P.part + (int64_t)r * P.n_chunks + chunk, make_float2(M, S));
    }
    SD_TS(wg_id, 8);
    if constexpr (TAIL) {
        if (poll) return;   // the decider takes it from the records
        __shared__ int s_last;
        if (threadIdx.x == 0) s_last = arrive_last(seq_counter(P.cnt, 0, b), (uint32_t)(P.stat_slots * P.n_chunks));
        __syncthreads();
        SD_TS(wg_id, 2);
        if (!s_last) return;
        decide_seq(P, b, pf, wg_id, nullptr, true, true, nullptr);
        SD_TS(wg_id, 3);
    }
}

template <int DT, bool FAST, bool TAIL>
__global__ void __launch_bounds__(kThreads) SD_SGPR_CAP k_stats(Plan P, int slot_lo, int slot_cnt) {
    stats_body<DT, FAST, TAIL, false>(P, slot_lo, slot_cnt);
}

// The fused verify (stats_body with SAMP): grid = B x (spans + decider) then B x n_samp samplers (two
// 2048-element chunks each)
#ifndef SD_FUSED_VGPR
#define SD_FUSED_VGPR 0
#endif
#if SD_FUSED_VGPR > 0
#define SD_FUSED_VGPR_CAP __attribute__((amdgpu_waves_per_eu(SD_FUSED_VGPR)))
#else
#define SD_FUSED_VGPR_CAP
#endif
// TICKET: the ticket-order layout (fused_role; any batch): its own instantiation, so the block-id
// kernel of small batches carries neither the ticket code nor the multi-chunk samplers' registers
template <int DT, bool FAST, bool TICKET>
__global__ void __launch_bounds__(kThreads) SD_SGPR_CAP SD_FUSED_VGPR_CAP k_verify_fused(Plan P, int slot_lo, int slot_cnt) {
    stats_body<DT, FAST, true, true, TICKET>(P, slot_lo, slot_cnt);
}

// combine the chunk partials of row r (one wave)
__device__ __forceinline__ float2 combine_row(const Plan& P, int r) {
    const int lane = threadIdx.x & 63;
    const float2* pr = P.part + (int64_t)r * P.n_chunks;
    float m = -INFINITY;
    for (int c = lane; c < P.n_chunks; c += kWave) m = fmaxf(m, ld_coh(pr + c).x);
    m = wave_max(m);
    // fixed-order sum: lane-strided partial sums, then a fixed butterfly
    float s = 0.f;
    for (int c = lane; c < P.n_chunks; c += kWave) {
        const float2 v = ld_coh(pr + c);
        if (v.x > -INFINITY) s += v.y * sd_exp(v.x - m);
    }
    s = wave_sum(s);
    return make_float2(m, s);
}

template <int DT>
__device__ __forceinline__ float prob_at(const void* row, int64_t j, float T, bool has_keep, const RowKeep& kp,
                                         float2 ms) {
    const float y = process_value<DT>(load_one<DT>(row, j), j, T, has_keep, kp);
    return round_dt<DT>(sd_exp(y - ms.x) / ms.y);
}

__device__ __forceinline__ float prob_dyn(int dt, const void* row, int64_t j, float T, bool has_keep,
                                          const RowKeep& kp, float2 ms) {
    if (dt == SD_BF16) return prob_at<SD_BF16>(row, j, T, has_keep, kp, ms);
    if (dt == SD_F32) return prob_at<SD_F32>(row, j, T, has_keep, kp, ms);
    return prob_at<SD_F16>(row, j, T, has_keep, kp, ms);
}

// ------------------------------------------------------------------ decide (row stats, p/q, walk)
// Row statistics of every slot of sequence b, combined from the k_stats partials into LDS
// (all waves of the block).  Stats stay in LDS for the block's own use: re-reading them from
// global memory after a barrier could hit a line another block on this CU cached earlier.
__device__ __forceinline__ void seq_stats(const Plan& P, int b, float2* lstat, bool publish) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    // drafter rows whose stats came with their draws (sd_sample row_stats): no partials
    for (int s = P.stat_slots + (int)threadIdx.x; s < P.slots; s += (int)blockDim.x) {
        const float2 ms = P.dstats[(int64_t)(s - P.n_tslots) * P.dstats_stride + b];
        lstat[s] = ms;
        if (publish) P.rowstat[b * P.slots + s] = ms;
    }
    if (P.n_chunks <= kWave) {
        // one partial per lane per slot: issue every slot's load of this wave (a group of up to
        // kGroup slots per wave: 2γ + 1 <= 33 slots in one group) before reducing
        constexpr int kGroup = (2 * kFastSlots - 1 + 3) / 4;
        for (int g0 = 0; g0 < P.stat_slots; g0 += kGroup * nw) {
            float2 v[kGroup];
#pragma unroll
            for (int k = 0; k < kGroup; ++k) {
                const int s = g0 + w + k * nw;
                v[k] = (s < P.stat_slots && lane < P.n_chunks) ? ld_coh(P.part + (int64_t)(b * P.slots + s) * P.n_chunks + lane)
                                                          : make_float2(-INFINITY, 0.f);
            }
#pragma unroll
            for (int k = 0; k < kGroup; ++k) {
                const int s = g0 + w + k * nw;
                if (s >= P.stat_slots) break;
                const float m = wave_max(v[k].x);
                const float sum = wave_sum(v[k].x > -INFINITY ? v[k].y * sd_exp(v[k].x - m) : 0.f);
                if (lane == 0) {
                    lstat[s] = make_float2(m, sum);
                    if (publish) P.rowstat[b * P.slots + s] = make_float2(m, sum);   // read by later launches only
                }
            }
        }
        return;
    }
    for (int s = w; s < P.stat_slots; s += nw) {
        const float2 ms = combine_row(P, b * P.slots + s);
        if (lane == 0) {
            lstat[s] = ms;
            if (publish) P.rowstat[b * P.slots + s] = ms;
        }
    }
}

// Raw target / drafter values at drafted id tok of draft i (0 for an out-of-range id).
__device__ __forceinline__ void fetch_drafted(const Plan& P, int b, int i, int64_t tok, float* xt, float* xd) {
    *xt = 0.f;
    *xd = 0.f;
    if (tok >= 0 && tok < P.V) {
        int dt; float T; bool keep;
        *xt = load_dyn(P.tdt, row_ptr(P, b * P.slots + i, &dt, &T, &keep), tok);
        if (P.draft_is_probs) *xd = static_cast<const float*>(P.drow[i])[b * P.dstride + tok];
        else *xd = load_dyn(P.ddt, row_ptr(P, b * P.slots + P.n_tslots + i, &dt, &T, &keep), tok);
    }
}

// p(x_i), q(x_i) of the γ drafts (threads < γ; call after seq_stats + barrier)
__device__ void seq_ratios(const Plan& P, int b, const float2* lstat, float* lp, float* lq) {
    if (threadIdx.x >= P.gamma) return;
    const int i = threadIdx.x;
    const int64_t tok = P.draft_tokens[b * P.tok_stride + i];
    int dt; float T; bool keep;
    const int rt = b * P.slots + i;
    const void* trow = row_ptr(P, rt, &dt, &T, &keep);
    const RowKeep kt = keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    float p = 0.f, q = 0.f;
    if (tok >= 0 && tok < P.V) {
        p = prob_dyn(dt, trow, tok, T, keep, kt, lstat[i]);
        if (P.draft_is_probs) {
            q = static_cast<const float*>(P.drow[i])[b * P.dstride + tok];
        } else {
            const int rd = b * P.slots + P.n_tslots + i;
            const void* drow = row_ptr(P, rd, &dt, &T, &keep);
            const RowKeep kd = keep ? keep_of(P, rd) : RowKeep{-INFINITY, INT_MAX, 0, 0};
            q = prob_dyn(dt, drow, tok, T, keep, kd, lstat[P.n_tslots + i]);
        }
    }
    lp[i] = p;
    lq[i] = q;
}

// grid (B): STREAM-mode stage 1 — row stats and p/q ratios to global memory for the serial walk.
__global__ void __launch_bounds__(256) k_decide(Plan P) {
    __shared__ float2 lstat[2 * SD_MAX_GAMMA + 1];
    const int b = blockIdx.x;
    seq_stats(P, b, lstat, true);
    __syncthreads();
    seq_ratios(P, b, lstat, P.rp + b * P.gamma, P.rq + b * P.gamma);
}

// ------------------------------------------------------------------ walk
__device__ __forceinline__ float draw_uniform(const Plan& P, int b, int i, int64_t woff, bool* overrun) {
    if (P.noise.mode == SD_NOISE_STREAM) {
        if (woff >= stream_cap(P.noise)) { *overrun = true; return 0.f; }
        return uniform_from_word(stream_ptr(P.noise)[woff]);
    }
    const uint4 q = philox_block(P.noise, (uint32_t)b, kSiteAccept, (uint32_t)(i >> 2));   // 4 drafts per block
    return uniform_from_word((i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w);
}

// accept test of draft i given p(x_i), q(x_i) and its uniform
__device__ __forceinline__ bool accept_draft(const Plan& P, float p, float q, float u) {
    if (P.rule == SD_RULE_SPEC) return !(u > p / q);   // sampling/speculative_decoding.py:141-145 (fp32)
    const double ap = (double)q <= 0.0 ? 1.0 : fmin(1.0, (double)p / (double)q);   // infer_engine.py:303-305
    return (double)u < ap;
}

// The accept rule for one sequence given p(x_i), q(x_i); woff = its first noise word (STREAM).
// accm (has_acc): accept flags of the γ drafts precomputed in parallel, bit i = draft i (k_walk)
// lstop (nullable): per-draft "is a stop token" flags, precomputed alongside them
__device__ Decision walk_core(const Plan& P, int b, const float* rp, const float* rq, int64_t woff, int64_t* used_out,
                              bool has_acc = false, uint64_t accm = 0, const uint8_t* lstop = nullptr) {
    Decision d{};
    d.stop_index = -1;
    d.noise_off = 0;
    int64_t used = 0;
    bool overrun = false;
    const int g = P.gamma;
    const int64_t sample_words = 2ll * P.V;
    if (P.rule == SD_RULE_SPEC) {
        // sampling/speculative_decoding.py:139-145: r = rand(γ'); n = first i with r_i > p_i/q_i
        int n = g;
        for (int i = 0; i < g; ++i) {
            const bool acc = has_acc ? ((accm >> i) & 1u) != 0
                                     : accept_draft(P, rp[i], rq[i], draw_uniform(P, b, i, woff + i, &overrun));
            if (!acc && n == g) n = i;
        }
        used = g;
        d.n = n;
        // :150-155 stop token among the accepted drafts -> the reference returns before sampling
        // (the first-LISTED stop token that occurs, at its first position: stop_rank)
        int best = INT_MAX;
        for (int j = 0; j < n; ++j) {
            const int r = lstop && lstop[j] < 255 ? (lstop[j] == 0 ? INT_MAX : (int)lstop[j] - 1)
                                                  : stop_rank(P, P.draft_tokens[b * P.tok_stride + j]);
            if (r < best) { best = r; d.stop_index = j; }
        }
        if (d.stop_index >= 0) {
            d.mode = kModeNone;
            d.status = SD_ROW_DONE | SD_ROW_STOP_IN_DRAFTS;
        } else {
            if (n == g) { d.mode = kModeBonus; d.slot = g; d.status = SD_ROW_DONE | SD_ROW_BONUS; }
            else if (P.skip_adj) { d.mode = kModePRow; d.slot = n; d.status = SD_ROW_DONE | SD_ROW_FALLBACK_P; }
            else { d.mode = kModeResid; d.slot = n; d.status = SD_ROW_DONE | SD_ROW_RESIDUAL; }
            d.noise_off = woff + used;
            if (P.t_stoch) used += sample_words;
        }
    } else {
        // engine/infer_engine.py:287-330
        const bool act = P.active == nullptr || P.active[b] != 0;
        d.mode = kModeNone;
        d.n = 0;
        if (act) {
            d.status = SD_ROW_DONE;
            for (int i = 0; i < g; ++i) {
                const bool acc = has_acc ? ((accm >> i) & 1u) != 0
                                         : accept_draft(P, rp[i], rq[i], draw_uniform(P, b, i, woff + used, &overrun));
                used += 1;
                if (acc) {
                    d.n += 1;
                    if (lstop ? lstop[i] != 0 : is_stop(P, P.draft_tokens[b * P.tok_stride + i])) {
                        d.status |= SD_ROW_FINISHED;
                        break;
                    }
                } else {
                    d.mode = kModeResid;
                    d.slot = i;
                    d.status |= SD_ROW_RESIDUAL;
                    d.noise_off = woff + used;
                    used += sample_words;
                    break;
                }
            }
        }
    }
    if (overrun || (P.noise.mode == SD_NOISE_STREAM && d.mode != kModeNone && P.t_stoch &&
                    d.noise_off + sample_words > stream_cap(P.noise)))
        d.status |= SD_ROW_NOISE_OVERRUN;
    if (d.mode != kModeNone) {   // the sampled rows' stats travel with the decision (pick_wave reads them)
        d.mst = P.rowstat[b * P.slots + d.slot];
        d.msd = d.mode == kModeResid && !P.draft_is_probs ? P.rowstat[b * P.slots + P.n_tslots + d.slot]
                                                          : make_float2(0.f, 1.f);
    }
    *used_out = used;
    return d;
}

__device__ __forceinline__ void publish_decision(const Plan& P, int b, const Decision& d) {
    const int g = P.gamma;
    const bool pruned = P.rule == SD_RULE_SPEC && d.n < g && d.stop_index < 0;   // the engine never prunes
    if (P.prune_drafter) P.prune_drafter[b] = pruned ? g - d.n : 0;
    if (P.prune_target) P.prune_target[b] = pruned ? g - d.n + 1 : 0;
    P.dec[b] = d;
    P.n_accepted[b] = d.n;
    if (P.stop_index) P.stop_index[b] = d.stop_index;
}

__device__ int64_t walk_seq(const Plan& P, int b, int64_t woff) {
    int64_t used;
    const Decision d = walk_core(P, b, P.rp + b * P.gamma, P.rq + b * P.gamma, woff, &used);
    publish_decision(P, b, d);
    return used;
}

// The walk's accept tests on the raw words: torch.rand's u = m 2^-24, m = word & 0xffffff (exact in
// fp32), so u < t (ENGINE, accept_draft) is m < ceil(t 2^24) and !(u > t) (SPEC, a NaN t accepts) is
// m < floor(t 2^24) + 1 — t 2^24 is exact in fp64 — clamped to [0, 2^24].  The serial chain then
// compares integers (it converted each word and compared in fp64).
__device__ __forceinline__ uint32_t walk_thr_word(bool spec, double t) {
    constexpr double k24 = 16777216.0;
    if (t != t) return spec ? (1u << 24) : 0u;
    if (spec ? !(t >= 0.0) : !(t > 0.0)) return 0u;
    if (t >= 1.0) return 1u << 24;
    const double x = t * k24;
    return (uint32_t)(spec ? floor(x) + 1.0 : ceil(x));
}

// STREAM k_walk's LDS budget: the uniform windows of a block of rows (words), and the block's
// per-draft inputs (rows x gamma)
constexpr int kWalkWords = 12288;
constexpr int kWalkDrafts = 1024;

__global__ void __launch_bounds__(256) k_walk(Plan P) {
    if (P.noise.mode == SD_NOISE_STREAM) {
        // The reference draws row after row from one generator (engine/infer_engine.py:280-330;
        // sampling/speculative_decoding.py:139-171): the rows' word offsets form a serial chain.
        // Row b's words start at off + a + 2V k, where a counts the uniforms the earlier rows of the
        // block drew (<= g per row) and k the Exp(1) rows they drew (<= 1 per row).  So every
        // uniform a block of nb rows can read lies in nb windows [off + 2V k, off + 2V k + nb g).
        //   1. the workgroup loads those windows, and the block's accept thresholds (fp64 min(1,p/q)
        //      / fp32 p/q, divided in parallel), stop and active flags, into LDS: one round trip;
        //   2. wave 0 walks the chain from LDS — a row per step, its drafts on the lanes (one LDS
        //      load and two ballots per row), only the offsets (a, k) carried;
        //   3. every row's decision is rebuilt from its (a, k) and published in parallel.
        // (Before: one dependent global round trip per row, ~3 us each.)
        __shared__ uint32_t lw[kWalkWords];
        __shared__ uint32_t lthr[kWalkDrafts];   // accept iff (word & 0xffffff) < lthr (walk_thr_word)
        __shared__ float lrp[kWalkDrafts], lrq[kWalkDrafts];
        __shared__ uint8_t lstop[kWalkDrafts], lact[kWalkDrafts];
        __shared__ int32_t la[kWalkDrafts], lk[kWalkDrafts];
        __shared__ uint64_t lstpm[kWalkDrafts];   // row bi: bit i = draft i is a stop token
        __shared__ int64_t s_off;
        __shared__ int64_t s_stops[kLdsStops];
        const int tid = threadIdx.x, lane = tid & 63, g = P.gamma;
        const int64_t V2 = 2ll * P.V;
        const bool spec = P.rule == SD_RULE_SPEC;
        int nbmax = 1;
        while ((nbmax + 1) * (nbmax + 1) * g <= kWalkWords && (nbmax + 1) * g <= kWalkDrafts) ++nbmax;
        if (tid == 0) s_off = 0;
        const bool lds_stops = P.n_stop <= kLdsStops;
        if (lds_stops && tid < P.n_stop) s_stops[tid] = P.stops[tid];
        SD_TS(8000, 0);
        __syncthreads();
        for (int b0 = 0; b0 < P.B; b0 += nbmax) {
            const int nb = min(nbmax, P.B - b0), W = nb * g;
            const int64_t off = s_off;
            {   // every load of the block in flight at once — the windows' words (window k, word j at
                // lw[k W + j]; the window index by an exact fp32 reciprocal, not an integer division
                // per load), the drafts' p/q, ids and the rows' active flags — then the LDS writes
                // (a load behind a per-load branch, or a loop of load -> store pairs, paid one round
                // trip each)
                // the drafts' inputs first: in flight with the windows' first round
                constexpr int kPerD = kWalkDrafts / 256;
                float rp[kPerD], rq[kPerD];
                int64_t tok[kPerD];
                int32_t act[kPerD];
#pragma unroll
                for (int q = 0; q < kPerD; ++q) {
                    const int i = tid + q * 256;
                    const int bi = i / g, d = i - bi * g, b = b0 + (i < W ? bi : 0);
                    const int e = b * g + (i < W ? d : 0);
                    rp[q] = P.rp[e];
                    rq[q] = P.rq[e];
                    tok[q] = P.draft_tokens[b * P.tok_stride + (i < W ? d : 0)];
                    act[q] = P.active == nullptr ? 1 : P.active[b] != 0;
                }
                // The nb windows are W-word runs 2V words apart: each is read as nv aligned 16-byte
                // vectors (the first and last partly outside it; its own shift sh, as 2V words need
                // not be a multiple of 4), eight per thread per round, all in flight before their
                // words go to LDS.  Vectors that reach past the words the call may read (stream_cap)
                // take guarded word loads.
                const uint32_t* pw = stream_ptr(P.noise);
                const int64_t pcap = stream_cap(P.noise);
                const int sh0 = (int)((reinterpret_cast<uintptr_t>(pw + off) >> 2) & 3);   // window 0's shift
                const int nv = (W + 6) >> 2;   // covers W words after any shift <= 3
                const float invNv = 1.0f / (float)nv;
                const int nvec = nb * nv;
                constexpr int kVr = 8;
                for (int r0 = 0; r0 < nvec; r0 += kVr * 256) {
                    uint4 vv[kVr];
                    int kq[kVr], jq[kVr];
                    int64_t wq[kVr];
#pragma unroll
                    for (int q = 0; q < kVr; ++q) {
                        const int t = r0 + tid + q * 256;
                        const int tc = t < nvec ? t : nvec - 1;
                        const int k = (int)(((float)tc + 0.5f) * invNv), v = tc - k * nv;   // exact: tc, nv < 2^14
                        const int sh = (sh0 + (int)((V2 * k) & 3)) & 3;        // window k's shift
                        const int64_t w0 = off + V2 * k + 4 * v - sh;      // the vector's first word
                        kq[q] = t < nvec ? k : -1;
                        jq[q] = 4 * v - sh;
                        // unconditional loads (a vector outside the readable words reads the pool's
                        // first one instead and is patched below, word by word)
                        wq[q] = w0;
                        const bool whole = w0 >= 0 && w0 + 4 <= pcap;
                        vv[q] = *reinterpret_cast<const uint4*>(whole ? pw + w0 : P.noise.words);
                    }
#pragma unroll
                    for (int q = 0; q < kVr; ++q) {
                        if (kq[q] < 0) continue;
                        uint32_t e[4] = {vv[q].x, vv[q].y, vv[q].z, vv[q].w};
                        const int64_t w0 = wq[q];
                        if (!(w0 >= 0 && w0 + 4 <= pcap)) {   // the readable words' edge (rare)
#pragma unroll
                            for (int c = 0; c < 4; ++c) e[c] = w0 + c >= 0 && w0 + c < pcap ? pw[w0 + c] : 0u;
                        }
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const int j = jq[q] + c;
                            if (j >= 0 && j < W) lw[kq[q] * W + j] = e[c];
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < kPerD; ++q) {
                    const int i = tid + q * 256;
                    if (i >= W) continue;
                    const float p = rp[q], qq = rq[q];
                    lrp[i] = p;
                    lrq[i] = qq;
                    // accept iff u <= p/q (fp32, SPEC) / u < min(1, p/q) (fp64, ENGINE): accept_draft's rules
                    lthr[i] = walk_thr_word(spec, spec ? (double)(p / qq) : ((double)qq <= 0.0 ? 1.0 : fmin(1.0, (double)p / (double)qq)));
                    uint32_t r8 = 0;   // stop_rank8 from the staged list
                    if (lds_stops) {
                        for (int k = P.n_stop - 1; k >= 0; --k)
                            if (s_stops[k] == tok[q]) r8 = k < 254 ? (uint32_t)k + 1u : 255u;
                    } else {
                        r8 = stop_rank8(P, tok[q]);
                    }
                    lstop[i] = (uint8_t)r8;
                    lact[i] = (uint8_t)act[q];
                }
            }
            __syncthreads();
            for (int bi = tid; bi < nb; bi += blockDim.x) {   // the rows' stop masks (off the chain)
                uint64_t m = 0;
                for (int i = 0; i < g; ++i) m |= lstop[bi * g + i] != 0 ? 1ull << i : 0ull;
                lstpm[bi] = m;
            }
            __syncthreads();
            SD_TS(8000, 1);
            if (tid < kWave) {   // the chain: (a, k) of every row; per row only the uniforms' LDS read
                // depends on the previous row — the next row's threshold / flags are loaded during
                // this one, and rows < 64 keep their (a, k) in lane bi's registers (no LDS write on
                // the chain)
                int a = 0, k = 0, my_a = 0, my_k = 0;
                const bool in = lane < g;
                const bool t_stoch = P.t_stoch != 0;
                uint32_t t = lthr[in ? lane : 0];
                uint64_t stp = lstpm[0];
                bool ract = lact[0] != 0;
                for (int bi = 0; bi < nb; ++bi) {
                    const uint32_t m = lw[k * W + a + (in ? lane : 0)] & 0xFFFFFFu;   // u = m 2^-24
                    const int bn = bi + 1 < nb ? bi + 1 : bi;
                    const uint32_t t_n = lthr[bn * g + (in ? lane : 0)];
                    const uint64_t stp_n = lstpm[bn];
                    const bool ract_n = lact[bn * g] != 0;
                    if (bi < kWave && lane == bi) { my_a = a; my_k = k; }
                    if (bi >= kWave && lane == 0) { la[bi] = a; lk[bi] = k; }
                    const bool acc = m < t;
                    const uint64_t rej = __ballot(in && !acc);
                    const int f = rej ? __builtin_ctzll(rej) : g;              // first rejected draft
                    const uint64_t before = f >= 64 ? ~0ull : ((1ull << f) - 1ull);
                    const uint64_t stop_acc = stp & before;
                    // the row's outcome as selects, no branch on the chain: SPEC draws g uniforms and
                    // (stochastic rows, no stop among the accepted) one residual / bonus row; the
                    // ENGINE's active row stops at an accepted end token, or at the first rejection
                    // (+ the residual row), else takes all g
                    const int stop_i = stop_acc ? (int)__builtin_ctzll(stop_acc) : g;
                    const int da_e = stop_acc ? stop_i + 1 : (f < g ? f + 1 : g);
                    const int dk_e = !stop_acc && f < g ? 1 : 0;
                    const int da = spec ? g : (ract ? da_e : 0);
                    const int dk = spec ? (t_stoch && !stop_acc ? 1 : 0) : (ract ? dk_e : 0);
                    a += da;
                    k += dk;
                    t = t_n;
                    stp = stp_n;
                    ract = ract_n;
                }
                if (lane < nb) { la[lane] = my_a; lk[lane] = my_k; }
                if (lane == 0) s_off = off + a + V2 * k;
            }
            __syncthreads();
            SD_TS(8000, 2);
            // every row's decision from its offsets (walk_core's rules), published in parallel
            for (int bi = tid; bi < nb; bi += blockDim.x) {
                const int b = b0 + bi;
                const int64_t woff = off + la[bi] + V2 * lk[bi];
                uint64_t accm = 0;   // bit i: draft i accepted
                bool ovr = false;
                int64_t used;
                for (int i = 0; i < g; ++i) {
                    if ((lw[lk[bi] * W + la[bi] + i] & 0xFFFFFFu) < lthr[bi * g + i]) accm |= 1ull << i;
                }
                Decision d = walk_core(P, b, lrp + bi * g, lrq + bi * g, woff, &used, true, accm, lstop + bi * g);
                const bool sampled = spec ? (d.mode != kModeNone && P.t_stoch) : d.mode == kModeResid;
                const int64_t n_u = used - (sampled ? V2 : 0);
                const int64_t cap = stream_cap(P.noise);
                for (int i = 0; i < n_u; ++i) ovr |= woff + i >= cap;
                if (ovr) d.status |= SD_ROW_NOISE_OVERRUN;
                publish_decision(P, b, d);
            }
            __syncthreads();
            SD_TS(8000, 3);
        }
        if (tid == 0 && P.words_used) *P.words_used = s_off;
    } else {
        for (int b = threadIdx.x; b < P.B; b += blockDim.x) walk_seq(P, b, 0);
        if (threadIdx.x == 0 && P.words_used) *P.words_used = 0;
    }
}

// p(x_i), q(x_i) of draft i from its prefetch and the rows' (m, S)
template <int DT = -1, bool FAST = false>
__device__ __forceinline__ void draft_ratio(const Plan& P, int b, int i, const DraftPf& pf, float2 mst, float2 msd,
                                            float& p, float& q) {
    p = 0.f;
    q = 0.f;
    if (pf.tok < 0 || pf.tok >= P.V) return;
    if constexpr (DT >= 0 && FAST) {   // both rows of dtype DT, unprocessed, drafter logits
        p = round_dt<DT>(sd_exp(pf.xt - mst.x) / mst.y);
        q = round_dt<DT>(sd_exp(pf.xd - msd.x) / msd.y);
        return;
    }
    const int rt = b * P.slots + i;
    if constexpr (DT >= 0) {   // both rows of dtype DT, drafter logits (the fused / lean launches)
        const RowKeep kt = P.t_keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
        p = round_dt<DT>(sd_exp(process_value<DT>(pf.xt, pf.tok, P.tT, P.t_keep, kt) - mst.x) / mst.y);
        const int rd = b * P.slots + P.n_tslots + i;
        const RowKeep kd = P.d_keep ? keep_of(P, rd) : RowKeep{-INFINITY, INT_MAX, 0, 0};
        q = round_dt<DT>(sd_exp(process_value<DT>(pf.xd, pf.tok, P.dT, P.d_keep, kd) - msd.x) / msd.y);
        return;
    }
    const RowKeep kt = P.t_keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const float yt = P.tdt == SD_BF16 ? process_value<SD_BF16>(pf.xt, pf.tok, P.tT, P.t_keep, kt)
                   : P.tdt == SD_F32 ? process_value<SD_F32>(pf.xt, pf.tok, P.tT, P.t_keep, kt)
                                     : process_value<SD_F16>(pf.xt, pf.tok, P.tT, P.t_keep, kt);
    p = round_dyn(P.tdt, sd_exp(yt - mst.x) / mst.y);
    if (P.draft_is_probs) {
        q = pf.xd;
        return;
    }
    const int rd = b * P.slots + P.n_tslots + i;
    const RowKeep kd = P.d_keep ? keep_of(P, rd) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const float yd = P.ddt == SD_BF16 ? process_value<SD_BF16>(pf.xd, pf.tok, P.dT, P.d_keep, kd)
                   : P.ddt == SD_F32 ? process_value<SD_F32>(pf.xd, pf.tok, P.dT, P.d_keep, kd)
                                     : process_value<SD_F16>(pf.xd, pf.tok, P.dT, P.d_keep, kd);
    q = round_dyn(P.ddt, sd_exp(yd - msd.x) / msd.y);
}

// The perf-mode walk (walk_core's rules) from two ballots over the drafts' accept and stop flags
// (wave 0; lane 0 builds the Decision, carrying the sampled rows' (m, S) from lstat).
__device__ __forceinline__ void walk_decision(const Plan& P, int b, const uint8_t* lacc, const uint8_t* lstop, bool act,
                                              const float2* lstat, Decision* out, bool publish,
                                              int32_t extra_status = 0) {
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < kWave) {
        const int g = P.gamma;
        const bool in = lane < g;
        const bool acc = in && lacc[lane] != 0;
        const uint64_t rejm = __ballot(in && !acc), stopm = __ballot(in && lstop[lane] != 0);
        const int f_rej = rejm ? __builtin_ctzll(rejm) : g;             // first rejected draft (g: none)
        const uint64_t before = f_rej >= 64 ? ~0ull : ((1ull << f_rej) - 1ull);
        const uint64_t stop_acc = stopm & before;                        // stop tokens among the accepted
        // SPEC: the first-LISTED stop token among the accepted drafts, at its first position (the
        // reference's row-major nonzero, stop_rank); the ENGINE ends a row at its first accepted stop
        int spec_stop = -1;
        if (P.rule == SD_RULE_SPEC && stop_acc) {   // wave-uniform
            const bool sa = ((stop_acc >> lane) & 1ull) != 0;
            const int key = wave_min_i(sa ? ((int)lstop[lane] << 8) | lane : INT_MAX);
            spec_stop = key & 0xff;
            if ((key >> 8) == 255 && lane == 0) {   // saturated ranks (> 253 stop tokens): exact
                int best = INT_MAX;
                for (uint64_t m = stop_acc; m; m &= m - 1) {
                    const int j = __builtin_ctzll(m);
                    const int r = stop_rank(P, P.draft_tokens[b * P.tok_stride + j]);
                    if (r < best) { best = r; spec_stop = j; }
                }
            }
        }
        if (lane != 0) return;
        Decision d{};
        d.stop_index = -1;
        d.noise_off = 0;
        if (P.rule == SD_RULE_SPEC) {
            d.n = f_rej;
            if (stop_acc) {
                d.stop_index = spec_stop;
                d.mode = kModeNone;
                d.status = SD_ROW_DONE | SD_ROW_STOP_IN_DRAFTS;
            } else {
                if (f_rej == g) { d.mode = kModeBonus; d.slot = g; d.status = SD_ROW_DONE | SD_ROW_BONUS; }
                else if (P.skip_adj) { d.mode = kModePRow; d.slot = f_rej; d.status = SD_ROW_DONE | SD_ROW_FALLBACK_P; }
                else { d.mode = kModeResid; d.slot = f_rej; d.status = SD_ROW_DONE | SD_ROW_RESIDUAL; }
                d.noise_off = g;
            }
        } else {
            d.mode = kModeNone;
            d.n = 0;
            if (act) {
                d.status = SD_ROW_DONE;
                if (stop_acc) {
                    d.n = __builtin_ctzll(stop_acc) + 1;
                    d.status |= SD_ROW_FINISHED;
                } else if (f_rej < g) {
                    d.n = f_rej;
                    d.mode = kModeResid;
                    d.slot = f_rej;
                    d.status |= SD_ROW_RESIDUAL;
                    d.noise_off = f_rej + 1;
                } else {
                    d.n = g;
                }
            }
        }
        if (d.status & SD_ROW_DONE) d.status |= extra_status;   // e.g. a span record that never arrived
        if (d.mode != kModeNone) {   // the sampled rows' stats travel with the decision
            d.mst = lstat[d.slot];
            d.msd = d.mode == kModeResid && !P.draft_is_probs ? lstat[P.n_tslots + d.slot] : make_float2(0.f, 1.f);
        }
        if (out) *out = d;
        if (publish) {
            publish_decision(P, b, d);
            if (P.words_used && b == 0) *P.words_used = 0;
        }
    }
}

// Perf-mode decision of sequence b by one 256-thread workgroup (the k_stats tail, or every k_sample
// workgroup of the sequence when the decision is replicated there: out = its LDS copy, publish only
// from one of them): row stats
// from the partials (published to rowstat), p/q at the drafted ids, the accept tests on Philox
// uniforms, the walk.  Every per-draft input was prefetched during the stream (DraftPf), so the
// tail has one memory round trip (the partials).  With the drafter stats prefetched (P.dstats)
// the wave that reduces target slot i tests draft i at once: one barrier before the walk.
// DT >= 0 (the fused verify's decider): rows of that dtype, FAST rows unprocessed, the drafter
// stats from the draws and the one-round-trip record path guaranteed by the launch — only that
// path is compiled (a shorter, branch-free critical path after the records)
template <int DT, bool FAST>
__device__ __forceinline__ void decide_seq(const Plan& P, int b, const DraftPf& pf, int wg_id, Decision* out, bool publish, bool coh,
                           const uint32_t* poll_epoch) {
    __shared__ float2 lstat[2 * SD_MAX_GAMMA + 1];
    __shared__ float lp[SD_MAX_GAMMA], lq[SD_MAX_GAMMA];
    __shared__ uint8_t lacc[SD_MAX_GAMMA], lstop[SD_MAX_GAMMA];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = kThreads / kWave;
    const int i = pf_draft(P);
    if (i >= 0) lstop[i] = pf.stop;
    if (DT >= 0 || (P.dstats && P.n_chunks <= kWave && P.n_tslots <= kFastSlots)) {
        if (i >= 0) {
            lstat[P.n_tslots + i] = pf.ds;
            if (publish) P.rowstat[b * P.slots + P.n_tslots + i] = pf.ds;
        }
        constexpr int kMaxSlotsPerWave = (kFastSlots + 3) / 4;
        float2 v[kMaxSlotsPerWave];
        bool lost = false;   // a span record that never arrived: the row's outputs are invalid
        if (poll_epoch) {   // poll mode: each record re-read until it carries this call's tag (bounded)
            static_assert(kMaxSlotsPerWave <= 5, "ld_coh16x5");
            const uint32_t ep = *poll_epoch;
            // the wave's records all in flight at once (one round trip), then the stragglers
            const uint4* rp[5];
            bool need[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int s = w + k * nw;
                need[k] = k < kMaxSlotsPerWave && s < P.n_tslots && lane < P.n_chunks;
                rp[k] = need[k] ? stats_rec(P, b, s, lane) : stats_rec(P, b, 0, 0);
            }
            uint4 r[5];
            ld_coh16x5(rp[0], rp[1], rp[2], rp[3], rp[4], r);
            SD_TS(wg_id, 9);
#pragma unroll
            for (int k = 0; k < kMaxSlotsPerWave; ++k) {
                const int s = w + k * nw;
                v[k] = make_float2(-INFINITY, 0.f);
                if (need[k]) {
                    const uint32_t tag = stats_tag(ep, b, s, lane);
                    uint4 rr = r[k];
                    uint64_t sw_ = 0; for (int spin = 0; rr.z != tag && spin_more(spin, P.spin_limit, sw_); ++spin) {
                        __builtin_amdgcn_s_sleep(1);
                        rr = ld_coh16(rp[k]);
                    }
                    // spin limit < 0 (the test hook): every record counts as lost, as in the draws'
                    // and the samplers' polls — not only the ones still missing at the first read
                    const bool got = rr.z == tag && P.spin_limit >= 0;
                    v[k] = got ? make_float2(__uint_as_float(rr.x), __uint_as_float(rr.y))
                               : make_float2(0.f, NAN);   // timeout: the row is flagged invalid
                    lost |= !got;
                }
            }
            SD_TS(wg_id, 11);
        } else {
#pragma unroll
            for (int k = 0; k < kMaxSlotsPerWave; ++k) {
                const int s = w + k * nw;
                v[k] = (s < P.n_tslots && lane < P.n_chunks) ? ld_x(P.part + (int64_t)(b * P.slots + s) * P.n_chunks + lane, coh)
                                                             : make_float2(-INFINITY, 0.f);
            }
        }
#pragma unroll
        for (int k = 0; k < kMaxSlotsPerWave; ++k) {
            const int s = w + k * nw;
            if (s >= P.n_tslots) break;
            const float m = wave_max(v[k].x);
            const float sum = wave_sum(v[k].x > -INFINITY ? v[k].y * sd_exp(v[k].x - m) : 0.f);
            const float2 ms = make_float2(m, sum);
            if (lane == 0) {
                lstat[s] = ms;
                if (publish) P.rowstat[b * P.slots + s] = ms;
            }
            if (k == 0) SD_TS(wg_id, 13);
            if (lane == k && i == s) {   // i < γ: this thread holds draft s
                float p, q;
                draft_ratio<DT, FAST>(P, b, i, pf, ms, pf.ds, p, q);
                if (k == 0 && s == 0) SD_TS(wg_id, 14);
                lp[i] = p;
                lq[i] = q;
                lacc[i] = accept_draft(P, p, q, pf.u);
                if (k == 0 && s == 0) SD_TS(wg_id, 15);
            }
        }
        __shared__ int32_t s_lost[kThreads / kWave];
        if (lane == 0) s_lost[w] = __ballot(lost) != 0;
        SD_TS(wg_id, 10);
        __syncthreads();
        SD_TS(wg_id, 4);
        int32_t xs = 0;
#pragma unroll
        for (int k = 0; k < kThreads / kWave; ++k) xs |= s_lost[k];
        walk_decision(P, b, lacc, lstop, pf.act, lstat, out, publish,
                      xs ? SD_ROW_EXCHANGE_TIMEOUT | SD_ROW_INVALID_DIST : 0);
        SD_TS(wg_id, 5);
        return;
    } else {
        seq_stats(P, b, lstat, publish);   // every wave reduces partials
        __syncthreads();
        SD_TS(wg_id, 4);
        if (i >= 0) {
            float p, q;
            draft_ratio(P, b, i, pf, lstat[i], P.draft_is_probs ? make_float2(0.f, 1.f) : lstat[P.n_tslots + i], p, q);
            lp[i] = p;
            lq[i] = q;
            lacc[i] = accept_draft(P, p, q, pf.u);
        }
        __syncthreads();
        SD_TS(wg_id, 5);
    }
    walk_decision(P, b, lacc, lstop, pf.act, lstat, out, publish);
}

// STREAM exponential race of one chunk: the exact argmax (first index on ties) of
// round_dt(p_j / round_dt(E_j)), p_j = round_dt(exp(y_j - M) / S) the processed probability and
// E_j torch's exponential_ value from words woff + 2j (exp1_from_words, fp64 log1p).  Screened in
// fp32: a_j = p'_j / E'_j with a cheap E' and, for 16-bit rows, the unrounded p' = e^(y_j - M)
// (the common 1/S drops out of the comparison).  The exact values differ from a_j by at most the
// dt roundings and the screening errors, so every element that can be the chunk's exact maximum
// has a_j >= max_chunk(a) (1 - tol); only those take the exact path.  Whole workgroup; returns the
// chunk's (value, index) in pv / pi.
template <int DT>
__device__ __forceinline__ float race_tol() {
    // tol >= 4.2 u_dt + 2 (screening errors of p and E); about twice that, for margin
    return DT == SD_BF16 ? 0.0625f : (DT == SD_F16 ? 0.0078125f : 7.62939453125e-06f);
}
template <int DT, int EPT>
__device__ __forceinline__ void stream_race(const sd_noise& nz, int64_t woff, const float* y, const bool* ok,
                                            const uint32_t* wd, const int64_t* jj, float M, float S, float invS,
                                            float& pv, int32_t& pi, float* ldsf, int32_t* ldsi) {
    float a[EPT];
    float am = 0.f;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        const bool inw = woff + 2 * jj[k] + 1 < nz.n_words;
        float e, p;
        if constexpr (DT == SD_F32) {
            e = exp1_fast_from_words(wd[2 * k], wd[2 * k + 1]);
            p = prob_exact<DT>(y[k], M, S, invS);
        } else {
            e = exp1_screen16(wd[2 * k], wd[2 * k + 1]);
            p = __builtin_amdgcn_exp2f((y[k] - M) * kLog2e);
        }
        a[k] = ok[k] ? p * __builtin_amdgcn_rcpf(inw ? e : 1.f) : -INFINITY;
        am = fmaxf(am, a[k]);
    }
    const float bm = block_reduce(am, FMax(), ldsf);
    const float thr = bm * (1.0f - race_tol<DT>());
    pv = -INFINITY;
    pi = INT_MAX;
    // candidates; an all-zero chunk keeps each thread's first element (exact value 0)
    uint32_t cm = 0;
    bool first = true;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        if (!ok[k]) continue;
        if (a[k] >= thr && (a[k] > 0.f || first)) cm |= 1u << k;
        first = false;
    }
    // the exact values, one candidate at a time (one copy of the fp64 code; registers selected by
    // an unrolled compare so nothing is indexed dynamically)
    while (cm) {
        const int k = __builtin_ctz(cm);
        cm &= cm - 1u;
        float yk = 0.f;
        uint32_t h = 0u, l = 0u;
        int64_t j = 0;
#pragma unroll
        for (int kk = 0; kk < EPT; ++kk)
            if (kk == k) { yk = y[kk]; h = wd[2 * kk]; l = wd[2 * kk + 1]; j = jj[kk]; }
        const float pk = prob_exact<DT>(yk, M, S, invS);
        const float eb = round_dt<DT>(woff + 2 * j + 1 < nz.n_words ? exp1_from_words(h, l) : 1.f);
        const float val = div_round<DT>(pk, eb, __builtin_amdgcn_rcpf(eb));
        if (arg_better(val, (int32_t)j, pv, pi)) { pv = val; pi = (int32_t)j; }
    }
    block_argmax(pv, pi, ldsf, ldsi);
}

// ------------------------------------------------------------------ k_resample
// grid (chunk, B).  RESID: Σ(p_n - q_n)+ and the argmax candidates of fl(fl(res/S)/E) in one pass
// over the two rows; BONUS / PROW: argmax of the multinomial (or greedy) value of the target row.
// candidates within 64 ulp of the max: the roundings of fl(fl(res/S)/E) (<= a few ulp) and, under
// STREAM noise, the fp32 screening value of E (exp1_fast_from_words, <= 8 ulp, on both sides)
constexpr float kCandTol = 1.0f - 64.0f * 5.9604645e-08f;

template <int TDT, int DDT, int NZ, int EPT, bool FAST>
__device__ __forceinline__ void resid_body(const Plan& P, const Decision& d, int b, int c, float2 mst, float2 msd_in) {
    __shared__ float ldsf[8];
    __shared__ int32_t lcount;
    __shared__ float lres[kMaxCand], le[kMaxCand];
    __shared__ int32_t lidx[kMaxCand];
    constexpr int VEC = Elem<TDT>::kVec < Elem<DDT>::kVec ? Elem<TDT>::kVec : Elem<DDT>::kVec;
    constexpr int NV = EPT / VEC;
    const int rt = b * P.slots + d.slot;
    const void* trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (TDT == SD_F32 ? 4 : 2);
    const bool t_al = (reinterpret_cast<uintptr_t>(trow) & 15) == 0;
    const RowKeep kt = P.t_keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const bool stoch = P.t_stoch != 0;
    const int64_t base = (int64_t)c * P.rchunk;
    const void* drow;
    RowKeep kd{-INFINITY, INT_MAX, 0, 0};
    const float2 msd = msd_in;
    if (P.draft_is_probs) {
        drow = static_cast<const float*>(P.drow[d.slot]) + b * P.dstride;
    } else {
        const int rd = b * P.slots + P.n_tslots + d.slot;
        drow = static_cast<const char*>(P.drow[d.slot]) + b * P.dstride * (DDT == SD_F32 ? 4 : 2);
        if (P.d_keep) kd = keep_of(P, rd);
    }
    const bool d_al = (reinterpret_cast<uintptr_t>(drow) & 15) == 0;
    const float t_inv = 1.0f / mst.y, d_inv = 1.0f / msd.y;

    float sum = 0.f, wmax = 0.f;
    float res[EPT], ev[EPT];
    // STREAM: the words stay in registers; ev holds the fp32 screening value of E, and the exact
    // value is formed for the candidates only
    uint32_t wd[NZ == SD_NOISE_STREAM ? 2 * EPT : 1];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float xt[VEC], xd[VEC], e[VEC];
        load_vecn<TDT, VEC>(trow, e0, P.V, t_al, xt);
        load_vecn<DDT, VEC>(drow, e0, P.V, d_al, xd);   // draft_is_probs dispatches DDT = F32
        if constexpr (NZ == SD_NOISE_STREAM) {
            if (stoch) {
                stream_words<VEC>(P.noise, d.noise_off, e0, wd + 2 * v * VEC);
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    e[k] = d.noise_off + 2 * (e0 + k) + 1 < stream_cap(P.noise)
                               ? exp1_fast_from_words(wd[2 * (v * VEC + k)], wd[2 * (v * VEC + k) + 1]) : 1.f;
            }
        } else {
            if (stoch) exp_noise_vec<VEC, NZ>(P.noise, d.noise_off, b, e0, P.V, e);
        }
        if constexpr (!FAST) {
            process_vec<TDT, VEC>(xt, e0, P.tT, P.t_keep, kt);
            if (!P.draft_is_probs) process_vec<DDT, VEC>(xd, e0, P.dT, P.d_keep, kd);
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            const float yt = xt[k];
            const float p = prob_exact<TDT>(yt, mst.x, mst.y, t_inv);
            float q;
            if (P.draft_is_probs) {
                q = xd[k];
            } else {
                const float yd = xd[k];
                q = prob_exact<DDT>(yd, msd.x, msd.y, d_inv);
            }
            const float diff = p - q;                                 // bf16/fp32 - fp32 -> fp32
            const float rr = (j < P.V && diff > 0.f) ? diff : 0.f;     // max_fn numerator, :317 clamp
            res[v * VEC + k] = rr;
            ev[v * VEC + k] = stoch ? e[k] : 1.f;
            sum += rr;
            wmax = fmaxf(wmax, stoch ? rr * __builtin_amdgcn_rcpf(e[k]) : rr);
        }
    }
    const float bsum = block_reduce(sum, FSum(), ldsf, kThreads / kWave);
    const float bw = block_reduce(wmax, FMax(), ldsf, kThreads / kWave);
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    // any j whose exact fl(fl(res/S)/E) can tie the maximum has res/E within a few ulp of it
    const float thr = bw * kCandTol;
    if (bw > 0.f) {
        uint32_t cm = 0;
#pragma unroll
        for (int idx = 0; idx < EPT; ++idx) {
            const float w = stoch ? res[idx] * __builtin_amdgcn_rcpf(ev[idx]) : res[idx];
            if (res[idx] > 0.f && w >= thr) cm |= 1u << idx;
        }
        while (cm) {   // one candidate at a time (registers selected by an unrolled compare)
            const int idx = __builtin_ctz(cm);
            cm &= cm - 1u;
            float rr = 0.f, ee = 1.f;
            uint32_t h = 0u, l = 0u;
#pragma unroll
            for (int kk = 0; kk < EPT; ++kk)
                if (kk == idx) {
                    rr = res[kk];
                    ee = ev[kk];
                    if constexpr (NZ == SD_NOISE_STREAM) { h = wd[2 * kk]; l = wd[2 * kk + 1]; }
                }
            const int v = idx / VEC, k = idx - v * VEC;
            const int64_t j = base + ((int64_t)v * kThreads + threadIdx.x) * VEC + k;
            const int slot = atomicAdd(&lcount, 1);
            if (slot < kMaxCand) {
                if constexpr (NZ == SD_NOISE_STREAM)   // the exact value, for the candidates only
                    if (stoch) ee = d.noise_off + 2 * j + 1 < stream_cap(P.noise) ? exp1_from_words(h, l) : 1.f;
                lres[slot] = rr;
                le[slot] = ee;
                lidx[slot] = (int32_t)j;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ResPart& o = P.rpart[(int64_t)b * P.rn_chunks + c];
        st_coh(&o.sum, bsum);
        st_coh(&o.wmax, bw);
        st_coh(&o.ncand, lcount);
        for (int k = 0; k < kMaxCand && k < lcount; ++k) {
            st_coh(&o.cres[k], lres[k]);
            st_coh(&o.ce[k], le[k]);
            st_coh(&o.cidx[k], lidx[k]);
        }
    }
}

template <int TDT, int NZ, int EPT, bool FAST>
__device__ __forceinline__ void prow_body(const Plan& P, const Decision& d, int b, int c, float2 mst) {
    __shared__ float ldsf[8];
    __shared__ int32_t ldsi[8];
    constexpr int VEC = Elem<TDT>::kVec, NV = EPT / VEC;
    const int rt = b * P.slots + d.slot;
    const void* trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (TDT == SD_F32 ? 4 : 2);
    const bool t_al = (reinterpret_cast<uintptr_t>(trow) & 15) == 0;
    const RowKeep kt = P.t_keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const bool stoch = P.t_stoch != 0;
    const int64_t base = (int64_t)c * P.rchunk;
    const float t_inv = 1.0f / mst.y;
    float pv = -INFINITY;
    int32_t pi = INT_MAX;
    if constexpr (NZ == SD_NOISE_STREAM) {
        if (stoch) {   // the screened exponential race (stream_race)
            float pr[EPT];
            uint32_t wd[2 * EPT];
            int64_t jj[EPT];
            bool ok[EPT];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
                float xt[VEC];
                load_vec<TDT>(trow, e0, P.V, t_al, xt);
                stream_words<VEC>(P.noise, d.noise_off, e0, wd + 2 * v * VEC);
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const int64_t j = e0 + k;
                    jj[v * VEC + k] = j;
                    ok[v * VEC + k] = j < P.V;
                    pr[v * VEC + k] = FAST ? xt[k] : process_value<TDT>(xt[k], j, P.tT, P.t_keep, kt);   // y
                }
            }
            stream_race<TDT, EPT>(P.noise, d.noise_off, pr, ok, wd, jj, mst.x, mst.y, t_inv, pv, pi, ldsf, ldsi);
            if (threadIdx.x == 0) {
                ResPart& o = P.rpart[(int64_t)b * P.rn_chunks + c];
                st_coh(&o.pval, pv);
                st_coh(&o.pidx, pi);
            }
            return;
        }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float xt[VEC], e[VEC];
        load_vec<TDT>(trow, e0, P.V, t_al, xt);
        if (stoch) exp_noise_vec<VEC, NZ>(P.noise, d.noise_off, b, e0, P.V, e);
        if constexpr (!FAST) process_vec<TDT, VEC>(xt, e0, P.tT, P.t_keep, kt);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= P.V) continue;
            const float p = prob_exact<TDT>(xt[k], mst.x, mst.y, t_inv);
            float val = p;
            if (stoch) {   // multinomial: round_dt(p / round_dt(E))
                const float eb = round_dt<TDT>(e[k]);
                val = div_round<TDT>(p, eb, __builtin_amdgcn_rcpf(eb));
            }
            if (arg_better(val, (int32_t)j, pv, pi)) { pv = val; pi = (int32_t)j; }
        }
    }
    block_argmax(pv, pi, ldsf, ldsi, kThreads / kWave);
    if (threadIdx.x == 0) {
        ResPart& o = P.rpart[(int64_t)b * P.rn_chunks + c];
        st_coh(&o.pval, pv);
        st_coh(&o.pidx, pi);
    }
}

// STREAM (parity) mode: the decision comes from the serial k_decide -> k_walk stages.
template <int TDT, int DDT, int EPT, bool FAST>
__global__ void __launch_bounds__(kThreads) SD_SGPR_CAP k_resample(Plan P) {
    const int b = blockIdx.y, c = blockIdx.x;
    const Decision d = P.dec[b];
    if (d.mode == kModeNone || (d.status & SD_ROW_NOISE_OVERRUN)) return;
    const float2 mst = P.rowstat[b * P.slots + d.slot];
    float2 msd = make_float2(0.f, 1.f);
    if (d.mode == kModeResid && !P.draft_is_probs) msd = P.rowstat[b * P.slots + P.n_tslots + d.slot];
    if (d.mode == kModeResid) resid_body<TDT, DDT, SD_NOISE_STREAM, EPT, FAST>(P, d, b, c, mst, msd);
    else prow_body<TDT, SD_NOISE_STREAM, EPT, FAST>(P, d, b, c, mst);
}

// ------------------------------------------------------------------ finalize
// Σ residual over the chunk partials of sequence b, fixed order (lane-strided, then a butterfly).
__device__ __forceinline__ float resid_mass(const Plan& P, int b, float* wmax) {
    const int lane = threadIdx.x & 63;
    const ResPart* rp = P.rpart + (int64_t)b * P.rn_chunks;
    float s = 0.f, wm = 0.f;
    for (int c = lane; c < P.rn_chunks; c += kWave) {
        s += ld_coh(&rp[c].sum);
        if (wmax) wm = fmaxf(wm, ld_coh(&rp[c].wmax));
    }
    if (wmax) *wmax = wave_max(wm);
    return wave_sum(s);
}

// The token of sequence b from the argmax-candidate partials (one wave): residual candidates
// evaluated exactly as fl(fl(res / S) / E), the engine's multinomial(p) fallback, bonus / p-row
// argmax.  x = -1 when nothing is sampled.
__device__ __forceinline__ void pick_wave(const Plan& P, int b, const Decision& d, int64_t& x, float& mass, int32_t& status) {
    const int lane = threadIdx.x & 63;
    const ResPart* rp = P.rpart + (int64_t)b * P.rn_chunks;
    if (d.mode == kModeResid) {
        int overflow = 0;
        float wm;
        const float s = resid_mass(P, b, &wm);
        mass = s;
        const int rt = b * P.slots + d.slot;
        const RowKeep kt = P.t_keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
        const void* trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
        const float2 mst = d.mst;   // the decision carries the rows' (m, S): no read of rowstat, which
                                    // k_verify_lean writes in this same launch
        if (P.rule == SD_RULE_ENGINE && (double)s <= 1e-12) {
            // engine/infer_engine.py:319-321: multinomial(p) over the target row (rare: p ~= q)
            float bv = -INFINITY;
            int32_t bi = INT_MAX;
            for (int64_t j = lane; j < P.V; j += kWave) {
                const float p = prob_dyn(P.tdt, trow, j, P.tT, P.t_keep, kt, mst);
                const float v = round_dyn(P.tdt, p / round_dyn(P.tdt, exp_noise(P.noise, d.noise_off, b, j)));
                if (arg_better(v, (int32_t)j, bv, bi)) { bv = v; bi = (int32_t)j; }
            }
            wave_argmax(bv, bi);
            x = bi;
            status = (status & ~SD_ROW_RESIDUAL) | SD_ROW_FALLBACK_P;
        } else if (s == 0.f || (P.t_stoch && !(s > 0.f && s < INFINITY))) {
            // max_fn divides by zero (all-NaN distribution) or by NaN / inf: torch raises
            // (sampling/speculative_decoding.py:171; engine/infer_engine.py:325 with den NaN)
            if (P.t_stoch) status |= SD_ROW_INVALID_DIST;
            else x = 0;   // torch.argmax over an all-NaN row
        } else {
            // exact evaluation of the candidates: v = fl(fl(res / S) / E)
            const float thr = wm * kCandTol;
            float bv = -INFINITY;
            int32_t bi = INT_MAX;
            for (int c = lane; c < P.rn_chunks; c += kWave) {
                const ResPart& o = rp[c];
                if (ld_coh(&o.wmax) < thr) continue;
                const int nc = ld_coh(&o.ncand);
                if (nc > kMaxCand) { overflow = 1; continue; }
                for (int k = 0; k < nc; ++k) {
                    const float pr = ld_coh(&o.cres[k]) / s;
                    const float v = P.t_stoch ? pr / ld_coh(&o.ce[k]) : pr;
                    const int32_t ci = ld_coh(&o.cidx[k]);
                    if (arg_better(v, ci, bv, bi)) { bv = v; bi = ci; }
                }
            }
            wave_argmax(bv, bi);
            // chunks with too many near-equal values (e.g. ties) are re-scanned exactly
            overflow = __any(overflow);
            if (overflow) {
                const void* drow;
                RowKeep kd{-INFINITY, INT_MAX, 0, 0};
                float2 msd = make_float2(0.f, 1.f);
                int ddt = SD_F32;
                if (P.draft_is_probs) drow = static_cast<const float*>(P.drow[d.slot]) + b * P.dstride;
                else {
                    const int rd = b * P.slots + P.n_tslots + d.slot;
                    drow = static_cast<const char*>(P.drow[d.slot]) + b * P.dstride * (P.ddt == SD_F32 ? 4 : 2);
                    if (P.d_keep) kd = keep_of(P, rd);
                    msd = d.msd;
                    ddt = P.ddt;
                }
                for (int64_t j = lane; j < P.V; j += kWave) {
                    const float p = prob_dyn(P.tdt, trow, j, P.tT, P.t_keep, kt, mst);
                    const float q = P.draft_is_probs ? static_cast<const float*>(drow)[j]
                                                     : prob_dyn(ddt, drow, j, P.dT, P.d_keep, kd, msd);
                    const float diff = p - q;
                    const float rr = diff > 0.f ? diff : 0.f;
                    const float pr = rr / s;
                    const float v = P.t_stoch ? pr / exp_noise(P.noise, d.noise_off, b, j) : pr;
                    if (arg_better(v, (int32_t)j, bv, bi)) { bv = v; bi = (int32_t)j; }
                }
                wave_argmax(bv, bi);
            }
            x = bi;
        }
    } else {
        // bonus / p-row: argmax across chunks
        float pv = -INFINITY;
        int32_t pi = INT_MAX;
        for (int c = lane; c < P.rn_chunks; c += kWave) {
            const float v = ld_coh(&rp[c].pval);
            const int32_t i = ld_coh(&rp[c].pidx);
            if (arg_better(v, i, pv, pi)) { pv = v; pi = i; }
        }
        wave_argmax(pv, pi);
        x = pi;
        // multinomial over a row whose softmax is NaN / inf (a NaN or +inf logit): torch raises
        // (utils/logits_processor.py:48-49); torch.argmax (greedy) does not
        const float2 ms = d.mst;
        if (P.t_stoch && !(ms.y > 0.f && ms.y < INFINITY)) status |= SD_ROW_INVALID_DIST;
    }
}

// Outputs of sequence b (one thread): token, mass, engine state (engine/infer_engine.py:307-336
// applied in place), row status with the threshold flags.
__device__ void finalize_write(const Plan& P, int b, const Decision& d, int64_t x, float mass, int32_t status,
                               int64_t acc0, const int64_t* lstops = nullptr) {
    const int g = P.gamma;
    P.next_token[b * P.next_token_stride] = x;
    if (P.resample_mass) P.resample_mass[b] = mass;
    const bool engine_state = P.rule == SD_RULE_ENGINE && P.generated != nullptr;
    if (engine_state && (status & SD_ROW_DONE)) {
        int64_t* gen = P.generated + b * P.gen_stride;
        if (d.mode == kModeResid && x >= 0) {
            gen[P.step + d.n] = x;
            if (is_stop_l(P, x, lstops)) status |= SD_ROW_FINISHED;
        }
        if (d.n < g)
            for (int t = P.step + d.n + 1; t < P.step + g; ++t) gen[t] = 0;
        if (status & SD_ROW_FINISHED) P.finished[b] = 1;
        P.accepted_count[b] = acc0 + d.n;
    } else if (P.rule == SD_RULE_ENGINE && d.mode == kModeResid && x >= 0 && is_stop_l(P, x, lstops)) {
        status |= SD_ROW_FINISHED;
    }
    if (P.t_keep)
        for (int s2 = 0; s2 < P.n_tslots; ++s2) status |= keep_of(P, b * P.slots + s2).flags;
    if (P.d_keep)
        for (int s2 = P.n_tslots; s2 < P.slots; ++s2) status |= keep_of(P, b * P.slots + s2).flags;
    P.row_status[b] = status;
    flag_error(P.status_or, status);
    if (P.row_counts && (status & SD_ROW_DONE)) {   // one writer per row per call (stream-ordered calls)
        int64_t* rc = P.row_counts + 2 * (int64_t)b;
        rc[0] += d.n;
        rc[1] += d.n + (d.mode != kModeNone && x >= 0 ? 1 : 0);
    }
}

// STREAM mode: grid (B), one wave.
__global__ void __launch_bounds__(64) k_finalize(Plan P) {
    const int b = blockIdx.x;
    const Decision d = P.dec[b];
    int64_t x = -1;
    float mass = NAN;
    int32_t status = d.status;
    if (d.mode != kModeNone && !(status & SD_ROW_NOISE_OVERRUN)) pick_wave(P, b, d, x, mass, status);
    if (threadIdx.x == 0) {
        const bool engine_state = P.rule == SD_RULE_ENGINE && P.generated != nullptr;
        finalize_write(P, b, d, x, mass, status, engine_state && (status & SD_ROW_DONE) ? P.accepted_count[b] : 0);
    }
}

// ------------------------------------------------------------------ k_sample (PHILOX / perf mode)
// The row to sample from and its weights: RESID -> (p_n - q_n)+ (max_fn's numerator,
// sampling/speculative_decoding.py:180-186, engine/infer_engine.py:313-324); BONUS / PROW -> p.
struct PairRows {
    const void* trow;
    const void* drow;
    RowKeep kt, kd;
    float2 mst, msd;
    float t_inv, d_inv;
    float tT, dT;
    int32_t V;
    bool t_al, d_al, resid, t_keep, d_keep, dprobs;
};

template <int TDT, int DDT>
__device__ __forceinline__ PairRows pair_rows(const Plan& P, const Decision& d, int b) {
    PairRows R;
    R.resid = d.mode == kModeResid;
    const int rt = b * P.slots + d.slot;
    R.trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (TDT == SD_F32 ? 4 : 2);
    R.kt = P.t_keep ? keep_of(P, rt) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    R.kd = RowKeep{-INFINITY, INT_MAX, 0, 0};
    R.mst = d.mst;   // perf mode: carried by the decision (no dependent rowstat load)
    R.msd = make_float2(0.f, 1.f);
    R.drow = nullptr;
    if (R.resid) {
        if (P.draft_is_probs) {
            R.drow = static_cast<const float*>(P.drow[d.slot]) + b * P.dstride;
        } else {
            const int rd = b * P.slots + P.n_tslots + d.slot;
            R.drow = static_cast<const char*>(P.drow[d.slot]) + b * P.dstride * (DDT == SD_F32 ? 4 : 2);
            if (P.d_keep) R.kd = keep_of(P, rd);
            R.msd = d.msd;
        }
    }
    R.t_al = (reinterpret_cast<uintptr_t>(R.trow) & 15) == 0;
    R.d_al = (reinterpret_cast<uintptr_t>(R.drow) & 15) == 0;
    R.t_inv = 1.0f / R.mst.y;
    R.d_inv = 1.0f / R.msd.y;
    R.tT = P.tT;
    R.dT = P.dT;
    R.V = P.V;
    R.t_keep = P.t_keep;
    R.d_keep = P.d_keep;
    R.dprobs = P.draft_is_probs;
    return R;
}

template <int TDT, int DDT>
struct PairVec {
    static constexpr int kVec = Elem<TDT>::kVec < Elem<DDT>::kVec ? Elem<TDT>::kVec : Elem<DDT>::kVec;
};

template <int TDT, int DDT, bool FAST>
__device__ __forceinline__ void pair_weights_from(const PairRows& R, int64_t e0, const float* xt, const float* xd,
                                                  float* w, float* pw);

// weights of the VEC elements starting at e0 (0 past the vocabulary)
template <int TDT, int DDT, bool FAST>
__device__ __forceinline__ void pair_weights(const PairRows& R, int64_t e0, float* w, float* pw = nullptr) {
    constexpr int VEC = PairVec<TDT, DDT>::kVec;
    float xt[VEC], xd[VEC];
    if (VEC == Elem<TDT>::kVec && VEC == Elem<DDT>::kVec && R.t_al && (!R.resid || R.d_al) && R.V >= VEC) {
        // both rows' vectors in flight together (ld16_clamped), one round trip
        const uint4 wt = ld16_clamped<TDT>(R.trow, e0, last_whole_vec<TDT>(R.V));
        uint4 wd = make_uint4(0u, 0u, 0u, 0u);
        if (R.resid) wd = ld16_clamped<DDT>(R.drow, e0, last_whole_vec<DDT>(R.V));
        finish16<TDT>(wt, R.trow, e0, R.V, xt);
        if (R.resid) finish16<DDT>(wd, R.drow, e0, R.V, xd);
    } else {
        load_vecn<TDT, VEC>(R.trow, e0, R.V, R.t_al, xt);
        if (R.resid) {
            load_vecn<DDT, VEC>(R.drow, e0, R.V, R.d_al, xd);   // dprobs dispatches DDT = F32
        }
    }
    pair_weights_from<TDT, DDT, FAST>(R, e0, xt, xd, w, pw);
}

// the weights of pair_weights from the loaded values
template <int TDT, int DDT, bool FAST>
__device__ __forceinline__ void pair_weights_from(const PairRows& R, int64_t e0, const float* xt, const float* xd,
                                                  float* w, float* pw) {
    constexpr int VEC = PairVec<TDT, DDT>::kVec;
    float yt_v[VEC], yd_v[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) { yt_v[k] = xt[k]; yd_v[k] = R.resid ? xd[k] : 0.f; }
    if constexpr (!FAST) {
        process_vec<TDT, VEC>(yt_v, e0, R.tT, R.t_keep, R.kt);
        if (R.resid && !R.dprobs) process_vec<DDT, VEC>(yd_v, e0, R.dT, R.d_keep, R.kd);
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const int64_t j = e0 + k;
        const float yt = yt_v[k];
        const float p = prob_fast<TDT>(yt, R.mst.x, R.t_inv);
        float v = p;
        if (R.resid) {
            float q;
            if (R.dprobs) {
                q = xd[k];
            } else {
                q = prob_fast<DDT>(yd_v[k], R.msd.x, R.d_inv);
            }
            const float diff = p - q;
            v = diff > 0.f ? diff : 0.f;
        }
        w[k] = j < R.V ? v : 0.f;
        if (pw) pw[k] = j < R.V ? p : 0.f;
    }
}

// Poll-mode tag of k_sample's chunk record c of sequence b (k_draw_lean's protocol): the sequence's
// epoch (counter set 3, advanced by its consumer after every call) hashed with b and c, salted
// apart from k_draw_lean's row records, which share the region.
__device__ __forceinline__ uint32_t sample_tag(uint32_t epoch, int b, int c) {
    uint32_t h = epoch * 0x9E3779B1u + (uint32_t)b * 0x85EBCA77u + (uint32_t)c * 0xC2B2AE3Du + 0x5A3B1E7Du;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;   // murmur3 fmix32
    return h | 1u;   // never 0 (the counter path's records carry 0)
}

// Perf-mode sampling is a two-level inverse CDF.  Each sampling chunk c draws its own candidate
// j_c with an independent Philox U'_c (chunk_pick, on the weights it holds in registers); the
// sequence's tail then picks the chunk on the fp64 running sum of the chunk totals with U
// (pick_chunk) and returns j_c.  P(c) = S_c / ΣS and P(j | c) = w_j / S_c, so the draw is w_j / Σw
// up to the rounding of the chunk totals (~1e-7 relative), with no per-element noise and no
// dependent reload of the chosen chunk.

// The element of one chunk (whole workgroup; the thread's EPT weights in registers) whose interval
// of the fp64 running sum in (thread, k) order holds u * total.  Every element's interval has its
// exact fp32 weight as width.  Returns the position tid * EPT + k (uniform), -1 without positive
// weight; total: the chunk's fp64 Σ weight, ptotal: the block sum of pextra (fixed order).
// chunk_pick_tot: the same with the thread's total given (k_draw's lean path sums its weights in
// fp32: the walk's fp64 intervals then tile the thread's interval up to that rounding, ~EPT ulp).
template <int EPT>
__device__ __forceinline__ int chunk_pick_tot(const float* wv, double tot, double u, float pextra, double& total,
                                              float& ptotal, uint4* early = nullptr, uint32_t early_tag = 0u) {
    constexpr int NW = kThreads / kWave;
    __shared__ double s_wtot[NW];
    __shared__ float s_ptot[NW];
    __shared__ int s_pos[NW], s_lastp[NW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // exclusive fp64 prefix of the thread totals in thread order: DPP scan, wave offsets via LDS
    const double wincl = wave_incl_scan_d(tot);
    double excl = dpp_d<0x138, 0xF, true>(0.0, wincl);   // wave_shr:1 -> the previous lane's inclusive
    const float wp = wave_sum(pextra);
    if (lane == 63) {
        s_wtot[w] = wincl;
        s_ptot[w] = wp;
    }
    __syncthreads();
    // wave offset first, then the lane's bounds from it: lane 63's end is the next wave's offset
    double T = 0.0, woff = 0.0;
    float PT = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        if (k == w) woff = T;
        T += s_wtot[k];
        PT += s_ptot[k];
    }
    excl += woff;
    const double end = woff + wincl;
    total = T;
    ptotal = PT;
    // split records (fused verify): the chunk's totals go out now, before the in-chunk walk, so the
    // finisher can pick the chunk while the candidates are still being drawn
    if (early && threadIdx.x == 0)
        st_coh16(early, make_uint4(__float_as_uint((float)T), __float_as_uint(PT), 0xffffffffu, early_tag));
    const double t = u * T;
    // Thread intervals [excl, end) tile the running total exactly (end is the scan's own inclusive
    // value, which is the next thread's excl), so at most one thread holds t and only it walks its
    // elements; the wave's last thread with positive weight finds its last positive element for
    // the rounding fallback.  Every other lane skips the per-element loop.
    const bool hit = tot > 0.0 && excl <= t && t < end;
    const uint64_t hm = __ballot(hit), lm = __ballot(tot > 0.0);
    const int last_lane = lm ? 63 - __builtin_clzll(lm) : -1;
    if (hit || lane == last_lane) {
        int mypos = INT_MAX, lastp = -1;
        double run = excl;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            run += (double)wv[k];
            if (wv[k] > 0.f) {
                lastp = threadIdx.x * EPT + k;
                if (run > t && mypos == INT_MAX) mypos = threadIdx.x * EPT + k;
            }
        }
        // the hit thread's own rounding fallback: its last positive element
        if (hit) s_pos[w] = mypos != INT_MAX ? mypos : lastp;
        if (lane == last_lane) s_lastp[w] = lastp;
    }
    if (lane == 0) {
        if (!hm) s_pos[w] = INT_MAX;
        if (!lm) s_lastp[w] = -1;
    }
    __syncthreads();
    int pos = INT_MAX, lp = -1;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        pos = s_pos[k] < pos ? s_pos[k] : pos;
        lp = s_lastp[k] > lp ? s_lastp[k] : lp;
    }
    // rounding can leave t at/after the running total's end: the last positive element
    return pos == INT_MAX ? lp : pos;
}
template <int EPT>
__device__ __forceinline__ int chunk_pick(const float* wv, double u, float pextra, double& total, float& ptotal,
                                          uint4* early = nullptr, uint32_t early_tag = 0u) {
    double tot = 0.0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) tot += (double)wv[k];
    return chunk_pick_tot<EPT>(wv, tot, u, pextra, total, ptotal, early, early_tag);
}

// vocabulary index of chunk_pick's position in the chunk starting at base
template <int TDT, int DDT, int EPT>
__device__ __forceinline__ int64_t chunk_elem(int64_t base, int pos) {
    constexpr int VEC = PairVec<TDT, DDT>::kVec;
    const int tid = pos / EPT, k = pos - tid * EPT, v = k / VEC;
    return base + ((int64_t)v * kThreads + tid) * VEC + (k - v * VEC);
}

// The chunk of sequence b (whole workgroup; chunk totals lw staged in LDS): the first whose fp64
// running total in chunk order exceeds u * Σ, u = cdf_uniform(noise, b) (Philox U[0,1) at 53 bits,
// computed by the caller ahead of the tail); -1: no positive total.
__device__ __forceinline__ int pick_chunk(const Plan& P, double u, const float* lw) {
    __shared__ int s_chunk;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < kWave && P.rn_chunks <= kWave) {   // one scan serves both passes
        const float sv = lane < P.rn_chunks ? lw[lane] : 0.f;
        const double incl = wave_incl_scan_d((double)sv);
        const double t = u * lane_d(incl, 63);
        const uint64_t hit = __ballot(incl > t && sv > 0.f), pos = __ballot(sv > 0.f);
        if (lane == 0) s_chunk = hit ? __builtin_ctzll(hit) : (pos ? 63 - __builtin_clzll(pos) : -1);
    } else if (threadIdx.x < kWave) {
        int chunk = -1, lastpos = -1;
        double total = 0.0;
        for (int c0 = 0; c0 < P.rn_chunks; c0 += kWave) {   // pass 1 (one group for V <= 128 Ki)
            const float sv = c0 + lane < P.rn_chunks ? lw[c0 + lane] : 0.f;
            total = lane_d(total + wave_incl_scan_d((double)sv), 63);
        }
        const double t = u * total;
        double base = 0.0;
        for (int c0 = 0; c0 < P.rn_chunks && chunk < 0; c0 += kWave) {
            const float sv = c0 + lane < P.rn_chunks ? lw[c0 + lane] : 0.f;
            const double incl = base + wave_incl_scan_d((double)sv);
            const uint64_t hit = __ballot(incl > t && sv > 0.f);
            const uint64_t pos = __ballot(sv > 0.f);
            if (pos) lastpos = c0 + 63 - __builtin_clzll(pos);
            if (hit) chunk = c0 + __builtin_ctzll(hit);
            base = lane_d(incl, 63);
        }
        // rounding can leave t at/after the total: the last positive chunk
        if (lane == 0) s_chunk = chunk >= 0 ? chunk : lastpos;
    }
    __syncthreads();
    return s_chunk;
}

// Token of sequence b once every chunk partial has landed (whole workgroup): the chunk pick over
// the staged chunk totals and that chunk's own candidate for stochastic rows, the exact
// argmax-candidate pick for greedy ones; then the outputs and the engine state.  One memory round
// trip: engine-state read issued first, every chunk partial staged into LDS in one cooperative
// load.  Only the engine's den <= 1e-12 fallback re-reads a chunk (its p weights).
template <int TDT, int DDT, bool FAST, bool STOCH, int EPT = 8>
__device__ __forceinline__ void sample_finish(const Plan& P, const Decision& d, int b, PairRows R, double u_row,
                                              int wg_id, const uint32_t* poll_epoch = nullptr) {
    constexpr int VEC = PairVec<TDT, DDT>::kVec, NV = EPT / VEC;
    const bool engine_state = P.rule == SD_RULE_ENGINE && P.generated != nullptr;
    int64_t acc0 = 0;
    if (threadIdx.x == 0 && engine_state && (d.status & SD_ROW_DONE)) acc0 = P.accepted_count[b];   // early
    // the stop list into registers now, into LDS after the partials' loads are issued (one round trip)
    __shared__ int64_t lstops[kLdsStops];   // read by thread 0 at the end
    const bool stop_lane = threadIdx.x < P.n_stop && threadIdx.x < kLdsStops;
    const int64_t stop_v = stop_lane ? P.stops[threadIdx.x] : 0;
    int64_t x = -1;
    float mass = NAN;
    int32_t status = d.status;
    __shared__ int32_t s_xstat;   // poll mode: a record that never arrived
    if (threadIdx.x == 0) s_xstat = 0;
    if (poll_epoch) __syncthreads();
    if constexpr (STOCH) {
        __shared__ float l_sum[kTailChunks], l_pv[kTailChunks];
        __shared__ int32_t l_cand[kTailChunks];
        __shared__ float s_mass;
        if (d.mode != kModeNone) {
            const float4* rp = reinterpret_cast<const float4*>(P.sprec) + (int64_t)b * P.rn_chunks;
            for (int k = threadIdx.x; k < P.rn_chunks; k += kThreads) {
                uint4 v = ld_coh16(rp + k);
                if (poll_epoch) {   // poll mode: re-read until the record carries this call's tag (bounded)
                    const uint32_t tag = sample_tag(*poll_epoch, b, k);
                    uint64_t sw_ = 0; for (int spin = 0; v.w != tag; ++spin) {
                        if (!spin_more(spin, P.spin_limit, sw_)) { atomicOr(&s_xstat, SD_ROW_EXCHANGE_TIMEOUT | SD_ROW_INVALID_DIST); break; }
                        __builtin_amdgcn_s_sleep(1);
                        v = ld_coh16(rp + k);
                    }
                }
                l_sum[k] = __uint_as_float(v.x);
                l_pv[k] = __uint_as_float(v.y);
                l_cand[k] = (int32_t)v.z;
                if ((int32_t)v.z == kLostDecision) atomicOr(&s_xstat, SD_ROW_EXCHANGE_TIMEOUT | SD_ROW_INVALID_DIST);
            }
            if (stop_lane) lstops[threadIdx.x] = stop_v;
            __syncthreads();
            if (threadIdx.x < kWave) {   // Σ residual, fixed order (lane-strided, then a butterfly)
                float sacc = 0.f;
                for (int k = threadIdx.x; k < P.rn_chunks; k += kWave) sacc += l_sum[k];
                sacc = wave_sum(sacc);
                if (threadIdx.x == 0) s_mass = sacc;
            }
            __syncthreads();
            const float S = s_mass;
            SD_TS(wg_id, 4);
            // engine/infer_engine.py:319-321: den <= 1e-12 -> multinomial(p) over the target row
            const bool fallback = d.mode == kModeResid && P.rule == SD_RULE_ENGINE && (double)S <= 1e-12;
            const int c = pick_chunk(P, u_row, fallback ? l_pv : l_sum);
            SD_TS(wg_id, 7);
            if (c >= 0 && !fallback && P.crec && poll_epoch) {
                // split records: the picked chunk's candidate (bounded wait; a lost one flags the row)
                __shared__ int32_t s_cand;
                if (threadIdx.x == 0) {
                    const uint4* cr = P.crec + (int64_t)b * P.rn_chunks + c;
                    const uint32_t tag = sample_tag(*poll_epoch, b, c) ^ 0x5bd1e995u;
                    uint4 v = ld_coh16(cr);
                    uint64_t sw_ = 0; for (int spin = 0; v.w != tag && spin_more(spin, P.spin_limit, sw_); ++spin) {
                        __builtin_amdgcn_s_sleep(1);
                        v = ld_coh16(cr);
                    }
                    if (v.w != tag) s_xstat |= SD_ROW_EXCHANGE_TIMEOUT | SD_ROW_INVALID_DIST;
                    s_cand = v.w == tag ? (int32_t)v.x : -1;
                }
                __syncthreads();
                x = s_cand;
            } else if (c >= 0 && !fallback) {
                x = l_cand[c];
            } else if (c >= 0) {
                // the chosen chunk's p weights, re-read, and the same in-chunk draw as k_sample's
                R.resid = false;   // same slot, same row stats: weights p
                status = (status & ~SD_ROW_RESIDUAL) | SD_ROW_FALLBACK_P;
                const int64_t base = (int64_t)c * P.rchunk;
                float wv[EPT];
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    pair_weights<TDT, DDT, FAST>(R, base + ((int64_t)v * kThreads + threadIdx.x) * VEC, wv + v * VEC);
                double T;
                float PT;
                const int pos = chunk_pick<EPT>(wv, cdf_uniform(P.noise, (uint32_t)b, 1u + (uint32_t)c), 0.f, T, PT);
                x = pos < 0 ? -1 : chunk_elem<TDT, DDT, EPT>(base, pos);
            } else if (fallback) {
                status = (status & ~SD_ROW_RESIDUAL) | SD_ROW_FALLBACK_P;
            }
            SD_TS(wg_id, 5);
            if (d.mode == kModeResid) mass = S;
            if (x < 0) status |= SD_ROW_INVALID_DIST;   // no positive weight: torch.multinomial raises
        }
    } else {
        if (d.mode != kModeNone && threadIdx.x < kWave) pick_wave(P, b, d, x, mass, status);
    }
    if (poll_epoch) {
        __syncthreads();
        status |= s_xstat;
    }
    if (threadIdx.x == 0) finalize_write(P, b, d, x, mass, status, acc0, lstops);
    SD_TS(wg_id, 6);
}

__device__ __forceinline__ Decision load_decision(const Plan& P, int b) {
    Decision d = P.dec[b];
    if (d.mode < kModeNone || d.mode > kModePRow || d.slot < 0 || d.slot >= P.n_tslots) d.mode = kModeNone;
    return d;
}

// Stochastic sampling chunk c of sequence b (whole workgroup): the chunk's Σ weight, Σ p, and its own
// inverse-CDF candidate (pick_chunk's comment), published as one 16-byte record (k_draw's layout;
// .w = the poll-mode tag, or 0).
// chunk c's draw from weights already in registers (sample_chunk's second half)
template <int TDT, int DDT, int EPT>
__device__ __forceinline__ void sample_chunk_pick(const Plan& P, int b, int c, const float* wv, float psum, uint32_t tag,
                                                  int wg_id, double u) {
    const int64_t base = (int64_t)c * P.rchunk;
    double T;
    float PT;
    uint4* rec = P.sprec + (int64_t)b * P.rn_chunks + c;
    const int pos = chunk_pick<EPT>(wv, u, psum, T, PT, P.crec ? rec : nullptr, tag);
    SD_TS(wg_id, 9);
    const uint32_t cand = (uint32_t)(pos < 0 ? -1 : (int32_t)chunk_elem<TDT, DDT, EPT>(base, pos));
    if (threadIdx.x == 0) {
        if (P.crec)   // split: the candidate on its own record, its own tag
            st_coh16(P.crec + (int64_t)b * P.rn_chunks + c, make_uint4(cand, 0u, 0u, tag ^ 0x5bd1e995u));
        else          // {Σ w, Σ p, candidate, tag}
            st_coh16(rec, make_uint4(__float_as_uint((float)T), __float_as_uint(PT), cand, tag));
    }
}

template <int TDT, int DDT, bool FAST, int EPT = 8>
__device__ __forceinline__ void sample_chunk(const Plan& P, const PairRows& R, int b, int c, uint32_t tag, int wg_id = 0,
                                             double u = -1.0) {
    constexpr int VEC = PairVec<TDT, DDT>::kVec, NV = EPT / VEC;
    // the chunk's uniform (its Philox offset may be a device load) before the rows' loads
    if (u < 0.0) u = cdf_uniform(P.noise, (uint32_t)b, 1u + (uint32_t)c);
    float psum = 0.f;
    const int64_t base = (int64_t)c * P.rchunk;
    float wv[EPT];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        float pv[VEC];
        pair_weights<TDT, DDT, FAST>(R, base + ((int64_t)v * kThreads + threadIdx.x) * VEC, wv + v * VEC, pv);
#pragma unroll
        for (int k = 0; k < VEC; ++k) psum += pv[k];
    }
    SD_TS(wg_id, 8);
    sample_chunk_pick<TDT, DDT, EPT>(P, b, c, wv, psum, tag, wg_id, u);
}

// grid (chunk, B).  STOCH: chunk Σ weight; greedy (!STOCH): the exact argmax-candidate bodies.
// The last workgroup of each sequence (poll mode: its last chunk) runs sample_finish.  (A variant
// that moved the decision into every sampling workgroup measured 63.9 vs 61.9 us per step and was
// removed in round 5, with the own-launch decide / finish kernels.)
template <int TDT, int DDT, bool FAST, bool STOCH>
__global__ void __launch_bounds__(kThreads) SD_SGPR_CAP k_sample(Plan P) {
    constexpr int EPT = 8;
    constexpr bool TAIL = true;
    const int wg_id = 8192 + blockIdx.y * gridDim.x + blockIdx.x;
    int b, c;
    if (P.xcd_affine) affine_split(wg_id - 8192, (int)gridDim.x, b, c);
    else { b = blockIdx.y; c = blockIdx.x; }
    SD_TS(wg_id, 0);
    const Decision d = load_decision(P, b);
    // the tail's chunk-pick uniform, computed while the decision load is in flight
    const double u_row = STOCH ? cdf_uniform(P.noise, (uint32_t)b) : 0.0;
    // poll mode (stochastic tails): this call's epoch of sequence b, read beside the decision load
    const bool poll = STOCH && P.spoll;
    uint32_t epoch = 0;
    if (poll) epoch = seq_epoch(P, b);
    PairRows R{};
    if (d.mode != kModeNone) {
        if constexpr (STOCH) {
            // RESID also sums p: the engine's den <= 1e-12 fallback samples the target row itself
            R = pair_rows<TDT, DDT>(P, d, b);
            SD_TS(wg_id, 1);
            sample_chunk<TDT, DDT, FAST>(P, R, b, c, poll ? sample_tag(epoch, b, c) : 0u, wg_id);
        } else {
            const float2 mst = P.rowstat[b * P.slots + d.slot];
            const float2 msd = d.mode == kModeResid && !P.draft_is_probs ? P.rowstat[b * P.slots + P.n_tslots + d.slot]
                                                                         : make_float2(0.f, 1.f);
            if (d.mode == kModeResid) resid_body<TDT, DDT, SD_NOISE_PHILOX, EPT, FAST>(P, d, b, c, mst, msd);
            else prow_body<TDT, SD_NOISE_PHILOX, EPT, FAST>(P, d, b, c, mst);
        }
    }
    SD_TS(wg_id, 2);
    if constexpr (TAIL) {
        if (poll) {
            // the sequence's last chunk (the ragged one: least work) is its consumer; the others
            // have published their records and are done — no counter, no write-ack wait
            if (c != P.rn_chunks - 1) return;
            __shared__ uint32_t s_epoch;
            if (threadIdx.x == 0) s_epoch = epoch;
            __syncthreads();
            sample_finish<TDT, DDT, FAST, STOCH>(P, d, b, R, u_row, wg_id, &s_epoch);
            if (threadIdx.x == 0)
                seq_advance(P, b, epoch);
            return;
        }
        __shared__ int s_last;
        if (threadIdx.x == 0) s_last = arrive_last(seq_counter(P.cnt, 1, b), (uint32_t)P.rn_chunks);
        __syncthreads();
        SD_TS(wg_id, 3);
        if (!s_last) return;
        sample_finish<TDT, DDT, FAST, STOCH>(P, d, b, R, u_row, wg_id);
    }
}

// ------------------------------------------------------------------ fused verify (k_stats<.., SAMP>)
// The decider hands its decision to the sequence's sampling workgroups as two tagged 16-byte records
// (k_draw_lean's protocol: write-through stores, each record validated by its own tag):
//   A = {mode | slot << 8, mst.x, mst.y, tag}, B = {msd.x, msd.y, 0, tag}.
// A sampler publishes its chunk record (sample_chunk) — or, for a sequence with nothing to sample,
// an empty one — so the decider always waits for every sampler before it advances the epoch.
#ifndef SD_SAMP_SLEEP
#define SD_SAMP_SLEEP 1   // fused samplers' decision poll interval (s_sleep units of 64 clocks)
#endif
constexpr int kFusedEpt = 8;                       // k_sample's chunking: 2048-element chunks, the same draws

__device__ __forceinline__ uint32_t dec_tag(uint32_t epoch, int b, int k) {
    uint32_t h = epoch * 0x9E3779B1u + (uint32_t)b * 0x85EBCA77u + (uint32_t)k * 0xC2B2AE3Du + 0x1B873593u;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;   // murmur3 fmix32
    return h | 1u;
}

// pair_weights_from's FAST weights of one 16-bit vector pair (T = 1, no processor, drafter logits),
// the same values and psum order, with the row's mode (RESID) and the chunk's raggedness (WHOLE:
// every element inside the vocabulary) out of the element loop
template <int DT, bool RESID, bool WHOLE>
__device__ __forceinline__ void fused_weights_v(const PairRows& R, int64_t e0, uint4 rt, uint4 rd, float* w, float& psum) {
    constexpr int VEC = Elem<DT>::kVec;
    float xt[VEC], xd[VEC];
    if (WHOLE) unpack16<DT>(rt, xt);
    else finish16<DT>(rt, R.trow, e0, R.V, xt);
    if (RESID) {
        if (WHOLE) unpack16<DT>(rd, xd);
        else finish16<DT>(rd, R.drow, e0, R.V, xd);
    }
    psum = 0.f;
    if constexpr (DT == SD_BF16) {
        // pairs on packed fp32 (v_pk_add / v_pk_mul: the same IEEE operations as prob_fast's, two
        // lanes per instruction) and one v_cvt_pk_bf16_f32 per pair
        typedef float f2 __attribute__((ext_vector_type(2)));
        typedef __bf16 h2 __attribute__((ext_vector_type(2)));
        constexpr float kL2e = 1.44269502162933349609375f;
        auto prob2 = [](f2 y, float m, float inv) {
            f2 e = (y - m) * kL2e;
            e.x = __builtin_amdgcn_exp2f(e.x);
            e.y = __builtin_amdgcn_exp2f(e.y);
            return __builtin_convertvector(__builtin_convertvector(e * inv, h2), f2);
        };
#pragma unroll
        for (int k = 0; k < VEC; k += 2) {
            f2 p = prob2(f2{xt[k], xt[k + 1]}, R.mst.x, R.t_inv);
            f2 v = p;
            if (RESID) {
                const f2 diff = p - prob2(f2{xd[k], xd[k + 1]}, R.msd.x, R.d_inv);
                v.x = diff.x > 0.f ? diff.x : 0.f;
                v.y = diff.y > 0.f ? diff.y : 0.f;
            }
            if (!WHOLE) {
                if (!(e0 + k < R.V)) v.x = p.x = 0.f;
                if (!(e0 + k + 1 < R.V)) v.y = p.y = 0.f;
            }
            w[k] = v.x;
            w[k + 1] = v.y;
            psum += p.x;
            psum += p.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            float p = prob_fast<DT>(xt[k], R.mst.x, R.t_inv);
            float v = p;
            if (RESID) {
                const float diff = p - prob_fast<DT>(xd[k], R.msd.x, R.d_inv);
                v = diff > 0.f ? diff : 0.f;
            }
            if (!WHOLE && !(e0 + k < R.V)) v = p = 0.f;
            w[k] = v;
            psum += p;
        }
    }
}
template <int DT>
__device__ __forceinline__ void fused_weights(const PairRows& R, int cc, int rchunk, int64_t e0, uint4 rt, uint4 rd,
                                              float* w, float& psum) {
    const bool whole = (int64_t)(cc + 1) * rchunk <= R.V;
    if (R.resid) {
        if (whole) fused_weights_v<DT, true, true>(R, e0, rt, rd, w, psum);
        else fused_weights_v<DT, true, false>(R, e0, rt, rd, w, psum);
    } else {
        if (whole) fused_weights_v<DT, false, true>(R, e0, rt, rd, w, psum);
        else fused_weights_v<DT, false, false>(R, e0, rt, rd, w, psum);
    }
}

template <int DT, bool FAST, int MAXP>
__device__ __forceinline__ void fused_sampler(const Plan& P, int b, int c, int wg_id) {
    __shared__ uint4 s_rec[2];
    __shared__ uint32_t s_ep;
    __shared__ int32_t s_ok;
    SD_TS(wg_id, 0);
    // sampler c draws chunks [c * cps, c * cps + cps) of the sequence's rn_chunks, in pairs (pair q:
    // chunks 2q, 2q + 1 of the row); the chunks, their uniforms and their records are k_sample's,
    // so the grouping never changes a draw
    const int cps = P.samp_cps, q0 = c * (cps >> 1), nq = cps >> 1;
    // the first pair's in-chunk uniforms depend on (b, chunk) only: computed (and the Philox offset,
    // a device load under graph replays, fetched) while the decision is still being made
    double u0 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 1u + 2u * (uint32_t)q0));
    double u1 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 2u + 2u * (uint32_t)q0));
    if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        uint32_t ep = 0;
        if (lane == 0) ep = seq_epoch(P, b);
        ep = __builtin_amdgcn_readfirstlane(ep);
        bool have = lane >= 2;
        uint4 r = make_uint4(0u, 0u, 0u, 0u);
        const uint32_t tag = lane < 2 ? dec_tag(ep, b, lane) : 0u;
        uint64_t sw_ = 0; for (int spin = 0;; ++spin) {
            if (!have && P.spin_limit >= 0) {   // < 0: the test hook, the decision counts as lost
                r = ld_coh16(P.drec + 2 * b + lane);
                have = r.w == tag;
            }
            if (__all(have)) break;
            if (!spin_more(spin, P.spin_limit, sw_)) break;   // bounded: the finisher flags the row
            __builtin_amdgcn_s_sleep(SD_SAMP_SLEEP);   // the decision is microseconds away
        }
        if (lane < 2) s_rec[lane] = r;
        if (lane == 0) { s_ep = ep; s_ok = __all(have) ? 1 : 0; }
    }
    __syncthreads();
    SD_TS(wg_id, 1);
    const uint32_t ep = s_ep;
    const uint4 A = s_rec[0], Bq = s_rec[1];
    Decision d{};
    d.mode = (int32_t)(A.x & 0xffu);
    d.slot = (int32_t)(A.x >> 8);
    d.mst = make_float2(__uint_as_float(A.y), __uint_as_float(A.z));
    d.msd = make_float2(__uint_as_float(Bq.x), __uint_as_float(Bq.y));
    const bool ok = s_ok != 0;
    // The decision never came: publish NOTHING.  The epoch this sampler read may already be the next
    // call's (it was dispatched after its decider gave up waiting and advanced it), and a record
    // tagged with it would pass the next call's check; the decider's own bounded wait flags the row
    // (SD_ROW_EXCHANGE_TIMEOUT) without it.
    if (!ok) return;
    if (d.mode <= kModeNone || d.mode > kModePRow || d.slot < 0 || d.slot >= P.n_tslots) {
        // nothing to draw: empty records for every chunk of this sampler (the decider waits for all)
        if ((int)threadIdx.x < cps && 2 * q0 + (int)threadIdx.x < P.rn_chunks) {
            const int cc = 2 * q0 + (int)threadIdx.x;
            st_coh16(reinterpret_cast<float4*>(P.sprec) + (int64_t)b * P.rn_chunks + cc,
                     make_uint4(0u, 0u, (uint32_t)-1, sample_tag(ep, b, cc)));
        }
        return;
    }
    const PairRows R = pair_rows<DT, DT>(P, d, b);
    constexpr int VEC = Elem<DT>::kVec, NV = kFusedEpt / VEC;
    if (!(R.t_al && (!R.resid || R.d_al) && P.V >= VEC)) {   // misaligned rows: one chunk at a time
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            const int q = q0 + k, c0 = 2 * q, c1 = 2 * q + 1;
            if (k >= nq || c0 >= P.rn_chunks) break;
            if (k > 0) {
                u0 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 1u + 2u * (uint32_t)q));
                u1 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 2u + 2u * (uint32_t)q));
            }
            sample_chunk<DT, DT, FAST, kFusedEpt>(P, R, b, c0, sample_tag(ep, b, c0), wg_id, u0);
            if (c1 < P.rn_chunks) sample_chunk<DT, DT, FAST, kFusedEpt>(P, R, b, c1, sample_tag(ep, b, c1), wg_id, u1);
        }
        return;
    }
    const int64_t lastv = last_whole_vec<DT>(P.V);
    float wv[kFusedEpt], psum;
    if constexpr (NV == 1 && FAST) {
        // 16-bit rows (one vector per thread and chunk): a pair's four vectors in flight at once, the
        // next pair's issued before this pair's weights and draws (the sampled row's mode and the
        // chunk's raggedness hoisted out of the element loop)
        const int64_t tid8 = (int64_t)threadIdx.x * VEC;
        auto ld_pair = [&](int q, uint4& t0, uint4& d0, uint4& t1, uint4& d1) {
            const int64_t e0 = (int64_t)(2 * q) * P.rchunk + tid8, e1 = e0 + P.rchunk;
            t0 = ld16_clamped<DT>(R.trow, e0, lastv);
            d0 = R.resid ? ld16_clamped<DT>(R.drow, e0, lastv) : make_uint4(0u, 0u, 0u, 0u);
            t1 = make_uint4(0u, 0u, 0u, 0u);
            d1 = t1;
            if (2 * q + 1 < P.rn_chunks) {
                t1 = ld16_clamped<DT>(R.trow, e1, lastv);
                if (R.resid) d1 = ld16_clamped<DT>(R.drow, e1, lastv);
            }
        };
        // one pair in flight ahead (ticket order: the next pair's vectors load while this pair's
        // weights and draws run)
        uint4 t0, d0, t1, d1;
        ld_pair(q0, t0, d0, t1, d1);
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            const int q = q0 + k, c0 = 2 * q, c1 = 2 * q + 1;
            if (k >= nq || c0 >= P.rn_chunks) break;
            if (!SD_SAMP_PREFETCH && k > 0) ld_pair(q, t0, d0, t1, d1);
            uint4 nt0 = t0, nd0 = d0, nt1 = t1, nd1 = d1;
            if (SD_SAMP_PREFETCH && k + 1 < MAXP && k + 1 < nq && 2 * (q + 1) < P.rn_chunks) ld_pair(q + 1, nt0, nd0, nt1, nd1);
            if (k > 0) {
                u0 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 1u + 2u * (uint32_t)q));
                u1 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 2u + 2u * (uint32_t)q));
            }
            const int64_t e0 = (int64_t)c0 * P.rchunk + tid8, e1 = e0 + P.rchunk;
            fused_weights<DT>(R, c0, P.rchunk, e0, t0, d0, wv, psum);
            SD_TS(wg_id, 8);
            sample_chunk_pick<DT, DT, kFusedEpt>(P, b, c0, wv, psum, sample_tag(ep, b, c0), wg_id, u0);
            if (c1 < P.rn_chunks) {
                fused_weights<DT>(R, c1, P.rchunk, e1, t1, d1, wv, psum);
                sample_chunk_pick<DT, DT, kFusedEpt>(P, b, c1, wv, psum, sample_tag(ep, b, c1), wg_id, u1);
            }
            t0 = nt0; d0 = nd0; t1 = nt1; d1 = nd1;
        }
        SD_TS(wg_id, 2);
        return;
    }
    uint4 rt[NV], rd[NV];
    auto issue = [&](int cc) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t e0 = (int64_t)cc * P.rchunk + ((int64_t)v * kThreads + threadIdx.x) * VEC;
            rt[v] = ld16_clamped<DT>(R.trow, e0, lastv);
            rd[v] = R.resid ? ld16_clamped<DT>(R.drow, e0, lastv) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto weights = [&](int cc, float* wv, float& psum) {
        psum = 0.f;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t e0 = (int64_t)cc * P.rchunk + ((int64_t)v * kThreads + threadIdx.x) * VEC;
            float xt[VEC], xd[VEC], pv[VEC];
            finish16<DT>(rt[v], R.trow, e0, P.V, xt);
            if (R.resid) finish16<DT>(rd[v], R.drow, e0, P.V, xd);
            pair_weights_from<DT, DT, FAST>(R, e0, xt, xd, wv + v * VEC, pv);
#pragma unroll
            for (int k = 0; k < VEC; ++k) psum += pv[k];
        }
    };
    // the general rows (fp32, processors): chunk c0's vectors, its weights, then chunk c1's loads go
    // out before c0's draw; only the weights of one chunk and the raw vectors of the other are live
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
        const int q = q0 + k, c0 = 2 * q, c1 = 2 * q + 1;
        if (k >= nq || c0 >= P.rn_chunks) break;
        const bool has1 = c1 < P.rn_chunks;
        if (k > 0) {
            u0 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 1u + 2u * (uint32_t)q));
            u1 = uniform_d(cdf_uniform(P.noise, (uint32_t)b, 2u + 2u * (uint32_t)q));
        }
        issue(c0);
        weights(c0, wv, psum);
        if (NV == 1 && has1) issue(c1);   // fp32 rows (two vectors per chunk): after the draw, no spills
        SD_TS(wg_id, 8);
        sample_chunk_pick<DT, DT, kFusedEpt>(P, b, c0, wv, psum, sample_tag(ep, b, c0), wg_id, u0);
        if (has1) {
            if (NV != 1) issue(c1);
            weights(c1, wv, psum);
            sample_chunk_pick<DT, DT, kFusedEpt>(P, b, c1, wv, psum, sample_tag(ep, b, c1), wg_id, u1);
        }
    }
    SD_TS(wg_id, 2);
}

// The decider after deciding (whole workgroup): the decision records for the samplers, then their
// chunk records (always every one of them, so none is left polling an advanced epoch) and the
// token / outputs as k_sample's tail writes them.
template <int DT, bool FAST>
__device__ __forceinline__ void fused_finish(const Plan& P, int b, const Decision& d0, uint32_t epoch, int wg_id,
                                             double u_row) {
    Decision d = d0;
    if (d.mode < kModeNone || d.mode > kModePRow || d.slot < 0 || d.slot >= P.n_tslots) d.mode = kModeNone;
    if (threadIdx.x == 0) {
        const uint32_t mslot = (uint32_t)(d.mode & 0xff) | ((uint32_t)(d.mode != kModeNone ? d.slot : 0) << 8);
        st_coh16(P.drec + 2 * b, make_uint4(mslot, __float_as_uint(d.mst.x), __float_as_uint(d.mst.y), dec_tag(epoch, b, 0)));
        st_coh16(P.drec + 2 * b + 1, make_uint4(__float_as_uint(d.msd.x), __float_as_uint(d.msd.y), 0u, dec_tag(epoch, b, 1)));
    }
    PairRows R{};
    if (d.mode != kModeNone) R = pair_rows<DT, DT>(P, d, b);
    if (d.mode == kModeNone) {
        // every sampler's (empty) record before the epoch moves on
        const float4* rp = reinterpret_cast<const float4*>(P.sprec) + (int64_t)b * P.rn_chunks;
        for (int k = threadIdx.x; k < P.rn_chunks; k += kThreads) {
            const uint32_t tag = sample_tag(epoch, b, k);
            uint64_t sw_ = 0; for (int spin = 0; ld_coh16(rp + k).w != tag && spin_more(spin, P.spin_limit, sw_); ++spin)
                __builtin_amdgcn_s_sleep(1);
        }
    }
    __shared__ uint32_t s_ep2;
    if (threadIdx.x == 0) s_ep2 = epoch;
    // (phase timestamps: the finish's on a row of its own, 4096 + wg)
    sample_finish<DT, DT, FAST, true, kFusedEpt>(P, d, b, R, u_row, wg_id + 4096, &s_ep2);
}

// ------------------------------------------------------------------ sd_sample kernels
// grid (chunk, R): argmax of round_dt(p / round_dt(E)) (multinomial) or p (greedy).
template <int DT, int NZ, int EPT, bool FAST = false>
__device__ void rowsample_body(const Plan& P, int r, int c) {
    __shared__ float ldsf[8];
    __shared__ int32_t ldsi[8];
    __shared__ float2 lms;
    constexpr int VEC = Elem<DT>::kVec, NV = EPT / VEC;
    if constexpr (NZ == SD_NOISE_STREAM) {
        if (P.t_stoch) {
            // the chunk's logits and noise words are loaded first (independent of the row stats),
            // then the stats, then the screened race
            const int ts_wg = r * P.rn_chunks + c;
            SD_TS(ts_wg, 0);
            const void* row = static_cast<const char*>(P.trow[0]) + r * P.tstride * (DT == SD_F32 ? 4 : 2);
            const bool al = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
            const int64_t base = (int64_t)c * P.rchunk;
            const int64_t woff = 2ll * P.V * r;
            float x[EPT];
            uint32_t wd[2 * EPT];
            int64_t jj[EPT];
            bool ok[EPT];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
                load_vec<DT>(row, e0, P.V, al, x + v * VEC);
                stream_words<VEC>(P.noise, woff, e0, wd + 2 * v * VEC);
#pragma unroll
                for (int k = 0; k < VEC; ++k) { jj[v * VEC + k] = e0 + k; ok[v * VEC + k] = e0 + k < P.V; }
            }
            if (threadIdx.x < 64) {
                const float2 ms = combine_row(P, r);
                if (threadIdx.x == 0) lms = ms;
            }
            __syncthreads();
            SD_TS(ts_wg, 1);
            const float2 ms = lms;
            const float inv_s = 1.0f / ms.y;
            if (!FAST) {   // the processed values y (T, top-k / nucleus mask)
                const RowKeep kp = P.t_keep ? keep_of(P, r) : RowKeep{-INFINITY, INT_MAX, 0, 0};
#pragma unroll
                for (int k = 0; k < EPT; ++k) x[k] = process_value<DT>(x[k], jj[k], P.tT, P.t_keep, kp);
            }
            SD_TS(ts_wg, 2);
            float pv;
            int32_t pi;
            stream_race<DT, EPT>(P.noise, woff, x, ok, wd, jj, ms.x, ms.y, inv_s, pv, pi, ldsf, ldsi);
            SD_TS(ts_wg, 3);
            if (threadIdx.x == 0) {
                ResPart& o = P.rpart[(int64_t)r * P.rn_chunks + c];
                o.pval = pv;
                o.pidx = pi;
            }
            return;
        }
    }
    if (threadIdx.x < 64) {
        const float2 ms = combine_row(P, r);
        if (threadIdx.x == 0) lms = ms;
    }
    __syncthreads();
    const float2 ms = lms;
    const void* row = static_cast<const char*>(P.trow[0]) + r * P.tstride * (DT == SD_F32 ? 4 : 2);
    const bool al = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
    const RowKeep kp = P.t_keep ? keep_of(P, r) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const int64_t base = (int64_t)c * P.rchunk;
    const int64_t woff = 2ll * P.V * r;
    const float inv_s = 1.0f / ms.y;
    float pv = -INFINITY;
    int32_t pi = INT_MAX;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float x[VEC], e[VEC];
        load_vec<DT>(row, e0, P.V, al, x);
        if (P.t_stoch) exp_noise_vec<VEC, NZ>(P.noise, woff, r, e0, P.V, e);
        process_vec<DT, VEC>(x, e0, P.tT, P.t_keep, kp);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= P.V) continue;
            const float p = prob_exact<DT>(x[k], ms.x, ms.y, inv_s);
            float val = p;
            if (P.t_stoch) {
                const float eb = round_dt<DT>(e[k]);
                val = div_round<DT>(p, eb, __builtin_amdgcn_rcpf(eb));
            }
            if (arg_better(val, (int32_t)j, pv, pi)) { pv = val; pi = (int32_t)j; }
        }
    }
    block_argmax(pv, pi, ldsf, ldsi);
    if (threadIdx.x == 0) {
        ResPart& o = P.rpart[(int64_t)r * P.rn_chunks + c];
        o.pval = pv;
        o.pidx = pi;
    }
}

template <int DT, int NZ, int EPT, bool FAST = false>
__global__ void __launch_bounds__(kThreads) k_rowsample(Plan P) {
    rowsample_body<DT, NZ, EPT, FAST>(P, blockIdx.y, blockIdx.x);
}

__global__ void __launch_bounds__(64) k_sample_finalize(Plan P) {
    const int r = blockIdx.x, lane = threadIdx.x;
    const ResPart* rp = P.rpart + (int64_t)r * P.rn_chunks;
    float pv = -INFINITY;
    int32_t pi = INT_MAX;
    for (int c = lane; c < P.rn_chunks; c += kWave)
        if (arg_better(rp[c].pval, rp[c].pidx, pv, pi)) { pv = rp[c].pval; pi = rp[c].pidx; }
    wave_argmax(pv, pi);
    const float2 ms = combine_row(P, r);
    if (lane == 0) {
        int32_t st = SD_ROW_DONE;
        if (P.t_stoch && !(ms.y > 0.f && ms.y < INFINITY)) st |= SD_ROW_INVALID_DIST;   // NaN / inf / zero mass
        if (P.t_keep) st |= keep_of(P, r).flags;
        if (P.noise.mode == SD_NOISE_STREAM && P.t_stoch && 2ll * P.V * P.B > stream_cap(P.noise))
            st |= SD_ROW_NOISE_OVERRUN;
        // no candidate at all (an all-NaN / all -inf row: the race's threshold is NaN) is an invalid
        // distribution too; a failed row's token is -1, never an index a forward could be fed
        if (pi < 0 || pi >= P.V) st |= SD_ROW_INVALID_DIST;
        if (st & SD_ROW_INVALID_DIST) pi = -1;
        P.next_token[r * P.next_token_stride] = pi;
        if (P.token_prob) {
            const void* row = static_cast<const char*>(P.trow[0]) + r * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
            const RowKeep kp = P.t_keep ? keep_of(P, r) : RowKeep{-INFINITY, INT_MAX, 0, 0};
            P.token_prob[r] = (pi >= 0 && pi < P.V) ? prob_dyn(P.tdt, row, pi, P.tT, P.t_keep, kp, ms) : NAN;
        }
        if (P.row_stats) P.row_stats[r] = ms;
        if (P.row_status) P.row_status[r] = st;
        flag_error(P.status_or, st);
        if (P.keep_out && P.t_keep) P.keep_out[r] = keep_of(P, r);
        if (r == 0 && P.words_used) *P.words_used = P.t_stoch ? 2ll * P.V * P.B : 0;
    }
}

// ------------------------------------------------------------------ k_draw (perf-mode sd_sample)
// One launch, one pass over each row: LogitsProcessor.__call__ + MultinomialProcessor.sample
// (utils/logits_processor.py:13-15,39-49) for PHILOX noise, plus the row's (max, Σexp) for the
// verify step (sd_verify_args.draft_row_stats).  grid (span, R): a workgroup holds NST stages of
// 2048 elements of row r in registers, takes their max m_c and weights w = exp(y - m_c), and
// draws its own candidate j_c by inverse CDF with U'_c (chunk_pick); it publishes
// (m_c, S_c, j_c, y_{j_c}).  The row's last arrival combines M = max m_c, S = Σ S_c·e^{m_c-M},
// picks span c with probability S_c·e^{m_c-M} / S (U, pick_chunk) and returns j_c:
// P(j) = e^{y_j-M} / S, the softmax of the processed row, with no second pass over it.
// Greedy rows keep the exact two-pass argmax (rounded-probability ties need (M, S) first).
template <int DT, bool FAST, int NST>
__global__ void __launch_bounds__(kThreads) SD_SGPR_CAP k_draw(Plan P) {
    constexpr int VEC = Elem<DT>::kVec, STEP = kThreads * VEC, EPT = NST * VEC;
    __shared__ float lm[kThreads / kWave];
    const int wg_id = blockIdx.y * gridDim.x + blockIdx.x;
    SD_TS(wg_id, 0);
    int r, c;
    if (P.xcd_affine) affine_split(wg_id, (int)gridDim.x, r, c);
    else { r = blockIdx.y; c = blockIdx.x; }
    const void* row = static_cast<const char*>(P.trow[0]) + r * P.tstride * (DT == SD_F32 ? 4 : 2);
    const bool al = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
    const RowKeep kp = (!FAST && P.t_keep) ? keep_of(P, r) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const int64_t base = (int64_t)c * NST * STEP;
    // The Philox uniforms run on the scalar unit, which every wave of the CU shares: computed by
    // each wave ahead of its loads (as the compiler scheduled them) they held back the launch's
    // load issue by ~0.7 us.  So: loads first, the span's in-chunk uniform by wave 0 alone (into
    // LDS; the span-max barrier publishes it), the tail's chunk-pick uniform by the tail's wave 1.
    __shared__ double s_u;
    double u_c;
    float y[EPT];
    float wv[EPT];
    double T;
    float PT;
    int pos;
    float m;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // lean path (T = 1, no processor, 16-bit rows, aligned, the span wholly inside the row — every
    // span of a row but its ragged last one): no per-element bounds, NaN or keep tests; the
    // compute phase is VALU-bound (every workgroup of the launch reaches it at once), so each
    // element costs an unpack, a max3 third, a subtract, a multiply, an exp and an fp32 add.
    // A NaN / +inf anywhere makes the fp32 total NaN, which flags the row as the general path does.
    constexpr bool kLeanOk = FAST && DT != SD_F32;
    if (kLeanOk && al && base + (int64_t)NST * STEP <= P.V) {
        uint4 raw[NST];
#pragma unroll
        for (int v = 0; v < NST; ++v)
            raw[v] = *reinterpret_cast<const uint4*>(static_cast<const char*>(row) + (base + (int64_t)v * STEP + threadIdx.x * VEC) * 2);
        if (w == 0) {
            const double u = cdf_uniform(P.noise, (uint32_t)r, 1u + (uint32_t)c);
            if (lane == 0) s_u = u;
        }
#pragma unroll
        for (int v = 0; v < NST; ++v) unpack16<DT>(raw[v], y + v * VEC);
        float mv = y[0];
#pragma unroll
        for (int k = 1; k + 1 < EPT; k += 2) mv = fmaxf(mv, fmaxf(y[k], y[k + 1]));
        if constexpr (EPT % 2 == 0) mv = fmaxf(mv, y[EPT - 1]);
        mv = wave_max(mv);
        if (lane == 0) lm[w] = mv;
        __syncthreads();
        m = lm[0];
#pragma unroll
        for (int k = 1; k < kThreads / kWave; ++k) m = fmaxf(m, lm[k]);
        u_c = s_u;
        SD_TS(wg_id, 1);
        float t32 = 0.f;
        if (m > -INFINITY) {
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                wv[k] = __builtin_amdgcn_exp2f((y[k] - m) * kLog2e);
                t32 += wv[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < EPT; ++k) wv[k] = 0.f;
        }
        SD_TS(wg_id, 7);
        pos = chunk_pick_tot<EPT>(wv, (double)t32, u_c, 0.f, T, PT);
        if (T != T) PT = 1.f;   // NaN / +inf in the span: the general path's flag
    } else {
    auto take = [&](int v, int64_t e0, const float* x) {
        float yv[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) yv[k] = x[k];
        if constexpr (!FAST) process_vec<DT, VEC>(yv, e0, P.tT, P.t_keep, kp);
#pragma unroll
        for (int k = 0; k < VEC; ++k) y[v * VEC + k] = e0 + k < P.V ? yv[k] : -INFINITY;
    };
    if (al && P.V >= VEC) {   // every stage's vector in flight at once (ld16_clamped)
        const int64_t last = last_whole_vec<DT>(P.V);
        uint4 raw[NST];
#pragma unroll
        for (int v = 0; v < NST; ++v) raw[v] = ld16_clamped<DT>(row, base + (int64_t)v * STEP + threadIdx.x * VEC, last);
#pragma unroll
        for (int v = 0; v < NST; ++v) {
            const int64_t e0 = base + (int64_t)v * STEP + threadIdx.x * VEC;
            float x[VEC];
            finish16<DT>(raw[v], row, e0, P.V, x);
            take(v, e0, x);
        }
    } else {
#pragma unroll
        for (int v = 0; v < NST; ++v) {
            const int64_t e0 = base + (int64_t)v * STEP + threadIdx.x * VEC;
            float x[VEC];
            load_vec<DT>(row, e0, P.V, al, x);
            take(v, e0, x);
        }
    }
    if (w == 0) {
        const double u = cdf_uniform(P.noise, (uint32_t)r, 1u + (uint32_t)c);
        if (lane == 0) s_u = u;
    }
    // span max (NaN sticks: fmaxf drops it, so track it apart)
    float mv = -INFINITY;
    bool nan = false;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        mv = fmaxf(mv, y[k]);
        nan |= y[k] != y[k];
    }
    mv = wave_max(mv);
    if (lane == 0) lm[w] = mv;
    __syncthreads();
    m = lm[0];
#pragma unroll
    for (int k = 1; k < kThreads / kWave; ++k) m = fmaxf(m, lm[k]);
    u_c = s_u;
    SD_TS(wg_id, 1);
#pragma unroll
    for (int k = 0; k < EPT; ++k) wv[k] = m > -INFINITY ? __builtin_amdgcn_exp2f((y[k] - m) * kLog2e) : 0.f;
    pos = chunk_pick<EPT>(wv, u_c, nan ? 1.f : 0.f, T, PT);
    }
    SD_TS(wg_id, 2);
    // the candidate's processed value, from the thread that holds it
    __shared__ float s_ycand;
    if (pos >= 0 && threadIdx.x == pos / EPT) {
        const int k = pos - threadIdx.x * EPT;
        float yc = y[0];
#pragma unroll
        for (int kk = 1; kk < EPT; ++kk) yc = kk == k ? y[kk] : yc;
        s_ycand = yc;
    }
    __syncthreads();
    SD_TS(wg_id, 8);
    // partial (m_c, S_c | j_c, y_{j_c}) as one 16-byte write-through store into the span's slot
    float2* slot = reinterpret_cast<float2*>(reinterpret_cast<float4*>(P.rpart) + (int64_t)r * P.n_chunks + c);
    if (threadIdx.x == 0) {
        const float S = PT > 0.f ? NAN : (float)T;   // PT counts NaN lanes
        st_coh16(slot, make_uint4(__float_as_uint(PT > 0.f && !(m > -INFINITY) ? 0.f : m), __float_as_uint(S),
                                  (uint32_t)(pos < 0 ? -1 : (int32_t)chunk_elem<DT, DT, EPT>(base, pos)),
                                  __float_as_uint(pos < 0 ? -INFINITY : s_ycand)));
    }
    __shared__ int s_last;
    if (threadIdx.x == 0) s_last = arrive_last(seq_counter(P.cnt, 0, r), (uint32_t)P.n_chunks);
    __syncthreads();
    SD_TS(wg_id, 3);
    if (!s_last) return;

    // ---- tail: the row's last arrival
    __shared__ float l_w[kTailChunks], l_s[kTailChunks], l_y[kTailChunks];
    __shared__ int32_t l_cand[kTailChunks];
    __shared__ float2 s_ms;
    {   // every span's partial in one staged round trip
        const float2* pr = reinterpret_cast<const float2*>(reinterpret_cast<const float4*>(P.rpart) + (int64_t)r * P.n_chunks);
        for (int k = threadIdx.x; k < P.n_chunks; k += kThreads) {
            const uint4 v = ld_coh16(pr + 2 * k);
            const float2 ms = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
            const float2 jy = make_float2(__uint_as_float(v.z), __uint_as_float(v.w));
            l_w[k] = ms.x;   // m_c for now; weights below
            l_s[k] = ms.y;
            l_cand[k] = __float_as_int(jy.x);
            l_y[k] = jy.y;
        }
    }
    __syncthreads();
    SD_TS(wg_id, 4);
    if (w == 1) {   // the chunk-pick uniform, beside wave 0's combine
        const double u = cdf_uniform(P.noise, (uint32_t)r);
        if (lane == 0) s_u = u;
    }
    if (threadIdx.x < kWave) {
        float M = -INFINITY;
        for (int k = lane; k < P.n_chunks; k += kWave) M = fmaxf(M, l_w[k]);
        M = wave_max(M);
        float S = 0.f;
        for (int k = lane; k < P.n_chunks; k += kWave) {
            const float wc = l_w[k] > -INFINITY || l_s[k] != l_s[k] ? l_s[k] * sd_exp(l_w[k] - M) : 0.f;
            l_w[k] = wc;
            S += wc;
        }
        S = wave_sum(S);
        if (lane == 0) s_ms = make_float2(M, S);
    }
    __syncthreads();
    const float2 ms = s_ms;
    const int cp = pick_chunk(P, s_u, l_w);
    SD_TS(wg_id, 5);
    if (threadIdx.x == 0) {
        int32_t st = SD_ROW_DONE;
        if (!(ms.y > 0.f) || ms.y != ms.y || ms.y == INFINITY) st |= SD_ROW_INVALID_DIST;   // torch raises
        if (P.t_keep) st |= keep_of(P, r).flags;
        int64_t x = cp >= 0 ? (int64_t)l_cand[cp] : -1;
        if (x < 0) st |= SD_ROW_INVALID_DIST;
        if (st & SD_ROW_INVALID_DIST) x = -1;   // a failed row's token is -1, never a usable index
        P.next_token[r * P.next_token_stride] = x;
        if (P.token_prob) P.token_prob[r] = x >= 0 ? prob_exact<DT>(l_y[cp], ms.x, ms.y, 1.0f / ms.y) : NAN;
        if (P.row_stats) P.row_stats[r] = ms;
        if (P.row_status) P.row_status[r] = st;
        flag_error(P.status_or, st);
        if (P.keep_out && P.t_keep) P.keep_out[r] = keep_of(P, r);
        if (r == 0 && P.words_used) *P.words_used = 0;
    }
    SD_TS(wg_id, 6);
}
static_assert(sizeof(ResPart) >= sizeof(float4), "k_draw keeps a 16-byte partial per span in the ResPart region");
static_assert(2 * sizeof(ResPart) >= 8 * sizeof(float4), "k_draw_lean's line-padded rows fit the (nc + 1) ResParts per row");

// ------------------------------------------------------------------ k_draw_lean
// The bench's draw (and the drop-in loops' common case): T = 1, no processor, 16-bit rows,
// 16-byte aligned.  Same draw and outputs as k_draw, restructured for the latency chain that
// bounds a 8 MB launch (scripts/microbench/draw_shapes.hip: a bare span pass over the same rows
// takes 3.5 us):
//   * a compact kernel-argument block (one scalar-load batch, no hidden-argument division);
//   * spans of NST x 2048 elements, every vector in flight at once, no per-element tests except
//     in a row's ragged last span;
//   * the thread holding the span's candidate stores the partial itself (no candidate barrier)
//     and its wave alone continues: arrival, and — for the row's last arrival — the whole tail
//     in that one wave (64 lanes stage up to 64 partials per pass; wave reductions and a DPP
//     scan; no barrier).
struct DrawLean {
    const char* rows;
    int64_t stride_bytes;
    float4* part;
    uint32_t* cnt;
    int64_t* next_token;
    int64_t nt_stride;
    float* token_prob;
    float2* row_stats;
    int32_t* row_status;
    int64_t* words_used;
    sd_noise noise;
    int32_t V, n_span;
    int32_t pstride;   // float4 partials per row: n_span rounded up to whole 128-B lines
    int32_t poll;      // 1: the row's last span polls tagged partials (no arrival counter)
    int32_t spin_limit;   // bounded poll (sd_set_poll_policy)
    int32_t* status_or;   // the caller's sticky error word (nullable)
    uint64_t* ts;         // phase timestamps (SD_PHASE_TIMING builds only)
};

// phase timestamps of k_draw_lean (diagnostic builds): slot wg = r * n_span + c
#ifdef SD_PHASE_TIMING
#define SD_TSL(wg, ph)                                                                                 \
    do {                                                                                               \
        if (threadIdx.x == 0 && A.ts) A.ts[(size_t)(wg) * 16 + (ph)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define SD_TSL(wg, ph) \
    do {               \
        (void)(wg);    \
    } while (0)
#endif

// Poll-mode record tag: the row's epoch (counter set 2, advanced by the row's consumer after every
// draw) hashed with the row, the span and the span count.  Every row advances its epoch in step,
// and other shapes place other rows' records at these addresses, so the epoch alone would match
// a record another row left here; bytes from other kernels match only by a 2^-32 accident.
__device__ __forceinline__ uint32_t draw_tag(uint32_t epoch, int r, int c, int n_span) {
    uint32_t h = epoch * 0x9E3779B1u + (uint32_t)r * 0x85EBCA77u + (uint32_t)c * 0xC2B2AE3Du + (uint32_t)n_span * 0x27D4EB2Fu;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;   // murmur3 fmix32
    return h | 1u;   // never 0 (zero-filled workspace)
}

// GREEDY (argmax of the rounded probabilities, first index on ties — GreedyProcessor.sample on
// softmax(l) in the row's dtype, utils/logits_processor.py:26-36) in the same single pass: the
// rounded probability is monotone in the logit, so the winner lies in a span whose max m_c rounds
// to the row's top probability P* = p(M).  Each span publishes m_c, the first index of m_c, and
// whether any OTHER value lies strictly within kGreedyDelta below m_c (two probabilities that round
// to one bf16 value differ by < 2^-7 relative, e^-0.0079; fp16 subnormal tops of flat rows at
// V <= 256 Ki by < 1.6%; kGreedyDelta = 1/32 leaves a margin for both).  The
// tail takes the first index of every clean qualifying span; a qualifying span with such close
// values (rare) is rescanned by the tail wave with the exact rule, and so is the whole row when
// its normaliser is not finite (NaN / inf logits).
constexpr float kGreedyDelta = 1.0f / 32.0f;

// Variants measured slower and parked as patches (scripts/experiments/draw_lean_variants.patch):
// the claiming wave publishing the span's record itself (6.8 vs 6.5 us per bench draw), two
// staggered polls in flight (7.2 vs 6.65 us), an fp64 CDF span pick instead of the Gumbel race, and
// fmaxf wave maxima with a per-element -inf select (6.80 vs 6.50 us).

template <int DT, int NST>
__device__ int greedy_rescan(const DrawLean& A, const char* row, int c, float M, float S) {
    constexpr int VEC = 8, STEP = kThreads * VEC, SPAN = NST * STEP, PER = SPAN / kWave;
    const int lane = threadIdx.x & 63;
    const int64_t base = (int64_t)c * SPAN;
    const float inv = 1.0f / S;
    float bv = -INFINITY;
    int32_t bi = INT_MAX;
    for (int k0 = 0; k0 < PER; k0 += VEC) {
        const int64_t e0 = base + (int64_t)lane * PER + k0;   // lane-contiguous runs: index order per lane
        float x[VEC];
        load_vec<DT>(row, e0, A.V, true, x);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= A.V) continue;
            const float p = prob_exact<DT>(x[k], M, S, inv);
            if (arg_better(p, (int32_t)j, bv, bi)) { bv = p; bi = (int32_t)j; }
        }
    }
    wave_argmax(bv, bi);
    return bi;
}

// Element k of a lane's NST packed 16-byte vectors (16-bit rows): the loaded bits stay packed in
// registers and every pass over the span unpacks them again (one shift or mask for bf16), so a
// 4-stage span holds 16 VGPRs of row data instead of 32 floats plus 32 weights (90 -> <= 64 VGPRs:
// 8 workgroups per CU instead of 5, the large-batch draws' bytes in flight).
template <int DT>
__device__ __forceinline__ float lean_elem(const uint4* raw, int k) {
    const uint4 q = raw[k >> 3];
    const int i = (k & 7) >> 1;
    const uint32_t wd = i == 0 ? q.x : (i == 1 ? q.y : (i == 2 ? q.z : q.w));
    if constexpr (DT == SD_BF16) return __uint_as_float((k & 1) ? (wd & 0xffff0000u) : (wd << 16));
    else return __half2float(__ushort_as_half((unsigned short)((k & 1) ? (wd >> 16) : (wd & 0xffffu))));
}

// The ragged last span's vector at e0 in packed form: elements at or past the row end become -inf
// (bf16 0xff80, fp16 0xfc00), and a vector the clamped load could not fetch whole is rebuilt from
// guarded 16-bit loads — the same values finish16 + the -inf mask gave as floats.
template <int DT>
__device__ __forceinline__ uint4 lean_finish16(uint4 w, const char* row, int64_t e0, int vocab) {
    if (e0 + 8 <= vocab) return w;
    constexpr uint32_t kNegInf = DT == SD_BF16 ? 0xff80u : 0xfc00u;
    const uint16_t* h = reinterpret_cast<const uint16_t*>(row);
    uint32_t ws[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t e = e0 + 2 * k;
        const uint32_t lo = e < vocab ? (uint32_t)h[e] : kNegInf, hi = e + 1 < vocab ? (uint32_t)h[e + 1] : kNegInf;
        ws[k] = lo | (hi << 16);
    }
    return make_uint4(ws[0], ws[1], ws[2], ws[3]);
}

template <int DT, int NST, bool GREEDY = false>
__global__ void __launch_bounds__(kThreads) k_draw_lean(DrawLean A) {
    constexpr int VEC = 8, STEP = kThreads * VEC, EPT = NST * VEC, NW = kThreads / kWave;
    // (XCD-affine placement of a row's spans measured slower, 6.6 vs 6.4 us: plain grid order)
    const int c = blockIdx.x, r = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ts_wg = r * A.n_span + c;
    SD_TSL(ts_wg, 0);
    const char* row = A.rows + (int64_t)r * A.stride_bytes;
    const int64_t base = (int64_t)c * NST * STEP;
    uint4 raw[NST];
    if (base + (int64_t)NST * STEP <= A.V) {
#pragma unroll
        for (int v = 0; v < NST; ++v)
            raw[v] = *reinterpret_cast<const uint4*>(row + (base + (int64_t)v * STEP + threadIdx.x * VEC) * 2);
    } else {   // the row's ragged last span
        const int64_t last = last_whole_vec<DT>(A.V);
#pragma unroll
        for (int v = 0; v < NST; ++v) raw[v] = ld16_clamped<DT>(row, base + (int64_t)v * STEP + threadIdx.x * VEC, last);
#pragma unroll
        for (int v = 0; v < NST; ++v)
            raw[v] = lean_finish16<DT>(raw[v], row, base + (int64_t)v * STEP + threadIdx.x * VEC, A.V);
    }
    auto y = [&](int k) { return lean_elem<DT>(raw, k); };
    // an empty asm that "rewrites" the packed vectors: the passes after it cannot reuse values the
    // compiler derived from them before (it would keep every unpacked element and weight live)
    // (one or two stages fit 64 VGPRs as they are: those draws keep the compiler's schedule — the
    // re-derived values cost the 2-stage draw 1 us at B = 128)
    auto fence_raw = [&]() {
        if constexpr (NST >= 4)
#pragma unroll
        for (int v = 0; v < NST; ++v) asm volatile("" : "+v"(raw[v].x), "+v"(raw[v].y), "+v"(raw[v].z), "+v"(raw[v].w));
    };
    __shared__ float l_m[NW], l_s[NW];
    __shared__ double l_u;
    __shared__ int32_t l_j;
    __shared__ float l_y;
    __shared__ int32_t l_fi[NW], l_dirty[NW];
    uint32_t epoch = 0;   // poll mode: this launch's epoch of row r (read by wave 0, beside the loads)
    if (w == 0) {   // the span's in-chunk uniform: one wave's scalar unit, while the loads fly
        if (A.poll) epoch = __hip_atomic_load(seq_counter(A.cnt, 2, r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double u = GREEDY ? 0.0 : cdf_uniform(A.noise, (uint32_t)r, 1u + (uint32_t)c);
        if (lane == 0) { l_u = u; l_j = -1; l_y = -INFINITY; }
    }
    // per-wave max and weights: no barrier before the exps
    float mv = y(0);
#pragma unroll
    for (int k = 1; k < EPT; ++k) mv = fmaxf(mv, y(k));
    // integer-key wave max; a wave of -inf entries subtracts 0 (its weights are exp2(-inf) = 0),
    // so no per-element select, and a NaN entry always makes its own weight NaN (the span's S_c
    // NaN flags the row)
    fence_raw();
    const float mw = wave_max_ord(mv);
    const float mws = mw > -INFINITY ? mw : 0.f;
    SD_TSL(ts_wg, 1);
    // element k's weight, recomputed where it is needed again (the claiming lane's walk): the same
    // instruction on the same input, so the walk sees exactly the summed values
    auto wv = [&](int k) { return __builtin_amdgcn_exp2f((y(k) - mws) * kLog2e); };
    float tl = 0.f;
#pragma unroll
    for (int k = 0; k < EPT; ++k) tl += wv(k);
    fence_raw();
    const float incl = wave_incl_scan(tl);             // lane order, relative to mw
    const float prev = dpp_f<0x138, 0xF, true>(0.f, incl);   // wave_shr:1 -> the previous lane's incl
    if (lane == 63) { l_m[w] = mw; l_s[w] = incl; }
    __syncthreads();
    // every thread: span max, wave weights, offsets and total in one fixed order (uniform)
    float m = l_m[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) m = fmaxf(m, l_m[k]);
    float off = 0.f, my_off = 0.f, my_sc = 0.f, my_W = 0.f;
    int lastw = -1;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const float sc = l_m[k] > -INFINITY ? __builtin_amdgcn_exp2f((l_m[k] - m) * kLog2e) : 0.f;
        const float Wk = l_s[k] * sc;
        if (k == w) { my_off = off; my_sc = sc; my_W = Wk; }
        if (Wk > 0.f) lastw = k;
        off += Wk;
    }
    const float T = off;
    if constexpr (GREEDY) {
        // first index of the span max and whether another value lies within kGreedyDelta of it
        int32_t fi = INT_MAX;
        bool dirty = false;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int v = k / VEC;
            const int32_t j = (int32_t)(base + ((int64_t)v * kThreads + threadIdx.x) * VEC + (k - v * VEC));
            if (y(k) == m && fi == INT_MAX) fi = j;
            dirty |= y(k) > m - kGreedyDelta && y(k) != m;
        }
        fi = wave_min_i(fi);
        const bool dw = __ballot(dirty) != 0;
        if (lane == 0) { l_fi[w] = fi; l_dirty[w] = dw; }
    }
    const float t = (float)(l_u * (double)T);
    // the claiming wave (rounding past the end: the last wave with weight)
    const bool claim = !GREEDY && my_W > 0.f && ((t >= my_off && t < my_off + my_W) ||
                                                 (w == lastw && t >= my_off + my_W));
    int32_t cj = -1;   // the claiming lane's element and its logit
    float cy = -INFINITY;
    int hl = -1;
    if (claim) {
        const float a = fmaf(incl, my_sc, my_off), a0 = lane == 0 ? my_off : fmaf(prev, my_sc, my_off);
        const uint64_t hit = __ballot(a > t && tl > 0.f), posm = __ballot(tl > 0.f);
        hl = hit ? __builtin_ctzll(hit) : (posm ? 63 - __builtin_clzll(posm) : -1);
        if (lane == hl) {
            float run = a0;
            int kk = -1, lastk = -1;
#pragma unroll
            for (int k = 0; k < EPT; ++k) {
                const float wk = wv(k);
                run = fmaf(wk, my_sc, run);
                if (wk > 0.f) {
                    lastk = k;
                    if (kk < 0 && run > t) kk = k;
                }
            }
            if (kk < 0) kk = lastk;
            if (kk >= 0) {
                const int v = kk / VEC;
                float yk = y(0);
#pragma unroll
                for (int k = 1; k < EPT; ++k) yk = k == kk ? y(k) : yk;
                cj = (int32_t)(base + ((int64_t)v * kThreads + threadIdx.x) * VEC + (kk - v * VEC));
                cy = yk;
            }
        }
    }
    if (claim && lane == hl) { l_j = cj; l_y = cy; }
    __syncthreads();
    SD_TSL(ts_wg, 2);
    if (w != 0) return;
    const bool bad = T != T;   // NaN / +inf in the span: S_c NaN flags the row
    const float m_pub = bad && !(m > -INFINITY) ? 0.f : m, s_pub = bad ? NAN : T;
    int32_t j_pub = l_j;
    float y_pub = l_y;
    int32_t g_dirty = 0;   // GREEDY: another value within kGreedyDelta of the span max
    if constexpr (GREEDY) {
        j_pub = l_fi[0];
        for (int k = 1; k < NW; ++k) j_pub = l_fi[k] < j_pub ? l_fi[k] : j_pub;
        for (int k = 0; k < NW; ++k) g_dirty |= l_dirty[k];
        if (j_pub == INT_MAX) j_pub = -1;
        y_pub = m;
    }
    float4* part_row = A.part + (int64_t)r * A.pstride;
    int32_t xstat = 0;
    if (A.poll) {
        // Poll mode: every span but the row's last publishes one tagged 16-byte record
        // {m_c, S_c, (j_c - base + 1) | raw y << 16, tag} (write-through) and is done; the last
        // span's wave 0 polls the records until every tag is this launch's (bounded), then runs
        // the tail and advances the row's epoch.  No counter, no write-ack wait on the path.
        const uint32_t tag = draw_tag(epoch, r, c, A.n_span);
        if (c != A.n_span - 1) {
            if (lane == 0) {
                const uint32_t yraw = DT == SD_BF16 ? (__float_as_uint(y_pub) >> 16)
                                                    : (uint32_t)__half_as_ushort(__float2half_rn(y_pub));
                const uint32_t off = j_pub >= 0 ? (uint32_t)(j_pub - base) + 1u : 0u;   // <= NST * 2048
                const uint32_t gd = GREEDY && g_dirty ? 0x8000u : 0u;
                st_coh16(part_row + c, make_uint4(__float_as_uint(m_pub), __float_as_uint(s_pub), off | gd | (yraw << 16), tag));
            }
            SD_TSL(ts_wg, 3);
            return;
        }
    } else {
        // counter mode (many rows: more consumers than resident workgroups could spin): thread 0
        // publishes {m_c, S_c, j_c, y_{j_c}} and arrives; the last arrival runs the tail
        uint32_t last = 0;
        if (lane == 0) {
            st_coh16(part_row + c, make_uint4(__float_as_uint(m_pub), __float_as_uint(s_pub), (uint32_t)j_pub,
                                              GREEDY ? (uint32_t)g_dirty : __float_as_uint(y_pub)));
            last = arrive_last(seq_counter(A.cnt, 0, r), (uint32_t)A.n_span) ? 1u : 0u;
        }
        if (!__builtin_amdgcn_readlane(last, 0)) return;
    }

    // ---- tail (one wave): every span's partial, M, S, the span pick, the outputs
    // (SD_TAIL_PRIO: the row's one latency-critical wave wins VALU issue over the co-resident
    // producers' compute bursts — priority first, then age, MI355X_MICROARCH.md)
    if (SD_TAIL_PRIO) __builtin_amdgcn_s_setprio(3);
    const float2* pr = reinterpret_cast<const float2*>(A.part + (int64_t)r * A.pstride);
    float M = -INFINITY;
    float mk[2], sk[2], yk[2];
    int32_t jk[2];
    bool dk[2] = {false, false};   // GREEDY: the span's dirty flag
    const int npass = (A.n_span + kWave - 1) / kWave;   // <= 2 (host: n_span <= 128)
    // the span race's Gumbel noise, one span per lane and pass, before the wait (off the chain)
    float gk[2] = {0.f, 0.f};
    if constexpr (!GREEDY) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int k = q * kWave + lane;
            if (q < npass && k < A.n_span) gk[q] = span_gumbel(A.noise, (uint32_t)r, (uint32_t)k);
        }
    }
    if (A.poll) {
        // every other span's record, re-read until its tag is this launch's; this span's own from
        // registers (the lane that would hold it)
        bool have[2];
        uint4 rec[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int k = q * kWave + lane;
            have[q] = !(q < npass && k < A.n_span) || k == c;
            rec[q] = make_uint4(0u, 0u, 0u, 0u);
        }
        uint64_t sw_ = 0; for (int spin = 0;; ++spin) {
            if (A.spin_limit >= 0) {   // < 0: the test hook, every record counts as lost
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (!have[q]) {
                        rec[q] = ld_coh16(pr + 2 * (q * kWave + lane));
                        have[q] = rec[q].w == draw_tag(epoch, r, q * kWave + lane, A.n_span);
                    }
                }
                if (__all(have[0] && have[1])) break;
            }
            if (!spin_more(spin, A.spin_limit, sw_)) {   // bounded: ~tens of ms; the row is flagged, never a hang
                xstat = SD_ROW_EXCHANGE_TIMEOUT | SD_ROW_INVALID_DIST;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        SD_TSL(ts_wg, 4);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int k = q * kWave + lane;
            mk[q] = -INFINITY; sk[q] = 0.f; yk[q] = -INFINITY; jk[q] = -1;
            if (k == c) {
                mk[q] = m_pub; sk[q] = s_pub; jk[q] = j_pub; yk[q] = y_pub; dk[q] = g_dirty != 0;
            } else if (q < npass && k < A.n_span && have[q]) {
                mk[q] = __uint_as_float(rec[q].x); sk[q] = __uint_as_float(rec[q].y);
                dk[q] = GREEDY && (rec[q].z & 0x8000u) != 0;
                const uint32_t off = rec[q].z & (GREEDY ? 0x7fffu : 0xffffu), yraw = rec[q].z >> 16;
                jk[q] = off ? (int32_t)((int64_t)k * NST * STEP + off - 1) : -1;
                yk[q] = DT == SD_BF16 ? __uint_as_float(yraw << 16) : __half2float(__ushort_as_half((unsigned short)yraw));
            }
            M = fmaxf(M, mk[q]);
        }
    } else {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int k = q * kWave + lane;
        mk[q] = -INFINITY; sk[q] = 0.f; yk[q] = -INFINITY; jk[q] = -1;
        if (q < npass && k < A.n_span) {
            const uint4 v = ld_coh16(pr + 2 * k);
            mk[q] = __uint_as_float(v.x); sk[q] = __uint_as_float(v.y);
            jk[q] = (int32_t)v.z; yk[q] = GREEDY ? mk[q] : __uint_as_float(v.w);
            dk[q] = GREEDY && v.w != 0u;
        }
        M = fmaxf(M, mk[q]);
    }
    }
    M = wave_max_ord(M);   // the tail's maxima: finite or -inf records, never NaN
    float wk[2], S = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        wk[q] = mk[q] > -INFINITY || sk[q] != sk[q] ? sk[q] * sd_exp(mk[q] - M) : 0.f;
        S += wk[q];
    }
    S = wave_sum(S);
    if constexpr (GREEDY) {
        const bool ok = S > 0.f && S != INFINITY && M == M;
        const float inv = 1.0f / S;
        const float pst = ok ? prob_exact<DT>(M, M, S, inv) : 0.f;
        int32_t cand = INT_MAX;
        bool resc[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int k = q * kWave + lane;
            const bool in = q < npass && k < A.n_span;
            const bool qual = in && (!ok || (mk[q] > -INFINITY && prob_exact<DT>(mk[q], M, S, inv) == pst));
            resc[q] = qual && (!ok || dk[q] || jk[q] < 0);
            if (qual && !resc[q]) cand = jk[q] < cand ? jk[q] : cand;
        }
        cand = wave_min_i(cand);
        // rescans (rare): the exact rule over each flagged span; an invalid row is scanned whole
        float bv = -INFINITY;
        int32_t bi = INT_MAX;
        if (cand != INT_MAX) { bv = ok ? pst : -INFINITY; bi = cand; }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            uint64_t mask = __ballot(resc[q]);
            while (mask) {
                const int k = q * kWave + __builtin_ctzll(mask);
                mask &= mask - 1;
                const int32_t j = greedy_rescan<DT, NST>(A, row, k, M, S);
                if (j != INT_MAX) {
                    const float pv = prob_exact<DT>(load_one<DT>(row, j), M, S, inv);
                    if (arg_better(pv, j, bv, bi)) { bv = pv; bi = j; }
                }
            }
        }
        const int32_t x = bi == INT_MAX ? -1 : bi;
        if (lane == 0) {
            int32_t st = SD_ROW_DONE | xstat;
            if (!ok) st |= SD_ROW_INVALID_DIST;
            if (x < 0) st |= SD_ROW_INVALID_DIST;
            if (A.poll) __hip_atomic_store(seq_counter(A.cnt, 2, r), epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            A.next_token[r * A.nt_stride] = x;
            if (A.token_prob) A.token_prob[r] = x >= 0 ? bv : NAN;
            if (A.row_stats) A.row_stats[r] = make_float2(M, S);
            if (A.row_status) A.row_status[r] = st;
            flag_error(A.status_or, st);
            if (r == 0 && A.words_used) *A.words_used = 0;
        }
        return;
    }
    // span pick by a Gumbel race: argmax_c (m_c + ln S_c + g_c) picks span c with probability
    // S_c e^(m_c) / Σ — independent of M and S, so its wave max runs beside theirs (no fp64 scan)
    float key[2];
    float kmax = -INFINITY;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        key[q] = mk[q] > -INFINITY && sk[q] > 0.f ? mk[q] + __logf(sk[q]) + gk[q] : -INFINITY;
        kmax = fmaxf(kmax, key[q]);
    }
    kmax = wave_max_ord(kmax);
    int pick = -1;
    if (kmax > -INFINITY) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint64_t hit = __ballot(key[q] == kmax);
            if (pick < 0 && hit) pick = q * kWave + __builtin_ctzll(hit);
        }
    }
    int32_t x = -1;
    float yx = -INFINITY;
    if (pick >= 0) {
        const int q = pick / kWave, src = pick & 63;
        x = __builtin_amdgcn_readlane(q == 0 ? jk[0] : jk[1], src);
        yx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q == 0 ? yk[0] : yk[1]), src));
    }
    if (lane == 0) {
        int32_t st = SD_ROW_DONE | xstat;
        if (!(S > 0.f) || S != S || S == INFINITY) st |= SD_ROW_INVALID_DIST;   // torch raises
        if (x < 0) st |= SD_ROW_INVALID_DIST;
        if (st & SD_ROW_INVALID_DIST) x = -1;   // a failed row's token is -1, never a usable index
        if (A.poll) __hip_atomic_store(seq_counter(A.cnt, 2, r), epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        A.next_token[r * A.nt_stride] = x;
        if (A.token_prob) A.token_prob[r] = x >= 0 ? prob_exact<DT>(yx, M, S, 1.0f / S) : NAN;
        if (A.row_stats) A.row_stats[r] = make_float2(M, S);
        if (A.row_status) A.row_status[r] = st;
        flag_error(A.status_or, st);
        if (r == 0 && A.words_used) *A.words_used = 0;
    }
    SD_TSL(ts_wg, 5);
}

// ------------------------------------------------------------------ sd_probs kernel
template <int DT, int EPT>
__device__ void writeprobs_body(const Plan& P, void* out, int64_t ostride, int r, int c) {
    __shared__ float2 lms;
    constexpr int VEC = Elem<DT>::kVec, NV = EPT / VEC;
    if (threadIdx.x < 64) {
        const float2 ms = combine_row(P, r);
        if (threadIdx.x == 0) lms = ms;
    }
    __syncthreads();
    const float2 ms = lms;
    const void* row = static_cast<const char*>(P.trow[0]) + r * P.tstride * (DT == SD_F32 ? 4 : 2);
    const bool al = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
    const RowKeep kp = P.t_keep ? keep_of(P, r) : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const int64_t base = (int64_t)c * P.rchunk;
    char* orow = static_cast<char*>(out) + r * ostride * (DT == SD_F32 ? 4 : 2);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float x[VEC];
        load_vec<DT>(row, e0, P.V, al, x);
        process_vec<DT, VEC>(x, e0, P.tT, P.t_keep, kp);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= P.V) continue;
            const float p = round_dt<DT>(sd_exp(x[k] - ms.x) / ms.y);
            if constexpr (DT == SD_F32) reinterpret_cast<float*>(orow)[j] = p;
            else if constexpr (DT == SD_BF16) reinterpret_cast<uint16_t*>(orow)[j] = (uint16_t)(__float_as_uint(p) >> 16);
            else reinterpret_cast<__half*>(orow)[j] = __float2half_rn(p);
        }
    }
}

template <int DT, int EPT>
__global__ void __launch_bounds__(kThreads) k_writeprobs(Plan P, void* out, int64_t ostride) {
    writeprobs_body<DT, EPT>(P, out, ostride, blockIdx.y, blockIdx.x);
}

}  // namespace sd

// ====================================================================== host side
namespace {
thread_local hipError_t g_last_error = hipSuccess;

// In-launch exchange policy (sd_set_poll_policy): whether poll-mode exchanges may be chosen at all,
// and the bound of every poll.  Process-wide; SD_POLL / SD_POLL_SPIN_LIMIT set the initial values.
constexpr int kDefaultSpin = 2000000;   // us of wall clock per wait (2 s): outlasts a co-running kernel
std::atomic<int> g_allow_poll{-1};
std::atomic<int> g_spin_limit{kDefaultSpin};
std::once_flag g_policy_once;
// The only environment reads of the library: the poll policy's initial values, once per process
// (the DP runner's shared-device rehearsal sets SD_POLL=0 before the first call).
void policy_init() {
    std::call_once(g_policy_once, [] {
        int allow = 1;
        if (const char* e = getenv("SD_POLL")) allow = atoi(e) != 0;
        int expected = -1;
        g_allow_poll.compare_exchange_strong(expected, allow);
        if (const char* e = getenv("SD_POLL_SPIN_LIMIT")) {
            const int v = atoi(e);
            g_spin_limit.store(v == 0 ? kDefaultSpin : v);
        }
    });
}

// Dispatch options (sd_set_option), indexed by sd_option; relaxed reads on every call.
std::atomic<int> g_opt_fused{1}, g_opt_lean{-1}, g_opt_thr_poll{1}, g_opt_draw_stream{1}, g_opt_ticket{-1};
std::atomic<int> g_opt_draw_span{0}, g_opt_ticket_lag{0}, g_opt_samp_chunks{0};
// k_draw_lean: batches above kDrawSpan4MinB take 4 stages per workgroup (measured round 6, packed
// registers: B = 128 one stage 12.9 us, two 13.7, four 13.3; B = 512 four 33.5, one 38.7)
constexpr int kDrawSpan4MinB = 128;
std::atomic<int>* option_slot(int32_t opt) {
    switch (opt) {
        case SD_OPT_DRAW_SPAN: return &g_opt_draw_span;
        case SD_OPT_TICKET_LAG: return &g_opt_ticket_lag;
        case SD_OPT_SAMP_CHUNKS: return &g_opt_samp_chunks;
        case SD_OPT_FUSED_VERIFY: return &g_opt_fused;
        case SD_OPT_FUSED_TICKET: return &g_opt_ticket;
        case SD_OPT_LEAN_VERIFY: return &g_opt_lean;
        case SD_OPT_THRESHOLD_POLL: return &g_opt_thr_poll;
        case SD_OPT_DRAW_STREAM: return &g_opt_draw_stream;
        default: return nullptr;
    }
}
inline int opt(const std::atomic<int>& o) { return o.load(std::memory_order_relaxed); }

// the path of this thread's last sd_verify / sd_sample (sd_last_*_path)
thread_local int32_t g_verify_path = SD_PATH_NONE;
thread_local int32_t g_sample_path = SD_PATH_NONE;
bool poll_allowed() {
    policy_init();
    return g_allow_poll.load(std::memory_order_relaxed) > 0;
}
int spin_limit() {
    policy_init();
    return g_spin_limit.load(std::memory_order_relaxed);
}
int resident_cap(const void* kern, int threads = sd::kThreads, size_t dyn = 0);
}  // namespace

#include "sd_threshold.inc"
#include "sd_draw_nucleus.inc"
#include "sd_draw_stream.inc"
#include "sd_verify_lean.inc"

namespace {

using namespace sd;

constexpr int kEptSmall = 8;

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Carve {
    char* p;
    size_t used = 0;
    template <typename T>
    T* take(size_t n) {
        T* r = reinterpret_cast<T*>(p ? p + used : nullptr);
        used += align256(n * sizeof(T));
        return r;
    }
};

int max_chunks(int vocab) { return (vocab + kThreads * kEptSmall - 1) / (kThreads * kEptSmall); }

void carve(Plan& P, Carve& c, int rows_total, int B, int gamma, int vocab) {
    const int nc = max_chunks(vocab);
    // first, at a fixed offset (see kCntMax): sets 0 / 1 arrivals, 2 k_draw_lean row epochs,
    // 3 k_sample poll-mode sequence epochs
    P.cnt = c.take<uint32_t>(4 * (size_t)kCntMax * kCntStride);
    P.part = c.take<float2>((size_t)rows_total * nc);
    P.rowstat = c.take<float2>(rows_total);
    P.keep = c.take<RowKeep>(rows_total);
    P.rp = c.take<float>((size_t)B * gamma);
    P.rq = c.take<float>((size_t)B * gamma);
    P.dec = c.take<Decision>(B);
    // + 1 per row: room for 16-byte records padded to whole 128-B lines per row (k_draw_lean)
    P.rpart = c.take<ResPart>((size_t)(B > rows_total ? B : rows_total) * (nc + 1));
    P.srec = reinterpret_cast<uint4*>(P.rpart);
    P.sprec = reinterpret_cast<uint4*>(P.rpart);
    P.drec = nullptr;
    P.crec = nullptr;
    P.n_samp = 0;
    P.samp_cps = 2;
    P.keep_hist = c.take<int32_t>((size_t)rows_total * kThreshScratchInts);
    P.thr_part = c.take<uint32_t>((size_t)rows_total * kThrMaxSlices);
    P.thr_tail = c.take<float>((size_t)rows_total * kThrMaxSlices);
    P.thr_hist = c.take<int32_t>((size_t)rows_total * kThrWin);
    P.thr_shist = c.take<int32_t>((size_t)kThrShistSlots * kThrWin);
    P.thr = c.take<ThrRow>(rows_total);
}

bool valid_dtype(int dt) { return dt == SD_F32 || dt == SD_BF16 || dt == SD_F16; }
bool valid_proc(const sd_processor& p) {
    if (p.kind < SD_PROC_GREEDY || p.kind > SD_PROC_TOPK_NUCLEUS) return false;
    if ((p.kind == SD_PROC_TOPK || p.kind == SD_PROC_TOPK_NUCLEUS) && p.top_k <= 0) return false;
    return true;
}
bool needs_keep(const sd_processor& p) { return p.kind >= SD_PROC_TOPK; }

// Span of a k_stats workgroup: a multiple of one 2048-element stage, sized for about 512
// workgroups (2 per CU), all resident at once.  Measured at the bench shape (128 rows of 128256
// bf16): 512 workgroups 13.6 us, 1024 14.4, 2048 16.3, 384 14.7, 256 15.9 — longer spans mean
// fewer arrivals and partials per sequence for the decision tail, until the stream itself thins
// out.  Contiguous spans (interleaved stages measured 39.2 vs 38.4 us per step, removed).
// Other callers (sd_sample's greedy / STREAM statistics, A11) keep target_wgs = 2048.
void set_stats_chunks(sd::Plan& P, int rows, int target_wgs = 2048, int min_stages = 1) {
    const int64_t stage = kThreads * 8;
    const int64_t stages_per_row = (P.V + stage - 1) / stage;
    int64_t per_wg = (rows * stages_per_row + target_wgs - 1) / target_wgs;
    per_wg = per_wg < min_stages ? min_stages : per_wg;
    per_wg = per_wg < 1 ? 1 : (per_wg > 64 ? 64 : per_wg);
    P.chunk = (int32_t)(per_wg * stage);
    P.n_chunks = (P.V + P.chunk - 1) / P.chunk;
}

// Resample / sample passes: 1 or 2 stages of 2048 elements per workgroup, about 1024 workgroups so
// the whole grid is resident at once (these kernels carry more SGPRs, so fewer blocks fit per CU).
void set_rchunks(sd::Plan& P) {
    const int64_t stage = kThreads * kEptSmall;
    int64_t per_wg = ((int64_t)P.B * ((P.V + stage - 1) / stage) + 1023) / 1024;
    per_wg = 1;   // measured: 2 stages (116 VGPRs, 4 waves/SIMD) ran 1.8x slower than 1 stage at 8
    P.rchunk = (int32_t)(per_wg * stage);
    P.rn_chunks = (P.V + P.rchunk - 1) / P.rchunk;
}

int32_t launch_stats(const sd::Plan& P, void* stream, bool tail = false);

#define SD_LAUNCH(kern, grid, block, stream, ...)                                             \
    do {                                                                                      \
        hipLaunchKernelGGL(kern, grid, block, 0, (hipStream_t)stream, __VA_ARGS__);            \
        const hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess) { g_last_error = e_; return SD_ERR_LAUNCH; }                    \
    } while (0)

// errors left behind by earlier, unrelated runtime calls must not be blamed on our launches
inline void clear_stale_error() { (void)hipGetLastError(); }

bool sample_poll_ok(int B, const void* kern);

template <int DT, bool TAIL>
int32_t launch_stats_dt(const sd::Plan& P, bool fast, int slot_lo, int slot_cnt, void* stream) {
    const dim3 grid(P.n_chunks, P.B * slot_cnt);
    // poll-mode decide tail: the drafter stats came with the draws (target slots only, one launch)
    sd::Plan Q = P;
    Q.kpoll = TAIL && P.dstats && P.n_chunks <= kWave && P.stat_slots == P.n_tslots &&
              P.n_tslots <= sd::kFastSlots && slot_lo == 0 &&
              slot_cnt == P.stat_slots &&
              sample_poll_ok(P.B, fast ? (const void*)k_stats<DT, true, TAIL> : (const void*)k_stats<DT, false, TAIL>);
    // poll mode: a 1-D grid with one decider workgroup per sequence after its spans (k_stats)
    const dim3 g2 = Q.kpoll ? dim3(P.B * (slot_cnt * P.n_chunks + 1)) : grid;
    if (fast) SD_LAUNCH((k_stats<DT, true, TAIL>), g2, dim3(kThreads), stream, Q, slot_lo, slot_cnt);
    else SD_LAUNCH((k_stats<DT, false, TAIL>), g2, dim3(kThreads), stream, Q, slot_lo, slot_cnt);
    return SD_OK;
}

// resident capacity of a kernel's workgroups (256 threads unless given) on this device (occupancy x
// CUs), cached per (device, kernel, block, dynamic LDS) under a mutex: any host thread may call
int resident_cap(const void* kern, int threads, size_t dyn) {
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, int, size_t>, int> caps;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lk(mu);
    auto it = caps.find({dev, kern, threads, dyn});
    if (it == caps.end()) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, dyn) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            per_cu = cus = 0;
        it = caps.emplace(std::make_tuple(dev, kern, threads, dyn), per_cu * cus).first;
    }
    return it->second;
}

// The whole perf-mode verify of stochastic target rows in ONE launch (k_stats<.., TAIL, SAMP>): the
// spans, a decider and P.n_samp samplers per sequence, every workgroup resident (the decider and the
// samplers poll).  1 launched, 0 not applicable (the caller runs k_stats + k_sample), < 0 an error.
template <int DT>
int32_t launch_fused_dt(const sd::Plan& P, bool fast, void* stream) {
    const int64_t head = (int64_t)P.B * (P.n_tslots * P.n_chunks + 1);
    // ticket mode: every label gets ceil(B / labels) sequences' workgroups (stats_body)
    const int64_t seqs = P.ticket ? (int64_t)P.labels * ((P.B + P.labels - 1) / P.labels) : P.B;
    const int64_t total = P.ticket ? seqs * (P.n_tslots * P.n_chunks + 1 + P.n_samp) : head + (int64_t)P.B * P.n_samp;
    if (!poll_allowed()) return 0;
    sd::Plan Q = P;
    Q.kpoll = 1;
    if (P.ticket) {
        if (fast) SD_LAUNCH((k_verify_fused<DT, true, true>), dim3((uint32_t)total), dim3(kThreads), stream, Q, 0, P.n_tslots);
        else SD_LAUNCH((k_verify_fused<DT, false, true>), dim3((uint32_t)total), dim3(kThreads), stream, Q, 0, P.n_tslots);
    } else {
        if (fast) SD_LAUNCH((k_verify_fused<DT, true, false>), dim3((uint32_t)total), dim3(kThreads), stream, Q, 0, P.n_tslots);
        else SD_LAUNCH((k_verify_fused<DT, false, false>), dim3((uint32_t)total), dim3(kThreads), stream, Q, 0, P.n_tslots);
    }
    return 1;
}

// the block-id layout's kernel (its residency decides between the layouts, fused_layout)
const void* fused_kernel(const sd::Plan& P) {
    const bool fast = P.tT == 1.0f && P.dT == 1.0f && !P.t_keep && !P.d_keep;
    if (P.tdt == SD_BF16) return fast ? (const void*)k_verify_fused<SD_BF16, true, false> : (const void*)k_verify_fused<SD_BF16, false, false>;
    if (P.tdt == SD_F16) return fast ? (const void*)k_verify_fused<SD_F16, true, false> : (const void*)k_verify_fused<SD_F16, false, false>;
    return fast ? (const void*)k_verify_fused<SD_F32, true, false> : (const void*)k_verify_fused<SD_F32, false, false>;
}

int32_t launch_fused(const sd::Plan& P, void* stream) {
    const bool fast = P.tT == 1.0f && P.dT == 1.0f && !P.t_keep && !P.d_keep;
    if (P.tdt == SD_BF16) return launch_fused_dt<SD_BF16>(P, fast, stream);
    if (P.tdt == SD_F16) return launch_fused_dt<SD_F16>(P, fast, stream);
    return launch_fused_dt<SD_F32>(P, fast, stream);
}

// The fused verify's work layout for F (n_samp set): block-id order when the spans and deciders are
// resident at once with headroom (the deciders poll the spans; the samplers, after them in dispatch
// order, wait only for decisions and take freed slots) and the batch is small; otherwise ticket
// order (stats_body, fused_role) — at any batch, resident or not.  (From kTicketMinB sequences every
// perf-mode verify streams spans of kTicketSpan elements, sd_verify: the fused and the two-launch
// kernels then take the same row statistics, so their outputs stay identical.)
// SD_OPT_FUSED_TICKET: -1 auto, 0 never (a non-resident grid then takes the two launches), 1 always.
// false: no fused launch for this batch.
constexpr int kTicketMinB = 64;
constexpr int kTicketLabels = 64;   // labels (ticket counters) from B = 64; 8 below
constexpr int kTicketLag = 1;       // default lag (SD_OPT_TICKET_LAG pins it): B = 512 verify 173 us at 1, 179 at 2, 185 at 3
constexpr int kTicketSampChunks = 4;   // chunks per sampler in ticket order (SD_OPT_SAMP_CHUNKS pins it): 4 measured best at B = 128 / 512
constexpr int kTicketSpan = 16 * kThreads * 8;   // 32768 elements: 4 spans per Llama-3 row
bool fused_layout(sd::Plan& F) {
    const int cap = resident_cap(fused_kernel(F));
    const int64_t head = (int64_t)F.B * (F.n_tslots * F.n_chunks + 1);
    const bool resident = cap > 0 && 2 * head <= cap;
    const int tmode = opt(g_opt_ticket);
    F.ticket = tmode == 1 || (tmode < 0 && (F.B >= kTicketMinB || !resident));
    if (!F.ticket) return resident;
    if (cap <= 0) return false;
    F.labels = F.B >= kTicketLabels ? kTicketLabels : 8;
    // chunks per sampler: a large batch's samplers hold slots the spans could stream in, and each
    // one pays a decision poll and a dispatch — fewer, longer samplers (SD_OPT_SAMP_CHUNKS pins it)
    const int sc = opt(g_opt_samp_chunks);
    F.samp_cps = sc > 0 ? sc : kTicketSampChunks;
    F.n_samp = (F.rn_chunks + F.samp_cps - 1) / F.samp_cps;
    const int lg = opt(g_opt_ticket_lag);
    F.lag = lg > 0 ? lg : kTicketLag;
    // set 1's last `labels` counters (k_sample's arrivals of sequences B >= kCntMax - labels, which a
    // call of that size only uses in counter mode, where they are zero between launches too)
    F.ticket_ctr = F.cnt + ((size_t)1 * kCntMax + (kCntMax - F.labels)) * kCntStride;
    F.xcd_affine = 0;
    return true;
}

int32_t launch_stats_group(const sd::Plan& P, int dt, bool fast, int slot_lo, int slot_cnt, bool tail, void* stream) {
    if (slot_cnt <= 0) return SD_OK;
    if (tail) {
        if (dt == SD_BF16) return launch_stats_dt<SD_BF16, true>(P, fast, slot_lo, slot_cnt, stream);
        if (dt == SD_F32) return launch_stats_dt<SD_F32, true>(P, fast, slot_lo, slot_cnt, stream);
        return launch_stats_dt<SD_F16, true>(P, fast, slot_lo, slot_cnt, stream);
    }
    if (dt == SD_BF16) return launch_stats_dt<SD_BF16, false>(P, fast, slot_lo, slot_cnt, stream);
    if (dt == SD_F32) return launch_stats_dt<SD_F32, false>(P, fast, slot_lo, slot_cnt, stream);
    return launch_stats_dt<SD_F16, false>(P, fast, slot_lo, slot_cnt, stream);
}

// A poll-mode exchange (k_sample's finish, k_stats' decide tail) needs its B consumers plus producers
// resident: 2B <= the kernel's resident capacity (occupancy x CUs, per device and kernel, queried
// once); sd_set_poll_policy(0, ·) keeps the arrival counters
bool sample_poll_ok(int B, const void* kern) {
    if (!poll_allowed()) return false;
    return 2 * B <= resident_cap(kern);
}

template <int TDT, int DDT>
int32_t launch_resample_dd(const sd::Plan& P, void* stream) {
    const dim3 grid(P.rn_chunks, P.B);
    // FAST: T == 1 and no top-k / nucleus mask on either side (the engine rule, plain softmax)
    const bool fast = P.tT == 1.0f && P.dT == 1.0f && !P.t_keep && !P.d_keep;
    if (P.noise.mode == SD_NOISE_STREAM) {
        if (fast) SD_LAUNCH((k_resample<TDT, DDT, 8, true>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_resample<TDT, DDT, 8, false>), grid, dim3(kThreads), stream, P);
    } else if (P.t_stoch) {
        // poll-mode finish when the consumers (one per sequence) leave room for every producer
        sd::Plan Q = P;
        Q.spoll = sample_poll_ok(P.B, fast ? (const void*)k_sample<TDT, DDT, true, true>
                                           : (const void*)k_sample<TDT, DDT, false, true>);
        if (fast) SD_LAUNCH((k_sample<TDT, DDT, true, true>), grid, dim3(kThreads), stream, Q);
        else SD_LAUNCH((k_sample<TDT, DDT, false, true>), grid, dim3(kThreads), stream, Q);
    } else {
        if (fast) SD_LAUNCH((k_sample<TDT, DDT, true, false>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_sample<TDT, DDT, false, false>), grid, dim3(kThreads), stream, P);
    }
    return SD_OK;
}

template <int TDT>
int32_t launch_resample_t(const sd::Plan& P, int ddt, void* stream) {
    if (ddt == SD_BF16) return launch_resample_dd<TDT, SD_BF16>(P, stream);
    if (ddt == SD_F32) return launch_resample_dd<TDT, SD_F32>(P, stream);
    return launch_resample_dd<TDT, SD_F16>(P, stream);
}

int32_t launch_resample(const sd::Plan& P, void* stream) {
    const int ddt = P.draft_is_probs ? SD_F32 : P.ddt;
    if (P.tdt == SD_BF16) return launch_resample_t<SD_BF16>(P, ddt, stream);
    if (P.tdt == SD_F32) return launch_resample_t<SD_F32>(P, ddt, stream);
    return launch_resample_t<SD_F16>(P, ddt, stream);
}

template <int DT>
int32_t launch_rowsample_dt(const sd::Plan& P, void* stream) {
    const dim3 grid(P.rn_chunks, P.B);
    // FAST: T = 1 and no top-k / nucleus mask (the engine's plain softmax draws)
    const bool fast = P.tT == 1.0f && !P.t_keep;
    if (P.noise.mode == SD_NOISE_STREAM) {
        if (fast) SD_LAUNCH((k_rowsample<DT, SD_NOISE_STREAM, 8, true>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_rowsample<DT, SD_NOISE_STREAM, 8>), grid, dim3(kThreads), stream, P);
    } else {
        SD_LAUNCH((k_rowsample<DT, SD_NOISE_PHILOX, 8>), grid, dim3(kThreads), stream, P);
    }
    return SD_OK;
}

int32_t launch_rowsample(const sd::Plan& P, void* stream) {
    if (P.tdt == SD_BF16) return launch_rowsample_dt<SD_BF16>(P, stream);
    if (P.tdt == SD_F32) return launch_rowsample_dt<SD_F32>(P, stream);
    return launch_rowsample_dt<SD_F16>(P, stream);
}

// Row statistics for every slot: one launch when target and drafter rows share a dtype.
// tail: perf-mode decision in the last workgroup per sequence (both launches count arrivals; the
// second launch starts after the first has finished, so the last arrival is always in it).
int32_t launch_stats(const sd::Plan& P, void* stream, bool tail) {
    const bool t_fast = P.tT == 1.0f && !P.t_keep, d_fast = P.dT == 1.0f && !P.d_keep;
    const int d_cnt = P.stat_slots - P.n_tslots;   // drafter slots without stashed stats
    if (d_cnt == 0 || (P.tdt == P.ddt && t_fast == d_fast))
        return launch_stats_group(P, P.tdt, t_fast, 0, P.stat_slots, tail, stream);
    if (int32_t st = launch_stats_group(P, P.tdt, t_fast, 0, P.n_tslots, tail, stream)) return st;
    return launch_stats_group(P, P.ddt, d_fast, P.n_tslots, d_cnt, tail, stream);
}

// perf-mode sd_sample of stochastic rows: k_draw (one launch, one pass)
template <int DT>
int32_t launch_draw_dt(const sd::Plan& P, int nst, void* stream) {
    const dim3 grid(P.n_chunks, P.B);
    const bool fast = P.tT == 1.0f && !P.t_keep;
    if (nst == 1) {
        if (fast) SD_LAUNCH((k_draw<DT, true, 1>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_draw<DT, false, 1>), grid, dim3(kThreads), stream, P);
    } else if (nst == 4) {
        if (fast) SD_LAUNCH((k_draw<DT, true, 4>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_draw<DT, false, 4>), grid, dim3(kThreads), stream, P);
    } else {
        if (fast) SD_LAUNCH((k_draw<DT, true, 2>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_draw<DT, false, 2>), grid, dim3(kThreads), stream, P);
    }
    return SD_OK;
}

// k_draw_lean's cases: T = 1, no processor, 16-bit rows, every row 16-byte aligned, <= 128 spans
template <int DT, int NST, bool GREEDY = false>
int32_t launch_draw_lean_t(const sd::Plan& P, void* stream) {
    DrawLean A{};
    A.rows = static_cast<const char*>(P.trow[0]);
    A.stride_bytes = P.tstride * 2;
    A.part = reinterpret_cast<float4*>(P.rpart);
    A.cnt = P.cnt;
    A.next_token = P.next_token; A.nt_stride = P.next_token_stride;
    A.token_prob = P.token_prob; A.row_stats = P.row_stats; A.row_status = P.row_status; A.words_used = P.words_used;
    A.noise = P.noise;
    A.V = P.V;
    A.n_span = (int32_t)((P.V + NST * kThreads * 8 - 1) / (NST * kThreads * 8));
    A.pstride = (A.n_span + 7) & ~7;
    // poll mode needs every row's consumer resident while it waits: at most half the workgroups
    // the device holds at once (occupancy x CUs, queried once per device) are consumers
    const int cap = resident_cap((const void*)k_draw_lean<DT, NST, GREEDY>);
    A.poll = cap > 0 && 2 * P.B <= cap && poll_allowed();
    A.spin_limit = P.spin_limit;
    A.status_or = P.status_or;
    A.ts = P.ts;
    SD_LAUNCH((k_draw_lean<DT, NST, GREEDY>), dim3(A.n_span, P.B), dim3(kThreads), stream, A);
    return SD_OK;
}

// The one-launch verify of a few sequences (sd_verify_lean.inc): 1 launched, 0 not applicable (the
// caller runs k_stats + k_sample), < 0 a launch error.  Perf mode with the drafter stats from the
// draws, no top-k / nucleus, 16-bit rows of one dtype, V <= 64 spans, every row 16-byte aligned, and
// the whole grid resident (every workgroup polls).  Up to kLeanVerifyMaxB sequences by default;
// SD_OPT_LEAN_VERIFY = 0 turns it off, = 1 allows any batch the occupancy check admits (A/B, tests).
constexpr int kLeanVerifyMaxB = 8;

// why the lean verify was not taken (1..11), kept for diagnostics (a debugger / a printf build)
thread_local int g_lean_why = 0;
static void lean_why(int k) { g_lean_why = k; }

int32_t launch_verify_lean(const sd::Plan& P0, void* stream) {
    if (P0.noise.mode == SD_NOISE_STREAM) { lean_why(1); return 0; }
    // statistics: the target rows with the draws' drafter stats, or every row here; keep
    // predicates from this call's threshold search (P.keep) or the draws' (P.dkeep)
    if (P0.draft_is_probs || P0.stat_slots != (P0.dstats ? P0.n_tslots : P0.slots)) { lean_why(2); return 0; }
    if (P0.tdt != P0.ddt || (P0.tdt != SD_BF16 && P0.tdt != SD_F16)) { lean_why(3); return 0; }
    if (P0.n_tslots > sd::kLeanMaxT || P0.gamma > SD_LEAN_MAX_GAMMA || P0.B > kCntMax || !poll_allowed()) { lean_why(4); return 0; }
    const int mode = opt(g_opt_lean);
    if (mode == 0 || (mode < 0 && P0.B > kLeanVerifyMaxB)) { lean_why(5); return 0; }
    constexpr int kSpan = kThreads * 8;
    const int n_span = (P0.V + kSpan - 1) / kSpan;
    if (n_span > kWave || P0.rn_chunks != n_span || P0.rchunk != kSpan) { lean_why(6); return 0; }
    if ((P0.tstride * 2) % 16 || (P0.dstride * 2) % 16) { lean_why(7); return 0; }
    for (int t = 0; t < P0.n_tslots; ++t)
        if (reinterpret_cast<uintptr_t>(P0.trow[t]) & 15) { lean_why(8); return 0; }
    for (int t = 0; t < P0.gamma; ++t)
        if (reinterpret_cast<uintptr_t>(P0.drow[t]) & 15) { lean_why(9); return 0; }
    const bool fast = P0.tT == 1.0f && P0.dT == 1.0f && !P0.t_keep && !P0.d_keep;
    const bool stoch = P0.t_stoch != 0;
    const int di = P0.tdt == SD_BF16 ? 0 : 1;
    using K = void (*)(sd::Plan);
    static const K kerns[2][2][2] = {
        {{sd::k_verify_lean<SD_BF16, false, false>, sd::k_verify_lean<SD_BF16, false, true>},
         {sd::k_verify_lean<SD_BF16, true, false>, sd::k_verify_lean<SD_BF16, true, true>}},
        {{sd::k_verify_lean<SD_F16, false, false>, sd::k_verify_lean<SD_F16, false, true>},
         {sd::k_verify_lean<SD_F16, true, false>, sd::k_verify_lean<SD_F16, true, true>}}};
    const K kern = kerns[di][fast][stoch];
    // the staged spans: the target rows and the drafter rows the launch loads, 4 KB each
    const int nload = P0.n_tslots + ((stoch || !P0.dstats) ? P0.gamma : 0);
    const size_t dyn = (size_t)nload * kThreads * sizeof(uint4);
    static std::mutex mu;
    static std::map<std::tuple<int, const void*, size_t>, int> caps;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) { lean_why(10); return 0; }
    int cap;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = caps.find({dev, (const void*)kern, dyn});
        if (it == caps.end()) {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, sd::kLeanThreads, dyn) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                per_cu = cus = 0;
            it = caps.emplace(std::make_tuple(dev, (const void*)kern, dyn), per_cu * cus).first;
        }
        cap = it->second;
    }
    // headroom: every workgroup polls its sequence's others, so the whole grid must be resident; a
    // kernel of another stream holding some CUs must not push it past that, so the grid takes at
    // most half the device's slots (at V = 128256: up to 4 sequences); beyond, k_stats + k_sample
    if (2 * (int64_t)P0.B * n_span > cap && mode < 0) { lean_why(11); return 0; }
    if ((int64_t)P0.B * n_span > cap) { lean_why(11); return 0; }
    sd::Plan P = P0;
    P.n_chunks = n_span;
    P.chunk = kSpan;
    P.kpoll = 1;
    P.xcd_affine = 0;
    // the statistics records after the sampler's (ResPart-sized) chunk records, 16-byte aligned;
    // both fit the workspace's rpart region: B (2γ+1) (nc+1) ResParts >= B n_span (ResPart + 16 (2γ+1))
    const uintptr_t srec = reinterpret_cast<uintptr_t>(P0.rpart + (int64_t)P0.B * n_span);
    P.srec = reinterpret_cast<uint4*>((srec + 15) & ~uintptr_t(15));
    hipLaunchKernelGGL(kern, dim3(n_span, P.B), dim3(sd::kLeanThreads), (unsigned)dyn, (hipStream_t)stream, P);
    if (const hipError_t e = hipGetLastError(); e != hipSuccess) { g_last_error = e; return SD_ERR_LAUNCH; }
    lean_why(0);
    return 1;
}

// STREAM multinomial rows (T = 1, no processor, 16-bit, aligned) in one pass (k_draw_stream,
// sd_draw_stream.inc): 1 if launched, 0 if the shape needs the three-launch path (row statistics,
// k_rowsample, k_sample_finalize), < 0 on a launch error.  Poll mode only: the grid's consumers
// must leave room for every producer (the occupancy check), and sd_set_poll_policy must allow it;
// SD_OPT_DRAW_STREAM = 0 turns it off (A/B, tests).
int32_t launch_draw_stream(const sd::Plan& P, void* stream) {
    if (P.noise.mode != SD_NOISE_STREAM || !P.t_stoch || P.tT != 1.0f || P.t_keep || P.tdt == SD_F32) return 0;
    if (P.token_prob || P.keep_out || P.B > kCntMax || !poll_allowed() || opt(g_opt_draw_stream) == 0) return 0;
    const bool al = (reinterpret_cast<uintptr_t>(P.trow[0]) & 15) == 0 && (P.tstride * 2) % 16 == 0;
    const int n_span = (int)((P.V + kThreads * 8 - 1) / (kThreads * 8));
    if (!al || P.V < 8 || n_span > 128) return 0;
    if ((int64_t)n_span * sd::kDsRecs * 16 > (int64_t)(max_chunks(P.V) + 1) * (int64_t)sizeof(sd::ResPart)) return 0;
    const int cap = resident_cap(P.tdt == SD_BF16 ? (const void*)sd::k_draw_stream<SD_BF16>
                                                  : (const void*)sd::k_draw_stream<SD_F16>);
    if (cap <= 0 || 2 * P.B > cap) return 0;
    sd::DrawStream A{};
    A.rows = static_cast<const char*>(P.trow[0]);
    A.stride_bytes = P.tstride * 2;
    A.recs = reinterpret_cast<uint4*>(P.rpart);
    A.cnt = P.cnt;
    A.next_token = P.next_token;
    A.nt_stride = P.next_token_stride;
    A.row_stats = P.row_stats;
    A.row_status = P.row_status;
    A.words_used = P.words_used;
    A.status_or = P.status_or;
    A.ts = P.ts;
    A.noise = P.noise;
    A.V = P.V;
    A.n_span = n_span;
    A.spin_limit = P.spin_limit;
    A.rows_total = P.B;
    const dim3 grid(n_span, P.B);
    if (P.tdt == SD_BF16) SD_LAUNCH((sd::k_draw_stream<SD_BF16>), grid, dim3(kThreads), stream, A);
    else SD_LAUNCH((sd::k_draw_stream<SD_F16>), grid, dim3(kThreads), stream, A);
    return 1;
}

// greedy sd_sample rows in one pass (k_draw_lean<GREEDY>): 1 if launched, 0 if the shape needs the
// three-launch path (statistics, per-chunk argmax, finalize), < 0 on a launch error
int32_t launch_greedy_lean(const sd::Plan& P, void* stream) {
    const bool fast = P.tT == 1.0f && !P.t_keep && P.tdt != SD_F32;
    const bool al = (reinterpret_cast<uintptr_t>(P.trow[0]) & 15) == 0 && (P.tstride * 2) % 16 == 0;
    const int64_t span = (int64_t)kThreads * 8;
    if (!fast || !al || P.V < 8 || (P.V + span - 1) / span > 128) return 0;
    const int32_t st = P.tdt == SD_BF16 ? launch_draw_lean_t<SD_BF16, 1, true>(P, stream)
                                        : launch_draw_lean_t<SD_F16, 1, true>(P, stream);
    return st == SD_OK ? 1 : st;
}

int32_t launch_draw(sd::Plan& P, void* stream) {
    {
        const bool fast = P.tT == 1.0f && !P.t_keep && P.tdt != SD_F32;
        const bool al = (reinterpret_cast<uintptr_t>(P.trow[0]) & 15) == 0 && (P.tstride * 2) % 16 == 0;
        // one 2048-element span per workgroup (4096-element spans measured slower)
        const int64_t span = (int64_t)kThreads * 8;
        if (fast && al && P.V >= 8 && (P.V + span - 1) / span <= 128) {
            // stages per workgroup: one 2048-element span while the grid is a few thousand
            // workgroups; a large batch takes 2 or 4 stages per workgroup, so each holds more bytes
            // in flight and the grid stays a few resident rounds (SD_OPT_DRAW_SPAN pins it)
            int nst = opt(g_opt_draw_span);
            if (nst == 0) nst = P.B <= kDrawSpan4MinB ? 1 : 4;
            int32_t st;
            if (nst == 4) st = P.tdt == SD_BF16 ? launch_draw_lean_t<SD_BF16, 4>(P, stream) : launch_draw_lean_t<SD_F16, 4>(P, stream);
            else if (nst == 2) st = P.tdt == SD_BF16 ? launch_draw_lean_t<SD_BF16, 2>(P, stream) : launch_draw_lean_t<SD_F16, 2>(P, stream);
            else st = P.tdt == SD_BF16 ? launch_draw_lean_t<SD_BF16, 1>(P, stream) : launch_draw_lean_t<SD_F16, 1>(P, stream);
            if (st == SD_OK) g_sample_path = SD_PATH_SAMPLE_DRAW_LEAN;   // only once the launch succeeded
            return st;
        }
    }
    // spans of NST stages (2048 elements each): 2 once the grid passes ~1024 workgroups
    // (measured at 32 rows of 128256 bf16: NST 1 9.0 us, 2 8.5, 4 10.6 — its registers spill)
    const int64_t stage = kThreads * 8;
    const int64_t nst_row = (P.V + stage - 1) / stage;
    int nst = P.B * nst_row <= 1024 ? 1 : 2;
    if (P.tdt == SD_F32) nst = 2;   // fp32 stages hold 1024 elements: keep spans >= 2048 (workspace sizing)
    const int64_t step = kThreads * (int64_t)(P.tdt == SD_F32 ? 4 : 8);
    P.chunk = (int32_t)(nst * step);
    P.n_chunks = (int32_t)((P.V + P.chunk - 1) / P.chunk);
    P.rn_chunks = P.n_chunks;   // pick_chunk's count
    P.xcd_affine = P.B % 8 == 0;
    const int32_t st = P.tdt == SD_BF16 ? launch_draw_dt<SD_BF16>(P, nst, stream)
                     : P.tdt == SD_F32  ? launch_draw_dt<SD_F32>(P, nst, stream)
                                        : launch_draw_dt<SD_F16>(P, nst, stream);
    if (st == SD_OK) g_sample_path = SD_PATH_SAMPLE_DRAW;
    return st;
}

// The nucleus drafter draw by rejection (k_draw_nuc, sd_draw_nucleus.inc) in place of the threshold
// search + k_draw: PHILOX plain nucleus with top_p >= kNucMinP and T <= 1 (the proposal then keeps
// >= top_p of its mass on the nucleus), 16-bit rows, no token_prob / row_stats / row_keep asked
// (they need the nucleus' own normaliser), and the whole grid resident (its slices poll each other).
// 1: launched; 0: not applicable.
int32_t launch_draw_nuc(const sd::Plan& P, const sd_processor& proc, void* stream) {
    if (P.noise.mode != SD_NOISE_PHILOX || proc.kind != SD_PROC_NUCLEUS) return 0;
    if (!(proc.top_p >= sd::kNucMinP) || !(proc.temperature <= 1.f) || P.tdt == SD_F32) return 0;
    if (P.token_prob || P.row_stats || P.keep_out || !poll_allowed()) return 0;
    // the verify's threshold search must cut this row with the same normaliser: its sub-slice mode
    const int nsl = (P.V + sd::kNucSlice - 1) / sd::kNucSlice;
    if (nsl > kWave || P.B > kCntMax || sd::kThrSlice != 4 * sd::kSubSlice) return 0;
    // the records (kNucRecs x 16 B per slice) inside the row's share of the ResPart region
    if ((int64_t)nsl * sd::kNucRecs * 16 > (int64_t)(max_chunks(P.V) + 1) * (int64_t)sizeof(sd::ResPart)) return 0;
    const int cap = resident_cap((const void*)sd::k_draw_nuc<SD_BF16>, sd::kNucThreads);
    if (cap <= 0 || (int64_t)nsl * P.B > cap) return 0;
    sd::NucArgs A{};
    A.rows = static_cast<const char*>(P.trow[0]);
    A.stride_bytes = P.tstride * 2;
    A.cnt = P.cnt;
    A.rpart = reinterpret_cast<uint4*>(P.rpart);
    A.next_token = P.next_token;
    A.nt_stride = P.next_token_stride;
    A.row_status = P.row_status;
    A.words_used = P.words_used;
    A.ts = P.ts;
    A.noise = P.noise;
    A.V = P.V;
    A.T = proc.temperature;
    A.top_p = proc.top_p;
    A.spin_limit = P.spin_limit;
    A.status_or = P.status_or;
    const dim3 grid(nsl, P.B);
    if (P.tdt == SD_BF16)
        hipLaunchKernelGGL(sd::k_draw_nuc<SD_BF16>, grid, dim3(sd::kNucThreads), 0, (hipStream_t)stream, A);
    else
        hipLaunchKernelGGL(sd::k_draw_nuc<SD_F16>, grid, dim3(sd::kNucThreads), 0, (hipStream_t)stream, A);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { g_last_error = e; return SD_ERR_LAUNCH; }
    return 1;
}

}  // namespace

extern "C" {

int32_t sd_abi_version(void) { return SD_ABI_VERSION; }

int32_t sd_set_poll_policy(int32_t allow_poll, int32_t spin_limit_) {
    if (allow_poll != 0 && allow_poll != 1) return SD_ERR_INVALID;
    policy_init();
    g_allow_poll.store(allow_poll);
    g_spin_limit.store(spin_limit_ == 0 ? kDefaultSpin : spin_limit_);
    return SD_OK;
}

int32_t sd_get_poll_policy(int32_t* allow_poll, int32_t* spin_limit_) {
    if (!allow_poll || !spin_limit_) return SD_ERR_INVALID;
    *allow_poll = poll_allowed() ? 1 : 0;
    *spin_limit_ = spin_limit();
    return SD_OK;
}

const char* sd_last_hip_error(void) { return hipGetErrorString(g_last_error); }

int32_t sd_set_option(int32_t option, int32_t value) {
    std::atomic<int>* o = option_slot(option);
    if (!o) return SD_ERR_INVALID;
    const bool ok = option == SD_OPT_FUSED_VERIFY ? (value >= 0 && value <= 2)
                  : option == SD_OPT_LEAN_VERIFY || option == SD_OPT_FUSED_TICKET ? (value >= -1 && value <= 1)
                  : option == SD_OPT_DRAW_SPAN ? (value == 0 || value == 1 || value == 2 || value == 4)
                  : option == SD_OPT_TICKET_LAG ? (value >= 0 && value <= 64)
                  : option == SD_OPT_SAMP_CHUNKS ? (value == 0 || value == 2 || value == 4 || value == 8)
                                                 : (value == 0 || value == 1);
    if (!ok) return SD_ERR_INVALID;
    o->store(value, std::memory_order_relaxed);
    return SD_OK;
}

int32_t sd_get_option(int32_t option, int32_t* value) {
    std::atomic<int>* o = option_slot(option);
    if (!o || !value) return SD_ERR_INVALID;
    *value = o->load(std::memory_order_relaxed);
    return SD_OK;
}

int32_t sd_last_verify_path(void) { return g_verify_path; }
int32_t sd_last_sample_path(void) { return g_sample_path; }

const char* sd_status_string(int32_t s) {
    switch (s) {
        case SD_OK: return "ok";
        case SD_ERR_INVALID: return "invalid argument";
        case SD_ERR_WORKSPACE: return "workspace too small";
        case SD_ERR_LAUNCH: return "kernel launch failed";
        case SD_ERR_UNSUPPORTED: return "unsupported combination";
        default: return "unknown status";
    }
}

size_t sd_verify_workspace_size(int32_t batch, int32_t gamma, int32_t vocab) {
    if (batch <= 0 || gamma <= 0 || gamma > SD_MAX_GAMMA || vocab <= 0) return 0;
    Plan P{};
    Carve c{nullptr};
    carve(P, c, batch * (2 * gamma + 1), batch, gamma, vocab);
    return c.used;
}

int32_t sd_verify(const sd_verify_args* a, void* stream) {
    clear_stale_error();
    if (!a || a->batch <= 0 || a->gamma <= 0 || a->gamma > SD_MAX_GAMMA || a->vocab <= 0) return SD_ERR_INVALID;
    if (a->rule != SD_RULE_SPEC && a->rule != SD_RULE_ENGINE) return SD_ERR_INVALID;
    if (!valid_dtype(a->target_dtype) || (!a->draft_is_probs && !valid_dtype(a->draft_dtype))) return SD_ERR_INVALID;
    if (!valid_proc(a->target_proc) || !valid_proc(a->draft_proc)) return SD_ERR_INVALID;
    if (!a->draft_tokens || !a->n_accepted || !a->next_token || !a->row_status) return SD_ERR_INVALID;
    if (a->n_stop > 0 && !a->stop_tokens) return SD_ERR_INVALID;
    if (a->noise.mode == SD_NOISE_STREAM && !a->noise.words && a->noise.n_words > 0) return SD_ERR_INVALID;
    if (a->rule == SD_RULE_ENGINE && a->generated && (!a->finished || !a->accepted_count)) return SD_ERR_INVALID;
    const int n_t = a->rule == SD_RULE_SPEC ? a->gamma + 1 : a->gamma;
    for (int t = 0; t < n_t; ++t)
        if (!a->target_rows[t]) return SD_ERR_INVALID;
    for (int t = 0; t < a->gamma; ++t)
        if (!a->draft_rows[t]) return SD_ERR_INVALID;
    if (a->workspace_bytes < sd_verify_workspace_size(a->batch, a->gamma, a->vocab) || !a->workspace)
        return SD_ERR_WORKSPACE;
    if (a->noise.mode != SD_NOISE_STREAM &&
        (a->batch > kCntMax || (a->vocab + kThreads * kEptSmall - 1) / (kThreads * kEptSmall) > kTailChunks))
        return SD_ERR_UNSUPPORTED;

    g_verify_path = SD_PATH_NONE;
    Plan P{};
    static std::atomic<uint32_t> call_seq{0};
    P.call_nonce = 0x9E3779B9u * (call_seq.fetch_add(1, std::memory_order_relaxed) + 1u);
    P.B = a->batch; P.gamma = a->gamma; P.V = a->vocab; P.rule = a->rule;
    P.n_tslots = n_t;
    P.n_dslots = a->draft_is_probs ? 0 : a->gamma;
    P.slots = P.n_tslots + P.n_dslots;
    P.stat_slots = P.slots;
    P.tdt = a->target_dtype; P.ddt = a->draft_is_probs ? SD_F32 : a->draft_dtype;
    P.draft_is_probs = a->draft_is_probs; P.skip_adj = a->skip_sample_adjustment;
    P.t_keep = needs_keep(a->target_proc); P.d_keep = !a->draft_is_probs && needs_keep(a->draft_proc);
    P.t_stoch = a->rule == SD_RULE_ENGINE ? 1 : (a->target_proc.kind != SD_PROC_GREEDY);
    P.tT = a->target_proc.temperature; P.dT = a->draft_proc.temperature;
    if (!(P.tT > 0.f) || (!a->draft_is_probs && !(P.dT > 0.f))) return SD_ERR_INVALID;
    for (int t = 0; t < n_t; ++t) P.trow[t] = a->target_rows[t];
    P.tstride = a->target_stride_b;
    for (int t = 0; t < a->gamma; ++t) P.drow[t] = a->draft_rows[t];
    P.dstride = a->draft_stride_b;
    P.draft_tokens = a->draft_tokens; P.tok_stride = a->draft_tokens_stride_b;
    P.stops = a->stop_tokens; P.n_stop = a->n_stop;
    P.active = a->active; P.noise = a->noise;
    P.n_accepted = a->n_accepted; P.next_token = a->next_token; P.next_token_stride = 1;
    P.resample_mass = a->resample_mass; P.prune_drafter = a->prune_drafter; P.prune_target = a->prune_target;
    P.stop_index = a->stop_index; P.row_status = a->row_status; P.words_used = a->words_used;
    P.generated = a->generated; P.gen_stride = a->generated_stride_b; P.step = a->step;
    P.finished = a->finished; P.accepted_count = a->accepted_count;
    P.status_or = a->status_or;
    P.row_counts = a->row_counts;
    P.spin_limit = spin_limit();
    // drafter row stats that came with the draws (sd_sample row_stats): k_stats reads only the
    // target rows.  A top-k / nucleus drafter also needs the draws' keep predicates
    // (sd_sample row_keep): then the threshold search covers the target rows only.  Without
    // them the stats are a hint the call ignores.
    if (a->draft_row_stats && !a->draft_is_probs && (!P.d_keep || a->draft_row_keep)) {
        if (a->draft_row_stats_stride < a->batch) return SD_ERR_INVALID;
        P.dstats = reinterpret_cast<const float2*>(a->draft_row_stats);
        P.dstats_stride = a->draft_row_stats_stride;
        P.stat_slots = P.n_tslots;
        if (P.d_keep) P.dkeep = reinterpret_cast<const RowKeep*>(a->draft_row_keep);
    }

    // the rows k_stats streams; at least 8 stages per workgroup: few rows (batch 1) then take 8 spans
    // per row instead of 63 one-stage ones (configs[1] multinomial 36.1 -> 33.7 us per step)
    set_stats_chunks(P, P.B * P.stat_slots, 512, 8);
    if (a->noise.mode != SD_NOISE_STREAM && P.B >= kTicketMinB && P.chunk > kTicketSpan) {
        // large perf-mode batches: 4 spans per Llama-3 row instead of one workgroup per row (set_stats_
        // chunks' 512-workgroup target) — the ticket-order fused verify's layout, for both verify paths
        P.chunk = kTicketSpan;
        P.n_chunks = (P.V + P.chunk - 1) / P.chunk;
    }
    Carve c{static_cast<char*>(a->workspace)};
    carve(P, c, a->batch * (2 * a->gamma + 1), a->batch, a->gamma, a->vocab);

    if (P.t_keep || (P.d_keep && !P.dkeep)) {
        Plan Q = P;                  // the drafter rows' keeps came with their draws: skip them
        if (P.dkeep) Q.d_keep = 0;
        const int32_t st = launch_threshold(Q, a->target_proc, a->draft_proc, stream);
        if (st != SD_OK) return st;
    }
    set_rchunks(P);
    const bool perf = P.noise.mode != SD_NOISE_STREAM;
#ifdef SD_PHASE_TIMING
    if (const char* e = getenv("SD_TS_PTR")) P.ts = reinterpret_cast<uint64_t*>(strtoull(e, nullptr, 0));
#endif
    // perf mode: decision / token in the last-arriving workgroups (tails)
    P.coh = perf;
    P.xcd_affine = perf && P.B % 8 == 0;
    if (!a->prof_stats_begin) {   // the batch-1 / few-sequence verify in one launch (sd_verify_lean.inc)
        const int32_t st = launch_verify_lean(P, stream);
        if (st < 0) return st;
        if (st) { g_verify_path = SD_PATH_VERIFY_LEAN; return SD_OK; }
    }
    // the verify in one launch (k_stats with a decider and samplers per sequence, fused_sampler): perf
    // mode, stochastic target rows of one dtype, the drafter stats from the draws.  SD_OPT_FUSED_VERIFY
    // = 0 turns it off; by default it takes B >= 8 (fewer sequences: k_verify_lean above), 2 any B.
    if (perf && P.t_stoch && P.tdt == P.ddt && !P.draft_is_probs && P.dstats &&
        P.stat_slots == P.n_tslots && P.n_tslots <= kFastSlots && P.n_chunks <= kWave && P.B <= kCntMax &&
        !a->prof_stats_begin) {
        const int fmode = opt(g_opt_fused);
        if (fmode == 2 || (fmode == 1 && P.B >= 8)) {
            Plan F = P;
            F.rchunk = kThreads * kFusedEpt;
            F.rn_chunks = (P.V + F.rchunk - 1) / F.rchunk;
            F.samp_cps = 2;                     // two chunks per sampler (fused_sampler); ticket order: below
            F.n_samp = (F.rn_chunks + 1) / 2;
            const bool layout_ok = fused_layout(F);   // block-id or ticket order; may re-cut the spans
            // records: the spans' (srec = rpart), the samplers' totals after them, the decisions, the candidates
            const size_t n_srec = (size_t)P.B * P.stat_slots * F.n_chunks;
            const size_t need = n_srec + 2 * (size_t)P.B * F.rn_chunks + 2 * (size_t)P.B + 8;
            const size_t have = (size_t)(P.B > a->batch * (2 * a->gamma + 1) ? P.B : a->batch * (2 * a->gamma + 1)) *
                                (max_chunks(P.V) + 1) * sizeof(ResPart) / sizeof(uint4);
            if (layout_ok && F.rn_chunks <= kTailChunks && need <= have) {
                F.sprec = F.srec + n_srec;
                F.drec = F.sprec + (size_t)P.B * F.rn_chunks;
                // chunk candidates in records of their own (sample_chunk_pick): the totals go out
                // before the pick's second pass, so the decider's Σ starts earlier (-0.45 us at B=32)
                F.crec = F.drec + 2 * (size_t)P.B;
                const int32_t st = launch_fused(F, stream);
                if (st < 0) return st;
                if (st) { g_verify_path = F.ticket ? SD_PATH_VERIFY_FUSED_TICKET : SD_PATH_VERIFY_FUSED; return SD_OK; }
            }
        }
    }
    if (a->prof_stats_begin) (void)hipEventRecord((hipEvent_t)a->prof_stats_begin, (hipStream_t)stream);
    const int reps = a->prof_stats_begin && a->prof_stats_repeat > 1 ? a->prof_stats_repeat : 1;
    for (int rep = 0; rep < reps; ++rep)
        if (int32_t st = launch_stats(P, stream, perf)) return st;
    if (a->prof_stats_end) (void)hipEventRecord((hipEvent_t)a->prof_stats_end, (hipStream_t)stream);
    if (!perf) {   // parity mode: the reference's serial noise order
        SD_LAUNCH(k_decide, dim3(P.B), dim3(256), stream, P);
        SD_LAUNCH(k_walk, dim3(1), dim3(256), stream, P);
    }
    if (int32_t st = launch_resample(P, stream)) return st;   // perf mode: k_sample finalizes in its tail
    if (!perf) SD_LAUNCH(k_finalize, dim3(P.B), dim3(64), stream, P);
    g_verify_path = perf ? SD_PATH_VERIFY_TWO_LAUNCH : SD_PATH_VERIFY_STREAM;
    return SD_OK;
}

size_t sd_sample_workspace_size(int32_t rows, int32_t vocab) {
    if (rows <= 0 || vocab <= 0) return 0;
    Plan P{};
    Carve c{nullptr};
    carve(P, c, rows, rows, 1, vocab);
    return c.used;
}

int32_t sd_sample(const sd_sample_args* a, void* stream) {
    clear_stale_error();
    if (!a || a->rows <= 0 || a->vocab <= 0 || !a->logits || !a->tokens) return SD_ERR_INVALID;
    if (!valid_dtype(a->dtype) || !valid_proc(a->proc) || !(a->proc.temperature > 0.f)) return SD_ERR_INVALID;
    if (a->noise.mode == SD_NOISE_STREAM && a->proc.kind != SD_PROC_GREEDY && !a->noise.words) return SD_ERR_INVALID;
    if (a->workspace_bytes < sd_sample_workspace_size(a->rows, a->vocab) || !a->workspace) return SD_ERR_WORKSPACE;
    Plan P{};
    P.B = a->rows; P.gamma = 1; P.V = a->vocab; P.rule = -1;
    P.n_tslots = 1; P.n_dslots = 0; P.slots = 1; P.stat_slots = 1;
    P.tdt = a->dtype; P.ddt = a->dtype;
    P.t_keep = needs_keep(a->proc); P.t_stoch = a->proc.kind != SD_PROC_GREEDY;
    P.tT = a->proc.temperature; P.dT = 1.f;
    P.trow[0] = a->logits; P.tstride = a->stride_r;
    P.noise = a->noise;
    P.next_token = a->tokens; P.next_token_stride = a->tokens_stride;
    P.token_prob = a->token_prob; P.row_status = a->row_status; P.words_used = a->words_used;
    P.row_stats = reinterpret_cast<float2*>(a->row_stats);
    P.keep_out = reinterpret_cast<RowKeep*>(a->row_keep);
    P.status_or = a->status_or;
    P.spin_limit = spin_limit();
    set_stats_chunks(P, P.B);
    Carve c{static_cast<char*>(a->workspace)};
    carve(P, c, a->rows, a->rows, 1, a->vocab);
#ifdef SD_PHASE_TIMING
    if (const char* e = getenv("SD_TS_PTR")) P.ts = reinterpret_cast<uint64_t*>(strtoull(e, nullptr, 0));
#endif
    g_sample_path = SD_PATH_NONE;
    if (const int32_t st = launch_draw_nuc(P, a->proc, stream)) {
        if (st < 0) return st;
        g_sample_path = SD_PATH_SAMPLE_NUCLEUS;
        return SD_OK;
    }
    if (P.t_keep) {
        const int32_t st = launch_threshold(P, a->proc, a->proc, stream);
        if (st != SD_OK) return st;
    }
    if (P.noise.mode == SD_NOISE_PHILOX && P.t_stoch) {
        if (P.B > kCntMax || max_chunks(P.V) > kTailChunks) return SD_ERR_UNSUPPORTED;
        return launch_draw(P, stream);   // one pass; the row's last arrival writes the outputs
    }
    if (const int32_t st = launch_draw_stream(P, stream)) {   // STREAM, one pass
        if (st < 0) return st;
        g_sample_path = SD_PATH_SAMPLE_STREAM;
        return SD_OK;
    }
    if (!P.t_stoch && P.B <= kCntMax) {   // greedy (either noise mode: no noise is drawn)
        const int32_t st = launch_greedy_lean(P, stream);
        if (st < 0) return st;
        if (st == 1) { g_sample_path = SD_PATH_SAMPLE_GREEDY_LEAN; return SD_OK; }
    }
    set_rchunks(P);
    if (int32_t st = launch_stats(P, stream)) return st;
    if (int32_t st = launch_rowsample(P, stream)) return st;
    SD_LAUNCH(k_sample_finalize, dim3(P.B), dim3(64), stream, P);
    g_sample_path = SD_PATH_SAMPLE_MULTI;
    return SD_OK;
}

size_t sd_probs_workspace_size(int32_t rows, int32_t vocab) { return sd_sample_workspace_size(rows, vocab); }

int32_t sd_probs(const sd_probs_args* a, void* stream) {
    clear_stale_error();
    if (!a || a->rows <= 0 || a->vocab <= 0 || !a->logits || !a->probs) return SD_ERR_INVALID;
    if (!valid_dtype(a->dtype) || !valid_proc(a->proc) || !(a->proc.temperature > 0.f)) return SD_ERR_INVALID;
    if (a->workspace_bytes < sd_probs_workspace_size(a->rows, a->vocab) || !a->workspace) return SD_ERR_WORKSPACE;
    Plan P{};
    P.B = a->rows; P.gamma = 1; P.V = a->vocab; P.rule = -1;
    P.n_tslots = 1; P.n_dslots = 0; P.slots = 1; P.stat_slots = 1;
    P.tdt = a->dtype; P.ddt = a->dtype;
    P.t_keep = needs_keep(a->proc);
    P.tT = a->proc.temperature; P.dT = 1.f;
    P.trow[0] = a->logits; P.tstride = a->stride_r;
    P.spin_limit = spin_limit();
    set_stats_chunks(P, P.B);
    Carve c{static_cast<char*>(a->workspace)};
    carve(P, c, a->rows, a->rows, 1, a->vocab);
    if (P.t_keep) {
        const int32_t st = launch_threshold(P, a->proc, a->proc, stream);
        if (st != SD_OK) return st;
    }
    set_rchunks(P);
    if (int32_t st = launch_stats(P, stream)) return st;
    P.rchunk = kThreads * kEptSmall;   // plain streaming write: one stage per workgroup
    P.rn_chunks = (P.V + P.rchunk - 1) / P.rchunk;
    const dim3 wg(P.rn_chunks, P.B);
    if (P.tdt == SD_BF16) SD_LAUNCH((k_writeprobs<SD_BF16, 8>), wg, dim3(kThreads), stream, P, a->probs, a->probs_stride_r);
    else if (P.tdt == SD_F32) SD_LAUNCH((k_writeprobs<SD_F32, 8>), wg, dim3(kThreads), stream, P, a->probs, a->probs_stride_r);
    else SD_LAUNCH((k_writeprobs<SD_F16, 8>), wg, dim3(kThreads), stream, P, a->probs, a->probs_stride_r);
    return SD_OK;
}

}  // extern "C"

#include "sd_ngram.inc"
