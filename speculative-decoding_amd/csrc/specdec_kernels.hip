// specdec_kernels.hip — fused speculative verify/accept/resample for MI355X (gfx950).
//
// One verify step (sd_verify) is a short chain of memory-bound kernels on one stream,
// with no host sync and no allocation:
//
//   k_threshold  (top-k / nucleus rows only) radix descent for the keep threshold   -> RowKeep
//   k_stats      grid (chunk, row): per-chunk max / Σexp of the processed row      -> partials
//   k_decide     grid (B): combine partials -> (M, S) per row; p(x_i), q(x_i)
//   k_walk       accept rule walk (A8 / A10), noise offsets, per-row decision
//   k_resample   grid (chunk, B): Σ(p_n - q_n)+ and exact argmax candidates of the
//                residual / bonus / p-row sample, in ONE pass over the two rows
//   k_finalize   grid (B): combine, exact candidate evaluation, outputs, engine state
//
// Every logit row is read once by k_stats (the algorithmic bytes); k_resample re-reads
// at most two rows per sequence (served from the 256 MiB Infinity Cache).  See DESIGN.md.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>

#include "sd_device.h"

namespace sd {

constexpr int kMaxCand = 8;

struct Decision {
    int32_t n;          // accepted drafts
    int32_t mode;       // kModeNone / Bonus / Resid / PRow
    int32_t slot;       // target slot sampled from (bonus: gamma, resid/prow: n)
    int32_t status;     // SD_ROW_* bits
    int64_t noise_off;  // STREAM: word offset of the Exp noise; PHILOX: unused
    int32_t stop_index;
    int32_t pad;
};
enum { kModeNone = 0, kModeBonus = 1, kModeResid = 2, kModePRow = 3 };

struct ResPart {
    float sum;                 // Σ residual over the chunk
    float wmax;                // max residual / E
    int32_t ncand;             // candidates kept (> kMaxCand => overflow)
    float pval;                // argmax value (bonus / p-row / engine p fallback)
    int32_t pidx;
    float cres[kMaxCand];      // candidate residual value
    float ce[kMaxCand];        // candidate noise value
    int32_t cidx[kMaxCand];
};

struct Plan {
    int32_t B, gamma, V, rule;
    int32_t n_tslots, n_dslots, slots, n_chunks, chunk;
    int32_t rn_chunks, rchunk;   // chunking of the resample / sample passes
    int32_t diag;                // SD_DIAG tuning bits (0 in production)
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
    int32_t* keep_hist;   // threshold scratch
};

__device__ __forceinline__ const void* row_ptr(const Plan& P, int r, int* dt, float* T, bool* keep) {
    const int b = r / P.slots, s = r - b * P.slots;
    if (s < P.n_tslots) {
        *dt = P.tdt; *T = P.tT; *keep = P.t_keep;
        return static_cast<const char*>(P.trow[s]) + b * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
    }
    *dt = P.ddt; *T = P.dT; *keep = P.d_keep;
    return static_cast<const char*>(P.drow[s - P.n_tslots]) + b * P.dstride * (P.ddt == SD_F32 ? 4 : 2);
}

__device__ __forceinline__ bool is_stop(const Plan& P, int64_t tok) {
    for (int k = 0; k < P.n_stop; ++k)
        if (P.stops[k] == tok) return true;
    return false;
}

// ------------------------------------------------------------------ block helpers
template <typename F>
__device__ __forceinline__ float block_reduce(float v, F op, float* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, kWave));
    __syncthreads();
    if (lane == 0) lds[w] = v;
    __syncthreads();
    float r = lds[0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = op(r, lds[k]);
    return r;
}

__device__ __forceinline__ void block_argmax(float& v, int32_t& i, float* ldsv, int32_t* ldsi) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    wave_argmax(v, i);
    __syncthreads();
    if (lane == 0) { ldsv[w] = v; ldsi[w] = i; }
    __syncthreads();
    v = ldsv[0]; i = ldsi[0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
        if (arg_better(ldsv[k], ldsi[k], v, i)) { v = ldsv[k]; i = ldsi[k]; }
}

struct FMax { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
struct FSum { __device__ float operator()(float a, float b) const { return a + b; } };

// ------------------------------------------------------------------ k_stats
// grid (span, row-of-group): running max / Σexp of y = round_dt(_process(x)/T) over one span of a
// row, streamed through a 4-deep register pipeline (16 B per lane per stage, 16 KiB per
// workgroup in flight) with an online rescaled sum, so loads stay in flight while exp() runs.
constexpr int kPipe = 4;
constexpr float kLog2e = 1.44269502162933349609375f;

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    const float mn = fmaxf(m, m2);
    if (mn == -INFINITY) return;
    s = (m > -INFINITY ? s * sd_exp(m - mn) : 0.f) + (m2 > -INFINITY ? s2 * sd_exp(m2 - mn) : 0.f);
    m = mn;
}

__device__ __forceinline__ const void* slot_row(const Plan& P, int b, int s) {
    if (s < P.n_tslots)
        return static_cast<const char*>(P.trow[s]) + b * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
    return static_cast<const char*>(P.drow[s - P.n_tslots]) + b * P.dstride * (P.ddt == SD_F32 ? 4 : 2);
}

// <= 80 SGPRs keeps 8 workgroups of 256 threads resident per CU (MI355X_MICROARCH.md, residency)
template <int DT, bool FAST>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_num_sgpr(80))) k_stats(Plan P, int slot_lo, int slot_cnt) {
    __shared__ float lm[4], ls[4];
    constexpr int VEC = Elem<DT>::kVec;
    constexpr int STEP = kThreads * VEC;                      // elements per workgroup stage
    const int b = blockIdx.y / slot_cnt, s = slot_lo + blockIdx.y % slot_cnt;
    const int r = b * P.slots + s;
    const void* row = slot_row(P, b, s);
    const bool is_t = s < P.n_tslots;
    const float T = is_t ? P.tT : P.dT;
    const bool has_keep = !FAST && (is_t ? P.t_keep : P.d_keep);
    const RowKeep kp = has_keep ? P.keep[r] : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const int64_t lo = (int64_t)blockIdx.x * P.chunk;
    const int64_t hi = lo + P.chunk < P.V ? lo + P.chunk : P.V;
    const bool aligned = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
    const int nit = (int)((hi - lo + STEP - 1) / STEP);
    float m = -INFINITY, acc = 0.f;

    // Terms are exp(y - m) = exp2((y - m) * log2e): subtract, multiply, v_exp_f32.  y - m is exact
    // for bf16/fp16 values (and for fp32 ones within 2^24 of each other); the multiply's rounding
    // gives each term an independent ~|y-m|*6e-8 relative error that averages down in the sum, and
    // no rounded product is shared by all terms, so S carries no common bias.  Consumers compute
    // numerators with the compensated sd_exp.  The running reference m may trail the true max by
    // up to 20 (terms stay <= e^20): rescales become rare after the first vectors, and every
    // consumer uses (m, S) as a pair.
    auto consume = [&](const float* x, int64_t e0) {
        float y[VEC];
        float vm = -INFINITY;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            y[k] = (e0 + k < hi) ? (FAST ? x[k] : process_value<DT>(x[k], e0 + k, T, has_keep, kp)) : -INFINITY;
            vm = fmaxf(vm, y[k]);
        }
        if (vm > m + 20.f) {
            acc = m > -INFINITY ? acc * sd_exp(m - vm) : 0.f;
            m = vm;
        }
        if (m > -INFINITY) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) acc += __builtin_amdgcn_exp2f((y[k] - m) * kLog2e);
        }
    };
    // steady state: stages where every lane's 16-byte vector is in range.  Loads are issued
    // unconditionally (the prefetch index is clamped), so the compiler keeps kPipe of them in
    // flight with counted vmcnt waits instead of draining to vmcnt(0) each stage.
    const int nfull = aligned ? (int)((hi - lo) / STEP) : 0;
    if (nfull > 0) {
        const uint4* vb = reinterpret_cast<const uint4*>(static_cast<const char*>(row) + lo * Elem<DT>::kBytes) +
                          threadIdx.x;
        uint4 buf[kPipe];
#pragma unroll
        for (int d = 0; d < kPipe; ++d) buf[d] = vb[(d < nfull ? d : nfull - 1) * kThreads];
        int it = 0;
        for (; it + kPipe <= nfull; it += kPipe) {
#pragma unroll
            for (int d = 0; d < kPipe; ++d) {
                const uint4 v = buf[d];
                const int nx = it + d + kPipe;
                buf[d] = vb[(nx < nfull ? nx : nfull - 1) * kThreads];
                float x[VEC];
                unpack16<DT>(v, x);
                consume(x, lo + ((int64_t)(it + d) * kThreads + threadIdx.x) * VEC);
            }
        }
#pragma unroll
        for (int d = 0; d < kPipe; ++d) {
            if (it + d < nfull) {
                float x[VEC];
                unpack16<DT>(buf[d], x);
                consume(x, lo + ((int64_t)(it + d) * kThreads + threadIdx.x) * VEC);
            }
        }
    }
    // ragged tail (and misaligned rows): guarded element loads
    for (int it = nfull; it < nit; ++it) {
        const int64_t e0 = lo + ((int64_t)it * kThreads + threadIdx.x) * VEC;
        float x[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = (e0 + k < hi) ? load_one<DT>(row, e0 + k) : 0.f;
        consume(x, e0);
    }
    // workgroup combine (fixed order)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, kWave), s2 = __shfl_xor(acc, o, kWave);
        online_merge(m, acc, m2, s2);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { lm[w] = m; ls[w] = acc; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = lm[0], S = ls[0];
        for (int k = 1; k < kThreads / kWave; ++k) online_merge(M, S, lm[k], ls[k]);
        P.part[(int64_t)r * P.n_chunks + blockIdx.x] = make_float2(M, S);
    }
}

// combine the chunk partials of row r (one wave)
__device__ __forceinline__ float2 combine_row(const Plan& P, int r) {
    const int lane = threadIdx.x & 63;
    const float2* pr = P.part + (int64_t)r * P.n_chunks;
    float m = -INFINITY;
    for (int c = lane; c < P.n_chunks; c += kWave) m = fmaxf(m, pr[c].x);
    m = wave_max(m);
    // fixed-order sum: lane-strided partial sums, then a fixed butterfly
    float s = 0.f;
    for (int c = lane; c < P.n_chunks; c += kWave)
        if (pr[c].x > -INFINITY) s += pr[c].y * sd_exp(pr[c].x - m);
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
__device__ void seq_stats(const Plan& P, int b, float2* lstat, bool publish) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (P.n_chunks <= kWave) {
        // one partial per lane per slot: issue every slot's load of this wave before reducing
        constexpr int kMaxSlotsPerWave = (2 * SD_MAX_GAMMA + 1 + 3) / 4;
        float2 v[kMaxSlotsPerWave];
#pragma unroll
        for (int k = 0; k < kMaxSlotsPerWave; ++k) {
            const int s = w + k * nw;
            v[k] = (s < P.slots && lane < P.n_chunks) ? P.part[(int64_t)(b * P.slots + s) * P.n_chunks + lane]
                                                      : make_float2(-INFINITY, 0.f);
        }
#pragma unroll
        for (int k = 0; k < kMaxSlotsPerWave; ++k) {
            const int s = w + k * nw;
            if (s >= P.slots) break;
            const float m = wave_max(v[k].x);
            const float sum = wave_sum(v[k].x > -INFINITY ? v[k].y * sd_exp(v[k].x - m) : 0.f);
            if (lane == 0) {
                lstat[s] = make_float2(m, sum);
                if (publish) P.rowstat[b * P.slots + s] = make_float2(m, sum);   // read by later launches only
            }
        }
        return;
    }
    for (int s = w; s < P.slots; s += nw) {
        const float2 ms = combine_row(P, b * P.slots + s);
        if (lane == 0) {
            lstat[s] = ms;
            if (publish) P.rowstat[b * P.slots + s] = ms;
        }
    }
}

// Raw logits at the drafted ids (threads < γ): issued before seq_stats so both load chains overlap.
__device__ void seq_fetch(const Plan& P, int b, float* lxt, float* lxd) {
    if (threadIdx.x >= P.gamma) return;
    const int i = threadIdx.x;
    const int64_t tok = P.draft_tokens[b * P.tok_stride + i];
    float xt = 0.f, xd = 0.f;
    if (tok >= 0 && tok < P.V) {
        int dt; float T; bool keep;
        xt = load_dyn(P.tdt, row_ptr(P, b * P.slots + i, &dt, &T, &keep), tok);
        if (P.draft_is_probs) xd = static_cast<const float*>(P.drow[i])[b * P.dstride + tok];
        else xd = load_dyn(P.ddt, row_ptr(P, b * P.slots + P.n_tslots + i, &dt, &T, &keep), tok);
    }
    lxt[i] = xt;
    lxd[i] = xd;
}

// p(x_i), q(x_i) from the fetched raw values and the row stats (threads < γ; after a barrier)
__device__ void seq_ratios_from(const Plan& P, int b, const float2* lstat, const float* lxt, const float* lxd,
                                float* lp, float* lq) {
    if (threadIdx.x >= P.gamma) return;
    const int i = threadIdx.x;
    const int64_t tok = P.draft_tokens[b * P.tok_stride + i];
    float p = 0.f, q = 0.f;
    if (tok >= 0 && tok < P.V) {
        const int rt = b * P.slots + i;
        const RowKeep kt = P.t_keep ? P.keep[rt] : RowKeep{-INFINITY, INT_MAX, 0, 0};
        const float yt = P.tdt == SD_BF16 ? process_value<SD_BF16>(lxt[i], tok, P.tT, P.t_keep, kt)
                       : P.tdt == SD_F32 ? process_value<SD_F32>(lxt[i], tok, P.tT, P.t_keep, kt)
                                         : process_value<SD_F16>(lxt[i], tok, P.tT, P.t_keep, kt);
        p = round_dyn(P.tdt, sd_exp(yt - lstat[i].x) / lstat[i].y);
        if (P.draft_is_probs) {
            q = lxd[i];
        } else {
            const int rd = b * P.slots + P.n_tslots + i;
            const RowKeep kd = P.d_keep ? P.keep[rd] : RowKeep{-INFINITY, INT_MAX, 0, 0};
            const float2 sd = lstat[P.n_tslots + i];
            const float yd = P.ddt == SD_BF16 ? process_value<SD_BF16>(lxd[i], tok, P.dT, P.d_keep, kd)
                           : P.ddt == SD_F32 ? process_value<SD_F32>(lxd[i], tok, P.dT, P.d_keep, kd)
                                             : process_value<SD_F16>(lxd[i], tok, P.dT, P.d_keep, kd);
            q = round_dyn(P.ddt, sd_exp(yd - sd.x) / sd.y);
        }
    }
    lp[i] = p;
    lq[i] = q;
}

// p(x_i), q(x_i) of the γ drafts (threads < γ; call after seq_stats + barrier)
__device__ void seq_ratios(const Plan& P, int b, const float2* lstat, float* lp, float* lq) {
    if (threadIdx.x >= P.gamma) return;
    const int i = threadIdx.x;
    const int64_t tok = P.draft_tokens[b * P.tok_stride + i];
    int dt; float T; bool keep;
    const int rt = b * P.slots + i;
    const void* trow = row_ptr(P, rt, &dt, &T, &keep);
    const RowKeep kt = keep ? P.keep[rt] : RowKeep{-INFINITY, INT_MAX, 0, 0};
    float p = 0.f, q = 0.f;
    if (tok >= 0 && tok < P.V) {
        p = prob_dyn(dt, trow, tok, T, keep, kt, lstat[i]);
        if (P.draft_is_probs) {
            q = static_cast<const float*>(P.drow[i])[b * P.dstride + tok];
        } else {
            const int rd = b * P.slots + P.n_tslots + i;
            const void* drow = row_ptr(P, rd, &dt, &T, &keep);
            const RowKeep kd = keep ? P.keep[rd] : RowKeep{-INFINITY, INT_MAX, 0, 0};
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
        if (woff >= P.noise.n_words) { *overrun = true; return 0.f; }
        return uniform_from_word(P.noise.words[woff]);
    }
    return uniform_from_word(philox_block(P.noise, (uint32_t)b, kSiteAccept, (uint32_t)i).x);
}

// The accept rule for one sequence given p(x_i), q(x_i); woff = its first noise word (STREAM).
__device__ Decision walk_core(const Plan& P, int b, const float* rp, const float* rq, int64_t woff, int64_t* used_out) {
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
            const float r = draw_uniform(P, b, i, woff + i, &overrun);
            const float frac = rp[i] / rq[i];
            if (r > frac && n == g) n = i;
        }
        used = g;
        d.n = n;
        // :150-155 stop token among the accepted drafts -> the reference returns before sampling
        for (int j = 0; j < n; ++j)
            if (is_stop(P, P.draft_tokens[b * P.tok_stride + j])) { d.stop_index = j; break; }
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
                const int64_t tok = P.draft_tokens[b * P.tok_stride + i];
                const double p = rp[i], q = rq[i];
                const double ap = q <= 0.0 ? 1.0 : fmin(1.0, p / q);
                const float u = draw_uniform(P, b, i, woff + used, &overrun);
                used += 1;
                if ((double)u < ap) {
                    d.n += 1;
                    if (is_stop(P, tok)) { d.status |= SD_ROW_FINISHED; break; }
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
                    d.noise_off + sample_words > P.noise.n_words))
        d.status |= SD_ROW_NOISE_OVERRUN;
    *used_out = used;
    return d;
}

__device__ void publish_decision(const Plan& P, int b, const Decision& d) {
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

__global__ void __launch_bounds__(256) k_walk(Plan P) {
    if (P.noise.mode == SD_NOISE_STREAM) {
        // the reference draws row after row from one generator: serial by construction
        if (threadIdx.x == 0) {
            int64_t off = 0;
            for (int b = 0; b < P.B; ++b) off += walk_seq(P, b, off);
            if (P.words_used) *P.words_used = off;
        }
    } else {
        for (int b = threadIdx.x; b < P.B; b += blockDim.x) walk_seq(P, b, 0);
        if (threadIdx.x == 0 && P.words_used) *P.words_used = 0;
    }
}

// ------------------------------------------------------------------ k_resample
// grid (chunk, B).  RESID: Σ(p_n - q_n)+ and the argmax candidates of fl(fl(res/S)/E) in one pass
// over the two rows; BONUS / PROW: argmax of the multinomial (or greedy) value of the target row.
constexpr float kCandTol = 1.0f - 16.0f * 5.9604645e-08f;   // candidates within 16 ulp of the max

template <int TDT, int DDT, int NZ, int EPT, bool FAST>
__device__ void resid_body(const Plan& P, const Decision& d, int b, int c, float2 mst, float2 msd_in) {
    __shared__ float ldsf[8];
    __shared__ int32_t lcount;
    __shared__ float lres[kMaxCand], le[kMaxCand];
    __shared__ int32_t lidx[kMaxCand];
    constexpr int VEC = Elem<TDT>::kVec < Elem<DDT>::kVec ? Elem<TDT>::kVec : Elem<DDT>::kVec;
    constexpr int NV = EPT / VEC;
    const int rt = b * P.slots + d.slot;
    const void* trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (TDT == SD_F32 ? 4 : 2);
    const bool t_al = (reinterpret_cast<uintptr_t>(trow) & 15) == 0;
    const RowKeep kt = P.t_keep ? P.keep[rt] : RowKeep{-INFINITY, INT_MAX, 0, 0};
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
        if (P.d_keep) kd = P.keep[rd];
    }
    const bool d_al = (reinterpret_cast<uintptr_t>(drow) & 15) == 0;
    const float t_inv = 1.0f / mst.y, d_inv = 1.0f / msd.y;

    float sum = 0.f, wmax = 0.f;
    float res[EPT], ev[EPT];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float xt[VEC], xd[VEC], e[VEC];
        load_vec<TDT>(trow, e0, P.V, t_al, xt);
        if (P.draft_is_probs) load_vec<SD_F32>(drow, e0, P.V, d_al, xd);
        else load_vec<DDT>(drow, e0, P.V, d_al, xd);
        if (stoch) exp_noise_vec<VEC, NZ>(P.noise, d.noise_off, b, e0, P.V, e);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            const float yt = FAST ? xt[k] : process_value<TDT>(xt[k], j, P.tT, P.t_keep, kt);
            const float p = prob_exact<TDT>(yt, mst.x, mst.y, t_inv);
            float q;
            if (P.draft_is_probs) {
                q = xd[k];
            } else {
                const float yd = FAST ? xd[k] : process_value<DDT>(xd[k], j, P.dT, P.d_keep, kd);
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
    const float bsum = block_reduce(sum, FSum(), ldsf);
    const float bw = block_reduce(wmax, FMax(), ldsf);
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    // any j whose exact fl(fl(res/S)/E) can tie the maximum has res/E within a few ulp of it
    const float thr = bw * kCandTol;
    if (bw > 0.f) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const int idx = v * VEC + k;
                const float w = stoch ? res[idx] * __builtin_amdgcn_rcpf(ev[idx]) : res[idx];
                if (res[idx] > 0.f && w >= thr) {
                    const int slot = atomicAdd(&lcount, 1);
                    if (slot < kMaxCand) {
                        lres[slot] = res[idx];
                        le[slot] = ev[idx];
                        lidx[slot] = (int32_t)(base + ((int64_t)v * kThreads + threadIdx.x) * VEC + k);
                    }
                }
            }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ResPart& o = P.rpart[(int64_t)b * P.rn_chunks + c];
        o.sum = bsum;
        o.wmax = bw;
        o.ncand = lcount;
        for (int k = 0; k < kMaxCand && k < lcount; ++k) { o.cres[k] = lres[k]; o.ce[k] = le[k]; o.cidx[k] = lidx[k]; }
    }
}

template <int TDT, int NZ, int EPT, bool FAST>
__device__ void prow_body(const Plan& P, const Decision& d, int b, int c, float2 mst) {
    __shared__ float ldsf[8];
    __shared__ int32_t ldsi[8];
    constexpr int VEC = Elem<TDT>::kVec, NV = EPT / VEC;
    const int rt = b * P.slots + d.slot;
    const void* trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (TDT == SD_F32 ? 4 : 2);
    const bool t_al = (reinterpret_cast<uintptr_t>(trow) & 15) == 0;
    const RowKeep kt = P.t_keep ? P.keep[rt] : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const bool stoch = P.t_stoch != 0;
    const int64_t base = (int64_t)c * P.rchunk;
    const float t_inv = 1.0f / mst.y;
    float pv = -INFINITY;
    int32_t pi = INT_MAX;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float xt[VEC], e[VEC];
        load_vec<TDT>(trow, e0, P.V, t_al, xt);
        if (stoch) exp_noise_vec<VEC, NZ>(P.noise, d.noise_off, b, e0, P.V, e);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= P.V) continue;
            const float p = prob_exact<TDT>(FAST ? xt[k] : process_value<TDT>(xt[k], j, P.tT, P.t_keep, kt),
                                            mst.x, mst.y, t_inv);
            float val = p;
            if (stoch) {   // multinomial: round_dt(p / round_dt(E))
                const float eb = round_dt<TDT>(e[k]);
                val = div_round<TDT>(p, eb, __builtin_amdgcn_rcpf(eb));
            }
            if (arg_better(val, (int32_t)j, pv, pi)) { pv = val; pi = (int32_t)j; }
        }
    }
    block_argmax(pv, pi, ldsf, ldsi);
    if (threadIdx.x == 0) {
        ResPart& o = P.rpart[(int64_t)b * P.rn_chunks + c];
        o.pval = pv;
        o.pidx = pi;
    }
}

// FUSED (perf mode): every workgroup of sequence b first re-derives the decision itself — row
// stats from the k_stats partials, p(x_i)/q(x_i), the accept walk on Philox uniforms — which is
// cheap next to a kernel boundary; chunk 0 publishes it for k_finalize.  STREAM (parity) mode
// reads the decision of the serial k_decide -> k_walk stages instead.
template <int TDT, int DDT, int NZ, bool FUSED, int EPT, bool FAST>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_num_sgpr(80))) k_resample(Plan P) {
    __shared__ float2 lstat[2 * SD_MAX_GAMMA + 1];
    __shared__ float lp[SD_MAX_GAMMA], lq[SD_MAX_GAMMA];
    __shared__ Decision ldec;
    const int b = blockIdx.y, c = blockIdx.x;
    Decision d;
    float2 mst, msd = make_float2(0.f, 1.f);
    if (P.diag & 1) {   // diagnostic: decision = residual at slot 0, stats from the previous call
        d = Decision{};
        d.mode = kModeResid;
        d.slot = 0;
        d.status = SD_ROW_DONE | SD_ROW_RESIDUAL;
        mst = P.rowstat[b * P.slots];
        msd = P.rowstat[b * P.slots + P.n_tslots];
        if (P.diag & 2) return;
        resid_body<TDT, DDT, NZ, EPT, FAST>(P, d, b, c, mst, msd);
        return;
    }
    if constexpr (FUSED) {
        __shared__ float lxt[SD_MAX_GAMMA], lxd[SD_MAX_GAMMA];
        seq_fetch(P, b, lxt, lxd);          // threads < γ: drafted ids -> raw logits (2 dependent loads)
        seq_stats(P, b, lstat, c == 0);     // meanwhile every wave reduces k_stats partials
        __syncthreads();
        seq_ratios_from(P, b, lstat, lxt, lxd, lp, lq);
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t used;
            ldec = walk_core(P, b, lp, lq, 0, &used);
            if (c == 0) {
                publish_decision(P, b, ldec);
                if (P.words_used && b == 0) *P.words_used = 0;
            }
        }
        __syncthreads();
        d = ldec;
        if (d.mode == kModeNone || (P.diag & 2)) return;
        mst = lstat[d.slot];
        if (d.mode == kModeResid && !P.draft_is_probs) msd = lstat[P.n_tslots + d.slot];
    } else {
        d = P.dec[b];
        if (d.mode == kModeNone || (d.status & SD_ROW_NOISE_OVERRUN)) return;
        mst = P.rowstat[b * P.slots + d.slot];
        if (d.mode == kModeResid && !P.draft_is_probs) msd = P.rowstat[b * P.slots + P.n_tslots + d.slot];
    }
    if (d.mode == kModeResid) resid_body<TDT, DDT, NZ, EPT, FAST>(P, d, b, c, mst, msd);
    else prow_body<TDT, NZ, EPT, FAST>(P, d, b, c, mst);
}

// ------------------------------------------------------------------ k_finalize
// grid (B), one wave.
__global__ void __launch_bounds__(64) k_finalize(Plan P) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const Decision d = P.dec[b];
    const int g = P.gamma;
    int64_t x = -1;
    float mass = NAN;
    int32_t status = d.status;
    if (d.mode != kModeNone && !(status & SD_ROW_NOISE_OVERRUN)) {
        const ResPart* rp = P.rpart + (int64_t)b * P.rn_chunks;
        if (d.mode == kModeResid) {
            // fixed-order residual sum (lane-strided over chunks, then a fixed butterfly)
            float s = 0.f, wm = 0.f;
            int overflow = 0;
            for (int c = lane; c < P.rn_chunks; c += kWave) {
                s += rp[c].sum;
                wm = fmaxf(wm, rp[c].wmax);
            }
            s = wave_sum(s);
            wm = wave_max(wm);
            mass = s;
            const int rt = b * P.slots + d.slot;
            const RowKeep kt = P.t_keep ? P.keep[rt] : RowKeep{-INFINITY, INT_MAX, 0, 0};
            const void* trow = static_cast<const char*>(P.trow[d.slot]) + b * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
            const float2 mst = P.rowstat[rt];
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
            } else if (s == 0.f) {
                // max_fn divides by zero: all-NaN distribution
                if (P.t_stoch) status |= SD_ROW_INVALID_DIST;
                else x = 0;   // torch.argmax over an all-NaN row
            } else {
                // exact evaluation of the candidates: v = fl(fl(res / S) / E)
                const float thr = wm * kCandTol;
                float bv = -INFINITY;
                int32_t bi = INT_MAX;
                for (int c = lane; c < P.rn_chunks; c += kWave) {
                    const ResPart& o = rp[c];
                    if (o.wmax < thr) continue;
                    if (o.ncand > kMaxCand) { overflow = 1; continue; }
                    for (int k = 0; k < o.ncand; ++k) {
                        const float pr = o.cres[k] / s;
                        const float v = P.t_stoch ? pr / o.ce[k] : pr;
                        if (arg_better(v, o.cidx[k], bv, bi)) { bv = v; bi = o.cidx[k]; }
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
                        if (P.d_keep) kd = P.keep[rd];
                        msd = P.rowstat[rd];
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
            for (int c = lane; c < P.rn_chunks; c += kWave)
                if (arg_better(rp[c].pval, rp[c].pidx, pv, pi)) { pv = rp[c].pval; pi = rp[c].pidx; }
            wave_argmax(pv, pi);
            x = pi;
        }
    }
    if (lane == 0) {
        P.next_token[b * P.next_token_stride] = x;
        if (P.resample_mass) P.resample_mass[b] = mass;
        // engine/infer_engine.py:307-336 applied in place
        const bool engine_state = P.rule == SD_RULE_ENGINE && P.generated != nullptr;
        if (engine_state && (status & SD_ROW_DONE)) {
            int64_t* gen = P.generated + b * P.gen_stride;
            if (d.mode == kModeResid && x >= 0) {
                gen[P.step + d.n] = x;
                if (is_stop(P, x)) status |= SD_ROW_FINISHED;
            }
            if (d.n < g)
                for (int t = P.step + d.n + 1; t < P.step + g; ++t) gen[t] = 0;
            if (status & SD_ROW_FINISHED) P.finished[b] = 1;
            P.accepted_count[b] += d.n;
        } else if (P.rule == SD_RULE_ENGINE && d.mode == kModeResid && x >= 0 && is_stop(P, x)) {
            status |= SD_ROW_FINISHED;
        }
        if (P.t_keep)
            for (int s2 = 0; s2 < P.n_tslots; ++s2) status |= P.keep[b * P.slots + s2].flags;
        if (P.d_keep)
            for (int s2 = P.n_tslots; s2 < P.slots; ++s2) status |= P.keep[b * P.slots + s2].flags;
        P.row_status[b] = status;
    }
}

// ------------------------------------------------------------------ sd_sample kernels
// grid (chunk, R): argmax of round_dt(p / round_dt(E)) (multinomial) or p (greedy).
template <int DT, int NZ, int EPT>
__device__ void rowsample_body(const Plan& P, int r, int c) {
    __shared__ float ldsf[8];
    __shared__ int32_t ldsi[8];
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
    const RowKeep kp = P.t_keep ? P.keep[r] : RowKeep{-INFINITY, INT_MAX, 0, 0};
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
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= P.V) continue;
            const float p = prob_exact<DT>(process_value<DT>(x[k], j, P.tT, P.t_keep, kp), ms.x, ms.y, inv_s);
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

template <int DT, int NZ, int EPT>
__global__ void __launch_bounds__(kThreads) k_rowsample(Plan P) {
    rowsample_body<DT, NZ, EPT>(P, blockIdx.y, blockIdx.x);
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
        if (P.t_stoch && (!(ms.y > 0.f) || ms.y != ms.y)) st |= SD_ROW_INVALID_DIST;
        if (P.t_keep) st |= P.keep[r].flags;
        if (P.noise.mode == SD_NOISE_STREAM && P.t_stoch && 2ll * P.V * P.B > P.noise.n_words)
            st |= SD_ROW_NOISE_OVERRUN;
        P.next_token[r * P.next_token_stride] = pi;
        if (P.token_prob) {
            const void* row = static_cast<const char*>(P.trow[0]) + r * P.tstride * (P.tdt == SD_F32 ? 4 : 2);
            const RowKeep kp = P.t_keep ? P.keep[r] : RowKeep{-INFINITY, INT_MAX, 0, 0};
            P.token_prob[r] = (pi >= 0 && pi < P.V) ? prob_dyn(P.tdt, row, pi, P.tT, P.t_keep, kp, ms) : NAN;
        }
        if (P.row_status) P.row_status[r] = st;
        if (r == 0 && P.words_used) *P.words_used = P.t_stoch ? 2ll * P.V * P.B : 0;
    }
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
    const RowKeep kp = P.t_keep ? P.keep[r] : RowKeep{-INFINITY, INT_MAX, 0, 0};
    const int64_t base = (int64_t)c * P.rchunk;
    char* orow = static_cast<char*>(out) + r * ostride * (DT == SD_F32 ? 4 : 2);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t e0 = base + ((int64_t)v * kThreads + threadIdx.x) * VEC;
        float x[VEC];
        load_vec<DT>(row, e0, P.V, al, x);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int64_t j = e0 + k;
            if (j >= P.V) continue;
            const float p = round_dt<DT>(sd_exp(process_value<DT>(x[k], j, P.tT, P.t_keep, kp) - ms.x) / ms.y);
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
}  // namespace

#include "sd_threshold.inc"

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
    P.part = c.take<float2>((size_t)rows_total * nc);
    P.rowstat = c.take<float2>(rows_total);
    P.keep = c.take<RowKeep>(rows_total);
    P.rp = c.take<float>((size_t)B * gamma);
    P.rq = c.take<float>((size_t)B * gamma);
    P.dec = c.take<Decision>(B);
    P.rpart = c.take<ResPart>((size_t)(B > rows_total ? B : rows_total) * nc);
    P.keep_hist = c.take<int32_t>((size_t)rows_total * kThreshScratchInts);
}

bool valid_dtype(int dt) { return dt == SD_F32 || dt == SD_BF16 || dt == SD_F16; }
bool valid_proc(const sd_processor& p) {
    if (p.kind < SD_PROC_GREEDY || p.kind > SD_PROC_TOPK_NUCLEUS) return false;
    if ((p.kind == SD_PROC_TOPK || p.kind == SD_PROC_TOPK_NUCLEUS) && p.top_k <= 0) return false;
    return true;
}
bool needs_keep(const sd_processor& p) { return p.kind >= SD_PROC_TOPK; }

// Span of a k_stats workgroup: a multiple of one 2048-element stage, sized so the whole grid is
// resident at once (<= 2048 workgroups = 256 CUs x 8): a grid a little over one residency
// wave would run its remainder on 1/8 of the chip.  SD_STATS_STAGES overrides (tuning).
void set_stats_chunks(sd::Plan& P, int rows) {
    const int64_t stage = kThreads * 8;
    const int64_t stages_per_row = (P.V + stage - 1) / stage;
    int64_t per_wg = (rows * stages_per_row + 2047) / 2048;
    if (const char* e = getenv("SD_STATS_STAGES")) per_wg = atoi(e);
    per_wg = per_wg < 1 ? 1 : (per_wg > 16 ? 16 : per_wg);
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

int32_t launch_stats(const sd::Plan& P, void* stream);

#define SD_LAUNCH(kern, grid, block, stream, ...)                                             \
    do {                                                                                      \
        hipLaunchKernelGGL(kern, grid, block, 0, (hipStream_t)stream, __VA_ARGS__);            \
        const hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess) { g_last_error = e_; return SD_ERR_LAUNCH; }                    \
    } while (0)

// errors left behind by earlier, unrelated runtime calls must not be blamed on our launches
inline void clear_stale_error() { (void)hipGetLastError(); }

template <int DT>
int32_t launch_stats_dt(const sd::Plan& P, bool fast, int slot_lo, int slot_cnt, void* stream) {
    const dim3 grid(P.n_chunks, P.B * slot_cnt);
    if (fast) SD_LAUNCH((k_stats<DT, true>), grid, dim3(kThreads), stream, P, slot_lo, slot_cnt);
    else SD_LAUNCH((k_stats<DT, false>), grid, dim3(kThreads), stream, P, slot_lo, slot_cnt);
    return SD_OK;
}

int32_t launch_stats_group(const sd::Plan& P, int dt, bool fast, int slot_lo, int slot_cnt, void* stream) {
    if (slot_cnt <= 0) return SD_OK;
    if (dt == SD_BF16) return launch_stats_dt<SD_BF16>(P, fast, slot_lo, slot_cnt, stream);
    if (dt == SD_F32) return launch_stats_dt<SD_F32>(P, fast, slot_lo, slot_cnt, stream);
    return launch_stats_dt<SD_F16>(P, fast, slot_lo, slot_cnt, stream);
}

template <int TDT, int DDT>
int32_t launch_resample_dd(const sd::Plan& P, void* stream) {
    const dim3 grid(P.rn_chunks, P.B);
    // FAST: T == 1 and no top-k / nucleus mask on either side (the engine rule, plain softmax)
    const bool fast = P.tT == 1.0f && P.dT == 1.0f && !P.t_keep && !P.d_keep;
    if (P.noise.mode == SD_NOISE_STREAM) {
        if (fast) SD_LAUNCH((k_resample<TDT, DDT, SD_NOISE_STREAM, false, 8, true>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_resample<TDT, DDT, SD_NOISE_STREAM, false, 8, false>), grid, dim3(kThreads), stream, P);
    } else {
        if (fast) SD_LAUNCH((k_resample<TDT, DDT, SD_NOISE_PHILOX, true, 8, true>), grid, dim3(kThreads), stream, P);
        else SD_LAUNCH((k_resample<TDT, DDT, SD_NOISE_PHILOX, true, 8, false>), grid, dim3(kThreads), stream, P);
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
    if (P.noise.mode == SD_NOISE_STREAM) SD_LAUNCH((k_rowsample<DT, SD_NOISE_STREAM, 8>), grid, dim3(kThreads), stream, P);
    else SD_LAUNCH((k_rowsample<DT, SD_NOISE_PHILOX, 8>), grid, dim3(kThreads), stream, P);
    return SD_OK;
}

int32_t launch_rowsample(const sd::Plan& P, void* stream) {
    if (P.tdt == SD_BF16) return launch_rowsample_dt<SD_BF16>(P, stream);
    if (P.tdt == SD_F32) return launch_rowsample_dt<SD_F32>(P, stream);
    return launch_rowsample_dt<SD_F16>(P, stream);
}

// Row statistics for every slot: one launch when target and drafter rows share a dtype.
int32_t launch_stats(const sd::Plan& P, void* stream) {
    const bool t_fast = P.tT == 1.0f && !P.t_keep, d_fast = P.dT == 1.0f && !P.d_keep;
    if (P.n_dslots == 0 || (P.tdt == P.ddt && t_fast == d_fast))
        return launch_stats_group(P, P.tdt, t_fast, 0, P.slots, stream);
    if (int32_t st = launch_stats_group(P, P.tdt, t_fast, 0, P.n_tslots, stream)) return st;
    return launch_stats_group(P, P.ddt, d_fast, P.n_tslots, P.n_dslots, stream);
}

}  // namespace

extern "C" {

int32_t sd_abi_version(void) { return SD_ABI_VERSION; }

const char* sd_last_hip_error(void) { return hipGetErrorString(g_last_error); }

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

    Plan P{};
    P.B = a->batch; P.gamma = a->gamma; P.V = a->vocab; P.rule = a->rule;
    P.n_tslots = n_t;
    P.n_dslots = a->draft_is_probs ? 0 : a->gamma;
    P.slots = P.n_tslots + P.n_dslots;
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

    const int rows = P.B * P.slots;
    set_stats_chunks(P, rows);
    Carve c{static_cast<char*>(a->workspace)};
    carve(P, c, a->batch * (2 * a->gamma + 1), a->batch, a->gamma, a->vocab);

    if (P.t_keep || P.d_keep) {
        const int32_t st = launch_threshold(P, a->target_proc, a->draft_proc, stream);
        if (st != SD_OK) return st;
    }
    set_rchunks(P);
    if (const char* e = getenv("SD_DIAG")) P.diag = atoi(e);
    if (a->prof_stats_begin) (void)hipEventRecord((hipEvent_t)a->prof_stats_begin, (hipStream_t)stream);
    if (int32_t st = launch_stats(P, stream)) return st;
    if (a->prof_stats_end) (void)hipEventRecord((hipEvent_t)a->prof_stats_end, (hipStream_t)stream);
    if (P.noise.mode == SD_NOISE_STREAM) {   // parity mode: the reference's serial noise order
        SD_LAUNCH(k_decide, dim3(P.B), dim3(256), stream, P);
        SD_LAUNCH(k_walk, dim3(1), dim3(256), stream, P);
    }
    if (int32_t st = launch_resample(P, stream)) return st;
    SD_LAUNCH(k_finalize, dim3(P.B), dim3(64), stream, P);
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
    P.n_tslots = 1; P.n_dslots = 0; P.slots = 1;
    P.tdt = a->dtype; P.ddt = a->dtype;
    P.t_keep = needs_keep(a->proc); P.t_stoch = a->proc.kind != SD_PROC_GREEDY;
    P.tT = a->proc.temperature; P.dT = 1.f;
    P.trow[0] = a->logits; P.tstride = a->stride_r;
    P.noise = a->noise;
    P.next_token = a->tokens; P.next_token_stride = a->tokens_stride;
    P.token_prob = a->token_prob; P.row_status = a->row_status; P.words_used = a->words_used;
    set_stats_chunks(P, P.B);
    Carve c{static_cast<char*>(a->workspace)};
    carve(P, c, a->rows, a->rows, 1, a->vocab);
    if (P.t_keep) {
        const int32_t st = launch_threshold(P, a->proc, a->proc, stream);
        if (st != SD_OK) return st;
    }
    set_rchunks(P);
    if (int32_t st = launch_stats(P, stream)) return st;
    if (int32_t st = launch_rowsample(P, stream)) return st;
    SD_LAUNCH(k_sample_finalize, dim3(P.B), dim3(64), stream, P);
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
    P.n_tslots = 1; P.n_dslots = 0; P.slots = 1;
    P.tdt = a->dtype; P.ddt = a->dtype;
    P.t_keep = needs_keep(a->proc);
    P.tT = a->proc.temperature; P.dT = 1.f;
    P.trow[0] = a->logits; P.tstride = a->stride_r;
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
