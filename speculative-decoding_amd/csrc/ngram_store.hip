// Device-resident n-gram drafter store: the reference's
// OneLevelNGramStorage / NGramStorage (ngram_assisted/ngram_storage.py:71-249) as two open-
// addressing hash tables in HBM, updated and queried by kernels, so a batch of histories is
// recorded in two launches instead of a Python loop over every position and gram order.
//
// The reference's rule (ngram_storage.py:118-125, 131-138, 207-216, 232-241): a gram's best token
// starts as the first token recorded for it and changes only when another token's count becomes
// STRICTLY larger than the best's.  So the best always holds the running maximum count, and it is
// the token that FIRST reached the final maximum.  With every record stamped by its position ts in
// the reference's processing order, a token reached its current count at its latest record, so
//     best = argmax over the gram's tokens of (count, -latest ts)
// which no longer depends on the order the records are applied in.  A batch of records is applied
// in two launches: (1) every record inserts its gram and (gram, token) pair, adds 1 to the pair's
// count and raises the pair's latest ts; (2) every record re-reads its pair and raises the gram's
// packed (count, ~ts, token) key with one 64-bit atomicMax.  Keys only grow (counts only grow), so
// pairs untouched by a batch keep their earlier contribution.
//
// Layout (caller-owned device memory, zero-filled once; sd_ngram_store in specdec.h):
//   gram table: key u64 = 1<<63 | level<<51 | t0 | t1<<17 | t2<<34 (a gram is 1..3 token ids of
//               17 bits, level = its order j, so the orders of NGramStorage share one table);
//               best u64 = count<<44 | (2^27-1-ts)<<17 | token
//   pair table: key u64 = 1<<63 | gram_slot<<17 | token; count u32; latest ts u32
// Linear probing from a splitmix64 hash; 0 = empty.  A full table sets SD_NGRAM_FULL in *status.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "specdec.h"

namespace {

constexpr int kThreads = 256;
constexpr uint64_t kUsed = 1ull << 63;
constexpr uint32_t kTokBits = 17, kTokMask = (1u << kTokBits) - 1;
constexpr uint64_t kTsMax = (1ull << 27) - 1;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// key of the gram seq[e - j .. e) of order j (1 <= j <= 3); false if a token is out of range
__device__ __forceinline__ bool gram_key(const int64_t* seq, int64_t e, int j, int level, uint64_t& key) {
    uint64_t k = kUsed | ((uint64_t)level << 51);
    for (int t = 0; t < j; ++t) {
        const int64_t v = seq[e - j + t];
        if (v < 0 || v > (int64_t)kTokMask) return false;
        k |= (uint64_t)v << (kTokBits * t);
    }
    key = k;
    return true;
}

// gram_key over the last j of C register-held ids (ctx[C-1] newest): static indices only, so
// the ids stay in registers (a runtime index into ctx[] put them in scratch)
template <int C>
__device__ __forceinline__ bool gram_key_ctx(const int64_t (&ctx)[C], int j, uint64_t& key) {
    uint64_t k = kUsed | ((uint64_t)j << 51);
    bool ok = true;
#pragma unroll
    for (int t = 0; t < C; ++t) {
        if (t >= C - j) {
            const int64_t v = ctx[t];
            ok &= v >= 0 && v <= (int64_t)kTokMask;
            k |= (uint64_t)(v & kTokMask) << (kTokBits * (t - (C - j)));
        }
    }
    key = k;
    return ok;
}

// slot of key (inserted when absent if INSERT), -1 when absent (lookup) or the table is full
template <bool INSERT>
__device__ __forceinline__ int64_t probe(uint64_t* keys, int64_t cap, uint64_t key, int32_t* status) {
    int64_t s = (int64_t)(mix64(key) & (uint64_t)(cap - 1));
    for (int64_t n = 0; n < cap; ++n) {
        uint64_t cur = __hip_atomic_load(keys + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == key) return s;
        if (cur == 0) {
            if (!INSERT) return -1;
            cur = atomicCAS((unsigned long long*)(keys + s), 0ull, (unsigned long long)key);
            if (cur == 0 || cur == key) return s;
        }
        s = (s + 1) & (cap - 1);
    }
    if (INSERT) atomicOr(status, SD_NGRAM_FULL);
    return -1;
}

struct Rec {
    bool ok;
    const int64_t* seq;
    int64_t end;    // the gram is seq[end - j .. end)
    int j;
    int64_t token;
    uint32_t ts;
};

// Record r of an initialize (ngram_storage.py:128-142 one-level, 227-243 all orders):
// r = (b * len + i) * n_orders + o, the token at position i after the gram of order j ending there.
__device__ __forceinline__ Rec init_rec(const sd_ngram_store& S, const int64_t* ids, int64_t len, int64_t stride,
                                        int64_t ts_base, int64_t r) {
    Rec R{};
    const int n_orders = S.one_level ? 1 : S.n - 2;
    const int64_t o = r % n_orders, bi = r / n_orders, i = bi % len, b = bi / len;
    R.j = S.one_level ? S.n - 1 : 2 + (int)o;
    // one level: positions i >= n-1; all orders: j <= min(n-1, i)
    R.ok = i >= R.j;
    R.seq = ids + b * stride;
    R.end = i;
    R.token = R.seq[i];
    R.ts = (uint32_t)(ts_base + bi);
    return R;
}

// Record r of an update (ngram_storage.py:106-126, 196-217): next_tokens[b, k] after the gram of
// order j ending the history; r = (b * n_orders + o) * k_tok + k
__device__ __forceinline__ Rec update_rec(const sd_ngram_store& S, const int64_t* ids, int64_t len, int64_t stride,
                                          const int64_t* next, int64_t k_tok, int64_t nstride, int64_t ts_base,
                                          int64_t r) {
    Rec R{};
    const int n_orders = S.one_level ? 1 : S.n - 2;
    const int64_t k = r % k_tok, bo = r / k_tok, o = bo % n_orders, b = bo / n_orders;
    R.j = S.one_level ? S.n - 1 : 2 + (int)o;
    // one level: skipped when len < n (:109-110); all orders: j <= min(n-1, len)
    R.ok = S.one_level ? len >= S.n : R.j <= len;
    R.seq = ids + b * stride;
    R.end = len;
    R.token = next[b * nstride + k];
    R.ts = (uint32_t)(ts_base + b * k_tok + k);
    return R;
}

template <int PHASE>
__device__ __forceinline__ void apply(const sd_ngram_store& S, const Rec& R) {
    if (!R.ok) return;
    uint64_t gk;
    if (!gram_key(R.seq, R.end, R.j, R.j, gk) || R.token < 0 || R.token > (int64_t)kTokMask) {
        atomicOr(S.status, SD_NGRAM_BAD_TOKEN);
        return;
    }
    const int64_t gs = probe<PHASE == 1>(S.gram_keys, S.gram_capacity, gk, S.status);
    if (gs < 0) return;
    const uint64_t pk = kUsed | ((uint64_t)gs << kTokBits) | (uint64_t)R.token;
    const int64_t ps = probe<PHASE == 1>(S.pair_keys, S.pair_capacity, pk, S.status);
    if (ps < 0) return;
    if (PHASE == 1) {
        atomicAdd(S.pair_count + ps, 1u);
        atomicMax(S.pair_ts + ps, R.ts);
    } else {
        const uint64_t cnt = S.pair_count[ps], ts = S.pair_ts[ps];
        const uint64_t packed = (cnt << 44) | ((kTsMax - ts) << kTokBits) | (uint64_t)R.token;
        atomicMax((unsigned long long*)(S.gram_best + gs), (unsigned long long)packed);
    }
}

template <int PHASE>
__global__ void __launch_bounds__(kThreads) k_ng_init(sd_ngram_store S, const int64_t* ids, int64_t len, int64_t stride,
                                                      int64_t ts_base, int64_t n_rec) {
    const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (r < n_rec) apply<PHASE>(S, init_rec(S, ids, len, stride, ts_base, r));
}

template <int PHASE>
__global__ void __launch_bounds__(kThreads) k_ng_update(sd_ngram_store S, const int64_t* ids, int64_t len, int64_t stride,
                                                        const int64_t* next, int64_t k_tok, int64_t nstride,
                                                        int64_t ts_base, int64_t n_rec) {
    const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (r < n_rec) apply<PHASE>(S, update_rec(S, ids, len, stride, next, k_tok, nstride, ts_base, r));
}

// next_token (ngram_storage.py:76-90, 162-177): the longest known order's best token; out[b] holds
// the caller's fallback draw and is overwritten only for a known gram
__global__ void __launch_bounds__(kThreads) k_ng_next(sd_ngram_store S, const int64_t* ids, int32_t batch, int64_t len,
                                                      int64_t stride, int64_t* out, uint8_t* known) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= batch) return;
    const int64_t* seq = ids + (int64_t)b * stride;
    int hi, lo;
    if (S.one_level) hi = lo = len >= S.n - 1 ? S.n - 1 : 0;
    else { hi = (int)(len < S.n - 1 ? len : S.n - 1); lo = 2; }
    uint8_t kn = 0;
    for (int j = hi; j >= lo && j >= 1; --j) {
        uint64_t gk;
        if (!gram_key(seq, len, j, j, gk)) break;
        const int64_t gs = probe<false>(S.gram_keys, S.gram_capacity, gk, S.status);
        if (gs < 0) continue;
        const uint64_t best = S.gram_best[gs];
        if (best == 0) continue;
        out[b] = (int64_t)(best & kTokMask);
        kn = 1;
        break;
    }
    known[b] = kn;
}

// The n-gram loop's drafting (ngram_assisted/ngram_assisted.py:94-101): gamma chained next_token
// calls, each on the history extended by the previous drafts, in one thread per history: the
// last n-1 ids ride in registers.  fallback[b, k] = the k-th call's torch.randint draw.  Every
// draft is produced (the caller truncates at the first unknown for stop_if_unknown).
__global__ void __launch_bounds__(kThreads) k_ng_draft(sd_ngram_store S, const int64_t* ids, int32_t batch, int64_t len,
                                                       int64_t stride, int32_t gamma, const int64_t* fallback,
                                                       int64_t fstride, int64_t* drafts, int64_t dstride,
                                                       uint8_t* known) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= batch) return;
    const int64_t* seq = ids + (int64_t)b * stride;
    int64_t ctx[SD_NGRAM_MAX_N - 1];   // ctx[SD_NGRAM_MAX_N - 2] = newest id
    constexpr int C = SD_NGRAM_MAX_N - 1;
#pragma unroll
    for (int t = 0; t < C; ++t) ctx[t] = len - C + t >= 0 ? seq[len - C + t] : -1;
    for (int k = 0; k < gamma; ++k) {
        const int64_t L = len + k;
        int hi, lo;
        if (S.one_level) hi = lo = L >= S.n - 1 ? S.n - 1 : 0;
        else { hi = (int)(L < S.n - 1 ? L : S.n - 1); lo = 2; }
        int64_t tok = fallback[(int64_t)b * fstride + k];
        uint8_t kn = 0;
        for (int j = hi; j >= lo && j >= 1; --j) {
            uint64_t gk;
            if (!gram_key_ctx(ctx, j, gk)) break;
            const int64_t gs = probe<false>(S.gram_keys, S.gram_capacity, gk, S.status);
            if (gs < 0) continue;
            const uint64_t best = S.gram_best[gs];
            if (best == 0) continue;
            tok = (int64_t)(best & kTokMask);
            kn = 1;
            break;
        }
        drafts[(int64_t)b * dstride + k] = tok;
        known[(int64_t)b * gamma + k] = kn;
#pragma unroll
        for (int t = 0; t + 1 < C; ++t) ctx[t] = ctx[t + 1];
        ctx[C - 1] = tok;
    }
}

// has_gram (ngram_storage.py:92-102, 179-194): the gram is the LAST j ids of the n-gram, its last
// token included, as in the reference; true if that token was recorded after it
__global__ void k_ng_has(sd_ngram_store S, const int64_t* ngram, int64_t len, uint8_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint8_t res = 0;
    int hi, lo;
    if (S.one_level) {
        hi = lo = S.n - 1;
        if (len < S.n) hi = 0;
    } else {
        hi = (int)(len < S.n - 1 ? len : S.n - 1);
        lo = 2;
    }
    const int64_t last = len > 0 ? ngram[len - 1] : -1;
    for (int j = hi; j >= lo && j >= 1 && !res; --j) {
        uint64_t gk;
        if (!gram_key(ngram, len, j, j, gk) || last < 0 || last > (int64_t)kTokMask) break;
        const int64_t gs = probe<false>(S.gram_keys, S.gram_capacity, gk, S.status);
        if (gs < 0) continue;
        const uint64_t pk = kUsed | ((uint64_t)gs << kTokBits) | (uint64_t)last;
        res = probe<false>(S.pair_keys, S.pair_capacity, pk, S.status) >= 0;
    }
    *out = res;
}

bool valid_store(const sd_ngram_store* s) {
    if (!s || !s->gram_keys || !s->gram_best || !s->pair_keys || !s->pair_count || !s->pair_ts || !s->status)
        return false;
    auto pow2 = [](int64_t c) { return c > 0 && (c & (c - 1)) == 0; };
    if (!pow2(s->gram_capacity) || !pow2(s->pair_capacity) || s->gram_capacity > (1ll << 40)) return false;
    if (s->n < 2 || s->n > SD_NGRAM_MAX_N || s->vocab < 1 || s->vocab > (1 << kTokBits)) return false;
    return true;
}

int64_t blocks(int64_t n) { return (n + kThreads - 1) / kThreads; }

int32_t launched() { return hipGetLastError() == hipSuccess ? SD_OK : SD_ERR_LAUNCH; }

}  // namespace

extern "C" {

int32_t sd_ngram_store_initialize(const sd_ngram_store* s, const int64_t* ids, int32_t batch, int32_t len,
                                  int64_t stride_b, int64_t ts_base, void* stream) {
    if (!valid_store(s) || batch < 0 || len < 0 || (batch && len && !ids) || ts_base < 0) return SD_ERR_INVALID;
    const int n_orders = s->one_level ? 1 : s->n - 2;
    const int64_t n_rec = (int64_t)batch * len * n_orders;
    if (ts_base + (int64_t)batch * len > (int64_t)kTsMax) return SD_ERR_UNSUPPORTED;
    if (n_rec == 0) return SD_OK;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL((k_ng_init<1>), dim3(blocks(n_rec)), dim3(kThreads), 0, st, *s, ids, (int64_t)len, stride_b, ts_base, n_rec);
    hipLaunchKernelGGL((k_ng_init<2>), dim3(blocks(n_rec)), dim3(kThreads), 0, st, *s, ids, (int64_t)len, stride_b, ts_base, n_rec);
    return launched();
}

int32_t sd_ngram_store_update(const sd_ngram_store* s, const int64_t* ids, int32_t batch, int32_t len, int64_t stride_b,
                              const int64_t* next_tokens, int32_t k, int64_t next_stride_b, int64_t ts_base,
                              void* stream) {
    if (!valid_store(s) || batch < 0 || len < 0 || k < 1 || (batch && (!next_tokens || (len && !ids))) || ts_base < 0)
        return SD_ERR_INVALID;
    const int n_orders = s->one_level ? 1 : s->n - 2;
    const int64_t n_rec = (int64_t)batch * n_orders * k;
    if (ts_base + (int64_t)batch * k > (int64_t)kTsMax) return SD_ERR_UNSUPPORTED;
    if (n_rec == 0) return SD_OK;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL((k_ng_update<1>), dim3(blocks(n_rec)), dim3(kThreads), 0, st, *s, ids, (int64_t)len, stride_b,
                       next_tokens, (int64_t)k, next_stride_b, ts_base, n_rec);
    hipLaunchKernelGGL((k_ng_update<2>), dim3(blocks(n_rec)), dim3(kThreads), 0, st, *s, ids, (int64_t)len, stride_b,
                       next_tokens, (int64_t)k, next_stride_b, ts_base, n_rec);
    return launched();
}

int32_t sd_ngram_store_next_token(const sd_ngram_store* s, const int64_t* ids, int32_t batch, int32_t len,
                                  int64_t stride_b, int64_t* out, uint8_t* known, void* stream) {
    if (!valid_store(s) || batch < 0 || len < 0 || (batch && (!out || !known || (len && !ids)))) return SD_ERR_INVALID;
    if (batch == 0) return SD_OK;
    hipLaunchKernelGGL(k_ng_next, dim3(blocks(batch)), dim3(kThreads), 0, (hipStream_t)stream, *s, ids, batch,
                       (int64_t)len, stride_b, out, known);
    return launched();
}

int32_t sd_ngram_store_draft(const sd_ngram_store* s, const int64_t* ids, int32_t batch, int32_t len, int64_t stride_b,
                             int32_t gamma, const int64_t* fallback, int64_t fallback_stride_b, int64_t* drafts,
                             int64_t drafts_stride_b, uint8_t* known, void* stream) {
    if (!valid_store(s) || batch < 0 || len < 0 || gamma < 0 ||
        (batch && gamma && (!fallback || !drafts || !known || (len && !ids))))
        return SD_ERR_INVALID;
    if (batch == 0 || gamma == 0) return SD_OK;
    hipLaunchKernelGGL(k_ng_draft, dim3(blocks(batch)), dim3(kThreads), 0, (hipStream_t)stream, *s, ids, batch,
                       (int64_t)len, stride_b, gamma, fallback, fallback_stride_b, drafts, drafts_stride_b, known);
    return launched();
}

int32_t sd_ngram_store_has_gram(const sd_ngram_store* s, const int64_t* ngram, int32_t len, uint8_t* out, void* stream) {
    if (!valid_store(s) || len < 0 || !out || (len && !ngram)) return SD_ERR_INVALID;
    hipLaunchKernelGGL(k_ng_has, dim3(1), dim3(64), 0, (hipStream_t)stream, *s, ngram, (int64_t)len, out);
    return launched();
}

}  // extern "C"
