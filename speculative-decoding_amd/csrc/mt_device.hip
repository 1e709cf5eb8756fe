// mt_device.hip — torch's CPU generator (ATen mt19937) run on the GPU: the STREAM noise words the
// verify / sample kernels consume, bit-identical to what torch.rand / torch.multinomial draw on
// the host under torch.manual_seed (the reference's noise), without the single host thread.
//
// The generator's untempered sequence obeys x[k+624] = x[k+397] ^ mag(upper(x[k]) | lower(x[k+1]))
// and is consumed from position tau0 of the current 624-word block (sd_mt_state).  A fill of n
// words is cut into substreams of `stride` words; substream s starts at x[tau0 + s*stride],
// reached by a jump-ahead polynomial c_s (csrc/mt_jump.cpp):
//     W(tau0 + s*stride) = XOR over i in c_s of W(tau0 + 1 + i),     W(m) = x[m .. m+623],
// so every start is a GF(2) combination of windows of ONE base sequence.  Three launches:
//   k_mt_base  one workgroup: the untempered x[0 .. 21760) from the block (an LDS ring, 2 words
//              per thread per barrier: position q depends on q-227 — the thread's own previous
//              word — and on q-624 / q-623, made before the last barrier);
//   k_mt_jump  (substream, bit chunk) per wave: 640 window words per wave, 10 per lane in a
//              rotating register window that slides one position per polynomial bit (one LDS
//              word per lane per bit, the layout transposed mod 10 so the reads are
//              conflict-free), XORed into 10 accumulators when the bit is set; partial windows
//              per chunk go to the workspace;
//   k_mt_gen   one workgroup per substream: XOR the chunk partials (substream 0 reads its window
//              from the base), then run the recurrence, tempering into the output.
// k_mt_commit moves the state past the words a consumer used (a count on the host, or the
// words_used a verify kernel wrote on the device — no host sync).  Integer work, HBM-light:
// the output words are written once (4 B each) and read once by the consumer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "specdec.h"

namespace {

constexpr int kN = 624, kM = 397, kLag = kN - kM;         // 227 = largest independent batch
constexpr int kJW = SD_MT_JUMP_WORDS;                      // 320 u64 per jump polynomial
constexpr int kJBits = kJW * 64;                           // 20480 coefficient slots (>= 19937)
constexpr int kBaseLen = kN + 1 + kJBits + 640 + 15;       // 21760: covers tau0 + 1 + i + j
constexpr int kRing = 2048;
constexpr int kK = 10;                                     // window words per lane in k_mt_jump

// A workgroup barrier for LDS hand-offs only.  __syncthreads() also orders the threads' GLOBAL
// stores at workgroup scope, i.e. waits for every output store of the round to be acknowledged
// (vmcnt(0)) before the barrier — ~1000 cycles per recurrence round in k_mt_gen, whose rounds only
// exchange words through LDS.  Here: LDS operations complete (lgkmcnt(0)), then s_barrier; the
// "memory" clobber keeps the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ uint32_t mag(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// (s & k) ^ y in one v_bitop3_b32 (truth table 0x6c over (s, y, k)); k lives in an SGPR
__device__ __forceinline__ uint32_t and_xor(uint32_t s, uint32_t y, uint32_t k) {
    return __builtin_amdgcn_bitop3_b32(s, y, k, 0x6c);
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y = and_xor(y << 7, y, 0x9d2c5680u);
    y = and_xor(y << 15, y, 0xefc60000u);
    y ^= (y >> 18);
    return y;
}

// x[q-681] ^ mag(a0, b0) ^ mag(a1, b1) ^ mag(a2, b2) with the three mags folded together: the
// shifted halves XOR linearly, (upper(A) | lower(B)) >> 1 with A, B the XORs of the a's and b's,
// and the matrix term is taken once on the parity of the b's low bits (bit 0 of that same word).
// Seven VALU operations for the round's word instead of ~20.
__device__ __forceinline__ uint32_t mag3(uint32_t c, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                                         uint32_t a2, uint32_t b2) {
    const uint32_t A = __builtin_amdgcn_bitop3_b32(a0, a1, a2, 0x96);           // a0 ^ a1 ^ a2
    const uint32_t B = __builtin_amdgcn_bitop3_b32(b0, b1, b2, 0x96);
    const uint32_t Y = __builtin_amdgcn_bitop3_b32(A, B, 0x80000000u, 0xe4);   // upper(A) | lower(B)
    const uint32_t m = (uint32_t)((int32_t)(Y << 31) >> 31);                    // -(Y & 1)
    return and_xor(m, (Y >> 1) ^ c, 0x9908b0dfu);
}

__device__ __forceinline__ uint32_t untemper(uint32_t y) {
    y ^= y >> 18;
    y ^= (y << 15) & 0xefc60000u;
    uint32_t t = y;
#pragma unroll
    for (int i = 0; i < 4; ++i) t = y ^ ((t << 7) & 0x9d2c5680u);
    y = t;
#pragma unroll
    for (int i = 0; i < 2; ++i) t = y ^ (t >> 11);
    return t;
}

// ---------------------------------------------------------------------------------- recurrence
// Unrolling the recurrence three times,
//     x[q] = x[q-681] ^ F(q-1078) ^ F(q-851) ^ F(q-624),      F(p) = mag(x[p], x[p+1]),
// every input of position q is at least 623 positions back: the 623 positions of a round are
// independent, one barrier per round (the plain recurrence makes 454 per barrier, two of them
// chained in each thread).  The LDS ring is double-mapped — x[q] at r[q & 2047] and
// r[(q & 2047) + 2048] — so a round's seven reads are one base address plus immediate offsets.
// Reads cover [q0 - 1078, q0), writes [q0, q0 + 623): disjoint modulo 2048, hence one barrier.
constexpr int kBlk = kN - 1;           // 623 positions per round
constexpr int kMtThreads = 640;        // 10 waves: a round's 623 positions, one per thread
constexpr int kBack = 1078;            // the oldest input of a round, q - 1078

__device__ __forceinline__ void ring_put(uint32_t* r, int q, uint32_t x) {
    const int i = q & (kRing - 1);
    r[i] = x;
    r[i + kRing] = x;
}

// Extend the ring holding x[0 .. 624) to x[len), calling out(q, x) for q in [624, len).  Whole
// workgroup of kMtThreads; the caller put x[0 .. 624) in the ring and synchronised.  Positions are
// 32-bit (a substream is at most a few million words): the round's index math stays in one VGPR.
template <typename Out>
__device__ __forceinline__ void mt_extend(uint32_t* r, int len, Out out) {
    const int t = threadIdx.x;
    // [624, 1078): the plain recurrence, one round of two chained positions per thread
    if (t < kLag) {
        const int q1 = kN + t, q2 = q1 + kLag;
        const uint32_t x1 = r[kM + t] ^ mag(r[t], r[t + 1]);
        const uint32_t x2 = x1 ^ mag(r[q2 - kN], r[q2 - kN + 1]);
        ring_put(r, q1, x1);
        ring_put(r, q2, x2);
        out(q1, x1);
        out(q2, x2);
    }
    lds_barrier();
    const bool act = t < kBlk;
    for (int q0 = kBack, q = kBack + t; q0 < len; q0 += kBlk, q += kBlk) {
        if (act) {
            const uint32_t* b = r + (q & (kRing - 1)) + kRing - kBack;   // b[k] = x[q - 1078 + k]
            const uint32_t x = mag3(b[397], b[0], b[1], b[227], b[228], b[454], b[455]);
            ring_put(r, q, x);
            out(q, x);
        }
        lds_barrier();
    }
}

// ---------------------------------------------------------------------------------------- base
__global__ void __launch_bounds__(kMtThreads) k_mt_base(const sd_mt_state* __restrict__ st, uint32_t* __restrict__ base) {
    __shared__ uint32_t ring[2 * kRing];
    const int t = threadIdx.x;
    if (t < kN) {
        const uint32_t w = st->mt[t];
        ring_put(ring, t, w);
        base[t] = w;
    }
    __syncthreads();
    mt_extend(ring, kBaseLen, [&](int q, uint32_t x) {
        if (q < kBaseLen) base[q] = x;
    });
}

// ---------------------------------------------------------------------------------------- jump
// grid (chunk, substream-1); one wave.  Chunk ch covers polynomial bits [ch*I, ch*I + I).
template <int I>
__global__ void __launch_bounds__(64) k_mt_jump(const sd_mt_state* __restrict__ st, const uint32_t* __restrict__ base,
                                                const uint64_t* __restrict__ table, uint32_t* __restrict__ partial) {
    static_assert(I % kK == 0 && kJBits % I == 0, "chunking");
    constexpr int kSeg = I + 64 * kK + kK;                 // base words a chunk touches
    constexpr int kStr = kSeg / kK + 1;
    __shared__ uint32_t seg[kK * kStr];                    // seg word m at [(m % 10) * kStr + m / 10]
    const int ch = blockIdx.x, s = blockIdx.y + 1, nch = gridDim.x;
    const int l = threadIdx.x;
    const int tau0 = st->tau0;
    const int i0 = ch * I;
    const uint32_t* src = base + tau0 + 1 + i0;            // seg[m] = x[tau0 + 1 + i0 + m]
    for (int m = l; m < kSeg; m += 64) seg[(m % kK) * kStr + m / kK] = src[m];
    __syncthreads();
    uint32_t ring[kK], acc[kK];
#pragma unroll
    for (int k = 0; k < kK; ++k) {
        ring[k] = seg[k * kStr + l];                       // seg[10 l + k]
        acc[k] = 0u;
    }
    const uint64_t* c = table + (size_t)(s - 1) * kJW;
    for (int blk = 0; blk < I / kK; ++blk) {
        const int i = i0 + blk * kK;                       // bits i .. i+9 (never straddle 3 words)
        const uint64_t w0 = c[i >> 6];
        const uint64_t w1 = (i & 63) > 64 - kK ? c[(i >> 6) + 1] : 0ull;
        const uint32_t bits = (uint32_t)(((w0 >> (i & 63)) | ((i & 63) ? (w1 << (64 - (i & 63))) : 0ull)) & 0x3ffu);
#pragma unroll
        for (int tt = 0; tt < kK; ++tt) {
            if ((bits >> tt) & 1u) {
#pragma unroll
                for (int r = 0; r < kK; ++r) acc[r] ^= ring[(tt + r) % kK];
            }
            ring[tt] = seg[tt * kStr + blk + 1 + l];       // seg[10 (blk + 1) + 10 l + tt]
        }
    }
    uint32_t* out = partial + ((size_t)(s - 1) * nch + ch) * kN;
#pragma unroll
    for (int r = 0; r < kK; ++r) {
        const int j = kK * l + r;
        if (j < kN) out[j] = acc[r];
    }
}

// ----------------------------------------------------------------------------------------- gen
__global__ void __launch_bounds__(kMtThreads) k_mt_gen(const sd_mt_state* __restrict__ st, const uint32_t* __restrict__ base,
                                                       const uint32_t* __restrict__ partial, int /*nch: SD_MT_JUMP_CHUNKS*/, uint32_t* __restrict__ out,
                                                       int64_t n, int64_t stride) {
    __shared__ uint32_t ring[2 * kRing];
    const int s = blockIdx.x, t = threadIdx.x;
    const int64_t lo = (int64_t)s * stride;
    const int64_t len = n - lo < stride ? n - lo : stride;
    uint32_t* o = out + lo;
    if (t < kN) {
        uint32_t w;
        if (s == 0) {
            w = base[st->tau0 + t];
        } else {
            // every chunk partial in flight at once (a load -> xor loop waited for each in turn:
            // 16 dependent round trips before the first round)
            w = 0u;
            const uint32_t* p = partial + (size_t)(s - 1) * SD_MT_JUMP_CHUNKS * kN + t;
            uint32_t pv[SD_MT_JUMP_CHUNKS];
#pragma unroll
            for (int c = 0; c < SD_MT_JUMP_CHUNKS; ++c) pv[c] = p[(size_t)c * kN];
#pragma unroll
            for (int c = 0; c < SD_MT_JUMP_CHUNKS; ++c) w ^= pv[c];
        }
        ring_put(ring, t, w);
        if (t < len) o[t] = temper(w);
    }
    __syncthreads();
    mt_extend(ring, (int)len, [&](int q, uint32_t x) {
        if (q < (int)len) o[(uint32_t)q] = temper(x);
    });
}

// -------------------------------------------------------------------------------------- commit
__global__ void __launch_bounds__(256) k_mt_commit(sd_mt_state* __restrict__ st, const uint32_t* __restrict__ words,
                                                   int64_t n_words, const int64_t* __restrict__ used_dev, int64_t used,
                                                   int32_t* __restrict__ status) {
    const int t = threadIdx.x;
    const int64_t u = used + (used_dev ? used_dev[0] : 0);   // host-known prefix + the device count
    const int tau0 = st->tau0;
    __syncthreads();                                       // every thread has read tau0
    if (u <= 0) return;
    const int64_t end = tau0 + u;                          // one past the last consumed position
    if (end <= kN) {                                       // still inside the current block
        if (t == 0) st->tau0 = (int)end;
        return;
    }
    const int64_t b = (end - 1) / kN;                      // block holding the last consumed word
    const int64_t first = b * kN - tau0;                   // its first word in `words`
    if (first + kN > n_words) {                            // not generated: leave the state alone
        if (t == 0 && status) atomicOr(status, 1);
        return;
    }
    for (int j = t; j < kN; j += 256) st->mt[j] = untemper(words[first + j]);
    if (t == 0) st->tau0 = (int)(end - b * kN);
}

inline bool launch_ok() { return hipGetLastError() == hipSuccess; }

}  // namespace

extern "C" {

size_t sd_mt19937_generate_workspace_size(int64_t n_words, int64_t stride_words) {
    if (n_words < 0 || stride_words < kN) return 0;
    const int64_t S = n_words > 0 ? (n_words + stride_words - 1) / stride_words : 1;
    const size_t base = ((size_t)kBaseLen * 4 + 255) & ~(size_t)255;
    return base + (size_t)(S > 1 ? S - 1 : 0) * SD_MT_JUMP_CHUNKS * kN * 4 + 256;
}

int32_t sd_mt19937_generate(const sd_mt_generate_args* a, void* stream) {
    if (!a || !a->state || (a->n_words > 0 && !a->words) || a->n_words < 0 || a->stride_words < kN ||
        a->stride_words > (int64_t)1 << 30)
        return SD_ERR_INVALID;
    if (a->n_words == 0) return SD_OK;
    const int64_t S = (a->n_words + a->stride_words - 1) / a->stride_words;
    if (S > 1 && (!a->jump_table || a->jump_count < S - 1)) return SD_ERR_INVALID;
    if (S > 65535) return SD_ERR_UNSUPPORTED;
    const size_t need = sd_mt19937_generate_workspace_size(a->n_words, a->stride_words);
    if (!a->workspace || a->workspace_bytes < need) return SD_ERR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    uint32_t* base = (uint32_t*)a->workspace;
    uint32_t* partial = (uint32_t*)((char*)a->workspace + (((size_t)kBaseLen * 4 + 255) & ~(size_t)255));
    hipLaunchKernelGGL(k_mt_base, dim3(1), dim3(kMtThreads), 0, s, a->state, base);
    if (!launch_ok()) return SD_ERR_LAUNCH;
    if (S > 1) {
        hipLaunchKernelGGL((k_mt_jump<kJBits / SD_MT_JUMP_CHUNKS>), dim3(SD_MT_JUMP_CHUNKS, (unsigned)(S - 1)), dim3(64),
                           0, s, a->state, base, a->jump_table, partial);
        if (!launch_ok()) return SD_ERR_LAUNCH;
    }
    hipLaunchKernelGGL(k_mt_gen, dim3((unsigned)S), dim3(kMtThreads), 0, s, a->state, base, partial, SD_MT_JUMP_CHUNKS,
                       a->words, a->n_words, a->stride_words);
    return launch_ok() ? SD_OK : SD_ERR_LAUNCH;
}

int32_t sd_mt19937_commit(sd_mt_state* state, const uint32_t* words, int64_t n_words, const int64_t* used_dev,
                          int64_t used, int32_t* status, void* stream) {
    if (!state || n_words < 0 || (n_words > 0 && !words) || used < 0) return SD_ERR_INVALID;
    hipLaunchKernelGGL(k_mt_commit, dim3(1), dim3(256), 0, (hipStream_t)stream, state, words, n_words, used_dev, used,
                       status);
    return launch_ok() ? SD_OK : SD_ERR_LAUNCH;
}

}  // extern "C"
