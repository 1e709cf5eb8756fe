// sd_device.h — device helpers shared by the specdec kernels (gfx950 / CDNA4, wave64).
//
// Numerics mirror torch-CPU semantics of the reference's ops:
//   * `logits / T`            -> round_dt(float(x) / float(T))      (true IEEE division)
//   * `softmax` in dtype      -> round_dt(exp(y - M) / S), fp32 internals
//   * `multinomial(p, 1)`     -> argmax(round_dt(p / round_dt(E))), E ~ Exp(1), first max wins
//   * torch.rand (fp32)       -> (w & 0xFFFFFF) * 2^-24 from one mt19937 word
//   * exponential_            -> float(-log1p(-u53)), u53 from two words (hi first)
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "specdec.h"

namespace sd {

constexpr int kWave = 64;
constexpr int kThreads = 256;            // 4 waves per workgroup
constexpr float kNegFill = -1e20f;       // utils/logits_processor.py:62,79

// ---------------------------------------------------------------- dtype handling
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ float round_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return __uint_as_float(u | 0x00400000u);  // NaN stays NaN
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    return __uint_as_float(u);
}

__device__ __forceinline__ float round_f16(float f) { return __half2float(__float2half_rn(f)); }

template <int DT>
__device__ __forceinline__ float round_dt(float f) {
    if constexpr (DT == SD_BF16) return round_bf16(f);
    else if constexpr (DT == SD_F16) return round_f16(f);
    else return f;
}

__device__ __forceinline__ float round_dyn(int dt, float f) {
    return dt == SD_BF16 ? round_bf16(f) : (dt == SD_F16 ? round_f16(f) : f);
}

template <int DT> struct Elem;
template <> struct Elem<SD_F32> { static constexpr int kVec = 4; static constexpr int kBytes = 4; };
template <> struct Elem<SD_BF16> { static constexpr int kVec = 8; static constexpr int kBytes = 2; };
template <> struct Elem<SD_F16> { static constexpr int kVec = 8; static constexpr int kBytes = 2; };

template <int DT>
__device__ __forceinline__ float load_one(const void* row, int64_t i) {
    if constexpr (DT == SD_F32) return static_cast<const float*>(row)[i];
    else if constexpr (DT == SD_BF16) return bf16_bits_to_f32(static_cast<const uint16_t*>(row)[i]);
    else return __half2float(static_cast<const __half*>(row)[i]);
}

__device__ __forceinline__ float load_dyn(int dt, const void* row, int64_t i) {
    return dt == SD_F32 ? load_one<SD_F32>(row, i)
                        : (dt == SD_BF16 ? load_one<SD_BF16>(row, i) : load_one<SD_F16>(row, i));
}

// Unpack one 16-byte vector into kVec floats.
template <int DT>
__device__ __forceinline__ void unpack16(const uint4 w, float* out) {
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
    if constexpr (DT == SD_F32) {
#pragma unroll
        for (int k = 0; k < 4; ++k) out[k] = __uint_as_float(ws[k]);
    } else if constexpr (DT == SD_BF16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            out[2 * k] = __uint_as_float(ws[k] << 16);
            out[2 * k + 1] = __uint_as_float(ws[k] & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            out[2 * k] = __half2float(__ushort_as_half((unsigned short)(ws[k] & 0xffffu)));
            out[2 * k + 1] = __half2float(__ushort_as_half((unsigned short)(ws[k] >> 16)));
        }
    }
}

// Load one 16-byte vector (kVec elements) starting at element e0, or the in-range part of it.
template <int DT>
__device__ __forceinline__ void load_vec(const void* row, int64_t e0, int vocab, bool aligned, float* out) {
    constexpr int V = Elem<DT>::kVec;
    if (aligned && e0 + V <= vocab) {
        const uint4 w = *reinterpret_cast<const uint4*>(static_cast<const char*>(row) + e0 * Elem<DT>::kBytes);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        if constexpr (DT == SD_F32) {
#pragma unroll
            for (int k = 0; k < 4; ++k) out[k] = __uint_as_float(ws[k]);
        } else if constexpr (DT == SD_BF16) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                out[2 * k] = __uint_as_float(ws[k] << 16);
                out[2 * k + 1] = __uint_as_float(ws[k] & 0xffff0000u);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                out[2 * k] = __half2float(__ushort_as_half((unsigned short)(ws[k] & 0xffffu)));
                out[2 * k + 1] = __half2float(__ushort_as_half((unsigned short)(ws[k] >> 16)));
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < V; ++k) out[k] = (e0 + k < vocab) ? load_one<DT>(row, e0 + k) : 0.f;
    }
}

// ---------------------------------------------------------------- exp
// e^x with v_exp_f32 (2^t) and the rounding error of t = x*log2(e) folded back in by FMA:
// ~1 ulp like ocml's expf but without its range/denormal branches.  Every kernel uses this
// one function, so a row's normaliser and its probabilities are computed consistently.
__device__ __forceinline__ float sd_exp(float x) {
    constexpr float kL = 1.44269502162933349609375f;       // log2(e) rounded to fp32
    constexpr float kLlo = 1.925963033500011e-08f;          // log2(e) - kL
    x = x < -1000.f ? -1000.f : x;                          // -inf -> 0 (not inf-inf = NaN); NaN stays NaN
    const float t = x * kL;
    const float err = fmaf(x, kL, -t) + x * kLlo;           // x*log2(e) - t
    const float r = __builtin_amdgcn_exp2f(t);
    return fmaf(r, err * 0.693147180559945309f, r);
}

// round_dt(num / den) with inv_den = 1/den.  bf16: the product num*inv_den is within ~2 fp32 ulp
// of the true quotient, so it rounds to the same bf16 unless its low 16 bits sit within a few
// units of the round-to-nearest-even tie (0x8000); only then is the IEEE division done.
template <int DT>
__device__ __forceinline__ float div_round(float num, float den, float inv_den) {
    if constexpr (DT == SD_BF16) {
        const float q = num * inv_den;
        const uint32_t low = __float_as_uint(q) & 0xffffu;
        if (low - 0x7ff0u > 0x20u) return round_bf16(q);
        return round_bf16(num / den);
    } else {
        return round_dt<DT>(num / den);
    }
}

// Probability p = round_dt(exp(y - m) / S), bit-exact, cheap for bf16: e' = exp2((y - m)*log2e)
// (v_exp_f32 on a once-rounded argument) is within ~48 fp32 ulp of exp(y - m) for arguments above
// -126 (no denormal results), so e'*invS rounds to the same bf16 unless its low 16 bits sit
// within 64 units of the tie; only then (and for tiny arguments) the compensated exp + IEEE
// division run.  Arguments below -1000 (masked logits) give exactly 0.
template <int DT>
__device__ __forceinline__ float prob_exact(float y, float m, float S, float invS) {
    if constexpr (DT == SD_BF16) {
        const float t = (y - m) * 1.44269502162933349609375f;
        if (t >= -126.f) {
            const float q = __builtin_amdgcn_exp2f(t) * invS;
            const uint32_t low = __float_as_uint(q) & 0xffffu;
            if (low - 0x7fc0u > 0x80u) return round_bf16(q);
        } else if (t < -1000.f) {
            return 0.f;
        }
        return round_bf16(sd_exp(y - m) / S);
    } else {
        return round_dt<DT>(sd_exp(y - m) / S);
    }
}

// ---------------------------------------------------------------- processors
// Per-row keep predicate produced by the top-k / nucleus threshold search:
// kept(j) <=> x_j > tau || (x_j == tau && j <= tie_idx).   tau=-inf, tie=INT_MAX keeps all.
struct RowKeep {
    float tau;
    int32_t tie_idx;
    int32_t flags;
    int32_t pad;
};

struct ProcParams {
    float inv_unused;
    float temperature;
    int32_t kind;
    int32_t has_keep;   // top-k / nucleus rows carry a RowKeep
};

// processed value y = round_dt(_process(x) / T)  (utils/logits_processor.py:13-15)
template <int DT>
__device__ __forceinline__ float process_value(float x, int64_t j, float T, bool has_keep, const RowKeep& keep) {
    float v = x;
    if (has_keep && !(x > keep.tau || (x == keep.tau && j <= keep.tie_idx))) v = round_dt<DT>(kNegFill);
    if (T != 1.0f) v = round_dt<DT>(v / T);
    return v;
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// torch.argmax semantics: NaN is the maximum; among equal maxima the first index wins.
__device__ __forceinline__ bool arg_better(float a, int32_t ia, float b, int32_t ib) {
    const bool na = a != a, nb = b != b;
    if (na || nb) return na && (!nb || ia < ib);
    return a > b || (a == b && ia < ib);
}

__device__ __forceinline__ void wave_argmax(float& v, int32_t& i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, kWave);
        const int32_t oi = __shfl_xor(i, o, kWave);
        if (arg_better(ov, oi, v, i)) { v = ov; i = oi; }
    }
}

// ---------------------------------------------------------------- noise
__device__ __forceinline__ float uniform_from_word(uint32_t w) {   // torch.rand fp32 (1 word)
    return (float)(w & 0xFFFFFFu) * 5.9604644775390625e-08f;          // 2^-24
}

__device__ __forceinline__ float exp1_from_words(uint32_t hi, uint32_t lo) {  // exponential_ (2 words)
    const uint64_t v = ((((uint64_t)hi) << 32) | lo) & ((1ull << 53) - 1);
    const double u = (double)v * 1.1102230246251565e-16;                        // 2^-53
    return (float)(-log1p(-u));
}

// Philox4x32-10 (Salmon et al., SC'11), counter-based: perf-mode noise.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

enum PhiloxSite : uint32_t { kSiteAccept = 1, kSiteSample = 2 };

__device__ __forceinline__ uint4 philox_block(const sd_noise& nz, uint32_t row, uint32_t site, uint32_t idx) {
    const uint4 c = make_uint4(idx, (row & 0x00ffffffu) | (site << 24), (uint32_t)nz.offset,
                               (uint32_t)(nz.offset >> 32));
    return philox4x32_10(c, make_uint2((uint32_t)nz.seed, (uint32_t)(nz.seed >> 32)));
}

// perf-mode Exp(1) from one 32-bit word: u in (0,1) at 24 bits, E = -ln(u) in fp32
__device__ __forceinline__ float exp1_from_word(uint32_t w) {
    const float u = (float)(w >> 8) * 5.9604644775390625e-08f + 2.98023223876953125e-08f;
    return -__logf(u);
}

// Exp(1) noise of element j of a sampled row.  STREAM: torch's exponential_ draw for element j
// (2 words at woff + 2j).  PHILOX: word (j & 3) of block (row, sample, j >> 2).
__device__ __forceinline__ float exp_noise(const sd_noise& nz, int64_t woff, int row, int64_t j) {
    if (nz.mode == SD_NOISE_STREAM) {
        const int64_t w = woff + 2 * j;
        if (w + 1 >= nz.n_words) return 1.f;   // overrun is flagged by the caller
        return exp1_from_words(nz.words[w], nz.words[w + 1]);
    }
    const uint4 q = philox_block(nz, (uint32_t)row, kSiteSample, (uint32_t)(j >> 2));
    const uint32_t w = (j & 3) == 0 ? q.x : (j & 3) == 1 ? q.y : (j & 3) == 2 ? q.z : q.w;
    return exp1_from_word(w);
}

// The same values for VEC consecutive elements starting at e0 (e0 % 4 == 0), vectorised; the
// noise mode NZ is a compile-time parameter so perf-mode kernels carry no fp64 log1p code.
template <int VEC, int NZ>
__device__ __forceinline__ void exp_noise_vec(const sd_noise& nz, int64_t woff, int row, int64_t e0, int vocab,
                                              float* out) {
    if constexpr (NZ == SD_NOISE_STREAM) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) out[k] = (e0 + k < vocab) ? exp_noise(nz, woff, row, e0 + k) : 1.f;
    } else {
#pragma unroll
        for (int q = 0; q < VEC / 4; ++q) {
            const uint4 r = philox_block(nz, (uint32_t)row, kSiteSample, (uint32_t)((e0 >> 2) + q));
            out[4 * q + 0] = exp1_from_word(r.x);
            out[4 * q + 1] = exp1_from_word(r.y);
            out[4 * q + 2] = exp1_from_word(r.z);
            out[4 * q + 3] = exp1_from_word(r.w);
        }
    }
}

}  // namespace sd
