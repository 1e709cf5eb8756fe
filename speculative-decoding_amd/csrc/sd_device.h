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
#include <climits>

#include "specdec.h"

namespace sd {

constexpr int kWave = 64;
constexpr int kThreads = 256;            // 4 waves per workgroup
constexpr float kNegFill = -1e20f;       // utils/logits_processor.py:62,79

// ---------------------------------------------------------------- dtype handling
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

// fp32 -> bf16 -> fp32, round to nearest even: gfx950's v_cvt_pk_bf16_f32 (two instructions per
// value; the integer form with its NaN branch cost ~13, the sampling passes' VALU bound).  Equal to
// the integer rounding on all 2^32 inputs, NaN for NaN (scripts/microbench/bf16_round.hip).
__device__ __forceinline__ float round_bf16(float f) { return (float)(__bf16)f; }

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

// Split loads: a thread that needs several 16-byte vectors issues them all before it uses any
// (load_vec's in-range test is a branch, and the compiler waits for each vector before the next
// branch, so a loop of load_vec calls pays one memory round trip per vector).  ld16_clamped
// loads the vector at e0, or — past the last whole vector of the row — that last whole vector,
// so every load is unconditional and in bounds (caller: 16-byte aligned row, vocab >= kVec);
// finish16 unpacks it and patches a vector that is not wholly inside [0, vocab) with guarded
// element loads (only a ragged row end takes that second round trip).
template <int DT>
__device__ __forceinline__ int64_t last_whole_vec(int vocab) {
    return ((int64_t)vocab / Elem<DT>::kVec - 1) * Elem<DT>::kVec;
}
template <int DT>
__device__ __forceinline__ uint4 ld16_clamped(const void* row, int64_t e0, int64_t last) {
    return *reinterpret_cast<const uint4*>(static_cast<const char*>(row) + (e0 < last ? e0 : last) * Elem<DT>::kBytes);
}
template <int DT>
__device__ __forceinline__ void finish16(uint4 w, const void* row, int64_t e0, int vocab, float* out) {
    constexpr int V = Elem<DT>::kVec;
    unpack16<DT>(w, out);
    if (e0 + V > vocab) {
#pragma unroll
        for (int k = 0; k < V; ++k) out[k] = (e0 + k < vocab) ? load_one<DT>(row, e0 + k) : 0.f;
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

// Load N consecutive elements starting at e0 (N a divisor of kVec, e0 a multiple of N): one
// 16-, 8- or 4-byte vector when the row is 16-byte aligned and in range, else guarded scalars.
// Mixed-width pairs (bf16 target with fp32 drafter) step both rows by the narrower vector.
template <int DT, int N>
__device__ __forceinline__ void load_vecn(const void* row, int64_t e0, int vocab, bool aligned, float* out) {
    static_assert(Elem<DT>::kVec % N == 0, "N must divide the 16-byte vector");
    if constexpr (N == Elem<DT>::kVec) {
        load_vec<DT>(row, e0, vocab, aligned, out);
    } else {
        constexpr int kB = N * Elem<DT>::kBytes;
        if (aligned && e0 + N <= vocab) {
            const char* a = static_cast<const char*>(row) + e0 * Elem<DT>::kBytes;
            uint32_t ws[4];
            if constexpr (kB == 8) {
                const uint2 w = *reinterpret_cast<const uint2*>(a);
                ws[0] = w.x; ws[1] = w.y;
            } else {
                static_assert(kB == 4, "unsupported width");
                ws[0] = *reinterpret_cast<const uint32_t*>(a);
            }
#pragma unroll
            for (int k = 0; k < kB / 4; ++k) {
                if constexpr (DT == SD_F32) {
                    out[k] = __uint_as_float(ws[k]);
                } else if constexpr (DT == SD_BF16) {
                    out[2 * k] = __uint_as_float(ws[k] << 16);
                    out[2 * k + 1] = __uint_as_float(ws[k] & 0xffff0000u);
                } else {
                    out[2 * k] = __half2float(__ushort_as_half((unsigned short)(ws[k] & 0xffffu)));
                    out[2 * k + 1] = __half2float(__ushort_as_half((unsigned short)(ws[k] >> 16)));
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) out[k] = (e0 + k < vocab) ? load_one<DT>(row, e0 + k) : 0.f;
        }
    }
}

// ---------------------------------------------------------------- cross-workgroup exchange
// Data handed between workgroups of ONE kernel (the last-arrival tails) goes through
// agent-coherent stores / loads (relaxed agent-scope atomics: `sc1` on gfx950, write-through /
// bypass of the per-XCD L2 for these few words) instead of an agent-scope release / acquire,
// which on gfx950 is a whole-L2 writeback + invalidate (buffer_wbl2 / buffer_inv) per workgroup.
__device__ __forceinline__ void st_coh(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(float2* p, float2 v) {
    const uint64_t u = ((uint64_t)__float_as_uint(v.y) << 32) | __float_as_uint(v.x);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coh(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<uint32_t*>(const_cast<float*>(p)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ int32_t ld_coh(const int32_t* p) {
    return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_coh(const float2* p) {
    const uint64_t u = __hip_atomic_load(reinterpret_cast<uint64_t*>(const_cast<float2*>(p)), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((uint32_t)u), __uint_as_float((uint32_t)(u >> 32)));
}
// coherent only when another workgroup of the SAME launch may have written p (last-arrival tails);
// data from an earlier launch is read with plain (cacheable) loads
template <typename T>
__device__ __forceinline__ T ld_x(const T* p, bool coh) { return coh ? ld_coh(p) : *p; }

// One 16-byte record per write-through store / coherent load (global_*_dwordx4 sc1): a scalar
// sc1 store is one fabric write each (dword ~6x the dwordx4 time per byte, MI355X_MICROARCH.md),
// so a tail's partial {a, b, c, d} travels as one.  p must be 16-byte aligned.  The load waits for
// itself (vmcnt(0)): the compiler does not track inline-asm loads.
typedef uint32_t sd_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_coh16(void* p, uint4 v) {
    const sd_u32x4 w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ uint4 ld_coh16(const void* p) {
    sd_u32x4 w;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(w) : "v"(p) : "memory");
    return make_uint4(w.x, w.y, w.z, w.w);
}

// five coherent 16-byte loads in flight together, one wait (pollers that read several records:
// separate ld_coh16 calls cost one round trip each).  Unused slots take any valid address.
__device__ __forceinline__ void ld_coh16x5(const void* p0, const void* p1, const void* p2, const void* p3,
                                           const void* p4, uint4* out) {
    sd_u32x4 a, b, c, d, e;
    asm volatile(
        "global_load_dwordx4 %0, %5, off sc1\n\t"
        "global_load_dwordx4 %1, %6, off sc1\n\t"
        "global_load_dwordx4 %2, %7, off sc1\n\t"
        "global_load_dwordx4 %3, %8, off sc1\n\t"
        "global_load_dwordx4 %4, %9, off sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "=&v"(e)
        : "v"(p0), "v"(p1), "v"(p2), "v"(p3), "v"(p4)
        : "memory");
    out[0] = make_uint4(a.x, a.y, a.z, a.w);
    out[1] = make_uint4(b.x, b.y, b.z, b.w);
    out[2] = make_uint4(c.x, c.y, c.z, c.w);
    out[3] = make_uint4(d.x, d.y, d.z, d.w);
    out[4] = make_uint4(e.x, e.y, e.z, e.w);
}

// this wave's coherent stores have completed (s_waitcnt 0), and the compiler keeps order
__device__ __forceinline__ void coh_wait() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// A row's error bits (SD_ROW_ERROR_MASK) into the caller's sticky word: one device atomic, and
// only for a failed row (the success path issues nothing).  Called by the one thread that writes
// the row's status.
__device__ __forceinline__ void flag_error(int32_t* acc, int32_t status) {
    const int32_t e = status & SD_ROW_ERROR_MASK;
    if (acc && e) __hip_atomic_fetch_or(acc, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded polls, by WALL CLOCK: a wait gives up after `limit_us` microseconds (the host's poll
// bound, sd_set_poll_policy; default 2 s) of s_memrealtime (a constant 100 MHz clock), so a grid
// that shares the GPU with a long kernel of another stream waits for it instead of flagging its
// rows.  The clock is read once every 64 re-reads (the start of the wait at the 64th: the common
// short waits never read it); t0 is the caller's per-wait state, zero before the loop.  A negative
// limit gives up at once (tests force the timeout path with it).
__device__ __forceinline__ bool spin_more(int spin, int limit_us, uint64_t& t0) {
    if (limit_us < 0) return false;
    if ((spin & 63) != 63) return true;
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (spin == 63) t0 = t;
    return t - t0 < (uint64_t)limit_us * 100u;
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

// Perf-mode sampling weight: the dtype-rounded probability from one exp2 and the reciprocal of S,
// without prob_exact's correctly-rounded re-evaluation near a rounding boundary (fp32 error of a
// few ulp: ~2e-4 of bf16 values land one ulp off, which moves a sampling weight by <= 2^-8 of
// itself).  Decisions (p(x)/q(x)) and greedy picks keep prob_exact.
template <int DT>
__device__ __forceinline__ float prob_fast(float y, float m, float invS) {
    return round_dt<DT>(__builtin_amdgcn_exp2f((y - m) * 1.44269502162933349609375f) * invS);
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
    if (has_keep && !(x > keep.tau || (x == keep.tau && (int32_t)j <= keep.tie_idx))) v = round_dt<DT>(kNegFill);   // j < 2^31
    if (T != 1.0f) v = round_dt<DT>(v / T);
    // A NaN / +inf logit under a top-k / nucleus keep stays NaN whether the cut keeps it or not:
    // torch's topk and sort rank NaN first and keep +inf, whose softmax is NaN (inf - inf), so the
    // reference's processed row is NaN throughout (utils/logits_processor.py:59-63,73-81).  Every
    // consumer of a processed row takes its (max, Σexp) over all of it, and a NaN element makes
    // those NaN: the row then behaves exactly as a NaN row (draws flag SD_ROW_INVALID_DIST, accept
    // ratios are NaN as the reference's).
    if (has_keep && !(x <= 3.402823466e38f)) v = __builtin_nanf("");
    return v;
}

// process_value over N consecutive elements (indices e0 ..): the keep mask and NaN rule per element,
// then the temperature behind ONE wave-uniform branch — the same values as N process_value calls
// (a masked value divided by T either way; NaN / T stays NaN), without a branch per element
// The keep mask and NaN rule of process_value over N consecutive elements (indices e0 ..): the tie
// index compare becomes one 32-bit compare against a per-vector constant (element k is an allowed
// tie iff k <= tie_idx - e0; indices are < 2^31)
template <int DT, int N>
__device__ __forceinline__ void keep_vec(float* x, int64_t e0, const RowKeep& keep) {
    const int32_t jr = keep.tie_idx - (int32_t)e0;
    const float fill = round_dt<DT>(kNegFill);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const float xv = x[k];
        const float v = (xv > keep.tau || (xv == keep.tau && k <= jr)) ? xv : fill;
        x[k] = xv <= 3.402823466e38f ? v : __builtin_nanf("");
    }
}
template <int DT, int N>
__device__ __forceinline__ void process_vec(float* x, int64_t e0, float T, bool has_keep, const RowKeep& keep) {
    if (has_keep) keep_vec<DT, N>(x, e0, keep);
    if (T != 1.0f) {
#pragma unroll
        for (int k = 0; k < N; ++k) x[k] = round_dt<DT>(x[k] / T);
    }
}

// ---------------------------------------------------------------- wave primitives (DPP)
// Cross-lane steps use DPP lane shuffles (a VALU operand modifier, a few cycles) instead of
// __shfl (ds_bpermute through the LDS crossbar, ~100 cycles per dependent step).  Reductions:
// quad_perm x2, row_half_mirror, row_mirror (every lane holds its row's result), then
// row_bcast15 / row_bcast31 fold rows 0..3 into lane 63, broadcast with readlane.  Scans:
// row_shr 1,2,4,8 (Hillis-Steele inside each 16-lane row), then row_bcast15 / row_bcast31.
// The combining order is fixed, so results are deterministic.  Call with all 64 lanes active.
enum : int {
    kDppQuad1032 = 0xB1, kDppQuad2301 = 0x4E, kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114,
    kDppRowShr8 = 0x118, kDppRowMirror = 0x140, kDppRowHalfMirror = 0x141, kDppRowBcast15 = 0x142,
    kDppRowBcast31 = 0x143
};

template <int CTRL, int ROWS = 0xF, bool BOUND0 = false>
__device__ __forceinline__ int dpp_i(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xF, BOUND0);
}
template <int CTRL, int ROWS = 0xF, bool BOUND0 = false>
__device__ __forceinline__ float dpp_f(float old, float v) {
    return __int_as_float(dpp_i<CTRL, ROWS, BOUND0>(__float_as_int(old), __float_as_int(v)));
}
template <int CTRL, int ROWS = 0xF, bool BOUND0 = false>
__device__ __forceinline__ double dpp_d(double old, double v) {
    const uint64_t o = __double_as_longlong(old), x = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)dpp_i<CTRL, ROWS, BOUND0>((int)(uint32_t)o, (int)(uint32_t)x);
    const uint32_t hi = (uint32_t)dpp_i<CTRL, ROWS, BOUND0>((int)(uint32_t)(o >> 32), (int)(uint32_t)(x >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ float lane63_f(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63)); }
__device__ __forceinline__ int lane63_i(int v) { return __builtin_amdgcn_readlane(v, 63); }

// all-lanes reduction of v with op (identity id): the result is uniform across the wave
template <typename Op>
__device__ __forceinline__ float wave_reduce(float v, float id, Op op) {
    v = op(v, dpp_f<kDppQuad1032>(id, v));
    v = op(v, dpp_f<kDppQuad2301>(id, v));
    v = op(v, dpp_f<kDppRowHalfMirror>(id, v));
    v = op(v, dpp_f<kDppRowMirror>(id, v));
    v = op(v, dpp_f<kDppRowBcast15, 0xA>(id, v));
    v = op(v, dpp_f<kDppRowBcast31, 0xC>(id, v));
    return lane63_f(v);
}
template <typename Op>
__device__ __forceinline__ int wave_reduce_i(int v, int id, Op op) {
    v = op(v, dpp_i<kDppQuad1032>(id, v));
    v = op(v, dpp_i<kDppQuad2301>(id, v));
    v = op(v, dpp_i<kDppRowHalfMirror>(id, v));
    v = op(v, dpp_i<kDppRowMirror>(id, v));
    v = op(v, dpp_i<kDppRowBcast15, 0xA>(id, v));
    v = op(v, dpp_i<kDppRowBcast31, 0xC>(id, v));
    return lane63_i(v);
}

__device__ __forceinline__ float wave_max(float v) {
    return wave_reduce(v, -INFINITY, [](float a, float b) { return fmaxf(a, b); });
}
// wave max on order-preserving integer keys (k_draw_lean's hot path): v_max_i32 needs no NaN
// canonicalisation, so each step is one DPP-fused instruction instead of four.  A NaN input may win
// or lose the max (fmaxf drops it); the callers flag such rows from their NaN weights either way.
__device__ __forceinline__ float wave_max_ord(float v) {
    int k = __float_as_int(v);
    k ^= (k >> 31) & 0x7fffffff;
    auto mx = [](int a, int b) { return a > b ? a : b; };
    k = mx(k, dpp_i<kDppQuad1032>(INT_MIN, k));
    k = mx(k, dpp_i<kDppQuad2301>(INT_MIN, k));
    k = mx(k, dpp_i<kDppRowHalfMirror>(INT_MIN, k));
    k = mx(k, dpp_i<kDppRowMirror>(INT_MIN, k));
    k = mx(k, dpp_i<kDppRowBcast15, 0xA>(INT_MIN, k));
    k = mx(k, dpp_i<kDppRowBcast31, 0xC>(INT_MIN, k));
    k = lane63_i(k);
    k ^= (k >> 31) & 0x7fffffff;
    return __int_as_float(k);
}
__device__ __forceinline__ float wave_sum(float v) {
    return wave_reduce(v, 0.f, [](float a, float b) { return a + b; });
}
__device__ __forceinline__ int wave_min_i(int v) {
    return wave_reduce_i(v, INT_MAX, [](int a, int b) { return a < b ? a : b; });
}
__device__ __forceinline__ int wave_sum_i(int v) {
    return wave_reduce_i(v, 0, [](int a, int b) { return a + b; });
}
__device__ __forceinline__ int wave_max_i(int v) {
    return wave_reduce_i(v, INT_MIN, [](int a, int b) { return a > b ? a : b; });
}

// inclusive prefix sums across the wave (lane order)
__device__ __forceinline__ float wave_incl_scan(float v) {
    v += dpp_f<kDppRowShr1, 0xF, true>(0.f, v);
    v += dpp_f<kDppRowShr2, 0xF, true>(0.f, v);
    v += dpp_f<kDppRowShr4, 0xF, true>(0.f, v);
    v += dpp_f<kDppRowShr8, 0xF, true>(0.f, v);
    v += dpp_f<kDppRowBcast15, 0xA>(0.f, v);
    v += dpp_f<kDppRowBcast31, 0xC>(0.f, v);
    return v;
}
__device__ __forceinline__ int wave_incl_scan_i(int v) {   // integer inclusive scan (lane order)
    v += dpp_i<kDppRowShr1, 0xF, true>(0, v);
    v += dpp_i<kDppRowShr2, 0xF, true>(0, v);
    v += dpp_i<kDppRowShr4, 0xF, true>(0, v);
    v += dpp_i<kDppRowShr8, 0xF, true>(0, v);
    v += dpp_i<kDppRowBcast15, 0xA>(0, v);
    v += dpp_i<kDppRowBcast31, 0xC>(0, v);
    return v;
}
__device__ __forceinline__ double wave_incl_scan_d(double v) {
    v += dpp_d<kDppRowShr1, 0xF, true>(0.0, v);
    v += dpp_d<kDppRowShr2, 0xF, true>(0.0, v);
    v += dpp_d<kDppRowShr4, 0xF, true>(0.0, v);
    v += dpp_d<kDppRowShr8, 0xF, true>(0.0, v);
    v += dpp_d<kDppRowBcast15, 0xA>(0.0, v);
    v += dpp_d<kDppRowBcast31, 0xC>(0.0, v);
    return v;
}
// a wave-uniform double into scalar registers (no VGPRs held across a long wait)
__device__ __forceinline__ double uniform_d(double v) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double lane_d(double v, int lane) {
    const uint64_t x = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// torch.argmax semantics: NaN is the maximum; among equal maxima the first index wins.
__device__ __forceinline__ bool arg_better(float a, int32_t ia, float b, int32_t ib) {
    const bool na = a != a, nb = b != b;
    if (na || nb) return na && (!nb || ia < ib);
    return a > b || (a == b && ia < ib);
}

// (v, i) argmax across the wave (arg_better order); the result is uniform across the wave
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ void argmax_step(float& v, int32_t& i) {
    const float ov = dpp_f<CTRL, ROWS>(-INFINITY, v);
    const int32_t oi = dpp_i<CTRL, ROWS>(INT_MAX, i);
    if (arg_better(ov, oi, v, i)) { v = ov; i = oi; }
}
__device__ __forceinline__ void wave_argmax(float& v, int32_t& i) {
    argmax_step<kDppQuad1032>(v, i);
    argmax_step<kDppQuad2301>(v, i);
    argmax_step<kDppRowHalfMirror>(v, i);
    argmax_step<kDppRowMirror>(v, i);
    argmax_step<kDppRowBcast15, 0xA>(v, i);
    argmax_step<kDppRowBcast31, 0xC>(v, i);
    v = lane63_f(v);
    i = lane63_i(i);
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

// The same Exp(1) value in fp32 arithmetic, for SCREENING only (relative error <= 2^-21 against
// exp1_from_words): u < 1/2 as -log1p(-u) with u rounded to fp32 (log1p stays well conditioned),
// u >= 1/2 as -log(1 - u) with 1 - u formed exactly in integers and rounded once.  The kernels
// find the few elements that can win an exponential race with it, and evaluate only those with
// the exact fp64 form — so torch's values decide the race, at fp32 cost per element.
constexpr float kExpFastRelErr = 4.76837158203125e-07f;   // 2^-21
__device__ __forceinline__ float exp1_fast_from_words(uint32_t hi, uint32_t lo) {
    const uint64_t v = ((((uint64_t)hi) << 32) | lo) & ((1ull << 53) - 1);
    if (v < (1ull << 52)) return -log1pf(-(float)v * 1.1102230246251565e-16f);
    return -__logf((float)((1ull << 53) - v) * 1.1102230246251565e-16f);
}

// A cheaper screening value for 16-bit rows (relative error <= 2^-11 against exp1_from_words; the
// races over bf16 / fp16 values tolerate far more): u < 2^-10 as u (1 + u/2), u < 1/2 as
// -ln(1 - u) with 1 - u rounded once in fp32, u >= 1/2 as -ln of 1 - u formed from the words with
// one rounding; v_log_f32 for the logarithm.  About ten VALU instructions, no branches.
constexpr float kExpScreen16RelErr = 4.8828125e-04f;   // 2^-11
__device__ __forceinline__ float exp1_screen16(uint32_t hi, uint32_t lo) {
    const uint32_t h = hi & 0x1FFFFFu;                  // the top 21 of the 53 bits
    const float lof = (float)lo * 1.1102230246251565e-16f;   // lo * 2^-53
    const float u = fmaf((float)h, 4.76837158203125e-07f, lof);                    // h * 2^-21 + lo * 2^-53
    const float w = h < (1u << 20) ? 1.0f - u : fmaf((float)((1u << 21) - h), 4.76837158203125e-07f, -lof);
    const float big = -__builtin_amdgcn_logf(w) * 0.693147180559945309f;            // -ln(w)
    return u < 9.765625e-04f ? u * fmaf(0.5f, u, 1.0f) : big;
}

// STREAM (ABI 11): word i of a call is words[stream_base(nz) + i], base = offset + *offset_dev (both
// optional): a noise session hands every call its pool and the call's start inside it — the host
// part (draws of known size) in `offset`, the part only the device knows (what the previous verify
// consumed) in `offset_dev` — so a pool generated ahead, on another stream, needs no host sync.
// n_words is the pool's capacity from words[0].
__device__ __forceinline__ int64_t stream_base(const sd_noise& nz) {
    return (int64_t)nz.offset + (nz.offset_dev ? (int64_t)*reinterpret_cast<const int64_t*>(nz.offset_dev) : 0);
}
__device__ __forceinline__ const uint32_t* stream_ptr(const sd_noise& nz) { return nz.words + stream_base(nz); }
__device__ __forceinline__ int64_t stream_cap(const sd_noise& nz) { return nz.n_words - stream_base(nz); }

// torch's exponential_ words of VEC consecutive elements (two per element, from woff + 2 e0): 16-byte
// loads when aligned and in range, else per-word loads; words past the buffer read as 0 (the
// callers flag the overrun).
template <int VEC>
__device__ __forceinline__ void stream_words(const sd_noise& nz, int64_t woff, int64_t e0, uint32_t* w) {
    const int64_t w0 = woff + 2 * e0;
    const uint32_t* src = stream_ptr(nz) + w0;
    const int64_t cap = stream_cap(nz);
    const int s = (int)((reinterpret_cast<uintptr_t>(src) >> 2) & 3);   // words past a 16-byte boundary
    if (s == 0 && w0 + 2 * VEC <= cap) {
#pragma unroll
        for (int q = 0; q < VEC / 2; ++q) {
            const uint4 t = reinterpret_cast<const uint4*>(src)[q];
            w[4 * q] = t.x; w[4 * q + 1] = t.y; w[4 * q + 2] = t.z; w[4 * q + 3] = t.w;
        }
    } else if (s != 0 && w0 - s + 2 * VEC + 4 <= cap) {
        // a call that starts mid-vector (a pipelined pool's offset is what the verifies consumed):
        // one more aligned vector, and the words picked by a shift that is uniform per call (the
        // row's offset sets it; e0 is a multiple of VEC), so per-word loads are never needed
        uint32_t u[2 * VEC + 4];
        const uint4* a = reinterpret_cast<const uint4*>(src - s);
#pragma unroll
        for (int q = 0; q <= VEC / 2; ++q) {
            const uint4 t = a[q];
            u[4 * q] = t.x; u[4 * q + 1] = t.y; u[4 * q + 2] = t.z; u[4 * q + 3] = t.w;
        }
        if (s == 1) {
#pragma unroll
            for (int k = 0; k < 2 * VEC; ++k) w[k] = u[k + 1];
        } else if (s == 2) {
#pragma unroll
            for (int k = 0; k < 2 * VEC; ++k) w[k] = u[k + 2];
        } else {
#pragma unroll
            for (int k = 0; k < 2 * VEC; ++k) w[k] = u[k + 3];
        }
    } else {
#pragma unroll
        for (int k = 0; k < 2 * VEC; ++k) w[k] = w0 + k < cap ? src[k] : 0u;
    }
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

enum PhiloxSite : uint32_t { kSiteAccept = 1, kSiteSample = 2, kSiteCdf = 3 };

// counter (idx, global row | site << 24, offset): row is the call-local row, nz.row_base its base
__device__ __forceinline__ uint4 philox_block(const sd_noise& nz, uint32_t row, uint32_t site, uint32_t idx) {
    const uint32_t grow = (uint32_t)(nz.row_base + row);
    // offset_dev: a device-resident base added to the call's offset (graph replays move it on the device)
    const uint64_t off = nz.offset + (nz.offset_dev ? *nz.offset_dev : 0ull);
    const uint4 c = make_uint4(idx, (grow & 0x00ffffffu) | (site << 24), (uint32_t)off, (uint32_t)(off >> 32));
    return philox4x32_10(c, make_uint2((uint32_t)nz.seed, (uint32_t)(nz.seed >> 32)));
}

// perf-mode U[0,1) at 53 bits for the inverse-CDF draws of row `row`: idx 0 picks the chunk,
// idx 1 + c the element inside chunk c (independent blocks)
__device__ __forceinline__ double cdf_uniform(const sd_noise& nz, uint32_t row, uint32_t idx = 0u) {
    const uint4 q = philox_block(nz, row, kSiteCdf, idx);
    return (double)(((((uint64_t)q.x) << 32) | q.y) >> 11) * 1.1102230246251565e-16;   // 2^-53
}

// perf-mode Exp(1) from one 32-bit word: u in (0,1) at 24 bits, E = -ln(u) in fp32
__device__ __forceinline__ float exp1_from_word(uint32_t w) {
    const float u = (float)(w >> 8) * 5.9604644775390625e-08f + 2.98023223876953125e-08f;
    return -__logf(u);
}

// perf-mode span race of row `row` (k_draw_lean): Gumbel noise g_c = -ln E_c of span c from word z of
// the span's cdf block (words x, y are its in-span uniform, cdf_uniform(row, 1 + c)); the row's span
// is argmax_c (m_c + ln S_c + g_c), i.e. span c with probability S_c e^(m_c) / Σ (Gumbel-max)
__device__ __forceinline__ float span_gumbel(const sd_noise& nz, uint32_t row, uint32_t c) {
    return -__logf(exp1_from_word(philox_block(nz, row, kSiteCdf, 1u + c).z));
}

// Exp(1) noise of element j of a sampled row.  STREAM: torch's exponential_ draw for element j
// (2 words at woff + 2j).  PHILOX: word (j & 3) of block (row, sample, j >> 2).
__device__ __forceinline__ float exp_noise(const sd_noise& nz, int64_t woff, int row, int64_t j) {
    if (nz.mode == SD_NOISE_STREAM) {
        const int64_t w = woff + 2 * j;
        if (w + 1 >= stream_cap(nz)) return 1.f;   // overrun is flagged by the caller
        const uint32_t* ws = stream_ptr(nz);
        return exp1_from_words(ws[w], ws[w + 1]);
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
