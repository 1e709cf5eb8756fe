// mt_jump.cpp — jump-ahead polynomials for torch's CPU generator (ATen mt19937), host side of the
// device STREAM noise generator (csrc/mt_device.hip).
//
// The generator's untempered sequence obeys x[k+624] = x[k+397] ^ f(upper(x[k]), lower(x[k+1])),
// a linear map A over GF(2) on the 624-word window W(m) = x[m .. m+623].  On windows that are
// images of A (every W(m), m >= 1) A satisfies its characteristic polynomial P (degree 19937,
// primitive), so for J >= 1:   W(m + J) = A^(J-1) W(m + 1) = sum_i c_i W(m + 1 + i),
// with c = x^(J-1) mod P.  The device XORs the windows of one shared base sequence selected by
// c's bits to start every substream of a fill at its own offset (one jump per substream).
//
// P is found once per process by Berlekamp–Massey on one output bit of the generator; the jump
// polynomials for offsets s * stride (s = 1..count) follow by repeated multiplication with
// x^stride mod P (carry-less products, Barrett reduction).  CPU tests check every piece against
// straight generation (tests/test_mt_jump_cpu.py).
#include <cstring>
#include <mutex>
#include <vector>

#include "specdec.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr int kDeg = 19937;                 // degree of P
constexpr int kW = (kDeg + 63) / 64;        // 312 words hold a polynomial of degree < kDeg

using Poly = std::vector<uint64_t>;         // bit i of word i/64 = coefficient of x^i

// -------------------------------------------------------------------------- carry-less products
uint64_t clmul_lo_sw(uint64_t a, uint64_t b, uint64_t* hi) {
    uint64_t lo = 0, h = 0;
    for (int i = 0; i < 64; ++i)
        if ((b >> i) & 1) {
            lo ^= a << i;
            if (i) h ^= a >> (64 - i);
        }
    *hi = h;
    return lo;
}

#if defined(__x86_64__)
typedef long long v2di __attribute__((vector_size(16)));
__attribute__((target("pclmul"))) uint64_t clmul_lo_hw(uint64_t a, uint64_t b, uint64_t* hi) {
    v2di x = {(long long)a, 0}, y = {(long long)b, 0};
    v2di r = __builtin_ia32_pclmulqdq128(x, y, 0x00);
    *hi = (uint64_t)r[1];
    return (uint64_t)r[0];
}
bool have_pclmul() {
    static const bool ok = __builtin_cpu_supports("pclmul");
    return ok;
}
#endif

// r = a * b (full product, a.size() + b.size() words)
void poly_mul(const uint64_t* a, int na, const uint64_t* b, int nb, uint64_t* r) {
    std::memset(r, 0, sizeof(uint64_t) * (na + nb));
#if defined(__x86_64__)
    if (have_pclmul()) {
        for (int i = 0; i < na; ++i) {
            if (!a[i]) continue;
            for (int j = 0; j < nb; ++j) {
                uint64_t hi, lo = clmul_lo_hw(a[i], b[j], &hi);
                r[i + j] ^= lo;
                r[i + j + 1] ^= hi;
            }
        }
        return;
    }
#endif
    for (int i = 0; i < na; ++i) {
        if (!a[i]) continue;
        for (int j = 0; j < nb; ++j) {
            uint64_t hi, lo = clmul_lo_sw(a[i], b[j], &hi);
            r[i + j] ^= lo;
            r[i + j + 1] ^= hi;
        }
    }
}

inline int bit(const uint64_t* p, long i) { return (int)((p[i >> 6] >> (i & 63)) & 1); }
inline void flip(uint64_t* p, long i) { p[i >> 6] ^= 1ull << (i & 63); }

// bits [lo, lo + n) of p as a new polynomial (shift right by lo)
void take_bits(const uint64_t* p, int np, long lo, int n, uint64_t* out) {
    const int nw = (n + 63) / 64;
    for (int w = 0; w < nw; ++w) {
        const long b = lo + 64L * w;
        const long wi = b >> 6;
        const int sh = (int)(b & 63);
        uint64_t v = wi < np ? p[wi] >> sh : 0;
        if (sh && wi + 1 < np) v |= p[wi + 1] << (64 - sh);
        out[w] = v;
    }
    const int tail = n & 63;
    if (tail) out[nw - 1] &= (1ull << tail) - 1;
}

struct Field {
    Poly P;        // degree kDeg, kW + 1 words
    Poly mu;       // floor(x^(2 kDeg) / P), degree kDeg
    bool ok = false;

    // r = a mod P for deg(a) < 2 kDeg (Barrett): q = floor(floor(a / x^n) * mu / x^n), r = a - q P
    void reduce(const uint64_t* a, int na, uint64_t* r) const {
        const int n = kDeg;
        std::vector<uint64_t> hi(kW + 1), t(2 * kW + 4), q(kW + 1), qp(2 * kW + 4);
        take_bits(a, na, n, n, hi.data());
        poly_mul(hi.data(), kW, mu.data(), kW + 1, t.data());
        take_bits(t.data(), 2 * kW + 1, n, n + 1, q.data());
        poly_mul(q.data(), kW + 1, P.data(), kW + 1, qp.data());
        for (int w = 0; w < kW; ++w) r[w] = (w < na ? a[w] : 0) ^ qp[w];
        r[kW - 1] &= (1ull << (kDeg & 63)) - 1;
    }

    void mulmod(const uint64_t* a, const uint64_t* b, uint64_t* r) const {
        std::vector<uint64_t> t(2 * kW);
        poly_mul(a, kW, b, kW, t.data());
        reduce(t.data(), 2 * kW, r);
    }

    // x^e mod P (square and multiply; e >= 0)
    Poly xpow(uint64_t e) const {
        Poly r(kW, 0);
        r[0] = 1;
        int top = 63;
        while (top >= 0 && !((e >> top) & 1)) --top;
        std::vector<uint64_t> t(2 * kW + 2);
        for (int b = top; b >= 0; --b) {
            mulmod(r.data(), r.data(), r.data());
            if ((e >> b) & 1) {    // r *= x
                std::memset(t.data(), 0, sizeof(uint64_t) * t.size());
                for (int w = 0; w < kW; ++w) {
                    t[w] |= r[w] << 1;
                    t[w + 1] |= r[w] >> 63;
                }
                reduce(t.data(), kW + 1, r.data());
            }
        }
        return r;
    }
};

// untempered words of a generator seeded the way torch seeds it (seed 5489), from x[1] on
void untempered_sequence(uint32_t* out, int n) {
    std::vector<uint32_t> x(n + kN + 1);
    x[0] = 5489u;
    for (int i = 1; i < kN; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    for (int k = 0; k + kN < n + kN + 1; ++k) {
        const uint32_t y = (x[k] & 0x80000000u) | (x[k + 1] & 0x7fffffffu);
        x[k + kN] = x[k + kM] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    std::memcpy(out, x.data() + 1, sizeof(uint32_t) * n);
}

// Berlekamp–Massey over GF(2) on bit 0 of the untempered sequence: the connection polynomial
// C(x) = 1 + c1 x + ... + cL x^L; P(x) = x^L C(1/x) is the characteristic polynomial.
bool characteristic_polynomial(Poly& P) {
    const int n = 2 * kDeg + 64;
    std::vector<uint32_t> seq(n);
    untempered_sequence(seq.data(), n);
    // R: the bit sequence reversed and packed, bit (n-1-k) = s[k]; then s[k-i] = R bit (n-1-k+i)
    const int nw = (n + 63) / 64 + 2;
    std::vector<uint64_t> R(nw, 0), C(nw, 0), B(nw, 0), T(nw), win(nw);
    for (int k = 0; k < n; ++k)
        if (seq[k] & 1u) flip(R.data(), n - 1 - k);
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int k = 0; k < n; ++k) {
        // d = sum_{i=0..L} C_i s[k-i]
        take_bits(R.data(), nw, n - 1 - k, L + 1, win.data());
        uint64_t acc = 0;
        for (int w = 0; w <= L / 64; ++w) acc ^= win[w] & C[w];
        if (!__builtin_parityll(acc)) { ++m; continue; }
        T = C;
        const int ws = m >> 6, bs = m & 63;   // C ^= B << m
        for (int w = nw - 1; w >= 0; --w) {
            uint64_t v = 0;
            if (w - ws >= 0) v = B[w - ws] << bs;
            if (bs && w - ws - 1 >= 0) v |= B[w - ws - 1] >> (64 - bs);
            C[w] ^= v;
        }
        if (2 * L <= k) {
            L = k + 1 - L;
            B = T;
            m = 1;
        } else {
            ++m;
        }
    }
    if (L != kDeg) return false;
    P.assign(kW + 1, 0);
    for (int i = 0; i <= L; ++i)
        if (bit(C.data(), i)) flip(P.data(), L - i);
    return true;
}

const Field& field() {
    static Field F;
    static std::once_flag once;
    std::call_once(once, [] {
        if (!characteristic_polynomial(F.P)) return;
        // mu = floor(x^(2n) / P) by long division (once)
        const int n = kDeg;
        std::vector<uint64_t> rem((2 * n + 64) / 64 + 1, 0);
        flip(rem.data(), 2L * n);
        F.mu.assign(kW + 1, 0);
        for (long d = 2L * n; d >= n; --d) {
            if (!bit(rem.data(), d)) continue;
            flip(F.mu.data(), d - n);
            for (long i = 0; i <= n; ++i)
                if (bit(F.P.data(), i)) flip(rem.data(), i + d - n);
        }
        F.ok = true;
    });
    return F;
}

inline uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// untempered words x[lo .. lo + n) continuing a window w[0..623] = x[lo - 624 .. lo)
void extend(std::vector<uint32_t>& x, size_t upto) {
    for (size_t k = x.size() - kN; x.size() < upto; ++k) {
        const uint32_t y = (x[k] & 0x80000000u) | (x[k + 1] & 0x7fffffffu);
        x.push_back(x[k + kM] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
}

}  // namespace

extern "C" {

int32_t sd_mt19937_jump_table(int64_t stride_words, int32_t count, uint64_t* out) {
    if (stride_words < 1 || count < 0 || (count > 0 && !out)) return SD_ERR_INVALID;
    static_assert(SD_MT_JUMP_WORDS >= kW, "jump polynomial slot");
    const Field& F = field();
    if (!F.ok) return SD_ERR_UNSUPPORTED;
    if (count == 0) return SD_OK;
    // c_s = x^(s*stride - 1) mod P: c_1 = x^(stride-1), c_(s+1) = c_s * x^stride
    Poly c = F.xpow((uint64_t)stride_words - 1);
    Poly step = F.xpow((uint64_t)stride_words);
    for (int s = 1; s <= count; ++s) {
        uint64_t* o = out + (size_t)(s - 1) * SD_MT_JUMP_WORDS;
        std::memcpy(o, c.data(), sizeof(uint64_t) * kW);
        std::memset(o + kW, 0, sizeof(uint64_t) * (SD_MT_JUMP_WORDS - kW));
        if (s < count) F.mulmod(c.data(), step.data(), c.data());
    }
    return SD_OK;
}

int32_t sd_mt19937_char_poly(uint64_t* out, size_t words) {
    const Field& F = field();
    if (!F.ok) return SD_ERR_UNSUPPORTED;
    if (!out || words < (size_t)kW + 1) return SD_ERR_INVALID;
    std::memcpy(out, F.P.data(), sizeof(uint64_t) * (kW + 1));
    return SD_OK;
}

}  // extern "C"

extern "C" {

/* Host restatement of the device fill's decomposition (csrc/mt_device.hip), for the CPU tests:
 * the block array arr[624] with the consumption position tau0 in [0, 624], n output words cut
 * into substreams of `stride` words, substream s >= 1 started by the jump polynomial table[s-1]
 * applied to windows of the base sequence.  out[o] = temper(x[tau0 + o]). */
int32_t sd_mt19937_fill_substreams(const uint32_t* arr, int32_t tau0, uint32_t* out, int64_t n, int64_t stride,
                                   const uint64_t* table, int32_t count) {
    if (!arr || tau0 < 0 || tau0 > kN || n < 0 || stride < kN || (n > 0 && !out)) return SD_ERR_INVALID;
    const int64_t S = n > 0 ? (n + stride - 1) / stride : 0;
    if (S > (int64_t)count + 1 || (S > 1 && !table)) return SD_ERR_INVALID;
    std::vector<uint32_t> base(arr, arr + kN);
    extend(base, (size_t)tau0 + kDeg + kN);
    for (int64_t s = 0; s < S; ++s) {
        std::vector<uint32_t> x(kN);
        if (s == 0) {
            std::memcpy(x.data(), base.data() + tau0, sizeof(uint32_t) * kN);
        } else {
            const uint64_t* c = table + (size_t)(s - 1) * SD_MT_JUMP_WORDS;
            std::fill(x.begin(), x.end(), 0u);
            for (long i = 0; i < kDeg; ++i)
                if (bit(c, i))
                    for (int j = 0; j < kN; ++j) x[j] ^= base[tau0 + 1 + i + j];
        }
        const int64_t lo = s * stride, hi = lo + stride < n ? lo + stride : n;
        extend(x, (size_t)(hi - lo));
        for (int64_t o = lo; o < hi; ++o) out[o] = temper(x[o - lo]);
    }
    return SD_OK;
}

}  // extern "C"
