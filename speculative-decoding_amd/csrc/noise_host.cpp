// noise_host.cpp — host-side mirror of torch's CPU generator (ATen mt19937) for the STREAM
// noise mode.  torch.Generator.get_state() serialises CPUGeneratorImplState (5056 bytes):
//   +0 int64 the_initial_seed, +8 int32 left, +12 int32 seeded, +16 uint64 next,
//   +24 uint64 state[624] (one 32-bit word per slot), +5016 normal-sample cache.
// The words produced here are exactly what torch.rand / exponential_ consume.
#include <cstring>

#include "specdec.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr size_t kStateBytes = 5056, kOffLeft = 8, kOffNext = 16, kOffState = 24;

struct Mt {
    uint32_t st[kN];
    int32_t left;
    uint32_t next;

    void twist() {
        for (int i = 0; i < kN; ++i) {
            const uint32_t y = (st[i] & 0x80000000u) | (st[(i + 1) % kN] & 0x7fffffffu);
            st[i] = st[(i + kM) % kN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        left = kN;
        next = 0;
    }
    uint32_t word() {
        if (--left == 0) twist();
        uint32_t y = st[next++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
};

bool load(Mt& m, const uint8_t* s, size_t len) {
    if (!s || len < kStateBytes) return false;
    std::memcpy(&m.left, s + kOffLeft, 4);
    uint64_t nx;
    std::memcpy(&nx, s + kOffNext, 8);
    if (m.left < 1 || m.left > kN || nx > (uint64_t)kN) return false;
    m.next = (uint32_t)nx;
    for (int i = 0; i < kN; ++i) {
        uint64_t w;
        std::memcpy(&w, s + kOffState + 8 * i, 8);
        m.st[i] = (uint32_t)w;
    }
    return true;
}

void store(const Mt& m, uint8_t* s) {
    std::memcpy(s + kOffLeft, &m.left, 4);
    const uint64_t nx = m.next;
    std::memcpy(s + kOffNext, &nx, 8);
    for (int i = 0; i < kN; ++i) {
        const uint64_t w = m.st[i];
        std::memcpy(s + kOffState + 8 * i, &w, 8);
    }
}

}  // namespace

extern "C" {

int32_t sd_mt19937_fill(const uint8_t* torch_state, size_t state_len, uint32_t* out, int64_t n) {
    Mt m;
    if (!load(m, torch_state, state_len) || n < 0 || (n > 0 && !out)) return SD_ERR_INVALID;
    for (int64_t i = 0; i < n; ++i) out[i] = m.word();
    return SD_OK;
}

/* torch state <-> the device generator's block + position (sd_mt_state, csrc/mt_device.hip).
 * torch twists lazily: left == 1 means the next word starts a new block (tau0 = 624); otherwise
 * the next word is state[next] and left == 625 - next. */
int32_t sd_mt19937_state_from_torch(const uint8_t* torch_state, size_t state_len, sd_mt_state* out) {
    Mt m;
    if (!out || !load(m, torch_state, state_len)) return SD_ERR_INVALID;
    if (m.left != 1 && m.left + (int32_t)m.next != kN + 1) return SD_ERR_INVALID;
    std::memcpy(out->mt, m.st, sizeof(m.st));
    out->tau0 = m.left == 1 ? kN : (int32_t)m.next;
    out->reserved[0] = out->reserved[1] = out->reserved[2] = 0;
    return SD_OK;
}

int32_t sd_mt19937_state_to_torch(const sd_mt_state* st, uint8_t* torch_state, size_t state_len) {
    Mt m;
    if (!st || !load(m, torch_state, state_len) || st->tau0 < 1 || st->tau0 > kN) return SD_ERR_INVALID;
    std::memcpy(m.st, st->mt, sizeof(m.st));
    m.next = (uint32_t)st->tau0;
    m.left = kN + 1 - st->tau0;
    store(m, torch_state);
    return SD_OK;
}

int32_t sd_mt19937_advance(uint8_t* torch_state, size_t state_len, int64_t n) {
    Mt m;
    if (!load(m, torch_state, state_len) || n < 0) return SD_ERR_INVALID;
    // whole blocks of 624 words: one twist each
    while (n > 0) {
        if (m.left > 1 && n >= m.left - 1) {     // consume the rest of the current block
            n -= m.left - 1;
            m.next += m.left - 1;
            m.left = 1;
        } else if (m.left == 1 && n >= kN) {
            m.twist();                             // left = 624, next = 0 -> emulate 624 draws
            m.left = 1;
            m.next = kN;
            n -= kN;
        } else {
            m.word();
            --n;
        }
    }
    store(m, torch_state);
    return SD_OK;
}

}  // extern "C"
