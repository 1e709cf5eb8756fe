// Host-side AddressSanitizer driver for the C ABI (SURVEY.md §5 "Race detection / sanitizers").
// Built by `make -C speculative-decoding_amd asan` from host-only objects (no device code, no GPU):
// every argument-validation path of the compute entry points, the workspace carving for many
// shapes, and the host mt19937 / jump-ahead code (torch state read from argv[1], words written to
// argv[2] for tests/test_asan_cpu.py to compare with torch).  Any ASan report aborts the run.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "specdec.h"

static int g_checks = 0, g_fail = 0;
#define CHECK(cond)                                                                  \
    do {                                                                             \
        ++g_checks;                                                                  \
        if (!(cond)) { ++g_fail; std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #cond); } \
    } while (0)

static void* fake(uintptr_t k) { return reinterpret_cast<void*>(0x100000 + 0x1000 * k); }   // never dereferenced

static void verify_rejections() {
    sd_verify_args a;
    std::memset(&a, 0, sizeof a);
    CHECK(sd_verify(nullptr, nullptr) == SD_ERR_INVALID);
    a.batch = 2; a.gamma = 4; a.vocab = 1000; a.rule = SD_RULE_SPEC;
    CHECK(sd_verify(&a, nullptr) == SD_ERR_INVALID);              // null rows / outputs
    for (int t = 0; t <= SD_MAX_GAMMA; ++t) a.target_rows[t] = fake(t);
    for (int t = 0; t < SD_MAX_GAMMA; ++t) a.draft_rows[t] = fake(20 + t);
    a.target_dtype = a.draft_dtype = SD_BF16;
    a.target_proc = a.draft_proc = sd_processor{SD_PROC_MULTINOMIAL, 1.f, 0, 1.f};
    a.draft_tokens = static_cast<const int64_t*>(fake(40));
    a.n_accepted = static_cast<int32_t*>(fake(41));
    a.next_token = static_cast<int64_t*>(fake(42));
    a.row_status = static_cast<int32_t*>(fake(43));
    a.noise.mode = SD_NOISE_PHILOX;
    CHECK(sd_verify(&a, nullptr) == SD_ERR_WORKSPACE);            // everything valid but the workspace
    const size_t need = sd_verify_workspace_size(2, 4, 1000);
    CHECK(need > 0);
    a.workspace = fake(50); a.workspace_bytes = need - 1;
    CHECK(sd_verify(&a, nullptr) == SD_ERR_WORKSPACE);
    sd_verify_args b = a;
    b.gamma = 0; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.gamma = SD_MAX_GAMMA + 1; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.vocab = 0; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.batch = -3; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.rule = 7; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.target_dtype = 9; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.target_proc.kind = 11; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.n_stop = 2; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);
    b = a; b.target_rows[4] = nullptr; CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);   // SPEC: γ+1 rows
    b = a; b.rule = SD_RULE_ENGINE; b.generated = static_cast<int64_t*>(fake(60));
    CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);            // engine state without finished / counts
    b = a; b.noise.mode = SD_NOISE_STREAM; b.noise.n_words = 10;
    CHECK(sd_verify(&b, nullptr) == SD_ERR_INVALID);            // stream words missing
}

static void sample_probs_rejections() {
    sd_sample_args s;
    std::memset(&s, 0, sizeof s);
    CHECK(sd_sample(nullptr, nullptr) == SD_ERR_INVALID);
    s.rows = 3; s.vocab = 5000; s.logits = fake(1); s.tokens = static_cast<int64_t*>(fake(2));
    s.dtype = SD_BF16; s.proc = sd_processor{SD_PROC_TOPK, 0.7f, 50, 1.f};
    s.noise.mode = SD_NOISE_PHILOX;
    CHECK(sd_sample(&s, nullptr) == SD_ERR_WORKSPACE);
    sd_sample_args t = s; t.proc.temperature = 0.f; CHECK(sd_sample(&t, nullptr) == SD_ERR_INVALID);
    t = s; t.dtype = -1; CHECK(sd_sample(&t, nullptr) == SD_ERR_INVALID);
    t = s; t.noise.mode = SD_NOISE_STREAM; CHECK(sd_sample(&t, nullptr) == SD_ERR_INVALID);
    sd_probs_args p;
    std::memset(&p, 0, sizeof p);
    CHECK(sd_probs(&p, nullptr) == SD_ERR_INVALID);
    p.rows = 2; p.vocab = 100; p.logits = fake(3); p.probs = fake(4); p.dtype = SD_F32;
    p.proc = sd_processor{SD_PROC_NUCLEUS, 1.f, 0, 0.9f};
    CHECK(sd_probs(&p, nullptr) == SD_ERR_WORKSPACE);
    sd_ngram_args n;
    std::memset(&n, 0, sizeof n);
    CHECK(sd_ngram_verify(&n, nullptr) == SD_ERR_INVALID);
    n.batch = 1; n.gamma = 3; n.vocab = 1000; n.filler_k = 9;
    CHECK(sd_ngram_verify(&n, nullptr) == SD_ERR_INVALID);
}

static void workspace_shapes() {
    const int32_t Bs[] = {1, 2, 31, 32, 512, 16384};
    const int32_t Vs[] = {1, 7, 2048, 50257, 128256, 262144};
    for (int32_t B : Bs)
        for (int32_t V : Vs) {
            for (int32_t g = 1; g <= SD_MAX_GAMMA; g += 5) {
                CHECK(sd_verify_workspace_size(B, g, V) > 0);
                CHECK(sd_ngram_workspace_size(B, g, V) > 0);
            }
            CHECK(sd_sample_workspace_size(B, V) > 0);
            CHECK(sd_probs_workspace_size(B, V) > 0);
        }
    CHECK(sd_verify_workspace_size(0, 4, 10) == 0);
    CHECK(sd_verify_workspace_size(1, SD_MAX_GAMMA + 1, 10) == 0);
    CHECK(sd_sample_workspace_size(1, 0) == 0);
}

static std::vector<uint8_t> read_file(const char* path) {
    std::vector<uint8_t> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    uint8_t buf[4096];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
    std::fclose(f);
    return v;
}

static void mt_host(const char* state_path, const char* out_path) {
    std::vector<uint8_t> st = read_file(state_path);
    CHECK(!st.empty());
    if (st.empty()) return;
    const int64_t n = 3 * 65536 + 1234;
    std::vector<uint32_t> words(n), again(n);
    CHECK(sd_mt19937_fill(st.data(), st.size(), words.data(), n) == SD_OK);
    CHECK(sd_mt19937_fill(st.data(), st.size() - 1, words.data(), n) != SD_OK);   // short state
    // the device path's host pieces: torch state <-> sd_mt_state, jump table, substreams
    sd_mt_state ms;
    CHECK(sd_mt19937_state_from_torch(st.data(), st.size(), &ms) == SD_OK);
    const int64_t stride = 65536;
    const int32_t count = 3;
    std::vector<uint64_t> table((size_t)count * SD_MT_JUMP_WORDS);
    CHECK(sd_mt19937_jump_table(stride, count, table.data()) == SD_OK);
    CHECK(sd_mt19937_fill_substreams(ms.mt, ms.tau0, again.data(), n, stride, table.data(), count) == SD_OK);
    CHECK(std::memcmp(words.data(), again.data(), n * sizeof(uint32_t)) == 0);
    std::vector<uint8_t> st2(st.size());
    std::memcpy(st2.data(), st.data(), st.size());
    CHECK(sd_mt19937_state_to_torch(&ms, st2.data(), st2.size()) == SD_OK);
    std::vector<uint32_t> w2(64);
    CHECK(sd_mt19937_fill(st2.data(), st2.size(), w2.data(), 64) == SD_OK);
    CHECK(std::memcmp(w2.data(), words.data(), 64 * sizeof(uint32_t)) == 0);
    // advance by k, then the next words are words[k..]
    CHECK(sd_mt19937_advance(st2.data(), st2.size(), 70001) == SD_OK);
    CHECK(sd_mt19937_fill(st2.data(), st2.size(), w2.data(), 64) == SD_OK);
    CHECK(std::memcmp(w2.data(), words.data() + 70001, 64 * sizeof(uint32_t)) == 0);
    std::vector<uint64_t> poly(313);
    CHECK(sd_mt19937_char_poly(poly.data(), poly.size()) == SD_OK);
    CHECK(sd_mt19937_char_poly(poly.data(), 10) != SD_OK);
    FILE* f = std::fopen(out_path, "wb");
    CHECK(f != nullptr);
    if (f) {
        std::fwrite(words.data(), sizeof(uint32_t), n, f);
        std::fclose(f);
    }
}

int main(int argc, char** argv) {
    CHECK(sd_abi_version() == SD_ABI_VERSION);
    verify_rejections();
    sample_probs_rejections();
    workspace_shapes();
    if (argc >= 3) mt_host(argv[1], argv[2]);
    std::printf("abi_asan: %d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
