/*
 * specdec.h — C ABI of the MI355X-native speculative verify/accept path.
 *
 * The reference (dadiaokua/speculative-decoding) is pure Python and has no FFI; this
 * library sits under the Python entry points it exposes for the hot path, which keep
 * their signatures (the specdec_amd Python package):
 *
 *   sd_verify      replaces the per-step verify block of
 *                    sampling/speculative_decoding.py:129-187   (rule SD_RULE_SPEC,   "A8")
 *                    engine/infer_engine.py:265-336             (rule SD_RULE_ENGINE, "A10")
 *                  including the processors it calls (utils/logits_processor.py:13-103),
 *                  max_fn (sampling/speculative_decoding.py:10-19) and the prune lengths fed
 *                  to utils/caching.py:6-24 (sampling/speculative_decoding.py:163-165).
 *   sd_sample      replaces LogitsProcessor.__call__ + .sample on the drafter / first-target
 *                  rows (sampling/speculative_decoding.py:95-96,120-123; engine/infer_engine.py:241-246).
 *   sd_mt19937_*   host-side mirror of torch's CPU generator (ATen mt19937) that feeds the
 *                  "stream" noise mode, so GPU results equal the reference's under a fixed
 *                  torch.manual_seed (torch.rand: engine/infer_engine.py:305,
 *                  sampling/speculative_decoding.py:139; torch.multinomial's Exp(1) noise).
 *
 * Conventions: all tensor pointers are device pointers (hipMalloc / torch CUDA memory);
 * the vocab axis has unit stride; other strides are in ELEMENTS.  Every entry point
 * returns SD_OK or a negative sd_status, never aborts, never allocates, never syncs the
 * host; kernels are enqueued on `stream` (a hipStream_t, passed as void*).  Per-row
 * failures (e.g. an all-zero residual under multinomial, which makes torch raise) are
 * reported in `row_status`, read back by the caller.
 */
#ifndef SPECDEC_H
#define SPECDEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SD_ABI_VERSION 11
#define SD_MAX_GAMMA 32          /* drafts per call; specdec_amd.ops chunks longer windows */
#define SD_NGRAM_MAX_FILLER 64   /* sd_ngram_verify filler ids per pass; filler_k itself may be
                                    anything up to vocab (ABI 11: one more launch pair per 64)  */

typedef enum {
    SD_OK = 0,
    SD_ERR_INVALID = -1,      /* bad argument (null pointer, bad shape, bad enum)        */
    SD_ERR_WORKSPACE = -2,    /* workspace too small (see sd_*_workspace_size)            */
    SD_ERR_LAUNCH = -3,       /* hipLaunchKernel / hip runtime error                      */
    SD_ERR_UNSUPPORTED = -4,  /* combination not implemented                              */
} sd_status;

typedef enum { SD_F32 = 0, SD_BF16 = 1, SD_F16 = 2 } sd_dtype;

/* utils/logits_processor.py: GreedyProcessor :26, MultinomialProcessor :39, TopKProcessor :52,
 * NucleusProcessor :66, TopKNucleusProcessor :84.                                          */
typedef enum {
    SD_PROC_GREEDY = 0,
    SD_PROC_MULTINOMIAL = 1,
    SD_PROC_TOPK = 2,
    SD_PROC_NUCLEUS = 3,
    SD_PROC_TOPK_NUCLEUS = 4,
} sd_proc_kind;

typedef struct {
    int32_t kind;         /* sd_proc_kind                       */
    float temperature;    /* LogitsProcessor.temperature        */
    int32_t top_k;        /* TopK*.top_k                         */
    float top_p;          /* Nucleus*.top_p                      */
} sd_processor;

typedef enum {
    SD_RULE_SPEC = 0,     /* sampling/speculative_decoding.py:139-171: accept iff r <= p/q (fp32),
                             bonus sample on full accept, (p-q)+ residual on reject           */
    SD_RULE_ENGINE = 1,   /* engine/infer_engine.py:287-336: accept iff u < min(1,p/q) (fp64),
                             q<=0 accepts, eos ends the row, no bonus, residual on reject     */
} sd_rule;

typedef enum {
    SD_NOISE_STREAM = 0,  /* words[] = mt19937 outputs of torch's CPU generator (parity mode) */
    SD_NOISE_PHILOX = 1,  /* in-kernel Philox4x32-10 keyed by seed, counter offset (perf mode) */
} sd_noise_mode;

typedef struct {
    int32_t mode;            /* sd_noise_mode                                                 */
    const uint32_t* words;   /* STREAM: device buffer of generator words, consumed from [0]   */
    int64_t n_words;         /* STREAM: capacity; overrun => row_status SD_ROW_NOISE_OVERRUN  */
    uint64_t seed;           /* PHILOX: key                                                   */
    uint64_t offset;         /* PHILOX: per-call counter offset (caller advances it)          */
    int64_t row_base;        /* PHILOX: global id of row 0 of this call — noise is keyed by
                                (seed, offset, global row), so a batch sharded across ranks
                                draws exactly what one call over the whole batch draws     */
    const uint64_t* offset_dev;  /* PHILOX (nullable): device uint64 added to `offset` when the
                                kernels run — a captured hipGraph replays with fresh noise once
                                the caller advances it on the device between replays        */
} sd_noise;

/* row_status bits */
#define SD_ROW_DONE           0x1   /* the row was processed                                  */
#define SD_ROW_STOP_IN_DRAFTS 0x2   /* SPEC: an accepted draft is a stop token: the reference
                                       returns before sampling (speculative_decoding.py:150-155);
                                       stop_index holds its draft position                   */
#define SD_ROW_FINISHED       0x4   /* ENGINE: the row hit an end token (infer_engine.py:310,328) */
#define SD_ROW_RESIDUAL       0x8   /* x was drawn from the (p-q)+ residual                    */
#define SD_ROW_BONUS          0x10  /* x was drawn from the bonus row (full accept, SPEC)      */
#define SD_ROW_FALLBACK_P     0x20  /* ENGINE: residual mass <= 1e-12, x drawn from p (:319-321);
                                       SPEC skip_sample_adjustment: x drawn from p_n (:169-170) */
#define SD_ROW_INVALID_DIST   0x40  /* multinomial over NaN/zero mass: torch raises RuntimeError */
#define SD_ROW_NOISE_OVERRUN  0x80  /* STREAM noise buffer too short                           */
#define SD_ROW_NUCLEUS_INEXACT 0x100 /* nucleus cut computed where fp32 cumsum rounding could not
                                       be reproduced exactly           */
#define SD_ROW_EXCHANGE_TIMEOUT 0x200 /* a workgroup's partial never arrived within the bounded
                                       wait of an in-launch exchange (k_draw_lean); the row's
                                       outputs are invalid (also flagged SD_ROW_INVALID_DIST)    */
/* The bits that make a row's outputs unusable: the reference raises in these cases (torch.multinomial
 * on NaN / inf / zero mass, engine/infer_engine.py:246,321-325; sampling/speculative_decoding.py:171),
 * so callers must treat them as errors, never as tokens.  Every entry point that takes a
 * `status_or` word ORs the error bits of each of its rows into it (one device atomic per failed
 * row; nothing on the success path), so a decode loop can test ONE word where it already syncs. */
#define SD_ROW_ERROR_MASK (SD_ROW_INVALID_DIST | SD_ROW_NOISE_OVERRUN | SD_ROW_EXCHANGE_TIMEOUT)

/* A top-k / nucleus row's keep predicate (the threshold search's result): token j is kept iff
 * x_j > tau || (x_j == tau && j <= tie_idx), x_j the row's logit (tau = -inf, tie_idx = INT_MAX
 * keeps all).  flags: SD_ROW_* bits the search raised (SD_ROW_NUCLEUS_INEXACT).  16 bytes.   */
typedef struct sd_row_keep {
    float tau;
    int32_t tie_idx;
    int32_t flags;
    int32_t reserved;
} sd_row_keep;

typedef struct {
    /* shape */
    int32_t batch;               /* B                                                         */
    int32_t gamma;               /* γ' (drafts verified this step), 1..SD_MAX_GAMMA           */
    int32_t vocab;               /* V                                                         */
    int32_t rule;                /* sd_rule                                                   */

    /* target logits: rows t = 0..gamma (gamma+1 rows; row gamma is the bonus row, read only
       under SD_RULE_SPEC).  Row t of sequence b is target_rows[t] + b * target_stride_b.     */
    const void* target_rows[SD_MAX_GAMMA + 1];
    int64_t target_stride_b;
    int32_t target_dtype;        /* sd_dtype                                                  */

    /* drafter: rows d = 0..gamma-1; logits (processed with draft_proc) or, when
       draft_is_probs, fp32 probabilities (the reference's q buffer).                         */
    const void* draft_rows[SD_MAX_GAMMA];
    int64_t draft_stride_b;
    int32_t draft_dtype;
    int32_t draft_is_probs;

    const int64_t* draft_tokens; /* [B, >=gamma] drafted ids                                  */
    int64_t draft_tokens_stride_b;

    sd_processor target_proc;    /* SPEC: the loop's logits_processor; ENGINE: plain softmax  */
    sd_processor draft_proc;

    int32_t skip_sample_adjustment;  /* SPEC: sample from p_n instead of max_fn(p_n - q_n)    */
    const int64_t* stop_tokens;      /* device [n_stop] eos ids (SPEC stop scan / ENGINE end)  */
    int32_t n_stop;

    const uint8_t* active;       /* ENGINE: [B] rows still generating (nullable = all)        */

    sd_noise noise;

    /* outputs, device, [B] */
    int32_t* n_accepted;         /* accepted drafts n                                         */
    int64_t* next_token;         /* token written at position cur+n (-1 if none)              */
    float* resample_mass;        /* Σ (p_n - q_n)+ when a residual was formed, else NaN        */
    int32_t* prune_drafter;      /* SPEC: γ'-n on reject, else 0 (utils/caching.py input)      */
    int32_t* prune_target;       /* SPEC: γ'-n+1 on reject, else 0                            */
    int32_t* stop_index;         /* SPEC: draft position of the first accepted stop token, -1  */
    int32_t* row_status;         /* SD_ROW_* bits                                             */
    int64_t* words_used;         /* STREAM: [1] words consumed by this call (nullable)         */

    /* optional in-place engine state (ENGINE rule; nullable): applies
       engine/infer_engine.py:307-336 on the device — generated[b, step+n] = x on reject,
       zero the tail, finished[b] |= end token, accepted[b] += n.                             */
    int64_t* generated;          /* [B, gen_len]                                              */
    int64_t generated_stride_b;
    int32_t step;
    uint8_t* finished;           /* [B]                                                       */
    int64_t* accepted_count;     /* [B]                                                       */

    void* workspace;
    size_t workspace_bytes;

    /* optional instrumentation: hipEvent_t recorded on `stream` right before / after the
       row-statistics kernel (the pass that reads every logit row once); nullable.  With the
       events set, the kernel is launched prof_stats_repeat (>= 1) times between them, back to
       back (every repeat rewrites the same partials and decisions), so the event pair's own
       cost is amortised over the repeats.                                                   */
    void* prof_stats_begin;
    void* prof_stats_end;
    int32_t prof_stats_repeat;

    /* optional (nullable): (max, Σexp) of each processed drafter row as sd_sample returned it
       with the draw (sd_sample_args.row_stats), pairs of floats; row d of sequence b at
       draft_row_stats + 2 * (d * draft_row_stats_stride + b), stride >= batch.  With it the
       row-statistics pass reads only the target rows — the drafter rows were read by their
       draws (sampling/speculative_decoding.py:120-123, engine/infer_engine.py:241-247) — and
       the residual still reads drafter row n.  A hint: ignored with draft_is_probs or a
       top-k / nucleus drafter processor.                                                      */
    const float* draft_row_stats;
    int64_t draft_row_stats_stride;
    /* optional (nullable, read only with draft_row_stats): the keep predicates of a top-k /
       nucleus drafter's rows as sd_sample returned them with the draws (sd_sample_args.row_keep),
       at draft_row_stats' layout: row d of sequence b at draft_row_keep[d * stride + b].  With
       both, the drafter rows are neither re-read for their statistics nor re-searched for their
       thresholds: the keep is a function of the row and draft_proc alone, so the draw's equals
       the one the verify would compute (utils/logits_processor.py:52-101).                    */
    const struct sd_row_keep* draft_row_keep;
    /* optional (nullable): device int32 [1]; the call ORs every row's SD_ROW_ERROR_MASK bits into
       it (never cleared by the library: the caller zeroes it, e.g. once per decode loop)        */
    int32_t* status_or;
    /* optional (nullable): device int64 [B, 2]; the call ADDS (accepted drafts n, tokens emitted)
       to row b's pair — emitted = n plus the resampled / bonus token when one was drawn.  The
       acceptance / throughput bookkeeping (engine/infer_engine.py:258,308; engine/metrics.py:100-129)
       kept on the device with no extra launch.                                                  */
    int64_t* row_counts;
} sd_verify_args;

typedef struct {
    int32_t rows;                /* R rows sampled independently                               */
    int32_t vocab;
    const void* logits;          /* row r at logits + r * stride_r                            */
    int64_t stride_r;
    int32_t dtype;
    sd_processor proc;
    sd_noise noise;              /* STREAM: torch.multinomial on [R, V]: 2 words per element   */
    int64_t* tokens;             /* [R] sampled ids (token r at tokens[r * tokens_stride])     */
    int64_t tokens_stride;
    float* token_prob;           /* [R] processed probability of the sampled id (nullable)     */
    int32_t* row_status;         /* [R] (nullable)                                             */
    int64_t* words_used;         /* [1] (nullable)                                             */
    void* workspace;
    size_t workspace_bytes;
    float* row_stats;            /* [R][2] (max, Σexp) of each processed row, the softmax
                                    normaliser pair sd_verify takes as draft_row_stats (nullable).
                                    PHILOX stochastic rows: ONE pass (k_draw) — each span draws
                                    its own candidate, the row's last workgroup picks the span  */
    struct sd_row_keep* row_keep; /* [R] keep predicate of each row under a top-k / nucleus
                                    processor, the input sd_verify takes as draft_row_keep
                                    (nullable; not written for other processors)               */
    int32_t* status_or;          /* [1] (nullable): every row's SD_ROW_ERROR_MASK bits ORed in    */
} sd_sample_args;

/* LogitsProcessor.__call__ (utils/logits_processor.py:13-15) materialised: probs = softmax(_process(l)/T)
 * in the logits dtype, row r written at probs + r * probs_stride_r.                        */
typedef struct {
    int32_t rows;
    int32_t vocab;
    const void* logits;
    int64_t stride_r;
    int32_t dtype;
    sd_processor proc;
    void* probs;
    int64_t probs_stride_r;
    void* workspace;
    size_t workspace_bytes;
} sd_probs_args;

int32_t sd_abi_version(void);
const char* sd_status_string(int32_t status);

/* In-launch exchanges.  Several kernels exchange per-row partials inside ONE launch by polling
 * tagged records ("poll mode"; k_draw_lean, k_draw_nuc, k_thr_hist, the k_stats / k_sample tails)
 * when the host's occupancy check says the whole grid is resident.  A grid that shares the GPU
 * with other work (another process, RCCL kernels, a side stream) may not be: the bounded polls
 * then flag rows SD_ROW_EXCHANGE_TIMEOUT.  allow_poll = 0 selects the arrival-counter exchanges
 * everywhere (no kernel waits on another workgroup); 1 (default) lets the occupancy check decide.
 * spin_limit bounds every poll in MICROSECONDS OF WALL CLOCK (ABI 11; the device's constant
 * 100 MHz s_memrealtime): 0 = the default 2,000,000 (2 s), < 0 = give up at once — a test hook
 * that forces the timeout path.  A grid that shares the GPU with a long kernel of another stream
 * therefore waits for that kernel (its producers are dispatched in order behind it) instead of
 * flagging rows; only a record that never comes costs the bound.  Process-wide; the environment
 * variables SD_POLL (0/1) and SD_POLL_SPIN_LIMIT set the initial values.                       */
int32_t sd_set_poll_policy(int32_t allow_poll, int32_t spin_limit);
int32_t sd_get_poll_policy(int32_t* allow_poll, int32_t* spin_limit);
const char* sd_last_hip_error(void);   /* hipGetErrorString of the last failed launch (this thread) */

/* Dispatch options (ABI 10, 11): switches between kernel paths that compute the same outputs, for
 * A/B runs and for tests that compare the paths.  Process-wide, set by the caller; no entry point
 * reads the environment (SD_POLL / SD_POLL_SPIN_LIMIT seed the poll policy once, at first use).
 * sd_set_option returns SD_ERR_INVALID for an unknown option or value.                        */
typedef enum {
    SD_OPT_FUSED_VERIFY = 1,    /* 1 (default): k_verify_fused for B >= 8; 2: any B; 0: never    */
    SD_OPT_LEAN_VERIFY = 2,     /* -1 (default): k_verify_lean for <= 8 sequences; 1: any batch
                                   the occupancy check admits; 0: never                           */
    SD_OPT_THRESHOLD_POLL = 3,  /* 1 (default): the top-k / nucleus search in one launch when its
                                   grid is resident; 0: the launch-per-phase design               */
    SD_OPT_DRAW_STREAM = 4,     /* 1 (default): STREAM multinomial draws in one pass
                                   (k_draw_stream); 0: statistics + race + finalize launches      */
    SD_OPT_FUSED_TICKET = 5,    /* ABI 11. -1 (default): k_verify_fused in ticket order (work items
                                   by arrival ticket: any batch, resident or not) for B >= 64 or a
                                   grid too big to be resident; 0: block-id order only (a grid
                                   that is not resident takes k_stats + k_sample); 1: always      */
    SD_OPT_DRAW_SPAN = 6,       /* ABI 11. 0 (default): k_draw_lean's span per workgroup chosen by
                                   the batch (2048 elements, more for large batches); 1 / 2 / 4:
                                   that many 2048-element stages per workgroup                    */
    SD_OPT_TICKET_LAG = 7,      /* ABI 11. 0 (default, 1): in the ticket-order fused verify, how many
                                   sequences of a label stream before an earlier one's samplers  */
    SD_OPT_SAMP_CHUNKS = 8,     /* ABI 11. 0 (default: 2, 4 in ticket order): 2048-element chunks each
                                   sampling workgroup of the fused verify draws; 2, 4 or 8 pin it
                                   (the same chunks and draws whatever the grouping)              */
} sd_option;
int32_t sd_set_option(int32_t option, int32_t value);
int32_t sd_get_option(int32_t option, int32_t* value);

/* The kernel path the CALLING THREAD's last successful sd_verify / sd_sample took (so a test or a
 * bench can tell which kernel it measured without reading the dispatch rules).                 */
typedef enum {
    SD_PATH_NONE = 0,
    SD_PATH_VERIFY_LEAN = 1,        /* k_verify_lean: one launch, <= 8 sequences                 */
    SD_PATH_VERIFY_FUSED = 2,       /* k_verify_fused: one launch                                 */
    SD_PATH_VERIFY_TWO_LAUNCH = 3,  /* k_stats (+ decider) then k_sample                          */
    SD_PATH_VERIFY_STREAM = 4,      /* STREAM: k_stats, k_decide, k_walk, k_resample, k_finalize  */
    SD_PATH_VERIFY_FUSED_TICKET = 5,/* k_verify_fused in ticket order (ABI 11): one launch, any B  */
    SD_PATH_SAMPLE_DRAW_LEAN = 16,  /* k_draw_lean (PHILOX multinomial, T = 1, 16-bit)           */
    SD_PATH_SAMPLE_DRAW = 17,       /* k_draw (PHILOX, processors / fp32)                          */
    SD_PATH_SAMPLE_NUCLEUS = 18,    /* k_draw_nuc (PHILOX nucleus by rejection)                    */
    SD_PATH_SAMPLE_STREAM = 19,     /* k_draw_stream (STREAM one pass)                             */
    SD_PATH_SAMPLE_GREEDY_LEAN = 20,/* k_draw_lean<GREEDY>                                          */
    SD_PATH_SAMPLE_MULTI = 21,      /* row statistics + k_rowsample + k_sample_finalize            */
} sd_path;
int32_t sd_last_verify_path(void);
int32_t sd_last_sample_path(void);

/* Workspaces: device memory of at least sd_*_workspace_size bytes, ZERO-FILLED ONCE when
 * allocated (hipMemset).  Its first block holds per-sequence arrival counters that the PHILOX
 * verify path uses to run each sequence's decision / sampling in the last workgroup to finish;
 * every call leaves them at zero again, so one workspace can serve any sequence of
 * sd_verify / sd_sample / sd_probs calls on one stream (not concurrent calls).
 * PHILOX verify supports batch <= 16384 per call (SD_ERR_UNSUPPORTED beyond).
 *
 * PHILOX sampling draws the residual / bonus / p-row token by inverse CDF on one Philox U[0,1)
 * (53 bits) per row: distributionally the reference's multinomial, not its bit stream.  Greedy
 * rows are bit-exact in both noise modes; STREAM mode reproduces torch's CPU draws exactly.  */
size_t sd_verify_workspace_size(int32_t batch, int32_t gamma, int32_t vocab);
int32_t sd_verify(const sd_verify_args* args, void* stream);

size_t sd_sample_workspace_size(int32_t rows, int32_t vocab);
int32_t sd_sample(const sd_sample_args* args, void* stream);

size_t sd_probs_workspace_size(int32_t rows, int32_t vocab);
int32_t sd_probs(const sd_probs_args* args, void* stream);

/* The n-gram-assisted verify step (rule A11, ngram_assisted/ngram_assisted.py:111-164): sample-
 * and-compare of γ' drafts against the processed target rows, then an independent draw x from the
 * mismatch row (or the bonus row), no residual.  STREAM noise follows the reference's draw order
 * (one full-row Exp draw per compare sample, then x: words_used = draws × 2V); filler ids =
 * topk(filler_k) of every processed row (lowest index first among equal probabilities).        */
typedef struct {
    int32_t batch;               /* B (the reference is batch 1)                               */
    int32_t gamma;               /* γ' drafts, 0..SD_MAX_GAMMA                                  */
    int32_t vocab;
    const void* target_rows[SD_MAX_GAMMA + 1];   /* rows 0..γ'-1 verify draft i, row γ' = bonus */
    int64_t target_stride_b;
    int32_t target_dtype;
    const int64_t* draft_tokens; /* [B, >=γ']                                                  */
    int64_t draft_tokens_stride_b;
    sd_processor proc;           /* the loop's logits_processor                                */
    const int64_t* stop_tokens;
    int32_t n_stop;
    int32_t filler_k;            /* 0..vocab (ABI 11; p.topk(filler_top_k), any k)             */
    sd_noise noise;
    /* outputs, device */
    int32_t* n_accepted;         /* [B] n                                                      */
    int64_t* next_token;         /* [B] x, -1 when a stop token among the accepted drafts ends  */
    int32_t* prune_target;       /* [B] γ'-n+1 on a mismatch (:139-141), else 0                 */
    int32_t* stop_index;         /* [B] first accepted stop draft, -1                           */
    int32_t* row_status;         /* [B] SD_ROW_* (BONUS: x from the bonus row; FALLBACK_P: p_n) */
    int64_t* words_used;         /* [1] STREAM words consumed (batch 1 semantics)               */
    int64_t* filler_ids;         /* [B, γ'+1, filler_k] at + b * filler_stride_b + i * filler_k */
    int64_t filler_stride_b;
    void* workspace;
    size_t workspace_bytes;
    int32_t* status_or;          /* [1] (nullable): every row's SD_ROW_ERROR_MASK bits ORed in    */
} sd_ngram_args;

size_t sd_ngram_workspace_size(int32_t batch, int32_t gamma, int32_t vocab);
int32_t sd_ngram_verify(const sd_ngram_args* args, void* stream);

/* Device n-gram drafter store under the reference's OneLevelNGramStorage /
 * NGramStorage (ngram_assisted/ngram_storage.py:71-249): initialize / update / next_token /
 * has_gram keep their meaning; the host keeps the record clock (ts) and the fallback draws.
 *   sd_ngram_store_initialize  replaces ngram_storage.py:128-142 (one level), 227-243 (all orders)
 *   sd_ngram_store_update      replaces ngram_storage.py:106-126, 196-217
 *   sd_ngram_store_next_token  replaces ngram_storage.py:76-90, 162-177 (out[] holds the caller's
 *                              torch.randint fallback draws on entry, overwritten for known grams)
 *   sd_ngram_store_has_gram    replaces ngram_storage.py:92-102, 179-194 (writes 0/1 to *out)
 *   sd_ngram_store_draft       replaces the loop's gamma chained next_token calls
 *                              (ngram_assisted/ngram_assisted.py:94-101): drafts[b, k] and known[b, k]
 *                              (known: [B, gamma] contiguous) for the history extended by drafts
 *                              0..k-1; fallback[b, k] = the k-th call's torch.randint draw
 * Records are stamped ts = ts_base + their index in the reference's processing order (initialize:
 * b * len + i; update: b * k + j); the caller advances ts_base by batch * len / batch * k after
 * each call.  Tables: caller-owned device memory, zero-filled once, capacities powers of two.
 * Token ids must lie in [0, 2^17), n in [2, SD_NGRAM_MAX_N]; a full table or a bad token sets a
 * bit in *status (the call still returns SD_OK: the condition is found on the device).          */
#define SD_NGRAM_MAX_N 4
#define SD_NGRAM_FULL 1
#define SD_NGRAM_BAD_TOKEN 2
typedef struct {
    uint64_t* gram_keys;         /* [gram_capacity] 0 = empty                                   */
    uint64_t* gram_best;         /* [gram_capacity] count<<44 | (2^27-1-ts)<<17 | token           */
    int64_t gram_capacity;
    uint64_t* pair_keys;         /* [pair_capacity] (gram slot, token)                            */
    uint32_t* pair_count;        /* [pair_capacity]                                               */
    uint32_t* pair_ts;           /* [pair_capacity] latest record ts                              */
    int64_t pair_capacity;
    int32_t* status;             /* [1] SD_NGRAM_* bits                                           */
    int32_t n;                   /* the reference's n                                             */
    int32_t one_level;           /* 1: OneLevelNGramStorage, 0: NGramStorage                      */
    int32_t vocab;               /* <= 2^17                                                       */
} sd_ngram_store;

int32_t sd_ngram_store_initialize(const sd_ngram_store* store, const int64_t* ids, int32_t batch, int32_t len,
                                  int64_t stride_b, int64_t ts_base, void* stream);
int32_t sd_ngram_store_update(const sd_ngram_store* store, const int64_t* ids, int32_t batch, int32_t len,
                              int64_t stride_b, const int64_t* next_tokens, int32_t k, int64_t next_stride_b,
                              int64_t ts_base, void* stream);
int32_t sd_ngram_store_next_token(const sd_ngram_store* store, const int64_t* ids, int32_t batch, int32_t len,
                                  int64_t stride_b, int64_t* out, uint8_t* known, void* stream);
int32_t sd_ngram_store_draft(const sd_ngram_store* store, const int64_t* ids, int32_t batch, int32_t len,
                             int64_t stride_b, int32_t gamma, const int64_t* fallback, int64_t fallback_stride_b,
                             int64_t* drafts, int64_t drafts_stride_b, uint8_t* known, void* stream);
int32_t sd_ngram_store_has_gram(const sd_ngram_store* store, const int64_t* ngram, int32_t len, uint8_t* out,
                                void* stream);

/* Host side: torch CPU generator state (torch.Generator.get_state(), 5056 bytes) <-> words. */
int32_t sd_mt19937_fill(const uint8_t* torch_state, size_t state_len, uint32_t* out, int64_t n);
int32_t sd_mt19937_advance(uint8_t* torch_state, size_t state_len, int64_t n);

/* ---- STREAM noise generated on the device (csrc/mt_device.hip, csrc/mt_jump.cpp) ----------------
 * The same words as sd_mt19937_fill, produced by the GPU: the generator state lives in device
 * memory as an sd_mt_state (the current 624-word block of untempered words and the position tau0
 * in [0, 624] of the next word to consume; tau0 = 624 means the next word starts a new block).
 * sd_mt19937_generate writes the next n words (tempered, as torch.rand / exponential_ read them)
 * WITHOUT moving the state; sd_mt19937_commit then moves it past the words a consumer used — a
 * host count, or the device int64 a verify kernel wrote to words_used (no host sync).  A fill is
 * cut into substreams of stride_words words; substream s >= 1 starts at a jump of s*stride_words
 * words, given by jump polynomial s-1 of a table from sd_mt19937_jump_table (host; copy it to the
 * device once per stride).  Replaces the host-thread generation behind torch.rand
 * (sampling/speculative_decoding.py:139, engine/infer_engine.py:305) and torch.multinomial's
 * Exp(1) noise (utils/logits_processor.py:48-49, engine/infer_engine.py:246,322-324). */
#define SD_MT_JUMP_WORDS 320   /* uint64 per jump polynomial (degree < 19937, zero-padded)        */
#define SD_MT_JUMP_CHUNKS 16   /* polynomial bit chunks per jump (one wave each)                 */

typedef struct {
    uint32_t mt[624];      /* the current block x[624 b .. 624 b + 623], untempered               */
    int32_t tau0;          /* next word = x[624 b + tau0]; 624: the next word starts block b + 1   */
    int32_t reserved[3];
} sd_mt_state;

typedef struct {
    sd_mt_state* state;          /* device                                                     */
    const uint64_t* jump_table;  /* device, jump_count * SD_MT_JUMP_WORDS                     */
    int32_t jump_count;          /* >= ceil(n_words / stride_words) - 1                       */
    int64_t stride_words;        /* >= 624; the table's stride                                */
    uint32_t* words;             /* device out, n_words                                      */
    int64_t n_words;
    void* workspace;             /* device, sd_mt19937_generate_workspace_size bytes          */
    size_t workspace_bytes;
} sd_mt_generate_args;

/* host */
int32_t sd_mt19937_state_from_torch(const uint8_t* torch_state, size_t state_len, sd_mt_state* out);
int32_t sd_mt19937_state_to_torch(const sd_mt_state* state, uint8_t* torch_state, size_t state_len);
int32_t sd_mt19937_jump_table(int64_t stride_words, int32_t count, uint64_t* out);  /* count * SD_MT_JUMP_WORDS */
int32_t sd_mt19937_char_poly(uint64_t* out, size_t words);                         /* >= 313 words           */
int32_t sd_mt19937_fill_substreams(const uint32_t* block, int32_t tau0, uint32_t* out, int64_t n,
                                   int64_t stride_words, const uint64_t* table, int32_t count);
/* device.  sd_mt19937_commit moves the state past `used` + *used_dev words (used_dev nullable): a
 * host-known prefix (e.g. the draws of an engine window, 2·B·V words each) plus the count a verify
 * wrote on the device.                                                                           */
size_t sd_mt19937_generate_workspace_size(int64_t n_words, int64_t stride_words);
int32_t sd_mt19937_generate(const sd_mt_generate_args* args, void* stream);
int32_t sd_mt19937_commit(sd_mt_state* state, const uint32_t* words, int64_t n_words, const int64_t* used_dev,
                          int64_t used, int32_t* status, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SPECDEC_H */
