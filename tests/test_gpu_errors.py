"""The reference's error contract on the GPU path, and the in-launch exchange policy.

Where the reference's torch.multinomial raises — NaN / inf / all-zero probabilities
(engine/infer_engine.py:246,321-325; sampling/speculative_decoding.py:96,123,171;
ngram_assisted/ngram_assisted.py:89,117,141) — the drop-ins raise too, and
run_batch_speculative returns None as the reference's does (:144-146).  The kernels OR every
failed row's SD_ROW_ERROR_MASK bits into one device word (`status_or`) that the loops read where
they already sync; a failed draw's -1 never reaches a forward.

The in-launch exchange policy (sd_set_poll_policy): a forced poll timeout (spin limit < 0)
surfaces as an exception, never as tokens; with polling switched off (the counter exchanges) the
same calls return exactly what the poll-mode kernels return, and the keep sets of the threshold
kernels stay exact when every slice's poll gives up (the row-uniform radix hand-over).
"""
import contextlib
import dataclasses
from types import SimpleNamespace

import pytest
import torch

from fakelm import FakeLM, make_pair
from oracle import specdec_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@contextlib.contextmanager
def poll_policy(allow, spin):
    from specdec_amd import get_poll_policy, set_poll_policy
    old = get_poll_policy()
    set_poll_policy(allow, spin)
    try:
        yield
    finally:
        set_poll_policy(*old)


def nan_pair(V=4096, where="drafter"):
    target, drafter = make_pair(V, dtype=torch.bfloat16, device=DEV, pos_mult=0)
    lm = drafter if where == "drafter" else target
    lm.bank[:, 0] = float("nan")                    # every row: softmax NaN -> torch.multinomial raises
    return target, drafter


def engine_ctx(target, drafter, gamma=4, gen_len=16, graph=False):
    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=gamma, gen_len=gen_len, end_tokens=[1])
    if graph:
        K = target.bank.shape[0]
        ctx.drafter_step = lambda prev, d, step_dev: drafter.bank[(prev * 31) % K]
        ctx.target_rows = lambda tokens, step_dev: target.bank[(tokens * 31) % K]
    return ctx


def prompt(B=6, V=4096, seed=11):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(3, V, (B, 6), generator=g).to(DEV)


@pytest.mark.parametrize("mode", ["stream", "philox", "philox-graph"])
def test_engine_invalid_drafter_distribution_returns_none(mode):
    """A NaN drafter row: the reference's multinomial(q) raises (:246) and run_batch_speculative
    returns None (:144-146)."""
    from specdec_amd import RowError, set_noise_mode
    from specdec_amd.engine.infer_engine import batch_speculative_generate, run_batch_speculative
    target, drafter = nan_pair(where="drafter")
    ids = prompt()
    ctx = engine_ctx(target, drafter, graph=mode == "philox-graph")
    set_noise_mode("stream" if mode == "stream" else "philox", seed=3)
    try:
        with pytest.raises(RowError, match="nan"):
            batch_speculative_generate(ctx, ids, torch.ones_like(ids), ids.shape[0])
        assert run_batch_speculative(ctx, ids, torch.ones_like(ids), ids.shape[0]) is None   # :144-146
    finally:
        set_noise_mode("stream")
    torch.cuda.synchronize()   # no device fault was left behind (a -1 never reached an embedding)


@pytest.mark.parametrize("mode", ["stream", "philox"])
def test_engine_nan_target_accepts_like_the_reference(mode):
    """A NaN target row does NOT raise in the reference's engine: accept_prob = min(1.0, nan) is
    1.0 in Python (:303), so every draft is accepted and no residual is ever drawn.  The fp64
    accept test here is fmin(1, p/q) — also 1 for a NaN ratio — so the drop-in decodes the same
    way: no error, every row's acceptance rate 1.0, the drafts are the output."""
    from specdec_amd import set_noise_mode
    from specdec_amd.engine.infer_engine import run_batch_speculative
    target, drafter = nan_pair(where="target")
    ids = prompt()
    ctx = engine_ctx(target, drafter)
    set_noise_mode("stream" if mode == "stream" else "philox", seed=3)
    try:
        bm = run_batch_speculative(ctx, ids, torch.ones_like(ids), ids.shape[0])
    finally:
        set_noise_mode("stream")
    assert bm is not None
    assert all(r.acceptance_rate == 1.0 for r in bm.requests)


@pytest.mark.parametrize("mode", ["stream", "philox"])
@pytest.mark.parametrize("where", ["drafter", "target"])
def test_speculative_generate_raises_like_torch(mode, where):
    from specdec_amd import RowError, set_noise_mode
    from specdec_amd.sampling import speculative_generate
    from specdec_amd.utils.logits_processor import MultinomialProcessor
    target, drafter = nan_pair(where=where)
    set_noise_mode("stream" if mode == "stream" else "philox", seed=3)
    try:
        with pytest.raises(RowError, match="nan"):
            speculative_generate([5, 9, 13], drafter, target, gamma=4, logits_processor=MultinomialProcessor(1.0),
                                 max_gen_len=12, first_target=where == "drafter")
    finally:
        set_noise_mode("stream")
    torch.cuda.synchronize()


@pytest.mark.parametrize("kind", ["multinomial", "nucleus"])
def test_ngram_loop_raises_like_torch(kind):
    """A NaN column in the target bank (under a nucleus processor: masked by the cut in most rows,
    but torch's processed row is NaN all the same)."""
    from specdec_amd import RowError, set_noise_mode
    from specdec_amd.ngram_assisted import NGramStorage, ngram_assisted_speculative_generate
    from specdec_amd.utils.logits_processor import MultinomialProcessor, NucleusProcessor
    target, _ = nan_pair(where="target")
    proc = MultinomialProcessor(1.0) if kind == "multinomial" else NucleusProcessor(1.0, 0.9)
    set_noise_mode("stream")
    with pytest.raises(RowError, match="nan"):
        ngram_assisted_speculative_generate([5, 9, 13, 5, 9], NGramStorage(n=3, vocab_size=4096), target, gamma=4,
                                            logits_processor=proc, max_gen_len=10)


@pytest.mark.parametrize("graph", [False, True])
def test_forced_poll_timeout_raises_not_tokens(graph):
    """spin limit < 0: every in-launch poll gives up at once.  The engine's Philox draws (k_draw_lean,
    poll mode at this batch) flag their rows SD_ROW_EXCHANGE_TIMEOUT; the loop raises, and
    run_batch_speculative returns None."""
    from specdec_amd import RowError, set_noise_mode
    from specdec_amd.engine.infer_engine import batch_speculative_generate, run_batch_speculative
    target, drafter = make_pair(4096, dtype=torch.bfloat16, device=DEV, pos_mult=0)
    ids = prompt()
    ctx = engine_ctx(target, drafter, graph=graph)
    set_noise_mode("philox", seed=8)
    try:
        with poll_policy(True, -1):
            with pytest.raises(RowError, match="exchange timed out"):
                batch_speculative_generate(ctx, ids, torch.ones_like(ids), ids.shape[0])
            assert run_batch_speculative(ctx, ids, torch.ones_like(ids), ids.shape[0]) is None
    finally:
        set_noise_mode("stream")


@pytest.mark.parametrize("kind", ["multinomial", "greedy"])
def test_counter_exchanges_equal_poll_mode(kind):
    """allow_poll = 0 (the residency-safe mode a shared GPU needs): every exchange uses arrival
    counters, and the draws, row stats and verify outputs equal the poll-mode kernels' exactly —
    even with a spin limit that would make any poll give up."""
    from specdec_amd import PhiloxNoise, _lib, ops
    g = torch.Generator(device=DEV).manual_seed(21)
    B, gm, V = 16, 4, 128256
    tl = (torch.randn(B, gm, V, generator=g, device=DEV) * 3).to(torch.bfloat16)
    dl = (tl.float() + torch.randn(B, gm, V, generator=g, device=DEV)).to(torch.bfloat16)
    spec = ops.ProcSpec(kind, 1.0)

    def run():
        noise = PhiloxNoise(seed=99)
        draft = torch.zeros(B, gm, dtype=torch.long, device=DEV)
        stats = torch.zeros(gm, B, 2, device=DEV)
        sts = []
        for d in range(gm):
            _, _, st = ops.sample_rows(dl[:, d], spec, noise, tokens_out=draft[:, d],
                                       row_stats_out=None if spec.keeps else stats[d])
            sts.append(st)
        out = ops.verify([tl[:, t] for t in range(gm)], [dl[:, t] for t in range(gm)], draft, _lib.SD_RULE_ENGINE,
                         spec, spec, noise, draft_row_stats=None if spec.keeps else stats)
        torch.cuda.synchronize()
        return draft.cpu(), stats.cpu(), torch.stack(sts).cpu(), out.n_accepted.cpu(), out.next_token.cpu()

    want = run()
    with poll_policy(False, -1):
        got = run()
    for a, b in zip(want, got):
        assert torch.equal(a, b)
    assert not (want[2] & _lib.SD_ROW_ERROR_MASK).any()


def test_thresholds_exact_when_every_slice_poll_gives_up(monkeypatch):
    """k_thr_hist in poll mode with every slice-max poll giving up: every slice skips its histogram
    flush and the row takes the radix descent — the keep sets still equal the exact oracle (a
    row is never cut from a partial histogram)."""
    from specdec_amd import _lib, ops
    assert _lib.get_option(_lib.SD_OPT_THRESHOLD_POLL) == 1
    g = torch.Generator().manual_seed(4)
    rows = (torch.randn(3, 128256, generator=g) * 3).to(torch.bfloat16)
    for proc in (ref.Processor("nucleus", 1.0, 0, 0.9), ref.Processor("topk", 1.0, 50)):
        spec = ops.ProcSpec(proc.kind, 1.0, proc.top_k, proc.top_p)
        with poll_policy(True, -1):
            got = ops.probs_rows(rows.cuda(), spec).float().cpu() > 0
        exact = dataclasses.replace(proc, stable_ties=True)
        for r in range(rows.shape[0]):
            want = ref.process(rows[r:r + 1], exact, exact=True)[0].float() > 0
            assert torch.equal(got[r], want), (proc.kind, r)


def test_status_or_collects_only_error_bits():
    from specdec_amd import PhiloxNoise, _lib, ops
    x = (torch.randn(8, 4096, device=DEV) * 3).to(torch.bfloat16)
    x[3, 17] = float("nan")
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    _, _, st = ops.sample_rows(x, ops.PLAIN_SOFTMAX, PhiloxNoise(seed=1), status_or=err)
    st = st.cpu()
    assert st[3] & _lib.SD_ROW_INVALID_DIST
    assert not (st[torch.arange(8) != 3] & _lib.SD_ROW_ERROR_MASK).any()
    assert int(err.item()) == _lib.SD_ROW_INVALID_DIST
    with pytest.raises(ValueError):
        ops.sample_rows(x, ops.PLAIN_SOFTMAX, PhiloxNoise(seed=1), status_or=err.long())


@pytest.mark.parametrize("block", [(5 * 2048, 512), (7 * 2048 + 1536, 512), (3 * 2048, 2048)])
def test_nan_block_flags_like_a_nan_row(block):
    """A run of NaN logits covering one wave's elements (or a whole span) of a 128256-wide row: the
    draws flag the row (torch.multinomial raises on its NaN softmax),
    and the batch-1 one-launch verify treats a target row with such a block exactly as a row that
    is NaN throughout (its softmax is NaN either way)."""
    from specdec_amd import PhiloxNoise, StreamNoise, _lib, ops
    V, g = 128256, 4
    gen = torch.Generator().manual_seed(5)
    tl = (torch.randn(1, g + 1, V, generator=gen) * 3).to(torch.bfloat16)
    dl = (tl[:, :g].float() + torch.randn(1, g, V, generator=gen)).to(torch.bfloat16)
    tl, dl = tl.to(DEV), dl.to(DEV)
    off, n = block
    # (plain rows in both noise modes; nucleus rows through the Philox rejection draw; the masked
    # NaN under a top-k / nucleus keep: test_nan_under_keep_is_a_nan_row below)
    cases = [(ops.PLAIN_SOFTMAX, PhiloxNoise(seed=3)), (ops.PLAIN_SOFTMAX, StreamNoise(torch.Generator().manual_seed(3))),
             (ops.ProcSpec("nucleus", 1.0, 0, 0.9), PhiloxNoise(seed=3))]
    for spec, noise in cases:
        x = torch.cat([dl[:, 0], dl[:, 1]]).contiguous()
        x[0, off:off + n] = float("nan")
        _, _, st = ops.sample_rows(x, spec, noise)
        st = st.cpu()
        what = (spec.kind, type(noise).__name__, int(st[0]), int(st[1]))
        assert st[0] & _lib.SD_ROW_INVALID_DIST, what
        assert not st[1] & _lib.SD_ROW_ERROR_MASK, what

    def run(trows):
        stats = torch.empty(g, 1, 2, dtype=torch.float32, device=DEV)
        ids = torch.empty(1, g, dtype=torch.long, device=DEV)
        noise = PhiloxNoise(seed=9)
        for d in range(g):
            tok, _, _ = ops.sample_rows(dl[:, d], ops.PLAIN_SOFTMAX, noise, row_stats_out=stats[d])
            ids[:, d] = tok
        return ops.verify([trows[:, t] for t in range(g + 1)], [dl[:, d] for d in range(g)], ids,
                          _lib.SD_RULE_SPEC, ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX,
                          PhiloxNoise(seed=9, offset=noise.offset), draft_row_stats=stats)

    for slot in (0, g):
        tb, tw = tl.clone(), tl.clone()
        tb[0, slot, off:off + n] = float("nan")
        tw[0, slot, :] = float("nan")
        a, b = run(tb), run(tw)
        mask = _lib.SD_ROW_ERROR_MASK
        assert int(a.row_status[0]) & mask == int(b.row_status[0]) & mask, (slot, int(a.row_status[0]), int(b.row_status[0]))
        assert int(a.n_accepted[0]) == int(b.n_accepted[0]), slot


@pytest.mark.parametrize("fill", ["nan", "-inf"])
def test_stream_race_invalid_row_token_is_minus_one(fill):
    """The STREAM three-launch draw (T != 1 takes it): an all-NaN or all -inf row has no race
    candidate at all.  torch.multinomial raises on it; here the row is flagged invalid and its token
    is -1 (never an index past the vocabulary that a clamp(min=0) would let into a forward)."""
    from specdec_amd import StreamNoise, _lib, ops
    x = (torch.randn(3, 4096, device=DEV) * 3).to(torch.bfloat16)
    x[1] = float(fill)
    tok, _, st = ops.sample_rows(x, ops.ProcSpec("multinomial", 0.7), StreamNoise(torch.Generator().manual_seed(2)))
    tok, st = tok.cpu(), st.cpu()
    assert int(tok[1]) == -1 and st[1] & _lib.SD_ROW_INVALID_DIST
    assert all(0 <= int(tok[r]) < 4096 for r in (0, 2))
    assert not (st[torch.tensor([0, 2])] & _lib.SD_ROW_ERROR_MASK).any()


KEEP_PROCS = [("topk", 1.0, 50, 0.0), ("nucleus", 1.0, 0, 0.9), ("topknucleus", 1.0, 50, 0.9), ("topk", 0.7, 50, 0.0),
              ("nucleus", 0.7, 0, 0.9)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("fill", ["nan", "inf"])
def test_nan_under_keep_is_a_nan_row(dtype, fill):
    """A NaN or +inf logit that the top-k / nucleus cut would mask out: torch's topk / sort rank it
    first (NaN) or keep it (+inf, whose softmax is NaN), so the reference's processed row is NaN
    throughout and torch.multinomial raises on it (utils/logits_processor.py:59-63,73-81; checked on
    the oracle below).  The HIP path: sd_probs returns an all-NaN row, every draw of it — both noise
    modes, the threshold path and the Philox rejection draw — is SD_ROW_INVALID_DIST with token -1,
    and the verify treats such a target row exactly as a NaN row; the clean row beside it is
    untouched."""
    from specdec_amd import PhiloxNoise, StreamNoise, _lib, ops
    V, g = 128256, 4
    gen = torch.Generator().manual_seed(31)
    x = (torch.randn(2, V, generator=gen) * 3).to(dtype)
    lo = int(x[0].float().argmin())                  # far below any cut: masked by every processor
    x[0, lo] = float(fill)
    for kind, T, k, p in KEEP_PROCS:
        proc = ref.Processor(kind, T, k, p)
        want = ref.process(x[:1], proc)
        assert want.isnan().all(), kind                  # the reference's processed row is NaN
        spec = ops.ProcSpec(kind, T, k, p)
        got = ops.probs_rows(x.to(DEV), spec).float().cpu()
        assert got[0].isnan().all(), (kind, T)
        assert not got[1].isnan().any(), (kind, T)
        for noise in (PhiloxNoise(seed=5), StreamNoise(torch.Generator().manual_seed(5))):
            tok, _, st = ops.sample_rows(x.to(DEV), spec, noise)
            tok, st = tok.cpu(), st.cpu()
            what = (kind, T, type(noise).__name__, int(st[0]), int(tok[0]))
            assert st[0] & _lib.SD_ROW_INVALID_DIST and int(tok[0]) == -1, what
            assert not st[1] & _lib.SD_ROW_ERROR_MASK and 0 <= int(tok[1]) < V, what

    # the verify: a target row with the masked NaN / inf equals a NaN row (status and accept count)
    if dtype != torch.bfloat16:
        return
    tl = (torch.randn(1, g + 1, V, generator=gen) * 3).to(dtype)
    dl = (tl[:, :g].float() + torch.randn(1, g, V, generator=gen)).to(dtype)
    tl, dl = tl.to(DEV), dl.to(DEV)
    for kind, T, k, p in KEEP_PROCS[:3]:
        spec = ops.ProcSpec(kind, T, k, p)
        for mode in ("philox", "stream"):
            def run(trows):
                noise = PhiloxNoise(seed=9) if mode == "philox" else StreamNoise(torch.Generator().manual_seed(9))
                ids = torch.empty(1, g, dtype=torch.long, device=DEV)
                for d in range(g):
                    tok, _, _ = ops.sample_rows(dl[:, d], spec, noise)
                    ids[:, d] = tok
                return ops.verify([trows[:, t] for t in range(g + 1)], [dl[:, d] for d in range(g)], ids,
                                  _lib.SD_RULE_SPEC, spec, spec, noise)
            for slot in (0, g):
                tb, tw = tl.clone(), tl.clone()
                tb[0, slot, int(tl[0, slot].float().argmin())] = float(fill)
                tw[0, slot, :] = float("nan")
                a, b = run(tb), run(tw)
                mask = _lib.SD_ROW_ERROR_MASK
                assert int(a.row_status[0]) & mask == int(b.row_status[0]) & mask, (kind, mode, slot)
                assert int(a.n_accepted[0]) == int(b.n_accepted[0]), (kind, mode, slot)


@pytest.mark.parametrize("mode", ["stream", "philox"])
@pytest.mark.parametrize("kind", ["topk", "nucleus"])
def test_speculative_generate_raises_on_masked_nan(mode, kind):
    """The drop-in loop under a top-k / nucleus processor with one NaN logit per row (column 0,
    masked by the cut in almost every bank row): the reference raises in torch.multinomial, and so
    does speculative_generate (RowError, a RuntimeError)."""
    from specdec_amd import RowError, set_noise_mode
    from specdec_amd.sampling import speculative_generate
    from specdec_amd.utils.logits_processor import NucleusProcessor, TopKProcessor
    target, drafter = nan_pair(where="drafter")
    proc = TopKProcessor(1.0, 20) if kind == "topk" else NucleusProcessor(1.0, 0.9)
    set_noise_mode(mode, seed=3)
    try:
        with pytest.raises(RowError, match="nan"):
            speculative_generate([5, 9, 13], drafter, target, gamma=4, logits_processor=proc, max_gen_len=12)
    finally:
        set_noise_mode("stream")
    torch.cuda.synchronize()
