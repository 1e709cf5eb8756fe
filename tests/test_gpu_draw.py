"""PHILOX (perf) mode of sd_sample — k_draw, the one-pass drafter draw — and
the verify step that takes the draws' row statistics instead of re-reading the drafter rows.

* draws are checked in distribution (chi-square against the exact processed softmax:
  utils/logits_processor.py:13-15 + MultinomialProcessor.sample :39-49), across spans too;
* the returned (max, Σexp) must reproduce the exact softmax (fp64 oracle) and token_prob the
  processed probability of the drawn token;
* verify(draft_row_stats=...) must decide as the host walk on the exact p/q does, and agree with
  the call that computes the drafter statistics itself.
"""
import dataclasses
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import specdec_ref as ref
from parity_stats import DRAW_CLOSE_CALLS

pytestmark = pytest.mark.gpu
DEV = "cuda"
CHI2_P_MIN = 1e-4


@pytest.fixture(scope="module")
def sd():
    from specdec_amd import _lib, ops
    from specdec_amd.noise import PhiloxNoise
    return SimpleNamespace(lib=_lib, ops=ops, PhiloxNoise=PhiloxNoise)


def spec_of(sd, p):
    return sd.ops.ProcSpec(p.kind, p.temperature, p.top_k, p.top_p)


def rand_logits(shape, dtype, seed, scale=3.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def peaked_logits(V, n_hot, seed, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(V, generator=g)
    hot = torch.randperm(V, generator=g)[:n_hot]
    x[hot] += 8.0 + torch.rand(n_hot, generator=g) * 2.0
    return x.to(dtype)


def chi2_check(samples, probs, label):
    from scipy.stats import chisquare
    probs = np.asarray(probs, dtype=np.float64)
    probs = probs / probs.sum()
    n = len(samples)
    counts = np.bincount(np.asarray(samples), minlength=len(probs)).astype(np.float64)
    assert counts[probs == 0].sum() == 0, f"{label}: sampled a zero-probability token"
    exp = probs * n
    big = exp >= 5
    obs_b = np.append(counts[big], counts[~big].sum())
    exp_b = np.append(exp[big], exp[~big].sum())
    if exp_b[-1] < 5:
        k = np.argmax(exp_b[:-1])
        obs_b[k] += obs_b[-1]
        exp_b[k] += exp_b[-1]
        obs_b, exp_b = obs_b[:-1], exp_b[:-1]
    stat, pval = chisquare(obs_b, exp_b)
    print(f"[draw] {label}: n={n} bins={len(obs_b)} chi2={stat:.1f} p={pval:.3g}")
    assert pval > CHI2_P_MIN, (label, stat, pval)


def processed_values(row, proc):
    """y = _process(x) / T in the row dtype (the exact oracle's processed logits), fp64."""
    p = ref.process(row, proc, exact=True).double()
    return p


@pytest.mark.parametrize("label,proc,V,dtype", [
    ("multi_t1_v64", ref.Processor("multinomial", 1.0), 64, torch.bfloat16),
    ("multi_t1_v8192", ref.Processor("multinomial", 1.0), 8192, torch.bfloat16),
    ("multi_t1_v128256", ref.Processor("multinomial", 1.0), 128256, torch.bfloat16),   # the bench's rows
    ("multi_t07_v50257_f32", ref.Processor("multinomial", 0.7), 50257, torch.float32),
    ("topk50_v8192", ref.Processor("topk", 0.8, 50), 8192, torch.bfloat16),
    ("nucleus09_v8192", ref.Processor("nucleus", 1.0, 0, 0.9), 8192, torch.bfloat16),
])
def test_draw_distribution(sd, label, proc, V, dtype):
    R = 4096
    row = peaked_logits(V, 40, 3).to(dtype) if V > 64 else rand_logits((V,), dtype, 4, 1.5)
    logits = row.view(1, V).expand(R, V).contiguous().to(DEV)
    pproc = ref.Processor(proc.kind, proc.temperature, proc.top_k, proc.top_p, stable_ties=True)
    probs = ref.process(row, pproc, exact=True).double()
    noise = sd.PhiloxNoise(seed=31337)
    xs = []
    for _ in range(4):
        tok, prob, st = sd.ops.sample_rows(logits, spec_of(sd, proc), noise, want_prob=True)
        assert ((st & sd.lib.SD_ROW_DONE) != 0).all()
        assert ((st & sd.lib.SD_ROW_INVALID_DIST) == 0).all()
        t = tok.cpu()
        # token_prob = the processed probability of the drawn token (exact oracle, dtype-rounded)
        want = probs[t].float()
        got = prob.cpu()
        assert torch.allclose(got, want, rtol=1e-2, atol=0), label
        xs.append(t.numpy())
    chi2_check(np.concatenate(xs), probs.numpy(), label)


@pytest.mark.parametrize("R,V,dtype,offset", [(32, 128256, torch.bfloat16, 0), (5, 50257, torch.float32, 0),
                                              (3, 1000, torch.bfloat16, 0), (4, 4099, torch.bfloat16, 1),
                                              (8, 50257, torch.float16, 0),
                                              # k_draw_lean's 2- and 4-stage spans (large batches)
                                              (100, 128256, torch.bfloat16, 0), (300, 128256, torch.bfloat16, 0)])
def test_draw_row_stats_reproduce_softmax(sd, R, V, dtype, offset):
    """(M, S) from the draw: exp(y - M) / S is the softmax of the row (fp64 oracle) to 2e-6
    relative on the largest probabilities; misaligned rows (offset 1) and ragged V included."""
    base = rand_logits((R, V + offset), dtype, 5 + V)
    x = base.to(DEV)[:, offset:]
    stats = torch.empty(R, 2, dtype=torch.float32, device=DEV)
    proc = ref.Processor("multinomial", 1.0)
    tok, prob, st = sd.ops.sample_rows(x, spec_of(sd, proc), sd.PhiloxNoise(seed=7), want_prob=True,
                                       row_stats_out=stats)
    assert ((st & sd.lib.SD_ROW_INVALID_DIST) == 0).all()
    xc = base[:, offset:].double()
    M, S = stats[:, 0].double().cpu(), stats[:, 1].double().cpu()
    p = torch.exp(xc - M[:, None]) / S[:, None]
    exact = torch.softmax(xc, dim=-1)
    top = exact >= exact.max(dim=-1, keepdim=True).values * 1e-3
    rel = ((p - exact).abs() / exact)[top]
    assert float(rel.max()) < 2e-6, float(rel.max())
    t = tok.cpu()
    assert ((t >= 0) & (t < V)).all()
    want = ref.softmax(base[:, offset:], True).float()
    got = prob.cpu()
    for r in range(R):
        assert got[r] == want[r, t[r]] or abs(float(got[r]) - float(want[r, t[r]])) <= 1e-2 * float(want[r, t[r]])


def test_draw_invalid_rows_flagged(sd):
    """A NaN logit or an all -inf row: torch.multinomial raises; the draw flags the row."""
    V = 4096
    x = rand_logits((3, V), torch.bfloat16, 9)
    x[0, 77] = float("nan")
    x[1, :] = float("-inf")
    tok, _, st = sd.ops.sample_rows(x.to(DEV), spec_of(sd, ref.Processor("multinomial", 1.0)), sd.PhiloxNoise(seed=1))
    st = st.cpu()
    assert st[0] & sd.lib.SD_ROW_INVALID_DIST
    assert st[1] & sd.lib.SD_ROW_INVALID_DIST
    assert not st[2] & sd.lib.SD_ROW_INVALID_DIST
    assert 0 <= int(tok[2]) < V


def test_draw_graph_replay_deterministic(sd):
    """The one-pass draw's arrival counters re-arm: eager repeats and graph replays give the
    first call's tokens and statistics."""
    R, V = 32, 128256
    x = rand_logits((R, V), torch.bfloat16, 12).to(DEV)
    spec = spec_of(sd, ref.Processor("multinomial", 1.0))
    stats = torch.empty(R, 2, dtype=torch.float32, device=DEV)

    def call():
        tok, _, _ = sd.ops.sample_rows(x, spec, sd.PhiloxNoise(seed=5, offset=9), row_stats_out=stats)
        return tok.clone(), stats.clone()

    t0, s0 = call()
    for _ in range(20):
        t, s = call()
        assert torch.equal(t, t0) and torch.equal(s.view(torch.int32), s0.view(torch.int32))
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        call()
        with torch.cuda.graph(graph, stream=stream):
            tok, _, _ = sd.ops.sample_rows(x, spec, sd.PhiloxNoise(seed=5, offset=9), row_stats_out=stats)
    torch.cuda.current_stream().wait_stream(stream)
    for _ in range(20):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(tok, t0) and torch.equal(stats.view(torch.int32), s0.view(torch.int32))


def _walk_engine(p, q, u, toks, ends):
    n = 0
    for i in range(len(p)):
        ap = 1.0 if q[i] <= 0 else min(1.0, p[i] / q[i])
        if u[i] < ap:
            n += 1
            if int(toks[i]) in ends:
                return n
        else:
            return n
    return n


@pytest.mark.parametrize("rule", ["engine", "spec"])
def test_verify_with_draw_stats(sd, rule):
    """The bench's step: γ draws (each returning its row stats), then verify with
    draft_row_stats.  Decisions must agree with the verify that recomputes the drafter
    statistics itself on all rows but those whose accept test sits within fp32 rounding."""
    import philox_ref as ph
    B, g, V = 32, 4, 128256
    tl = rand_logits((B, g + 1, V), torch.bfloat16, 71).to(DEV)
    dl = (tl[:, :g].float() + rand_logits((B, g, V), torch.float32, 72, 1.0).to(DEV)).to(torch.bfloat16)
    proc = ref.Processor("multinomial", 0.9 if rule == "spec" else 1.0)
    spec = spec_of(sd, proc)
    noise = sd.PhiloxNoise(seed=11)
    stats = torch.empty(g, B, 2, dtype=torch.float32, device=DEV)
    ids = torch.empty(B, g, dtype=torch.long, device=DEV)
    for d in range(g):
        tok, _, _ = sd.ops.sample_rows(dl[:, d], spec, noise, row_stats_out=stats[d])
        ids[:, d] = tok
    r = sd.lib.SD_RULE_ENGINE if rule == "engine" else sd.lib.SD_RULE_SPEC
    trows = [tl[:, t] for t in range(g if rule == "engine" else g + 1)]
    drows = [dl[:, d] for d in range(g)]
    off = noise.offset
    a = sd.ops.verify(trows, drows, ids, r, spec, spec, sd.PhiloxNoise(seed=11, offset=off), draft_row_stats=stats)
    b = sd.ops.verify(trows, drows, ids, r, spec, spec, sd.PhiloxNoise(seed=11, offset=off))
    na, nb = a.n_accepted.cpu(), b.n_accepted.cpu()
    assert int((na != nb).sum()) <= 1
    same = na == nb
    assert int((a.next_token.cpu()[same] != b.next_token.cpu()[same]).sum()) <= 1
    # a row whose decision differs must be a close call: at its first differing draft the accept
    # uniform sits within fp32 rounding of the exact p/q (the two calls differ only in how the
    # drafter's Σexp was summed)
    pp = ref.process(tl[:, :g].cpu(), proc, exact=True).double()
    qq = ref.process(dl.cpu(), proc, exact=True).double()
    ih = ids.cpu()
    for s in (~same).nonzero().flatten().tolist():
        i = min(int(na[s]), int(nb[s]))
        p_i, q_i = float(pp[s, i, ih[s, i]]), float(qq[s, i, ih[s, i]])
        ratio = min(1.0, p_i / q_i) if q_i > 0 else 1.0
        u = float(ph.accept_uniform(11, off, s, i))   # both rules test the same uniform against p/q
        assert abs(u - ratio) <= 1e-5 * ratio + 1e-7, (s, i, u, ratio)
        DRAW_CLOSE_CALLS.append(f"{rule} row={s} draft={i} p/q={ratio:.9g} u={u:.9g}")
    assert ((a.row_status.cpu() & sd.lib.SD_ROW_DONE) != 0).all()
    if rule == "engine":   # host walk on the exact p / q
        pt = ref.softmax(tl[:, :g].cpu(), True).float()
        qd = ref.softmax(dl.cpu(), True).float()
        ih = ids.cpu()
        bad = 0
        for s in range(B):
            p = [float(pt[s, i, ih[s, i]]) for i in range(g)]
            q = [float(qd[s, i, ih[s, i]]) for i in range(g)]
            u = [float(ph.accept_uniform(11, off, s, i)) for i in range(g)]
            bad += _walk_engine(p, q, u, ih[s], []) != int(na[s])
        assert bad <= 1


def kept_count(x, keep):
    """tokens a row's sd_row_keep keeps: x_j > tau or (x_j == tau and j <= tie_idx)"""
    tau = keep[0:1].view(torch.float32)
    tie = int(keep[1])
    xf = x.float()
    j = torch.arange(x.numel())
    return int(((xf > tau) | ((xf == tau) & (j <= tie))).sum())


@pytest.mark.parametrize("proc", [ref.Processor("nucleus", 1.0, 0, 0.9), ref.Processor("topk", 0.8, 50),
                                  ref.Processor("topknucleus", 1.0, 200, 0.8)], ids=lambda p: p.kind)
@pytest.mark.parametrize("dtype,V", [(torch.bfloat16, 128256), (torch.float16, 32000)])
def test_verify_with_draw_keeps(sd, proc, dtype, V):
    """A top-k / nucleus drafter: each draw also returns its row's keep predicate
    (sample_rows(row_keep_out=...)), and verify(draft_row_stats, draft_row_keep) searches the
    thresholds of the target rows only.  The keeps count what the oracle's processor keeps
    (utils/logits_processor.py:52-101), the same rows drawn again return the same keeps, and the
    decisions equal the verify that recomputes everything but where the accept uniform sits
    within fp32 rounding of p/q (the drafter's Σexp summed in another order)."""
    import philox_ref as ph
    B, g = 4, 4
    tl = rand_logits((B, g + 1, V), dtype, 81).to(DEV)
    dl = (tl[:, :g].float() + rand_logits((B, g, V), torch.float32, 82, 1.0).to(DEV)).to(dtype)
    spec = spec_of(sd, proc)
    noise = sd.PhiloxNoise(seed=13)
    stats = torch.empty(g, B, 2, dtype=torch.float32, device=DEV)
    keeps = torch.empty(g, B, 4, dtype=torch.int32, device=DEV)
    ids = torch.empty(B, g, dtype=torch.long, device=DEV)
    for d in range(g):
        tok, _, _ = sd.ops.sample_rows(dl[:, d], spec, noise, row_stats_out=stats[d], row_keep_out=keeps[d])
        ids[:, d] = tok
    again = torch.empty_like(keeps[0])
    sd.ops.sample_rows(dl[:, 1], spec, sd.PhiloxNoise(seed=99), row_keep_out=again)
    assert torch.equal(again, keeps[1])
    kc, dlc = keeps.cpu(), dl.cpu()
    exact = dataclasses.replace(proc, stable_ties=True)   # the cut in exact arithmetic (test_gpu_threshold)
    # fp16 rows: the reference cannot fill -1e20 into fp16 (torch raises); top-k ranks values only,
    # so its count is checked on the same values in fp32, the nucleus cut has no fp16 reference
    orows = dlc.float() if dtype == torch.float16 else dlc
    for d in range(g if dtype != torch.float16 or proc.kind == "topk" else 0):
        want = (ref.processed_logits(orows[:, d], exact, exact=True).float() > -1e19).sum(-1)
        for b in range(B):
            if not int(kc[d, b, 2]) & sd.lib.SD_ROW_NUCLEUS_INEXACT:
                assert kept_count(dlc[b, d], kc[d, b]) == int(want[b]), (d, b)
    trows = [tl[:, t] for t in range(g + 1)]
    drows = [dl[:, d] for d in range(g)]
    off = noise.offset
    r = sd.lib.SD_RULE_SPEC
    a = sd.ops.verify(trows, drows, ids, r, spec, spec, sd.PhiloxNoise(seed=13, offset=off), draft_row_stats=stats,
                      draft_row_keep=keeps)
    b = sd.ops.verify(trows, drows, ids, r, spec, spec, sd.PhiloxNoise(seed=13, offset=off))
    assert torch.equal(a.row_status.cpu() & 0x1, b.row_status.cpu() & 0x1)
    na, nb = a.n_accepted.cpu(), b.n_accepted.cpu()
    same = na == nb
    assert torch.equal(a.next_token.cpu()[same], b.next_token.cpu()[same])
    tlc = tl[:, :g].cpu()
    pp = ref.process(tlc.float() if dtype == torch.float16 else tlc, proc, exact=True).double()
    qq = ref.process(orows, proc, exact=True).double()
    tol = 1e-5 if dtype != torch.float16 else 2e-3     # fp16: p/q of the fp32-processed rows
    ih = ids.cpu()
    for s in (~same).nonzero().flatten().tolist():
        i = min(int(na[s]), int(nb[s]))
        p_i, q_i = float(pp[s, i, ih[s, i]]), float(qq[s, i, ih[s, i]])
        ratio = min(1.0, p_i / q_i) if q_i > 0 else 1.0
        u = float(ph.accept_uniform(13, off, s, i))
        assert abs(u - ratio) <= tol * ratio + 1e-7, (s, i, u, ratio)
        DRAW_CLOSE_CALLS.append(f"keep {proc.kind} row={s} draft={i} p/q={ratio:.9g} u={u:.9g}")
    with pytest.raises(ValueError):   # keeps come with the stats
        sd.ops.verify(trows, drows, ids, r, spec, spec, sd.PhiloxNoise(seed=13), draft_row_keep=keeps)


def nucleus_case(kind, V, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    if kind == "peaked":        # ~30 hot tokens carry the mass
        x = peaked_logits(V, 30, seed, dtype).float()
    elif kind == "ties":        # few distinct values: the cut falls inside a run of equal values
        x = (torch.randint(0, 6, (V,), generator=g).float() * 0.75)
        x[torch.randperm(V, generator=g)[:40]] += 9.0
    else:                       # the bench's Llama-3 shaped rows (std 3): the nucleus holds thousands
        x = torch.randn(V, generator=g) * 3.0
    return x.to(dtype)


@pytest.mark.parametrize("kind,V,dtype,T,top_p", [
    ("peaked", 128256, torch.bfloat16, 1.0, 0.9), ("peaked", 32000, torch.float16, 0.7, 0.9),
    ("ties", 128256, torch.bfloat16, 1.0, 0.8), ("peaked", 50257, torch.bfloat16, 1.0, 0.5),
    ("peaked", 4096, torch.bfloat16, 0.9, 0.95)])
def test_nucleus_rejection_draw(sd, kind, V, dtype, T, top_p):
    """k_draw_nuc (sample_rows of a nucleus processor without token_prob / row_stats / row_keep,
    PHILOX, top_p >= 0.5, T <= 1): draws from the whole row's softmax and keeps a draw iff the
    T = 1 mass before it does not cross top_p.  The draws follow the processed distribution
    (utils/logits_processor.py:66-81 + :39-49; chi-square, never a token outside the nucleus)."""
    x = nucleus_case(kind, V, dtype, 3 + V % 97)
    proc = ref.Processor("nucleus", T, 0, top_p)
    spec = spec_of(sd, proc)
    R, calls = 8, 128      # 8 rows x 16 slices: the whole grid resident (one 1024-thread slice per CU)
    rows = x.view(1, -1).repeat(R, 1).to(DEV)
    noise = sd.PhiloxNoise(seed=1234)
    samples = []
    for _ in range(calls):
        tok, prob, st = sd.ops.sample_rows(rows, spec, noise)
        assert prob is None
        stc = st.cpu()
        assert bool(((stc & sd.lib.SD_ROW_DONE) != 0).all()) and not bool((stc & 0x40).any())
        samples += tok.cpu().tolist()
    # the nucleus the verify's threshold search cuts for this row (k_thr_hist, the same slice
    # normaliser; test_gpu_threshold holds it to the exact oracle): every draw inside it, and the
    # draws distributed as the processed softmax over it
    keep = torch.empty(R, 4, dtype=torch.int32, device=DEV)
    sd.ops.sample_rows(rows, spec, sd.PhiloxNoise(seed=5), row_stats_out=torch.empty(R, 2, device=DEV),
                       row_keep_out=keep)
    kc = keep.cpu()
    assert all(torch.equal(kc[i], kc[0]) for i in range(R))
    tau, tie = float(kc[0, 0:1].view(torch.float32)), int(kc[0, 1])
    xf = x.float()
    j = torch.arange(V)
    kept = (xf > tau) | ((xf == tau) & (j <= tie))
    y = (xf / T).to(dtype).double() if T != 1.0 else xf.double()
    want = torch.where(kept, torch.exp(y - y[kept].max()), torch.zeros_like(y))
    chi2_check(samples, (want / want.sum()).numpy(), f"nucleus-reject {kind} V={V}")
    # and the cut is the exact oracle's where the search calls it exact (no SD_ROW_NUCLEUS_INEXACT:
    # a cut among p < 2^-17, where fp32 cumsum rounding decides, is flagged instead)
    if not int(kc[0, 2]) & sd.lib.SD_ROW_NUCLEUS_INEXACT:
        orow = x.float() if dtype == torch.float16 else x
        exact = ref.processed_logits(orow.view(1, -1), dataclasses.replace(proc, stable_ties=True), exact=True)[0]
        assert int(kept.sum()) == int((exact.float() > -1e19).sum())


def test_nucleus_rejection_draw_flags_bad_rows(sd):
    x = torch.randn(3, 128256).to(torch.bfloat16)
    x[1, 5] = float("nan")
    x[2, 77] = float("inf")
    x[0, 9] = float("-inf")   # -inf is a zero-probability token, not an error
    spec = sd.ops.ProcSpec("nucleus", 1.0, 0, 0.9)
    tok, _, st = sd.ops.sample_rows(x.to(DEV), spec, sd.PhiloxNoise(seed=3))
    st, tok = st.cpu(), tok.cpu()
    assert int(st[0]) & 0x40 == 0 and int(tok[0]) != 9
    assert int(st[1]) & 0x40 and int(st[2]) & 0x40
    assert int(tok[1]) == -1 and int(tok[2]) == -1
