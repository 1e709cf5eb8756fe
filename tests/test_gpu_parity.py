"""HIP path vs the CPU oracle (and, through it, the reference) on identical inputs and noise.

Noise: the HIP side runs in STREAM mode, reading the raw mt19937 words of a torch CPU
generator; the oracle draws from an identically seeded generator with torch.rand /
exponential_.  Integer outputs (accept counts, token ids, stop positions, generator advance)
must match the oracle exactly.

Two oracles: ``exact=False`` is torch-CPU arithmetic (= the reference, pinned by the golden
vectors); ``exact=True`` computes every softmax in fp64 and rounds once.  torch-CPU's fp32
softmax normaliser carries a ~4e-6 relative summation error at V=128256 that moves ~0.5 % of
bf16 probabilities by one ulp, so on rare inputs the reference's own rounding flips a decision.
An integer result may therefore equal EITHER oracle; every such divergence is counted and
reported, and must equal the exact-arithmetic result.  The residual mass must be within 1e-5
of the exact value (north-star tolerance) and within 1e-4 of torch-CPU's.
"""
import dataclasses
import json
import os
from types import SimpleNamespace

import pytest
import torch

from fakelm import make_pair
from oracle import specdec_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
MASS_TOL = 1e-5
KINDS = {
    "greedy": ref.Processor("greedy"),
    "multi_t1": ref.Processor("multinomial", 1.0),
    "multi_t07": ref.Processor("multinomial", 0.7),
    "topk20": ref.Processor("topk", 1.0, 20),
    "topk50_t08": ref.Processor("topk", 0.8, 50),
    "nucleus09": ref.Processor("nucleus", 1.0, 0, 0.9),
    "nucleus05_t07": ref.Processor("nucleus", 0.7, 0, 0.5),
    "topknucleus": ref.Processor("topknucleus", 1.0, 50, 0.9),
}


@pytest.fixture(scope="module")
def sd():
    import specdec_amd
    from specdec_amd import _lib, ops
    from specdec_amd.noise import PhiloxNoise, StreamNoise
    return SimpleNamespace(lib=_lib, ops=ops, StreamNoise=StreamNoise, PhiloxNoise=PhiloxNoise, pkg=specdec_amd)


def spec_of(sd, p: ref.Processor):
    return sd.ops.ProcSpec(p.kind, p.temperature, p.top_k, p.top_p)


def rand_logits(shape, dtype, seed, scale=3.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def draft_case(B, gamma, V, dtype, seed, proc, sigma=1.0, peaked=False):
    """target [B, γ+1, V], drafter [B, γ, V] logits and draft ids sampled from the drafter."""
    scale = 6.0 if peaked else 3.0
    tl = rand_logits((B, gamma + 1, V), dtype, seed, scale)
    dl = (tl[:, :gamma].float() + rand_logits((B, gamma, V), torch.float32, seed + 777, sigma)).to(dtype)
    g = torch.Generator().manual_seed(seed + 99)
    ids = torch.empty(B, gamma, dtype=torch.long)
    for b in range(B):
        q = ref.process(dl[b], proc)
        if proc.stochastic:
            ids[b] = ref.multinomial(q, torch.empty(q.shape).exponential_(generator=g)).squeeze(-1)
        else:
            ids[b] = q.argmax(-1)
    # a few off-distribution drafts so rejects happen under greedy too
    ids[:, -1] = torch.randint(0, V, (B,), generator=g)
    return tl, dl, ids


# ---------------------------------------------------------------- SPEC rule (A8)
SPEC_GRID = [
    # (B, gamma, V, dtype, kind, seed)
    (1, 4, 4096, torch.bfloat16, "greedy", 0),
    (1, 4, 4096, torch.bfloat16, "multi_t1", 1),
    (1, 4, 4096, torch.bfloat16, "multi_t07", 2),
    (1, 1, 4096, torch.bfloat16, "multi_t1", 3),
    (1, 8, 4096, torch.bfloat16, "multi_t1", 4),
    (3, 4, 4096, torch.float32, "multi_t1", 5),
    (2, 4, 4096, torch.float32, "greedy", 6),
    (1, 4, 50257, torch.float32, "greedy", 7),
    (1, 4, 50257, torch.float32, "multi_t1", 8),
    (1, 4, 128256, torch.bfloat16, "greedy", 9),
    (1, 4, 128256, torch.bfloat16, "multi_t1", 10),
    (2, 4, 128256, torch.bfloat16, "multi_t07", 11),
    (1, 4, 4096, torch.bfloat16, "topk20", 12),
    (1, 4, 4096, torch.bfloat16, "topk50_t08", 13),
    (1, 4, 4096, torch.bfloat16, "nucleus09", 14),
    (1, 4, 4096, torch.bfloat16, "nucleus05_t07", 15),
    (1, 4, 4096, torch.bfloat16, "topknucleus", 16),
    (1, 4, 4096, torch.float32, "nucleus09", 17),
    (1, 4, 128256, torch.bfloat16, "topk50_t08", 18),
    (1, 8, 128256, torch.bfloat16, "nucleus09", 19),
    (1, 4, 4096, torch.float16, "multi_t1", 20),
    # nucleus at the production shape (Llama-3 vocab, bf16): >= 16 rows through check_spec
    (4, 4, 128256, torch.bfloat16, "nucleus09", 21),
    (4, 4, 128256, torch.bfloat16, "nucleus05_t07", 22),
    (4, 4, 128256, torch.bfloat16, "topknucleus", 23),
    (4, 8, 128256, torch.bfloat16, "nucleus09", 24),
    # more than one wave of rows in one STREAM k_walk block
    (96, 1, 2048, torch.bfloat16, "multi_t1", 25),
    (80, 2, 2048, torch.bfloat16, "multi_t07", 26),
]


from parity_stats import DIVERGENCES, NUCLEUS_ROWS, TIE_DIVERGENCES  # noqa: E402
from custom_procs import golden_processor  # noqa: E402


def run_spec_oracle(tl, dl, ids, proc, gen, stops, skip=False, exact=False):
    res = []
    for b in range(tl.shape[0]):
        g = ids.shape[1]
        q = ref.process(dl[b], proc, exact).float()
        r = torch.rand(g, generator=gen)
        n, p = ref.spec_accept(tl[b], q, ids[b].tolist(), proc, r, exact)
        hit = [ref.stop_location(ids[b, :n].tolist(), stops)]
        hit = [h for h in hit if h >= 0]
        if hit:
            res.append(dict(n=n, x=-1, stop=hit[0], mass=float("nan")))
            continue
        E = torch.empty(tl.shape[-1]).exponential_(generator=gen) if proc.stochastic else None
        st = ref.spec_resample(tl[b], q, p, n, proc, E, skip, exact)
        res.append(dict(n=n, x=st.x, stop=-1, mass=st.residual_mass, kd=st.prune_drafter, kt=st.prune_target))
    return res


def run_spec_hip(sd, tl, dl, ids, proc, gen, stops, skip=False):
    g = ids.shape[1]
    tld, dld, idd = tl.to(DEV), dl.to(DEV), ids.to(DEV)
    out = sd.ops.verify([tld[:, t, :] for t in range(g + 1)], [dld[:, d, :] for d in range(g)], idd,
                        sd.lib.SD_RULE_SPEC, spec_of(sd, proc), spec_of(sd, proc), sd.StreamNoise(gen),
                        torch.tensor(stops, dtype=torch.long, device=DEV), skip_sample_adjustment=skip)
    torch.cuda.synchronize()
    return out


def _ints(w):
    return (w["n"], w["stop"]) + ((w["x"], w["kd"], w["kt"]) if w["stop"] < 0 else ())




def oracle_variants(proc):
    """(label, processor, exact) oracles a HIP result may equal, in order of preference."""
    out = [("cpu", proc, False), ("exact", proc, True)]
    if proc.kind in ("nucleus", "topknucleus"):
        st = dataclasses.replace(proc, stable_ties=True)
        out += [("cpu-stable-ties", st, False), ("exact-stable-ties", st, True)]
    return out


def note_divergence(label, what):
    if label == "cpu":
        return
    if "stable" in label:
        TIE_DIVERGENCES.append(what)
    else:
        DIVERGENCES.append(what)
    print(f"[parity] {what}: HIP matched the {label} oracle, not torch-CPU arithmetic")


def check_spec(sd, tl, dl, ids, proc, seed, stops=(), skip=False):
    variants = []
    for label, pv, exact in oracle_variants(proc):
        g = torch.Generator().manual_seed(1000 + seed)
        variants.append((label, run_spec_oracle(tl, dl, ids, pv, g, list(stops), skip, exact), g.get_state()))
    g2 = torch.Generator().manual_seed(1000 + seed)
    out = run_spec_hip(sd, tl, dl, ids, proc, g2, list(stops), skip)
    n = out.n_accepted.cpu().tolist()
    x = out.next_token.cpu().tolist()
    st = out.row_status.cpu().tolist()
    si = out.stop_index.cpu().tolist()
    mass = out.resample_mass.cpu().tolist()
    kd = out.prune_drafter.cpu().tolist()
    kt = out.prune_target.cpu().tolist()
    for b in range(tl.shape[0]):
        got = (n[b], si[b]) + ((x[b], kd[b], kt[b]) if si[b] < 0 else ())
        match = [label for label, res, _ in variants if _ints(res[b]) == got]
        assert match, (b, got, [(label, res[b]) for label, res, _ in variants], hex(st[b]))
        note_divergence(match[0], f"spec seed={seed} row={b}")
        if proc.kind in ("nucleus", "topknucleus"):
            NUCLEUS_ROWS["checked"] += 1
            NUCLEUS_ROWS[f"variant={proc.kind}(T={proc.temperature:g},k={proc.top_k},p={proc.top_p:g})"
                         f"@V{tl.shape[-1]}"] += 1
            if st[b] & sd.lib.SD_ROW_NUCLEUS_INEXACT:   # held to the same integer match, and counted
                NUCLEUS_ROWS["inexact"] += 1
                NUCLEUS_ROWS["inexact=" + match[0]] += 1
        # mass vs the exact-arithmetic oracle with the kernel's tie rule (lowest index first)
        ex_label = "exact-stable-ties" if proc.kind in ("nucleus", "topknucleus") else "exact"
        wx = dict((label, res) for label, res, _ in variants)[ex_label][b]
        if si[b] < 0 and wx["mass"] == wx["mass"] and _ints(wx) == got:
            assert abs(mass[b] - wx["mass"]) <= MASS_TOL, (mass[b], wx["mass"])
        assert not (st[b] & sd.lib.SD_ROW_NOISE_OVERRUN)
    # identical generator advance: the kernels consumed exactly the reference's draws
    assert any(torch.equal(g2.get_state(), state) for _, _, state in variants)
    return st


@pytest.mark.parametrize("B,gamma,V,dtype,kind,seed", SPEC_GRID)
def test_spec_verify_matches_oracle(sd, B, gamma, V, dtype, kind, seed):
    proc = KINDS[kind]
    tl, dl, ids = draft_case(B, gamma, V, dtype, seed, proc)
    before = NUCLEUS_ROWS["inexact"]
    st = check_spec(sd, tl, dl, ids, proc, seed)
    if proc.kind in ("nucleus", "topknucleus"):
        # every row (INEXACT or not) equalled an oracle inside check_spec; the flag count is exact
        flagged = sum(1 for s in st if s & sd.lib.SD_ROW_NUCLEUS_INEXACT)
        assert NUCLEUS_ROWS["inexact"] - before == flagged


def test_spec_verify_full_accept_bonus(sd):
    # drafter == target and greedy drafts: everything is accepted, x comes from the bonus row
    proc = KINDS["multi_t1"]
    tl = rand_logits((1, 5, 4096), torch.bfloat16, 41)
    dl = tl[:, :4].clone()
    ids = torch.stack([ref.process(dl[0], proc).argmax(-1)])
    st = check_spec(sd, tl, dl, ids, proc, 41)
    assert st[0] & sd.lib.SD_ROW_BONUS


def test_spec_verify_stop_in_drafts(sd):
    proc = KINDS["greedy"]
    tl = rand_logits((1, 5, 4096), torch.bfloat16, 42)
    dl = tl[:, :4].clone()
    ids = torch.stack([ref.process(dl[0], proc).argmax(-1)])
    st = check_spec(sd, tl, dl, ids, proc, 42, stops=[int(ids[0, 1])])
    assert st[0] & sd.lib.SD_ROW_STOP_IN_DRAFTS


def test_spec_verify_skip_sample_adjustment(sd):
    proc = KINDS["multi_t1"]
    for seed in range(3):
        tl, dl, ids = draft_case(1, 4, 4096, torch.bfloat16, 50 + seed, proc, sigma=3.0)
        check_spec(sd, tl, dl, ids, proc, 50 + seed, skip=True)


@pytest.mark.parametrize("B,gamma,kind,seed", [(1, 40, "multi_t1", 70), (1, 48, "greedy", 71), (3, 40, "multi_t1", 72),
                                              (2, 64, "multi_t07", 73), (1, 33, "nucleus09", 74)])
def test_spec_verify_chunked_window(sd, B, gamma, kind, seed):
    """γ > SD_MAX_GAMMA (specdec_amd/chunked.py): the window in chunks of <= 32 drafts equals one
    reference verify over all γ — accept count, token, prune lengths and the generator's advance
    (γ uniforms, then the sample's 2V words).  Drafter = target + N(0, 0.05²), so the accept walks
    cross the chunk boundary; one row's last draft off-distribution so rejects land late."""
    proc = KINDS[kind]
    tl, dl, ids = draft_case(B, gamma, 4096, torch.bfloat16, seed, proc, sigma=0.05)
    st = check_spec(sd, tl, dl, ids, proc, seed)
    assert all(s & sd.lib.SD_ROW_DONE for s in st)


def test_spec_verify_chunked_window_stops(sd):
    """A stop token in the second chunk's accepted drafts, with the walk still accepting: the stop
    return, at the reference's position (the first-listed stop token that occurs)."""
    proc = KINDS["greedy"]
    tl = rand_logits((1, 41, 4096), torch.bfloat16, 75)
    dl = tl[:, :40].clone()
    ids = torch.stack([ref.process(dl[0], proc).argmax(-1)])
    st = check_spec(sd, tl, dl, ids, proc, 75, stops=[int(ids[0, 35]), int(ids[0, 37])])
    assert st[0] & sd.lib.SD_ROW_STOP_IN_DRAFTS


@pytest.mark.parametrize("fused", [0, 1], ids=["two-launch", "fused"])
def test_spec_verify_stop_list_order(sd, fused):
    """sampling/speculative_decoding.py:150-152 scans eq(drafts[1, n], stop_tokens[S, 1]) row-major:
    with several listed stop tokens among the accepted drafts the return is at the first-LISTED one
    (here the later position), not the earliest stop position.  STREAM (check_spec) and Philox, the
    latter with the drafter stats from draws so B = 8 takes the one-launch kernels."""
    proc = KINDS["greedy"]
    tl = rand_logits((8, 9, 4096), torch.bfloat16, 76)
    dl = tl[:, :8].clone()
    ids = torch.stack([ref.process(dl[b], proc).argmax(-1) for b in range(8)])
    stops = [int(ids[0, 5]), int(ids[0, 2])]
    st = check_spec(sd, tl, dl, ids, proc, 76, stops=stops)
    assert st[0] & sd.lib.SD_ROW_STOP_IN_DRAFTS
    tld, dld, idd = tl.to(DEV), dl.to(DEV), ids.to(DEV)
    stats = torch.empty(8, 8, 2, device=DEV)
    for d in range(8):
        sd.ops.sample_rows(dld[:, d], spec_of(sd, proc), sd.PhiloxNoise(seed=1), row_stats_out=stats[d])
    with sd.lib.option(sd.lib.SD_OPT_FUSED_VERIFY, 2 if fused else 0), sd.lib.option(sd.lib.SD_OPT_LEAN_VERIFY, 0):
        out = sd.ops.verify([tld[:, t] for t in range(9)], [dld[:, d] for d in range(8)], idd, sd.lib.SD_RULE_SPEC,
                            spec_of(sd, proc), spec_of(sd, proc), sd.PhiloxNoise(seed=5),
                            torch.tensor(stops, dtype=torch.long, device=DEV), draft_row_stats=stats)
    for b in range(8):
        want = ref.stop_location(ids[b].tolist(), stops)
        assert int(out.stop_index[b]) == want, (b, int(out.stop_index[b]), want)
    assert int(out.stop_index[0]) == 5


@pytest.mark.parametrize("seed", range(12))
def test_spec_verify_many_seeds(sd, seed):
    proc = [KINDS["greedy"], KINDS["multi_t1"], KINDS["multi_t07"]][seed % 3]
    tl, dl, ids = draft_case(2, 4, 8192, torch.bfloat16, 300 + seed, proc, sigma=1.5)
    check_spec(sd, tl, dl, ids, proc, 300 + seed)


# ---------------------------------------------------------------- ENGINE rule (A10)
ENGINE_GRID = [
    (1, 4, 4096, torch.bfloat16, 0),
    (6, 4, 4096, torch.float32, 1),
    (6, 1, 2048, torch.float32, 2),
    (5, 3, 2048, torch.bfloat16, 3),
    (32, 4, 128256, torch.bfloat16, 4),
    (8, 4, 50257, torch.float32, 5),
    # more than one wave of rows in one k_walk block (STREAM): rows >= 64 walk off lane registers
    (96, 1, 2048, torch.bfloat16, 9),
    (80, 2, 2048, torch.bfloat16, 10),
    (128, 4, 4096, torch.bfloat16, 11),
]


@pytest.mark.parametrize("B,gamma,V,dtype,seed", ENGINE_GRID)
def test_engine_verify_matches_oracle(sd, B, gamma, V, dtype, seed):
    _engine_case(sd, B, gamma, V, dtype, seed)


@pytest.mark.parametrize("B,gamma,V,dtype,seed", [(3, 40, 2048, torch.float32, 6), (4, 48, 4096, torch.bfloat16, 7),
                                                  (1, 70, 2048, torch.float32, 8)])
def test_engine_verify_chunked_window(sd, B, gamma, V, dtype, seed):
    """γ > SD_MAX_GAMMA (specdec_amd/chunked.py): the engine window in chunks of <= 32 drafts, row by
    row under STREAM, equals the reference's walk over all γ (engine state, counts, generator)."""
    _engine_case(sd, B, gamma, V, dtype, seed, sigma=0.05, late_stop=True)


def _engine_case(sd, B, gamma, V, dtype, seed, sigma=1.0, late_stop=False):
    plain = ref.Processor("multinomial", 1.0)
    tl, dl, ids = draft_case(B, gamma, V, dtype, seed, plain, sigma=sigma)
    tl = tl[:, :gamma]
    gen_len, step = gamma * 3, gamma
    end_tokens = [int(ids[0, min(1, gamma - 1)]), int(ids[min(2, B - 1), 0])]
    if late_stop:   # an end token past the first chunk (row 0), so the walks cross the chunk boundary
        end_tokens = [int(ids[0, gamma - 4])]
    finished = torch.zeros(B, dtype=torch.bool)
    finished[B // 2] = True if B > 2 else False
    generated = torch.zeros(B, gen_len, dtype=torch.long)
    generated[:, step:step + gamma] = torch.where(finished[:, None], generated[:, step:step + gamma], ids)
    acc = torch.zeros(B, dtype=torch.long)
    # oracles (torch-CPU arithmetic and exact-softmax arithmetic)
    res = {}
    for exact in (False, True):
        g1 = torch.Generator().manual_seed(2000 + seed)
        p = ref.softmax(tl, exact)
        q = ref.softmax(dl, exact).float()
        gen_o, fin_o, acc_o = generated.clone(), finished.clone(), acc.clone()
        n_o = ref.engine_verify_rows(p, q, ids, fin_o, end_tokens, step, gen_o, acc_o, ref.TorchNoise(g1), exact)
        res[exact] = (gen_o, fin_o, acc_o, n_o, g1.get_state())
    # HIP
    g2 = torch.Generator().manual_seed(2000 + seed)
    gen_d, fin_d, acc_d = generated.to(DEV), finished.to(torch.uint8).to(DEV), acc.to(DEV)
    tld, dld = tl.to(DEV), dl.to(DEV)
    plain_spec = sd.ops.PLAIN_SOFTMAX
    out = sd.ops.verify([tld[:, t, :] for t in range(gamma)], [dld[:, d, :] for d in range(gamma)], ids.to(DEV),
                        sd.lib.SD_RULE_ENGINE, plain_spec, plain_spec, sd.StreamNoise(g2),
                        torch.tensor(end_tokens, dtype=torch.long, device=DEV),
                        active=(fin_d == 0).to(torch.uint8),
                        engine_state=dict(generated=gen_d, step=step, finished=fin_d, accepted=acc_d))
    torch.cuda.synchronize()
    n_h = out.n_accepted.cpu().tolist()

    def same(r):
        gen_o, fin_o, acc_o, n_o, state = r
        return (torch.equal(gen_d.cpu(), gen_o) and torch.equal(fin_d.cpu().bool(), fin_o)
                and torch.equal(acc_d.cpu(), acc_o) and all(n_h[b] == n_o[b] for b in range(B) if n_o[b] >= 0)
                and torch.equal(g2.get_state(), state))

    if not same(res[False]):
        assert same(res[True])
        note_divergence("exact", f"engine seed={seed}")


@pytest.mark.parametrize("B,V,dtype,seed", [(6, 4096, torch.bfloat16, 60), (4, 50257, torch.float32, 61),
                                            (8, 128256, torch.bfloat16, 62)])
def test_engine_verify_draft_probs(sd, B, V, dtype, seed):
    """The reference's q buffer handed over as fp32 probabilities (draft_is_probs): mixed-width
    rows (bf16 target, fp32 drafter) must match the oracle fed the same q."""
    plain = ref.Processor("multinomial", 1.0)
    gamma = 4
    tl, dl, ids = draft_case(B, gamma, V, dtype, seed, plain)
    tl = tl[:, :gamma]
    q = ref.softmax(dl, True).float()
    g1 = torch.Generator().manual_seed(3000 + seed)
    n_o = {}
    for exact in (False, True):
        g1 = torch.Generator().manual_seed(3000 + seed)
        gen_o = torch.zeros(B, gamma * 2, dtype=torch.long)
        n_o[exact] = (ref.engine_verify_rows(ref.softmax(tl, exact), q, ids, torch.zeros(B, dtype=torch.bool), [],
                                             0, gen_o, torch.zeros(B, dtype=torch.long), ref.TorchNoise(g1), exact),
                      gen_o[:, :gamma], g1.get_state())
    g2 = torch.Generator().manual_seed(3000 + seed)
    tld, qd = tl.to(DEV), q.to(DEV)
    out = sd.ops.verify([tld[:, t, :] for t in range(gamma)], [qd[:, d, :] for d in range(gamma)], ids.to(DEV),
                        sd.lib.SD_RULE_ENGINE, sd.ops.PLAIN_SOFTMAX, sd.ops.PLAIN_SOFTMAX, sd.StreamNoise(g2),
                        torch.tensor([], dtype=torch.long, device=DEV), draft_is_probs=True)
    n_h = out.n_accepted.cpu().tolist()
    x_h = out.next_token.cpu().tolist()

    def same(r):
        n, gen, state = r
        xs = [int(gen[b, n[b]]) if n[b] < gamma else -1 for b in range(B)]
        return n_h == n and x_h == xs and torch.equal(g2.get_state(), state)

    if not same(n_o[False]):
        assert same(n_o[True]), (n_h, x_h, n_o[True][0])
        note_divergence("exact", f"engine probs seed={seed}")


# ---------------------------------------------------------------- sample / probs kernels
@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("dtype,V,R", [(torch.bfloat16, 4096, 3), (torch.float32, 50257, 2),
                                       (torch.bfloat16, 128256, 4)])
def test_sample_rows_matches_oracle(sd, kind, dtype, V, R):
    proc = KINDS[kind]
    x = rand_logits((R, V), dtype, hash((kind, V)) % 1000)
    g2 = torch.Generator().manual_seed(7)
    tok, prob, st = sd.ops.sample_rows(x.to(DEV), spec_of(sd, proc), sd.StreamNoise(g2), want_prob=True)
    tok = tok.cpu()
    match = []
    for label, pv, exact in oracle_variants(proc):
        g1 = torch.Generator().manual_seed(7)
        want = ref.sample(ref.process(x, pv, exact), pv, ref.TorchNoise(g1)).squeeze(-1)
        if torch.equal(tok, want):
            match.append(label)
    assert match, (kind, V, tok)
    note_divergence(match[0], f"sample {kind} V={V}")
    assert torch.equal(g1.get_state(), g2.get_state())


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("dtype,V", [(torch.bfloat16, 4096), (torch.float32, 4096), (torch.bfloat16, 128256)])
def test_probs_rows_close_to_oracle(sd, kind, dtype, V):
    proc = dataclasses.replace(KINDS[kind], stable_ties=True)
    x = rand_logits((3, V), dtype, 11)
    want = ref.process(x, proc)
    got = sd.ops.probs_rows(x.to(DEV), spec_of(sd, proc)).cpu()
    # same support (processor mask) ...
    assert torch.equal(got > 0, want > 0)
    # ... and values equal up to the last-bit rounding of the fp32 softmax internals
    if dtype == torch.float32:
        torch.testing.assert_close(got, want, rtol=2e-6, atol=1e-12)
    else:
        diff = (got.float() - want.float()).abs() > 0
        assert diff.float().mean().item() < 2e-3
        torch.testing.assert_close(got.float(), want.float(), rtol=8e-3, atol=1e-9)


# ---------------------------------------------------------------- full loops vs reference goldens
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DT = {"bf16": torch.bfloat16, "fp32": torch.float32}
with open(os.path.join(GOLD, "spec_loops.json")) as f:
    SPEC = json.load(f)
with open(os.path.join(GOLD, "engine_loops.json")) as f:
    ENGINE = json.load(f)


def make_proc(sd, pp):
    """The record's processor on the drop-in classes (custom:* = a user _process override,
    tests/custom_procs.py)."""
    from specdec_amd.utils import logits_processor as lp
    return golden_processor(lp, pp)


@pytest.mark.parametrize("case", sorted(SPEC))
def test_speculative_generate_matches_reference(sd, case):
    from specdec_amd.sampling import speculative_generate
    c = SPEC[case]
    target, drafter = make_pair(c["vocab"], dtype=DT[c["dtype"]], device=DEV, sigma=c.get("sigma", 1.0))
    eos = c["eos"] if len(c["eos"]) > 1 else c["eos"][0]
    torch.manual_seed(c["seed"])
    out, rate = speculative_generate(c["prompt"], drafter, target, gamma=c["gamma"],
                                     logits_processor=make_proc(sd, c["processor"]), max_gen_len=c["max_gen_len"],
                                     eos_tokens_id=eos, skip_sample_adjustment=c["skip_sample_adjustment"])
    if (out, rate) != (c["tokens"], c["acceptance_rate"]):
        tc, dc = make_pair(c["vocab"], dtype=DT[c["dtype"]], sigma=c.get("sigma", 1.0))
        pp = c["processor"]
        match = []
        for label, pv, exact in oracle_variants(golden_processor(ref, pp))[1:]:
            torch.manual_seed(c["seed"])
            want = ref.speculative_generate(c["prompt"], dc, tc, gamma=c["gamma"], proc=pv,
                                            max_gen_len=c["max_gen_len"], eos_tokens_id=eos,
                                            skip_sample_adjustment=c["skip_sample_adjustment"], exact=exact)
            if (out, rate) == want:
                match.append(label)
                break
        assert match, (case, out, c["tokens"])
        note_divergence(match[0], f"spec loop {case}")


@pytest.mark.parametrize("case", sorted(ENGINE))
def test_batch_speculative_generate_matches_reference(sd, case):
    from specdec_amd.engine.infer_engine import batch_speculative_generate
    c = ENGINE[case]
    target, drafter = make_pair(c["vocab"], dtype=DT[c["dtype"]], device=DEV, pos_mult=c["pos_mult"],
                                sigma=c.get("sigma", 1.0))
    ids = torch.tensor(c["prompt"], dtype=torch.long, device=DEV)
    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=c["gamma"], gen_len=c["gen_len"],
                          end_tokens=c["end_tokens"])
    torch.manual_seed(c["seed"])
    outs, rates = batch_speculative_generate(ctx, ids, torch.ones_like(ids), c["batch"])
    if c["raised"]:
        # the reference crashed here (bf16, B>=2); the drop-in must run and agree with the oracle
        tc, dc = make_pair(c["vocab"], dtype=DT[c["dtype"]], pos_mult=c["pos_mult"], sigma=c.get("sigma", 1.0))
        octx = SimpleNamespace(drafter=dc, target=tc, gamma=c["gamma"], gen_len=c["gen_len"],
                               end_tokens=c["end_tokens"])
        torch.manual_seed(c["seed"])
        want, wrates = ref.batch_speculative_generate(octx, ids.cpu(), torch.ones_like(ids.cpu()), c["batch"])
        assert [o.tolist() for o in outs] == [w.tolist() for w in want]
        assert rates == wrates
        return
    if ([o.cpu().tolist() for o in outs], rates) != (c["outputs"], c["rates"]):
        tc, dc = make_pair(c["vocab"], dtype=DT[c["dtype"]], pos_mult=c["pos_mult"], sigma=c.get("sigma", 1.0))
        octx = SimpleNamespace(drafter=dc, target=tc, gamma=c["gamma"], gen_len=c["gen_len"],
                               end_tokens=c["end_tokens"])
        torch.manual_seed(c["seed"])
        want, wrates = ref.batch_speculative_generate(octx, ids.cpu(), torch.ones_like(ids.cpu()), c["batch"],
                                                      exact=True)
        assert [o.cpu().tolist() for o in outs] == [w.tolist() for w in want] and rates == wrates
        note_divergence("exact", f"engine loop {case}")


def test_use_cache_equals_no_cache(sd):
    from specdec_amd.sampling import speculative_generate
    from specdec_amd.utils.logits_processor import MultinomialProcessor
    target, drafter = make_pair(4096, dtype=torch.bfloat16, device=DEV)
    prompt = list(range(10, 18))
    res = []
    for uc in (False, True):
        torch.manual_seed(3)
        res.append(speculative_generate(prompt, drafter, target, gamma=4, logits_processor=MultinomialProcessor(1.0),
                                        max_gen_len=40, use_cache=uc))
    assert res[0] == res[1]


def test_philox_mode_runs_and_is_deterministic(sd):
    from specdec_amd.noise import PhiloxNoise
    proc = KINDS["multi_t1"]
    tl, dl, ids = draft_case(4, 4, 8192, torch.bfloat16, 77, proc)
    outs = []
    for _ in range(2):
        out = sd.ops.verify([tl.to(DEV)[:, t, :] for t in range(5)], [dl.to(DEV)[:, d, :] for d in range(4)],
                            ids.to(DEV), sd.lib.SD_RULE_SPEC, spec_of(sd, proc), spec_of(sd, proc),
                            PhiloxNoise(seed=123))
        outs.append((out.n_accepted.cpu(), out.next_token.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert ((outs[0][1] >= 0) & (outs[0][1] < 8192)).all()


def test_divergence_budget():
    """Rounding divergences from torch-CPU must stay rare (each one already matched the exact oracle);
    nucleus tie-order divergences are reported (torch's unstable sort order is implementation-defined)."""
    print(f"[parity] torch-CPU rounding divergences: {len(DIVERGENCES)} {DIVERGENCES}")
    print(f"[parity] nucleus tie-order divergences: {len(TIE_DIVERGENCES)} {TIE_DIVERGENCES}")
    print(f"[parity] nucleus rows: {dict(NUCLEUS_ROWS)}")
    assert len(DIVERGENCES) <= 6


# ---------------------------------------------------------------- n-gram verify (A11)
NGRAM_STEP_GRID = [
    # (g, V, dtype, kind, match drafts, stop at)
    (4, 4096, torch.bfloat16, "greedy", 2, None),
    (4, 4096, torch.bfloat16, "multi_t1", 3, None),
    (8, 4096, torch.bfloat16, "nucleus09", 8, None),
    (8, 4096, torch.bfloat16, "multi_t07", 1, None),
    (4, 4096, torch.bfloat16, "topk20", 4, None),
    (1, 4096, torch.float32, "multi_t1", 1, None),
    (0, 4096, torch.bfloat16, "multi_t1", 0, None),
    (4, 4096, torch.bfloat16, "greedy", 4, 1),
    (4, 128256, torch.bfloat16, "multi_t1", 2, None),
]


@pytest.mark.parametrize("g,V,dtype,kind,match,stop_at", NGRAM_STEP_GRID)
def test_ngram_verify_step_matches_oracle(sd, g, V, dtype, kind, match, stop_at):
    proc = KINDS[kind]
    seed = g * 31 + V % 97
    x = rand_logits((g + 1, V), torch.float32, seed, 3.0)
    hot = torch.randint(0, V, (g + 1,), generator=torch.Generator().manual_seed(seed + 1))
    x[torch.arange(g + 1), hot] += 25.0            # peaked rows: samples equal the argmax almost surely
    x = x.to(dtype)
    drafts = [int(hot[i]) if i < match else (int(hot[i]) + 1) % V for i in range(g)]
    stops = [drafts[stop_at]] if stop_at is not None else [3]
    K = 3
    variants = {}
    for exact in (False, True):
        gen = torch.Generator().manual_seed(5000 + seed)
        noise = ref.TorchNoise(gen)
        n, xo = ref.ngram_verify_step(x, drafts, proc, noise) if g > 0 else (0, None)
        if g == 0:
            xo = int(ref.sample(ref.process(x[0:1], proc, exact), proc, noise).reshape(-1)[0])
        stop = ref.stop_location(drafts[:n], stops)
        variants[exact] = (n, xo, stop, gen.get_state())
    gen2 = torch.Generator().manual_seed(5000 + seed)
    rows = [x[i:i + 1].to(DEV) for i in range(g + 1)]
    dt = torch.tensor([drafts], dtype=torch.long, device=DEV) if g else None
    out = sd.ops.ngram_verify(rows, dt, spec_of(sd, proc), sd.StreamNoise(gen2),
                              torch.tensor(stops, dtype=torch.long, device=DEV), filler_k=K)
    torch.cuda.synchronize()
    n, xg, stop = int(out.n_accepted[0]), int(out.next_token[0]), int(out.stop_index[0])
    ok = []
    for exact, (n_o, x_o, stop_o, state) in variants.items():
        # a stop among the accepted drafts returns before x is drawn: the oracle step drew x anyway
        want = (n_o, -1 if stop_o >= 0 else x_o, stop_o)
        if (n, xg, stop) == want:
            ok.append(exact)
            if stop_o < 0:
                assert torch.equal(gen2.get_state(), state)
    assert ok, ((n, xg, stop), variants)
    # filler ids: the top-K processed probabilities of every row (equal values may come in any order)
    p = ref.process(x, proc, True).float()
    got = out.filler_ids[0].cpu()
    for i in range(g + 1):
        want_vals = p[i].topk(K).values
        assert torch.equal(p[i][got[i]], want_vals), (i, got[i], p[i].topk(K))


with open(os.path.join(os.path.dirname(__file__), "golden", "ngram_loops.json")) as f:
    NGRAM_GOLDEN = json.load(f)


@pytest.mark.parametrize("store_kind", ["host", "device"])
@pytest.mark.parametrize("case", sorted(NGRAM_GOLDEN))
def test_ngram_loop_matches_reference(sd, case, store_kind):
    """The drop-in loop against the reference's own outputs, with the host drafter and with the
    device store (sd_ngram_store_*: draft_chain drafts the gamma tokens of a step in one launch)."""
    from specdec_amd.ngram_assisted import (DeviceNGramStorage, DeviceOneLevelNGramStorage, NGramStorage,
                                            OneLevelNGramStorage, ngram_assisted_speculative_generate)
    if store_kind == "device":
        NGramStorage, OneLevelNGramStorage = DeviceNGramStorage, DeviceOneLevelNGramStorage   # noqa: N806
    from specdec_amd.utils import logits_processor as lp
    c = NGRAM_GOLDEN[case]
    DTm = {"bf16": torch.bfloat16, "fp32": torch.float32}
    target, _ = make_pair(c["vocab"], dtype=DTm[c["dtype"]], device=DEV, pos_mult=c["pos_mult"], peak=c["peak"])
    pp = c["processor"]
    proc = golden_processor(lp, pp)
    store = (NGramStorage if c["storage"] == "multi" else OneLevelNGramStorage)(c["n"], c["vocab"])
    eos = c["eos"] if len(c["eos"]) > 1 else c["eos"][0]
    torch.manual_seed(c["seed"])
    out, rate = ngram_assisted_speculative_generate(c["prompt"], store, target, gamma=c["gamma"],
                                                    filler_top_k=c["filler_top_k"], logits_processor=proc,
                                                    max_gen_len=c["max_gen_len"], eos_tokens_id=eos,
                                                    stop_if_unknown=c["stop_if_unknown"])
    if out != c["tokens"] or rate != c["acceptance_rate"]:
        # a torch-CPU rounding flip: then the exact-arithmetic oracle must agree
        cpu_target, _ = make_pair(c["vocab"], dtype=DTm[c["dtype"]], pos_mult=c["pos_mult"], peak=c["peak"])
        kp = dataclasses.replace(golden_processor(ref, pp), stable_ties=True)
        torch.manual_seed(c["seed"])
        noise = ref.TorchNoise(None)
        st = ref.NgramStore(c["storage"], c["n"], c["vocab"], noise)
        want = ref.ngram_assisted_generate(c["prompt"], st, cpu_target, c["gamma"], c["filler_top_k"], kp,
                                           c["max_gen_len"], eos, 0, True, c["stop_if_unknown"], noise, exact=True)
        assert (out, rate) == want
        note_divergence("exact", f"ngram loop {case}")
