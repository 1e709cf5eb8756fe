"""PHILOX (perf) mode of sd_verify: the decision runs in the tail of the row-statistics kernel
and the token is drawn by inverse CDF in the tail of the sampling kernel.

* accept walks are recomputed on the host from the exact-arithmetic oracle's p(x_i), q(x_i)
  and the numpy Philox (tests/philox_ref.py, pinned by Random123's known answers);
* greedy rows use no noise and must equal the oracle bit for bit;
* sampled tokens are checked in distribution (chi-square against the exact residual / p row),
  since perf mode reproduces the reference's multinomial, not torch's bit stream.

Each walk runs twice: without and with the drafter rows' statistics from real sd_sample draws of the
same rows (``draws``), as the decode loops pass them.  With them every B >= 8 call takes the one-launch
fused verify (k_verify_fused) — the kernel behind the bench's headline — and the tests assert that
path from sd_last_verify_path, so the fused kernel is pinned to the oracle directly, not only to the
two-launch path (tests/test_gpu_fused.py).
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import philox_ref as ph
from oracle import specdec_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
CHI2_P_MIN = 1e-4          # false-failure rate per distribution test


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
    """N(0,1) logits with n_hot tokens (spread over the whole row) boosted by ~8: most mass sits
    on a few dozen tokens in different sampling chunks."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(V, generator=g)
    hot = torch.randperm(V, generator=g)[:n_hot]
    x[hot] += 8.0 + torch.rand(n_hot, generator=g) * 2.0
    return x.to(dtype), hot


def draft_stats(sd, dl, proc, seed=4242):
    """(stats [γ, B, 2], keeps [γ, B, 4] or None) of the drafter rows dl [B, γ, V] as sd_sample returns
    them with its draws (the decode loops' draft_row_stats / draft_row_keep); the drawn tokens are
    discarded — the tests choose the drafts."""
    B, g = dl.shape[0], dl.shape[1]
    spec = spec_of(sd, proc)
    stats = torch.empty(g, B, 2, device=DEV)
    keeps = torch.empty(g, B, 4, dtype=torch.int32, device=DEV) if spec.keeps else None
    noise = sd.PhiloxNoise(seed=seed)
    for d in range(g):
        sd.ops.sample_rows(dl[:, d, :].contiguous(), spec, noise, row_stats_out=stats[d],
                           row_keep_out=keeps[d] if keeps is not None else None)
    return stats, keeps


def verify(sd, tl, dl, ids, rule, proc, noise, stops=(), draft_is_probs=False, draws=False, **kw):
    n_t = tl.shape[1]
    g = dl.shape[1]
    if draws:
        kw["draft_row_stats"], kw["draft_row_keep"] = draft_stats(sd, dl, proc)
    out = sd.ops.verify([tl[:, t, :] for t in range(n_t)], [dl[:, d, :] for d in range(g)], ids, rule,
                        spec_of(sd, proc), spec_of(sd, proc), noise,
                        torch.tensor(list(stops), dtype=torch.long, device=DEV),
                        draft_is_probs=draft_is_probs, **kw)
    out.path = sd.lib.last_verify_path()
    return out


def expect_path(sd, out, B, draws, stochastic=True):
    """With the draws' stats, B >= 8 stochastic calls take k_verify_fused (in ticket order from B = 64),
    B <= 8 k_verify_lean (where both apply, the lean kernel first: B == 8 bf16 plain rows)."""
    if not draws or not stochastic:
        return
    if B == 8:
        want = (sd.lib.SD_PATH_VERIFY_FUSED, sd.lib.SD_PATH_VERIFY_LEAN)
    elif B >= 64:
        want = (sd.lib.SD_PATH_VERIFY_FUSED_TICKET,)
    else:
        want = (sd.lib.SD_PATH_VERIFY_FUSED if B > 8 else sd.lib.SD_PATH_VERIFY_LEAN,)
    assert out.path in want, sd.lib.PATH_NAMES.get(out.path)


def flip_slack(logits_row, dtype):
    """Σ over the row's elements of how far its rounded probability can move when the softmax
    normaliser is off by 1e-6 (relative): the exact fp64 value, scaled by 1 ± 1e-6, rounded to the
    row's dtype both ways."""
    v = torch.softmax(logits_row.double(), dim=-1)
    return float(((v * (1 + 1e-6)).to(dtype).double() - (v * (1 - 1e-6)).to(dtype).double()).sum())


def chi2_check(samples, probs, label):
    """Pearson chi-square of integer samples against probabilities (bins with expected < 5 pooled)."""
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
    if exp_b[-1] < 5:   # too little pooled mass: fold it into the largest bin
        k = np.argmax(exp_b[:-1])
        obs_b[k] += obs_b[-1]
        exp_b[k] += exp_b[-1]
        obs_b, exp_b = obs_b[:-1], exp_b[:-1]
    stat, pval = chisquare(obs_b, exp_b)
    print(f"[perf] {label}: n={n} bins={len(obs_b)} chi2={stat:.1f} p={pval:.3g}")
    assert pval > CHI2_P_MIN, (label, stat, pval)


# ---------------------------------------------------------------- accept walk
def host_walk_spec(p, q, seed, off, b, g):
    """sampling/speculative_decoding.py:139-145 on Philox uniforms: n, and whether any comparison
    sat within fp32 rounding of the threshold (then the device may legitimately differ)."""
    n, close = g, False
    for i in range(g):
        r = ph.accept_uniform(seed, off, b, i)
        frac = np.float32(p[i]) / np.float32(q[i]) if q[i] != 0 else np.float32(np.inf if p[i] > 0 else np.nan)
        close |= bool(abs(float(r) - float(frac)) <= 1e-6 * max(1.0, float(frac)))
        if r > frac and n == g:
            n = i
    return n, close


def host_walk_engine(p, q, toks, ends, seed, off, b, g):
    """engine/infer_engine.py:297-330 on Philox uniforms: (n, rejected, finished, close)."""
    n, close = 0, False
    for i in range(g):
        u = float(ph.accept_uniform(seed, off, b, i))
        ap = 1.0 if q[i] <= 0 else min(1.0, float(p[i]) / float(q[i]))
        close |= abs(u - ap) <= 1e-6
        if u < ap:
            n += 1
            if int(toks[i]) in ends:
                return n, False, True, close
        else:
            return n, True, False, close
    return n, False, False, close


@pytest.mark.parametrize("draws", [False, True], ids=["stats-in-verify", "stats-from-draws"])
@pytest.mark.parametrize("kind,V,B,dtype", [("multi_t1", 4096, 64, torch.bfloat16),
                                            ("multi_t07", 4096, 16, torch.float32),
                                            ("topk50_t08", 8192, 16, torch.bfloat16),
                                            ("nucleus09", 4096, 8, torch.bfloat16),
                                            ("multi_t1", 128256, 32, torch.bfloat16),
                                            ("multi_t1", 50257, 8, torch.bfloat16),
                                            ("multi_t07", 50257, 32, torch.bfloat16)])
def test_perf_spec_accept_walk(sd, kind, V, B, dtype, draws):
    procs = {"multi_t1": ref.Processor("multinomial", 1.0), "multi_t07": ref.Processor("multinomial", 0.7),
             "topk50_t08": ref.Processor("topk", 0.8, 50), "nucleus09": ref.Processor("nucleus", 1.0, 0, 0.9)}
    proc = procs[kind]
    g = 4
    tl = rand_logits((B, g + 1, V), dtype, 11)
    dl = (tl[:, :g].float() + rand_logits((B, g, V), torch.float32, 12, 1.5)).to(dtype)
    gen = torch.Generator().manual_seed(13)
    ids = torch.randint(0, V, (B, g), generator=gen)
    # half the drafts from the drafter's top tokens so accepts happen
    ids[: B // 2] = dl[: B // 2].float().topk(2, dim=-1).indices[..., 1]
    noise = sd.PhiloxNoise(seed=0x1234_5678_9ABC, offset=5)
    off = noise.offset
    out = verify(sd, tl.to(DEV), dl.to(DEV), ids.to(DEV), sd.lib.SD_RULE_SPEC, proc, noise, draws=draws)
    expect_path(sd, out, B, draws)
    n = out.n_accepted.cpu().tolist()
    st = out.row_status.cpu().tolist()
    kd, kt = out.prune_drafter.cpu().tolist(), out.prune_target.cpu().tolist()
    x = out.next_token.cpu().tolist()
    stable = kind.startswith("nucleus")
    pproc = ref.Processor(proc.kind, proc.temperature, proc.top_k, proc.top_p, stable_ties=stable)
    close_rows = 0
    for b in range(B):
        pt = ref.process(tl[b, :g], pproc, exact=True).float()
        qd = ref.process(dl[b], pproc, exact=True).float()
        p = [float(pt[i, ids[b, i]]) for i in range(g)]
        q = [float(qd[i, ids[b, i]]) for i in range(g)]
        want, close = host_walk_spec(p, q, noise.seed, off, b, g)
        if n[b] != want:
            assert close, (b, n[b], want, p, q)
            close_rows += 1
            continue
        assert st[b] & sd.lib.SD_ROW_DONE
        if want == g:
            assert st[b] & sd.lib.SD_ROW_BONUS and kd[b] == 0 and kt[b] == 0
        else:
            assert st[b] & sd.lib.SD_ROW_RESIDUAL and kd[b] == g - want and kt[b] == g - want + 1
            # the residual token has positive residual weight
            pn = ref.process(tl[b, want], pproc, exact=True).float()
            assert float(pn[x[b]]) > float(qd[want, x[b]]), (b, x[b])
        assert 0 <= x[b] < V
    assert close_rows <= 1


@pytest.mark.parametrize("draws", [False, True], ids=["stats-in-verify", "stats-from-draws"])
@pytest.mark.parametrize("B,V,dtype", [(16, 4096, torch.bfloat16), (32, 128256, torch.bfloat16),
                                       (8, 50257, torch.float32), (8, 128256, torch.bfloat16),
                                       (32, 50257, torch.bfloat16),
                                       # the large-batch sweep's shapes (ticket-order fused verify)
                                       (128, 128256, torch.bfloat16), (512, 32768, torch.bfloat16)])
def test_perf_engine_accept_walk_and_state(sd, B, V, dtype, draws):
    g, step, gen_len = 4, 4, 12
    tl = rand_logits((B, g, V), dtype, 21)
    dl = (tl.float() + rand_logits((B, g, V), torch.float32, 22, 1.0)).to(dtype)
    gq = torch.Generator().manual_seed(23)
    qf = ref.softmax(dl, True).float()
    ids = torch.stack([torch.multinomial(qf[b], 1, generator=gq).squeeze(-1) for b in range(B)])
    ends = [int(ids[0, 1]), int(ids[3 % B, 0])]
    generated = torch.zeros(B, gen_len, dtype=torch.long)
    generated[:, step:step + g] = ids
    fin = torch.zeros(B, dtype=torch.uint8)
    acc = torch.full((B,), 7, dtype=torch.long)
    gen_d, fin_d, acc_d = generated.to(DEV), fin.to(DEV), acc.to(DEV)
    noise = sd.PhiloxNoise(seed=99, offset=1 << 33)
    off = noise.offset
    out = verify(sd, tl.to(DEV), dl.to(DEV), ids.to(DEV), sd.lib.SD_RULE_ENGINE, ref.Processor("multinomial", 1.0),
                 noise, stops=ends, engine_state=dict(generated=gen_d, step=step, finished=fin_d, accepted=acc_d),
                 draws=draws)
    expect_path(sd, out, B, draws)
    n = out.n_accepted.cpu().tolist()
    x = out.next_token.cpu().tolist()
    st = out.row_status.cpu().tolist()
    mass = out.resample_mass.cpu().tolist()
    gen_h, fin_h, acc_h = gen_d.cpu(), fin_d.cpu(), acc_d.cpu()
    pt = ref.softmax(tl, True).float()
    close_rows = 0
    for b in range(B):
        p = [float(pt[b, i, ids[b, i]]) for i in range(g)]
        q = [float(qf[b, i, ids[b, i]]) for i in range(g)]
        want, rejected, finished, close = host_walk_engine(p, q, ids[b], ends, noise.seed, off, b, g)
        if n[b] != want:
            assert close, (b, n[b], want)
            close_rows += 1
            continue
        assert int(acc_h[b]) == 7 + want
        expect = generated[b].clone()          # engine/infer_engine.py:326, :333-336
        if rejected:
            assert st[b] & (sd.lib.SD_ROW_RESIDUAL | sd.lib.SD_ROW_FALLBACK_P)
            assert 0 <= x[b] < V
            expect[step + want] = x[b]
            res = (pt[b, want].double() - qf[b, want].double()).clamp(min=0)
            # 1e-5 (the north star's tolerance) plus what one-ulp rounding flips of p and q can move:
            # the kernels' softmax normaliser is within ~1e-7 of the exact one, so an element whose
            # exact probability lies within 1e-6 (relative) of a rounding boundary may round either
            # way (at V = 32768, B = 512 such a flip of a large p moved one row's mass by 1.3e-5)
            slack = flip_slack(tl[b, want], dtype) + flip_slack(dl[b, want], dtype)
            assert abs(mass[b] - float(res.sum())) <= 1e-5 + slack, (b, mass[b], float(res.sum()), slack)
            assert float(res[x[b]]) > 0
            assert bool(fin_h[b]) == (x[b] in ends)
        else:
            assert x[b] == -1
            assert bool(fin_h[b]) == finished
        if want < g:
            expect[step + want + 1: step + g] = 0
        assert torch.equal(gen_h[b], expect), (b, gen_h[b], expect)
    assert close_rows <= 1


def test_perf_greedy_is_bit_exact(sd):
    """Greedy rows draw nothing: Philox mode must give the oracle's tokens exactly."""
    proc = ref.Processor("greedy")
    for seed, (B, V, dtype) in enumerate([(8, 4096, torch.bfloat16), (4, 50257, torch.float32),
                                          (4, 128256, torch.bfloat16)]):
        g = 4
        tl = rand_logits((B, g + 1, V), dtype, 31 + seed)
        dl = (tl[:, :g].float() + rand_logits((B, g, V), torch.float32, 41 + seed, 2.0)).to(dtype)
        ids = dl.float().argmax(-1)
        ids[:, -1] = torch.randint(0, V, (B,), generator=torch.Generator().manual_seed(seed))
        out = verify(sd, tl.to(DEV), dl.to(DEV), ids.to(DEV), sd.lib.SD_RULE_SPEC, proc, sd.PhiloxNoise(seed=5))
        got = list(zip(out.n_accepted.cpu().tolist(), out.next_token.cpu().tolist()))
        for b in range(B):
            wants = []
            for exact in (False, True):
                q = ref.process(dl[b], proc, exact).float()
                n, p = ref.spec_accept(tl[b], q, ids[b].tolist(), proc, torch.zeros(g) + 0.5, exact)
                st = ref.spec_resample(tl[b], q, p, n, proc, None, False, exact)
                wants.append((n, st.x))
            assert got[b] in wants, (seed, b, got[b], wants)


# ---------------------------------------------------------------- sampled distributions
def _collect(sd, calls, run):
    xs = []
    noise = sd.PhiloxNoise(seed=2024)
    for _ in range(calls):
        xs.append(run(noise))
    return np.concatenate(xs)


@pytest.mark.parametrize("V,n_hot", [(64, 0), (8192, 40), (128256, 60)])
def test_perf_residual_distribution(sd, V, n_hot):
    """SPEC reject at slot 0: the token must follow (p0 - q0)+ / Σ — across sampling chunks too."""
    proc = ref.Processor("multinomial", 1.0)
    B = 4096
    if n_hot:
        t0, hot = peaked_logits(V, n_hot, 1)
        d0 = t0.float().clone()
        d0[hot[: n_hot // 2]] += 1.5     # drafter over-weights half of the hot tokens
        d0 = d0.to(torch.bfloat16)
    else:
        t0, d0 = rand_logits((V,), torch.bfloat16, 2, 1.5), rand_logits((V,), torch.bfloat16, 3, 1.5)
    p0 = ref.process(t0, proc, exact=True).double()
    q0 = ref.process(d0, proc, exact=True).double()
    x = int(torch.argmax(q0 - p0))           # drafted token: q >> p, so most rows reject
    res = (p0.float() - q0.float()).clamp(min=0).double()
    tl = torch.stack([t0, t0]).unsqueeze(0).expand(B, 2, V).contiguous().to(DEV)
    dl = d0.view(1, 1, V).expand(B, 1, V).contiguous().to(DEV)
    ids = torch.full((B, 1), x, dtype=torch.long, device=DEV)

    def run(noise):
        out = verify(sd, tl, dl, ids, sd.lib.SD_RULE_SPEC, proc, noise)
        rej = (out.row_status & sd.lib.SD_ROW_RESIDUAL) != 0
        assert torch.allclose(out.resample_mass[rej].double().cpu(), res.sum().expand(int(rej.sum())), atol=1e-5)
        return out.next_token[rej].cpu().numpy()

    samples = _collect(sd, 6, run)
    assert len(samples) > B
    chi2_check(samples, res.numpy(), f"residual V={V}")


def test_perf_bonus_distribution(sd):
    """Full accept (q == p): the bonus token must follow the target's last row p_γ."""
    proc = ref.Processor("multinomial", 1.0)
    B, V = 4096, 8192
    t0, _ = peaked_logits(V, 30, 7)
    t1, _ = peaked_logits(V, 30, 8)
    tl = torch.stack([t0, t1]).unsqueeze(0).expand(B, 2, V).contiguous().to(DEV)
    dl = t0.view(1, 1, V).expand(B, 1, V).contiguous().to(DEV)
    ids = torch.full((B, 1), int(torch.argmax(t0.float())), dtype=torch.long, device=DEV)

    def run(noise):
        out = verify(sd, tl, dl, ids, sd.lib.SD_RULE_SPEC, proc, noise)
        assert ((out.row_status & sd.lib.SD_ROW_BONUS) != 0).all()
        return out.next_token.cpu().numpy()

    p1 = ref.process(t1, proc, exact=True).double()
    chi2_check(_collect(sd, 4, run), p1.numpy(), "bonus")


@pytest.mark.parametrize("case", ["residual", "bonus"])
def test_fused_verify_distributions(sd, case):
    """k_verify_fused's samplers (two 2048-element chunks per workgroup, the decider's chunk pick over
    the 63 chunk totals of a V=128256 row) at the bench's B=32: the residual token of a reject at
    slot 0 must follow (p0 - q0)+ / Σ, the bonus token of a full accept p1 — chi-square over many
    calls (each call draws with a fresh Philox offset).  sampling/speculative_decoding.py:139-171."""
    proc = ref.Processor("multinomial", 1.0)
    B, V = 32, 128256
    t0, hot = peaked_logits(V, 60, 21)
    t1, _ = peaked_logits(V, 60, 22)
    if case == "residual":
        d0 = t0.float().clone()
        d0[hot[:30]] += 1.5            # the drafter over-weights half of the hot tokens
        d0 = d0.to(torch.bfloat16)
        p0 = ref.process(t0, proc, exact=True).double()
        q0 = ref.process(d0, proc, exact=True).double()
        x = int(torch.argmax(q0 - p0))  # q >> p at the draft: most rows reject at slot 0
        want = (p0.float() - q0.float()).clamp(min=0).double()
        calls = 200
    else:
        d0 = t0                        # q == p: every draft accepted, the bonus row drawn
        x = int(torch.argmax(t0.float()))
        want = ref.process(t1, proc, exact=True).double()
        calls = 160
    tl = torch.stack([t0, t1]).unsqueeze(0).expand(B, 2, V).contiguous().to(DEV)
    dl = d0.view(1, 1, V).expand(B, 1, V).contiguous().to(DEV)
    ids = torch.full((B, 1), x, dtype=torch.long, device=DEV)
    stats, _ = draft_stats(sd, dl, proc)
    noise = sd.PhiloxNoise(seed=77)
    xs = []
    for _ in range(calls):
        out = verify(sd, tl, dl, ids, sd.lib.SD_RULE_SPEC, proc, noise, draft_row_stats=stats)
        assert out.path == sd.lib.SD_PATH_VERIFY_FUSED, sd.lib.PATH_NAMES.get(out.path)
        flag = sd.lib.SD_ROW_RESIDUAL if case == "residual" else sd.lib.SD_ROW_BONUS
        sel = (out.row_status & flag) != 0
        assert not (out.row_status & sd.lib.SD_ROW_ERROR_MASK).any()
        if case == "residual":
            assert torch.allclose(out.resample_mass[sel].double().cpu(), want.sum().expand(int(sel.sum())), atol=1e-5)
        else:
            assert sel.all()
        xs.append(out.next_token[sel].cpu().numpy())
    samples = np.concatenate(xs)
    assert len(samples) > 0.5 * B * calls
    chi2_check(samples, want.numpy(), f"fused {case} V={V} B={B}")


def test_perf_engine_fallback_distribution(sd):
    """ENGINE reject with Σ(p - q)+ == 0 (q = p except q(x) = 2 p(x), fp32 probabilities): the
    reference falls back to multinomial(p) (engine/infer_engine.py:319-321)."""
    B, V = 4096, 8192
    t0, hot = peaked_logits(V, 30, 9)
    p0 = ref.softmax(t0, True)                       # bf16 probabilities
    x = int(hot[0])
    q0 = p0.float().clone()
    q0[x] *= 2.0
    tl = t0.view(1, 1, V).expand(B, 1, V).contiguous().to(DEV)
    ql = q0.view(1, 1, V).expand(B, 1, V).contiguous().to(DEV)
    ids = torch.full((B, 1), x, dtype=torch.long, device=DEV)

    def run(noise):
        out = verify(sd, tl, ql, ids, sd.lib.SD_RULE_ENGINE, ref.Processor("multinomial", 1.0), noise,
                     draft_is_probs=True)
        rej = out.n_accepted == 0
        assert ((out.row_status[rej] & sd.lib.SD_ROW_FALLBACK_P) != 0).all()
        assert (out.resample_mass[rej] == 0).all()
        return out.next_token[rej].cpu().numpy()

    samples = _collect(sd, 4, run)
    assert 0.4 * 4 * B < len(samples) < 0.6 * 4 * B      # reject probability 1 - p/q = 1/2
    chi2_check(samples, p0.double().numpy(), "engine fallback")


def test_perf_workspace_counters_survive_mixed_calls(sd):
    """Calls of different shapes (and sd_sample) sharing the workspace leave the arrival counters
    consistent: a repeated call reproduces its first result."""
    proc = ref.Processor("multinomial", 1.0)

    def case(B, V, seed):
        tl = rand_logits((B, 5, V), torch.bfloat16, seed)
        dl = (tl[:, :4].float() + rand_logits((B, 4, V), torch.float32, seed + 1, 1.0)).to(torch.bfloat16)
        ids = dl.float().argmax(-1)
        return tl.to(DEV), dl.to(DEV), ids.to(DEV)

    a = case(8, 8192, 1)
    first = verify(sd, *a, sd.lib.SD_RULE_SPEC, proc, sd.PhiloxNoise(seed=3, offset=0))
    verify(sd, *case(2, 4096, 2), sd.lib.SD_RULE_SPEC, proc, sd.PhiloxNoise(seed=4))
    sd.ops.sample_rows(rand_logits((3, 4096), torch.bfloat16, 5).to(DEV), spec_of(sd, proc), sd.PhiloxNoise(seed=6))
    tl, dl, ids = case(40, 2048, 7)
    verify(sd, tl[:, :4].contiguous(), dl, ids, sd.lib.SD_RULE_ENGINE, proc, sd.PhiloxNoise(seed=8))
    again = verify(sd, *a, sd.lib.SD_RULE_SPEC, proc, sd.PhiloxNoise(seed=3, offset=0))
    for f in ("n_accepted", "next_token", "row_status", "prune_drafter", "prune_target"):
        assert torch.equal(getattr(first, f), getattr(again, f)), f


def test_perf_repeat_and_graph_replay_are_deterministic(sd):
    """The bench shape (B=32, γ=4, V=128256 bf16, engine rule), same inputs and Philox offset:
    40 eager calls and 40 hipGraph replays must all give the first call's outputs — a stale
    cross-XCD read of a partial would show up as a changed decision or token."""
    B, g, V = 32, 4, 128256
    tl = rand_logits((B, g, V), torch.bfloat16, 51).to(DEV)
    dl = (tl.float() + rand_logits((B, g, V), torch.float32, 52, 1.0).to(DEV)).to(torch.bfloat16)
    ids = dl.float().argmax(-1)
    proc = ref.Processor("multinomial", 1.0)
    fields = ("n_accepted", "next_token", "row_status", "resample_mass")

    def call():
        out = verify(sd, tl, dl, ids, sd.lib.SD_RULE_ENGINE, proc, sd.PhiloxNoise(seed=77, offset=3))
        # bit patterns: resample_mass is NaN on rows without a residual
        return [getattr(out, f).clone().view(torch.int32) if f == "resample_mass" else getattr(out, f).clone()
                for f in fields]

    want = call()
    assert ((want[2] & sd.lib.SD_ROW_RESIDUAL) != 0).any()
    for _ in range(40):
        got = call()
        for f, a, b in zip(fields, want, got):
            assert torch.equal(a, b), f
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        call()                                     # warm the workspace on this stream
        with torch.cuda.graph(graph, stream=stream):
            outs = call()
    torch.cuda.current_stream().wait_stream(stream)
    for _ in range(40):
        graph.replay()
        torch.cuda.synchronize()
        for f, a, b in zip(fields, want, outs):
            assert torch.equal(a, b), f


def test_perf_sharded_calls_equal_one_call(sd):
    """Data-parallel shards: verifying rows [0, 13) and [13, 32) in two calls with
    row_base = shard start gives exactly the one-call outputs — noise is keyed by the global row."""
    B, g, V = 32, 4, 8192
    tl = rand_logits((B, g, V), torch.bfloat16, 61).to(DEV)
    dl = (tl.float() + rand_logits((B, g, V), torch.float32, 62, 1.0).to(DEV)).to(torch.bfloat16)
    ids = dl.float().argmax(-1)
    proc = ref.Processor("multinomial", 1.0)
    fields = ("n_accepted", "next_token", "row_status")
    whole = verify(sd, tl, dl, ids, sd.lib.SD_RULE_ENGINE, proc, sd.PhiloxNoise(seed=9, offset=4))
    parts = []
    for lo, hi in ((0, 13), (13, 32)):
        parts.append(verify(sd, tl[lo:hi], dl[lo:hi], ids[lo:hi], sd.lib.SD_RULE_ENGINE, proc,
                            sd.PhiloxNoise(seed=9, offset=4), row_base=lo))
    for f in fields:
        assert torch.equal(getattr(whole, f), torch.cat([getattr(p, f) for p in parts])), f
    # drafter sampling shards the same way
    tok_all, _, _ = sd.ops.sample_rows(dl[:, 0], spec_of(sd, proc), sd.PhiloxNoise(seed=3))
    tok_a, _, _ = sd.ops.sample_rows(dl[:13, 0], spec_of(sd, proc), sd.PhiloxNoise(seed=3))
    tok_b, _, _ = sd.ops.sample_rows(dl[13:, 0], spec_of(sd, proc), sd.PhiloxNoise(seed=3), row_base=13)
    assert torch.equal(tok_all, torch.cat([tok_a, tok_b]))


def test_batches_beyond_one_call_are_row_sharded(sd):
    """More sequences than one Philox call holds (16384, the kernels' arrival-counter block): ops
    splits the batch into row shards that share the call's noise offset (noise keyed by the global
    row), so every shard equals the direct call over its rows with row_base = its first row."""
    B, g, V = sd.ops.MAX_ROWS_PER_CALL + 40, 2, 256
    tl = rand_logits((B, g, V), torch.bfloat16, 91).to(DEV)
    dl = (tl.float() + rand_logits((B, g, V), torch.float32, 92, 1.0).to(DEV)).to(torch.bfloat16)
    ids = dl.float().argmax(-1)
    proc = ref.Processor("multinomial", 1.0)
    out = verify(sd, tl, dl, ids, sd.lib.SD_RULE_ENGINE, proc, sd.PhiloxNoise(seed=12, offset=7))
    assert ((out.row_status & sd.lib.SD_ROW_DONE) != 0).all()
    lo = sd.ops.MAX_ROWS_PER_CALL - 8
    part = verify(sd, tl[lo:], dl[lo:], ids[lo:], sd.lib.SD_RULE_ENGINE, proc, sd.PhiloxNoise(seed=12, offset=7),
                  row_base=lo)
    for f in ("n_accepted", "next_token", "row_status"):
        assert torch.equal(getattr(out, f)[lo:], getattr(part, f)), f
    tok, _, st = sd.ops.sample_rows(dl[:, 0].contiguous(), spec_of(sd, proc), sd.PhiloxNoise(seed=3))
    tok2, _, _ = sd.ops.sample_rows(dl[lo:, 0].contiguous(), spec_of(sd, proc), sd.PhiloxNoise(seed=3), row_base=lo)
    assert torch.equal(tok[lo:], tok2) and (st & sd.lib.SD_ROW_DONE).all()
