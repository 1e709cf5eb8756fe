"""The one-launch fused verify (k_verify_fused: spans, a decider and two-chunk samplers per sequence,
csrc/specdec_kernels.hip) against the two-launch verify (k_stats + k_sample, SD_OPT_FUSED_VERIFY = 0) on identical
inputs and Philox noise.

Both take the decision from the same row statistics (the same k_stats span code and decide tail),
sample the decided row in the same 2048-element chunks with the same chunk uniforms and pick the
chunk with the same fp64 scan, so their outputs are identical, row for row — including the engine
state the verify updates in place and the per-row counters.  Also: the path is taken (B >= 8,
sd_last_verify_path) and a poll that gives up (spin limit < 0) flags rows instead of returning tokens.
The fused kernel's outputs are also checked against the oracle directly: tests/test_gpu_perfmode.py
(the accept walks with the drafter stats from the draws, and the residual / bonus chi-squares)."""
import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def fused(value):
    from specdec_amd import _lib
    return _lib.option(_lib.SD_OPT_FUSED_VERIFY, value)


def inputs(B, g, V, rule, seed):
    gen = torch.Generator(device=DEV).manual_seed(seed)
    n_t = g + 1 if rule == "spec" else g
    tl = (torch.randn(B, n_t, V, generator=gen, device=DEV) * 3).to(torch.bfloat16)
    dl = (tl[:, :g].float() + torch.randn(B, g, V, generator=gen, device=DEV)).to(torch.bfloat16)
    return tl, dl


def run(tl, dl, rule, spec, seed, engine=False, verify_ctx=contextlib.nullcontext):
    from specdec_amd import PhiloxNoise, _lib, ops
    B, g = dl.shape[0], dl.shape[1]
    noise = PhiloxNoise(seed=seed)
    draft = torch.zeros(B, g, dtype=torch.long, device=DEV)
    stats = torch.empty(g, B, 2, device=DEV)
    keep = torch.empty(g, B, 4, dtype=torch.int32, device=DEV) if spec.keeps else None
    for d in range(g):
        ops.sample_rows(dl[:, d], spec, noise, tokens_out=draft[:, d], row_stats_out=stats[d],
                        row_keep_out=keep[d] if keep is not None else None)
    r = _lib.SD_RULE_SPEC if rule == "spec" else _lib.SD_RULE_ENGINE
    extra = {}
    state = None
    if engine:
        gen_ids = torch.zeros(B, 3 * g, dtype=torch.long, device=DEV)
        state = dict(generated=gen_ids, step=g, finished=torch.zeros(B, dtype=torch.uint8, device=DEV),
                     accepted=torch.zeros(B, dtype=torch.long, device=DEV))
        extra = dict(engine_state=state, active=(torch.arange(B, device=DEV) % 5 != 3).to(torch.uint8))
    counts = torch.zeros(B, 2, dtype=torch.long, device=DEV)
    torch.cuda.synchronize()
    with verify_ctx():
        out = ops.verify([tl[:, t] for t in range(tl.shape[1])], [dl[:, d] for d in range(g)], draft, r, spec, spec,
                         noise, torch.tensor([int(draft[0, 1])], device=DEV), draft_row_stats=stats,
                         draft_row_keep=keep, row_counts=counts, **extra)
        torch.cuda.synchronize()
    res = {k: getattr(out, k).cpu() for k in ("n_accepted", "next_token", "row_status", "resample_mass")}
    res["path"] = torch.tensor(_lib.last_verify_path())
    res["counts"] = counts.cpu()
    if state is not None:
        res.update({k: v.cpu() for k, v in state.items() if torch.is_tensor(v)})
    return res


PROCS = [("multinomial", 1.0, 0, 0.0), ("multinomial", 0.7, 0, 0.0), ("topk", 1.0, 50, 0.0)]


def ticket(value):
    from specdec_amd import _lib
    return _lib.option(_lib.SD_OPT_FUSED_TICKET, value)


def samp_chunks(value):
    from specdec_amd import _lib
    return _lib.option(_lib.SD_OPT_SAMP_CHUNKS, value)


@pytest.mark.parametrize("B,V,tk,sc", [(8, 128256, -1, 0), (32, 128256, -1, 0), (16, 50257, -1, 0),
                                       # ticket order: forced at small batches, by default from B = 64
                                       (8, 128256, 1, 0), (32, 128256, 1, 0), (128, 128256, -1, 0),
                                       (300, 50257, -1, 0),
                                       # chunks per sampler (ticket order; 4 by default there)
                                       (128, 128256, -1, 2), (128, 128256, -1, 8), (300, 50257, -1, 2),
                                       (8, 128256, 1, 4)])
@pytest.mark.parametrize("rule", ["engine", "spec"])
@pytest.mark.parametrize("proc", PROCS, ids=[f"{p[0]}-T{p[1]}" for p in PROCS])
def test_fused_verify_equals_two_launch_verify(B, V, tk, sc, rule, proc):
    from specdec_amd import ops
    spec = ops.ProcSpec(*proc)
    seed = 31 * B + V % 89 + (1 if rule == "spec" else 2)
    tl, dl = inputs(B, 4, V, rule, seed)
    engine = rule == "engine"
    from specdec_amd import _lib
    with fused(1), ticket(tk), samp_chunks(sc):
        a = run(tl, dl, rule, spec, seed, engine)
    with fused(0):
        b = run(tl, dl, rule, spec, seed, engine)
    want = _lib.SD_PATH_VERIFY_FUSED_TICKET if tk == 1 or B >= 64 else _lib.SD_PATH_VERIFY_FUSED
    pa = int(a.pop("path"))
    assert pa == want, _lib.PATH_NAMES.get(pa)
    assert int(b.pop("path")) == _lib.SD_PATH_VERIFY_TWO_LAUNCH
    for k in a:
        assert torch.equal(a[k].nan_to_num(), b[k].nan_to_num()), (k, a[k], b[k])
    active = (torch.arange(B) % 5 != 3) if engine else torch.ones(B, dtype=torch.bool)
    assert (a["row_status"][active] & 0x1).all()          # every active row decided
    assert not (a["row_status"][~active] & 0x1).any()     # inactive engine rows untouched (:250-258)
    assert not (a["row_status"] & 0x2C0).any()


def test_fused_verify_polls_are_bounded():
    """Every in-launch poll of the fused verify forced to give up (spin limit < 0, the draws before
    it under the normal policy): its rows come back flagged SD_ROW_EXCHANGE_TIMEOUT (+ invalid), the
    call returns — no hang, no tokens taken as valid."""
    from specdec_amd import _lib, get_poll_policy, ops, set_poll_policy
    spec = ops.ProcSpec("multinomial", 1.0)
    tl, dl = inputs(32, 4, 128256, "engine", 5)

    @contextlib.contextmanager
    def no_polls():
        old = get_poll_policy()
        set_poll_policy(True, -1)
        try:
            yield
        finally:
            set_poll_policy(*old)

    with fused(0):   # the two-launch path: an independent reference for every row
        two = run(tl, dl, "engine", spec, 5)
    with fused(1):
        ref = run(tl, dl, "engine", spec, 5)
        for k in ("n_accepted", "next_token", "row_status"):
            assert torch.equal(ref[k], two[k]), (k, (ref[k] != two[k]).nonzero().flatten(), ref["row_status"])
        a = run(tl, dl, "engine", spec, 5, verify_ctx=no_polls)
        # the next calls on the same workspace are healthy: nothing the timed-out call left behind (its
        # records, its samplers, its epoch) is taken as theirs — no flags, the same outputs as before
        b = run(tl, dl, "engine", spec, 5)
        c = run(tl, dl, "engine", spec, 5)
    assert int(a["path"]) == _lib.SD_PATH_VERIFY_FUSED
    # every row flagged: the hook makes every poll give up, the decider's span records included
    assert (a["row_status"] & _lib.SD_ROW_EXCHANGE_TIMEOUT).all(), a["row_status"]
    assert (a["row_status"] & _lib.SD_ROW_INVALID_DIST).all()
    for o in (b, c):
        assert int(o["path"]) == _lib.SD_PATH_VERIFY_FUSED
        assert not (o["row_status"] & (_lib.SD_ROW_EXCHANGE_TIMEOUT | _lib.SD_ROW_INVALID_DIST)).any()
        for k in ("n_accepted", "next_token", "row_status"):
            assert torch.equal(o[k], ref[k]), k
