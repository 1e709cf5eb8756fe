"""The one-launch verify of few sequences (k_verify_lean, csrc/sd_verify_lean.inc) against the
two-launch verify (k_stats + k_sample, SD_OPT_LEAN_VERIFY = 0) on identical inputs and Philox noise.

Both paths take the same decisions from the same row statistics up to the summation order of Σexp
(~1e-7 relative), draw the same Philox uniforms and split the rows into the same 2048-element
sampling chunks, so their outputs agree row for row; a row may differ only where p(x)/q(x) or a
chunk boundary of the inverse CDF sits within that rounding (allowed: 1 row in 64).  Covers both
rules, plain / temperature / greedy / top-k / nucleus processors (keep predicates from the
threshold search), the drafter statistics from the draws or computed in the launch, ragged V,
stop tokens, and that the launch runs at all (its own phase of the parity suite goes through it
for every call with B <= 8).
"""
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def sd():
    from specdec_amd import _lib, ops
    from specdec_amd.noise import PhiloxNoise
    return SimpleNamespace(lib=_lib, ops=ops, PhiloxNoise=PhiloxNoise)


def rows(B, n, V, seed, scale=3.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(B, n, V, generator=g) * scale).to(torch.bfloat16).to(DEV)


def run(sd, lean, tl, dl, ids, rule, proc, with_stats, seed, stops=()):
    with sd.lib.option(sd.lib.SD_OPT_LEAN_VERIFY, 1 if lean else 0):
        return _run(sd, tl, dl, ids, rule, proc, with_stats, seed, stops)


def _run(sd, tl, dl, ids, rule, proc, with_stats, seed, stops):
    ops = sd.ops
    B, g = ids.shape
    dstats = None
    if with_stats:   # the drafter rows' (max, Σexp) from draws of the same rows, as the loops do
        dstats = torch.empty(g, B, 2, device=DEV)
        nz0 = sd.PhiloxNoise(seed=seed + 1000)
        for d in range(g):
            ops.sample_rows(dl[:, d].contiguous(), proc, nz0, row_stats_out=dstats[d])
    noise = sd.PhiloxNoise(seed=seed)
    n_t = tl.shape[1]
    out = ops.verify([tl[:, t] for t in range(n_t)], [dl[:, d] for d in range(g)], ids, rule, proc, proc, noise,
                     torch.tensor(list(stops), dtype=torch.long, device=DEV), draft_row_stats=dstats)
    torch.cuda.synchronize()
    res = {k: getattr(out, k).cpu() for k in ("n_accepted", "next_token", "row_status")}
    res["path"] = sd.lib.last_verify_path()
    return res


PROCS = [("multinomial", 1.0, 0, 0.0), ("multinomial", 0.7, 0, 0.0), ("greedy", 1.0, 0, 0.0),
         ("topk", 1.0, 20, 0.0), ("nucleus", 1.0, 0, 0.9), ("topknucleus", 0.8, 50, 0.9)]


@pytest.mark.parametrize("B,V", [(1, 128256), (3, 32000), (4, 6149)])
@pytest.mark.parametrize("rule", ["spec", "engine"])
@pytest.mark.parametrize("proc", PROCS, ids=[f"{p[0]}-T{p[1]}" for p in PROCS])
def test_lean_verify_equals_two_launch_verify(sd, B, V, rule, proc):
    g = 4
    kind, T, k, p = proc
    spec = sd.ops.ProcSpec(kind, T, k, p)
    r = sd.lib.SD_RULE_SPEC if rule == "spec" else sd.lib.SD_RULE_ENGINE
    n_t = g + 1 if rule == "spec" else g
    seed = 17 * B + V % 97 + (3 if rule == "spec" else 5)
    tl = rows(B, n_t, V, seed)
    dl = (tl[:, :g].float() + rows(B, g, V, seed + 1, 1.0).float()).to(torch.bfloat16)
    ids = dl.float().argmax(-1)   # drafts the target mostly agrees with: long accept walks
    ids[:, -1] = torch.randint(0, V, (B,), generator=torch.Generator().manual_seed(seed)).to(DEV)
    with_stats = kind in ("multinomial", "greedy")
    stops = (int(ids[0, 2]),) if B > 1 else ()
    a = run(sd, True, tl, dl, ids, r, spec, with_stats, seed, stops)
    b = run(sd, False, tl, dl, ids, r, spec, with_stats, seed, stops)
    # the lean kernel needs 16-byte aligned rows: [B, n_t, V] bf16 rows are when V % 8 == 0 (V = 6149 runs the
    # two-launch path on both sides: the ragged-V case of the two-launch kernels)
    want = sd.lib.SD_PATH_VERIFY_LEAN if V % 8 == 0 else sd.lib.SD_PATH_VERIFY_TWO_LAUNCH
    assert a.pop("path") == want and b.pop("path") == sd.lib.SD_PATH_VERIFY_TWO_LAUNCH
    assert not ((a["row_status"] | b["row_status"]) & 0x2C0).any()
    same = (a["n_accepted"] == b["n_accepted"]) & (a["next_token"] == b["next_token"]) & (a["row_status"] == b["row_status"])
    assert int((~same).sum()) <= B // 64, (a, b)


def test_lean_verify_runs_for_small_batches(sd):
    """The launch is taken (sd_last_verify_path reports it) for a batch-1 call under the default
    option, and not with SD_OPT_LEAN_VERIFY = 0."""
    g, V = 4, 128256
    tl = rows(1, g + 1, V, 1)
    dl = rows(1, g, V, 2)
    ids = dl.float().argmax(-1)
    spec = sd.ops.ProcSpec("multinomial", 1.0)
    assert sd.lib.get_option(sd.lib.SD_OPT_LEAN_VERIFY) == -1
    assert _run(sd, tl, dl, ids, sd.lib.SD_RULE_SPEC, spec, True, 3, ())["path"] == sd.lib.SD_PATH_VERIFY_LEAN
    assert run(sd, False, tl, dl, ids, sd.lib.SD_RULE_SPEC, spec, True, 3)["path"] == sd.lib.SD_PATH_VERIFY_TWO_LAUNCH
