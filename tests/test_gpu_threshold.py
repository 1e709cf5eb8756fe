"""Top-k / nucleus keep sets of the 16-bit histogram threshold kernels (sd_threshold.inc) against
the exact-arithmetic oracle (utils/logits_processor.py:59-103 restated in oracle/specdec_ref.py,
fp64 softmax, equal values kept lowest index first), through sd_probs.

Every test runs on both designs: the in-launch exchanges of k_thr_hist (slice maxima, tie search
and radix hand-over through polled records) and the separate k_thr_max / k_thr_tie launches.
Covers every path: one and many slices per row, a partial last slice,
unaligned rows (scalar loads), fp16 keys (top-k: the reference's -1e20 fill raises in fp16),
cuts inside long runs of equal values (the sliced tie
search), and the rows handed to the radix descent (top-k rank or nucleus crossing below the
histogram window).  A kept element is one whose processed probability is positive in both.
"""
import dataclasses

import pytest
import torch

from oracle import specdec_ref as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from specdec_amd import ops
    return ops


@pytest.fixture(autouse=True, params=["in-launch", "launches"])
def thr_design(request, monkeypatch):
    """The slice maxima, tie search and radix hand-over inside k_thr_hist (polled records, the
    default when the grid is resident) or in k_thr_max / k_thr_tie launches of their own
    (SD_OPT_THRESHOLD_POLL = 0); the library reads the option on every call."""
    from specdec_amd import _lib
    with _lib.option(_lib.SD_OPT_THRESHOLD_POLL, 1 if request.param == "in-launch" else 0):
        yield request.param


def normal_rows(R, V, dtype, seed, scale=3.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(R, V, generator=g) * scale).to(dtype)


def tied_rows(R, V, dtype, seed):
    # values from a handful of levels: every cut falls inside a run of thousands of equal values
    g = torch.Generator().manual_seed(seed)
    return (torch.randint(0, 6, (R, V), generator=g).float() * 0.75).to(dtype)


def below_window_rows(R, V, dtype, seed):
    # a small positive max and the mass on ~3000 negative values: the nucleus crossing lies far below
    # the 8192 keys under the max (the radix fallback).  The rest sits at -40 (p ~ 1e-18), so every
    # kept p is >= 2^-17 and the reference's fp32 running sum is exact (an exactly comparable row).
    g = torch.Generator().manual_seed(seed)
    x = torch.full((R, V), -40.0)
    idx = torch.randperm(V, generator=g)[:3000]
    x[:, idx] = -1.0 + 0.3 * torch.randn(R, 3000, generator=g)
    x[:, 7] = 1e-3
    return x.to(dtype)


def check_rows(ops, rows, proc):
    spec = ops.ProcSpec(proc.kind, 1.0, proc.top_k, proc.top_p)
    got = ops.probs_rows(rows.cuda(), spec).float().cpu() > 0
    exact = dataclasses.replace(proc, stable_ties=True)
    # fp16 rows: the reference cannot fill -1e20 into fp16 (torch raises); top-k ranks values only,
    # so its keep set is checked on the same values in fp32
    orows = rows.float() if rows.dtype == torch.float16 else rows
    for r in range(rows.shape[0]):
        want = ref.process(orows[r:r + 1], exact, exact=True)[0].float() > 0
        diff = torch.nonzero(got[r] != want).flatten().tolist()
        assert not diff, (r, int(got[r].sum()), int(want.sum()), diff[:8])


PROCS = {
    "topk50": ref.Processor("topk", 1.0, 50),
    "topk100k": ref.Processor("topk", 1.0, 100000),   # rank below the window: radix fallback
    "nucleus09": ref.Processor("nucleus", 1.0, 0, 0.9),
    "nucleus05": ref.Processor("nucleus", 1.0, 0, 0.5),
    "topknucleus": ref.Processor("topknucleus", 1.0, 50, 0.9),
    "topk2000_nucleus099": ref.Processor("topknucleus", 1.0, 2000, 0.99),
}

CASES = [
    # (rows, V, dtype, maker, proc, seed)
    (9, 128256, torch.bfloat16, normal_rows, "topk50", 0),
    (9, 128256, torch.bfloat16, normal_rows, "nucleus09", 1),
    (3, 128256, torch.bfloat16, normal_rows, "nucleus05", 2),
    (3, 128256, torch.bfloat16, normal_rows, "topknucleus", 3),
    (2, 128256, torch.bfloat16, normal_rows, "topk2000_nucleus099", 4),
    (2, 128256, torch.bfloat16, normal_rows, "topk100k", 5),
    (3, 128256, torch.float16, normal_rows, "topk50", 7),
    (3, 50257, torch.bfloat16, normal_rows, "nucleus09", 8),        # unaligned rows, partial slice
    (2, 4096, torch.bfloat16, normal_rows, "topknucleus", 9),       # one slice
    (3, 128256, torch.bfloat16, tied_rows, "nucleus09", 10),
    (2, 128256, torch.bfloat16, tied_rows, "topknucleus", 11),
    (2, 128256, torch.bfloat16, below_window_rows, "nucleus09", 12),
]


@pytest.mark.parametrize("R,V,dtype,maker,pname,seed", CASES,
                         ids=[f"{c[0]}x{c[1]}-{str(c[2])[6:]}-{c[3].__name__}-{c[4]}" for c in CASES])
def test_keep_set_matches_exact_oracle(ops, R, V, dtype, maker, pname, seed):
    check_rows(ops, maker(R, V, dtype, seed), PROCS[pname])


def test_nan_and_inf_rows_take_the_radix_path(ops):
    rows = normal_rows(3, 128256, torch.bfloat16, 14)
    rows[1, 100] = float("inf")
    rows[2, 5] = float("nan")
    spec = ops.ProcSpec("nucleus", 1.0, 0, 0.9)
    p = ops.probs_rows(rows.cuda(), spec).float().cpu()
    # the clean row is exact; the others complete (no hang) with the radix path's result
    check_rows(ops, rows[:1], PROCS["nucleus09"])
    assert p.shape == rows.shape


def test_repeated_calls_identical(ops):
    rows = normal_rows(4, 128256, torch.bfloat16, 15).cuda()
    spec = ops.ProcSpec("topknucleus", 1.0, 50, 0.9)
    first = ops.probs_rows(rows, spec).clone()
    for _ in range(10):
        assert torch.equal(ops.probs_rows(rows, spec), first)
