"""The one-pass greedy draw (k_draw_lean<GREEDY>, sd_sample of greedy rows) against the oracle.

GreedyProcessor.sample = argmax of softmax(logits) in the row's dtype, first index on ties
(utils/logits_processor.py:26-36).  The kernel picks it in one pass from per-span maxima: the
winner lies in a span whose max rounds to the row's top probability, and a span holding other
values within 1/32 of its max is rescanned exactly.  The inputs here force every branch: ties of
the max across spans, distinct logits whose probabilities round to the same top value (the first
of them wins, not the largest logit), dense near-max values (rescans), flat rows (fp16
subnormal tops), -inf spans, NaN / inf rows, the ragged last span.
"""
import pytest
import torch

from oracle import specdec_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
GREEDY = ref.Processor("greedy")


def oracle_tokens(x):
    """token ids a correct result may equal: torch-CPU arithmetic (the reference) or exact softmax."""
    outs = []
    for exact in (False, True):
        p = ref.process(x, GREEDY, exact)
        outs.append(torch.argmax(p, dim=-1))
    return outs


def run(x):
    from specdec_amd import PhiloxNoise, ops
    R = x.shape[0]
    stats = torch.empty(R, 2, device=DEV)
    tok, prob, st = ops.sample_rows(x.to(DEV), ops.ProcSpec("greedy"), PhiloxNoise(1), want_prob=True,
                                    row_stats_out=stats)
    return tok.cpu(), prob.cpu(), st.cpu(), stats.cpu()


def rows_case(kind, V, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(4, V, generator=g) * 3.0
    if kind == "tie_across_spans":          # the max value repeated in later spans: the first wins
        m = float(x.max()) + 1.0
        for r in range(4):
            for j in sorted(torch.randint(0, V, (3,), generator=g).tolist()):
                x[r, j] = m
    elif kind == "rounding_ties":           # distinct logits whose probabilities round alike
        x = x - 20.0                        # a peaked row: the top probability is ~1 - tiny
        for r in range(4):
            js = torch.randint(0, V, (4,), generator=g).tolist()
            for k, j in enumerate(js):
                x[r, j] = 0.25 - 0.001 * k  # bf16 values within 2^-9 of each other
    elif kind == "dense_near_max":          # distinct values within 1/32 of the max in one span (rescans)
        x = x * 0.1
        for r in range(4):
            j0 = int(torch.randint(0, V - 2048, (1,), generator=g))
            x[r, j0:j0 + 2048] = 2.0 - torch.rand(2048, generator=g) * 0.03
    elif kind == "flat":                    # all equal: the top probability is 1/V (fp16 subnormal)
        x = torch.zeros(4, V)
    elif kind == "neg_inf_spans":           # whole spans masked out
        x[:, :4096] = float("-inf")
        x[:, 8192:12288] = float("-inf")
    return x.to(dtype)


@pytest.mark.parametrize("kind", ["random", "tie_across_spans", "rounding_ties", "dense_near_max", "flat",
                                  "neg_inf_spans"])
@pytest.mark.parametrize("dtype,V", [(torch.bfloat16, 128256), (torch.float16, 128256), (torch.bfloat16, 4096),
                                     (torch.bfloat16, 32000)])
def test_greedy_draw_equals_the_oracle(kind, dtype, V):
    if kind == "neg_inf_spans" and V < 16384:
        pytest.skip("needs several spans")
    x = rows_case(kind, V, dtype, hash((kind, V)) % 997)
    tok, prob, st, stats = run(x)
    wants = oracle_tokens(x)
    for r in range(x.shape[0]):
        assert any(int(tok[r]) == int(w[r]) for w in wants), (kind, r, int(tok[r]), [int(w[r]) for w in wants])
    assert bool(((st & 0x1) != 0).all()) and not bool((st & 0x40).any())
    # the token's processed probability and the row statistics
    p_exact = ref.process(x, GREEDY, True)
    got_p = p_exact.float().gather(1, tok.view(-1, 1)).squeeze(1)
    torch.testing.assert_close(prob, got_p, rtol=1e-2, atol=0)   # one bf16 / fp16 ulp
    xf = x.float()
    M = xf.max(dim=1).values
    S = torch.exp(xf - M[:, None]).sum(dim=1)
    assert torch.equal(stats[:, 0], M)
    torch.testing.assert_close(stats[:, 1], S, rtol=2e-6, atol=0)


def test_greedy_draw_flags_nan_rows():
    x = torch.randn(3, 128256).to(torch.bfloat16)
    x[1, 777] = float("nan")
    x[2, 5] = float("inf")
    tok, prob, st, stats = run(x)
    assert int(st[0]) & 0x40 == 0
    assert int(st[1]) & 0x40 and int(st[2]) & 0x40      # torch would see NaN probabilities
    want = oracle_tokens(x[:1])
    assert any(int(tok[0]) == int(w[0]) for w in want)


def test_greedy_draw_many_rows_counter_mode():
    """More rows than the poll mode's resident-consumer bound: the arrival-counter exchange."""
    x = (torch.randn(2048, 4096, generator=torch.Generator().manual_seed(3)) * 3).to(torch.bfloat16)
    tok, _, st, _ = run(x)
    wants = oracle_tokens(x)
    ok = (tok == wants[0]) | (tok == wants[1])
    assert bool(ok.all())
