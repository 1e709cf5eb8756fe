"""The benchmark-facing surface of the drop-in engine, on CPU, against the reference's own outputs
(tests/golden/engine_surface.json from make_golden.py --only surface):

* engine/metrics.py — BenchmarkResults.to_dict (every key and value) and the printed summaries of
  a fixed synthetic result set built with the drop-in's classes;
* the target-only baseline (engine/infer_engine.py:407-497) — outputs on FakeLM banks, greedy and
  multinomial T=0.7 (torch's CPU generator, the reference's draws);
* infer_batch with target_gen returns (None, BatchMetrics) like the reference (:80-84);
* run_batch_speculative's metrics rules on stubbed decode results (the decode itself is GPU-only:
  tests/test_gpu_engine_surface.py checks it against the reference's run_batch_speculative);
* prune_cache on a real transformers-5 DynamicCache against the tuple-cache golden shapes.
"""
import contextlib
import io
import json
import os
import sys
from types import SimpleNamespace

import pytest
import torch

from fakelm import TupleFakeLM, bank_digest, make_pair

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden import synthetic_results  # noqa: E402

from specdec_amd.engine import infer_engine as ie  # noqa: E402
from specdec_amd.engine import metrics as em  # noqa: E402
from specdec_amd.utils import caching  # noqa: E402

with open(os.path.join(HERE, "golden", "engine_surface.json")) as f:
    GOLD = json.load(f)
DT = {"bf16": torch.bfloat16, "fp32": torch.float32}


def test_benchmark_results_to_dict_matches_reference():
    res = synthetic_results(em)
    for method, want in GOLD["to_dict"].items():
        got = json.loads(json.dumps(res[method].to_dict()))
        assert got == want, method


def test_printed_summaries_match_reference():
    res = synthetic_results(em)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        em.print_benchmark_summary(res["speculative"])
        em.print_benchmark_summary(res["target_ar"])
        em.print_comparison(res["speculative"], res["target_ar"])
    assert buf.getvalue() == GOLD["printed"]


def test_save_json_round_trips(tmp_path):
    res = synthetic_results(em)["speculative"]
    p = tmp_path / "r.json"
    with contextlib.redirect_stdout(io.StringIO()):
        res.save_json(str(p))
    assert json.loads(p.read_text()) == GOLD["to_dict"]["speculative"]


def test_empty_results_are_zero_not_errors():
    r = em.BenchmarkResults(method="speculative")
    d = r.to_dict()
    assert d["overall_throughput"] == 0.0 and d["avg_ttft"] == 0.0 and d["avg_acceptance_rate"] == 0.0
    b = em.BatchMetrics()
    assert b.avg_ttft == 0.0 and b.avg_latency == 0.0 and b.throughput == 0.0


@pytest.mark.parametrize("case", sorted(GOLD["batch_autoregressive_generate"]))
def test_target_only_baseline_matches_reference(case):
    c = GOLD["batch_autoregressive_generate"][case]
    target, _ = make_pair(c["vocab"], dtype=DT[c["dtype"]], pos_mult=3)
    assert bank_digest(target) == c["target_digest"]
    tl = TupleFakeLM(target.bank, pos_mult=3, no_cache=c["cache"] == "none")
    ids = torch.tensor(c["prompt"])
    ctx = SimpleNamespace(target=tl, gen_len=c["gen_len"], end_tokens=c["end_tokens"],
                          processor=SimpleNamespace(temperature=c["temperature"]))
    torch.manual_seed(c["seed"])
    outs = ie.batch_autoregressive_generate(ctx, ids, torch.ones_like(ids), c["batch"])
    if c["raised"] is None:
        assert [o.tolist() for o in outs] == c["outputs"]
    else:
        # documented divergence: the reference's per-row cache scatter cannot hold a growing cache
        # (engine/infer_engine.py:466 raises); the drop-in hands the model its own cache back
        assert len(outs) == c["batch"] and all(len(o) > ids.shape[1] for o in outs)


class _Tok:
    """Whitespace tokenizer with the call surface decode_batch_with_chat_template uses."""

    def __call__(self, prompts, return_tensors="pt", padding=True, truncation=True, max_length=64):
        rows = [[3 + (hash(w) % 1000) for w in p.split()][:max_length] for p in prompts]
        L = max(len(r) for r in rows)
        ids = torch.zeros(len(rows), L, dtype=torch.long)
        mask = torch.zeros(len(rows), L, dtype=torch.long)
        for i, r in enumerate(rows):
            ids[i, L - len(r):] = torch.tensor(r)
            mask[i, L - len(r):] = 1
        return SimpleNamespace(input_ids=ids, attention_mask=mask)


def test_infer_batch_target_gen_returns_target_metrics():
    target, _ = make_pair(2048, dtype=torch.float32, pos_mult=3)
    ctx = SimpleNamespace(tokenizer=_Tok(), chat=False, max_batch_length=32, spec=False, target_gen=True,
                          reset_in_between=False, ngram=None, target=TupleFakeLM(target.bank, pos_mult=3),
                          gen_len=8, end_tokens=[1], processor=SimpleNamespace(temperature=0.0))
    spec_m, tgt_m = ie.infer_batch(ctx, ["a b c", "d e f g h"])
    assert spec_m is None and isinstance(tgt_m, em.BatchMetrics)
    assert tgt_m.batch_size == 2 and len(tgt_m.requests) == 2
    for r in tgt_m.requests:
        assert r.total_tokens == r.prompt_tokens + r.generated_tokens and r.generated_tokens > 0
    d = em.BenchmarkResults(method="target_ar", batches=[tgt_m]).to_dict()
    assert d["batches"][0]["requests"][0]["prompt_tokens"] == 3


def test_run_batch_speculative_metrics_rules(monkeypatch):
    """The request fields (engine/infer_engine.py:117-140) from stubbed decode results."""
    outs = [torch.arange(12), torch.arange(9)]

    def fake_generate(ctx, input_ids, attention_mask, batch_size, first_token_callback=None):
        first_token_callback(0)
        return outs, [0.5, 0.0]

    monkeypatch.setattr(ie, "batch_speculative_generate", fake_generate)
    mask = torch.tensor([[1, 1, 1, 1], [0, 0, 1, 1]])
    bm = ie.run_batch_speculative(SimpleNamespace(), torch.zeros(2, 4, dtype=torch.long), mask, 2)
    assert [r.prompt_tokens for r in bm.requests] == [4, 2]
    assert [r.generated_tokens for r in bm.requests] == [8, 7]
    assert [r.total_tokens for r in bm.requests] == [12, 9]
    assert [r.acceptance_rate for r in bm.requests] == [0.5, 0.0]
    assert bm.requests[0].first_token_time > 0 and bm.requests[1].first_token_time == 0.0
    res = em.BenchmarkResults(method="speculative", batches=[bm])
    assert res.avg_acceptance_rate == 0.5   # zero-rate rows are skipped (metrics.py:123-129)
    assert res.to_dict()["total_prompt_tokens"] == 6


def test_run_batch_speculative_returns_none_on_failure(monkeypatch):
    def boom(*a, **k):
        raise RuntimeError("x")
    monkeypatch.setattr(ie, "batch_speculative_generate", boom)
    with contextlib.redirect_stdout(io.StringIO()):
        assert ie.run_batch_speculative(SimpleNamespace(), torch.zeros(1, 2, dtype=torch.long),
                                        torch.ones(1, 2, dtype=torch.long), 1) is None


def _dyn_cache(layers=3, length=10):
    from transformers.cache_utils import DynamicCache
    c = DynamicCache()
    g = torch.Generator().manual_seed(0)
    kv = []
    for layer in range(layers):
        k, v = torch.randn(1, 2, length, 4, generator=g), torch.randn(1, 2, length, 4, generator=g)
        c.update(k, v, layer)
        kv.append((k, v))
    return c, tuple(kv)


def test_prune_dynamic_cache_matches_tuple_golden():
    with open(os.path.join(HERE, "golden", "caching.json")) as f:
        shapes = json.load(f)
    for k, want in shapes.items():
        c, kv = _dyn_cache()
        out = caching.prune_cache(c, int(k))
        assert out is c                                          # mutated in place (utils/caching.py:67)
        assert c.get_seq_length() == want[0][2]
        tup = caching.prune_cache(kv, int(k))                    # the tuple path, views
        assert [list(t.shape) for t in tup[0]] == want
        for layer in range(len(kv)):
            assert torch.equal(c.layers[layer].keys, tup[layer][0])
            assert torch.equal(c.layers[layer].values, tup[layer][1])


def test_prune_cache_rejects_unknown_and_passes_none():
    assert caching.prune_cache(None, 2) is None
    with pytest.raises(ValueError, match="Unsupported cache type"):
        caching.prune_cache([1, 2], 1)
