"""Generate the golden vectors that pin the oracle to the reference.

Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

It imports the REFERENCE itself (read-only, CPU, torch 2.10.0) with a stub for the
missing ``termcolor`` package, drives its hot-path entry points with the FakeLM
banks of tests/fakelm.py under fixed ``torch.manual_seed`` seeds, and writes:

* ``spec_loops.json``   — ``sampling.speculative_generate`` outputs (batch-1 rule A8)
* ``engine_loops.json`` — ``engine.infer_engine.batch_speculative_generate`` outputs (rule A10)
* ``processors.safetensors`` — ``utils.logits_processor`` probabilities on small rows
* ``caching.json``      — ``utils.caching.prune_tuple_cache`` shapes
* ``ngram_loops.json``  — ``ngram_assisted.ngram_assisted_speculative_generate`` outputs (rule A11)
* ``engine_surface.json`` — ``engine.metrics`` (``BenchmarkResults.to_dict`` and the printed
  summaries of a fixed synthetic result set), ``engine.infer_engine.run_batch_speculative``'s
  non-timing request fields and ``batch_autoregressive_generate`` outputs on FakeLM banks

``python tests/golden/make_golden.py --only surface`` regenerates just the last file.

Only data is committed (inputs are regenerated from seeds + checked by digest);
no reference source travels.  The GPU box never runs this script.
"""
from __future__ import annotations

import json
import os
import sys
import types
from types import SimpleNamespace

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.dirname(HERE))           # tests/ (fakelm)
from fakelm import make_pair, bank_digest, likely_tokens   # noqa: E402

SPEC_CASES = [
    # name, V, dtype, gamma, processor(kind, T, k, p), gen_len, eos, skip_adj, seeds
    ("greedy_g4_bf16", 4096, "bf16", 4, ("greedy", 1.0, 0, 1.0), 40, [1], False, [0, 1]),
    ("greedy_g1_bf16", 4096, "bf16", 1, ("greedy", 1.0, 0, 1.0), 24, [1], False, [0]),
    ("greedy_g8_bf16", 4096, "bf16", 8, ("greedy", 1.0, 0, 1.0), 40, [1], False, [0]),
    ("multi_t1_g4_bf16", 4096, "bf16", 4, ("multinomial", 1.0, 0, 1.0), 40, [1], False, [0, 1, 2]),
    ("multi_t07_g4_bf16", 4096, "bf16", 4, ("multinomial", 0.7, 0, 1.0), 40, [1], False, [0, 1]),
    ("multi_t1_g8_bf16", 4096, "bf16", 8, ("multinomial", 1.0, 0, 1.0), 40, [1], False, [3]),
    ("multi_t1_g4_bf16_skipadj", 4096, "bf16", 4, ("multinomial", 1.0, 0, 1.0), 40, [1], True, [0]),
    ("multi_t1_g4_bf16_eos", 4096, "bf16", 4, ("multinomial", 1.0, 0, 1.0), 60, "likely", False,
     [0, 1, 2, 3]),
    ("greedy_g4_bf16_eos", 4096, "bf16", 4, ("greedy", 1.0, 0, 1.0), 60, "likely", False, [0, 1]),
    ("topk20_g4_bf16", 4096, "bf16", 4, ("topk", 1.0, 20, 1.0), 40, [1], False, [0, 1]),
    ("topk50_t08_g4_bf16", 4096, "bf16", 4, ("topk", 0.8, 50, 1.0), 40, [1], False, [0]),
    ("nucleus09_g4_bf16", 4096, "bf16", 4, ("nucleus", 1.0, 0, 0.9), 40, [1], False, [0, 1]),
    ("nucleus08_t07_g4_bf16", 4096, "bf16", 4, ("nucleus", 0.7, 0, 0.8), 40, [1], False, [0]),
    ("topknucleus_g4_bf16", 4096, "bf16", 4, ("topknucleus", 1.0, 50, 0.9), 40, [1], False, [0]),
    ("greedy_g4_fp32", 4096, "fp32", 4, ("greedy", 1.0, 0, 1.0), 40, [1], False, [0]),
    ("multi_t1_g4_fp32", 4096, "fp32", 4, ("multinomial", 1.0, 0, 1.0), 40, [1], False, [0, 1]),
    ("nucleus09_g4_fp32", 4096, "fp32", 4, ("nucleus", 1.0, 0, 0.9), 32, [1], False, [0]),
    ("gpt2like_greedy_g4_fp32", 50257, "fp32", 4, ("greedy", 1.0, 0, 1.0), 32, [50256], False, [0]),
    ("llama_greedy_g4_bf16", 128256, "bf16", 4, ("greedy", 1.0, 0, 1.0), 24, [128001, 128009], False, [0]),
    ("llama_multi_g4_bf16", 128256, "bf16", 4, ("multinomial", 1.0, 0, 1.0), 24, [128001, 128009], False, [0]),
    # γ beyond 16 (SD_MAX_GAMMA = 32): the reference takes any γ (sampling/speculative_decoding.py:106)
    ("multi_t1_g20_bf16", 4096, "bf16", 20, ("multinomial", 1.0, 0, 1.0), 64, [1], False, [0, 1]),
    ("greedy_g32_bf16", 4096, "bf16", 32, ("greedy", 1.0, 0, 1.0), 80, [1], False, [0]),
    ("nucleus09_g20_bf16", 4096, "bf16", 20, ("nucleus", 1.0, 0, 0.9), 48, [1], False, [0]),
    # drafter = target + N(0, 0.05^2): drafts are accepted deep into the γ = 24 window
    ("multi_t1_g24_bf16_close", 4096, "bf16", 24, ("multinomial", 1.0, 0, 1.0), 96, [1], False, [0, 1], 0.05),
    ("greedy_g32_bf16_close", 4096, "bf16", 32, ("greedy", 1.0, 0, 1.0), 96, [1], False, [0], 0.05),
    # γ beyond SD_MAX_GAMMA = 32: specdec_amd.ops verifies the window in chunks of <= 32 drafts
    ("multi_t1_g48_bf16_close", 4096, "bf16", 48, ("multinomial", 1.0, 0, 1.0), 160, [1], False, [0, 1, 2], 0.05),
    ("greedy_g40_bf16_close", 4096, "bf16", 40, ("greedy", 1.0, 0, 1.0), 120, [1], False, [0], 0.05),
    ("nucleus09_g40_bf16_close", 4096, "bf16", 40, ("nucleus", 1.0, 0, 0.9), 120, [1], False, [0], 0.05),
    ("multi_t1_g48_bf16_close_eos", 4096, "bf16", 48, ("multinomial", 1.0, 0, 1.0), 200, "likely", False,
     [0, 1], 0.05),
    ("multi_t1_g40_bf16", 4096, "bf16", 40, ("multinomial", 1.0, 0, 1.0), 100, [1], False, [0]),
    # user processors overriding only _process (tests/custom_procs.py, on the reference's classes)
    ("custom_penalty_g4_bf16", 4096, "bf16", 4, ("custom:penalty", 1.0, 0, 1.0), 40, [1], False, [0, 1]),
    ("custom_banned_topk_t08_g4_bf16", 4096, "bf16", 4, ("custom:banned_topk", 0.8, 50, 1.0), 40, [1], False, [0]),
    ("custom_sharpen_greedy_g4_bf16", 4096, "bf16", 4, ("custom:sharpen_greedy", 1.0, 0, 1.0), 40, [1], False, [0]),
    ("custom_penalty_g4_fp32", 4096, "fp32", 4, ("custom:penalty", 0.7, 0, 1.0), 40, [1], False, [0]),
]

# The engine re-feeds the last prompt token to the drafter after its prefill (engine/infer_engine.py:206,231),
# so drafter and target see it at different positions; pos_mult=0 banks (logits depend on the token only)
# keep their distributions aligned so the accept branch is exercised.
ENGINE_CASES = [
    # name, V, dtype, B, gamma, gen_len, end_tokens, seeds[, pos_mult[, sigma]]
    ("b1_g4_bf16_pos7", 4096, "bf16", 1, 4, 32, [1], [0], 7),
    ("b1_g4_bf16", 4096, "bf16", 1, 4, 32, [1], [0, 1]),
    ("b1_g4_fp32", 4096, "fp32", 1, 4, 32, [1], [0]),
    ("b4_g4_fp32", 4096, "fp32", 4, 4, 32, [1], [0, 1]),
    ("b6_g4_fp32_eos", 2048, "fp32", 6, 4, 40, "likely", [0, 1]),
    ("b6_g1_fp32", 2048, "fp32", 6, 1, 16, [1], [0]),
    ("b5_g3_fp32_ragged", 2048, "fp32", 5, 3, 17, "likely", [2]),
    ("b1_g4_bf16_eos", 4096, "bf16", 1, 4, 40, "likely", [0, 1, 2]),
    ("b4_g4_bf16_refcrash", 4096, "bf16", 4, 4, 16, [1], [0]),
    ("llama_b2_g4_fp32", 128256, "fp32", 2, 4, 12, [128001, 128009], [0]),
    ("b4_g20_fp32", 2048, "fp32", 4, 20, 48, [1], [0]),
    ("b3_g32_fp32_eos", 2048, "fp32", 3, 32, 70, "likely", [1]),
    # γ beyond SD_MAX_GAMMA = 32 (chunked windows); drafter = target + N(0, 0.05^2): accepts reach chunk 2
    ("b3_g48_fp32_close", 2048, "fp32", 3, 48, 120, [1], [0, 1], 0, 0.05),
    ("b1_g48_bf16_close", 4096, "bf16", 1, 48, 120, [1], [0], 0, 0.05),
    ("b4_g40_fp32_close_eos", 2048, "fp32", 4, 40, 120, "likely", [1, 2], 0, 0.05),
    ("b2_g40_fp32", 2048, "fp32", 2, 40, 80, [1], [0]),
]

# ngram-assisted loop (rule A11): FakeLM target, the reference's n-gram storages as the drafter
NGRAM_PEAK = 20.0
NGRAM_CASES = [
    # name, V, dtype, storage(kind, n), gamma, processor, filler_top_k, stop_if_unknown, gen_len, eos, seeds
    ("ng_greedy_g4_n3", 4096, "bf16", ("multi", 3), 4, ("greedy", 1.0, 0, 1.0), 3, False, 48, [1], [0, 1]),
    ("ng_greedy_g8_n4_f1", 4096, "bf16", ("multi", 4), 8, ("greedy", 1.0, 0, 1.0), 1, False, 48, [1], [0]),
    ("ng_greedy_g4_one3_unknown", 4096, "bf16", ("one", 3), 4, ("greedy", 1.0, 0, 1.0), 3, True, 40, [1], [0, 1]),
    ("ng_multi_g4_n3", 4096, "bf16", ("multi", 3), 4, ("multinomial", 1.0, 0, 1.0), 3, False, 40, [1], [0, 1, 2]),
    ("ng_multi_t07_g8_n3", 4096, "bf16", ("multi", 3), 8, ("multinomial", 0.7, 0, 1.0), 3, False, 40, [1], [0]),
    ("ng_nucleus09_g8_n3", 4096, "bf16", ("multi", 3), 8, ("nucleus", 1.0, 0, 0.9), 3, False, 40, [1], [0, 1]),
    ("ng_topk20_g4_one3", 4096, "bf16", ("one", 3), 4, ("topk", 1.0, 20, 1.0), 3, False, 40, [1], [0]),
    ("ng_greedy_g4_n3_eos", 4096, "bf16", ("multi", 3), 4, ("greedy", 1.0, 0, 1.0), 3, False, 60, "likely", [0, 1]),
    ("ng_multi_g4_n3_fp32", 4096, "fp32", ("multi", 3), 4, ("multinomial", 1.0, 0, 1.0), 3, False, 40, [1], [0]),
    ("ng_llama_nucleus_g8", 128256, "bf16", ("multi", 3), 8, ("nucleus", 1.0, 0, 0.9), 3, False, 24,
     [128001, 128009], [0, 1, 2]),
    ("ng_multi_g20_n3", 4096, "bf16", ("multi", 3), 20, ("multinomial", 1.0, 0, 1.0), 3, False, 60, [1], [0]),
    # filler top-k beyond 8 (SD_NGRAM_MAX_FILLER = 64) and γ' beyond SD_MAX_GAMMA (chunked windows)
    ("ng_multi_g4_n3_f16", 4096, "bf16", ("multi", 3), 4, ("multinomial", 1.0, 0, 1.0), 16, False, 40, [1], [0, 1]),
    ("ng_greedy_g8_n3_f40", 4096, "bf16", ("multi", 3), 8, ("greedy", 1.0, 0, 1.0), 40, False, 40, [1], [0]),
    ("ng_greedy_g40_n3", 4096, "bf16", ("multi", 3), 40, ("greedy", 1.0, 0, 1.0), 3, False, 160, [1], [0, 1]),
    ("ng_multi_g48_n3_f16", 4096, "bf16", ("multi", 3), 48, ("multinomial", 1.0, 0, 1.0), 16, False, 160, [1],
     [0, 1]),
    ("ng_custom_penalty_g4_n3", 4096, "bf16", ("multi", 3), 4, ("custom:penalty", 1.0, 0, 1.0), 3, False, 40, [1],
     [0, 1]),
    # filler top-k beyond one 64-id pass (sd_ngram_verify runs a pass per 64 ids)
    ("ng_multi_g4_n3_f128", 4096, "bf16", ("multi", 3), 4, ("multinomial", 1.0, 0, 1.0), 128, False, 40, [1], [0, 1]),
    ("ng_greedy_g8_n3_f200", 4096, "bf16", ("multi", 3), 8, ("greedy", 1.0, 0, 1.0), 200, False, 40, [1], [0]),
]

DT = {"bf16": torch.bfloat16, "fp32": torch.float32}


def _import_reference():
    sys.modules.setdefault("termcolor", types.SimpleNamespace(colored=lambda s, *a, **k: s, cprint=print))
    sys.path.insert(0, REF)
    from sampling.speculative_decoding import speculative_generate      # noqa
    from utils import logits_processor as lp                             # noqa
    from utils.caching import prune_tuple_cache                          # noqa
    from engine.infer_engine import batch_speculative_generate           # noqa
    return speculative_generate, lp, prune_tuple_cache, batch_speculative_generate


def _import_reference_ngram():
    _import_reference()
    import ngram_assisted as ng                                          # noqa
    return ng


def prompt_for(V: int, seed: int, length: int = 8, batch: int = 1):
    g = torch.Generator().manual_seed(10_000 + seed)
    return torch.randint(3, V, (batch, length), generator=g)


def make_processor(lp, kind, T, k, p):
    if kind.startswith("custom:"):   # a user subclass overriding _process (tests/custom_procs.py)
        from custom_procs import make_custom
        return make_custom(lp, kind.split(":", 1)[1], T, k, p)
    return {"greedy": lambda: lp.GreedyProcessor(T),
            "multinomial": lambda: lp.MultinomialProcessor(T),
            "topk": lambda: lp.TopKProcessor(T, k),
            "nucleus": lambda: lp.NucleusProcessor(T, p),
            "topknucleus": lambda: lp.TopKNucleusProcessor(T, k, p)}[kind]()


def _merge(path, new, only):
    """--cases: the listed cases' records replace / join the file's, every other record is kept."""
    if only is None:
        return new
    with open(path) as f:
        old = json.load(f)
    old.update(new)
    return old


def main(only=None):
    """only: a set of case names (SPEC / ENGINE / NGRAM) to (re)generate into the existing files;
    None regenerates everything."""
    speculative_generate, lp, prune_tuple_cache, batch_speculative_generate = _import_reference()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    keep = (lambda name: True) if only is None else (lambda name: name in only)

    spec = {}
    for name, V, dt, gamma, (kind, T, k, p), gen_len, eos, skip, seeds, *sg in SPEC_CASES:
        if not keep(name):
            continue
        sigma = sg[0] if sg else 1.0
        target, drafter = make_pair(V, dtype=DT[dt], sigma=sigma)
        if eos == "likely":
            eos = likely_tokens(target)
        for seed in seeds:
            prompt = prompt_for(V, seed)[0].tolist()
            torch.manual_seed(seed)
            out, rate = speculative_generate(
                prompt, drafter, target, gamma=gamma, logits_processor=make_processor(lp, kind, T, k, p),
                max_gen_len=gen_len, eos_tokens_id=eos if len(eos) > 1 else eos[0], pad_token_id=0,
                skip_sample_adjustment=skip)
            spec[f"{name}/s{seed}"] = dict(
                vocab=V, dtype=dt, gamma=gamma, processor=dict(kind=kind, temperature=T, top_k=k, top_p=p),
                max_gen_len=gen_len, eos=eos, skip_sample_adjustment=skip, seed=seed, prompt=prompt, sigma=sigma,
                target_digest=bank_digest(target), drafter_digest=bank_digest(drafter),
                tokens=out, acceptance_rate=float(rate))
            print(name, seed, len(out), rate, flush=True)
    spec = _merge(os.path.join(HERE, "spec_loops.json"), spec, only)
    with open(os.path.join(HERE, "spec_loops.json"), "w") as f:
        json.dump(spec, f, indent=1)

    eng = {}
    for name, V, dt, B, gamma, gen_len, ends, seeds, *pm in ENGINE_CASES:
        if not keep(name):
            continue
        pos_mult = pm[0] if pm else 0
        sigma = pm[1] if len(pm) > 1 else 1.0
        target, drafter = make_pair(V, dtype=DT[dt], pos_mult=pos_mult, sigma=sigma)
        if ends == "likely":
            ends = likely_tokens(target)
        for seed in seeds:
            ids = prompt_for(V, seed, batch=B)
            mask = torch.ones_like(ids)
            ctx = SimpleNamespace(drafter=drafter, target=target, gamma=gamma, gen_len=gen_len,
                                  end_tokens=ends, target_device="cpu")
            torch.manual_seed(seed)
            rec = dict(vocab=V, dtype=dt, batch=B, gamma=gamma, gen_len=gen_len, end_tokens=ends, seed=seed,
                       pos_mult=pos_mult, sigma=sigma,
                       prompt=ids.tolist(), target_digest=bank_digest(target),
                       drafter_digest=bank_digest(drafter))
            try:
                outs, rates = batch_speculative_generate(ctx, ids, mask, B)
                rec.update(outputs=[o.tolist() for o in outs], rates=[float(r) for r in rates], raised=None)
            except Exception as e:  # the reference's bf16 B>=2 index_put crash (engine/infer_engine.py:254)
                rec.update(outputs=None, rates=None, raised=f"{type(e).__name__}: {e}")
            eng[f"{name}/s{seed}"] = rec
            print(name, seed, rec["raised"] or [len(o) for o in rec["outputs"]], flush=True)
    eng = _merge(os.path.join(HERE, "engine_loops.json"), eng, only)
    with open(os.path.join(HERE, "engine_loops.json"), "w") as f:
        json.dump(eng, f, indent=1)

    ng = _import_reference_ngram()
    ngl = {}
    for name, V, dt, (skind, sn), gamma, (kind, T, k, p), filler, unknown, gen_len, eos, seeds in NGRAM_CASES:
        if not keep(name):
            continue
        # next-token logits depend on the last token only, peaked so sampled continuations repeat
        target, _ = make_pair(V, dtype=DT[dt], pos_mult=0, peak=NGRAM_PEAK)
        if eos == "likely":
            eos = likely_tokens(target)
        for seed in seeds:
            prompt = prompt_for(V, seed, length=12)[0].tolist()
            prompt = prompt + prompt[:6]   # a repeat so the storage starts with known grams
            store = (ng.NGramStorage if skind == "multi" else ng.OneLevelNGramStorage)(sn, V)
            torch.manual_seed(seed)
            out, rate = ng.ngram_assisted_speculative_generate(
                prompt, store, target, gamma=gamma, filler_top_k=filler,
                logits_processor=make_processor(lp, kind, T, k, p), max_gen_len=gen_len,
                eos_tokens_id=eos if len(eos) > 1 else eos[0], pad_token_id=0, stop_if_unknown=unknown)
            ngl[f"{name}/s{seed}"] = dict(
                vocab=V, dtype=dt, storage=skind, n=sn, gamma=gamma, pos_mult=0, peak=NGRAM_PEAK,
                processor=dict(kind=kind, temperature=T, top_k=k, top_p=p), filler_top_k=filler,
                stop_if_unknown=unknown, max_gen_len=gen_len, eos=eos, seed=seed, prompt=prompt,
                target_digest=bank_digest(target), tokens=out, acceptance_rate=float(rate))
            print(name, seed, len(out), rate, flush=True)
    ngl = _merge(os.path.join(HERE, "ngram_loops.json"), ngl, only)
    with open(os.path.join(HERE, "ngram_loops.json"), "w") as f:
        json.dump(ngl, f, indent=1)
    if only is not None:
        return

    # processors on small rows
    from safetensors.torch import save_file
    tens = {}
    meta = {}
    g = torch.Generator().manual_seed(7)
    base = torch.randn(3, 1024, generator=g) * 3
    configs = [("greedy", 1.0, 0, 1.0), ("multinomial", 0.7, 0, 1.0), ("topk", 1.0, 20, 1.0),
               ("topk", 0.8, 50, 1.0), ("nucleus", 1.0, 0, 0.9), ("nucleus", 0.7, 0, 0.5),
               ("topknucleus", 1.0, 50, 0.9), ("topknucleus", 1.3, 10, 0.95)]
    for dt in ("bf16", "fp32"):
        x = base.to(DT[dt])
        tens[f"logits_{dt}"] = x.contiguous()
        for i, (kind, T, k, p) in enumerate(configs):
            proc = make_processor(lp, kind, T, k, p)
            tens[f"probs_{dt}_{i}"] = proc(x.clone()).contiguous()
            meta[f"{dt}_{i}"] = f"{kind},{T},{k},{p}"
    save_file(tens, os.path.join(HERE, "processors.safetensors"), metadata=meta)

    # prune_tuple_cache shapes
    cache = tuple((torch.zeros(1, 2, 10, 4), torch.zeros(1, 2, 10, 4)) for _ in range(3))
    shapes = {str(k): [list(t.shape) for t in prune_tuple_cache(cache, k)[0]] for k in (1, 3, 5)}
    with open(os.path.join(HERE, "caching.json"), "w") as f:
        json.dump(shapes, f, indent=1)


SURFACE_ENGINE_CASES = [
    # name, V, dtype, B, gamma, gen_len, end_tokens, seed, pos_mult
    ("rbs_b4_g4_fp32", 4096, "fp32", 4, 4, 24, [1], 0, 0),
    ("rbs_b6_g4_fp32_eos", 2048, "fp32", 6, 4, 40, "likely", 1, 0),
]
SURFACE_AR_CASES = [
    # name, V, dtype, B, gen_len, end_tokens, temperature, seed, cache ("none": the model returns no
    # cache; "tuple": a growing tuple cache, which the reference's scatter cannot hold -> it raises)
    ("ar_b3_greedy_fp32", 2048, "fp32", 3, 16, "likely", 0.0, 0, "none"),
    ("ar_b4_multi_t07_fp32", 2048, "fp32", 4, 16, "likely", 0.7, 1, "none"),
    ("ar_b2_greedy_bf16", 4096, "bf16", 2, 12, [1], 0.0, 2, "none"),
    ("ar_b3_greedy_fp32_tuplecache", 2048, "fp32", 3, 8, [1], 0.0, 0, "tuple"),
]


def synthetic_results(metrics_mod):
    """A fixed BenchmarkResults (two batches, one zero-rate request) built with `metrics_mod`'s
    classes; the test builds the same object with the drop-in's classes."""
    R, Bm, Res = metrics_mod.RequestMetrics, metrics_mod.BatchMetrics, metrics_mod.BenchmarkResults
    out = {}
    for method, scale in (("speculative", 1.0), ("target_ar", 1.7)):
        res = Res(method=method, total_requests=5, total_batches=2, start_time=100.0, end_time=100.0 + 3.5 * scale)
        for bi, sizes in enumerate(((11, 7, 13), (5, 9))):
            b = Bm(batch_size=len(sizes), batch_start_time=100.0 + bi, batch_end_time=100.0 + bi + 1.25 * scale)
            for ri, pt in enumerate(sizes):
                r = R(prompt_tokens=pt, generated_tokens=3 * pt + ri, total_tokens=4 * pt + ri,
                      ttft=0.01 * (ri + 1) * scale, total_latency=0.5 + 0.1 * ri * scale,
                      acceptance_rate=0.0 if (bi, ri) == (0, 1) else 0.25 + 0.1 * ri + 0.05 * bi,
                      drafts_generated=8 * pt, drafts_accepted=3 * pt)
                b.requests.append(r)
            res.batches.append(b)
        out[method] = res
    return out


def make_surface():
    """engine_surface.json: the benchmark-facing surface of the engine (metrics + run_batch_* +
    the target-only baseline), from the reference itself."""
    import contextlib
    import io
    _import_reference()
    import engine.infer_engine as ie                                    # noqa
    import engine.metrics as em                                         # noqa
    from fakelm import TupleFakeLM
    res = synthetic_results(em)
    rec = {"to_dict": {k: v.to_dict() for k, v in res.items()}}
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        em.print_benchmark_summary(res["speculative"])
        em.print_benchmark_summary(res["target_ar"])
        em.print_comparison(res["speculative"], res["target_ar"])
    rec["printed"] = buf.getvalue()

    rbs = {}
    for name, V, dt, B, gamma, gen_len, ends, seed, pos_mult in SURFACE_ENGINE_CASES:
        target, drafter = make_pair(V, dtype=DT[dt], pos_mult=pos_mult)
        if ends == "likely":
            ends = likely_tokens(target)
        ids = prompt_for(V, seed, batch=B)
        mask = torch.ones_like(ids)
        mask[0, :2] = 0      # a padded row: generated_tokens counts padding (:124-126)
        ctx = SimpleNamespace(drafter=drafter, target=target, gamma=gamma, gen_len=gen_len, end_tokens=ends,
                              target_device="cpu")
        torch.manual_seed(seed)
        bm = ie.run_batch_speculative(ctx, ids, mask, B)
        rbs[name] = dict(vocab=V, dtype=dt, batch=B, gamma=gamma, gen_len=gen_len, end_tokens=ends, seed=seed,
                         pos_mult=pos_mult, prompt=ids.tolist(), mask=mask.tolist(),
                         target_digest=bank_digest(target), drafter_digest=bank_digest(drafter),
                         requests=[dict(prompt_tokens=int(r.prompt_tokens), generated_tokens=int(r.generated_tokens),
                                        total_tokens=int(r.total_tokens), acceptance_rate=float(r.acceptance_rate))
                                   for r in bm.requests])
        print(name, [r["generated_tokens"] for r in rbs[name]["requests"]], flush=True)
    rec["run_batch_speculative"] = rbs

    ar = {}
    for name, V, dt, B, gen_len, ends, T, seed, cache in SURFACE_AR_CASES:
        target, _ = make_pair(V, dtype=DT[dt], pos_mult=3)
        if ends == "likely":
            ends = likely_tokens(target)
        tl = TupleFakeLM(target.bank, pos_mult=3, no_cache=cache == "none")
        ids = prompt_for(V, seed, batch=B)
        mask = torch.ones_like(ids)
        ctx = SimpleNamespace(target=tl, gen_len=gen_len, end_tokens=ends, processor=SimpleNamespace(temperature=T))
        torch.manual_seed(seed)
        rec_ar = dict(vocab=V, dtype=dt, batch=B, gen_len=gen_len, end_tokens=ends, temperature=T, seed=seed,
                      cache=cache, prompt=ids.tolist(), target_digest=bank_digest(target))
        try:
            outs = ie.batch_autoregressive_generate(ctx, ids, mask, B)
            rec_ar.update(outputs=[o.tolist() for o in outs], raised=None)
        except Exception as e:
            rec_ar.update(outputs=None, raised=f"{type(e).__name__}: {e}")
        ar[name] = rec_ar
        print(name, rec_ar["raised"] or [len(o) for o in rec_ar["outputs"]], flush=True)
    rec["batch_autoregressive_generate"] = ar
    with open(os.path.join(HERE, "engine_surface.json"), "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "surface":
        make_surface()
    elif "--cases" in sys.argv:   # e.g. --cases multi_t1_g20_bf16,b4_g20_fp32: merged into the files
        main(set(sys.argv[sys.argv.index("--cases") + 1].split(",")))
    else:
        main()
        make_surface()
