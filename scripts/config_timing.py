"""Per-configuration step latency of the sampling path (GPU box; BASELINE.json configs beyond bench.py's).

bench.py measures configs[2] (engine rule, 32 rows).  This script times the other verify-path
configurations on synthetic Llama-3 shaped logits resident in HBM, each step captured in a
hipGraph and replayed (PhiloxNoise), next to the oracle (torch-CPU, reference semantics) on the
same step:

  cfg1_*    configs[1]: batch 1, γ=4, rule A8 — γ drafter draws (sd_sample) + sd_verify over
            γ+1 target rows and γ drafter rows; greedy, multinomial T=1, nucleus top-p 0.9.
  cfg4_*    configs[4]: n-gram drafter, γ=8, top-p 0.9, filler top-3 — sd_ngram_verify over 9
            target rows (A11).
  sweep_b*  the SURVEY §8(d) roofline sweep: the engine step (γ draws + verify) at 128 / 512 rows.

Prints one JSON object per case (µs per step, algorithmic bytes per step, achieved GB/s, and the
oracle's ms per step on the host cores).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import torch  # noqa: E402

from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

V = 128256
dev = torch.device("cuda", 0)
STOPS = torch.tensor([128001, 128009], dtype=torch.long, device=dev)
CPU_THREADS = min(len(os.sched_getaffinity(0)), 16)


def logits(B, rows, seed, sigma=None, base=None):
    g = torch.Generator(device=dev).manual_seed(seed)
    if base is None:
        return (torch.randn(B, rows, V, generator=g, device=dev) * 3.0).to(torch.bfloat16)
    return (base[:, :rows].float() + sigma * torch.randn(B, rows, V, generator=g, device=dev)).to(torch.bfloat16)


def graph_time(step, steps=200, per_graph=20):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(per_graph):
            step()
    gr.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // per_graph):
        gr.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


def cpu_time(fn, seconds=3.0):
    if os.environ.get("CFG_NO_CPU"):   # GPU-only A/B runs
        return None
    torch.set_num_threads(CPU_THREADS)
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        if time.perf_counter() - t0 > seconds:
            break
    return (time.perf_counter() - t0) / n * 1e3


def report(name, us, alg_bytes, cpu_ms, extra=None):
    rec = {"case": name, "us_per_step": us, "alg_bytes_per_step": alg_bytes,
           "achieved_gbs": alg_bytes / (us * 1e-6) / 1e9, "frac_of_8tbs": alg_bytes / (us * 1e-6) / 8e12,
           "cpu_oracle_ms_per_step": cpu_ms, "cpu_threads": CPU_THREADS}
    rec.update(extra or {})
    print(json.dumps(rec), flush=True)


def cfg1(kind, top_p=1.0):
    from oracle import specdec_ref as ref
    g = 4
    proc = ops.ProcSpec(kind, 1.0, 0, top_p)
    tl = logits(1, g + 1, 11)
    dl = logits(1, g, 12, 1.0, tl)
    noise = PhiloxNoise(seed=7)
    draft = torch.zeros(1, g, dtype=torch.long, device=dev)
    trows = [tl[:, t] for t in range(g + 1)]
    drows = [dl[:, t] for t in range(g)]

    # as the drop-in loop does: the draws hand their rows' stats to the verify, except under a
    # top-k / nucleus processor; CFG_KEEP_STASH=1: those draws return stats and keeps too (the
    # threshold + k_draw path instead of k_draw_nuc), CFG_NO_STASH=1: no stats at all (A/B)
    stash = not os.environ.get("CFG_NO_STASH") and (not proc.keeps or os.environ.get("CFG_KEEP_STASH"))
    dstats = torch.empty(g, 1, 2, dtype=torch.float32, device=dev) if stash else None
    dkeep = torch.empty(g, 1, 4, dtype=torch.int32, device=dev) if stash and proc.keeps else None

    def step():
        for d in range(g):
            ops.sample_rows(drows[d], proc, noise, tokens_out=draft[:, d],
                            row_stats_out=dstats[d] if stash else None,
                            row_keep_out=dkeep[d] if dkeep is not None else None)
        return ops.verify(trows, drows, draft, _lib.SD_RULE_SPEC, proc, proc, noise, STOPS,
                          draft_row_stats=dstats, draft_row_keep=dkeep)

    us = graph_time(step)
    # oracle: drafter process + sample per position, then the A8 verify step (torch-CPU)
    rp = ref.Processor(kind, 1.0, 0, top_p)
    tlc, dlc = tl[0].cpu(), dl[0].cpu()
    nz = ref.TorchNoise(torch.Generator().manual_seed(0))

    def cpu_step():
        q = torch.empty(g, V)
        ids = []
        for d in range(g):
            qd = ref.process(dlc[d:d + 1], rp)
            q[d] = qd[0].float()
            ids.append(int(ref.sample(qd, rp, nz).reshape(-1)[0]))
        r = nz.uniform(g)
        E = nz.exponential((1, V)) if rp.stochastic else None
        ref.spec_verify_step(tlc, q, ids, rp, r, E)

    report(f"cfg1_{kind}{'_p%.1f' % top_p if top_p < 1 else ''}", us, (2 * g + 1) * V * 2, cpu_time(cpu_step),
           {"B": 1, "gamma": g, "rule": "A8"})


def cfg4():
    from oracle import specdec_ref as ref
    g = 8
    proc = ops.ProcSpec("nucleus", 1.0, 0, 0.9)
    tl = logits(1, g + 1, 21)
    draft = tl[0, :g].float().argmax(-1).unsqueeze(0).contiguous()   # drafts the target agrees with
    noise = PhiloxNoise(seed=9)
    trows = [tl[:, t] for t in range(g + 1)]

    def step():
        return ops.ngram_verify(trows, draft, proc, noise, STOPS, filler_k=3)

    us = graph_time(step)
    rp = ref.Processor("nucleus", 1.0, 0, 0.9)
    tlc, ids = tl[0].cpu(), draft[0].tolist()
    nz = ref.TorchNoise(torch.Generator().manual_seed(0))

    def cpu_step():
        ref.ngram_verify_step(tlc, ids, rp, nz)

    report("cfg4_ngram_nucleus_p0.9", us, (g + 1) * V * 2, cpu_time(cpu_step), {"B": 1, "gamma": g, "rule": "A11"})


def sweep(B):
    g = 4
    tl = logits(B, g, 31)
    dl = logits(B, g, 32, 1.0, tl)
    noise = PhiloxNoise(seed=5)
    draft = torch.empty(B, g, dtype=torch.long, device=dev)
    dstats = torch.empty(g, B, 2, dtype=torch.float32, device=dev)
    trows = [tl[:, t] for t in range(g)]
    drows = [dl[:, t] for t in range(g)]

    def step():
        for d in range(g):
            ops.sample_rows(drows[d], ops.PLAIN_SOFTMAX, noise, tokens_out=draft[:, d], row_stats_out=dstats[d])
        return ops.verify(trows, drows, draft, _lib.SD_RULE_ENGINE, ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise,
                          STOPS, draft_row_stats=dstats)

    us = graph_time(step, steps=100, per_graph=10)
    report(f"sweep_engine_b{B}", us, B * 2 * g * V * 2, None, {"B": B, "gamma": g, "rule": "A10"})


if __name__ == "__main__":
    which = sys.argv[1:] or ["cfg1", "cfg4", "sweep"]
    if "cfg1" in which:
        cfg1("greedy")
        cfg1("multinomial")
        cfg1("nucleus", 0.9)
    if "cfg4" in which:
        cfg4()
    if "sweep" in which:
        for B in (128, 512):
            sweep(B)
