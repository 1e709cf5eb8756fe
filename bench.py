#!/usr/bin/env python3
"""bench.py — throughput of the speculative verify/accept hot path on MI355X.

Workload (BASELINE.json configs[2], per GPU): the sampling hot path of one step of the batched
engine (engine/infer_engine.py:238-336, rule A10) over synthetic Llama-3 shaped logits resident
in HBM — target [B, γ, V] and drafter [B, γ, V] bf16, B = 32 rows per GPU, γ = 4, V = 128256.
A "step" is γ drafter draws (softmax + multinomial of each [B, V] drafter row, :241-247, one
sd_sample launch each, which also return the rows' softmax statistics) and one sd_verify call
(softmax statistics of the γ target rows, the fp64 accept test, the (p−q)⁺ residual resample
and the per-row outputs).  Every logit row is read once by the step, plus the two rows the
residual samples from.  Independent prompt batches shard data-parallel (one replica per GPU,
no collective on the data path), so scaling is weak: every rank verifies its own 32 rows.

value = output tokens (accepted drafts + resampled tokens, all ranks) / max-over-ranks wall
time of the K timed steps.  Steps run as hipGraph replays (the step is captured once per
`--graph-steps` steps), noise is in-kernel Philox (perf mode).  Also reported: acceptance
rate, the HBM roofline of the row-statistics kernel (HIP events around it, algorithmic bytes
= every logit row read once), and the CPU baseline = the oracle (reference semantics,
torch-CPU) timed on a bounded sample of the same workload on this host.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "speculative-decoding_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROF_REPEAT = 20       # k_stats launches per HIP-event pair (roofline timing)
METRIC = "output tokens/sec + acceptance rate, Llama-3-8B/1B γ=4 at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32, help="rows per GPU")
    ap.add_argument("--gamma", type=int, default=4)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--sigma", type=float, default=1.0, help="drafter = target + N(0, sigma^2)")
    ap.add_argument("--graph-steps", type=int, default=20)
    ap.add_argument("--prof-steps", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import specdec_amd
    from specdec_amd import _lib, dp, ops
    from specdec_amd.noise import PhiloxNoise

    # weak scaling: the global batch is args.batch rows per rank, split contiguously by row
    # (specdec_amd/dp.py); Philox noise is keyed by the global row id, so the shards draw what
    # one GPU verifying the whole batch would draw for the same rows.  No data-path collective.
    g, V = args.gamma, args.vocab
    row0, row1 = dp.shard_rows(args.batch * world, world, rank)
    B = row1 - row0
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    tl = (torch.randn(B, g, V, generator=gen, device=dev) * 3.0).to(torch.bfloat16)
    dl = (tl.float() + args.sigma * torch.randn(B, g, V, generator=gen, device=dev)).to(torch.bfloat16)
    noise = PhiloxNoise(seed=4242)
    draft = torch.empty(B, g, dtype=torch.long, device=dev)
    dstats = torch.empty(g, B, 2, dtype=torch.float32, device=dev)   # drafter rows' (max, Σexp)
    stops = torch.tensor([128001, 128009], dtype=torch.long, device=dev)
    trows = [tl[:, t, :] for t in range(g)]
    drows = [dl[:, t, :] for t in range(g)]

    def draws():
        # engine/infer_engine.py:241-247: softmax + multinomial of each drafter row, one launch per
        # draft position (in the engine a drafter forward sits between them)
        for d in range(g):
            ops.sample_rows(drows[d], ops.PLAIN_SOFTMAX, noise, tokens_out=draft[:, d], row_base=row0,
                            row_stats_out=dstats[d])

    def verify(prof=None):
        return ops.verify(trows, drows, draft, _lib.SD_RULE_ENGINE, ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise,
                          stops, prof_events=prof, row_base=row0, draft_row_stats=dstats)

    def step(prof=None):
        draws()
        return verify(prof)

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()

    # capture G steps per graph; K must be a multiple of G
    G = max(1, min(args.graph_steps, args.steps))
    while args.steps % G:
        G -= 1
    graph = torch.cuda.CUDAGraph()
    outs = []
    with torch.cuda.graph(graph):
        for _ in range(G):
            outs.append(step())
    graph.replay()   # untimed warm replay
    torch.cuda.synchronize()
    replays = args.steps // G

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(replays):
        graph.replay()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # the verify alone (same captured draws' outputs), for the per-phase breakdown
    vgraph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(vgraph):
        for _ in range(G):
            verify()
    vgraph.replay()
    torch.cuda.synchronize()
    tv = time.perf_counter()
    for _ in range(replays):
        vgraph.replay()
    torch.cuda.synchronize()
    verify_ms = (time.perf_counter() - tv) / args.steps * 1e3

    # output tokens per replay (identical every replay: same inputs, same captured noise offsets)
    acc = sum(int(o.n_accepted.sum()) for o in outs)
    resid = sum(int(((o.row_status & _lib.SD_ROW_RESIDUAL) != 0).sum()) for o in outs)
    tokens = (acc + resid) * replays
    drafted = B * g * G * replays
    elapsed, tot = dp.aggregate(elapsed, {"tokens": tokens, "accepted": acc * replays, "drafted": drafted}, dev, dist)
    tokens, accepted, drafted = tot["tokens"], tot["accepted"], tot["drafted"]

    # dominant kernel: row statistics of the target rows.  HIP events on its stream
    # around PROF_REPEAT back-to-back launches of it (sd_verify's prof_stats_repeat), so the
    # event pair's own cost (~3-6 us, context dependent) is amortised; the per-launch figure
    # still includes the launch-to-launch gaps, i.e. it errs on the slow side of rocprofv3's
    # kernel-trace average (profiles/).
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.prof_steps)]
    for e in ev:
        e[0].record()   # marks the torch events as recorded; sd_verify re-records them around k_stats
        e[1].record()
        verify(prof=(e[0], e[1], PROF_REPEAT))
    torch.cuda.synchronize()
    stats_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev) / PROF_REPEAT
    alg_bytes = B * g * V * 2               # k_stats: the γ target rows, once
    achieved = alg_bytes / (stats_ms * 1e-3) / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    step_bytes = B * 2 * g * V * 2          # the step: every target and drafter row once
    step_gbs = step_bytes / (ms_per_step * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(tl, dl, draft, args)

    if rank == 0:
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                rec = json.load(f)
            key = f"engine_drawstats_b{B}_g{g}_v{V}"
            if key in rec:
                traffic = rec[key]["hbm_bytes_per_launch"]
        line = {
            "metric": METRIC,
            "value": tokens / elapsed,
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (target logits ~ N(0,3^2), drafter = target + N(0,1), draft ids sampled from the drafter)",
            "config": {"workload": "configs[2]: Llama-3-8B/3.2-1B logit shapes, engine step sampling path: "
                                   "γ drafter draws + verify (rule A10)",
                       "rows_per_gpu": args.batch, "global_batch": args.batch * world, "gamma": g, "vocab": V,
                       "parallelism": f"dp{world}", "noise": "philox", "graph_steps": G},
            "acceptance_rate": accepted / drafted,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_stats", "kernel_ms": stats_ms, "launches_per_event_pair": PROF_REPEAT,
                         "alg_bytes_per_launch": alg_bytes,
                         "step_bytes": step_bytes, "step_achieved_gbs": step_gbs,
                         "step_frac": step_gbs / HBM_PEAK_GBS},
            "phases_ms": {"draws": ms_per_step - verify_ms, "verify": verify_ms},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline(tl, dl, draft, args):
    """Oracle (reference semantics, torch-CPU) on the same logits: the drafter draws
    (softmax + multinomial per draft position, engine/infer_engine.py:241-247), the target
    softmax and the per-row accept/resample loop of :276-336."""
    sys.path.insert(0, ROOT)
    from oracle import specdec_ref as ref
    cores = min(len(os.sched_getaffinity(0)), 16)
    torch.set_num_threads(cores)
    tlc, dlc, dc = tl.cpu(), dl.cpu(), draft.cpu()
    B, g, V = tlc.shape
    gen_cpu = torch.Generator().manual_seed(0)
    noise = ref.TorchNoise(gen_cpu)
    t0 = time.perf_counter()
    steps = tokens = 0
    while True:
        q = torch.softmax(dlc, dim=-1).float()
        for d in range(g):
            dc[:, d] = torch.multinomial(q[:, d], 1, generator=gen_cpu).squeeze(-1)
        p = torch.softmax(tlc, dim=-1)
        gen = torch.zeros(B, g, dtype=torch.long)
        gen[:, :] = dc
        fin = torch.zeros(B, dtype=torch.bool)
        acc = torch.zeros(B, dtype=torch.long)
        n = ref.engine_verify_rows(p, q, dc, fin, [128001, 128009], 0, gen, acc, noise)
        tokens += sum(min(k + 1, g) for k in n)
        steps += 1
        if time.perf_counter() - t0 > args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": tokens / dt, "unit": "tokens/s", "cores": cores, "kind": "port",
            "sample": f"{steps} engine steps (γ drafter draws + verify) of the same {B}x{g}x{V} bf16 logits "
                      "(oracle, torch-CPU)",
            "ms_per_step": dt / steps * 1e3}


if __name__ == "__main__":
    main()
