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

value = output tokens (accepted drafts + resampled tokens, all ranks, counted exactly by the
verify kernel itself: sd_verify_args.row_counts) / max-over-ranks wall time of the K timed steps,
per trial; the median of the trials' ratios is reported.
Steps run as hipGraph replays — G = --graph-steps steps (default 20) per captured graph, K/G replays per
timed trial; --trials trials of exactly K steps (median reported), each replay also timed by HIP events —
and noise is in-kernel Philox (perf mode).
Also reported in the same line: acceptance rate (engine/metrics.py:123-129) over >= 200 untimed
steps, per-kernel timings with the HBM roofline of the step's DOMINANT kernel (the largest
per-step share; HIP events on the launch stream, algorithmic bytes = every logit row the kernel
must read, once), the same step in STREAM mode (the reference's torch-generator noise, bit-exact
tokens, in a noise session as the drop-in engine runs it), the strong-scaling variant of
configs[2] (a global batch of --batch rows split over the ranks) when N > 1 and its 16 / 8 / 4-row
shards measured on one GPU when N = 1, the configs[1] batch-1 step latencies, the configs[4]
n-gram verify step, and the CPU baseline = the oracle (reference semantics, torch-CPU) timed on a
bounded sample of the same workload on this host.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
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
    ap.add_argument("--cpu-seconds", type=float, default=30.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stream-steps", type=int, default=5, help="STREAM-mode (bit-exact noise) steps; 0 = skip")
    ap.add_argument("--no-configs1", action="store_true", help="skip the configs[1] / configs[4] batch-1 lines")
    ap.add_argument("--no-shards", action="store_true", help="skip the 16 / 8 / 4-row shard lines")
    ap.add_argument("--sweep-batches", default="128,512",
                    help="rows per GPU of the large-batch roofline sweep (SURVEY §8(d)); empty = skip")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end line (random-init Llama-3-8B / 3.2-1B shaped models, drop-in engine)")
    ap.add_argument("--e2e-gen", type=int, default=64, help="new tokens per row in the end-to-end line")
    ap.add_argument("--trials", type=int, default=5,
                    help="timed trials of exactly --steps steps each (median reported)")
    ap.add_argument("--profile-only", action="store_true",
                    help="only the B-row engine step (no shards, configs[1]/[4], STREAM or CPU lines): every "
                         "sd:: launch of the run has the headline shape, for rocprofv3 / PMC passes")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="dispatch option for A/B runs (sd_set_option), e.g. FUSED_VERIFY=0 or LEAN_VERIFY=0")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank) or gloo (rehearsing N ranks on fewer GPUs)")
    a = ap.parse_args()
    a.sweep_batches = [int(x) for x in a.sweep_batches.split(",") if x.strip()]
    if a.profile_only:
        a.no_cpu_baseline = a.no_configs1 = a.no_shards = a.no_e2e = True
        a.stream_steps = 0
        a.sweep_batches = []
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def graph_steps(step, steps, per_graph, noise=None, calls_per_step=0, min_replays=1):
    """Capture G steps in one hipGraph (G <= per_graph, G divides steps, and at least min_replays
    replays when steps allows), replay once untimed.  Returns (graph, outputs of the captured
    steps, replays).  With a PhiloxNoise that has a device counter base, the graph ends by moving
    it past the captured calls, so every replay draws fresh noise (the outputs are those of the
    last replay)."""
    G = max(1, min(per_graph, steps, steps // max(min_replays, 1) or 1))
    while steps % G:
        G -= 1
    graph = torch.cuda.CUDAGraph()
    outs = []
    with torch.cuda.graph(graph):
        for _ in range(G):
            outs.append(step())
        if noise is not None and noise.offset_dev is not None:
            noise.advance_device(G * calls_per_step)
    graph.replay()
    torch.cuda.synchronize()
    return graph, outs, steps // G


def timed_replays(graph, replays, dist, per_replay=None):
    """Wall time of `replays` back-to-back replays, bracketed by a barrier and a device sync on both
    sides.  per_replay (a list): receives each replay's device time in ms, from HIP events recorded
    on the launch stream between the replays (no sync inside the timed region)."""
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(replays + 1)] if per_replay is not None else None
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    for i in range(replays):
        graph.replay()
        if evs:
            evs[i + 1].record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if evs:
        per_replay.extend(evs[i].elapsed_time(evs[i + 1]) for i in range(replays))
    return elapsed


def engine_logits(B, g, V, sigma, seed, dev):
    gen = torch.Generator(device=dev).manual_seed(seed)
    tl = (torch.randn(B, g, V, generator=gen, device=dev) * 3.0).to(torch.bfloat16)
    dl = (tl.float() + sigma * torch.randn(B, g, V, generator=gen, device=dev)).to(torch.bfloat16)
    return tl, dl


class EngineStep:
    """One engine step's sampling path over resident logits: γ drafter draws (sd_sample, one launch
    each, engine/infer_engine.py:241-247) + one sd_verify (rule A10, :276-336)."""

    def __init__(self, tl, dl, noise, row0, ops, _lib):
        self.ops, self.lib = ops, _lib
        B, g, V = tl.shape
        dev = tl.device
        self.B, self.g, self.V = B, g, V
        self.noise, self.row0 = noise, row0
        self.draft = torch.empty(B, g, dtype=torch.long, device=dev)
        self.stash = True   # the draws return their rows' (max, Σexp) in both noise modes
        self.dstats = torch.empty(g, B, 2, dtype=torch.float32, device=dev)   # drafter rows' (max, Σexp)
        self.stops = torch.tensor([128001, 128009], dtype=torch.long, device=dev)
        self.trows = [tl[:, t, :] for t in range(g)]
        self.drows = [dl[:, t, :] for t in range(g)]
        # per row (accepted drafts, tokens emitted), accumulated by the verify kernel itself: every
        # timed step's tokens are counted exactly, with no extra launch (sd_verify_args.row_counts)
        self.counts = torch.zeros(B, 2, dtype=torch.long, device=dev)

    def draw(self, d):
        self.ops.sample_rows(self.drows[d], self.ops.PLAIN_SOFTMAX, self.noise, tokens_out=self.draft[:, d],
                             row_base=self.row0, row_stats_out=self.dstats[d] if self.stash else None)

    def draw_rows(self, rows):
        """A draw of the slot-0 drafts from other [B, V] rows (the roofline's rotating draw loop)."""
        self.ops.sample_rows(rows, self.ops.PLAIN_SOFTMAX, self.noise, tokens_out=self.draft[:, 0],
                             row_base=self.row0, row_stats_out=self.dstats[0] if self.stash else None)

    def draws(self):
        for d in range(self.g):
            self.draw(d)

    def verify(self, prof=None):
        ops = self.ops
        return ops.verify(self.trows, self.drows, self.draft, self.lib.SD_RULE_ENGINE, ops.PLAIN_SOFTMAX,
                          ops.PLAIN_SOFTMAX, self.noise, self.stops, prof_events=prof, row_base=self.row0,
                          draft_row_stats=self.dstats if self.stash else None, row_counts=self.counts)

    def reserve(self):
        """STREAM: the step's words in one generation (γ draws of 2·B·V, the verify's <= B·(γ+2V)),
        as the drop-in engine reserves a window's words (noise.StreamNoise.reserve)."""
        if hasattr(self.noise, "reserve"):
            self.noise.reserve(self.g * 2 * self.B * self.V + self.B * (self.g + 2 * self.V), self.trows[0].device,
                               known=self.g * 2 * self.B * self.V)

    def __call__(self, prof=None):
        self.reserve()
        self.draws()
        return self.verify(prof)

    def read_counts(self):
        """(accepted drafts, tokens emitted) per row since the last reset, and reset."""
        c = self.counts.cpu()
        self.counts.zero_()
        return c


def positive_rate_sums(acc_rows, drafted_per_row):
    """engine/metrics.py:123-129 averages per-row acc/tot over the rows whose rate is > 0:
    returns (Σ positive rates, count) so ranks can be summed."""
    rates = acc_rows.double() / drafted_per_row
    pos = rates[rates > 0]
    return float(pos.sum()), int(pos.numel())


def kernel_events(fn, repeat, n_pairs):
    """Mean time of one `fn()` launch: torch events on the current stream (the one the ops launch
    on) around `repeat` back-to-back launches, averaged over n_pairs pairs."""
    ts = []
    for _ in range(n_pairs):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(repeat):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / repeat)
    return sum(ts) / len(ts)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    local = local % torch.cuda.device_count()   # == local on a node with a GPU per rank
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    import specdec_amd  # noqa: F401
    from specdec_amd import _lib, dp, ops
    from specdec_amd.noise import PhiloxNoise, StreamNoise

    for kv in args.option:   # A/B runs: another kernel path for the same outputs
        k, v = kv.split("=", 1)
        _lib.set_option(getattr(_lib, f"SD_OPT_{k.upper()}"), int(v))
    g, V = args.gamma, args.vocab
    # weak scaling (the value): args.batch rows per rank, the global batch split contiguously by row
    # (specdec_amd/dp.py); Philox noise is keyed by the global row id, so the shards draw what one GPU
    # verifying the whole batch would draw for the same rows.  No data-path collective.
    row0, row1 = dp.shard_rows(args.batch * world, world, rank)
    B = row1 - row0
    tl, dl = engine_logits(B, g, V, args.sigma, 1000 + rank, dev)
    # the Philox counter base lives on the device: every replay of the captured steps draws fresh noise
    noise = PhiloxNoise(seed=4242, offset_dev=torch.zeros(1, dtype=torch.long, device=dev))
    step = EngineStep(tl, dl, noise, row0, ops, _lib)
    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    # which verify kernels the step runs, as the library reports it (sd_last_verify_path)
    verify_path = _lib.last_verify_path()
    # the K timed steps: one captured graph of G steps (G = --graph-steps, dividing K), replayed K/G times
    # per trial; --trials trials of exactly K steps, each bracketed by a barrier and a device sync, the
    # median trial reported (every trial's tokens counted exactly by the verify kernel)
    graph, outs, replays = graph_steps(step, args.steps, args.graph_steps, noise, g + 1)
    G = len(outs)
    step.read_counts()                                   # drop the warm-up / capture replay's counts
    replay_ms, trial_s, trial_rate, trial_tok = [], [], [], []
    acc_t = torch.zeros(B, dtype=torch.long)
    for _ in range(max(args.trials, 1)):
        t = timed_replays(graph, replays, dist, replay_ms)
        c = step.read_counts()                           # exact: this trial's tokens (outside the timed region)
        acc_t += c[:, 0]
        t, tt = dp.aggregate(t, {"tokens": int(c[:, 1].sum())}, dev, dist)
        trial_s.append(t)
        trial_tok.append(tt["tokens"])
        trial_rate.append(tt["tokens"] / t)
    n_trials = len(trial_s)
    mid = sorted(range(n_trials), key=lambda i: trial_rate[i])[n_trials // 2]   # the median trial
    value = trial_rate[mid]
    elapsed = trial_s[mid]
    rsum_t, rcnt_t = positive_rate_sums(acc_t, g * args.steps * n_trials)

    # acceptance over a larger untimed sample (>= 200 steps of the same graph, fresh noise each)
    n_count = max(1, -(-max(200, args.steps) // G))
    for _ in range(n_count):
        graph.replay()
    counts_c = step.read_counts()
    rsum, rcnt = positive_rate_sums(counts_c[:, 0], g * G * n_count)

    # the verify alone (on the captured draws' outputs), for the per-phase breakdown
    vgraph, _, vrep = graph_steps(step.verify, args.steps, args.graph_steps)
    verify_ms = statistics.median(timed_replays(vgraph, vrep, None) for _ in range(3)) / args.steps * 1e3

    _, tot = dp.aggregate(elapsed, {"accepted": float(acc_t.sum()),
                                          "drafted": B * g * args.steps * n_trials, "rate_sum": rsum, "rate_cnt": rcnt,
                                          "rate_sum_t": rsum_t, "rate_cnt_t": rcnt_t,
                                          "accepted_c": float(counts_c[:, 0].sum()),
                                          "drafted_c": B * g * G * n_count}, dev, dist)

    # per-kernel timing (HIP events on the launch stream, back-to-back launches so the event pair's
    # own cost is amortised): k_draw (one per drafter draw), k_stats (sd_verify's prof hook, with its
    # decide tail), and the rest of the verify (k_sample with its tail) by difference.  The draws cycle
    # over 8 distinct [B, V] row sets (the 4 drafter and 4 target rows, 2x the 32 MiB of aggregate L2 at
    # the bench shape), so each launch reads its rows from Infinity Cache / HBM as in the step, not from
    # an L2 a back-to-back loop over one row set would keep hot.
    rot = step.drows + step.trows
    dgraph, _, _ = graph_steps(lambda it=iter(range(1 << 30)): step.draw_rows(rot[next(it) % len(rot)]),
                               PROF_REPEAT, PROF_REPEAT)   # launch-overhead free
    draw_ms = kernel_events(dgraph.replay, 1, args.prof_steps) / PROF_REPEAT
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.prof_steps)]
    for e in ev:
        e[0].record()   # marks the torch events as recorded; sd_verify re-records them around k_stats
        e[1].record()
        step.verify(prof=(e[0], e[1], PROF_REPEAT))
    torch.cuda.synchronize()
    stats_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev) / PROF_REPEAT
    sample_ms = max(verify_ms - stats_ms, 0.0)
    ms_per_step = elapsed / args.steps * 1e3
    row_bytes = B * V * 2
    kernels = {
        # per launch: algorithmic bytes = each logit row the kernel must read, once
        "k_draw": {"ms": (ms_per_step - verify_ms) / g, "launches_per_step": g, "alg_bytes_per_launch": row_bytes,
                   "isolated_ms": draw_ms,
                   "note": "ms: the timed region's draw phase per launch = (step - the verify's graph-timed "
                           "share) / γ; isolated_ms: 20 graph-replayed launches between HIP events, cycling over "
                           "8 row sets (no L2-hot reuse); both include the dispatch gap between launches"},
    }
    # sd_verify's dispatch as the library reported it for the step's verify (sd_last_verify_path)
    if verify_path == _lib.SD_PATH_VERIFY_FUSED:
        kernels["k_verify_fused"] = {
            "ms": verify_ms, "launches_per_step": 1, "alg_bytes_per_launch": (g + 1) * row_bytes,
            "note": "the whole verify in one launch (graph-replayed verify steps); algorithmic bytes = the γ target "
                    "rows once + the decided drafter row once (the decided target row is a re-read)"}
        kernels["k_stats"] = {"ms": stats_ms, "launches_per_step": 0, "alg_bytes_per_launch": g * row_bytes,
                              "note": "diagnostic: the two-launch path's statistics kernel (sd_verify's prof hook "
                                      "runs it, not the fused launch), 20 back-to-back launches"}
    elif verify_path == _lib.SD_PATH_VERIFY_LEAN:
        kernels["k_verify_lean"] = {"ms": verify_ms, "launches_per_step": 1, "alg_bytes_per_launch": g * row_bytes,
                                    "note": "the whole verify in one launch (graph-replayed verify steps)"}
    else:
        kernels["k_stats"] = {"ms": stats_ms, "launches_per_step": 1, "alg_bytes_per_launch": g * row_bytes}
        kernels["k_sample"] = {"ms": sample_ms, "launches_per_step": 1, "alg_bytes_per_launch": 2 * row_bytes,
                               "note": "verify minus k_stats (graph-timed); rows re-read from L2 / Infinity Cache"}
    for k in kernels.values():
        k["ms_per_step"] = k["ms"] * k["launches_per_step"]   # 0 for diagnostic entries
        k["achieved_gbs"] = k["alg_bytes_per_launch"] / (k["ms"] * 1e-3) / 1e9 if k["ms"] > 0 else None
        k["frac"] = k["achieved_gbs"] / HBM_PEAK_GBS if k["achieved_gbs"] else None
    dominant = max(kernels, key=lambda n: kernels[n]["ms_per_step"])

    # strong scaling (configs[2] as written: a GLOBAL batch of args.batch rows split over the ranks)
    strong = None
    if world > 1:
        s0, s1 = dp.shard_rows(args.batch, world, rank)
        stl, sdl = tl[:s1 - s0], dl[:s1 - s0]
        snoise = PhiloxNoise(seed=4343, offset_dev=torch.zeros(1, dtype=torch.long, device=dev))
        sstep = EngineStep(stl, sdl, snoise, s0, ops, _lib)
        for _ in range(max(args.warmup, 1)):
            sstep()
        torch.cuda.synchronize()
        sgraph, souts, sreplays = graph_steps(sstep, args.steps, args.graph_steps, snoise, g + 1, min_replays=5)
        sstep.read_counts()
        selapsed = timed_replays(sgraph, sreplays, dist)
        stoks = int(sstep.read_counts()[:, 1].sum())
        selapsed, stot = dp.aggregate(selapsed, {"tokens": stoks}, dev, dist)
        strong = {"value": stot["tokens"] / selapsed, "unit": "tokens/s", "global_batch": args.batch,
                  "rows_per_gpu": s1 - s0, "ms_per_step": selapsed / args.steps * 1e3}

    # configs[2]'s strong-scaling shards measured on this GPU: 32 / N rows per GPU at N = 2, 4, 8
    shards = None
    if rank == 0 and world == 1 and not args.no_shards:
        shards = shard_lines(tl, dl, args, ops, _lib, PhiloxNoise, EngineStep)

    sweep = None
    if rank == 0 and world == 1 and args.sweep_batches:
        sweep = sweep_lines(args, ops, _lib, PhiloxNoise, EngineStep, dev)

    stream = None
    if args.stream_steps > 0:   # every rank: batch-level data parallelism (bit-exact), weak scaling
        stream = stream_line(tl, dl, row0, args, ops, _lib, StreamNoise, dp, dev, dist, world, rank)
    cfg1 = cfg4 = None
    if rank == 0 and world == 1 and not args.no_configs1:
        cfg1 = configs1_lines(dev, args, ops, _lib, PhiloxNoise)
        cfg4 = configs4_line(dev, args, ops, _lib, PhiloxNoise)
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = e2e_line(args)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(tl, dl, step.draft, args)

    if rank == 0:
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                rec = json.load(f)
            key = f"{dominant}_engine_b{B}_g{g}_v{V}"
            if key in rec:
                traffic = rec[key]["hbm_bytes_per_launch"]
        dk = kernels[dominant]
        step_bytes = B * 2 * g * V * 2          # the step: every target and drafter row once
        step_gbs = step_bytes / (ms_per_step * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": value,
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
                       "parallelism": f"dp{world}", "noise": "philox", "graph_steps": G, "replays_per_trial": replays,
                       "trials": n_trials, "verify_path": _lib.PATH_NAMES.get(verify_path, str(verify_path))},
            # engine/metrics.py:123-129: mean of per-row acc/tot over the rows with a positive rate,
            # over >= 200 untimed steps of the same graph (the timed steps' own figure beside it)
            "acceptance_rate": tot["rate_sum"] / tot["rate_cnt"] if tot["rate_cnt"] else 0.0,
            "acceptance_rate_pooled": tot["accepted_c"] / tot["drafted_c"],
            "acceptance_steps": G * n_count,
            "acceptance_rate_timed": tot["rate_sum_t"] / tot["rate_cnt_t"] if tot["rate_cnt_t"] else 0.0,
            "tokens_timed": trial_tok[mid],
            "replays": {"count": replays * n_trials, "steps_per_replay": G,
                        "ms_median": statistics.median(replay_ms), "ms_min": min(replay_ms),
                        "ms_max": max(replay_ms),
                        "ms_per_step_median": statistics.median(replay_ms) / G,
                        "trial_ms_per_step": [t / args.steps * 1e3 for t in trial_s],
                        "trial_tokens_per_s": trial_rate,
                        "note": "HIP events between back-to-back replays of the captured steps (rank 0); "
                                "trial_ms_per_step: each trial's wall time / K; value = the median trial's "
                                "tokens / its time (ms_per_step is that trial's)"},
            "roofline": {"bound": "hbm", "achieved": dk["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": dk["frac"], "traffic": traffic,
                         "kernel": dominant, "kernel_ms": dk["ms"], "launches_per_step": dk["launches_per_step"],
                         "launches_per_event_pair": PROF_REPEAT,
                         "alg_bytes_per_launch": dk["alg_bytes_per_launch"],
                         "step_bytes": step_bytes, "step_achieved_gbs": step_gbs,
                         "step_frac": step_gbs / HBM_PEAK_GBS},
            "kernels": kernels,
            "phases_ms": {"draws": ms_per_step - verify_ms, "verify": verify_ms},
            "stream": stream,
            "sweep": sweep,
            "strong_scaling": strong,
            "shard_rows": shards,
            "configs1": cfg1,
            "configs4": cfg4,
            "e2e": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def stream_line(tl, dl, row0, args, ops, _lib, StreamNoise, dp, dev, dist, world, rank):
    """The same engine step in STREAM mode: the noise is the reference's own torch CPU generator
    stream (bit-exact tokens under torch.manual_seed), run as the drop-in engine runs it — inside
    a noise session (the generator state stays on the device) with one word reservation per step
    (StreamNoise.reserve: one jump-ahead + generation for the γ draws and the verify).  Eager
    steps: the session's host bookkeeping sits between the calls.  With N ranks this is the
    batch-level data parallelism of specdec_amd.engine.dp_runner (every rank decodes its own whole
    batch of --batch rows from a generator seeded per batch, as engine/benchmark_executor.py:79
    re-seeds; no exchange; exact per batch): weak scaling, 1 batch per rank; value = tokens of all
    ranks / the slowest rank's time."""
    gen = torch.Generator().manual_seed(1234 + rank)   # batch `rank`'s seed
    noise = StreamNoise(gen)
    step = EngineStep(tl, dl, noise, 0, ops, _lib)     # a whole batch: rows 0..B-1 of its own
    B, g, V = step.B, step.g, step.V
    with noise.session():
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        step.read_counts()
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.stream_steps):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        c = step.read_counts()
    rsum, rcnt = positive_rate_sums(c[:, 0], g * args.stream_steps)
    dt, tot = dp.aggregate(dt, {"tokens": int(c[:, 1].sum()), "rate_sum": rsum, "rate_cnt": rcnt}, dev, dist)
    ms = dt / args.stream_steps * 1e3
    words = g * 2 * B * V + B * (g + 2 * V)          # reserved per step (the verify's worst case)
    return {"noise": "stream", "value": tot["tokens"] / dt, "unit": "tokens/s", "ms_per_step": ms,
            "steps": args.stream_steps, "rows": B, "n_gpus": world, "batches_per_rank": 1,
            "scaling": "weak", "exact": "bit-exact with the reference per batch (each rank's batch from its own "
                                        "re-seeded torch generator: dp_runner's batch-level mode)",
            "acceptance_rate": tot["rate_sum"] / tot["rate_cnt"] if tot["rate_cnt"] else 0.0,
            "logit_bytes_per_step": 2 * g * B * V * 2, "noise_words_per_step": words,
            "noise_bytes_per_step": words * 4 * 2,
            "note": "torch CPU generator words (bit-exact with the reference) made on the GPU, one reservation "
                    "per step in a noise session (as the drop-in engine); noise bytes = words written + read"}


def shard_lines(tl, dl, args, ops, _lib, PhiloxNoise, EngineStep):
    """configs[2] as written is a GLOBAL batch of 32 rows over N GPUs: 16 / 8 / 4 rows per GPU at
    N = 2 / 4 / 8.  One GPU times the engine step at each shard size (hipGraph replays), which
    bounds the strong-scaling curve: projected N-GPU tokens/s = N x the shard's tokens/s."""
    res = {}
    for rows in (16, 8, 4):
        if rows >= tl.shape[0]:
            continue
        noise = PhiloxNoise(seed=4545 + rows, offset_dev=torch.zeros(1, dtype=torch.long, device=tl.device))
        st = EngineStep(tl[:rows], dl[:rows], noise, 0, ops, _lib)
        for _ in range(3):
            st()
        torch.cuda.synchronize()
        steps = 100
        graph, _, replays = graph_steps(st, steps, 20, noise, st.g + 1, min_replays=5)
        st.read_counts()
        dt = timed_replays(graph, replays, None)
        tokens = int(st.read_counts()[:, 1].sum())
        n_gpus = args.batch // rows
        res[f"rows{rows}"] = {"rows_per_gpu": rows, "n_gpus_for_global_32": n_gpus,
                              "ms_per_step": dt / steps * 1e3, "tokens_per_s_per_gpu": tokens / dt,
                              "projected_global_tokens_per_s": n_gpus * tokens / dt}
    return res


def sweep_lines(args, ops, _lib, PhiloxNoise, EngineStep, dev):
    """SURVEY §8(d)'s large-batch roofline: the same engine step (configs[2]'s γ, V, logit
    distributions, Philox noise) at B = --sweep-batches rows on this GPU, hipGraph replays, with the
    verify path the library reports.  step_bytes = every target and drafter row once (2·γ·B·V·2);
    traffic_bytes adds the one re-read the residual resample cannot avoid: the decided target and
    drafter row of each sequence (2·B·V·2), so frac_traffic is the fraction of HBM peak the step's
    necessary reads run at."""
    res = {}
    g, V = args.gamma, args.vocab
    for B in args.sweep_batches:
        tl, dl = engine_logits(B, g, V, args.sigma, 5000 + B, dev)
        noise = PhiloxNoise(seed=4646 + B, offset_dev=torch.zeros(1, dtype=torch.long, device=dev))
        st = EngineStep(tl, dl, noise, 0, ops, _lib)
        for _ in range(3):
            st()
        torch.cuda.synchronize()
        path = _lib.last_verify_path()
        steps = 40
        graph, _, replays = graph_steps(st, steps, 10, noise, g + 1, min_replays=4)
        st.read_counts()
        dts = [timed_replays(graph, replays, None) for _ in range(3)]
        c = st.read_counts()
        dt = statistics.median(dts)
        vgraph, _, vrep = graph_steps(st.verify, steps, 10)
        vdt = statistics.median(timed_replays(vgraph, vrep, None) for _ in range(3))
        step_bytes = 2 * g * B * V * 2
        traffic = step_bytes + 2 * B * V * 2
        ms = dt / steps * 1e3
        res[f"b{B}"] = {"rows": B, "verify_path": _lib.PATH_NAMES.get(path, str(path)), "ms_per_step": ms,
                        "ms_per_step_trials": [d / steps * 1e3 for d in dts],
                        "verify_ms": vdt / steps * 1e3, "draw_ms": (ms - vdt / steps * 1e3) / g,
                        "tokens_per_s": float(c[:, 1].sum()) / (3 * dt),
                        "step_bytes": step_bytes, "frac": step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "traffic_bytes": traffic, "frac_traffic": traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        del graph, vgraph, st, tl, dl
        torch.cuda.empty_cache()
    return res


def configs4_line(dev, args, ops, _lib, PhiloxNoise):
    """configs[4]: the n-gram-assisted verify step (ngram_assisted/ngram_assisted.py:111-164, rule
    A11) — γ=8, top-p 0.9, filler top-3 over 9 synthetic Llama-3 shaped target rows (batch 1);
    hipGraph replays, Philox noise.

    What is drafted: A11 accepts draft i iff a draw from the processed target row i equals it
    (sample-and-compare), so its accept rate is p_i(draft_i).  An LM's next-token rows are peaked (the
    loop goldens' token-Markov banks are, tests/fakelm.py); here every target row is N(0, 1) noise
    with ONE hot token at logit 12.9 + U(0, 1.5), whose probability after the top-p 0.9 cut is
    ~0.6-0.85, and the draft at each position is that hot token (an n-gram store that predicts the
    row's likeliest continuation).  So the timed steps run the accept walk over several positions,
    the filler over the accepted ones and the final draw — not the reject-at-0 path alone."""
    g, V = 8, args.vocab
    gen = torch.Generator(device=dev).manual_seed(21)
    x = torch.randn(1, g + 1, V, generator=gen, device=dev)
    hot = torch.randint(0, V, (1, g + 1), generator=gen, device=dev)
    boost = 12.9 + 1.5 * torch.rand(1, g + 1, generator=gen, device=dev)
    x.scatter_(2, hot.unsqueeze(-1), boost.unsqueeze(-1))
    tl = x.to(torch.bfloat16)
    draft = hot[:, :g].contiguous()
    stops = torch.tensor([128001, 128009], dtype=torch.long, device=dev)
    proc = ops.ProcSpec("nucleus", 1.0, 0, 0.9)
    noise = PhiloxNoise(seed=9, offset_dev=torch.zeros(1, dtype=torch.long, device=dev))
    trows = [tl[:, t] for t in range(g + 1)]

    def step():
        return ops.ngram_verify(trows, draft, proc, noise, stops, filler_k=3)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    graph, outs, replays = graph_steps(step, 200, 20, noise, 1)
    dt = timed_replays(graph, replays, None)
    steps = len(outs) * replays
    # the acceptance over 50 more replays (fresh Philox noise each): the captured outputs hold the
    # last replay's values, so read them after every replay
    acc = []
    for _ in range(50):
        graph.replay()
        acc.append(torch.stack([o.n_accepted.long() for o in outs]).sum())
    n = float(torch.stack(acc).sum().item()) / (50 * len(outs))
    return {"us_per_step": dt / steps * 1e6, "tokens_per_s": (n + 1) * steps / dt,
            "accepted_per_step": n, "alg_bytes_per_step": (g + 1) * V * 2,
            "gamma": g, "top_p": 0.9, "filler_top_k": 3, "rule": "A11",
            "drafts": "the hot token of each peaked target row (p after the top-p cut ~0.6-0.85)"}


def configs1_lines(dev, args, ops, _lib, PhiloxNoise):
    """configs[1]: batch 1, γ=4, rule A8 (sampling/speculative_decoding.py:105-187) over synthetic
    Llama-3 shaped rows: γ drafter draws + one sd_verify over γ+1 target rows; greedy,
    multinomial T=1 and nucleus top-p 0.9; hipGraph replays."""
    g, V = args.gamma, args.vocab
    tl, dl = engine_logits(1, g + 1, V, args.sigma, 11, dev)
    dl = dl[:, :g].contiguous()
    stops = torch.tensor([128001, 128009], dtype=torch.long, device=dev)
    trows = [tl[:, t] for t in range(g + 1)]
    drows = [dl[:, t] for t in range(g)]
    res = {}
    for name, proc in (("greedy", ops.ProcSpec("greedy")), ("multinomial", ops.ProcSpec("multinomial", 1.0)),
                       ("nucleus_p0.9", ops.ProcSpec("nucleus", 1.0, 0, 0.9))):
        noise = PhiloxNoise(seed=7, offset_dev=torch.zeros(1, dtype=torch.long, device=dev))
        draft = torch.zeros(1, g, dtype=torch.long, device=dev)
        # as the drop-in loop does: the draws hand their rows' stats to the verify, except under a
        # top-k / nucleus processor (the nucleus draw runs without a threshold search: k_draw_nuc)
        dstats = torch.empty(g, 1, 2, dtype=torch.float32, device=dev) if not proc.keeps else None

        def step():
            for d in range(g):
                ops.sample_rows(drows[d], proc, noise, tokens_out=draft[:, d],
                                row_stats_out=dstats[d] if dstats is not None else None)
            return ops.verify(trows, drows, draft, _lib.SD_RULE_SPEC, proc, proc, noise, stops,
                              draft_row_stats=dstats)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        graph, outs, replays = graph_steps(step, 200, 20, noise, g + 1)
        dt = timed_replays(graph, replays, None)
        n = torch.stack([o.n_accepted.long() for o in outs]).sum().item()
        tokens = (n + len(outs)) * replays        # accepted + the resampled / bonus token, every step
        res[name] = {"us_per_step": dt / (len(outs) * replays) * 1e6, "tokens_per_s": tokens / dt,
                     "alg_bytes_per_step": (2 * g + 1) * V * 2}
    return res


def e2e_line(args):
    """The whole loop end to end (engine/infer_engine.py:99-146, the metric's own definition:
    engine/metrics.py:100-105 output tokens / wall time): random-init Llama-3-8B / Llama-3.2-1B shaped
    transformers models (bf16, no checkpoint exists offline) driving the drop-in
    batch_speculative_generate at B = 32, γ = 4 in both noise modes, with the hot path's device time
    (HIP events around every sd_sample / sd_verify call) against the wall time.  Random weights make
    the acceptance rate meaningless; tokens/s and the hot path's share are the measurement."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import e2e_timing
    try:
        return e2e_timing.run(batch=args.batch, gen=args.e2e_gen, gamma=args.gamma)
    except Exception as e:   # reported, never fatal to the headline line
        return {"error": f"{type(e).__name__}: {e}"}


def cpu_model_name():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                return ln.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(tl, dl, draft, args):
    """Oracle (reference semantics, torch-CPU) on the same logits: the drafter draws
    (softmax + multinomial per draft position, engine/infer_engine.py:241-247), the target
    softmax and the per-row accept/resample loop of :276-336.  SURVEY §8(d): every host thread
    this process may use (OMP_NUM_THREADS when the box sets it — its CPU share — else the
    affinity mask), 3 warm-up steps, then the median of >= 20 steps (fewer only if a step takes
    longer than args.cpu_seconds / 20)."""
    sys.path.insert(0, ROOT)
    from oracle import specdec_ref as ref
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    torch.set_num_threads(cores)
    tlc, dlc, dc = tl.cpu(), dl.cpu(), draft.cpu()
    B, g, V = tlc.shape
    gen_cpu = torch.Generator().manual_seed(0)
    noise = ref.TorchNoise(gen_cpu)

    def one_step():
        q = torch.softmax(dlc, dim=-1).float()
        for d in range(g):
            dc[:, d] = torch.multinomial(q[:, d], 1, generator=gen_cpu).squeeze(-1)
        p = torch.softmax(tlc, dim=-1)
        gen = torch.zeros(B, g, dtype=torch.long)
        gen[:, :] = dc
        fin = torch.zeros(B, dtype=torch.bool)
        acc = torch.zeros(B, dtype=torch.long)
        n = ref.engine_verify_rows(p, q, dc, fin, [128001, 128009], 0, gen, acc, noise)
        return sum(min(k + 1, g) for k in n)

    for _ in range(3):
        one_step()
    times, toks = [], []
    t_all = time.perf_counter()
    while len(times) < 20:
        t0 = time.perf_counter()
        toks.append(one_step())
        times.append(time.perf_counter() - t0)
        if len(times) >= 5 and time.perf_counter() - t_all > args.cpu_seconds:
            break
    med = statistics.median(times)
    return {"value": (sum(toks) / len(toks)) / med, "unit": "tokens/s", "cores": cores, "kind": "port",
            "cpu": cpu_model_name(),
            "sample": f"median of {len(times)} engine steps (after 3 warm-up) — γ drafter draws + verify of the "
                      f"same {B}x{g}x{V} bf16 logits (oracle = reference semantics, torch-CPU, {cores} threads)",
            "ms_per_step": med * 1e3}


if __name__ == "__main__":
    main()
