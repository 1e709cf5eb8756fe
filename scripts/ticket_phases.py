"""Where the slots go in a ticket-order fused verify (diagnostic; GPU box).

Loads the SD_PHASE_TIMING build (make -C speculative-decoding_amd timing), runs the perf-mode
engine-rule verify at batch B (default 512; γ = 4, V = 128256 bf16, Philox, the drafter rows'
statistics from the draws as in bench.py's sweep) and reads back, per workgroup, its phase stamps
(s_memrealtime, 100 MHz) and the work item its ticket gave it (SD_TS_ROLE: ticket, sequence,
span / decider / sampler).  Prints each role's timings and the share of the launch's slot-time
(makespan x resident slots) each role holds — streaming, waiting or computing — and saves the
raw table to gpurun_out/ticket_phases_B<B>.npz.
"""
import os
import sys

os.environ.setdefault("SPECDEC_LIB", "libspecdec_ts.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

B, G, V = int(os.environ.get("B", 512)), 4, 128256
NWG = 32768
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
tl = (torch.randn(B, G, V, device=dev, generator=g) * 3).to(torch.bfloat16)
dl = (tl.float() + torch.randn(B, G, V, device=dev, generator=g)).to(torch.bfloat16)
noise = PhiloxNoise(seed=1)
dstats = torch.empty(G, B, 2, device=dev)
ids = torch.empty(B, G, dtype=torch.long, device=dev)
for d in range(G):
    ids[:, d] = ops.sample_rows(dl[:, d], ops.PLAIN_SOFTMAX, noise, row_stats_out=dstats[d])[0]
ts = torch.zeros(NWG * 16 + NWG, dtype=torch.int64, device=dev)
stops = torch.tensor([], dtype=torch.long, device=dev)


def step():
    return ops.verify([tl[:, t] for t in range(G)], [dl[:, t] for t in range(G)], ids, _lib.SD_RULE_ENGINE,
                      ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise, stops, draft_row_stats=dstats)


for _ in range(5):
    step()
torch.cuda.synchronize()
print("verify path:", _lib.PATH_NAMES.get(_lib.last_verify_path(), "?"), flush=True)
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
for rep in range(3):
    ts.zero_()
    torch.cuda.synchronize()
    step()   # the same step just before: the bench's regime (busy GPU)
    ts.zero_()
    step()
    torch.cuda.synchronize()
    raw = ts.cpu().numpy()
    t = raw[:NWG * 16].reshape(NWG, 16)
    role = raw[NWG * 16:]
    live = t[:, 0] > 0
    t0 = t[live, 0].min()
    # columns 12-15 of workgroups past 8192 hold s_memtime (shader clock) stamps: not times here
    d = (t[:, :12] - t0) / 100.0
    d[t[:, :12] == 0] = np.nan
    r = role & 0xfff
    kind = np.where(~live, -1, np.where(r & 0x800, 2, np.where(r & 0x400, 1, 0)))   # 0 span 1 decider 2 sampler
    end = np.nanmax(d, axis=1)
    span = (kind == 0)
    dec = (kind == 1)
    smp = (kind == 2)
    make = np.nanmax(end)
    print(f"--- rep {rep}: {live.sum()} workgroups ran ({span.sum()} spans, {dec.sum()} deciders, "
          f"{smp.sum()} samplers), makespan {make:.1f} us")

    def pr(name, v):
        v = v[~np.isnan(v)]
        if len(v):
            print(f"  {name:34s} n={len(v):6d} p10 {np.percentile(v, 10):7.2f} p50 {np.median(v):7.2f} "
                  f"p90 {np.percentile(v, 90):7.2f} max {v.max():7.2f}")

    pr("span start", d[span, 0])
    pr("span start -> stream done", d[span, 6] - d[span, 0])
    pr("span start -> record stored", d[span, 8] - d[span, 0])
    pr("decider start", d[dec, 0])
    pr("decider start -> spans polled", d[dec, 9] - d[dec, 0])
    pr("decider polled -> decided", d[dec, 3] - d[dec, 9])
    pr("decider start -> end", end[dec] - d[dec, 0])
    pr("sampler start", d[smp, 0])
    pr("sampler start -> saw decision", d[smp, 1] - d[smp, 0])
    pr("sampler decision -> done", d[smp, 2] - d[smp, 1])
    # slot-time shares: busy time of each role over makespan x the slots in use at the peak
    dur = end - d[:, 0]
    tot = np.nansum(dur[live])
    for nm, m in (("span", span), ("decider", dec), ("sampler", smp)):
        print(f"  slot-time {nm:8s} {np.nansum(dur[m]) / tot * 100:5.1f} %  ({np.nansum(dur[m]):9.0f} wg-us)")
    sw = np.nansum(d[smp, 1] - d[smp, 0])
    dw = np.nansum(d[dec, 9] - d[dec, 0]) + np.nansum(end[dec] - d[dec, 3])
    print(f"  of which waiting: samplers {sw / tot * 100:.1f} %, deciders {dw / tot * 100:.1f} %")
    # concurrency in 5 us bins: workgroups alive per role
    assert make < 1e5, make   # a stamp outside this launch: do not build a giant bin table
    bins = np.arange(0, make + 5, 5.0)
    rows = []
    for lo in bins[:-1]:
        hi = lo + 5.0
        al = (d[:, 0] < hi) & (end > lo)
        rows.append((lo, int((al & span).sum()), int((al & dec).sum()), int((al & smp).sum())))
    print("  t(us)  spans deciders samplers alive")
    for lo, a, b_, c in rows:
        print(f"  {lo:5.0f} {a:6d} {b_:8d} {c:8d}")
    if rep == 2:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"ticket_phases_B{B}.npz"), t=t, role=role)
