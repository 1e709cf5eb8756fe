"""Per-workgroup phase timing of one perf-mode verify step (diagnostic; GPU box).

Loads the SD_PHASE_TIMING build (make -C speculative-decoding_amd timing), runs the bench
shape (engine rule, B=32, γ=4, V=128256 bf16, Philox; B=1 RULE=spec: configs[1]'s multinomial
verify over γ+1 target rows; PROC=nucleus: configs[1]'s nucleus-0.9 verify, the drafter rows'
statistics reduced in the launch as the drop-in loop does for nucleus drafters) and prints, per kernel, when workgroups
start / reach each phase relative to the kernel's first start (µs, s_memrealtime = 100 MHz).
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

B, G, V = int(os.environ.get("B", 32)), 4, 128256
SPEC = os.environ.get("RULE", "engine") == "spec"
NT = G + 1 if SPEC else G
LEAN = B <= 8   # the default dispatch (SD_OPT_LEAN_VERIFY = -1): k_verify_lean for <= 8 sequences
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
tl = (torch.randn(B, NT, V, device=dev, generator=g) * 3).to(torch.bfloat16)
dl = (tl[:, :G].float() + torch.randn(B, G, V, device=dev, generator=g)).to(torch.bfloat16)
ids = dl.float().argmax(-1)
noise = PhiloxNoise(seed=1)
NUC = os.environ.get("PROC") == "nucleus"
proc = ops.ProcSpec("nucleus", 1.0, 0, 0.9) if NUC else ops.PLAIN_SOFTMAX
# the bench's verify: drafter rows' (max, Σexp) come from the draws, k_stats reads target rows only
dstats = None if NUC else torch.empty(G, B, 2, device=dev)
for d in range(G if not NUC else 0):
    ops.sample_rows(dl[:, d], ops.PLAIN_SOFTMAX, noise, row_stats_out=dstats[d])
ts = torch.zeros(16384 * 16, dtype=torch.int64, device=dev)


def step():
    return ops.verify([tl[:, t] for t in range(NT)], [dl[:, t] for t in range(G)], ids,
                      _lib.SD_RULE_SPEC if SPEC else _lib.SD_RULE_ENGINE,
                      proc, proc, noise, torch.tensor([], dtype=torch.long, device=dev),
                      draft_row_stats=dstats)


for _ in range(20):
    step()
torch.cuda.synchronize()
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
warm = torch.randn(8192, 8192, device=dev)
for rep in range(4):
    ts.zero_()
    torch.cuda.synchronize()
    if rep == 2:   # keep the GPU busy right up to the step (no idle gap before it; caches cold)
        for _ in range(20):
            warm = warm @ warm
            warm = warm / warm.norm()
    if rep == 3:   # the bench's regime: the same step just before (busy GPU, its rows cache-warm);
        step()     # every stamp slot is rewritten by the second step
    step()
    torch.cuda.synchronize()
    t = ts.view(-1, 16).cpu().numpy().astype(np.int64)
    print(f"--- rep {rep}")
    for name, lo, hi, phases in (("k_stats", 0, 8192, ["start", "merged", "arrived", "decided", "dec_stats", "dec_ratios",
                                                        "stream_done", "pf_late", "rec_stored", "dec_polled",
                                                        "-", "dec_tags_ok"]
                   if not LEAN else ["start", "merged", "rec_stored", "decided", "accepts", "-",
                                     "loads_landed", "rows_reduced"]),
                                 ("k_sample_finish", 16384 - 64, 16384, ["start", "prologue", "body_end", "arrived",
                                                            "tail_S", "cdf_pick", "finalized", "cdf_select",
                                                            "cdf_loaded", "cdf_wscan", "cdf_found", "cdf_1st"]),
                                 ("k_sample", 8192, 16384 - 64, ["start", "prologue", "body_end", "arrived",
                                                            "tail_S", "cdf_pick", "finalized", "cdf_select",
                                                            "weights", "chunk_pick", "-", "-"])):
        blk = t[lo:hi]
        blk = blk[blk[:, 0] > 0]
        if not len(blk):
            continue
        t0 = blk[:, 0].min()
        print(f"{name}: {len(blk)} workgroups")
        for k, ph in enumerate(phases):
            v = blk[:, k]
            v = v[v > 0]
            if len(v):
                d = (v - t0) / 100.0
                print(f"  {ph:10s} n={len(v):5d}  min {d.min():7.2f}  p50 {np.median(d):7.2f}  max {d.max():7.2f} us")
    # the fused verify (k_verify_fused, B >= 8): spans + a decider per sequence, then the samplers
    nsp = 16 if not SPEC else 20
    head = B * (nsp + 1)
    blk = t[:8192]
    if (blk[head:, 0] > 0).any() and not LEAN:
        t0 = blk[blk[:, 0] > 0, 0].min()
        d = (blk - t0) / 100.0
        d[blk == 0] = np.nan
        wgi = np.arange(8192)
        item = (wgi >> 3) % (nsp + 1)
        roles = {"span": (wgi < head) & (item < nsp), "decider": (wgi < head) & (item == nsp),
                 "sampler": (wgi >= head) & (wgi < 4096) & (blk[:, 0] > 0),
                 "finish": (wgi >= 4096) & (blk[:, 6] > 0)}
        names = {"span": {0: "start", 6: "stream_done", 1: "merged", 8: "rec_stored"},
                 "decider": {0: "start", 7: "pf_done", 9: "polled", 11: "tags_ok", 13: "reduced", 14: "ratio0", 15: "accept0", 10: "ratios", 4: "synced",
                             6: "ballots", 8: "built", 12: "published", 5: "walked", 3: "decided", 1: "drec_stored"},
                 "finish": {4: "tail_S", 7: "chunk_picked", 5: "candidate", 6: "finalized"},
                 "sampler": {0: "start", 1: "saw_decision", 8: "weights", 9: "chunk_pick", 2: "done"}}
        print("fused verify roles:")
        for r, m in roles.items():
            for col, nm in names[r].items():
                v = d[m, col]
                v = v[~np.isnan(v)]
                if len(v):
                    print(f"  {r:8s} {nm:13s} n={len(v):5d}  min {v.min():7.2f}  p50 {np.median(v):7.2f}  max {v.max():7.2f} us")
    if rep == 3:   # per-workgroup dump of the k_stats launch for offline analysis
        np.save(os.path.join(ROOT, "gpurun_out", "phase_kstats.npy"), t[:8192])
    blk = t[8192:16384]
    sel = (blk[:, 4] > 0) & (blk[:, 10] > 0)
    if sel.any():
        real = (blk[sel, 10] - blk[sel, 4]).astype(np.float64)       # 100 MHz ticks
        core = (blk[sel, 13] - blk[sel, 12]).astype(np.float64)      # shader clock ticks
        print(f"  tail shader clock: {np.median(core / real) * 100:.0f} MHz (median over {sel.sum()} tails)")
