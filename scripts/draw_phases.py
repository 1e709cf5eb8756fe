"""Per-workgroup phase timing of one k_draw_lean launch at the bench shape (diagnostic; GPU box).

Loads the SD_PHASE_TIMING build (make -C speculative-decoding_amd timing) and draws 32 rows of
128256 bf16 (T = 1, Philox) — the bench's drafter draw — and prints, for the producer spans and
for the rows' last spans (the pollers), when they reach each phase, µs after the launch's first
start (s_memrealtime, 100 MHz).  Phases: 0 start, 1 loads landed (wave max), 2 span pick done,
3 record stored (producers), 4 poll done (last spans), 5 outputs written.
(An XCD-affine placement of a row's spans was measured slower and removed in round 5.)
"""
import os
import sys

os.environ["SPECDEC_LIB"] = "libspecdec_ts.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

B, V = int(os.environ.get("DRAW_ROWS", "32")), 128256
NSPAN = (V + 2047) // 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(B, V, device=dev, generator=g) * 3).to(torch.bfloat16)
noise = PhiloxNoise(seed=1)
stats = torch.empty(B, 2, device=dev)
ts = torch.zeros(16384 * 16, dtype=torch.int64, device=dev)
for _ in range(20):
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, noise, row_stats_out=stats)
torch.cuda.synchronize()
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
names = ["start", "loaded", "picked", "rec_stored", "poll_done", "written"]
warm = torch.randn(4096, 4096, device=dev)
agg = {}
for rep in range(6):
    ts.zero_()
    torch.cuda.synchronize()
    if rep % 2:   # keep the GPU busy right up to the draw (no idle gap before it)
        for _ in range(10):
            warm = warm @ warm
            warm = warm / warm.norm()
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, noise, row_stats_out=stats)
    torch.cuda.synchronize()
    t = ts.view(-1, 16).cpu().numpy().astype(np.int64)[:B * NSPAN]
    t0 = t[t[:, 0] > 0, 0].min()
    last = np.zeros(B * NSPAN, dtype=bool)
    last[NSPAN - 1::NSPAN] = True
    print(f"--- rep {rep} ({'busy' if rep % 2 else 'idle'} before)")
    for who, sel in (("producers", ~last), ("last spans", last)):
        blk = t[sel]
        print(f" {who}: {len(blk)}")
        for k, name in enumerate(names):
            v = blk[:, k]
            v = v[v > 0]
            if len(v):
                d = (v - t0) / 100.0
                print(f"  {name:10s} n={len(v):5d}  min {d.min():6.2f}  p50 {np.median(d):6.2f}  max {d.max():6.2f} us")
                agg.setdefault((who, name), []).append(float(np.median(d)))
print("median of per-rep medians:", {f"{w}/{n}": round(float(np.median(v)), 2) for (w, n), v in agg.items()})
