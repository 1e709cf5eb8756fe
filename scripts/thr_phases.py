"""Per-workgroup phase timing of a configs[1] nucleus-0.9 drafter draw, one row of 128256 bf16
(diagnostic; GPU box, the SD_PHASE_TIMING build: make -C speculative-decoding_amd timing):
the threshold search (k_thr_hist, poll mode; the draw asks for row stats, so the threshold + k_draw
path runs) or, with THR_NUC=1, the rejection draw (k_draw_nuc).  THR_ROWS sets the row count.
Prints when the row's slice workgroups reach each phase, µs after the first start
(s_memrealtime, 100 MHz)."""
import os
import sys

os.environ.setdefault("SPECDEC_LIB", "libspecdec_ts.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

V = 128256
R = int(os.environ.get("THR_ROWS", "1"))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(R, V, device=dev, generator=g) * 3).to(torch.bfloat16)
proc = ops.ProcSpec("nucleus", 1.0, 0, 0.9)
NUC = os.environ.get("THR_NUC") == "1"   # the rejection draw (k_draw_nuc) instead of the threshold
noise = PhiloxNoise(seed=1)
ts = torch.zeros(16384 * 16, dtype=torch.int64, device=dev)
want = None if NUC else torch.empty(R, 2, device=dev)   # row stats: the threshold + k_draw path
for _ in range(20):
    ops.sample_rows(x, proc, noise, row_stats_out=want)
torch.cuda.synchronize()
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
PH = {0: "start", 1: "max_pub", 2: "loc_hist", 3: "max_exch", 4: "tail", 5: "tail_sync", 6: "flushed",
      7: "arrived", 8: "hist_read", 9: "norm_scan", 10: "mass_scan", 11: "decided", 12: "decision", 13: "tie_rec",
      14: "keep_out"}
if NUC:
    PH = {0: "start", 1: "max", 2: "s1+prefix", 3: "picks", 7: "B_polled", 4: "B_recs", 5: "C_sums", 8: "D_polled",
          6: "D_recs"}
for rep in range(4):
    ts.zero_()
    torch.cuda.synchronize()
    ops.sample_rows(x, proc, noise, row_stats_out=want)
    torch.cuda.synchronize()
    base = 15000 if NUC else 14000
    t = ts.view(-1, 16).cpu().numpy().astype(np.int64)[base:base + 64 * R]
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    print(f"--- rep {rep}: {len(t)} workgroups")
    for k, name in PH.items():
        v = t[:, k]
        v = v[v > 0]
        if len(v):
            d = (v - t0) / 100.0
            print(f"  {name:10s} n={len(v):3d}  min {d.min():6.2f}  p50 {np.median(d):6.2f}  max {d.max():6.2f} us")
