"""Per-workgroup phase timing of one perf-mode drafter draw (k_draw) at the bench shape
(R = 32 rows, V = 128256 bf16, Philox).  Diagnostic; needs the SD_PHASE_TIMING build
(make -C speculative-decoding_amd timing).  Prints when workgroups reach each phase, in µs
from the launch's first workgroup start (s_memrealtime, 100 MHz)."""
import os
import sys

os.environ["SPECDEC_LIB"] = "libspecdec_ts.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

R, V = int(os.environ.get("R", 32)), 128256
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(R, V, device=dev, generator=g) * 3).to(torch.bfloat16)
stats = torch.empty(R, 2, device=dev)
noise = PhiloxNoise(seed=1)
ts = torch.zeros(16384 * 16, dtype=torch.int64, device=dev)
for _ in range(20):
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, noise, row_stats_out=stats)
torch.cuda.synchronize()
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
warm = torch.randn(8192, 8192, device=dev)
phases = ["start", "y_ready", "picked", "arrived", "tail_staged", "tail_picked", "written", "exps_done", "cand_shared"]
for rep in range(3):
    ts.zero_()
    torch.cuda.synchronize()
    if rep == 2:   # GPU busy right up to the draw
        for _ in range(20):
            warm = warm @ warm
            warm = warm / warm.norm()
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, noise, row_stats_out=stats)
    torch.cuda.synchronize()
    t = ts.view(-1, 16).cpu().numpy().astype(np.int64)[:8192]
    if os.environ.get("TS_DUMP"):
        np.save(os.path.join(ROOT, "gpurun_out", f"draw_ts_rep{rep}.npy"), t)
    blk = t[t[:, 0] > 0]
    t0 = blk[:, 0].min()
    print(f"--- rep {rep}: {len(blk)} workgroups")
    for k, ph in enumerate(phases):
        v = blk[:, k]
        v = v[v > 0]
        if len(v):
            d = (v - t0) / 100.0
            print(f"  {ph:12s} n={len(v):5d}  min {d.min():7.2f}  p50 {np.median(d):7.2f}  max {d.max():7.2f} us")
