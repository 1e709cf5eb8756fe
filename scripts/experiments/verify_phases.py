"""Per-workgroup phase timeline of the one-launch verify (k_verify) at the bench shape (diagnostic,
GPU box; needs `make -C speculative-decoding_amd timing`).  Phases (µs after the kernel's first
workgroup start): 0 start, 1 stream end, 2 stats arrival, 3 decided (last arrival only),
6 decision known, 7 sampling chunks done, 8 sample arrival, 9 finish done (finish tail only)."""
import os
import sys

os.environ["SPECDEC_LIB"] = "libspecdec_ts.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

B, G, V = int(os.environ.get("B", 32)), 4, 128256
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
tl = (torch.randn(B, G, V, device=dev, generator=g) * 3).to(torch.bfloat16)
dl = (tl.float() + torch.randn(B, G, V, device=dev, generator=g)).to(torch.bfloat16)
ids = dl.float().argmax(-1)
noise = PhiloxNoise(seed=1)
dstats = torch.empty(G, B, 2, device=dev)
for d in range(G):
    ops.sample_rows(dl[:, d], ops.PLAIN_SOFTMAX, noise, row_stats_out=dstats[d])
ts = torch.zeros(16384 * 16, dtype=torch.int64, device=dev)


def step():
    return ops.verify([tl[:, t] for t in range(G)], [dl[:, t] for t in range(G)], ids, _lib.SD_RULE_ENGINE,
                      ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise, torch.tensor([], dtype=torch.long, device=dev),
                      draft_row_stats=dstats)


for _ in range(20):
    step()
torch.cuda.synchronize()
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
warm = torch.randn(8192, 8192, device=dev)
for rep in range(3):
    ts.zero_()
    torch.cuda.synchronize()
    for _ in range(20):
        warm = warm @ warm
        warm = warm / warm.norm()
    step()
    torch.cuda.synchronize()
    t = ts.view(-1, 16).cpu().numpy().astype(np.int64)
    wg = t[:8192]
    live = wg[:, 0] > 0
    t0 = wg[live, 0].min()
    print(f"--- rep {rep}: {live.sum()} workgroups")
    for ph, name in ((0, "start"), (1, "stream_end"), (2, "stats_arrived"), (3, "decided"), (6, "decision_known"), (10, "weights_done"),
                     (7, "chunks_done"), (8, "sample_arrived"), (9, "finish_done")):
        v = wg[live, ph]
        v = v[v > 0]
        if v.size:
            us = (v - t0) / 100.0
            print(f"  {name:15s} n={v.size:4d} min {us.min():6.2f} p50 {np.median(us):6.2f} max {us.max():6.2f}")
    fin = t[16384 - B:16384, 0]
    fin = fin[fin > 0]
    if fin.size:
        print(f"  finish_start    n={fin.size} min {(fin.min()-t0)/100:6.2f} max {(fin.max()-t0)/100:6.2f}")
