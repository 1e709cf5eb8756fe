"""Tuning sweep for the row-statistics pass (k_stats) on the bench workload: stage counts per
workgroup, against reference streaming kernels on the same bytes.  Prints GB/s per variant."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speculative-decoding_amd"))
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

B, g, V = int(os.environ.get("B", 32)), 4, 128256
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(0)
tl = (torch.randn(B, g, V, generator=gen, device=dev) * 3).to(torch.bfloat16)
dl = (tl.float() + torch.randn(B, g, V, generator=gen, device=dev)).to(torch.bfloat16)
draft = torch.randint(0, V, (B, g), device=dev)
noise = PhiloxNoise(seed=1)
alg = B * 2 * g * V * 2


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def stats_ms(n=50):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(); b.record()
        ops.verify([tl[:, t] for t in range(g)], [dl[:, t] for t in range(g)], draft, _lib.SD_RULE_ENGINE,
                   ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise, prof_events=(a, b))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev[5:]) / (n - 5)


for st in ["auto", "1", "2", "4", "8", "16"]:
    if st == "auto":
        os.environ.pop("SD_STATS_STAGES", None)
    else:
        os.environ["SD_STATS_STAGES"] = st
    ms = stats_ms()
    print(f"k_stats stages={st:>4}: {ms*1e3:7.1f} us  {alg/ms/1e6:7.0f} GB/s", flush=True)
os.environ.pop("SD_STATS_STAGES", None)
both = torch.stack([tl, dl])
buf = torch.empty_like(both)
ms = timed(lambda: buf.copy_(both))
print(f"torch copy (read+write {2*alg/1e6:.0f} MB): {ms*1e3:.1f} us  {2*alg/ms/1e6:.0f} GB/s")
ms = timed(lambda: both.sum(dtype=torch.float32))
print(f"torch sum (read {alg/1e6:.0f} MB): {ms*1e3:.1f} us  {alg/ms/1e6:.0f} GB/s")
big = torch.empty(512 * 2**20 // 2, dtype=torch.bfloat16, device=dev).normal_()
ms = timed(lambda: big.sum(dtype=torch.float32), 20)
print(f"torch sum 512 MiB (beyond MALL): {ms*1e3:.1f} us  {big.numel()*2/ms/1e6:.0f} GB/s")
ms = timed(lambda: ops.verify([tl[:, t] for t in range(g)], [dl[:, t] for t in range(g)], draft,
                              _lib.SD_RULE_ENGINE, ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise))
print(f"full verify step (eager, incl. host launch): {ms*1e3:.1f} us")
