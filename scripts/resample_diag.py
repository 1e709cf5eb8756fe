"""Diagnostic timing of one verify step with parts of k_resample disabled (SD_DIAG bits):
1 = skip the fused decide prologue, 2 = skip the residual body.  Tuning aid only."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "speculative-decoding_amd"))
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

B, g, V = 32, 4, 128256
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(0)
tl = (torch.randn(B, g, V, generator=gen, device=dev) * 3).to(torch.bfloat16)
dl = (tl.float() + torch.randn(B, g, V, generator=gen, device=dev)).to(torch.bfloat16)
draft = torch.randint(0, V, (B, g), device=dev)
noise = PhiloxNoise(seed=1)


def step():
    ops.verify([tl[:, t] for t in range(g)], [dl[:, t] for t in range(g)], draft, _lib.SD_RULE_ENGINE,
               ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise)


for diag in ["0", "2", "1", "3"]:
    os.environ["SD_DIAG"] = diag
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(20):
            step()
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        gr.replay()
    e.record()
    torch.cuda.synchronize()
    print(f"SD_DIAG={diag}: {s.elapsed_time(e) / 200 * 1e3:.1f} us per verify step", flush=True)
