"""STREAM-mode engine step (bench.py's stream line) repeated for a rocprofv3 kernel-trace summary
(GPU box): γ drafter draws + verify on the bench shape with torch-generator noise made on the GPU."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import torch  # noqa: E402

from bench import EngineStep, engine_logits  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import StreamNoise  # noqa: E402

dev = torch.device("cuda", 0)
B, g, V = int(os.environ.get("B", 32)), 4, 128256
tl, dl = engine_logits(B, g, V, 1.0, 1000, dev)
noise = StreamNoise(torch.Generator().manual_seed(1234))
step = EngineStep(tl, dl, noise, 0, ops, _lib)
with noise.session():
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = int(os.environ.get("STEPS", 20))
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    from specdec_amd import noise as nz
    print(f"STREAM engine step B={B} stride={nz.mt_stride(step.g * 2 * B * V + B * (step.g + 2 * V))}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms")
