"""Is the STREAM engine step (bench.py's stream line, eager in a noise session) bound by the host or
by the GPU?  Times N steps' enqueue on the host (no sync) against the same N steps end to end, and
the GPU's own time for them (events around the block)."""
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
B, g, V = 32, 4, 128256
tl, dl = engine_logits(B, g, V, 1.0, 1000, dev)
noise = StreamNoise(torch.Generator().manual_seed(1234))
step = EngineStep(tl, dl, noise, 0, ops, _lib)
N = int(os.environ.get("STEPS", 24))
with noise.session():
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for rep in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        for _ in range(N):
            step()
        b.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host enqueue {(t1 - t0) / N * 1e6:.1f} us/step, end to end {(t2 - t0) / N * 1e6:.1f} us/step, "
              f"GPU events {a.elapsed_time(b) / N * 1e3:.1f} us/step", flush=True)
