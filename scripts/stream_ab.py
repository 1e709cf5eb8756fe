"""STREAM engine step time (bench.py's stream line: eager steps in a noise session, 32 rows of
128256 bf16, γ = 4) for library A/B runs (GPU box; SPECDEC_LIB picks the library).  Prints one
JSON line: ms per step over 3 repeats of 20 steps, and the tokens checksum (bit-exact runs of two
libraries must agree)."""
import json
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
res = []
for rep in range(3):
    noise = StreamNoise(torch.Generator().manual_seed(1234))
    step = EngineStep(tl, dl, noise, 0, ops, _lib)
    with noise.session():
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        step.read_counts()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c = step.read_counts()
    res.append(dt / 20 * 1e3)
print(json.dumps({"lib": os.environ.get("SPECDEC_LIB", "libspecdec.so"), "ms_per_step": [round(x, 4) for x in res],
                  "tokens": int(c[:, 1].sum()), "accepted": int(c[:, 0].sum())}), flush=True)
