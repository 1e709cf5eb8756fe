"""Phase timing of the STREAM (bit-exact) draw's k_rowsample and the verify's k_walk (diagnostic;
GPU box, the SD_PHASE_TIMING build: make -C speculative-decoding_amd timing).  Bench shape: 32
rows of 128256 bf16.  k_rowsample phases: 0 start, 1 logits + words + row stats in, 2 probabilities,
3 race done; k_walk (slot 8000): 0 start, 1 windows loaded, 2 chain walked, 3 decisions published.
µs after the kernel's first start (s_memrealtime, 100 MHz)."""
import os
import sys

os.environ.setdefault("SPECDEC_LIB", "libspecdec_ts.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import EngineStep, engine_logits  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import StreamNoise  # noqa: E402

dev = torch.device("cuda", 0)
B, g, V = 32, 4, 128256
tl, dl = engine_logits(B, g, V, 1.0, 1000, dev)
noise = StreamNoise(torch.Generator().manual_seed(1234))
step = EngineStep(tl, dl, noise, 0, ops, _lib)
ts = torch.zeros(16384 * 16, dtype=torch.int64, device=dev)


def show(name, t, phases):
    t = t[t[:, 0] > 0]
    if not len(t):
        return
    t0 = t[:, 0].min()
    print(f" {name}: {len(t)} workgroups")
    for k, ph in enumerate(phases):
        v = t[:, k]
        v = v[v > 0]
        if len(v):
            d = (v - t0) / 100.0
            print(f"  {ph:10s} n={len(v):5d}  min {d.min():7.2f}  p50 {np.median(d):7.2f}  max {d.max():7.2f} us")


with noise.session():
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    os.environ["SD_TS_PTR"] = str(ts.data_ptr())
    for rep in range(3):
        step.reserve()
        ts.zero_()
        torch.cuda.synchronize()
        step.draw(0)                      # the STREAM draw: k_stats, k_rowsample, k_sample_finalize
        torch.cuda.synchronize()
        t = ts.view(-1, 16).cpu().numpy().astype(np.int64)
        print(f"--- rep {rep}")
        show("k_rowsample", t[:B * 63], ["start", "loaded", "probs", "raced"])
        for d in range(1, g):
            step.draw(d)
        ts.zero_()
        torch.cuda.synchronize()
        step.verify()
        torch.cuda.synchronize()
        t = ts.view(-1, 16).cpu().numpy().astype(np.int64)
        show("k_walk", t[8000:8001], ["start", "loaded", "chained", "published"])
