"""Device STREAM generator timing (GPU box): sd_mt19937_generate for one engine drafter draw's
words at several substream strides, HIP events on the launch stream.  Default n_words: one
bench-shape STREAM engine step's pool (4 drafter draws + verify at B = 32, V = 128256).

    STRIDES=131072,196608 python scripts/mt_timing.py [n_words]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import torch  # noqa: E402

from specdec_amd import noise as nz  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 41042048
strides = [int(x) for x in os.environ.get("STRIDES", "131072,196608,262144,327680,393216").split(",")]
g = torch.Generator().manual_seed(1)
for stride in strides:
    nz.MT_STRIDE, nz._STRIDE_ENV = stride, str(stride)
    d = nz._DeviceMT("cuda", g.get_state())
    t0 = time.perf_counter()
    d.fill(n)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    for _ in range(3):
        d.fill(n)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    a.record()
    for _ in range(reps):
        d.fill(n)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(json.dumps({"n_words": n, "stride": stride, "substreams": (n + 624 + stride - 1) // stride,
                      "us_per_fill": ms * 1e3, "gwords_per_s": n / ms / 1e6, "first_call_s": first}), flush=True)
