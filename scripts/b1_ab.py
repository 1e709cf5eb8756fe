"""configs[1] batch-1 step times (bench.configs1_lines: γ=4 draws + verify, hipGraph replays) under
environment A/B settings read at capture time (GPU box):

    python scripts/b1_ab.py "SD_STATS_STAGES=8" "SD_STATS_STAGES=1" ...
Each argument is a space-separated list of VAR=value pairs ("" = defaults); prints one JSON line each.
"""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

dev = torch.device("cuda", 0)
args = SimpleNamespace(gamma=4, vocab=128256, sigma=1.0)
for spec in sys.argv[1:] or [""]:
    saved = {}
    for kv in spec.split():
        k, v = kv.split("=", 1)
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    res = {}
    for rep in range(2):
        r = bench.configs1_lines(dev, args, ops, _lib, PhiloxNoise)
        for name, d in r.items():
            res.setdefault(name, []).append(round(d["us_per_step"], 2))
    print(json.dumps({"env": spec, "us_per_step": res}), flush=True)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
