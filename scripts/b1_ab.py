"""configs[1] batch-1 step times (bench.configs1_lines: γ=4 draws + verify, hipGraph replays) under
dispatch-option A/B settings (sd_set_option, applied at capture time; GPU box):

    python scripts/b1_ab.py "" "LEAN_VERIFY=0" ...
Each argument is a space-separated list of OPTION=value pairs ("" = defaults); prints one JSON line each.
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
        o = getattr(_lib, f"SD_OPT_{k.upper()}")
        saved[o] = _lib.get_option(o)
        _lib.set_option(o, int(v))
    res = {}
    for rep in range(2):
        r = bench.configs1_lines(dev, args, ops, _lib, PhiloxNoise)
        for name, d in r.items():
            res.setdefault(name, []).append(round(d["us_per_step"], 2))
    print(json.dumps({"env": spec, "us_per_step": res}), flush=True)
    for o, v in saved.items():
        _lib.set_option(o, v)
