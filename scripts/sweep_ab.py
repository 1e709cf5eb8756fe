#!/usr/bin/env python3
"""A/B of the large-batch engine step (bench.py's sweep) under dispatch options.

    python scripts/sweep_ab.py 128,512 "" "FUSED_TICKET=0" "DRAW_SPAN=1" ...

Each argument after the batch list is one configuration: comma-separated NAME=VALUE pairs for
sd_set_option ("" = the defaults).  Prints one JSON line per (configuration, batch)."""
import json
import os
import sys
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "speculative-decoding_amd"))
import bench  # noqa: E402


def main():
    batches = [int(x) for x in sys.argv[1].split(",")]
    confs = sys.argv[2:] or [""]
    from specdec_amd import _lib, ops
    from specdec_amd.noise import PhiloxNoise
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(gamma=4, vocab=128256, sigma=1.0, sweep_batches=batches)
    for conf in confs:
        olds = []
        for kv in filter(None, conf.split(",")):
            k, v = kv.split("=")
            o = getattr(_lib, f"SD_OPT_{k.upper()}")
            olds.append((o, _lib.get_option(o)))
            _lib.set_option(o, int(v))
        res = bench.sweep_lines(args, ops, _lib, PhiloxNoise, bench.EngineStep, dev)
        for k, r in res.items():
            print(json.dumps({"conf": conf, "batch": r["rows"], "path": r["verify_path"],
                              "ms_per_step": round(r["ms_per_step"], 5), "verify_ms": round(r["verify_ms"], 5),
                              "draw_ms": round(r["draw_ms"], 5), "frac": round(r["frac"], 4),
                              "frac_traffic": round(r["frac_traffic"], 4)}), flush=True)
        for o, v in olds:
            _lib.set_option(o, v)


if __name__ == "__main__":
    main()
