"""configs[1]'s batch-1 step pieces run eagerly in a loop, for rocprofv3 kernel traces and PMC
counters (GPU box): γ=4 drafter draws (sd_sample) + one SPEC-rule sd_verify over 5 target rows,
Llama-3 shaped bf16 rows, Philox noise.  PROC=greedy|multinomial (default multinomial)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import torch  # noqa: E402

from bench import engine_logits  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

dev = torch.device("cuda", 0)
g, V = 4, 128256
tl, dl = engine_logits(1, g + 1, V, 1.0, 11, dev)
dl = dl[:, :g].contiguous()
stops = torch.tensor([128001, 128009], dtype=torch.long, device=dev)
proc = ops.ProcSpec(os.environ.get("PROC", "multinomial"), 1.0) if os.environ.get("PROC") != "greedy" else ops.ProcSpec("greedy")
noise = PhiloxNoise(seed=7, offset_dev=torch.zeros(1, dtype=torch.long, device=dev))
draft = torch.zeros(1, g, dtype=torch.long, device=dev)
dstats = torch.empty(g, 1, 2, dtype=torch.float32, device=dev)
for _ in range(int(os.environ.get("STEPS", 50))):
    for d in range(g):
        ops.sample_rows(dl[:, d], proc, noise, tokens_out=draft[:, d], row_stats_out=dstats[d])
    ops.verify([tl[:, t] for t in range(g + 1)], [dl[:, t] for t in range(g)], draft, _lib.SD_RULE_SPEC, proc, proc,
               noise, stops, draft_row_stats=dstats)
torch.cuda.synchronize()
print("done")
