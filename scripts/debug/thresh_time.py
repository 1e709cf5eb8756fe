"""Diagnostic (GPU box): time sd_probs (threshold + stats + probs) on one / nine bf16 rows per
processor kind, to isolate the threshold kernel's cost."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]
import torch  # noqa: E402

from specdec_amd import ops  # noqa: E402

V = 128256
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(9, V, device="cuda", generator=g) * 3).to(torch.bfloat16)
for name, spec in (("multinomial", ops.ProcSpec("multinomial")), ("topk50", ops.ProcSpec("topk", 1.0, 50)),
                   ("nucleus0.9", ops.ProcSpec("nucleus", 1.0, 0, 0.9)),
                   ("topk50+nucleus0.9", ops.ProcSpec("topknucleus", 1.0, 50, 0.9))):
    for R in (1, 9):
        rows = x[:R]
        for _ in range(3):
            ops.probs_rows(rows, spec)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            ops.probs_rows(rows, spec)
        b.record()
        torch.cuda.synchronize()
        print(f"{name:20s} rows={R}: {a.elapsed_time(b) / 20 * 1e3:8.1f} us per sd_probs", flush=True)
