"""Which kernels the batch-1 (configs[1]) verify takes per processor: runs one bench-shaped step
and prints the library's own report (sd_last_verify_path / sd_last_sample_path)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]
import torch  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

dev = torch.device("cuda")
g, V = 4, 128256
gen = torch.Generator(device=dev).manual_seed(11)
tl = (torch.randn(1, g + 1, V, generator=gen, device=dev) * 3).to(torch.bfloat16)
dl = (tl[:, :g].float() + torch.randn(1, g, V, generator=gen, device=dev)).to(torch.bfloat16)
for name, proc in (("multinomial", ops.ProcSpec("multinomial", 1.0)), ("nucleus", ops.ProcSpec("nucleus", 1.0, 0, 0.9)),
                   ("topk", ops.ProcSpec("topk", 1.0, 50, 0.0))):
    noise = PhiloxNoise(seed=7)
    draft = torch.zeros(1, g, dtype=torch.long, device=dev)
    dstats = torch.empty(g, 1, 2, dtype=torch.float32, device=dev) if not proc.keeps else None
    for d in range(g):
        ops.sample_rows(dl[:, d], proc, noise, tokens_out=draft[:, d], row_stats_out=dstats[d] if dstats is not None else None)
    draw = _lib.PATH_NAMES.get(_lib.last_sample_path())
    ops.verify([tl[:, t] for t in range(g + 1)], [dl[:, t] for t in range(g)], draft, _lib.SD_RULE_SPEC, proc, proc,
               noise, torch.tensor([128001], device=dev), draft_row_stats=dstats)
    torch.cuda.synchronize()
    print(f"{name}: draws {draw}, verify {_lib.PATH_NAMES.get(_lib.last_verify_path())}", flush=True)
