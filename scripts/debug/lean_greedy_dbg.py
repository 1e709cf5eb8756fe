"""Debug: the greedy verify of tests/test_gpu_perfmode.py::test_perf_greedy_is_bit_exact (seed 0)
through the lean kernel and the two-launch path; prints both outputs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]
import torch  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

for seed, (B, V, dtype) in enumerate([(8, 4096, torch.bfloat16), (4, 128256, torch.bfloat16)]):
    g = 4
    gen = torch.Generator().manual_seed(31 + seed)
    tl = (torch.randn(B, g + 1, V, generator=gen) * 3).to(dtype)
    gen = torch.Generator().manual_seed(41 + seed)
    dl = (tl[:, :g].float() + torch.randn(B, g, V, generator=gen) * 2).to(dtype)
    ids = dl.float().argmax(-1)
    ids[:, -1] = torch.randint(0, V, (B,), generator=torch.Generator().manual_seed(seed))
    tl, dl, ids = tl.cuda(), dl.cuda(), ids.cuda()
    proc = ops.ProcSpec("greedy")
    for lean in ("1", "0"):
        os.environ["SD_LEAN_VERIFY"] = lean
        out = ops.verify([tl[:, t] for t in range(g + 1)], [dl[:, d] for d in range(g)], ids, _lib.SD_RULE_SPEC,
                         proc, proc, PhiloxNoise(seed=5), torch.tensor([], dtype=torch.long, device="cuda"))
        torch.cuda.synchronize()
        print(seed, "lean" if lean == "1" else "2lau", out.n_accepted.tolist(), out.next_token.tolist(),
              [hex(x) for x in out.row_status.tolist()], [round(x, 5) for x in out.resample_mass.tolist()], flush=True)
