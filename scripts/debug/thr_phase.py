"""Diagnostic (GPU box, SD_PHASE_TIMING build): per-workgroup phase times of k_thr_hist for one
top-k / nucleus sd_sample row (µs from the kernel's first start).  The k_thr_tie and k_stats
launches that follow overwrite the same slots of workgroups they share, so only phases of
k_thr_hist's own workgroups are read, right after a call that has no later launch reaching them."""
import os
import sys

os.environ["SPECDEC_LIB"] = "libspecdec_ts.so"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]
import torch  # noqa: E402

ts = torch.zeros(16384 * 16, dtype=torch.int64, device="cuda")
os.environ["SD_TS_PTR"] = str(ts.data_ptr())
from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

V = 128256
x = (torch.randn(1, V, device="cuda", generator=torch.Generator(device="cuda").manual_seed(0)) * 3).to(torch.bfloat16)
names = ["start", "sliced", "flushed", "arrived", "tail_read", "tail_topk", "done"]
for spec in (ops.ProcSpec("topk", 1.0, 50), ops.ProcSpec("nucleus", 1.0, 0, 0.9)):
    for rep in range(3):
        ts.zero_()
        ops.sample_rows(x, spec, PhiloxNoise(seed=1))
        torch.cuda.synchronize()
        t = ts.view(16384, 16)[:16, :7].cpu().double()
        t0 = t[:, 0][t[:, 0] > 0].min()
        print(spec.kind, "rep", rep)
        for ph, nm in enumerate(names):
            col = t[:, ph]
            col = col[col > 0]
            if col.numel():
                v = (col - t0) / 100.0
                print(f"  {nm:10s} n={col.numel():3d} min {v.min():7.2f} med {v.median():7.2f} max {v.max():7.2f} us")
