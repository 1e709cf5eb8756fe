"""Debug: k_draw_lean vs k_draw (SD_DRAW_NO_LEAN) token_prob on a peaked V=8192 row (GPU box)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402
from oracle import specdec_ref as ref  # noqa: E402
from test_gpu_draw import peaked_logits  # noqa: E402

V, R = 8192, 4096
row = peaked_logits(V, 40, 3).to(torch.bfloat16)
logits = row.view(1, V).expand(R, V).contiguous().cuda()
probs = ref.process(row, ref.Processor("multinomial", 1.0), exact=True).double()
stats = torch.empty(R, 2, device="cuda")
tok, prob, st = ops.sample_rows(logits, ops.PLAIN_SOFTMAX, PhiloxNoise(seed=31337), want_prob=True, row_stats_out=stats)
t = tok.cpu()
want = probs[t].float()
got = prob.cpu()
bad = (~torch.isclose(got, want, rtol=1e-2, atol=0)).nonzero().flatten()
print("lean" if not os.environ.get("SD_DRAW_NO_LEAN") else "old", "bad rows", len(bad))
for b in bad[:10].tolist():
    print(b, int(t[b]), float(got[b]), float(want[b]), stats[b].tolist(), hex(int(st[b])))
x = row.float()
M = float(x.max()); S = float(torch.exp(x - M).sum())
print("true M S", M, S)
