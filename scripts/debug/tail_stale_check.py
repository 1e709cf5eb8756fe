"""Debug: do last-arrival tails read stale partials?  Back-to-back sample_rows calls alternate
between two different logits sets (R rows each); every call's row stats must equal the truth of
the set it was given (GPU box)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]
import torch  # noqa: E402
from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

V, R = int(os.environ.get("V", 128256)), int(os.environ.get("R", 32))
g = torch.Generator(device="cuda").manual_seed(5)
sets = [(torch.randn(R, V, device="cuda", generator=g) * s).to(torch.bfloat16) for s in (3.0, 1.0)]
truth = []
for x in sets:
    xf = x.float()
    M = xf.max(-1).values
    truth.append((M, torch.exp(xf - M[:, None]).sum(-1)))
noise = PhiloxNoise(seed=3)
stats = [torch.empty(R, 2, device="cuda") for _ in range(40)]
for i in range(40):   # no host sync between calls
    ops.sample_rows(sets[i % 2], ops.PLAIN_SOFTMAX, noise, row_stats_out=stats[i])
torch.cuda.synchronize()
bad = 0
for i in range(40):
    M, S = truth[i % 2]
    okm = torch.isclose(stats[i][:, 0], M)
    oks = torch.isclose(stats[i][:, 1], S, rtol=1e-4)
    bad += int((~(okm & oks)).sum())
print(os.environ.get("TAG", ""), f"V={V} R={R}: bad row-stats {bad} of {40 * R}")
