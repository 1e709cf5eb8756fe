"""Diagnostic (GPU box): kept-set size of sd_probs under nucleus / top-k vs the exact oracle on the
parity-test rows of one seed; prints rows whose kept sets differ and the differing indices."""
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), os.path.join(ROOT, "tests"), ROOT]
import torch  # noqa: E402

from test_gpu_parity import KINDS, draft_case  # noqa: E402
from oracle import specdec_ref as ref  # noqa: E402
from specdec_amd import ops  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "nucleus09"
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 19
gamma = int(sys.argv[3]) if len(sys.argv) > 3 else 8
V = int(sys.argv[4]) if len(sys.argv) > 4 else 128256
proc = KINDS[kind]
tl, dl, ids = draft_case(1, gamma, V, torch.bfloat16, seed, proc)
pe = dataclasses.replace(proc, stable_ties=True)
spec = ops.ProcSpec(proc.kind, 1.0, proc.top_k, proc.top_p)   # keep set is T-independent
bad = 0
for name, rows in (("target", tl[0]), ("drafter", dl[0])):
    for r in range(rows.shape[0]):
        row = rows[r:r + 1]
        ke = ref.processed_logits(row, pe, exact=True)[0].float() > -1e19
        pg = ops.probs_rows(row.cuda(), spec)[0].float().cpu()
        kg = pg > 0
        # kept by the threshold but p rounded to 0 is possible: compare on the exact kept set's p > 0
        pe_ = ref.process(row, pe, exact=True)[0].float() > 0
        if not torch.equal(kg, pe_):
            bad += 1
            d = torch.nonzero(kg != pe_).flatten().tolist()
            x = row[0].float()
            print(name, r, "gpu", int(kg.sum()), "exact", int(pe_.sum()), "diff idx", d[:10],
                  "vals", [float(x[i]) for i in d[:10]])
print("rows differing:", bad)
