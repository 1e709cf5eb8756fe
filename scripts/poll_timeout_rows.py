"""Which rows does a fused verify write when every in-launch poll gives up at once (spin limit < 0)?
(diagnostic; GPU box)  The output buffer is pre-filled with a sentinel (-7): a row still holding it
after the call was never written.  Prints, per call, the rows whose outputs differ from a normal
call's and whether they carry the timeout flag."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from specdec_amd import _lib, get_poll_policy, ops, set_poll_policy  # noqa: E402
from test_gpu_fused import inputs, run, fused  # noqa: E402

orig = ops._verify_outputs


def sentinel_outputs(B, dev):
    out = orig(B, dev)
    for f in ("n_accepted", "next_token", "prune_drafter", "prune_target", "stop_index", "row_status"):
        getattr(out, f).fill_(-7)
    out.resample_mass.fill_(-7.0)
    return out


ops._verify_outputs = sentinel_outputs
spec = ops.ProcSpec("multinomial", 1.0)
for B in (32, 128):
    tl, dl = inputs(B, 4, 128256, "engine", 5)
    old = get_poll_policy()
    with fused(1):
        ref = run(tl, dl, "engine", spec, 5)
        for rep in range(3):
            set_poll_policy(True, -1)
            try:
                a = run(tl, dl, "engine", spec, 5)
            finally:
                set_poll_policy(*old)
            st = a["row_status"]
            unwritten = (st == -7).nonzero().flatten().tolist()
            flagged = ((st & _lib.SD_ROW_EXCHANGE_TIMEOUT) != 0) & (st != -7)
            clean = (~flagged) & (st != -7)
            diff = [int(r) for r in clean.nonzero().flatten()
                    if int(a["n_accepted"][r]) != int(ref["n_accepted"][r]) or
                    int(a["next_token"][r]) != int(ref["next_token"][r])]
            print(f"B={B} rep={rep} path={_lib.PATH_NAMES.get(int(a['path']))}: flagged {int(flagged.sum())}, "
                  f"clean {int(clean.sum())}, unwritten {unwritten}, clean rows differing from the normal call {diff}")
            for r in diff[:4]:
                print(f"   row {r}: status {int(st[r])} n_acc {int(a['n_accepted'][r])} (normal {int(ref['n_accepted'][r])}) "
                      f"next {int(a['next_token'][r])} (normal {int(ref['next_token'][r])})")
            b = run(tl, dl, "engine", spec, 5)
            assert torch.equal(b["n_accepted"], ref["n_accepted"]) and torch.equal(b["next_token"], ref["next_token"])
