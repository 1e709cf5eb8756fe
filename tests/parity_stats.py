"""Counters the GPU parity tests fill and conftest's terminal summary prints (so the counts show
in a `pytest -q` log): torch-CPU rounding divergences, nucleus tie-order divergences, and the
nucleus rows the kernels flagged SD_ROW_NUCLEUS_INEXACT with the oracle each one matched."""
from collections import Counter

DIVERGENCES = []            # HIP matched the exact-arithmetic oracle, not torch-CPU's rounding
TIE_DIVERGENCES = []        # HIP matched the stable-ties oracle (torch's sort order among equals)
NUCLEUS_ROWS = Counter()    # "checked" / "inexact" / "inexact=<oracle label>"
DRAW_CLOSE_CALLS = []       # perf-mode decisions that differ only inside fp32 rounding


def summary_lines():
    if not (DIVERGENCES or TIE_DIVERGENCES or NUCLEUS_ROWS or DRAW_CLOSE_CALLS):
        return []
    inexact = {k.split("=", 1)[1]: v for k, v in NUCLEUS_ROWS.items() if k.startswith("inexact=")}
    variants = {k.split("=", 1)[1]: v for k, v in sorted(NUCLEUS_ROWS.items()) if k.startswith("variant=")}
    return [
        f"torch-CPU rounding divergences: {len(DIVERGENCES)} (each equal to the exact oracle) {DIVERGENCES[:8]}",
        f"nucleus tie-order divergences: {len(TIE_DIVERGENCES)}",
        f"nucleus rows checked: {NUCLEUS_ROWS['checked']}, flagged INEXACT: {NUCLEUS_ROWS['inexact']}, "
        f"INEXACT rows by matching oracle: {inexact}",
        f"nucleus rows per processor variant: {variants}",
        f"perf-mode close calls (|u - p/q| within fp32 rounding): {len(DRAW_CLOSE_CALLS)} {DRAW_CLOSE_CALLS[:4]}",
    ]
