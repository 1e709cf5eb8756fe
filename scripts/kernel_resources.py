"""VGPR / SGPR / LDS / scratch of the library's gfx950 kernels (code-object notes), optionally
filtered by a substring: python scripts/kernel_resources.py [lib.so] [filter]"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests")]
from test_lib_cpu import kernel_notes  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else os.path.join(ROOT, "speculative-decoding_amd", "specdec_amd", "libspecdec.so")
flt = sys.argv[2] if len(sys.argv) > 2 else ""
notes = kernel_notes(lib, "/opt/rocm/lib/llvm/bin")
for blk in notes.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s*(\S+)", blk).group(1)
    if flt not in name:
        continue
    g = lambda k: (re.search(rf"\.{k}:\s*(\d+)", blk) or [None, "?"])[1]
    print(f"{g('vgpr_count'):>4} vgpr {g('sgpr_count'):>4} sgpr {g('group_segment_fixed_size'):>6} lds "
          f"{g('private_segment_fixed_size'):>4} scratch  {name}")
