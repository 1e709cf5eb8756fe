#!/bin/bash
# Register / LDS / spill usage of the perf-path kernels in the built gfx950 code object.
# usage: scripts/kres.sh [object]   (default: the in-tree build/specdec_kernels.o)
set -e
OBJ=${1:-$(dirname $0)/../speculative-decoding_amd/build/specdec_kernels.o}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin $OBJ
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c '
import sys, re
txt = sys.stdin.read()
for blk in txt.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not re.search(r"k_stats|k_draw|k_sample", name): continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    v, s_, l, vs, ss = (g(k) for k in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count"))
    print("%-60s vgpr %4s sgpr %4s lds %6s spill v%s s%s" % (name[:60], v, s_, l, vs, ss))
'
rm -rf $T
