"""k_draw launch time at the bench shape (R = 32 rows, V = 128256 bf16, Philox): 20 launches
between HIP events on the launch stream, median of 10 repeats.  SPECDEC_LIB picks the library
build (A/B of timing experiments: make variant NAME=x VFLAGS=...).  Diagnostic; GPU box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]

import torch  # noqa: E402

from specdec_amd import ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402

R, V = int(os.environ.get("R", 32)), int(os.environ.get("V", 128256))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(R, V, device=dev, generator=g) * 3).to(torch.bfloat16)
stats = torch.empty(R, 2, device=dev)
tok = torch.empty(R, dtype=torch.long, device=dev)
noise = PhiloxNoise(seed=1)
for _ in range(5):
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, noise, tokens_out=tok, row_stats_out=stats)
torch.cuda.synchronize()
# 20 launches captured in one hipGraph (eager launches are host-bound at ~11 us each)
graph = torch.cuda.CUDAGraph()
cs = torch.cuda.Stream()
cs.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(cs):
    with torch.cuda.graph(graph, stream=cs):
        for _ in range(20):
            ops.sample_rows(x, ops.PLAIN_SOFTMAX, noise, tokens_out=tok, row_stats_out=stats)
torch.cuda.current_stream().wait_stream(cs)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
for _ in range(5):
    graph.replay()
torch.cuda.synchronize()
res = []
for rep in range(15):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    graph.replay()
    b.record(s)
    b.synchronize()
    res.append(a.elapsed_time(b) / 20 * 1e3)
res.sort()
print(f"{os.environ.get('SPECDEC_LIB', 'libspecdec.so')}: k_draw {res[len(res) // 2]:.2f} us (min {res[0]:.2f}) "
      f"R={R} V={V}")
