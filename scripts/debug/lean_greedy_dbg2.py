"""Debug: tests/test_gpu_perfmode.py::test_perf_greedy_is_bit_exact's calls, printing every output
field, five repetitions each (GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT, os.path.join(ROOT, "tests")]
from types import SimpleNamespace  # noqa: E402
import torch  # noqa: E402
from specdec_amd import _lib, ops  # noqa: E402
from specdec_amd.noise import PhiloxNoise  # noqa: E402
import test_gpu_perfmode as T  # noqa: E402
from oracle import specdec_ref as ref  # noqa: E402

sd = SimpleNamespace(lib=_lib, ops=ops, PhiloxNoise=PhiloxNoise)
proc = ref.Processor("greedy")
for rep in range(5):
    for seed, (B, V, dtype) in enumerate([(8, 4096, torch.bfloat16), (4, 50257, torch.float32), (4, 128256, torch.bfloat16)]):
        g = 4
        tl = T.rand_logits((B, g + 1, V), dtype, 31 + seed)
        dl = (tl[:, :g].float() + T.rand_logits((B, g, V), torch.float32, 41 + seed, 2.0)).to(dtype)
        ids = dl.float().argmax(-1)
        ids[:, -1] = torch.randint(0, V, (B,), generator=torch.Generator().manual_seed(seed))
        out = T.verify(sd, tl.to("cuda"), dl.to("cuda"), ids.to("cuda"), _lib.SD_RULE_SPEC, proc, PhiloxNoise(seed=5))
        torch.cuda.synchronize()
        print(rep, seed, out.n_accepted.tolist(), out.next_token.tolist(), [hex(x) for x in out.row_status.tolist()],
              [round(x, 4) for x in out.resample_mass.tolist()], flush=True)
