import sys, torch
sys.path[:0] = ["tests", "speculative-decoding_amd", "."]
from specdec_amd import _lib, ops
from specdec_amd.noise import PhiloxNoise
from oracle import specdec_ref as ref
B, V = 8, 8192
g = torch.Generator().manual_seed(9)
t0 = (torch.randn(V, generator=g) * 2).to(torch.bfloat16)
p0 = ref.softmax(t0, True)
x = int(torch.argmax(p0.float()))
for scale in (1.0, 0.9):
    q0 = p0.float() * scale
    q0[x] = 2.0 * p0.float()[x]
    tl = t0.view(1, V).expand(B, V).contiguous().cuda()
    ql = q0.view(1, V).expand(B, V).contiguous().cuda()
    ids = torch.full((B, 1), x, dtype=torch.long, device="cuda")
    out = ops.verify([tl], [ql], ids, _lib.SD_RULE_ENGINE, ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, PhiloxNoise(seed=1),
                     torch.tensor([], dtype=torch.long, device="cuda"), draft_is_probs=True)
    torch.cuda.synchronize()
    print("scale", scale, "n", out.n_accepted.tolist(), "x", out.next_token.tolist(),
          "st", [hex(s) for s in out.row_status.tolist()], "mass", out.resample_mass.tolist())
    ws = next(w for (d, _), w in ops._WS.items() if d == torch.device("cuda", 0))
    # rowstat: after cnt (2*65536*4 B) and part (rows_total*nc float2): print the first floats of each region
    import numpy as np
    raw = ws.cpu().numpy()
    off = 2 * 65536 * 4
    nc = (V + 2047) // 2048
    rows_total = B * 3
    part_bytes = ((rows_total * nc * 8) + 255) & ~255
    rs = np.frombuffer(raw[off + part_bytes: off + part_bytes + 8 * B], dtype=np.float32)
    print("rowstat", rs.reshape(B, 2)[:2])
