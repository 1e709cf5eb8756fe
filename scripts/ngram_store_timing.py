"""Device n-gram store vs the host drafter (reference semantics) — GPU box diagnostic.

(1) initialize of B prompts x L tokens (NGramStorage n=3 and OneLevel n=3), (2) the batch-1 loop
pattern: one update + one next_token per call pair.  Device times include the H2D copy of the
histories and a final synchronize; host times are the Python dict store (specdec_amd's mirror of
ngram_assisted/ngram_storage.py, which equals the oracle)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd")]
import torch  # noqa: E402

from specdec_amd.ngram_assisted import (DeviceNGramStorage, DeviceOneLevelNGramStorage,  # noqa: E402
                                        NGramStorage, OneLevelNGramStorage)

V = 128256
res = {}
g = torch.Generator().manual_seed(0)
for B, L in ((1, 4096), (32, 2048)):
    ids = torch.randint(0, 2000, (B, L), generator=g)   # 2000 distinct ids: repeated grams
    for name, dev_cls, host_cls in (("multi_n3", DeviceNGramStorage, NGramStorage),
                                    ("one_n3", DeviceOneLevelNGramStorage, OneLevelNGramStorage)):
        d = dev_cls(3, V, device="cuda", gram_capacity=1 << 22, pair_capacity=1 << 22)
        d.initialize(ids)   # warm-up: module load, first-touch of the tables
        torch.cuda.synchronize()
        d.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.initialize(ids)
        torch.cuda.synchronize()
        t_dev = time.perf_counter() - t0
        h = host_cls(3, V)
        t0 = time.perf_counter()
        h.initialize(ids)
        t_host = time.perf_counter() - t0
        # agreement on every history's last position
        torch.manual_seed(0)
        a = d.next_token(ids)
        torch.manual_seed(0)
        b = h.next_token(ids)
        same = a[0].cpu().tolist() == b[0].tolist() and a[1].cpu().tolist() == b[1].tolist()
        res[f"initialize_{name}_B{B}_L{L}"] = {"device_ms": t_dev * 1e3, "host_ms": t_host * 1e3,
                                               "records": B * L, "agree": same, "status": d.status()}
# batch-1 loop pattern: update(history, [x]) then next_token(history + [x]), 200 times
hist = torch.randint(0, 2000, (1, 512), generator=g)
for name, obj in (("device", DeviceNGramStorage(3, V, device="cuda")), ("host", NGramStorage(3, V))):
    obj.initialize(hist)
    seq = hist
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        x = torch.tensor([[i % 2000]])
        obj.update(seq, x)
        seq = torch.cat([seq, x], 1)
        tok, known = obj.next_token(seq)
        int(tok[0])   # the loop reads the draft on the host
    torch.cuda.synchronize()
    res[f"loop_step_{name}_us"] = (time.perf_counter() - t0) / 200 * 1e6
# the n-gram loop's drafting step (configs[4]: gamma = 8): one update, then gamma chained lookups
# read back on the host -- the host store calls next_token 8 times, the device store drafts the
# chain in one launch (draft_chain)
G = 8
for name, obj in (("device", DeviceNGramStorage(3, V, device="cuda")), ("host", NGramStorage(3, V))):
    obj.initialize(hist)
    seq = hist
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        x = torch.tensor([[i % 2000]])
        obj.update(seq, x)
        seq = torch.cat([seq, x], 1)
        if name == "device":
            toks = obj.draft_chain(seq, G)[0][0].tolist()
        else:
            s = seq[0].tolist()
            for k in range(G):
                tok, known = obj.next_token(torch.tensor([s]))
                s.append(int(tok[0]))
    torch.cuda.synchronize()
    res[f"draft_step_g{G}_{name}_us"] = (time.perf_counter() - t0) / 200 * 1e6
print(json.dumps(res, indent=1))
