"""Drop-in engine surface on the GPU:

* run_batch_speculative's non-timing request fields (prompt / generated / total tokens,
  acceptance rate) equal the reference's own run_batch_speculative on the same FakeLM banks and
  seed (tests/golden/engine_surface.json; STREAM noise = the reference's torch CPU draws), and
  the BatchMetrics feed BenchmarkResults.to_dict;
* the data-parallel runner (specdec_amd.engine.dp_runner): two processes (gloo, both on cuda:0 —
  the GPU box has one card) decoding row shards of one batch under Philox noise return exactly
  what one process decoding the whole batch returns, for two batches in a row (the call offsets
  are agreed after each); STREAM noise is refused; ranks sharing the card run with the
  library's in-launch polls switched off (the counter exchanges).
"""
import json
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.multiprocessing as mp

from fakelm import make_pair

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "engine_surface.json")) as f:
    GOLD = json.load(f)
DT = {"bf16": torch.bfloat16, "fp32": torch.float32}
DEV = "cuda"


@pytest.mark.parametrize("case", sorted(GOLD["run_batch_speculative"]))
def test_run_batch_speculative_fields_match_reference(case):
    from specdec_amd import set_noise_mode
    from specdec_amd.engine import metrics as em
    from specdec_amd.engine.infer_engine import run_batch_speculative
    c = GOLD["run_batch_speculative"][case]
    set_noise_mode("stream")
    target, drafter = make_pair(c["vocab"], dtype=DT[c["dtype"]], device=DEV, pos_mult=c["pos_mult"])
    ids = torch.tensor(c["prompt"], dtype=torch.long, device=DEV)
    mask = torch.tensor(c["mask"], dtype=torch.long, device=DEV)
    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=c["gamma"], gen_len=c["gen_len"],
                          end_tokens=c["end_tokens"])
    torch.manual_seed(c["seed"])
    bm = run_batch_speculative(ctx, ids, mask, c["batch"])
    assert bm is not None
    got = [dict(prompt_tokens=r.prompt_tokens, generated_tokens=r.generated_tokens, total_tokens=r.total_tokens,
                acceptance_rate=r.acceptance_rate) for r in bm.requests]
    assert got == c["requests"]
    d = em.BenchmarkResults(method="speculative", batches=[bm], start_time=bm.batch_start_time,
                            end_time=bm.batch_end_time).to_dict()
    assert d["total_tokens"] == sum(r["generated_tokens"] for r in c["requests"])
    assert all(r["ttft"] >= 0 for r in d["batches"][0]["requests"])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _decode_setup(V=4096, B=6):
    target, drafter = make_pair(V, dtype=torch.bfloat16, device=DEV, pos_mult=0)
    g = torch.Generator().manual_seed(4321)
    ids = torch.randint(3, V, (B, 8), generator=g).to(DEV)
    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=4, gen_len=24, end_tokens=[1])
    return ctx, ids


def _dp_worker(rank, world, port, seed, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from specdec_amd import set_noise_mode
        from specdec_amd.engine.dp_runner import batch_speculative_generate_dp, run_batch_speculative_dp
        from specdec_amd import get_poll_policy
        ctx, ids = _decode_setup()
        # STREAM (the bit-exact default) is refused: independent ranks cannot share one generator
        set_noise_mode("stream")
        try:
            batch_speculative_generate_dp(ctx, ids, torch.ones_like(ids), dist)
            refused = False
        except RuntimeError:
            refused = True
        set_noise_mode("philox", seed=seed)
        outs, rates, _ = batch_speculative_generate_dp(ctx, ids, torch.ones_like(ids), dist)
        # a second batch without re-seeding: the ranks agreed on the call offset after the first
        outs2, _, _ = batch_speculative_generate_dp(ctx, ids.flip(0), torch.ones_like(ids), dist)
        set_noise_mode("philox", seed=seed)
        bm = run_batch_speculative_dp(ctx, ids, torch.ones_like(ids), ids.shape[0], dist)
        if rank == 0:
            out.put(([o.cpu().tolist() for o in outs], rates,
                     [(r.generated_tokens, r.acceptance_rate) for r in bm.requests],
                     [o.cpu().tolist() for o in outs2], refused, get_poll_policy()[0]))
    finally:
        dist.destroy_process_group()


def test_dp_runner_two_ranks_equal_one_process():
    from specdec_amd import set_noise_mode
    from specdec_amd.engine.infer_engine import batch_speculative_generate
    seed = 9090
    ctx, ids = _decode_setup()
    set_noise_mode("philox", seed=seed)
    want, wrates = batch_speculative_generate(ctx, ids, torch.ones_like(ids), ids.shape[0])
    want = [o.cpu().tolist() for o in want]
    want2, _ = batch_speculative_generate(ctx, ids.flip(0), torch.ones_like(ids), ids.shape[0])
    want2 = [o.cpu().tolist() for o in want2]
    set_noise_mode("stream")
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_dp_worker, args=(r, 2, port, seed, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, rates, reqs, got2, refused, polled = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want and rates == wrates
    assert got2 == want2            # the second batch too: the ranks' Philox call offsets agree
    assert refused                  # DP under STREAM noise raises
    assert polled is False          # both ranks on cuda:0: the runner switched in-launch polls off
    assert [g for g, _ in reqs] == [len(o) - ids.shape[1] for o in want]
    assert [a for _, a in reqs] == wrates


def _batches_setup(V=4096):
    target, drafter = make_pair(V, dtype=torch.bfloat16, device=DEV, pos_mult=0)
    g = torch.Generator().manual_seed(5151)
    batches = []
    for k in range(4):
        ids = torch.randint(3, V, (3 + k % 2, 6 + k), generator=g).to(DEV)
        batches.append((ids, torch.ones_like(ids)))
    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=4, gen_len=16, end_tokens=[1])
    return ctx, batches


def _batch_dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from specdec_amd import set_noise_mode
        from specdec_amd.engine.dp_runner import generate_batches_dp
        ctx, batches = _batches_setup()
        set_noise_mode("stream")
        torch.manual_seed(100 + rank)            # only the per-batch re-seed may align the ranks
        res, _ = generate_batches_dp(ctx, batches, dist, seed=42)
        if rank == 0:
            out.put([([o.tolist() for o in outs], rates) for outs, rates in res])
    finally:
        dist.destroy_process_group()


def test_batch_level_dp_two_ranks_bit_exact_under_stream():
    """Batch-level data parallelism on the real kernels: 4 prompt batches dealt over two processes
    (both on cuda:0), each re-seeded per batch as engine/benchmark_executor.py:79 does, under the
    bit-exact STREAM noise, equal one process's re-seeded loop batch for batch."""
    from specdec_amd import set_noise_mode
    from specdec_amd.engine.dp_runner import reseed
    from specdec_amd.engine.infer_engine import batch_speculative_generate
    ctx, batches = _batches_setup()
    set_noise_mode("stream")
    want = []
    for ids, mask in batches:
        reseed(42)
        outs, rates = batch_speculative_generate(ctx, ids, mask, ids.shape[0])
        want.append(([o.cpu().tolist() for o in outs], rates))
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_batch_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
    assert any(len(o) > batches[i][0].shape[1] for i, (outs, _) in enumerate(want) for o in outs)
