"""The product data-parallel runner (specdec_amd.engine.dp_runner) on two gloo ranks (127.0.0.1).

The HIP engine loop cannot run here, so `batch_speculative_generate` inside the runner is replaced
by a host stand-in with the same contract: it decodes the rows it is given from ctx.row_base (its
outputs depend on the GLOBAL row id, as Philox-keyed draws do) and consumes Philox call offsets
for as many windows as its slowest row needs — so shards stop at different offsets, as real
ranks do.  Everything else is the shipped code: the sharding, the STREAM refusal, the residency
switch for ranks that share a device, the call-offset agreement after every batch, the error
propagation (every rank raises, none hangs in the gather) and the global-order gather that
run_batch_speculative_dp turns into BatchMetrics.  The GPU counterpart with the real kernels is
tests/test_gpu_engine_surface.py::test_dp_runner_two_ranks_equal_one_process.
"""
import os
import socket
from types import SimpleNamespace

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def fake_engine(ctx, input_ids, attention_mask, batch_size, first_token_callback=None):
    """Stand-in for engine.infer_engine.batch_speculative_generate: row i of the shard is global row
    ctx.row_base + i; it 'generates' windows of tokens derived from the global row, and the call
    offsets advance by (γ + 1) per window until the shard's longest row is done."""
    from specdec_amd.noise import default_noise
    noise = default_noise()
    outs, rates = [], []
    windows = 0
    for i in range(batch_size):
        g = ctx.row_base + i
        if g == ctx.fail_row:
            raise RuntimeError(f"probability tensor contains either `inf`, `nan` or element < 0 (row {g})")
        n_win = 1 + (2 * g) % 5                      # rows finish after 1..5 windows
        windows = max(windows, n_win)
        gen = [100 + 10 * g + k + noise.offset for k in range(n_win)]
        outs.append(torch.cat([input_ids[i], torch.tensor(gen, dtype=torch.long)]))
        rates.append(1.0 / (1 + g))
        if first_token_callback is not None:
            first_token_callback(i)
    noise.offset += windows * (ctx.gamma + 1)
    return outs, rates


def one_process(B, L, gamma, batches):
    """What one process decoding every row (row_base 0) returns, batch after batch."""
    from specdec_amd import set_noise_mode
    from specdec_amd.noise import default_noise
    set_noise_mode("philox", seed=5)
    ctx = SimpleNamespace(gamma=gamma, row_base=0, fail_row=-1)
    res = []
    for k in range(batches):
        ids = torch.arange(B * L, dtype=torch.long).reshape(B, L) + 1000 * k
        outs, rates = fake_engine(ctx, ids, torch.ones_like(ids), B)
        res.append(([o.tolist() for o in outs], rates))
    return res, default_noise().offset


def _worker(rank, world, port, B, L, gamma, fail_row, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import specdec_amd
        from specdec_amd import set_noise_mode
        from specdec_amd.engine import dp_runner
        from specdec_amd.noise import default_noise
        dp_runner.batch_speculative_generate = fake_engine
        ctx = SimpleNamespace(gamma=gamma, fail_row=-1, spec=True)
        rec = {}
        # the bit-exact STREAM default is refused on every rank before any decoding
        set_noise_mode("stream")
        ids = torch.arange(B * L, dtype=torch.long).reshape(B, L)
        try:
            dp_runner.batch_speculative_generate_dp(ctx, ids, torch.ones_like(ids), dist)
            rec["stream"] = "no error"
        except RuntimeError as e:
            rec["stream"] = str(e)
        assert not hasattr(ctx, "row_base")
        # two Philox batches back to back, no re-seed in between
        set_noise_mode("philox", seed=5)
        rec["batches"] = []
        for k in range(2):
            ids = torch.arange(B * L, dtype=torch.long).reshape(B, L) + 1000 * k
            outs, rates, _ = dp_runner.batch_speculative_generate_dp(ctx, ids, torch.ones_like(ids), dist)
            rec["batches"].append(([o.tolist() for o in outs], rates))
        rec["offset"] = default_noise().offset
        rec["poll"] = specdec_amd.get_poll_policy()
        # BatchMetrics over the ranks: global row order, the job's latency
        bm = dp_runner.run_batch_speculative_dp(ctx, ids, torch.ones_like(ids), B, dist)
        rec["generated"] = [r.generated_tokens for r in bm.requests]
        rec["ttft_set"] = all(r.first_token_time is not None for r in bm.requests)
        # a row that fails on one rank: every rank raises (reference :144-146 -> None), none hangs
        ctx.fail_row = fail_row
        try:
            dp_runner.batch_speculative_generate_dp(ctx, ids, torch.ones_like(ids), dist)
            rec["fail"] = "no error"
        except RuntimeError as e:
            rec["fail"] = str(e)
        rec["fail_bm"] = dp_runner.run_batch_speculative_dp(ctx, ids, torch.ones_like(ids), B, dist)
        out.put((rank, rec))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dp_runner_orchestration_on_two_gloo_ranks():
    B, L, gamma, world = 7, 3, 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, L, gamma, 5, q)) for r in range(world)]
    for p in procs:
        p.start()
    recs = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want, want_offset = one_process(B, L, gamma, 2)
    for rank, rec in recs.items():
        assert "PHILOX" in rec["stream"], rec["stream"]
        assert rec["batches"] == [(o, r) for o, r in want]      # both batches: sharded == one process
        assert rec["offset"] == want_offset                      # the ranks agree on the call offset
        assert rec["poll"][0] is False                           # two ranks on one device: no polling
        assert rec["generated"] == [1 + (2 * g) % 5 for g in range(B)]
        assert rec["ttft_set"]
        assert "row 5" in rec["fail"] and "rank 1" in rec["fail"]
        assert rec["fail_bm"] is None


# ---------------------------------------------------------------------------------------------
# batch-level data parallelism: whole batches per rank, re-seeded per batch (bit-exact, STREAM)
# ---------------------------------------------------------------------------------------------

def stream_engine(ctx, input_ids, attention_mask, batch_size, first_token_callback=None):
    """Stand-in for batch_speculative_generate under the STREAM noise: every token comes from
    torch.default_generator in the serial order one process consumes it (the reference's draws),
    and the number of draws depends on the outcomes — so a batch's outputs depend on the generator
    state it starts from, which only the per-batch re-seed makes rank-independent."""
    outs, rates = [], []
    for i in range(batch_size):
        n = 1 + int(torch.randint(0, 4, (1,)))
        gen = torch.randint(3, 1000, (n,))
        outs.append(torch.cat([input_ids[i], gen]))
        rates.append(float(torch.rand(1)))
    return outs, rates


def stream_batches(n):
    g = torch.Generator().manual_seed(77)
    return [torch.randint(3, 500, (2 + k % 3, 4), generator=g) for k in range(n)]


def one_process_batches(batches, seed):
    from specdec_amd.engine import dp_runner
    res = []
    for ids in batches:
        dp_runner.reseed(seed)
        outs, rates = stream_engine(None, ids, torch.ones_like(ids), ids.shape[0])
        res.append(([o.tolist() for o in outs], rates))
    return res


def _batch_worker(rank, world, port, n_batches, seed, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from specdec_amd import set_noise_mode
        from specdec_amd.engine import dp_runner, infer_engine
        dp_runner.batch_speculative_generate = stream_engine
        set_noise_mode("stream")
        batches = [(ids, torch.ones_like(ids)) for ids in stream_batches(n_batches)]
        torch.manual_seed(rank + 1000)        # the ranks' generators start apart: only reseed aligns them
        res, _ = dp_runner.generate_batches_dp(SimpleNamespace(), batches, dist, seed=seed)
        rec = {"batches": [([o.tolist() for o in outs], rates) for outs, rates in res],
               "mine": dp_runner.batches_of_rank(n_batches, world, rank)}

        # infer_batches_dp: the executor loop's (spec, target) pairs in batch order
        def fake_infer(ctx, prompts):
            return (len(prompts), float(torch.rand(1))), None
        infer_engine.infer_batch = fake_infer
        pairs = dp_runner.infer_batches_dp(SimpleNamespace(), [["p"] * (k + 1) for k in range(n_batches)], dist,
                                           seed=seed)
        rec["pairs"] = pairs
        # a failing batch raises on every rank
        def bad_engine(ctx, input_ids, attention_mask, batch_size, first_token_callback=None):
            if int(input_ids[0, 0]) == int(batches[1][0][0, 0]):
                raise RuntimeError("probability tensor contains either `inf`, `nan` or element < 0")
            return stream_engine(ctx, input_ids, attention_mask, batch_size)
        dp_runner.batch_speculative_generate = bad_engine
        try:
            dp_runner.generate_batches_dp(SimpleNamespace(), batches, dist, seed=seed)
            rec["fail"] = "no error"
        except RuntimeError as e:
            rec["fail"] = str(e)

        # infer_batch raising outside the decode (tokenization, chat template, .to(device)) on one
        # rank's batch: every rank raises after the gather, none is left waiting in it
        def raising_infer(ctx, prompts):
            if len(prompts) == 2:                # batch 1, on rank 1
                raise ValueError("chat template missing")
            return (len(prompts), 0.0), None
        infer_engine.infer_batch = raising_infer
        try:
            dp_runner.infer_batches_dp(SimpleNamespace(), [["p"] * (k + 1) for k in range(n_batches)], dist,
                                       seed=seed)
            rec["infer_fail"] = "no error"
        except RuntimeError as e:
            rec["infer_fail"] = str(e)
        out.put((rank, rec))
    finally:
        dist.destroy_process_group()


def test_batch_level_dp_is_bit_exact_under_stream_noise():
    """4 and 5 batches over 2 gloo ranks (round-robin) equal one process's re-seeded batch loop,
    batch for batch, under the STREAM noise (engine/benchmark_executor.py:79 re-seeds per batch)."""
    from specdec_amd import set_noise_mode
    from specdec_amd.engine import dp_runner
    seed, world = 42, 2
    set_noise_mode("stream")
    assert dp_runner.batches_of_rank(5, 2, 0) == [0, 2, 4] and dp_runner.batches_of_rank(5, 2, 1) == [1, 3]
    for n_batches in (4, 5):
        want = one_process_batches(stream_batches(n_batches), seed)
        want_pairs = []
        for k in range(n_batches):
            dp_runner.reseed(seed)
            want_pairs.append(((k + 1, float(torch.rand(1))), None))
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_batch_worker, args=(r, world, port, n_batches, seed, q)) for r in range(world)]
        for p in procs:
            p.start()
        recs = dict(q.get(timeout=180) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert sorted(recs[0]["mine"] + recs[1]["mine"]) == list(range(n_batches))
        for rank, rec in recs.items():
            assert rec["batches"] == want, (n_batches, rank)
            assert [tuple(p[0]) for p in rec["pairs"]] == [p[0] for p in want_pairs]
            assert "batch 1" in rec["fail"] and "rank 1" in rec["fail"]
            assert "rank 1 batch 1: ValueError: chat template missing" in rec["infer_fail"], rec["infer_fail"]


def test_dp_runner_forwards_the_graph_paths_first_token_time(monkeypatch):
    """The graph-window engine path reports each row's first draw at its device completion time
    (callback(idx, t) when the callback declares accepts_time); the DP wrappers must forward it,
    not stamp the time the whole run returned (TTFT ~ batch latency otherwise)."""
    from specdec_amd import set_noise_mode
    from specdec_amd.engine import dp_runner

    def timed_engine(ctx, input_ids, attention_mask, batch_size, first_token_callback=None):
        assert getattr(first_token_callback, "accepts_time", False)
        for i in range(batch_size):
            first_token_callback(i, 1000.0 + ctx.row_base + i)
        return [torch.cat([input_ids[i], torch.tensor([5])]) for i in range(batch_size)], [0.5] * batch_size

    monkeypatch.setattr(dp_runner, "batch_speculative_generate", timed_engine)
    set_noise_mode("philox", seed=3)
    ids = torch.arange(12, dtype=torch.long).reshape(4, 3) + 10
    bm = dp_runner.run_batch_speculative_dp(SimpleNamespace(gamma=4), ids, torch.ones_like(ids), 4, None)
    assert [r.first_token_time for r in bm.requests] == [1000.0, 1001.0, 1002.0, 1003.0]
    set_noise_mode("stream")
