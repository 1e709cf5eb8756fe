"""Data-parallel path on CPU: world_size-2 gloo ranks (127.0.0.1), as the bench runs one rank
per GPU.  Checks the contiguous row sharding, the max-time / summed-counter aggregation bench.py
reports, and that per-row Philox noise keyed by the GLOBAL row id makes the sharded accept walk
identical to a single-process walk over the whole batch (the property SURVEY.md §8e asks for;
the GPU counterpart is tests/test_gpu_perfmode.py::test_perf_sharded_calls_equal_one_call)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import philox_ref as ph
from specdec_amd import dp


def test_shard_rows_cover_the_batch_contiguously():
    for rows in (0, 1, 7, 32, 33, 1000):
        for world in (1, 2, 3, 8):
            spans = [dp.shard_rows(rows, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == rows
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        dp.shard_rows(4, 2, 2)


def engine_walk(p, q, seed, offset, global_row, gamma):
    """Accept count of one engine row (engine/infer_engine.py:297-330) on Philox uniforms."""
    n = 0
    for i in range(gamma):
        u = float(ph.accept_uniform(seed, offset, global_row, i))
        ap = 1.0 if q[i] <= 0 else min(1.0, p[i] / q[i])
        if u < ap:
            n += 1
        else:
            break
    return n


def batch_inputs(rows, gamma, seed=0):
    g = torch.Generator().manual_seed(seed)
    p = torch.rand(rows, gamma, generator=g).double()
    q = (p * (0.5 + torch.rand(rows, gamma, generator=g))).double()
    return p, q


def _worker(rank, world, port, rows, gamma, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, stop = dp.shard_rows(rows, world, rank)
        p, q = batch_inputs(rows, gamma)
        n = [engine_walk(p[b].tolist(), q[b].tolist(), 77, 5, b, gamma) for b in range(start, stop)]
        # gather the shards (test only; the bench never gathers row outputs)
        sizes = [dp.shard_rows(rows, world, r) for r in range(world)]
        buf = torch.full((rows,), -1, dtype=torch.long)
        buf[start:stop] = torch.tensor(n, dtype=torch.long)
        dist.all_reduce(buf, op=dist.ReduceOp.MAX)
        elapsed, tot = dp.aggregate(0.5 + rank, {"tokens": 10.0 * (rank + 1), "drafted": float(stop - start)},
                                    torch.device("cpu"), dist)
        if rank == 0:
            out.put((buf.tolist(), elapsed, tot, sizes))
    finally:
        dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_gloo_ranks_equal_one_process():
    rows, gamma, world = 37, 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, rows, gamma, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got, elapsed, tot, sizes = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p, qq = batch_inputs(rows, gamma)
    want = [engine_walk(p[b].tolist(), qq[b].tolist(), 77, 5, b, gamma) for b in range(rows)]
    assert got == want
    assert elapsed == 1.5                                   # max over ranks
    assert tot == {"drafted": float(rows), "tokens": 30.0}  # sums over ranks
    assert sizes == [(0, 19), (19, 37)]

