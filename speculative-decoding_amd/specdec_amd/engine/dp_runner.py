"""Data-parallel runners for the drop-in engine: one process per GPU, no collective on the data path.

Two ways to split the work (INTEGRATION.md "Data parallelism" says which is exact):

* **Batch-level (bit-exact in both noise modes)** — ``infer_batches_dp`` / ``generate_batches_dp``.
  The reference's benchmark loop re-seeds before EVERY prompt batch (engine/benchmark_executor.py:79,
  ``runner._set_seed(42)`` -> engine/benchmark_runner.py:164-172) and runs each batch on its own
  (:72-83).  A batch's outputs therefore depend only on its prompts and the seed, so the batches can
  be dealt to the ranks round-robin (batch i on rank i % world), each rank re-seeding before each of
  its batches exactly as the reference does, and every batch's tokens equal one process's — also under
  the STREAM noise (the reference's own torch-generator draws).  Results are gathered in batch order
  with ``all_gather_object`` after decoding.

* **Row-level (Philox only; strong scaling of ONE batch)** — ``batch_speculative_generate_dp`` /
  ``run_batch_speculative_dp`` / ``infer_batch_dp``.  Every rank takes a contiguous row shard of the
  SAME tokenized global batch (the padding depends on the whole batch, so the batch is tokenized
  once, identically on every rank), runs ``batch_speculative_generate`` on it with ``ctx.row_base`` =
  its first global row, and the per-row outputs / rates / request metrics are gathered in global
  row order.  Philox draws are keyed by (seed, call offset, GLOBAL row), so the gathered outputs
  equal those of one process decoding the whole batch (tests/test_gpu_engine_surface.py); after
  every batch the ranks agree on the call offset (the largest any rank reached — what one process,
  which runs until its last row finishes, would hold), so later batches stay equal too.  The
  bit-exact STREAM mode draws from ONE torch generator in the reference's serial row order
  (engine/infer_engine.py:280-330): independent ranks would each replay the same words, so the
  row-level runner refuses it (RuntimeError) rather than return outputs that match neither the
  reference nor one process.

Ranks that share a GPU (more ranks than devices on a node) make the library's in-launch polls
unsafe (a grid can be starved by another process's kernels), so both runners switch them off
(``sd_set_poll_policy(allow_poll=0)``) when they see that.
"""
from __future__ import annotations

import random
import time
from typing import List, Optional, Sequence, Tuple

import torch

from .. import _lib, dp
from ..noise import PhiloxNoise, StreamNoise, default_noise
from .batch_decode import decode_batch_with_chat_template
from .infer_engine import _fill_batch_metrics, batch_speculative_generate
from .metrics import BatchMetrics


def _world(dist) -> Tuple[int, int]:
    if dist is None or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(), dist.get_rank()


def _gather(obj, dist):
    world, _ = _world(dist)
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


_SHARED_CHECKED = set()


def ranks_share_devices(dist, device) -> bool:
    """True when two ranks of `dist` run on the same GPU (same host, same device index)."""
    world, _ = _world(dist)
    if world == 1:
        return False
    import socket
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else (torch.cuda.current_device() if dev.type == "cuda" else 0)
    me = (socket.gethostname(), dev.type, idx)
    everyone = _gather(me, dist)
    return len(set(everyone)) < len(everyone)


def configure_residency(dist, device) -> bool:
    """Switch the library's in-launch polls off when ranks share a GPU (INTEGRATION.md
    "Residency"): a poll-mode grid assumes it is alone on the device.  Checked once per process
    group; returns whether polling stays allowed."""
    key = id(dist) if dist is not None else None
    if key not in _SHARED_CHECKED:
        _SHARED_CHECKED.add(key)
        if ranks_share_devices(dist, device):
            _lib.set_poll_policy(allow_poll=False, spin_limit=_lib.get_poll_policy()[1])
    return _lib.get_poll_policy()[0]


def _sync_philox_offset(noise, dist) -> None:
    """Every rank takes the largest call offset any rank reached: one process decoding the whole
    batch runs until its LAST row finishes, so it holds that offset; ranks whose rows finished
    earlier stopped calling sooner."""
    world, _ = _world(dist)
    if world == 1 or not isinstance(noise, PhiloxNoise):
        return
    noise.offset = max(_gather(int(noise.offset), dist))


def batch_speculative_generate_dp(ctx, input_ids: torch.Tensor, attention_mask: torch.Tensor, dist=None,
                                  first_token_callback=None) -> Tuple[List[torch.Tensor], List[float], float]:
    """Decode the global batch [B, L] sharded over the ranks of `dist`.

    Returns (outputs, rates, elapsed) for the WHOLE batch on every rank (outputs on this rank's
    device, global row order) and this rank's decode wall time.  `first_token_callback` gets
    GLOBAL row ids.  PHILOX noise only (module docstring): under the STREAM default every rank
    raises RuntimeError before decoding anything."""
    world, rank = _world(dist)
    noise = default_noise()
    if world > 1 and isinstance(noise, StreamNoise):
        raise RuntimeError("data-parallel decoding needs PHILOX noise (specdec_amd.set_noise_mode('philox')): "
                           "the bit-exact STREAM mode draws every row from one torch generator in the "
                           "reference's serial order, which independent ranks cannot share")
    configure_residency(dist, input_ids.device)
    B = input_ids.shape[0]
    start, stop = dp.shard_rows(B, world, rank)
    saved = getattr(ctx, "row_base", None)
    ctx.row_base = start
    cb = None
    if first_token_callback is not None:
        takes_time = getattr(first_token_callback, "accepts_time", False)

        def cb(i, t=None):   # local row -> global row; the graph path's device time is forwarded
            if takes_time:
                first_token_callback(start + i, t)
            else:
                first_token_callback(start + i)
        cb.accepts_time = takes_time
    err = None
    outs, rates = [], []
    t0 = time.time()
    try:
        if stop > start:
            outs, rates = batch_speculative_generate(ctx, input_ids[start:stop], attention_mask[start:stop],
                                                     stop - start, first_token_callback=cb)
    except Exception as e:   # reported after the gather, so no rank is left waiting in it
        err = f"rank {rank}: {type(e).__name__}: {e}"
    finally:
        if saved is None:
            del ctx.row_base
        else:
            ctx.row_base = saved
    elapsed = time.time() - t0
    _sync_philox_offset(noise, dist)
    shards = _gather((err, [o.cpu() for o in outs], rates), dist)
    errs = [s[0] for s in shards if s[0] is not None]
    if errs:
        raise RuntimeError("; ".join(errs))
    dev = input_ids.device
    outputs = [o.to(dev) for s in shards for o in s[1]]
    all_rates = [r for s in shards for r in s[2]]
    return outputs, all_rates, elapsed


def run_batch_speculative_dp(ctx, input_ids: torch.Tensor, attention_mask: torch.Tensor, batch_size: int,
                             dist=None) -> Optional[BatchMetrics]:
    """engine/infer_engine.py:99-146 over the ranks: every rank returns the GLOBAL BatchMetrics
    (requests in global row order; batch latency = the slowest rank's, i.e. the job's)."""
    bm = BatchMetrics(batch_size=batch_size)
    firsts: List[Optional[float]] = [None] * batch_size

    def first_token(idx, t=None):
        if idx < batch_size and firsts[idx] is None:
            firsts[idx] = time.time() if t is None else t
    first_token.accepts_time = True   # the graph path reports the first draw's device completion time

    ok = True
    t_start = time.time()
    try:
        outputs, rates, _ = batch_speculative_generate_dp(ctx, input_ids, attention_mask, dist,
                                                          first_token_callback=first_token)
    except Exception as e:  # the reference's contract (:144-146); every rank must still join the gather
        print(f"Batch speculative decoding failed: {type(e).__name__}: {e}")
        ok, outputs, rates = False, [], []
    t_end = time.time()
    meta = _gather((ok, t_start, t_end, firsts), dist)
    if not all(m[0] for m in meta):
        return None
    bm.batch_start_time = min(m[1] for m in meta)
    bm.batch_end_time = max(m[2] for m in meta)
    merged = [None] * batch_size
    for m in meta:
        for i, f in enumerate(m[3]):
            if f is not None and merged[i] is None:
                merged[i] = f
    starts = [bm.batch_start_time] * batch_size
    return _fill_batch_metrics(bm, outputs, attention_mask, starts, merged, rates)


def infer_batch_dp(ctx, prompts: List[str], dist=None) -> Tuple[Optional[BatchMetrics], Optional[BatchMetrics]]:
    """``infer_batch`` (engine/infer_engine.py:10-96) for a data-parallel job: same formatting and
    tokenization of the whole prompt batch on every rank, then the row-sharded speculative run.
    The target-only baseline is not sharded (it is outside the verify/accept path)."""
    if not ctx.spec:
        from .infer_engine import infer_batch
        return infer_batch(ctx, prompts)
    if ctx.chat:
        formatted = [ctx.tokenizer.apply_chat_template([{"role": "user", "content": p}],
                                                       add_generation_prompt=True, tokenize=False)
                     for p in prompts]
    else:
        formatted = prompts
    input_ids, attention_mask = decode_batch_with_chat_template(ctx.tokenizer, formatted,
                                                                max_length=ctx.max_batch_length, chat=False)
    drafter_device = getattr(ctx, "drafter_device", None)
    if drafter_device is not None:
        input_ids, attention_mask = input_ids.to(drafter_device), attention_mask.to(drafter_device)
    if getattr(ctx, "reset_in_between", False) and getattr(ctx, "ngram", None) is not None:
        ctx.ngram.reset()
    return run_batch_speculative_dp(ctx, input_ids, attention_mask, len(prompts), dist), None


# ---------------------------------------------------------------------------------------------
# batch-level data parallelism (bit-exact under STREAM and Philox)
# ---------------------------------------------------------------------------------------------

def reseed(seed: int) -> None:
    """engine/benchmark_runner.py:164-172 (``_set_seed``), run before every batch by
    engine/benchmark_executor.py:79: python, numpy and torch generators seeded.  The STREAM noise
    draws from torch.default_generator, so this fixes its words; a Philox default noise restarts
    its call counter (its seed is fixed by ``set_noise_mode``), the Philox analogue."""
    random.seed(seed)
    try:
        import numpy as np
        np.random.seed(seed)
    except ImportError:   # pragma: no cover - numpy is part of the image
        pass
    torch.manual_seed(seed)
    noise = default_noise()
    if isinstance(noise, PhiloxNoise):
        noise.offset = 0


def batches_of_rank(n_batches: int, world: int, rank: int) -> List[int]:
    """The batches rank `rank` decodes: i % world == rank (round-robin, so ranks stay balanced when
    the batch count is not a multiple of the world size)."""
    if world <= 0 or not 0 <= rank < world or n_batches < 0:
        raise ValueError(f"bad batch assignment: batches={n_batches} world={world} rank={rank}")
    return list(range(rank, n_batches, world))


def _gather_in_order(mine, n_batches: int, dist, what: str):
    """[(batch index, result or error text)] of every rank -> results in batch order; raises on
    every rank if any rank failed (after the gather, so no rank is left waiting in it)."""
    got = {}
    errs = []
    for part in _gather(mine, dist):
        for i, ok, res in part:
            if ok:
                got[i] = res
            else:
                errs.append(res)
    if errs:
        raise RuntimeError(f"{what}: " + "; ".join(errs))
    return [got[i] for i in range(n_batches)]


def generate_batches_dp(ctx, batches: Sequence[Tuple[torch.Tensor, torch.Tensor]], dist=None, seed: int = 42):
    """Decode whole prompt batches ``[(input_ids [B_i, L_i], attention_mask)]`` dealt round-robin
    over the ranks, re-seeding before each batch (``reseed(seed)``) as the reference's benchmark
    loop does.  Returns, on every rank, ``[(outputs, rates)]`` in batch order (outputs on the CPU)
    and this rank's decode wall time.  Bit-exact in both noise modes: every batch equals what one
    process running the same re-seeded loop returns."""
    world, rank = _world(dist)
    if batches:
        configure_residency(dist, batches[0][0].device)
    mine = []
    t0 = time.time()
    for i in batches_of_rank(len(batches), world, rank):
        ids, mask = batches[i]
        reseed(seed)
        try:
            outs, rates = batch_speculative_generate(ctx, ids, mask, ids.shape[0])
            mine.append((i, True, ([o.cpu() for o in outs], rates)))
        except Exception as e:   # reported after the gather
            mine.append((i, False, f"rank {rank} batch {i}: {type(e).__name__}: {e}"))
    elapsed = time.time() - t0
    return _gather_in_order(mine, len(batches), dist, "generate_batches_dp"), elapsed


def infer_batches_dp(ctx, prompt_batches: Sequence[List[str]], dist=None, seed: int = 42
                     ) -> List[Tuple[Optional[BatchMetrics], Optional[BatchMetrics]]]:
    """engine/benchmark_executor.py:72-83's batch loop, sharded by batch: rank r runs
    ``reseed(seed); infer_batch(ctx, prompts)`` for batches r, r + world, ...; every rank returns
    the ``(spec_metrics, target_metrics)`` pair of EVERY batch, in batch order (what the reference
    appends to its BenchmarkResults).  A failed batch is ``(None, None)``, as infer_batch returns it
    (:144-146).  An exception that escapes infer_batch on one rank (tokenization, the chat template,
    a device copy, the target-only path) is held until after the gather and then raised on EVERY
    rank, as generate_batches_dp does — no rank is left waiting in the gather."""
    from .infer_engine import infer_batch
    world, rank = _world(dist)
    dev = getattr(ctx, "drafter_device", None) or getattr(ctx, "target_device", None)
    if dev is not None:
        configure_residency(dist, dev)
    mine = []
    for i in batches_of_rank(len(prompt_batches), world, rank):
        try:
            reseed(seed)
            mine.append((i, True, infer_batch(ctx, list(prompt_batches[i]))))
        except Exception as e:   # reported after the gather
            mine.append((i, False, f"rank {rank} batch {i}: {type(e).__name__}: {e}"))
    return _gather_in_order(mine, len(prompt_batches), dist, "infer_batches_dp")
