"""Tensor-level wrappers over the C ABI (include/specdec.h).

Every call validates shapes, strides and dtypes on the host BEFORE a kernel is enqueued,
then launches on the current HIP stream of the tensors' device.  Nothing here syncs except
where noted: StreamNoise outside a ``session`` writes the moved generator state back to the
torch generator after each call (one device->host copy).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import lib
from .noise import PhiloxNoise, StreamNoise

_DT = {torch.float32: _lib.SD_F32, torch.bfloat16: _lib.SD_BF16, torch.float16: _lib.SD_F16}

KIND = {"greedy": _lib.SD_PROC_GREEDY, "multinomial": _lib.SD_PROC_MULTINOMIAL, "topk": _lib.SD_PROC_TOPK,
        "nucleus": _lib.SD_PROC_NUCLEUS, "topknucleus": _lib.SD_PROC_TOPK_NUCLEUS}
# the reference's class names (utils/logits_processor.py) and ours map to the same kinds
_CLASS_KIND = {"GreedyProcessor": "greedy", "MultinomialProcessor": "multinomial", "TopKProcessor": "topk",
               "NucleusProcessor": "nucleus", "TopKNucleusProcessor": "topknucleus"}


@dataclass(frozen=True)
class ProcSpec:
    kind: str = "greedy"
    temperature: float = 1.0
    top_k: int = 0
    top_p: float = 1.0

    @property
    def stochastic(self) -> bool:
        return self.kind != "greedy"

    @property
    def keeps(self) -> bool:
        """top-k / nucleus: rows carry a keep predicate (sd_row_keep)"""
        return KIND[self.kind] >= _lib.SD_PROC_TOPK

    def struct(self) -> _lib.sd_processor:
        return _lib.sd_processor(KIND[self.kind], float(self.temperature), int(self.top_k), float(self.top_p))


PLAIN_SOFTMAX = ProcSpec("multinomial", 1.0)   # engine/infer_engine.py:241,276 (T=1, no processor)


# the processor protocol's behaviour (utils/logits_processor.py:7-23): a subclass that redefines the
# softmax or the sampling rule computes something the kernels do not, so it is refused, never run as
# its base class.  _process is the protocol's extension point: a subclass's own _process runs as it
# is (torch ops on the device rows) and the kernels take its output (_user_process).
_PROC_REFUSED = ("__call__", "sample")


def _known_base(proc):
    """(index in the MRO, name) of the first of the five processor classes proc derives from."""
    mro = type(proc).__mro__
    for i, cls in enumerate(mro):
        if cls.__name__ in _CLASS_KIND:
            return i, cls.__name__
    return -1, type(proc).__name__


def _user_process(proc):
    """The bound ``_process`` of a user subclass of one of the five processors that overrides it (the
    reference's extension point, utils/logits_processor.py:18-20), else None."""
    if isinstance(proc, ProcSpec):
        return None
    i, _ = _known_base(proc)
    if i <= 0:
        return None
    return proc._process if any("_process" in vars(sub) for sub in type(proc).__mro__[:i]) else None


def proc_spec(proc) -> ProcSpec:
    """ProcSpec of one of the five processors (ours, the reference's, or a ProcSpec).

    A subclass of a known processor may override ``_process`` (its own processing — often
    ``super()._process`` plus more): the rows are then processed by running it (``processed_rows``)
    and the kernels apply the base class's sampling rule to them — softmax(y / T), then argmax
    (GreedyProcessor) or the multinomial draw.  A subclass that overrides ``__call__`` or ``sample``
    raises TypeError: the kernels fuse the softmax and the draw and cannot run user code there."""
    if isinstance(proc, ProcSpec):
        return proc
    i, name = _known_base(proc)
    if i < 0:
        raise TypeError(f"unsupported logits processor {type(proc).__name__}")
    mro = type(proc).__mro__
    for sub in mro[:i]:
        over = [m for m in _PROC_REFUSED if m in vars(sub)]
        if over:
            raise TypeError(f"unsupported logits processor {type(proc).__name__}: {sub.__name__} overrides "
                            f"{', '.join(over)} of {name}, which the fused kernels cannot run")
    T = float(getattr(proc, "temperature", 1.0))
    if _user_process(proc) is not None:   # user processing: only the base's sampling rule stays fused
        return ProcSpec("greedy" if name == "GreedyProcessor" else "multinomial", T)
    return ProcSpec(_CLASS_KIND[name], T, int(getattr(proc, "top_k", 0)), float(getattr(proc, "top_p", 1.0)))


def processed_rows(proc, rows):
    """The rows the kernels read for processor ``proc``: the rows themselves, or — for a subclass
    with its own ``_process`` — its output on a copy of each row (device torch ops; the caller's
    logits are never modified).  rows: a tensor [R, V] or a sequence of them."""
    fn = _user_process(proc)
    if fn is None:
        return rows

    def one(t):
        y = fn(t.clone())
        if not torch.is_tensor(y) or y.shape != t.shape or y.device != t.device:
            raise ValueError(f"{type(proc).__name__}._process must return a tensor of the input's shape and device")
        if y.dtype not in _DT:
            y = y.float()
        return y if y.stride(-1) == 1 else y.contiguous()

    return one(rows) if torch.is_tensor(rows) else [one(t) for t in rows]


# sequences one Philox call verifies / samples (the arrival-counter block, kCntMax in the kernels)
MAX_ROWS_PER_CALL = 16384


def _row_shards(B: int, noise):
    """Row shards of a Philox call over more than MAX_ROWS_PER_CALL sequences: [(r0, r1, noise)]
    with ONE call offset for all shards (noise keyed by the global row = row_base + r), so the
    shards draw what one call would.  None when the call fits (or is not Philox)."""
    if B <= MAX_ROWS_PER_CALL or not isinstance(noise, PhiloxNoise):
        return None
    o = noise.next_offset()
    return [(r0, min(B, r0 + MAX_ROWS_PER_CALL), PhiloxNoise(noise.seed, o, noise.offset_dev))
            for r0 in range(0, B, MAX_ROWS_PER_CALL)]


def _stream_ptr(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


# One workspace per (device, stream): it holds the arrival counters and partials of the calls in
# flight, so calls on different streams must not share one (they would mix their counters).  A
# workspace is allocated on the stream that uses it, so replacing it by a bigger one is
# stream-ordered by the caching allocator.  Graph capture reuses the device's largest eager
# workspace (the capture stream is a side stream; run the call eagerly once before capturing) and
# keeps it alive for as long as the process runs, since replays hold its address.
_WS: Dict[Tuple[torch.device, int], torch.Tensor] = {}
_GRAPH_WS: List[torch.Tensor] = []


def _workspace(nbytes: int, device) -> torch.Tensor:
    dev = torch.device(device)
    if torch.cuda.is_current_stream_capturing():
        cands = [w for (d, _), w in _WS.items() if d == dev]
        ws = max(cands, key=lambda w: w.numel()) if cands else None
        if ws is None or ws.numel() < nbytes:
            raise RuntimeError("specdec: a call captured into a hipGraph needs a workspace sized by an eager call "
                               "of the same shape first (run it once before capturing)")
        if not any(w is ws for w in _GRAPH_WS):
            _GRAPH_WS.append(ws)
        return ws
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nbytes:
        # zero-filled once: the library keeps its arrival counters (front of the workspace) at zero
        ws = torch.zeros(max(nbytes, 1 << 20), dtype=torch.uint8, device=dev)
        _WS[key] = ws
    return ws


def _require_rows(t: torch.Tensor, name: str, V: int) -> None:
    if t.dim() != 2 or t.shape[1] != V:
        raise ValueError(f"{name}: expected [rows, {V}], got {tuple(t.shape)}")
    if t.stride(1) != 1:
        raise ValueError(f"{name}: vocab axis must be contiguous")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a device tensor")
    if t.dtype not in _DT:
        raise ValueError(f"{name}: unsupported dtype {t.dtype}")


def _status_or_ptr(status_or: Optional[torch.Tensor], device):
    """Device address of a caller's sticky error word (int32 [1] on the call's device), or None."""
    if status_or is None:
        return None
    if status_or.dtype != torch.int32 or status_or.numel() < 1 or status_or.device != torch.device(device):
        raise ValueError("status_or must be an int32 [1] tensor on the call's device")
    return status_or.data_ptr()


def _noise_struct(noise, n_words_needed: int, device, row_base: int = 0):
    """(sd_noise, keepalive tensor) for a call that may consume up to n_words_needed words.
    row_base: global id of the call's row 0 (Philox noise is keyed by the global row)."""
    if isinstance(noise, StreamNoise):
        # the call's words start at words[offset + *offset_dev] (ABI 11; a pipelined session's pool)
        words, off, off_dev = noise.prepare_ex(n_words_needed, device)
        return _lib.sd_noise(_lib.SD_NOISE_STREAM, words.data_ptr(), words.numel(), 0, int(off), 0,
                             off_dev.data_ptr() if off_dev is not None else None), (words, off_dev)
    if isinstance(noise, PhiloxNoise):
        if not 0 <= row_base < (1 << 24):
            raise ValueError("row_base must be in [0, 2^24)")
        od = noise.offset_dev
        if od is not None and (od.dtype != torch.int64 or od.numel() != 1 or od.device != torch.device(device)):
            raise ValueError("PhiloxNoise.offset_dev must be an int64 [1] tensor on the call's device")
        return _lib.sd_noise(_lib.SD_NOISE_PHILOX, None, 0, noise.seed, noise.next_offset(), row_base,
                             od.data_ptr() if od is not None else None), None
    raise TypeError(f"unsupported noise source {type(noise).__name__}")


# --------------------------------------------------------------------------- sampling
def sample_rows(logits: torch.Tensor, proc, noise, tokens_out: Optional[torch.Tensor] = None,
                want_prob: bool = False, row_base: int = 0, row_stats_out: Optional[torch.Tensor] = None,
                row_keep_out: Optional[torch.Tensor] = None, status_or: Optional[torch.Tensor] = None):
    """LogitsProcessor.__call__ + .sample on every row of logits [R, V] (one sample per row).

    Returns (tokens int64 [R], token_prob fp32 [R] or None, row_status int32 [R]).  Under
    StreamNoise the generator advances by 2·R·V words (torch.multinomial's Exp noise).
    row_stats_out: optional fp32 [R, 2] device tensor (contiguous) that receives each processed
    row's (max, Σexp) — what ``verify(draft_row_stats=...)`` takes so the verify step does not
    re-read the drafter rows.  Under PhiloxNoise stochastic rows are drawn in ONE pass (k_draw).
    row_keep_out: optional int32 [R, 4] contiguous device tensor that receives a top-k / nucleus
    row's keep predicate (sd_row_keep: tau as fp32 bits, tie index, flags) — what
    ``verify(draft_row_keep=...)`` takes with the stats so the verify skips the drafter rows'
    threshold search.  Not written for other processors.
    status_or: optional int32 [1] device word; every row's SD_ROW_ERROR_MASK bits are ORed into it
    (the decode loops test it where they already sync instead of reading every row_status).
    """
    spec = proc_spec(proc)
    R, V = logits.shape
    _require_rows(logits, "logits", V)
    logits = processed_rows(proc, logits)
    proc = spec
    dev = logits.device
    shards = _row_shards(R, noise)
    if shards is not None:   # more rows than one call holds: row shards, one noise offset
        toks = tokens_out if tokens_out is not None else torch.empty(R, dtype=torch.long, device=dev)
        outs = [sample_rows(logits[r0:r1], proc, nz, toks[r0:r1], want_prob, row_base + r0,
                            None if row_stats_out is None else row_stats_out.view(-1, 2)[r0:r1],
                            None if row_keep_out is None else row_keep_out.view(-1, 4)[r0:r1], status_or)
                for r0, r1, nz in shards]
        return (toks, torch.cat([o[1] for o in outs]) if want_prob else None, torch.cat([o[2] for o in outs]))
    tokens = tokens_out if tokens_out is not None else torch.empty(R, dtype=torch.long, device=dev)
    if tokens.dtype != torch.long or tokens.numel() < R or not tokens.is_cuda:
        raise ValueError("tokens_out must be an int64 device tensor with >= rows elements")
    prob = torch.empty(R, dtype=torch.float32, device=dev) if want_prob else None
    status = torch.empty(R, dtype=torch.int32, device=dev)
    if row_stats_out is not None and (row_stats_out.dtype != torch.float32 or not row_stats_out.is_cuda
                                      or row_stats_out.numel() < 2 * R or not row_stats_out.is_contiguous()):
        raise ValueError("row_stats_out must be a contiguous fp32 device tensor with >= 2*rows elements")
    if row_keep_out is not None and (row_keep_out.dtype != torch.int32 or not row_keep_out.is_cuda
                                     or row_keep_out.numel() < 4 * R or not row_keep_out.is_contiguous()):
        raise ValueError("row_keep_out must be a contiguous int32 device tensor with >= 4*rows elements")
    need = 2 * R * V if spec.stochastic else 0
    nz, keep = _noise_struct(noise, need, dev, row_base)
    nbytes = lib.sd_sample_workspace_size(R, V)
    ws = _workspace(nbytes, dev)
    a = _lib.sd_sample_args(R, V, logits.data_ptr(), logits.stride(0), _DT[logits.dtype], spec.struct(), nz,
                            tokens.data_ptr(), tokens.stride(0) if tokens.dim() == 1 else 1,
                            prob.data_ptr() if prob is not None else None, status.data_ptr(), None,
                            ws.data_ptr(), ws.numel(),
                            row_stats_out.data_ptr() if row_stats_out is not None else None,
                            row_keep_out.data_ptr() if row_keep_out is not None else None,
                            _status_or_ptr(status_or, dev))
    _lib.check(lib.sd_sample(C.byref(a), C.c_void_p(_stream_ptr(dev))), "sd_sample")
    if isinstance(noise, StreamNoise):
        noise.consumed(count=need)
    del keep
    return tokens, prob, status


def probs_rows(logits: torch.Tensor, proc) -> torch.Tensor:
    """LogitsProcessor.__call__: softmax(_process(logits) / T) in the logits dtype, on the device."""
    spec = proc_spec(proc)
    shape = logits.shape
    x = processed_rows(proc, logits.reshape(-1, shape[-1]))
    if x.stride(-1) != 1:
        x = x.contiguous()
    R, V = x.shape
    _require_rows(x, "logits", V)
    out = torch.empty((R, V), dtype=x.dtype, device=x.device)
    ws = _workspace(lib.sd_probs_workspace_size(R, V), x.device)
    a = _lib.sd_probs_args(R, V, x.data_ptr(), x.stride(0), _DT[x.dtype], spec.struct(), out.data_ptr(),
                           out.stride(0), ws.data_ptr(), ws.numel())
    _lib.check(lib.sd_probs(C.byref(a), C.c_void_p(_stream_ptr(x.device))), "sd_probs")
    return out.reshape(shape)


# --------------------------------------------------------------------------- verify
@dataclass
class VerifyOut:
    n_accepted: torch.Tensor      # int32 [B]
    next_token: torch.Tensor      # int64 [B]
    resample_mass: torch.Tensor   # fp32  [B]
    prune_drafter: torch.Tensor   # int32 [B]
    prune_target: torch.Tensor    # int32 [B]
    stop_index: torch.Tensor      # int32 [B]
    row_status: torch.Tensor      # int32 [B]
    words_used: torch.Tensor      # int64 [1]


def _verify_outputs(B: int, dev) -> VerifyOut:
    """VerifyOut's eight tensors as views of one device buffer: int64 fields first (8-byte aligned),
    then the 4-byte ones."""
    buf = torch.empty(8 * (B + 1) + 4 * 6 * B, dtype=torch.uint8, device=dev)
    nxt = buf[:8 * B].view(torch.long)
    used = buf[8 * B:8 * (B + 1)].view(torch.long)
    f4 = buf[8 * (B + 1):].view(torch.int32)
    i32 = [f4[k * B:(k + 1) * B] for k in range(6)]
    return VerifyOut(i32[0], nxt, i32[1].view(torch.float32), i32[2], i32[3], i32[4], i32[5], used)


def verify(target_rows: Sequence[torch.Tensor], draft_rows: Sequence[torch.Tensor], draft_tokens: torch.Tensor,
           rule: int, target_proc, draft_proc, noise, stop_tokens: Optional[torch.Tensor] = None,
           skip_sample_adjustment: bool = False, draft_is_probs: bool = False,
           active: Optional[torch.Tensor] = None, engine_state: Optional[dict] = None,
           sync_noise: bool = True, prof_events=None, row_base: int = 0,
           draft_row_stats: Optional[torch.Tensor] = None,
           draft_row_keep: Optional[torch.Tensor] = None,
           status_or: Optional[torch.Tensor] = None,
           row_counts: Optional[torch.Tensor] = None) -> VerifyOut:
    """One verify step for B sequences.

    target_rows: γ+1 (SPEC) or γ (ENGINE) tensors [B, V] — row t of every sequence;
    draft_rows:  γ tensors [B, V] (logits, or fp32 probabilities with draft_is_probs);
    draft_tokens: int64 [B, >=γ].  Under StreamNoise the torch generator is advanced by the
    words the kernels consumed, which needs one device->host read (sync_noise).
    row_base: global row id of this call's row 0 under PhiloxNoise (data-parallel shards draw
    what one call over the whole batch would draw for the same rows).
    draft_row_stats: optional fp32 [γ, B, 2] (or [γ, S>=B, 2]) device tensor — the drafter rows'
    (max, Σexp) as ``sample_rows(row_stats_out=...)`` returned them with the draws; the
    row-statistics pass then reads only the target rows.  Ignored for a top-k / nucleus drafter
    unless draft_row_keep comes with it.
    draft_row_keep: optional int32 [γ, S, 4] device tensor at draft_row_stats' row layout — the
    drafter rows' keep predicates as ``sample_rows(row_keep_out=...)`` returned them; the
    threshold search then covers the target rows only.
    status_or: optional int32 [1] device word that collects every row's SD_ROW_ERROR_MASK bits.
    row_counts: optional int64 [B, 2] contiguous device tensor; each call ADDS (accepted drafts,
    tokens emitted) to every row's pair (the A12 bookkeeping, kept on the device).
    """
    gamma = len(draft_rows)
    if rule == _lib.SD_RULE_SPEC and (active is not None or engine_state is not None):
        # the batch-1 rule has no finished rows and no engine state (sampling/speculative_decoding.py:
        # 129-171); refused on every path, so a γ > SD_MAX_GAMMA window cannot drop them silently
        raise ValueError("active / engine_state belong to the ENGINE rule (SD_RULE_ENGINE)")
    # user _process overrides: the kernels read the processed rows (processed_rows)
    target_rows = processed_rows(target_proc, list(target_rows))
    if not draft_is_probs:
        draft_rows = processed_rows(draft_proc, list(draft_rows))
    target_proc, draft_proc = proc_spec(target_proc), proc_spec(draft_proc)
    if gamma > _lib.SD_MAX_GAMMA:   # the reference takes any γ: windows of <= SD_MAX_GAMMA drafts (chunked.py)
        if prof_events is not None:
            raise ValueError("prof_events needs gamma <= SD_MAX_GAMMA")
        from .chunked import verify_chunked
        return verify_chunked(target_rows, draft_rows, draft_tokens, rule, target_proc, draft_proc, noise,
                              stop_tokens, skip_sample_adjustment, draft_is_probs, active, engine_state, sync_noise,
                              row_base, draft_row_stats, draft_row_keep, status_or, row_counts)
    if not 1 <= gamma:
        raise ValueError(f"gamma must be >= 1, got {gamma}")
    n_t = gamma + 1 if rule == _lib.SD_RULE_SPEC else gamma
    if len(target_rows) != n_t:
        raise ValueError(f"expected {n_t} target rows, got {len(target_rows)}")
    B, V = target_rows[0].shape
    dev = target_rows[0].device
    shards = _row_shards(B, noise)
    if shards is not None:   # more sequences than one call holds: row shards, one noise offset
        outs = []
        for r0, r1, nz in shards:
            es = None
            if engine_state is not None:
                es = dict(generated=engine_state["generated"][r0:r1], step=engine_state["step"],
                          finished=engine_state["finished"][r0:r1], accepted=engine_state["accepted"][r0:r1])
            outs.append(verify([t[r0:r1] for t in target_rows], [d[r0:r1] for d in draft_rows], draft_tokens[r0:r1],
                               rule, target_proc, draft_proc, nz, stop_tokens, skip_sample_adjustment, draft_is_probs,
                               None if active is None else active[r0:r1], es, sync_noise, None, row_base + r0,
                               None if draft_row_stats is None else draft_row_stats[:, r0:r1],
                               None if draft_row_keep is None else draft_row_keep[:, r0:r1], status_or,
                               None if row_counts is None else row_counts[r0:r1]))
        cat = {f: torch.cat([getattr(o, f) for o in outs]) for f in VerifyOut.__dataclass_fields__ if f != "words_used"}
        return VerifyOut(**cat, words_used=torch.zeros(1, dtype=torch.long, device=dev))
    tdt = target_rows[0].dtype
    # the batch stride is shared by a row set (it is irrelevant when B == 1)
    t_stride = target_rows[0].stride(0) if B > 1 else 0
    d_stride = draft_rows[0].stride(0) if B > 1 else 0
    for i, t in enumerate(target_rows):
        _require_rows(t, f"target_rows[{i}]", V)
        if t.shape[0] != B or t.dtype != tdt or (B > 1 and t.stride(0) != t_stride) or t.device != dev:
            raise ValueError("target rows must share batch, dtype, batch stride and device")
    for i, d in enumerate(draft_rows):
        _require_rows(d, f"draft_rows[{i}]", V)
        if d.shape[0] != B or d.dtype != draft_rows[0].dtype or (B > 1 and d.stride(0) != d_stride) \
                or d.device != dev:
            raise ValueError("draft rows must share batch, dtype, batch stride and device")
    if draft_is_probs and draft_rows[0].dtype != torch.float32:
        raise ValueError("draft probabilities must be fp32")
    if draft_tokens.dtype != torch.long or draft_tokens.dim() != 2 or draft_tokens.shape[0] != B \
            or draft_tokens.shape[1] < gamma or draft_tokens.stride(1) != 1 or draft_tokens.device != dev:
        raise ValueError(f"draft_tokens must be int64 [B, >={gamma}] on {dev}")
    tspec, dspec = proc_spec(target_proc), proc_spec(draft_proc)
    stops = stop_tokens if stop_tokens is not None else torch.empty(0, dtype=torch.long, device=dev)
    if stops.dtype != torch.long or stops.device != dev:
        raise ValueError("stop_tokens must be an int64 device tensor")
    if active is not None and (active.dtype not in (torch.uint8, torch.bool) or active.numel() != B):
        raise ValueError("active must be uint8/bool [B]")
    if draft_row_stats is not None:
        ds = draft_row_stats
        if ds.dtype != torch.float32 or ds.dim() != 3 or ds.shape[0] < gamma or ds.shape[1] < B \
                or ds.shape[2] != 2 or ds.stride(2) != 1 or ds.stride(1) != 2 or ds.device != dev:
            raise ValueError(f"draft_row_stats must be fp32 [>={gamma}, >={B}, 2] with (max, sum) pairs on {dev}")
    if draft_row_keep is not None:
        dk = draft_row_keep
        if draft_row_stats is None or dk.dtype != torch.int32 or dk.dim() != 3 or dk.shape[0] < gamma \
                or dk.shape[1] < B or dk.shape[2] != 4 or dk.stride(2) != 1 or dk.stride(1) != 4 \
                or dk.stride(0) // 4 != draft_row_stats.stride(0) // 2 or dk.device != dev:
            raise ValueError("draft_row_keep must be int32 [>=gamma, >=B, 4] at draft_row_stats' row stride, "
                             "and comes with draft_row_stats")

    # every output is written by the kernels (no fill launches); one allocation, typed views of it
    # (eight caching-allocator calls per verify were a visible share of an eager step's host time)
    out = _verify_outputs(B, dev)
    stochastic = rule == _lib.SD_RULE_ENGINE or tspec.stochastic
    need = B * (gamma + (2 * V if stochastic else 0))
    nz, keep = _noise_struct(noise, need, dev, row_base)
    ws = _workspace(lib.sd_verify_workspace_size(B, gamma, V), dev)

    a = _lib.sd_verify_args()
    a.batch, a.gamma, a.vocab, a.rule = B, gamma, V, rule
    for i, t in enumerate(target_rows):
        a.target_rows[i] = t.data_ptr()
    a.target_stride_b, a.target_dtype = t_stride, _DT[tdt]
    for i, d in enumerate(draft_rows):
        a.draft_rows[i] = d.data_ptr()
    a.draft_stride_b, a.draft_dtype = d_stride, _DT[draft_rows[0].dtype]
    a.draft_is_probs = int(draft_is_probs)
    a.draft_tokens, a.draft_tokens_stride_b = draft_tokens.data_ptr(), draft_tokens.stride(0)
    a.target_proc, a.draft_proc = tspec.struct(), dspec.struct()
    a.skip_sample_adjustment = int(skip_sample_adjustment)
    a.stop_tokens, a.n_stop = (stops.data_ptr() if stops.numel() else None), stops.numel()
    a.active = active.data_ptr() if active is not None else None
    a.noise = nz
    a.n_accepted, a.next_token, a.resample_mass = out.n_accepted.data_ptr(), out.next_token.data_ptr(), \
        out.resample_mass.data_ptr()
    a.prune_drafter, a.prune_target = out.prune_drafter.data_ptr(), out.prune_target.data_ptr()
    a.stop_index, a.row_status, a.words_used = out.stop_index.data_ptr(), out.row_status.data_ptr(), \
        out.words_used.data_ptr()
    if engine_state is not None:
        gen, fin, acc = engine_state["generated"], engine_state["finished"], engine_state["accepted"]
        if gen.dtype != torch.long or gen.shape[0] != B or gen.stride(1) != 1:
            raise ValueError("engine generated must be int64 [B, gen_len]")
        if engine_state["step"] + gamma > gen.shape[1]:
            raise ValueError("engine step window exceeds generated length")
        if fin.dtype not in (torch.uint8, torch.bool) or acc.dtype != torch.long:
            raise ValueError("engine finished must be uint8/bool, accepted int64")
        a.generated, a.generated_stride_b, a.step = gen.data_ptr(), gen.stride(0), int(engine_state["step"])
        a.finished, a.accepted_count = fin.data_ptr(), acc.data_ptr()
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel()
    if draft_row_stats is not None:
        a.draft_row_stats, a.draft_row_stats_stride = draft_row_stats.data_ptr(), draft_row_stats.stride(0) // 2
    if draft_row_keep is not None:
        a.draft_row_keep = draft_row_keep.data_ptr()
    a.status_or = _status_or_ptr(status_or, dev)
    if row_counts is not None:
        if row_counts.dtype != torch.long or tuple(row_counts.shape) != (B, 2) or not row_counts.is_contiguous() \
                or row_counts.device != dev:
            raise ValueError(f"row_counts must be a contiguous int64 [{B}, 2] tensor on {dev}")
        a.row_counts = row_counts.data_ptr()
    if prof_events is not None:   # (torch.cuda.Event, torch.cuda.Event[, repeats]) around the row-stats kernel
        a.prof_stats_begin, a.prof_stats_end = prof_events[0].cuda_event, prof_events[1].cuda_event
        a.prof_stats_repeat = int(prof_events[2]) if len(prof_events) > 2 else 1
    _lib.check(lib.sd_verify(C.byref(a), C.c_void_p(_stream_ptr(dev))), "sd_verify")
    if isinstance(noise, StreamNoise) and sync_noise:
        noise.consumed(used_dev=out.words_used)
    del keep
    return out


# --------------------------------------------------------------------------- n-gram verify (A11)
@dataclass
class NgramOut:
    n_accepted: torch.Tensor      # int32 [B]
    next_token: torch.Tensor      # int64 [B] (-1: a stop token among the accepted drafts)
    prune_target: torch.Tensor    # int32 [B]
    stop_index: torch.Tensor      # int32 [B]
    row_status: torch.Tensor      # int32 [B]
    filler_ids: Optional[torch.Tensor]   # int64 [B, γ'+1, K]
    words_used: torch.Tensor      # int64 [1]


def ngram_verify(target_rows: Sequence[torch.Tensor], draft_tokens: Optional[torch.Tensor], proc, noise,
                 stop_tokens: Optional[torch.Tensor] = None, filler_k: int = 0, sync_noise: bool = True,
                 row_base: int = 0, status_or: Optional[torch.Tensor] = None) -> NgramOut:
    """ngram_assisted/ngram_assisted.py:111-164 verify step for B sequences.

    target_rows: γ'+1 tensors [B, V] — rows 0..γ'-1 verify drafts 0..γ'-1, row γ' is the bonus row;
    draft_tokens: int64 [B, >=γ'] (None when γ' == 0).  Under StreamNoise the torch generator
    advances by the words the draws consumed (the reference's order), one device->host read."""
    spec = proc_spec(proc)
    target_rows = processed_rows(proc, list(target_rows))   # a user _process override (processed_rows)
    proc = spec
    gamma = len(target_rows) - 1
    if not 0 <= filler_k <= target_rows[0].shape[-1]:   # p.topk(k) raises for k > V as well
        raise ValueError(f"filler_k must be in [0, vocab = {target_rows[0].shape[-1]}]")
    if gamma > _lib.SD_MAX_GAMMA:   # the reference takes any γ: windows of <= SD_MAX_GAMMA drafts (chunked.py)
        from .chunked import ngram_verify_chunked
        return ngram_verify_chunked(target_rows, draft_tokens, proc, noise, stop_tokens, filler_k, sync_noise,
                                    row_base, status_or)
    if not 0 <= gamma:
        raise ValueError(f"gamma must be >= 0, got {gamma}")
    B, V = target_rows[0].shape
    dev = target_rows[0].device
    tdt = target_rows[0].dtype
    t_stride = target_rows[0].stride(0) if B > 1 else 0
    for i, t in enumerate(target_rows):
        _require_rows(t, f"target_rows[{i}]", V)
        if t.shape[0] != B or t.dtype != tdt or (B > 1 and t.stride(0) != t_stride):
            raise ValueError("target rows must share batch, dtype and batch stride")
    if gamma > 0:
        if draft_tokens is None or draft_tokens.dtype != torch.long or draft_tokens.shape[0] != B \
                or draft_tokens.shape[1] < gamma or draft_tokens.stride(1) != 1:
            raise ValueError("draft_tokens must be int64 [B, >=gamma] with a contiguous last axis")
        draft_tokens = draft_tokens.to(dev)
    if stop_tokens is None:
        stop_tokens = torch.empty(0, dtype=torch.long, device=dev)
    stop_tokens = stop_tokens.to(device=dev, dtype=torch.long).contiguous()
    i32 = dict(dtype=torch.int32, device=dev)
    out = NgramOut(torch.empty(B, **i32), torch.empty(B, dtype=torch.long, device=dev), torch.empty(B, **i32),
                   torch.empty(B, **i32), torch.empty(B, **i32),
                   torch.empty(B, gamma + 1, filler_k, dtype=torch.long, device=dev) if filler_k else None,
                   torch.empty(1, dtype=torch.long, device=dev))
    need = B * (gamma + 1) * 2 * V if spec.stochastic else 0
    nz, keep = _noise_struct(noise, need, dev, row_base)
    ws = _workspace(lib.sd_ngram_workspace_size(B, gamma, V), dev)
    a = _lib.sd_ngram_args()
    a.batch, a.gamma, a.vocab = B, gamma, V
    for i, t in enumerate(target_rows):
        a.target_rows[i] = t.data_ptr()
    a.target_stride_b, a.target_dtype = t_stride, _DT[tdt]
    a.draft_tokens = draft_tokens.data_ptr() if gamma > 0 else None
    a.draft_tokens_stride_b = draft_tokens.stride(0) if gamma > 0 else 0
    a.proc, a.stop_tokens, a.n_stop, a.filler_k = spec.struct(), stop_tokens.data_ptr(), stop_tokens.numel(), filler_k
    a.noise = nz
    a.n_accepted, a.next_token = out.n_accepted.data_ptr(), out.next_token.data_ptr()
    a.prune_target, a.stop_index = out.prune_target.data_ptr(), out.stop_index.data_ptr()
    a.row_status, a.words_used = out.row_status.data_ptr(), out.words_used.data_ptr()
    a.filler_ids = out.filler_ids.data_ptr() if filler_k else None
    a.filler_stride_b = (gamma + 1) * filler_k
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel()
    a.status_or = _status_or_ptr(status_or, dev)
    _lib.check(lib.sd_ngram_verify(C.byref(a), C.c_void_p(_stream_ptr(dev))), "sd_ngram_verify")
    if isinstance(noise, StreamNoise) and sync_noise:
        noise.consumed(used_dev=out.words_used)
    del keep
    return out
