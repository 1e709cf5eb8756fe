"""Batched speculative decoding on the fused HIP path.

Drop-in for engine/infer_engine.py:10-359 (``infer_batch`` -> ``run_batch_speculative`` ->
``batch_speculative_generate``), same signatures and return values, same bookkeeping.

Per window the drafter runs γ_w single-token forwards with its KV cache; each ``[B, V]``
drafter row is softmax-sampled by ``sd_sample`` (T=1, :241-246).  The target runs once on the
whole sequence (no cache, as the reference, :270-276).  ONE ``sd_verify`` call (rule ENGINE)
then replaces the per-row / per-draft Python loop with its ``.item()`` syncs (:279-336): the
fp64 ``u < min(1, p/q)`` test, the eos stop, the (p-q)+ residual resample (or the p fallback
when Σ <= 1e-12) and the in-place updates of ``generated`` / ``finished`` / accepted counts —
all on the device.  The host syncs once per window (``finished.all()``, :212).

Reference quirks reproduced: no bonus token; zero "gaps" after a
reject; trailing zeros stripped; padding counted as generated tokens; the drafter cache is
never pruned.  Not reproduced: the bf16 B>=2 crash at :254 (there is nothing to crash on).
"""
from __future__ import annotations

import time
from typing import List, Optional, Tuple

import torch

from .. import _lib
from ..noise import PhiloxNoise, StreamNoise, default_noise, noise_session
from ..ops import PLAIN_SOFTMAX, sample_rows, verify
from .batch_decode import decode_batch_with_chat_template
from .graph_window import EngineWindow
from .metrics import BatchMetrics, RequestMetrics


def infer_batch(ctx, prompts: List[str]) -> Tuple[Optional[BatchMetrics], Optional[BatchMetrics]]:
    """engine/infer_engine.py:10-96: format, tokenize, dispatch."""
    if ctx.chat:
        formatted = [ctx.tokenizer.apply_chat_template([{"role": "user", "content": p}],
                                                       add_generation_prompt=True, tokenize=False)
                     for p in prompts]
    else:
        formatted = prompts
    input_ids, attention_mask = decode_batch_with_chat_template(ctx.tokenizer, formatted,
                                                                max_length=ctx.max_batch_length, chat=False)
    drafter_device = getattr(ctx, "drafter_device", None)
    if ctx.spec and drafter_device is not None:
        input_ids, attention_mask = input_ids.to(drafter_device), attention_mask.to(drafter_device)
    if getattr(ctx, "reset_in_between", False) and getattr(ctx, "ngram", None) is not None:
        ctx.ngram.reset()
    target_device = getattr(ctx, "target_device", None)
    if not ctx.spec and getattr(ctx, "target_gen", False) and target_device is not None:
        input_ids, attention_mask = input_ids.to(target_device), attention_mask.to(target_device)
    if ctx.spec:
        return run_batch_speculative(ctx, input_ids, attention_mask, len(prompts)), None
    if getattr(ctx, "target_gen", False):
        return None, run_batch_target(ctx, input_ids, attention_mask, len(prompts))
    print("Warning: No inference method enabled")
    return None, None


def _fill_batch_metrics(bm: BatchMetrics, outputs, attention_mask, starts, firsts, rates=None) -> BatchMetrics:
    """engine/infer_engine.py:117-140 / :380-399: per-request metrics, the reference's formulas."""
    prompt_tokens = attention_mask.sum(dim=1).tolist()
    for i in range(bm.batch_size):
        r = RequestMetrics()
        r.start_time = starts[i]
        r.prompt_tokens = int(prompt_tokens[i])
        r.generated_tokens = len(outputs[i]) - r.prompt_tokens
        r.total_tokens = len(outputs[i])
        if rates is not None:
            r.acceptance_rate = rates[i] if i < len(rates) else 0.0
        r.end_time = bm.batch_end_time
        if firsts[i] is not None:
            r.first_token_time = firsts[i]
            r.ttft = firsts[i] - starts[i]
        else:
            r.ttft = (bm.batch_end_time - starts[i]) / max(r.generated_tokens, 1)
        r.total_latency = bm.batch_end_time - starts[i]
        bm.requests.append(r)
    return bm


def run_batch_speculative(ctx, input_ids: torch.Tensor, attention_mask: torch.Tensor,
                          batch_size: int) -> Optional[BatchMetrics]:
    """engine/infer_engine.py:99-146: run the batch and fill BatchMetrics (same rules)."""
    bm = BatchMetrics(batch_size=batch_size)
    bm.batch_start_time = time.time()
    starts = [time.time()] * batch_size
    firsts: List[Optional[float]] = [None] * batch_size

    def first_token(idx, t=None):
        if idx < batch_size and firsts[idx] is None:
            firsts[idx] = time.time() if t is None else t
    first_token.accepts_time = True   # the graph path reports the first draw's device completion time

    try:
        outputs, rates = batch_speculative_generate(ctx, input_ids, attention_mask, batch_size,
                                                    first_token_callback=first_token)
    except Exception as e:  # the reference's contract: report and return None (:144-146)
        print(f"Batch speculative decoding failed: {type(e).__name__}: {e}")
        return None
    bm.batch_end_time = time.time()
    return _fill_batch_metrics(bm, outputs, attention_mask, starts, firsts, rates)


def run_batch_target(ctx, input_ids: torch.Tensor, attention_mask: torch.Tensor,
                     batch_size: int) -> Optional[BatchMetrics]:
    """engine/infer_engine.py:362-404: the target-only baseline, same metrics rules."""
    bm = BatchMetrics(batch_size=batch_size)
    bm.batch_start_time = time.time()
    starts = [time.time()] * batch_size
    firsts: List[Optional[float]] = [None] * batch_size

    def first_token(idx):
        if idx < batch_size and firsts[idx] is None:
            firsts[idx] = time.time()

    try:
        outputs = batch_autoregressive_generate(ctx, input_ids, attention_mask, batch_size,
                                                first_token_callback=first_token)
    except Exception as e:
        print(f"Batch target generation failed: {type(e).__name__}: {e}")
        return None
    bm.batch_end_time = time.time()
    return _fill_batch_metrics(bm, outputs, attention_mask, starts, firsts)


@torch.no_grad()
def batch_autoregressive_generate(ctx, input_ids: torch.Tensor, attention_mask: torch.Tensor, batch_size: int,
                                  first_token_callback=None) -> List[torch.Tensor]:
    """engine/infer_engine.py:407-497: target-only decoding, the baseline the benchmark compares
    against (outside the verify/accept path, so plain torch ops on the device).

    Same token rule: ``multinomial(softmax(logits / T))`` when the processor has T > 0, else
    ``argmax(logits)``, over the rows still active; a row finishes on an end token; outputs are
    the unpadded prompt + generated tokens up to the last nonzero one.  The reference gathers
    and scatters per-row tuple caches for the active rows; here every row keeps its cache
    position (the cache object is whatever the model returns) and only active rows' tokens are
    taken, which gives the active rows the same logits.
    """
    dev = input_ids.device
    gen_len = int(ctx.gen_len)
    generated = torch.zeros(batch_size, gen_len, dtype=torch.long, device=dev)
    finished = torch.zeros(batch_size, dtype=torch.bool, device=dev)
    ends = torch.tensor(list(ctx.end_tokens), dtype=torch.long, device=dev)
    temperature = float(getattr(ctx.processor, "temperature", 0.0) or 0.0)
    past = None
    for step in range(gen_len):
        if bool(finished.all()):
            break
        if step == 0:
            out = ctx.target(input_ids, attention_mask=attention_mask, use_cache=True)
        else:
            cur = generated[:, step - 1:step]
            out = ctx.target(cur, attention_mask=torch.ones_like(cur), past_key_values=past, use_cache=True)
        past = out.past_key_values
        active = ~finished
        logits = out.logits[:, -1, :][active]
        if temperature > 0:
            nxt = torch.multinomial(torch.softmax(logits / temperature, dim=-1), 1).squeeze(-1)
        else:
            nxt = torch.argmax(logits, dim=-1)
        nxt = nxt.to(dev)
        idx = torch.nonzero(active).flatten()
        generated[idx, step] = nxt
        if first_token_callback is not None and step == 0:
            for i in idx.tolist():
                first_token_callback(i)
        finished[idx] |= torch.isin(nxt, ends)
    outputs = []
    gen_host = generated.cpu()
    lens = attention_mask.sum(dim=1).tolist()
    for i in range(batch_size):
        nz = torch.nonzero(gen_host[i], as_tuple=True)[0]
        tail = gen_host[i, :int(nz[-1]) + 1] if nz.numel() > 0 else torch.empty(0, dtype=torch.long)
        outputs.append(torch.cat([input_ids[i][:int(lens[i])], tail.to(dev)]))
    return outputs


@torch.no_grad()
def batch_speculative_generate(ctx, input_ids: torch.Tensor, attention_mask: torch.Tensor, batch_size: int,
                               first_token_callback=None) -> Tuple[List[torch.Tensor], List[float]]:
    """engine/infer_engine.py:149-359 with the accept loop fused into sd_verify."""
    dev = input_ids.device
    if dev.type != "cuda":
        raise RuntimeError("specdec_amd.batch_speculative_generate runs on the GPU (HIP); input_ids are on "
                           f"{dev}. There is no CPU path.")
    noise = default_noise()
    with noise_session(noise):   # STREAM: the generator state stays on the device for the loop
        return _batch_speculative_generate(noise, ctx, input_ids, attention_mask, batch_size, first_token_callback)


def _batch_speculative_generate(noise, ctx, input_ids, attention_mask, batch_size, first_token_callback):
    dev = input_ids.device
    target_device = getattr(ctx, "target_device", dev)
    B = batch_size
    gen_len, gamma = int(ctx.gen_len), int(ctx.gamma)
    # data-parallel shards (specdec_amd.engine.dp_runner): Philox noise is keyed by the GLOBAL row,
    # so a shard starting at global row `row_base` draws what one process over the whole batch draws
    row_base = int(getattr(ctx, "row_base", 0))
    generated = torch.zeros(B, gen_len, dtype=torch.long, device=dev)
    finished = torch.zeros(B, dtype=torch.uint8, device=dev)
    drafted = torch.zeros(B, dtype=torch.long, device=dev)
    accepted = torch.zeros(B, dtype=torch.long, device=dev)
    stops = torch.tensor(list(ctx.end_tokens), dtype=torch.long, device=dev)
    # every draw's and every verify's failed rows (SD_ROW_ERROR_MASK) OR into one device word, read
    # where the loop already syncs; set bits raise as torch.multinomial does in the reference
    # (:246,321-325), and run_batch_speculative then returns None (:144-146)
    err = torch.zeros(1, dtype=torch.int32, device=dev)

    if isinstance(noise, PhiloxNoise) and getattr(ctx, "drafter_step", None) is not None \
            and getattr(ctx, "target_rows", None) is not None:
        # capturable drafter / target steps: the whole window replays from one hipGraph (graph_window.py)
        win = EngineWindow(ctx.drafter_step, ctx.target_rows, input_ids[:, -1], gamma, gen_len, ctx.end_tokens,
                           noise, row_base=row_base)
        # TTFT (:261-263: after step 0's first draft): the first draw's completion on the device,
        # placed on the host clock by one event synchronised before the window is queued — no sync
        # inside the loop.  A callback without a time argument is called after the run.
        ref = torch.cuda.Event(enable_timing=True)
        win.first_draw_event = torch.cuda.Event(enable_timing=True)
        if first_token_callback is not None:
            ref.record()
            ref.synchronize()
        t_ref = time.time()
        try:
            win.run()
        finally:
            noise.offset = win.o0 + win.windows_run * (gamma + 1)         # the calls the windows consumed
        outs = _collect(input_ids, win.generated, win.drafted, win.accepted, B, win.err)
        if first_token_callback is not None and win._first_recorded:     # gen_len 0: no first token
            t_first = t_ref + ref.elapsed_time(win.first_draw_event) / 1e3
            for idx in range(B):                                          # step 0: every row is active
                if getattr(first_token_callback, "accepts_time", False):
                    first_token_callback(idx, t_first)
                else:
                    first_token_callback(idx)
        return outs

    # each draw also returns its row's (max, Σexp) — free in the one-pass draws of both noise modes
    # (k_draw_lean, k_draw_stream) — so the verify's statistics pass reads only target rows
    stash = True
    dstats = torch.empty(max(gamma, 1), B, 2, dtype=torch.float32, device=dev) if stash else None
    past = ctx.drafter(input_ids, attention_mask=attention_mask, use_cache=True).past_key_values   # :206
    # Philox: the all-finished test of :212 is read one window late (pinned copy behind an event), so
    # the host queues the next window while the GPU runs this one.  A window over all-finished rows
    # changes nothing, so the outputs are the reference's.  STREAM keeps the exact check: such a
    # window would still consume generator words.
    probe = _FinishedProbe(finished, err) if isinstance(noise, PhiloxNoise) else None
    # Opt-in (ctx.cached_target = True): the target keeps a KV cache instead of re-encoding the whole
    # sequence every window (:269-273).  A window's positions are final only after its verify (the
    # rejected drafts are zeroed, :332-336), so the cache is cropped back to the start of the previous
    # window and each forward feeds that window's final tokens plus the new drafts: the same token
    # sequence and positions as the reference's full forward, its logits up to rounding.  Default: off
    # (the reference's uncached forward).
    cached = bool(getattr(ctx, "cached_target", False))
    t_past, t_valid = None, 0                                             # cache and its valid length
    step = 0
    while step < gen_len:                                                 # :211
        if probe is not None:
            if probe.done():
                break
        else:                                                             # one read: finished.all() and err
            done, bits = torch.stack([(finished != 0).all().to(torch.int32), err[0]]).tolist()
            _lib.raise_row_error(bits, "batch_speculative_generate")
            if done:
                break
        gw = min(gamma, gen_len - step)                                   # :216
        draft_tokens = torch.zeros(B, gw, dtype=torch.long, device=dev)
        active = finished == 0
        rows = []
        for d in range(gw):                                               # :224 (finished is constant here)
            if d == 0:
                prev = generated[:, step - 1] if step > 0 else input_ids[:, -1]
            else:
                prev = generated[:, step + d - 1]
            out = ctx.drafter(prev.unsqueeze(1), past_key_values=past, use_cache=True)   # :239
            logits = out.logits[:, -1, :]
            past = out.past_key_values
            if d == 0 and isinstance(noise, StreamNoise):
                # the window's words in one generation: γ_w draws of 2·B·V, the verify's <= B·(γ_w + 2V)
                V = logits.shape[-1]
                noise.reserve(gw * 2 * B * V + B * (gw + 2 * V), dev, known=gw * 2 * B * V)
            samples, _, _ = sample_rows(logits, PLAIN_SOFTMAX, noise,     # :241-246 softmax + multinomial
                                        row_base=row_base, row_stats_out=dstats[d] if stash else None,
                                        status_or=err)
            samples.clamp_(0, logits.shape[-1] - 1)   # a failed row's -1 (raised at the next read of err) never reaches a forward
            rows.append(logits)
            draft_tokens[:, d] = torch.where(active, samples, draft_tokens[:, d])          # :252
            generated[:, step + d] = torch.where(active, samples, generated[:, step + d])  # :257
            drafted += active.long()                                      # :258
            if first_token_callback is not None and d == 0 and step == 0:
                for idx in range(B):                                      # step 0: every row is active
                    first_token_callback(idx)
        verify_ids = torch.cat([input_ids, generated[:, :step + gw]], dim=1).to(target_device)  # :269-270
        L = verify_ids.shape[1]
        if cached:
            if t_past is not None:
                t_past.crop(t_valid)                                      # drop the previous window's drafts
            out = ctx.target(verify_ids[:, t_valid:], past_key_values=t_past, use_cache=True)
            t_logits, t_past, first = out.logits, out.past_key_values, t_valid
            t_valid = L - gw                                              # this window is final after its verify
        else:
            t_logits, first = ctx.target(verify_ids).logits, 0           # :273
        trows = [t_logits[:, L - gw - 1 + t - first, :] for t in range(gw)]   # :275 logits[:, -(γ+1):-1]
        if any(r.device != t_logits.device for r in rows):
            rows = [r.to(t_logits.device) for r in rows]
        verify(trows, rows, draft_tokens, _lib.SD_RULE_ENGINE, PLAIN_SOFTMAX, PLAIN_SOFTMAX, noise, stops,
               active=active.to(torch.uint8),
               engine_state=dict(generated=generated, step=step, finished=finished, accepted=accepted),
               row_base=row_base, draft_row_stats=dstats[:gw] if stash and t_logits.device == dev else None,
               status_or=err)
        if probe is not None:
            probe.record()
        step += gw                                                        # :338
    return _collect(input_ids, generated, drafted, accepted, B, err)


class _FinishedProbe:
    """finished.all() and the error word of the window before last, without a sync on the window
    just queued.  The lag costs at most one extra window after the last row finished (γ drafter
    forwards and one target forward over rows that are all inactive: they draw nothing into the
    outputs, so the tokens are the reference's; the Philox call offsets advance by that window's
    γ + 1 calls).  A failed row raises one window late; its -1 tokens were clamped before any
    forward saw them, and the batch's outputs are discarded with the exception."""

    def __init__(self, finished: torch.Tensor, err: torch.Tensor):
        self.finished, self.err = finished, err
        self.flags = [torch.zeros(2, dtype=torch.int32).pin_memory() for _ in range(2)]
        self.events: List[Optional[torch.cuda.Event]] = [None, None]
        self.w = 0

    def record(self) -> None:
        i = self.w % 2
        both = torch.cat([(self.finished != 0).all().to(torch.int32).reshape(1), self.err])
        self.flags[i].copy_(both, non_blocking=True)
        self.events[i] = torch.cuda.Event()
        self.events[i].record()
        self.w += 1

    def done(self) -> bool:
        ev = self.events[self.w % 2]                                      # window w - 2
        if ev is None:
            return False
        ev.synchronize()
        done, bits = self.flags[self.w % 2].tolist()
        _lib.raise_row_error(bits, "batch_speculative_generate")
        return bool(done)


def _collect(input_ids, generated, drafted, accepted, B, err=None):
    """engine/infer_engine.py:341-357: prompt + generated up to the last nonzero token, per-row rates.
    err: the loop's error word — a failed row raises here at the latest (torch raises in the
    reference's loop, :246,321-325)."""
    dev = input_ids.device
    if err is not None:
        _lib.raise_row_error(int(err.item()), "batch_speculative_generate")
    gen_host = generated.cpu()
    drafted_h, accepted_h = drafted.tolist(), accepted.tolist()
    outputs, rates = [], []
    for i in range(B):                                                    # :341-357
        nz = torch.nonzero(gen_host[i], as_tuple=True)[0]
        tail = gen_host[i, :int(nz[-1]) + 1] if nz.numel() > 0 else torch.empty(0, dtype=torch.long)
        outputs.append(torch.cat([input_ids[i], tail.to(dev)]))
        t, a = drafted_h[i], accepted_h[i]
        rates.append(a / t if t > 0 else 0.0)
    return outputs, rates
