"""The engine window as a replayable hipGraph (sync-free batched engine step).

engine/infer_engine.py:211-338 runs, per window of γ positions: γ drafter forwards, each
followed by a softmax + multinomial draw of its ``[B, V]`` row (:238-258), one target forward
(:265-276) and the per-row accept / residual loop with its state updates (:279-336).  Here the
whole window — draws, verify and state update — is captured ONCE into a hipGraph and replayed
per window, with nothing on the host between windows:

* the drafter and target forwards are caller-supplied capturable callables (static shapes,
  device-only work — e.g. a model with a static KV cache, or the seeded banks of the tests):
    ``drafter_step(prev [B] int64, d, step_dev) -> logits [B, V]`` and
    ``target_rows(tokens [B, γ] int64, step_dev) -> logits [B, γ, V]``, where ``tokens`` are the
    inputs at the γ verified positions (the window's previous token, then drafts 0..γ-2) —
    the rows ``logits[:, -(γ+1):-1]`` the reference takes from its full forward (:275);
* draws: ``sd_sample`` (k_draw, Philox) writes each draft straight into the window buffer;
  the verify (``sd_verify`` rule ENGINE) applies :307-336 in place on that buffer;
* the window's position lives on the device (``step_dev``): the window buffer is scattered
  into ``generated[:, step:step+γ]`` by a device index, and the Philox counter base
  (``PhiloxNoise.offset_dev``) moves by the window's γ+1 calls inside the graph, so every
  replay draws fresh noise — the SAME noise the eager drop-in loop draws for that window
  (calls take offsets o0 + w(γ+1) + i in both).

Early exit needs no sync either: after each window a copy of ``finished.all()`` goes to pinned
host memory behind an event, and the host reads it one window late.  A window run after every
row finished changes nothing (inactive rows draw into zeros, the verify skips them), so the
outputs are those of the reference's loop, which stops at the first all-finished check (:212).
A trailing window shorter than γ (gen_len % γ) runs eagerly with the same noise offsets.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch

from .. import _lib
from ..noise import PhiloxNoise
from ..ops import PLAIN_SOFTMAX, sample_rows, verify


class EngineWindow:
    """Replays engine windows of γ positions from a captured hipGraph (see the module docstring).

    After ``run()``: ``generated`` [B, gen_len], ``drafted`` / ``accepted`` [B] hold what the
    reference's loop holds at its end (engine/infer_engine.py:341-357 reads them)."""

    def __init__(self, drafter_step: Callable, target_rows: Callable, last_prompt_token: torch.Tensor, gamma: int,
                 gen_len: int, end_tokens, noise: PhiloxNoise, row_base: int = 0):
        if not isinstance(noise, PhiloxNoise):
            raise TypeError("EngineWindow replays Philox noise (the parity STREAM mode is host-ordered)")
        dev = last_prompt_token.device
        if dev.type != "cuda":
            raise RuntimeError("EngineWindow runs on the GPU (HIP)")
        self.drafter_step, self.target_rows = drafter_step, target_rows
        self.B, self.gamma, self.gen_len = last_prompt_token.shape[0], int(gamma), int(gen_len)
        self.row_base, self.dev = int(row_base), dev
        B, g = self.B, self.gamma
        self.generated = torch.zeros(B, self.gen_len, dtype=torch.long, device=dev)
        self.finished = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.drafted = torch.zeros(B, dtype=torch.long, device=dev)
        self.accepted = torch.zeros(B, dtype=torch.long, device=dev)
        self.stops = torch.tensor(list(end_tokens), dtype=torch.long, device=dev)
        self.last = last_prompt_token.to(torch.long).clone()        # generated[:, step-1] (:217-219)
        self.step_dev = torch.zeros(1, dtype=torch.long, device=dev)
        self.win = torch.zeros(B, g, dtype=torch.long, device=dev)
        self.inputs = torch.zeros(B, g, dtype=torch.long, device=dev)
        self.dstats = torch.empty(g, B, 2, dtype=torch.float32, device=dev)
        self.cols = torch.arange(g, dtype=torch.long, device=dev)
        self.idx = torch.empty(g, dtype=torch.long, device=dev)
        self.all_done = torch.zeros(1, dtype=torch.uint8, device=dev)
        # failed rows of every draw / verify (SD_ROW_ERROR_MASK), read with the finished flag
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.done_err = torch.zeros(2, dtype=torch.int32, device=dev)   # [all finished, err] per window
        self.o0 = noise.offset
        od = noise.offset_dev if noise.offset_dev is not None else torch.zeros(1, dtype=torch.long, device=dev)
        self.noise = PhiloxNoise(noise.seed, self.o0, od)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.windows_run = 0
        self.on_window: Optional[Callable[[int], None]] = None   # host hook after window w is queued
        self.first_draw_event: Optional[torch.cuda.Event] = None    # recorded after the first window's draw 0
        self._first_recorded = False

    # ---------------------------------------------------------------- one window, device-only
    def _window(self, gw: int) -> None:
        B = self.B
        self.noise.offset = self.o0                      # host offsets o0..o0+gw; the device base moves
        active = self.finished == 0                      # :213 (constant within the window)
        win = self.win[:, :gw]
        win.zero_()
        rows: List[torch.Tensor] = []
        prev = self.last
        for d in range(gw):                              # :224-258
            logits = self.drafter_step(prev, d, self.step_dev)
            samples, _, _ = sample_rows(logits, PLAIN_SOFTMAX, self.noise, row_base=self.row_base,
                                        row_stats_out=self.dstats[d], status_or=self.err)
            samples.clamp_(0, logits.shape[-1] - 1)      # a failed row's -1 never reaches a forward
            if d == 0 and self.first_draw_event is not None and not self._first_recorded \
                    and not torch.cuda.is_current_stream_capturing():
                self.first_draw_event.record()           # TTFT: the first draft of the first window
                self._first_recorded = True
            torch.where(active, samples, torch.zeros_like(samples), out=self.win[:, d])   # :252,:257
            rows.append(logits)
            prev = self.win[:, d]
        self.drafted.add_(active.long() * gw)            # :258
        ins = self.inputs[:, :gw]
        ins[:, 0].copy_(self.last)
        if gw > 1:
            ins[:, 1:].copy_(win[:, :gw - 1])
        t_logits = self.target_rows(ins, self.step_dev)   # [B, gw, V]: logits[:, -(gw+1):-1] (:275)
        trows = [t_logits[:, t, :] for t in range(gw)]
        # the window buffer is `generated` for the kernel (step 0): :307-336 applied in place
        verify(trows, rows, win, _lib.SD_RULE_ENGINE, PLAIN_SOFTMAX, PLAIN_SOFTMAX, self.noise, self.stops,
               active=active.to(torch.uint8),
               engine_state=dict(generated=self.win, step=0, finished=self.finished, accepted=self.accepted),
               row_base=self.row_base, draft_row_stats=self.dstats[:gw], status_or=self.err)
        idx = self.idx[:gw]
        torch.add(self.cols[:gw], self.step_dev, out=idx)
        self.generated.index_copy_(1, idx, win)          # generated[:, step:step+gw] = window
        self.last.copy_(win[:, gw - 1])
        self.step_dev.add_(gw)
        self.noise.advance_device(gw + 1)                # γ draws + 1 verify consumed
        self.all_done.copy_((self.finished != 0).all().to(torch.uint8).reshape(1))
        self.done_err[0].copy_(self.all_done[0])
        self.done_err[1].copy_(self.err[0])

    def capture(self) -> None:
        """Capture one full window.  Capturing records the launches without running them, so the
        decode state is untouched; run() captures after its eager first window has sized the
        workspaces and the allocator's blocks."""
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._window(self.gamma)

    def run(self, lag: int = 2, use_graph: bool = True) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Decode gen_len positions; returns (generated, drafted, accepted).  The all-finished
        flag of window w is read before window w + lag is launched (lag >= 1): the host keeps
        lag - 1 windows queued ahead of the GPU.  use_graph=False runs every window eagerly (the
        same launches; the parity reference for the replays)."""
        g = self.gamma
        lag = max(int(lag), 1)
        full, tail = divmod(self.gen_len, g)
        flags = [torch.zeros(2, dtype=torch.int32).pin_memory() for _ in range(lag)]
        events: List[Optional[torch.cuda.Event]] = [None] * lag
        self.first_window_done: Optional[torch.cuda.Event] = None

        def done_before(w: int) -> bool:   # the flags of window w - lag, if it ran; a failed row raises
            ev = events[w % lag]
            if ev is None:
                return False
            ev.synchronize()
            done, bits = flags[w % lag].tolist()
            _lib.raise_row_error(bits, "EngineWindow")
            return bool(done)

        for w in range(full):
            if done_before(w):                           # every row finished (:212)
                return self.generated, self.drafted, self.accepted
            if w == 0 or not use_graph:
                self._window(g)                          # eager first window
            else:
                if self.graph is None:
                    self.capture()
                self.graph.replay()
            self.windows_run += 1
            flags[w % lag].copy_(self.done_err, non_blocking=True)
            events[w % lag] = torch.cuda.Event()
            events[w % lag].record()
            if w == 0:
                self.first_window_done = events[0]
            if self.on_window is not None:
                self.on_window(w)
        if tail:
            torch.cuda.current_stream(self.dev).synchronize()
            _lib.raise_row_error(int(self.err.item()), "EngineWindow")
            if not bool(self.all_done.item()):
                self._window(tail)
                self.windows_run += 1
        return self.generated, self.drafted, self.accepted
