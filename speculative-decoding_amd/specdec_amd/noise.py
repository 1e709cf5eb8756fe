"""Noise sources for the verify / sample kernels.

StreamNoise  (parity mode)  feeds the kernels the raw mt19937 words of torch's CPU generator
             (torch.default_generator unless one is given), so every torch.rand / multinomial
             draw the reference makes is reproduced bit-exactly, in the reference's order, on
             the GPU.  The words are made ON THE GPU from the generator's state
             (sd_mt19937_generate: jump-ahead substreams, csrc/mt_device.hip) and the state is
             moved by exactly the words the kernels consumed (sd_mt19937_commit, device-side
             count); SPECDEC_STREAM_DEVICE=0 makes them on the host instead (sd_mt19937_fill).
PhiloxNoise  (perf mode)    counter-based Philox4x32-10 inside the kernels: no host work, no
             noise bytes in HBM; statistically equivalent, not stream-identical.

The mode used by the drop-in entry points is chosen by ``set_noise_mode`` or the
SPECDEC_NOISE environment variable (``stream`` | ``philox``; default ``stream``).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import lib


_DEVICE_GEN = os.environ.get("SPECDEC_STREAM_DEVICE", "1") != "0"
# Words per device substream.  Jump-ahead cost grows with the number of substreams (~0.33 us each),
# generation time with their length (one workgroup per substream, ~0.47 ns per word), and a
# substream per CU at most keeps every generation round uncontended (a CU running two is
# VALU-bound: 487 vs 292 ns per round, profiles/r3b_mt_gen_bench.txt).  So the stride is the
# smallest multiple of 64 Ki words that needs at most kMaxSubstreams substreams (an engine step's
# 41 M words at B = 32, V = 128256: 192 Ki words, 209 substreams).  SPECDEC_MT_STRIDE pins it.
_STRIDE_ENV = os.environ.get("SPECDEC_MT_STRIDE")
# steps per pipelined pool (StreamNoise.reserve(..., known=...) in a session); 0 = no pipeline
_PIPE_STEPS = int(os.environ.get("SPECDEC_STREAM_PIPELINE", "16"))
# HBM the two pools may take (words): fewer steps per pool for big steps, no pipeline beyond it
_PIPE_WORD_BUDGET = 1 << 30   # 4 GiB per pool


def pipeline_steps_for(n: int, known: int, steps: int) -> int:
    """Steps per pool for steps of n words (known host-known): the configured count, cut so a pool
    (steps + 2 steps' worst case + the verifies' slack) fits the budget; 0 when even one step does not."""
    w = n - known
    while steps > 0 and (steps + 2) * n + steps * w > _PIPE_WORD_BUDGET:
        steps -= 1
    return steps
MT_STRIDE = int(_STRIDE_ENV) if _STRIDE_ENV else 65536
MT_MAX_SUBSTREAMS = 240


def mt_stride(n_words: int) -> int:
    if _STRIDE_ENV:
        return MT_STRIDE
    per = -(-int(n_words) // MT_MAX_SUBSTREAMS)
    return max(MT_STRIDE, -(-per // 65536) * 65536)
_JUMP: Dict[Tuple[torch.device, int], torch.Tensor] = {}


def jump_table(device, stride: int, count: int) -> torch.Tensor:
    """Device copy of the jump polynomials for substreams 1..>=count of `stride` words (host
    computed once by libspecdec, grown geometrically)."""
    dev = torch.device(device)
    key = (dev, stride)
    t = _JUMP.get(key)
    if t is None or t.shape[0] < count:
        n = max(count, 2 * (t.shape[0] if t is not None else 0), 16)
        host = np.zeros((n, _lib.SD_MT_JUMP_WORDS), dtype=np.uint64)
        _lib.check(lib.sd_mt19937_jump_table(stride, n, host.ctypes.data), "sd_mt19937_jump_table")
        t = torch.from_numpy(host.view(np.int64)).to(dev)
        _JUMP[key] = t
    return t


def _mt_generate(state: torch.Tensor, words: torch.Tensor, n: int, ws_box: list, stream) -> None:
    """sd_mt19937_generate: the n words after `state` into words[:n] on `stream` (ws_box[0]: a
    workspace tensor grown in place, one per stream)."""
    dev = words.device
    stride = mt_stride(n)
    S = (n + stride - 1) // stride
    table = jump_table(dev, stride, max(S - 1, 1))
    need = lib.sd_mt19937_generate_workspace_size(n, stride)
    if ws_box[0] is None or ws_box[0].numel() < need:
        ws_box[0] = torch.empty(need + need // 4, dtype=torch.uint8, device=dev)
    a = _lib.sd_mt_generate_args(state.data_ptr(), table.data_ptr(), table.shape[0], stride, words.data_ptr(), n,
                                 ws_box[0].data_ptr(), ws_box[0].numel())
    _lib.check(lib.sd_mt19937_generate(C.byref(a), C.c_void_p(stream.cuda_stream)), "sd_mt19937_generate")


def _mt_commit(state: torch.Tensor, words: torch.Tensor, n_generated: int, used: int, used_dev, stream) -> None:
    """sd_mt19937_commit: move `state` past used + *used_dev of the n_generated words after it."""
    _lib.check(lib.sd_mt19937_commit(state.data_ptr(), words.data_ptr(), n_generated,
                                     used_dev.data_ptr() if used_dev is not None else None, int(used), None,
                                     C.c_void_p(stream.cuda_stream)), "sd_mt19937_commit")


class _Pool:
    """One pipelined pool: `cap` generator words (+ 624 of slack for commits) from the position whose
    generator state is `state`; `ready` is recorded on the generation stream once they are written."""

    def __init__(self, words: torch.Tensor, cap: int):
        self.words, self.cap = words, cap
        self.state: Optional[torch.Tensor] = None
        self.ready: Optional[torch.cuda.Event] = None
        # the anchor, in the previous pool's coordinates: host part snap_host + K, device part a_dev
        self.snap_host = 0
        self.K = 0
        self.a_dev: Optional[torch.Tensor] = None
        self.dev_since = 0     # upper bound of the device-counted words since the anchor snapshot


class _CudaBackend:
    """The stream / event / generation primitives the pipeline runs on (a CPU test substitutes a
    fake with the same methods: tests/test_stream_pipeline_cpu.py)."""

    @staticmethod
    def new_stream(dev):
        return torch.cuda.Stream(dev)

    @staticmethod
    def current(dev):
        return torch.cuda.current_stream(dev)

    @staticmethod
    def event_on(stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    @staticmethod
    def wait(stream, ev):
        stream.wait_event(ev)

    @staticmethod
    def on(stream):
        return torch.cuda.stream(stream)

    @staticmethod
    def keep(t, stream):
        t.record_stream(stream)

    generate = staticmethod(_mt_generate)
    commit = staticmethod(_mt_commit)


class _Pipeline:
    """STREAM words generated ahead, on a side stream, while the calls consume the current pool
    (DESIGN §4 "STREAM pool pipeline").  A session's steps (``reserve(n, known=...)``: n words at
    most, `known` of them host-known — the draws) consume consecutive generator positions; the call
    start inside the current pool is host_off + *rel_dev (the kernels add both, ABI 11), rel_dev
    summing the verifies' device counts, so nothing is read back.  The next pool is generated from
    an anchor no later than where the current pool will be left: the position at the switch into
    the current pool plus the host-known words of `steps` steps; it holds `steps` + 2 steps' worst
    case plus the verifies' slack, so the switch (after `steps` steps) always lands inside it and
    the pool after it is generated meanwhile, on the side stream, behind an event."""

    def __init__(self, dev: torch.device, state: torch.Tensor, n: int, known: int, steps: int, be=_CudaBackend):
        self.dev, self.be = dev, be
        self.steps = steps
        self.n, self.known = n, known
        # a pool is entered up to one step's host words plus `steps` verifies' slack past its anchor,
        # and serves `steps` steps (the switch is taken as soon as the walk passes the next anchor)
        self.cap = (steps + 2) * n + steps * (n - known)
        self.side = be.new_stream(dev)
        self.ws_main, self.ws_side = [None], [None]
        bufs = [torch.empty(self.cap + 624, dtype=torch.int32, device=dev) for _ in range(2)]
        self.pools = [_Pool(b, self.cap) for b in bufs]
        self.i = 0                                   # the current pool's buffer
        cur = self.pools[0]
        cur.state = state.clone()
        be.generate(cur.state, cur.words, self.cap + 624, self.ws_main, be.current(dev))   # the first pool: in line
        self.host_off = 0
        self.rel_dev = torch.zeros(1, dtype=torch.long, device=dev)
        self.dev_hi = 0                              # upper bound of *rel_dev
        self.nxt: Optional[_Pool] = None
        self._enqueue_next()

    @property
    def cur(self) -> _Pool:
        return self.pools[self.i]

    def _enqueue_next(self) -> None:
        """Generate the other buffer's pool on the side stream, anchored at host_off + K + *rel_dev
        (snapshot) of the current pool, K = the host-known words of `steps` steps."""
        be = self.be
        nxt = self.pools[1 - self.i]
        nxt.snap_host, nxt.K = self.host_off, self.steps * self.known
        nxt.a_dev = self.rel_dev.clone()             # snapshot (stream-ordered on the main stream)
        nxt.dev_since = 0
        nxt.state = self.cur.state.clone()
        # the event also orders the buffer's last readers (the pool before the current one) first
        be.wait(self.side, be.event_on(be.current(self.dev)))
        with be.on(self.side):
            be.keep(nxt.a_dev, self.side)
            be.keep(nxt.state, self.side)
            be.commit(nxt.state, self.cur.words, self.cap + 624, nxt.snap_host + nxt.K, nxt.a_dev, self.side)
            be.generate(nxt.state, nxt.words, self.cap + 624, self.ws_side, self.side)
            nxt.ready = be.event_on(self.side)
        self.nxt = nxt

    def fits(self, n: int) -> bool:
        return self.host_off + self.dev_hi + n <= self.cap

    def switch(self, n: int) -> bool:
        """Move to the next pool if the walk has passed its anchor and it holds n more words."""
        nxt = self.nxt
        if nxt is None or self.host_off < nxt.snap_host + nxt.K:
            return False
        new_host = self.host_off - nxt.snap_host - nxt.K
        if new_host + nxt.dev_since + n > self.cap:
            return False
        self.be.wait(self.be.current(self.dev), nxt.ready)
        self.rel_dev.sub_(nxt.a_dev)                 # exact, on the device: >= 0, <= nxt.dev_since
        self.host_off, self.dev_hi = new_host, nxt.dev_since
        self.i = 1 - self.i
        self.nxt = None
        self._enqueue_next()
        return True

    def take(self, n: int):
        """(pool words, host offset, device offset) for a call of up to n words, or None.  Moves to
        the next pool as soon as the walk has passed its anchor (so every pool is entered within one
        step of it), else stays while the call fits."""
        if not self.switch(n) and not self.fits(n):
            return None
        return self.cur.words, self.host_off, self.rel_dev

    def consumed(self, count: Optional[int], used_dev: Optional[torch.Tensor], worst: int) -> None:
        if used_dev is None:
            self.host_off += int(count or 0)
        else:
            self.rel_dev.add_(used_dev.view(1))
            self.dev_hi += worst
            if self.nxt is not None:
                self.nxt.dev_since += worst

    def final_state(self) -> torch.Tensor:
        """The generator state after every consumed word (device; stream-ordered)."""
        st = self.cur.state.clone()
        self.be.commit(st, self.cur.words, self.cap + 624, self.host_off, self.rel_dev, self.be.current(self.dev))
        return st


class _DeviceMT:
    """The generator state on one device (sd_mt_state) plus the word buffer and workspace of the
    last fill.  Fills and commits are stream-ordered; nothing here syncs except pull()."""

    def __init__(self, device, torch_state: torch.Tensor):
        self.device = torch.device(device)
        host = _lib.sd_mt_state()
        st = torch_state.contiguous()
        _lib.check(lib.sd_mt19937_state_from_torch(st.data_ptr(), st.numel(), C.byref(host)),
                   "sd_mt19937_state_from_torch")
        raw = np.frombuffer(bytes(host), dtype=np.uint8).copy()
        self._loaded = raw.tobytes()
        self.state = torch.from_numpy(raw).to(self.device)
        self.words = torch.empty(0, dtype=torch.int32, device=self.device)
        self.ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.n_generated = 0

    def fill(self, n_words: int) -> torch.Tensor:
        """The next n_words words (plus one block of slack for the commit), state unchanged."""
        n = max(int(n_words), 1) + 624
        if self.words.numel() < n:
            self.words = torch.empty(n + n // 4, dtype=torch.int32, device=self.device)
        stride = mt_stride(n)
        S = (n + stride - 1) // stride
        table = jump_table(self.device, stride, max(S - 1, 1))
        need = lib.sd_mt19937_generate_workspace_size(n, stride)
        if self.ws.numel() < need:
            self.ws = torch.empty(need + need // 4, dtype=torch.uint8, device=self.device)
        a = _lib.sd_mt_generate_args(self.state.data_ptr(), table.data_ptr(), table.shape[0], stride,
                                     self.words.data_ptr(), n, self.ws.data_ptr(), self.ws.numel())
        _lib.check(lib.sd_mt19937_generate(C.byref(a), C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "sd_mt19937_generate")
        self.n_generated = n
        return self.words[:n]

    def commit(self, count: Optional[int] = None, used_dev: Optional[torch.Tensor] = None) -> None:
        """Move the state past `count` (host) + *used_dev (device) words of the last fill."""
        used_ptr = used_dev.data_ptr() if used_dev is not None else None
        _lib.check(lib.sd_mt19937_commit(self.state.data_ptr(), self.words.data_ptr(), self.n_generated, used_ptr,
                                         int(count or 0), None,
                                         C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "sd_mt19937_commit")

    def pull(self, gen: torch.Generator) -> None:
        """Write the device state back into the torch generator (one device->host copy).  A state
        that consumed nothing is left as torch holds it: a freshly seeded torch state (left=1,
        next=0, block not yet twisted) and its converted form (tau0=624) are the same stream but
        not the same bytes."""
        raw = self.state.cpu().numpy().tobytes()
        if raw == self._loaded:
            return
        host = _lib.sd_mt_state.from_buffer_copy(raw)
        st = gen.get_state().clone()
        _lib.check(lib.sd_mt19937_state_to_torch(C.byref(host), st.data_ptr(), st.numel()),
                   "sd_mt19937_state_to_torch")
        gen.set_state(st)


class StreamNoise:
    """Parity noise: torch's CPU generator words (torch.default_generator unless one is given).

    device_generation (default on; SPECDEC_STREAM_DEVICE=0 turns it off): the words are made on
    the GPU by libspecdec's mt19937 kernels from the generator's state, and the state moves on
    the device by exactly the words the kernels consumed.  Outside a ``session`` every call loads
    the generator state, and writes the moved state back after the call (one host round trip per
    call, as the host path).  Inside ``with noise.session(device):`` the state stays on the device
    across calls (no host syncs) and is written back to the generator when the session ends —
    nothing else may draw from the generator meanwhile.
    """
    mode = _lib.SD_NOISE_STREAM

    def __init__(self, generator: Optional[torch.Generator] = None, device_generation: Optional[bool] = None,
                 pipeline_steps: Optional[int] = None):
        self.generator = generator
        self.device_generation = _DEVICE_GEN if device_generation is None else bool(device_generation)
        self._dev: Optional[_DeviceMT] = None
        self._depth = 0
        self._pool: Optional[Tuple[torch.Tensor, int]] = None   # (the reserved words, host cursor)
        # steps per pipelined pool (reserve(..., known=...) inside a session); 0 turns the pipeline off
        self.pipeline_steps = _PIPE_STEPS if pipeline_steps is None else int(pipeline_steps)
        self._pipe: Optional[_Pipeline] = None
        self._last_need = 0

    @property
    def gen(self) -> torch.Generator:
        return self.generator if self.generator is not None else torch.default_generator

    # ---- host path -------------------------------------------------------------------------
    def draw(self, n_words: int, device) -> torch.Tensor:
        """The next n_words generator words made on the HOST (the generator is NOT advanced)."""
        n = max(int(n_words), 1)
        st = self.gen.get_state().contiguous()
        host = np.empty(n, dtype=np.uint32)
        _lib.check(lib.sd_mt19937_fill(st.data_ptr(), st.numel(), host.ctypes.data, n), "sd_mt19937_fill")
        return torch.from_numpy(host.view(np.int32)).to(device)

    def advance(self, n_words: int) -> None:
        if n_words <= 0:
            return
        st = self.gen.get_state().clone()
        _lib.check(lib.sd_mt19937_advance(st.data_ptr(), st.numel(), int(n_words)), "sd_mt19937_advance")
        self.gen.set_state(st)

    # ---- the kernels' interface (ops.py) -----------------------------------------------------
    def _device_mt(self, dev: torch.device) -> _DeviceMT:
        if self._dev is None or self._dev.device != dev:
            if self._dev is not None:                   # moving devices mid-session: hand over
                self._leave_pipeline()
                self._close_pool()
                self._dev.pull(self.gen)
            self._dev = _DeviceMT(dev, self.gen.get_state())
        return self._dev

    def _leave_pipeline(self) -> None:
        """Back to the per-call generation: the device state moves to where the pipeline stands."""
        if self._pipe is None:
            return
        self._dev.state = self._pipe.final_state()
        self._pipe = None

    def reserve(self, n_words: int, device, known: Optional[int] = None) -> None:
        """As below; with `known` (the host-known part of n_words, e.g. the window's draws) the words
        come from the session's pool pipeline (_Pipeline): generated ahead on a side stream."""
        dev = torch.device(device)
        if known is not None and self._depth > 0 and self.device_generation and dev.type == "cuda" \
                and self.pipeline_steps > 0:
            self._close_pool()
            mt = self._device_mt(dev)
            p = self._pipe
            if p is not None and (p.dev != dev or p.n < n_words):   # pools sized for smaller steps
                self._leave_pipeline()
                p = None
            steps = pipeline_steps_for(int(n_words), int(known), self.pipeline_steps)
            if steps > 0:
                if p is None:
                    self._pipe = _Pipeline(dev, mt.state, int(n_words), int(known), steps)
                elif p.take(int(n_words)) is None:        # the pipeline lost its footing: start it again
                    self._leave_pipeline()
                    self._pipe = _Pipeline(dev, mt.state, int(n_words), int(known), steps)
                return
            self._leave_pipeline()
        self._reserve_pool(n_words, device)

    def _reserve_pool(self, n_words: int, device) -> None:
        """Inside a session: generate the words of SEVERAL calls in one go — an engine window's γ
        draws and its verify, whose word counts are known up front (2·B·V per draw, at most
        B·(γ + 2V) for the verify).  One set of jump-ahead substreams and one generation launch
        replace one per call; the calls then take consecutive slices (prepare) and the state is
        committed once, by the host-known prefix plus the last call's device count.  No-op
        outside a session or without device generation."""
        dev = torch.device(device)
        if self._depth == 0 or not self.device_generation or dev.type != "cuda":
            return
        self._leave_pipeline()
        self._close_pool()
        words = self._device_mt(dev).fill(int(n_words))
        self._pool = (words, 0)

    def _close_pool(self, used_dev: Optional[torch.Tensor] = None) -> None:
        """Commit a reserved pool by its host cursor (+ a device count) and drop it."""
        if self._pool is None:
            return
        _, cursor = self._pool
        self._pool = None
        if cursor or used_dev is not None:
            self._dev.commit(cursor, used_dev)

    def prepare_ex(self, n_words: int, device):
        """(words, host offset, device offset or None): the call's first word is
        words[offset + *offset_dev] (sd_noise, ABI 11)."""
        dev = torch.device(device)
        self._last_need = int(n_words)
        if self._pipe is not None:
            if self._pipe.dev == dev:
                got = self._pipe.take(max(int(n_words), 1))
                if got is not None:
                    return got
            self._leave_pipeline()
        return self.prepare(n_words, device), 0, None

    def prepare(self, n_words: int, device) -> torch.Tensor:
        """Device words for a call that may consume up to n_words words (the words start at [0])."""
        dev = torch.device(device)
        self._leave_pipeline()   # a caller that needs the words at [0] (chunked windows)
        if not self.device_generation or dev.type != "cuda":
            return self.draw(n_words, dev)
        if self._pool is not None:
            words, cursor = self._pool
            if self._dev.device == dev and cursor + max(int(n_words), 1) <= words.numel() - 624:
                return words[cursor:words.numel() - 624]   # the rest of the pool, minus the commit's slack
            self._close_pool()                          # exhausted: commit what was used, fill anew
        return self._device_mt(dev).fill(n_words)

    def consumed(self, count: Optional[int] = None, used_dev: Optional[torch.Tensor] = None) -> None:
        """The call consumed `count` words (or the device int64 `used_dev` holds the count)."""
        if self._dev is None:
            self.advance(int(used_dev.item()) if used_dev is not None else int(count or 0))
            return
        if self._pipe is not None:
            self._pipe.consumed(count, used_dev, self._last_need)
            return
        if self._pool is not None:
            words, cursor = self._pool
            if used_dev is None:                        # a host-known count: the cursor moves
                self._pool = (words, cursor + int(count or 0))
            else:                                       # a device count ends the pool (its size is
                self._close_pool(used_dev)              # unknown to the host until read)
        else:
            self._dev.commit(count, used_dev)
        if self._depth == 0:
            self._close_pool()
            self._dev.pull(self.gen)
            self._dev = None

    @contextlib.contextmanager
    def session(self):
        """Keep the generator state on the device across calls (see the class docstring)."""
        self._depth += 1
        try:
            yield self
        finally:
            self._depth -= 1
            if self._depth == 0 and self._dev is not None:
                self._leave_pipeline()
                self._close_pool()
                self._dev.pull(self.gen)
                self._dev = None


class PhiloxNoise:
    """Perf-mode noise: Philox4x32-10 keyed by (seed, call offset, global row) in the kernels.

    Every call takes the next host offset.  ``offset_dev`` (optional int64 [1] device tensor) is
    added to it by the kernels when they run: a hipGraph captures fixed host offsets, and
    advancing ``offset_dev`` on the device between replays (``advance_device``) gives every
    replay fresh noise without leaving the graph."""
    mode = _lib.SD_NOISE_PHILOX

    def __init__(self, seed: Optional[int] = None, offset: int = 0, offset_dev: Optional[torch.Tensor] = None):
        if seed is None:   # deterministic under torch.manual_seed
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.seed = seed & 0xFFFFFFFFFFFFFFFF
        self.offset = offset
        self.offset_dev = offset_dev

    def advance_device(self, calls: int) -> None:
        """Move the device base past `calls` host offsets (a stream-ordered add; capturable)."""
        if self.offset_dev is None:
            raise ValueError("PhiloxNoise has no offset_dev")
        self.offset_dev.add_(int(calls))

    def next_offset(self) -> int:
        o = self.offset
        self.offset += 1
        return o


_mode = os.environ.get("SPECDEC_NOISE", "stream").lower()
_philox: Optional[PhiloxNoise] = None


def set_noise_mode(mode: str, seed: Optional[int] = None) -> None:
    global _mode, _philox
    if mode not in ("stream", "philox"):
        raise ValueError(f"noise mode must be 'stream' or 'philox', got {mode!r}")
    _mode = mode
    _philox = PhiloxNoise(seed) if mode == "philox" else None


def default_noise():
    global _philox
    if _mode == "philox":
        if _philox is None:
            _philox = PhiloxNoise()
        return _philox
    return StreamNoise()


def noise_session(noise):
    """``noise.session()`` for StreamNoise (state kept on the device for a whole decode loop),
    a no-op context for PhiloxNoise."""
    return noise.session() if isinstance(noise, StreamNoise) else contextlib.nullcontext()
