"""The STREAM pool pipeline's bookkeeping (specdec_amd.noise._Pipeline), on the CPU.

In a noise session the drop-in loops reserve each step's words (``reserve(n, known=k)``) and the
pools come from a side stream, generated ahead from an anchor the host never reads back; a call's
first word is words[host offset + *device offset] (sd_noise, ABI 11).  The invariant that makes the
GPU path bit-exact is that this view always points at the generator position the reference's
sequential draws have reached.  Here the generator is a fake whose word i of a pool generated from
position s is s + i, and whose commit moves a position, so every view can be checked against the
true running position over long random sessions: steps of varying draws and verify consumption
(0 .. the worst case), steps that consume less than announced, calls without a reservation, and the
final state handed back to the generator."""
import contextlib
import random

import torch

from specdec_amd.noise import _Pipeline


class FakeBackend:
    """The pipeline's primitives with the generator replaced by positions: state = int64 [1]."""

    @staticmethod
    def new_stream(dev):
        return object()

    @staticmethod
    def current(dev):
        return None

    @staticmethod
    def event_on(stream):
        return None

    @staticmethod
    def wait(stream, ev):
        pass

    @staticmethod
    def on(stream):
        return contextlib.nullcontext()

    @staticmethod
    def keep(t, stream):
        pass

    @staticmethod
    def generate(state, words, n, ws_box, stream):
        words[:n] = state[0].to(torch.int32) + torch.arange(n, dtype=torch.int32)

    @staticmethod
    def commit(state, words, n_generated, used, used_dev, stream):
        state += int(used) + (int(used_dev[0]) if used_dev is not None else 0)


def view(pipe, n):
    got = pipe.take(n)
    if got is None:
        return None
    words, off, off_dev = got
    start = off + int(off_dev[0])
    assert 0 <= start and start + n <= words.numel(), (start, n, words.numel())
    return int(words[start])


def run_session(seed, steps_per_pool, B, V, gamma, n_steps, short=0.3):
    rnd = random.Random(seed)
    draw = 2 * B * V
    known = gamma * draw
    n = known + B * (gamma + 2 * V)
    pos = 1000                                   # the true generator position
    pipe = _Pipeline(torch.device("cpu"), torch.tensor([pos]), n, known, steps_per_pool, be=FakeBackend)
    restarts = 0
    for step in range(n_steps):
        g = gamma - 1 if gamma > 1 and rnd.random() < short else gamma   # short (final) windows too
        kn = g * draw
        if pipe.take(kn + B * (g + 2 * V)) is None:       # StreamNoise.reserve's restart
            pipe = _Pipeline(torch.device("cpu"), pipe.final_state(), n, known, steps_per_pool, be=FakeBackend)
            restarts += 1
        for _ in range(g):                                # the draws: host-known counts
            assert view(pipe, draw) == pos
            pipe.consumed(draw, None, draw)
            pos += draw
        if rnd.random() < 0.1:                            # a call outside the step accounting
            assert view(pipe, 7) == pos
            pipe.consumed(7, None, 7)
            pos += 7
        worst = B * (g + 2 * V)
        assert view(pipe, worst) == pos                   # the verify: a device count
        used = rnd.choice([0, worst, rnd.randrange(worst + 1), B * g])
        pipe.consumed(None, torch.tensor([used]), worst)
        pos += used
    assert int(pipe.final_state()[0]) == pos
    return restarts


def test_pipeline_views_follow_the_generator():
    for seed in range(6):
        run_session(seed, steps_per_pool=4, B=3, V=50, gamma=4, n_steps=60)


def test_pipeline_steady_state_never_restarts():
    """Full windows (the loops' steady state): the pools hand over without a restart (a restart
    regenerates in line, on the main stream, and only costs time)."""
    for seed in range(4):
        assert run_session(50 + seed, steps_per_pool=4, B=3, V=50, gamma=4, n_steps=60, short=0.0) == 0


def test_pipeline_small_pools_switch_often():
    for seed in range(4):
        run_session(100 + seed, steps_per_pool=1, B=2, V=17, gamma=2, n_steps=80)
        run_session(200 + seed, steps_per_pool=2, B=1, V=64, gamma=1, n_steps=80)
