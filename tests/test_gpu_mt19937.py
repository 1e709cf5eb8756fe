"""The device STREAM generator (csrc/mt_device.hip) against torch's own CPU generator words.

* sd_mt19937_generate writes exactly the words the host stream (sd_mt19937_fill, pinned to
  torch.rand / exponential_ in tests/test_lib_cpu.py) gives, from states at every block
  position, for fills inside one block, across block and substream boundaries, and at the
  bench's size (2 * 32 * 128256 words: one engine drafter draw);
* sd_mt19937_commit moves the device state by a host count or by a device-side count, landing on
  torch's state after the same number of draws;
* StreamNoise with device generation gives the same kernel outputs and the same generator
  state as host generation, per call and across a session.
"""
import numpy as np
import pytest
import torch

from specdec_amd import _lib, ops
from specdec_amd.noise import StreamNoise, _DeviceMT

pytestmark = pytest.mark.gpu
DEV = "cuda"


def gen_after(seed, skip):
    g = torch.Generator().manual_seed(seed)
    if skip:
        torch.rand(skip, generator=g)
    return g


def host_words(g, n):
    return StreamNoise(g, device_generation=False).draw(n, "cpu").numpy().view(np.uint32)


@pytest.mark.parametrize("skip", [0, 1, 300, 623, 624, 1000])
@pytest.mark.parametrize("n", [1, 623, 700, 5000, 65536 - 624, 65536 * 2 + 77, 3 * 65536 + 12345])
def test_generate_equals_host_stream(skip, n):
    g = gen_after(42, skip)
    d = _DeviceMT(DEV, g.get_state())
    got = d.fill(n).cpu().numpy().view(np.uint32)
    want = host_words(g, n + 624)
    assert got.shape == want.shape
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:5], bad.size)


def test_generate_engine_draw_size():
    n = 2 * 32 * 128256
    g = gen_after(7, 12345)
    d = _DeviceMT(DEV, g.get_state())
    got = d.fill(n).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, host_words(g, n + 624))


@pytest.mark.parametrize("skip,used", [(0, 1), (0, 624), (5, 619), (5, 620), (300, 5000), (624, 1),
                                       (100, 1248), (3, 2 * 65536 + 999)])
@pytest.mark.parametrize("device_count", [False, True])
def test_commit_moves_state_like_torch(skip, used, device_count):
    g = gen_after(3, skip)
    d = _DeviceMT(DEV, g.get_state())
    d.fill(used + 10)
    if device_count:
        d.commit(used_dev=torch.tensor([used], dtype=torch.long, device=DEV))
    else:
        d.commit(count=used)
    d.pull(g)
    ref = gen_after(3, skip)
    torch.rand(used, generator=ref)
    assert torch.equal(torch.rand(3000, generator=g), torch.rand(3000, generator=ref))


def test_repeated_fill_commit_in_a_session_equals_host():
    g_dev, g_host = gen_after(11, 77), gen_after(11, 77)
    nd = StreamNoise(g_dev)
    with nd.session():
        for n, used in ((1000, 400), (70000, 70000), (5, 0), (200000, 123457), (624, 624)):
            w = nd.prepare(n, DEV)[:n].cpu().numpy().view(np.uint32)
            assert np.array_equal(w, host_words(g_host, n))
            nd.consumed(count=used)
            StreamNoise(g_host, device_generation=False).advance(used)
    assert torch.equal(g_dev.get_state(), g_host.get_state())


@pytest.mark.parametrize("kind", ["multinomial", "nucleus"])
def test_device_and_host_generation_give_identical_calls(kind):
    V, B, g = 8192, 3, 4
    gen = torch.Generator().manual_seed(5)
    tl = (torch.randn(B, g + 1, V, generator=gen) * 3).to(torch.bfloat16).to(DEV)
    dl = (tl[:, :g].float() + torch.randn(B, g, V, generator=gen).to(DEV)).to(torch.bfloat16)
    spec = ops.ProcSpec(kind, 1.0, 0, 0.9)
    outs, states = [], []
    for devgen in (True, False):
        gs = torch.Generator().manual_seed(99)
        noise = StreamNoise(gs, device_generation=devgen)
        ids = torch.zeros(B, g, dtype=torch.long, device=DEV)
        for d in range(g):
            ops.sample_rows(dl[:, d], spec, noise, tokens_out=ids[:, d])
        o = ops.verify([tl[:, t] for t in range(g + 1)], [dl[:, d] for d in range(g)], ids, _lib.SD_RULE_SPEC,
                       spec, spec, noise)
        outs.append((ids.cpu(), o.n_accepted.cpu(), o.next_token.cpu(), int(o.words_used.item())))
        states.append(gs.get_state())
    assert all(torch.equal(a, b) for a, b in zip(outs[0][:3], outs[1][:3])) and outs[0][3] == outs[1][3]
    assert torch.equal(states[0], states[1])
