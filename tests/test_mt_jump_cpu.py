"""Host side of the device STREAM generator (csrc/mt_jump.cpp, noise_host.cpp), on CPU:

* the characteristic polynomial P of torch's mt19937 (Berlekamp–Massey) has degree 19937 and
  annihilates the generator's output bits;
* jump polynomials: the substream decomposition the GPU runs (sd_mt19937_fill_substreams — the
  same base-sequence windows, the same XOR of windows selected by x^(s*stride-1) mod P) gives
  exactly the words torch's generator produces, from real torch states at every block position;
* torch state <-> (block, tau0) round trips, and the commit rule (untemper the block holding the
  last consumed word) lands on torch's own state after the same number of draws.
The GPU kernels are checked against the same host stream in tests/test_gpu_mt19937.py.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from specdec_amd import _lib
from specdec_amd._lib import lib
from specdec_amd.noise import StreamNoise

W = _lib.SD_MT_JUMP_WORDS


def torch_state_after(seed, skip):
    g = torch.Generator().manual_seed(seed)
    if skip:
        torch.rand(skip, generator=g)
    return g


def block_of(gen):
    st = gen.get_state().contiguous()
    s = _lib.sd_mt_state()
    assert lib.sd_mt19937_state_from_torch(st.data_ptr(), st.numel(), C.byref(s)) == 0
    return np.frombuffer(bytes(s), dtype=np.uint32)[:624].copy(), s.tau0


def host_words(gen, n):
    return StreamNoise(gen, device_generation=False).draw(n, "cpu").numpy().view(np.uint32)


def untemper(y):
    y = y.astype(np.uint32)
    y ^= y >> np.uint32(18)
    y ^= (y << np.uint32(15)) & np.uint32(0xEFC60000)
    t = y.copy()
    for _ in range(4):
        t = y ^ ((t << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = t
    t = y.copy()
    for _ in range(2):
        t = y ^ (t >> np.uint32(11))
    return t


def test_characteristic_polynomial_annihilates_the_output_bits():
    P = np.zeros(313, dtype=np.uint64)
    assert lib.sd_mt19937_char_poly(P.ctypes.data, 313) == 0
    bits = np.unpackbits(P.view(np.uint8), bitorder="little")
    deg = int(np.nonzero(bits)[0].max())
    assert deg == 19937 and bits[0] == 1
    # sum_j p_j s[k+j] = 0 for the bit-0 sequence of the untempered words, at a few offsets k
    g = torch_state_after(7, 0)
    words = host_words(g, 19937 + 700)
    x = untemper(words)[1:]                                 # windows from x[1] on are in A's image
    s = (x & 1).astype(np.uint8)
    taps = np.nonzero(bits[:deg + 1])[0]
    for k in (0, 5, 333, 650):
        assert int(s[k + taps].sum()) % 2 == 0


@pytest.mark.parametrize("skip", [0, 1, 300, 623, 624, 625, 1247, 5000])
def test_substream_decomposition_equals_torch_words(skip):
    stride, count = 4096, 8
    table = np.zeros((count, W), dtype=np.uint64)
    assert lib.sd_mt19937_jump_table(stride, count, table.ctypes.data) == 0
    assert not table[:, 312:].any()                          # zero padding past degree 19937
    g = torch_state_after(11, skip)
    block, tau0 = block_of(g)
    n = stride * 7 + 1234
    out = np.zeros(n, dtype=np.uint32)
    assert lib.sd_mt19937_fill_substreams(block.ctypes.data, tau0, out.ctypes.data, n, stride,
                                          table.ctypes.data, count) == 0
    assert np.array_equal(out, host_words(g, n))


def test_jump_table_rejects_bad_args_and_is_deterministic():
    t1 = np.zeros((3, W), dtype=np.uint64)
    t2 = np.zeros((5, W), dtype=np.uint64)
    assert lib.sd_mt19937_jump_table(65536, 3, t1.ctypes.data) == 0
    assert lib.sd_mt19937_jump_table(65536, 5, t2.ctypes.data) == 0
    assert np.array_equal(t1, t2[:3])
    assert lib.sd_mt19937_jump_table(0, 3, t1.ctypes.data) == _lib.SD_ERR_INVALID


@pytest.mark.parametrize("skip", [0, 1, 623, 624, 9999])
def test_state_round_trip(skip):
    g = torch_state_after(5, skip)
    st = g.get_state().contiguous()
    s = _lib.sd_mt_state()
    assert lib.sd_mt19937_state_from_torch(st.data_ptr(), st.numel(), C.byref(s)) == 0
    assert 1 <= s.tau0 <= 624
    back = st.clone()                                       # left / next are rewritten from tau0
    assert lib.sd_mt19937_state_to_torch(C.byref(s), back.data_ptr(), back.numel()) == 0
    if skip == 0:
        # a fresh seed is (left 1, next 0); the round trip writes the equivalent (left 1, next 624)
        assert s.tau0 == 624
        g2 = torch.Generator()
        g2.set_state(back)
        assert torch.equal(torch.rand(700, generator=g2), torch.rand(700, generator=torch_state_after(5, 0)))
    else:
        assert torch.equal(back, st)


@pytest.mark.parametrize("skip,used", [(0, 1), (0, 624), (5, 619), (5, 620), (300, 5000), (624, 1), (100, 1248)])
def test_commit_rule_lands_on_torch_state(skip, used):
    """k_mt_commit restated: the block holding the last consumed word, untempered from the fill's
    words, with tau0' = end - 624 b (or tau0 + used inside the current block)."""
    g = torch_state_after(3, skip)
    block, tau0 = block_of(g)
    words = host_words(g, used + 624)
    end = tau0 + used
    if end <= 624:
        new_block, new_tau0 = block, end
    else:
        b = (end - 1) // 624
        first = b * 624 - tau0
        new_block, new_tau0 = untemper(words[first:first + 624]), end - b * 624
    s = _lib.sd_mt_state()
    C.memmove(C.addressof(s), new_block.astype(np.uint32).tobytes(), 624 * 4)
    s.tau0 = int(new_tau0)
    st = g.get_state().clone()
    assert lib.sd_mt19937_state_to_torch(C.byref(s), st.data_ptr(), st.numel()) == 0
    ref = torch_state_after(3, skip)
    torch.rand(used, generator=ref)
    g2 = torch.Generator()
    g2.set_state(st)
    assert torch.equal(torch.rand(2000, generator=g2), torch.rand(2000, generator=ref))
