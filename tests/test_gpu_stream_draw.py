"""The one-pass STREAM draw (k_draw_stream, csrc/sd_draw_stream.inc) against the oracle and the
three-launch STREAM path (row statistics + k_rowsample + k_sample_finalize, SD_OPT_DRAW_STREAM = 0).

torch.multinomial(softmax(l), 1) on [R, V] rows with the generator's words (the reference's draw,
engine/infer_engine.py:241-246; utils/logits_processor.py:39-49) must come out bit-exact: the same
token as torch-CPU (or, where torch-CPU's own fp32 normaliser rounds a probability the other way,
as the exact-arithmetic oracle), the generator advanced by exactly 2·R·V words, and the same tokens
as the three-launch path.  Covers Llama-3 rows at the bench batch, fp16, a ragged last span, and
rows of a few repeated values (every span overflows its candidate slots: the tail's exact rescan).
The (max, Σexp) the draw returns for the verify equal the exact row statistics.
"""
import pytest
import torch

from oracle import specdec_ref as ref
from parity_stats import DIVERGENCES

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rows(R, V, dtype, seed, kind="normal", pad=0):
    g = torch.Generator().manual_seed(seed)
    if kind == "ties":   # a handful of levels: thousands of equal values per span
        x = torch.randint(0, 5, (R, V), generator=g).float() * 0.5
    else:
        x = torch.randn(R, V, generator=g) * 3.0
    if pad:   # rows of V elements at a padded (16-byte aligned) stride, on the device
        buf = torch.zeros(R, V + pad)
        buf[:, :V] = x
        return buf.to(dtype).to(DEV)[:, :V]
    return x.to(dtype).to(DEV)


def hip_draw(x, seed, one_pass, monkeypatch):
    from specdec_amd import _lib, ops
    from specdec_amd.noise import StreamNoise
    g = torch.Generator().manual_seed(seed)
    xd = x
    stats = torch.zeros(x.shape[0], 2, device=DEV)
    with _lib.option(_lib.SD_OPT_DRAW_STREAM, 1 if one_pass else 0):
        tok, _, st = ops.sample_rows(xd, ops.PLAIN_SOFTMAX, StreamNoise(g), row_stats_out=stats)
    if one_pass:
        assert _lib.last_sample_path() == _lib.SD_PATH_SAMPLE_STREAM
    else:
        assert _lib.last_sample_path() == _lib.SD_PATH_SAMPLE_MULTI
    torch.cuda.synchronize()
    return tok.cpu(), st.cpu(), stats.cpu(), g.get_state()


CASES = [
    # (R, V, dtype, kind, pad, seed)
    (32, 128256, torch.bfloat16, "normal", 0, 1),
    (4, 128256, torch.float16, "normal", 0, 2),
    (8, 4096, torch.bfloat16, "normal", 0, 3),
    (3, 6149, torch.bfloat16, "normal", 11, 4),     # ragged last span, rows 16-byte aligned
    (3, 128256, torch.bfloat16, "ties", 0, 5),
    (1, 128256, torch.bfloat16, "normal", 0, 6),
]


@pytest.mark.parametrize("R,V,dtype,kind,pad,seed", CASES, ids=[f"{c[0]}x{c[1]}-{str(c[2])[6:]}-{c[3]}" for c in CASES])
def test_one_pass_stream_draw_is_the_reference_draw(R, V, dtype, kind, pad, seed, monkeypatch):
    x = rows(R, V, dtype, seed, kind, pad)
    tok1, st1, stats1, state1 = hip_draw(x, 100 + seed, True, monkeypatch)
    tok3, st3, stats3, state3 = hip_draw(x, 100 + seed, False, monkeypatch)
    # the generator moved by exactly the reference's 2·R·V words, on both paths
    g = torch.Generator().manual_seed(100 + seed)
    torch.empty(R, V).exponential_(generator=g)
    assert torch.equal(state1, g.get_state()) and torch.equal(state3, g.get_state())
    assert not ((st1 | st3) & 0x2C0).any()      # no INVALID / OVERRUN / TIMEOUT
    # the oracle: torch-CPU arithmetic, or the exact-softmax variant where torch's normaliser rounds
    proc = ref.Processor("multinomial", 1.0)
    xc = x.cpu().contiguous()
    want = {}
    for exact in (False, True):
        gg = torch.Generator().manual_seed(100 + seed)
        want[exact] = ref.sample(ref.process(xc, proc, exact), proc, ref.TorchNoise(gg)).squeeze(-1)
    for r in range(R):
        got = int(tok1[r])
        assert got in (int(want[False][r]), int(want[True][r])), (r, got, int(want[False][r]), int(want[True][r]))
        if got != int(want[False][r]):
            DIVERGENCES.append(f"stream draw {kind} V={V} row={r}")
    assert torch.equal(tok1, tok3)
    # row statistics: the exact max, and Σexp within fp32 accumulation error of the fp64 value
    xf = xc.double()
    M = xf.max(-1).values
    S = torch.exp(xf - M[:, None]).sum(-1)
    assert torch.equal(stats1[:, 0].double(), M)
    assert torch.allclose(stats1[:, 1].double(), S, rtol=2e-6, atol=0)
