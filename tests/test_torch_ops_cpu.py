"""torch.library registration: torch.ops.specdec.sample / .verify exist and their
fake implementations give the output shapes and dtypes without a GPU (meta tensors)."""
import torch

import specdec_amd  # noqa: F401  (registers the ops)


def test_sample_op_fake_shapes():
    x = torch.empty(4, 1000, device="meta", dtype=torch.bfloat16)
    tok, stats, st = torch.ops.specdec.sample(x, 1, 1.0, 0, 1.0, 1, 0, 0)
    assert (tok.shape, tok.dtype) == ((4,), torch.long)
    assert (stats.shape, stats.dtype) == ((4, 2), torch.float32)
    assert (st.shape, st.dtype) == ((4,), torch.int32)


def test_verify_op_fake_shapes():
    t = torch.empty(3, 5, 1000, device="meta", dtype=torch.bfloat16)
    d = torch.empty(3, 4, 1000, device="meta", dtype=torch.bfloat16)
    ids = torch.empty(3, 4, dtype=torch.long, device="meta")
    stops = torch.empty(2, dtype=torch.long, device="meta")
    outs = torch.ops.specdec.verify(t, d, ids, stops, 0, 1, 1.0, 0, 1.0, 7, 0, 0)
    assert [o.shape for o in outs] == [(3,)] * 7
    assert [o.dtype for o in outs] == [torch.int32, torch.long, torch.float32] + [torch.int32] * 4
