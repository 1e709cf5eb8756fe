"""Poll-mode kernels beside a long kernel of another stream (VERDICT r5 "spurious timeouts").

The in-launch exchanges (k_draw_lean's row records, k_verify_fused's span / decision / chunk
records) have a consumer workgroup wait for producers of the same launch.  Workgroups are
dispatched in order per XCD, so a producer is always dispatched before its consumer — but when
another stream's kernel holds the CUs of some XCDs, producers there wait for it, and their
consumers elsewhere spin meanwhile.  Round 5 bounded that spin by a count (~50 ms), so a
co-running kernel longer than that turned into SD_ROW_EXCHANGE_TIMEOUT / RowError with the data
fine.  The bound is now wall clock (2 s default, sd_set_poll_policy): here a helper kernel
(tests/busy/busy.hip) fills every CU of half the XCDs for 300 ms while a lean draw and a fused
verify run on the default stream; their outputs must equal an idle-GPU call's, with no flagged row.
"""
import ctypes as C
import os
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))


def busy_lib():
    path = os.path.join(HERE, "busy", "libsd_busy.so")
    if not os.path.exists(path):
        pytest.fail("tests/busy/libsd_busy.so is not built (make -C speculative-decoding_amd testhelpers)")
    lib = C.CDLL(path)
    lib.sd_test_busy.restype = C.c_int32
    lib.sd_test_busy.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    return lib


def step(ops, _lib, PhiloxNoise, tl, dl, seed, status_or):
    """4 lean draws + one fused verify (the bench's engine step), fixed Philox offsets."""
    B, g, V = tl.shape
    noise = PhiloxNoise(seed=seed, offset=0)
    draft = torch.empty(B, g, dtype=torch.long, device=DEV)
    stats = torch.empty(g, B, 2, dtype=torch.float32, device=DEV)
    for d in range(g):
        ops.sample_rows(dl[:, d], ops.PLAIN_SOFTMAX, noise, tokens_out=draft[:, d], row_stats_out=stats[d],
                        status_or=status_or)
    paths = [_lib.last_sample_path()]
    out = ops.verify([tl[:, t] for t in range(g)], [dl[:, d] for d in range(g)], draft, _lib.SD_RULE_ENGINE,
                     ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, noise, torch.tensor([128001], device=DEV),
                     draft_row_stats=stats, status_or=status_or)
    paths.append(_lib.last_verify_path())
    return draft, out, paths


def test_poll_kernels_beside_a_busy_stream():
    from specdec_amd import _lib, ops
    from specdec_amd.noise import PhiloxNoise
    lib = busy_lib()
    B, g, V = 32, 4, 128256
    gen = torch.Generator(device=DEV).manual_seed(5)
    tl = (torch.randn(B, g, V, generator=gen, device=DEV) * 3).to(torch.bfloat16)
    dl = (tl.float() + torch.randn(B, g, V, generator=gen, device=DEV)).to(torch.bfloat16)
    so_idle = torch.zeros(1, dtype=torch.int32, device=DEV)
    want_draft, want, paths = step(ops, _lib, PhiloxNoise, tl, dl, 77, so_idle)
    torch.cuda.synchronize()
    assert paths == [_lib.SD_PATH_SAMPLE_DRAW_LEAN, _lib.SD_PATH_VERIFY_FUSED], paths
    assert int(so_idle) == 0

    side = torch.cuda.Stream()
    ran = torch.zeros(1, dtype=torch.int32, device=DEV)
    busy_us = 300_000
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    so = torch.zeros(1, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    # every CU of the odd XCDs, 4 workgroups deep (the later ones queue behind the first), 160 KiB each
    st = lib.sd_test_busy(4 * cus, 0xAA, busy_us, 160 * 1024, ran.data_ptr(), side.cuda_stream)
    assert st == 0, st
    t0 = time.perf_counter()
    got_draft, got, _ = step(ops, _lib, PhiloxNoise, tl, dl, 77, so)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"[busy] step beside the busy kernel: {dt * 1e3:.1f} ms, busy workgroups {int(ran)}")
    assert int(ran) > 0                    # the helper did occupy CUs
    assert int(so) == 0, hex(int(so))       # no flagged row: the waits outlasted the busy kernel
    assert torch.equal(got_draft, want_draft)
    for f in ("n_accepted", "next_token", "row_status"):
        assert torch.equal(getattr(got, f), getattr(want, f)), f
