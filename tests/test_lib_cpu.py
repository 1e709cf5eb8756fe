"""CPU-side checks of the C ABI: the library loads, exports every symbol include/specdec.h
declares, its ctypes mirror has the C layout, and the host mt19937 stream equals torch's."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "specdec.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|size_t|const char\*)\s+(sd_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from specdec_amd import _lib
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(_lib.lib, n), n
    assert set(names) == set(_lib.EXPORTS)
    assert _lib.lib.sd_abi_version() == _lib.SD_ABI_VERSION


C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "specdec.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("sd_verify_args %zu\n", sizeof(sd_verify_args));
  printf("sd_sample_args %zu\n", sizeof(sd_sample_args));
  printf("sd_probs_args %zu\n", sizeof(sd_probs_args));
  printf("sd_noise %zu\n", sizeof(sd_noise));
  printf("sd_row_keep %zu\n", sizeof(sd_row_keep));
  printf("sd_ngram_args %zu\n", sizeof(sd_ngram_args));
  printf("sd_ngram_store %zu\n", sizeof(sd_ngram_store));
  F(sd_ngram_store, gram_capacity) F(sd_ngram_store, pair_keys) F(sd_ngram_store, pair_capacity)
  F(sd_ngram_store, status) F(sd_ngram_store, one_level) F(sd_ngram_store, vocab)
  F(sd_verify_args, draft_rows) F(sd_verify_args, draft_tokens) F(sd_verify_args, target_proc)
  F(sd_verify_args, noise) F(sd_verify_args, n_accepted) F(sd_verify_args, generated)
  F(sd_verify_args, step) F(sd_verify_args, workspace_bytes) F(sd_verify_args, prof_stats_end) F(sd_verify_args, prof_stats_repeat)
  F(sd_verify_args, draft_row_stats) F(sd_verify_args, draft_row_stats_stride) F(sd_verify_args, draft_row_keep)
  F(sd_sample_args, noise) F(sd_sample_args, tokens) F(sd_sample_args, workspace_bytes) F(sd_sample_args, row_stats) F(sd_sample_args, row_keep)
  F(sd_probs_args, probs) F(sd_probs_args, workspace_bytes) F(sd_noise, row_base)
  F(sd_ngram_args, target_rows) F(sd_ngram_args, draft_tokens) F(sd_ngram_args, proc) F(sd_ngram_args, noise)
  F(sd_ngram_args, filler_ids) F(sd_ngram_args, workspace_bytes)
  printf("sd_mt_state %zu\n", sizeof(sd_mt_state));
  printf("sd_mt_generate_args %zu\n", sizeof(sd_mt_generate_args));
  F(sd_mt_state, tau0) F(sd_mt_generate_args, jump_count) F(sd_mt_generate_args, stride_words)
  F(sd_mt_generate_args, n_words) F(sd_mt_generate_args, workspace_bytes)
  return 0;
}
"""


def test_ctypes_layout_matches_c_header():
    from specdec_amd import _lib
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write(C_LAYOUT)
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), src, "-o", exe])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = dict(line.rsplit(" ", 1) for line in out if line)
    for name, cls in [("sd_verify_args", _lib.sd_verify_args), ("sd_sample_args", _lib.sd_sample_args),
                      ("sd_probs_args", _lib.sd_probs_args), ("sd_noise", _lib.sd_noise),
                      ("sd_ngram_args", _lib.sd_ngram_args), ("sd_ngram_store", _lib.sd_ngram_store),
                      ("sd_mt_state", _lib.sd_mt_state), ("sd_mt_generate_args", _lib.sd_mt_generate_args)]:
        assert int(got[name]) == C.sizeof(cls), name
    for key, val in got.items():
        if "." in key:
            struct, field = key.split(".")
            assert getattr(getattr(_lib, struct), field).offset == int(val), key


def test_workspace_sizes_are_positive_and_reject_bad_shapes():
    from specdec_amd._lib import lib
    assert lib.sd_verify_workspace_size(32, 4, 128256) > 0
    assert lib.sd_verify_workspace_size(0, 4, 128256) == 0
    assert lib.sd_verify_workspace_size(1, 32, 128256) > 0
    assert lib.sd_verify_workspace_size(1, 33, 128256) == 0
    assert lib.sd_sample_workspace_size(4, 50257) > 0


def test_verify_rejects_invalid_args_without_touching_the_gpu():
    from specdec_amd import _lib
    a = _lib.sd_verify_args()
    a.batch, a.gamma, a.vocab = 1, 4, 100
    assert _lib.lib.sd_verify(C.byref(a), None) == _lib.SD_ERR_INVALID   # null pointers
    a.gamma = 99
    assert _lib.lib.sd_verify(C.byref(a), None) == _lib.SD_ERR_INVALID


@pytest.mark.parametrize("skip", [0, 3, 623, 624, 625, 5000])
def test_mt19937_stream_equals_torch_draws(skip):
    from specdec_amd.noise import StreamNoise
    g = torch.Generator().manual_seed(1234)
    torch.rand(skip, generator=g)
    n = StreamNoise(g)
    w = n.draw(4000, "cpu").numpy().view(np.uint32).astype(np.uint64)
    ref = torch.Generator().manual_seed(1234)
    torch.rand(skip, generator=ref)
    r = torch.rand(1000, generator=ref).numpy()
    assert np.array_equal(((w[:1000] & 0xFFFFFF) * 2.0 ** -24).astype(np.float32), r)
    e = torch.empty(1500).exponential_(generator=ref).numpy()
    u = (((w[1000:4000:2] << np.uint64(32)) | w[1001:4000:2]) & np.uint64((1 << 53) - 1)).astype(np.float64)
    assert np.array_equal((-np.log1p(-u * 2.0 ** -53)).astype(np.float32), e)
    n.advance(4000)
    assert torch.equal(g.get_state(), ref.get_state())


def test_mt19937_advance_large():
    from specdec_amd.noise import StreamNoise
    for k in (1, 624 * 3 + 7, 100_003):
        g = torch.Generator().manual_seed(99)
        StreamNoise(g).advance(k)
        r = torch.Generator().manual_seed(99)
        torch.rand(k, generator=r)
        assert torch.equal(g.get_state(), r.get_state())


def test_no_kernel_uses_scratch():
    """Every gfx950 kernel of libspecdec.so runs without private (scratch) memory: a kernel that
    spills pays ~20 us per dispatch on MI355X (an unrolled k_stats variant once
    gave the processor kernels 816 B of scratch and configs[1] nucleus +36 us per step)."""
    llvm = "/opt/rocm/lib/llvm/bin"
    from specdec_amd import _lib
    if not (os.path.exists(os.path.join(llvm, "clang-offload-bundler")) and os.path.exists(os.path.join(llvm, "llvm-readelf"))):
        pytest.skip("ROCm llvm tools not found")
    notes = kernel_notes(_lib.LIB_PATH, llvm)
    names = re.findall(r"\.name:\s*(\S+)", notes)
    assert any("k_mt_jump" in n for n in names) and any("k_stats" in n for n in names)
    sizes = re.findall(r"\.private_segment_fixed_size:\s*(\d+)", notes)
    assert len(sizes) > 100
    assert all(int(v) == 0 for v in sizes), sorted(set(sizes))


def kernel_notes(lib_path, llvm):
    """Code-object notes of every gfx950 bundle in the library's .hip_fatbin section (one bundle
    per HIP translation unit, concatenated by the linker)."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.check_call(["objcopy", "--dump-section", f".hip_fatbin={fb}", lib_path, os.path.join(d, "x.so")])
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for i, st in enumerate(starts):
            part, co = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"co{i}.o")
            open(part, "wb").write(data[st:starts[i + 1] if i + 1 < len(starts) else len(data)])
            subprocess.check_call([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", f"--input={part}",
                                   f"--output={co}", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"])
            out.append(subprocess.check_output([os.path.join(llvm, "llvm-readelf"), "--notes", co]).decode())
    return "\n".join(out)


def test_dispatch_options_round_trip_and_reject_bad_values():
    """sd_set_option / sd_get_option (ABI 10): the defaults, a scoped change, and refusals."""
    from specdec_amd import _lib
    defaults = {_lib.SD_OPT_FUSED_VERIFY: 1, _lib.SD_OPT_LEAN_VERIFY: -1, _lib.SD_OPT_THRESHOLD_POLL: 1,
                _lib.SD_OPT_DRAW_STREAM: 1}
    for o, v in defaults.items():
        assert _lib.get_option(o) == v, o
    with _lib.option(_lib.SD_OPT_FUSED_VERIFY, 0):
        assert _lib.get_option(_lib.SD_OPT_FUSED_VERIFY) == 0
    assert _lib.get_option(_lib.SD_OPT_FUSED_VERIFY) == 1
    for o, bad in ((99, 0), (_lib.SD_OPT_FUSED_VERIFY, 3), (_lib.SD_OPT_LEAN_VERIFY, 2),
                   (_lib.SD_OPT_THRESHOLD_POLL, -1), (_lib.SD_OPT_DRAW_STREAM, 2)):
        assert _lib.lib.sd_set_option(o, bad) == _lib.SD_ERR_INVALID, (o, bad)
    assert _lib.lib.sd_get_option(99, C.byref(C.c_int32())) == _lib.SD_ERR_INVALID
    for o, v in defaults.items():
        assert _lib.get_option(o) == v, o
    assert _lib.last_verify_path() == _lib.SD_PATH_NONE   # nothing ran on this thread
    assert _lib.last_sample_path() == _lib.SD_PATH_NONE


def test_no_environment_read_on_the_call_path():
    """The library reads the environment only for the poll policy's initial values (once, in
    policy_init) and, in SD_PHASE_TIMING diagnostic builds, the timestamp buffer: no getenv on the
    path of sd_verify / sd_sample / sd_ngram_verify — dispatch switches are sd_set_option."""
    csrc = os.path.join(ROOT, "speculative-decoding_amd", "csrc")
    found = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".hip", ".inc", ".cpp", ".h")):
            continue
        lines = open(os.path.join(csrc, name)).read().split("\n")
        depth_timing = 0
        func = None
        for ln, line in enumerate(lines, 1):
            s = line.strip()
            if s.startswith("#ifdef SD_PHASE_TIMING"):
                depth_timing += 1
            elif s.startswith("#endif") and depth_timing:
                depth_timing -= 1
            m = re.match(r"^[\w:<>\s\*&]+?\b(\w+)\s*\([^;]*\)\s*\{\s*$", line)
            if m and not line.startswith(" "):
                func = m.group(1)
            if "getenv(" in line:
                found.append((name, ln, func, bool(depth_timing), re.findall(r'getenv\("(\w+)"\)', line)))
    assert found, "scanner found no getenv at all (the poll policy's should be there)"
    for name, ln, func, timing, vars_ in found:
        if timing:
            assert vars_ == ["SD_TS_PTR"], (name, ln, vars_)
        else:
            assert func == "policy_init" and set(vars_) <= {"SD_POLL", "SD_POLL_SPIN_LIMIT"}, (name, ln, func, vars_)
