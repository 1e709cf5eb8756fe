"""The C ABI's host code under AddressSanitizer: `make asan` links the library's
objects (host side instrumented, -Xarch_host -fsanitize=address) into tests/asan/abi_asan.cpp,
which drives every argument-validation path, the workspace carving over many shapes, and the
host mt19937 / jump-ahead code; an ASan report aborts it.  Its generator words must equal torch's."""
import os
import subprocess

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "speculative-decoding_amd")
BIN = os.path.join(PKG, "build", "asan", "abi_asan")


def test_abi_host_code_is_asan_clean(tmp_path):
    r = subprocess.run(["make", "-C", PKG, "asan"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    g = torch.Generator().manual_seed(2024)
    torch.rand(17, generator=g)                      # a state mid-block
    state = tmp_path / "state.bin"
    state.write_bytes(g.get_state().numpy().tobytes())
    words = tmp_path / "words.bin"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0")
    r = subprocess.run([BIN, str(state), str(words)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr
    assert ", 0 failed" in r.stdout
    w = np.fromfile(words, dtype=np.uint32).astype(np.uint64)
    ref = torch.rand(2000, generator=g).numpy()
    assert np.array_equal(((w[:2000] & 0xFFFFFF) * 2.0 ** -24).astype(np.float32), ref)
