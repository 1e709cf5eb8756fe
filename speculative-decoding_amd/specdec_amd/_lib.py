"""ctypes binding of libspecdec.so (include/specdec.h).

The library is built in-tree (``make -C speculative-decoding_amd``) and loaded from this
package directory.  There is no fallback: if the library is missing or was built for a
different ABI, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

SD_ABI_VERSION = 11
SD_MAX_GAMMA = 32           # drafts per call (ops.verify / ngram_verify chunk longer windows)
SD_NGRAM_MAX_FILLER = 64

SD_OK, SD_ERR_INVALID, SD_ERR_WORKSPACE, SD_ERR_LAUNCH, SD_ERR_UNSUPPORTED = 0, -1, -2, -3, -4
SD_F32, SD_BF16, SD_F16 = 0, 1, 2
SD_PROC_GREEDY, SD_PROC_MULTINOMIAL, SD_PROC_TOPK, SD_PROC_NUCLEUS, SD_PROC_TOPK_NUCLEUS = range(5)
SD_RULE_SPEC, SD_RULE_ENGINE = 0, 1
SD_NOISE_STREAM, SD_NOISE_PHILOX = 0, 1

SD_ROW_DONE = 0x1
SD_ROW_STOP_IN_DRAFTS = 0x2
SD_ROW_FINISHED = 0x4
SD_ROW_RESIDUAL = 0x8
SD_ROW_BONUS = 0x10
SD_ROW_FALLBACK_P = 0x20
SD_ROW_INVALID_DIST = 0x40
SD_ROW_NOISE_OVERRUN = 0x80
SD_ROW_NUCLEUS_INEXACT = 0x100
SD_ROW_EXCHANGE_TIMEOUT = 0x200
# the bits that make a row's outputs unusable (the reference raises there): status_or collects them
SD_ROW_ERROR_MASK = SD_ROW_INVALID_DIST | SD_ROW_NOISE_OVERRUN | SD_ROW_EXCHANGE_TIMEOUT

# dispatch options (sd_set_option) and the paths sd_last_*_path reports
SD_OPT_FUSED_VERIFY, SD_OPT_LEAN_VERIFY, SD_OPT_THRESHOLD_POLL, SD_OPT_DRAW_STREAM = 1, 2, 3, 4
SD_OPT_FUSED_TICKET, SD_OPT_DRAW_SPAN, SD_OPT_TICKET_LAG, SD_OPT_SAMP_CHUNKS = 5, 6, 7, 8
SD_PATH_NONE = 0
SD_PATH_VERIFY_LEAN, SD_PATH_VERIFY_FUSED, SD_PATH_VERIFY_TWO_LAUNCH, SD_PATH_VERIFY_STREAM = 1, 2, 3, 4
SD_PATH_VERIFY_FUSED_TICKET = 5
SD_PATH_SAMPLE_DRAW_LEAN, SD_PATH_SAMPLE_DRAW, SD_PATH_SAMPLE_NUCLEUS, SD_PATH_SAMPLE_STREAM = 16, 17, 18, 19
SD_PATH_SAMPLE_GREEDY_LEAN, SD_PATH_SAMPLE_MULTI = 20, 21
PATH_NAMES = {SD_PATH_NONE: "none", SD_PATH_VERIFY_LEAN: "k_verify_lean", SD_PATH_VERIFY_FUSED: "k_verify_fused",
              SD_PATH_VERIFY_FUSED_TICKET: "k_verify_fused(ticket)",
              SD_PATH_VERIFY_TWO_LAUNCH: "k_stats+k_sample", SD_PATH_VERIFY_STREAM: "stream",
              SD_PATH_SAMPLE_DRAW_LEAN: "k_draw_lean", SD_PATH_SAMPLE_DRAW: "k_draw", SD_PATH_SAMPLE_NUCLEUS: "k_draw_nuc",
              SD_PATH_SAMPLE_STREAM: "k_draw_stream", SD_PATH_SAMPLE_GREEDY_LEAN: "k_draw_lean<greedy>",
              SD_PATH_SAMPLE_MULTI: "k_stats+k_rowsample+k_sample_finalize"}

# SPECDEC_LIB selects another in-tree build of the same ABI (e.g. the phase-timing variant)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("SPECDEC_LIB", "libspecdec.so"))

EXPORTS = ("sd_abi_version", "sd_status_string", "sd_last_hip_error", "sd_verify_workspace_size", "sd_verify",
           "sd_sample_workspace_size", "sd_sample", "sd_probs_workspace_size", "sd_probs",
           "sd_ngram_workspace_size", "sd_ngram_verify", "sd_mt19937_fill", "sd_mt19937_advance",
           "sd_ngram_store_initialize", "sd_ngram_store_update", "sd_ngram_store_next_token",
           "sd_ngram_store_has_gram", "sd_ngram_store_draft",
           "sd_mt19937_state_from_torch", "sd_mt19937_state_to_torch", "sd_mt19937_jump_table",
           "sd_mt19937_char_poly", "sd_mt19937_fill_substreams", "sd_mt19937_generate_workspace_size",
           "sd_mt19937_generate", "sd_mt19937_commit", "sd_set_poll_policy", "sd_get_poll_policy",
           "sd_set_option", "sd_get_option", "sd_last_verify_path", "sd_last_sample_path")

SD_MT_JUMP_WORDS = 320
SD_MT_JUMP_CHUNKS = 16
SD_MT_STATE_BYTES = 624 * 4 + 16


SD_NGRAM_MAX_N = 4
SD_NGRAM_FULL = 1
SD_NGRAM_BAD_TOKEN = 2


class sd_ngram_store(C.Structure):
    _fields_ = [("gram_keys", C.c_void_p), ("gram_best", C.c_void_p), ("gram_capacity", C.c_int64),
                ("pair_keys", C.c_void_p), ("pair_count", C.c_void_p), ("pair_ts", C.c_void_p),
                ("pair_capacity", C.c_int64), ("status", C.c_void_p), ("n", C.c_int32), ("one_level", C.c_int32),
                ("vocab", C.c_int32)]


class sd_mt_state(C.Structure):
    _fields_ = [("mt", C.c_uint32 * 624), ("tau0", C.c_int32), ("reserved", C.c_int32 * 3)]


class sd_mt_generate_args(C.Structure):
    _fields_ = [("state", C.c_void_p), ("jump_table", C.c_void_p), ("jump_count", C.c_int32),
                ("stride_words", C.c_int64), ("words", C.c_void_p), ("n_words", C.c_int64),
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t)]


class sd_processor(C.Structure):
    _fields_ = [("kind", C.c_int32), ("temperature", C.c_float), ("top_k", C.c_int32), ("top_p", C.c_float)]


class sd_noise(C.Structure):
    _fields_ = [("mode", C.c_int32), ("words", C.c_void_p), ("n_words", C.c_int64),
                ("seed", C.c_uint64), ("offset", C.c_uint64), ("row_base", C.c_int64),
                ("offset_dev", C.c_void_p)]


class sd_verify_args(C.Structure):
    _fields_ = [
        ("batch", C.c_int32), ("gamma", C.c_int32), ("vocab", C.c_int32), ("rule", C.c_int32),
        ("target_rows", C.c_void_p * (SD_MAX_GAMMA + 1)), ("target_stride_b", C.c_int64),
        ("target_dtype", C.c_int32),
        ("draft_rows", C.c_void_p * SD_MAX_GAMMA), ("draft_stride_b", C.c_int64),
        ("draft_dtype", C.c_int32), ("draft_is_probs", C.c_int32),
        ("draft_tokens", C.c_void_p), ("draft_tokens_stride_b", C.c_int64),
        ("target_proc", sd_processor), ("draft_proc", sd_processor),
        ("skip_sample_adjustment", C.c_int32), ("stop_tokens", C.c_void_p), ("n_stop", C.c_int32),
        ("active", C.c_void_p),
        ("noise", sd_noise),
        ("n_accepted", C.c_void_p), ("next_token", C.c_void_p), ("resample_mass", C.c_void_p),
        ("prune_drafter", C.c_void_p), ("prune_target", C.c_void_p), ("stop_index", C.c_void_p),
        ("row_status", C.c_void_p), ("words_used", C.c_void_p),
        ("generated", C.c_void_p), ("generated_stride_b", C.c_int64), ("step", C.c_int32),
        ("finished", C.c_void_p), ("accepted_count", C.c_void_p),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
        ("prof_stats_begin", C.c_void_p), ("prof_stats_end", C.c_void_p), ("prof_stats_repeat", C.c_int32),
        ("draft_row_stats", C.c_void_p), ("draft_row_stats_stride", C.c_int64),
        ("draft_row_keep", C.c_void_p),
        ("status_or", C.c_void_p), ("row_counts", C.c_void_p),
    ]


class sd_sample_args(C.Structure):
    _fields_ = [
        ("rows", C.c_int32), ("vocab", C.c_int32), ("logits", C.c_void_p), ("stride_r", C.c_int64),
        ("dtype", C.c_int32), ("proc", sd_processor), ("noise", sd_noise),
        ("tokens", C.c_void_p), ("tokens_stride", C.c_int64), ("token_prob", C.c_void_p),
        ("row_status", C.c_void_p), ("words_used", C.c_void_p),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
        ("row_stats", C.c_void_p), ("row_keep", C.c_void_p),
        ("status_or", C.c_void_p),
    ]


class sd_probs_args(C.Structure):
    _fields_ = [
        ("rows", C.c_int32), ("vocab", C.c_int32), ("logits", C.c_void_p), ("stride_r", C.c_int64),
        ("dtype", C.c_int32), ("proc", sd_processor), ("probs", C.c_void_p), ("probs_stride_r", C.c_int64),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
    ]


class sd_ngram_args(C.Structure):
    _fields_ = [
        ("batch", C.c_int32), ("gamma", C.c_int32), ("vocab", C.c_int32),
        ("target_rows", C.c_void_p * (SD_MAX_GAMMA + 1)), ("target_stride_b", C.c_int64),
        ("target_dtype", C.c_int32),
        ("draft_tokens", C.c_void_p), ("draft_tokens_stride_b", C.c_int64),
        ("proc", sd_processor), ("stop_tokens", C.c_void_p), ("n_stop", C.c_int32), ("filler_k", C.c_int32),
        ("noise", sd_noise),
        ("n_accepted", C.c_void_p), ("next_token", C.c_void_p), ("prune_target", C.c_void_p),
        ("stop_index", C.c_void_p), ("row_status", C.c_void_p), ("words_used", C.c_void_p),
        ("filler_ids", C.c_void_p), ("filler_stride_b", C.c_int64),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
        ("status_or", C.c_void_p),
    ]


def _share_torch_hip_runtime():
    """Load PyTorch-ROCm's bundled HIP runtime first, so libspecdec.so (NEEDED libamdhip64.so.7,
    which that copy's SONAME satisfies) binds to the SAME runtime torch uses instead of loading
    /opt/rocm's second copy (two runtimes in one process do not share devices or streams)."""
    try:
        import torch
    except ImportError:
        return
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if os.path.exists(path):
        C.CDLL(path, mode=C.RTLD_GLOBAL)


def _load():
    _share_torch_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"specdec_amd: {LIB_PATH} not found — build it with "
                          f"`make -C speculative-decoding_amd` (hipcc, gfx950)")
    lib = C.CDLL(LIB_PATH)
    for name in EXPORTS:
        if not hasattr(lib, name):
            raise ImportError(f"specdec_amd: {LIB_PATH} does not export {name}")
    lib.sd_abi_version.restype = C.c_int32
    lib.sd_status_string.restype = C.c_char_p
    lib.sd_status_string.argtypes = [C.c_int32]
    lib.sd_last_hip_error.restype = C.c_char_p
    for ws in ("sd_verify_workspace_size",):
        getattr(lib, ws).restype = C.c_size_t
        getattr(lib, ws).argtypes = [C.c_int32, C.c_int32, C.c_int32]
    lib.sd_ngram_workspace_size.restype = C.c_size_t
    lib.sd_ngram_workspace_size.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    lib.sd_ngram_verify.restype = C.c_int32
    lib.sd_ngram_verify.argtypes = [C.POINTER(sd_ngram_args), C.c_void_p]
    for ws in ("sd_sample_workspace_size", "sd_probs_workspace_size"):
        getattr(lib, ws).restype = C.c_size_t
        getattr(lib, ws).argtypes = [C.c_int32, C.c_int32]
    lib.sd_verify.restype = C.c_int32
    lib.sd_verify.argtypes = [C.POINTER(sd_verify_args), C.c_void_p]
    lib.sd_sample.restype = C.c_int32
    lib.sd_sample.argtypes = [C.POINTER(sd_sample_args), C.c_void_p]
    lib.sd_probs.restype = C.c_int32
    lib.sd_probs.argtypes = [C.POINTER(sd_probs_args), C.c_void_p]
    lib.sd_mt19937_fill.restype = C.c_int32
    lib.sd_mt19937_fill.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64]
    lib.sd_mt19937_advance.restype = C.c_int32
    lib.sd_mt19937_advance.argtypes = [C.c_void_p, C.c_size_t, C.c_int64]
    for name, res, args in (
            ("sd_mt19937_state_from_torch", C.c_int32, [C.c_void_p, C.c_size_t, C.c_void_p]),
            ("sd_mt19937_state_to_torch", C.c_int32, [C.c_void_p, C.c_void_p, C.c_size_t]),
            ("sd_mt19937_jump_table", C.c_int32, [C.c_int64, C.c_int32, C.c_void_p]),
            ("sd_mt19937_char_poly", C.c_int32, [C.c_void_p, C.c_size_t]),
            ("sd_mt19937_fill_substreams", C.c_int32, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64, C.c_int64,
                                                        C.c_void_p, C.c_int32]),
            ("sd_mt19937_generate_workspace_size", C.c_size_t, [C.c_int64, C.c_int64]),
            ("sd_mt19937_generate", C.c_int32, [C.POINTER(sd_mt_generate_args), C.c_void_p]),
            ("sd_mt19937_commit", C.c_int32, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                                              C.c_void_p])):
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    lib.sd_set_poll_policy.restype = C.c_int32
    lib.sd_set_poll_policy.argtypes = [C.c_int32, C.c_int32]
    lib.sd_get_poll_policy.restype = C.c_int32
    lib.sd_get_poll_policy.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.sd_set_option.restype = C.c_int32
    lib.sd_set_option.argtypes = [C.c_int32, C.c_int32]
    lib.sd_get_option.restype = C.c_int32
    lib.sd_get_option.argtypes = [C.c_int32, C.POINTER(C.c_int32)]
    for name in ("sd_last_verify_path", "sd_last_sample_path"):
        getattr(lib, name).restype = C.c_int32
        getattr(lib, name).argtypes = []
    P = C.POINTER(sd_ngram_store)
    for name, args in (("sd_ngram_store_initialize", [P, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_int64, C.c_void_p]),
                       ("sd_ngram_store_update", [P, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_int32,
                                                  C.c_int64, C.c_int64, C.c_void_p]),
                       ("sd_ngram_store_next_token", [P, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_void_p,
                                                      C.c_void_p, C.c_void_p]),
                       ("sd_ngram_store_has_gram", [P, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
                       ("sd_ngram_store_draft", [P, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_void_p,
                                                 C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p])):
        getattr(lib, name).restype = C.c_int32
        getattr(lib, name).argtypes = args
    if lib.sd_abi_version() != SD_ABI_VERSION:
        raise ImportError(f"specdec_amd: ABI mismatch ({lib.sd_abi_version()} != {SD_ABI_VERSION})")
    return lib


lib = _load()


class SpecdecError(RuntimeError):
    pass


def check(status: int, what: str):
    if status != SD_OK:
        msg = f"{what}: {lib.sd_status_string(status).decode()} ({status})"
        if status == SD_ERR_LAUNCH:
            msg += f": {lib.sd_last_hip_error().decode()}"
        raise SpecdecError(msg)


def set_poll_policy(allow_poll: bool = True, spin_limit: int = 0) -> None:
    """sd_set_poll_policy: whether kernels may exchange partials by polling inside one launch (the
    occupancy check still decides per launch), and the bound of every poll in microseconds of wall
    clock (0 = the default 2 s; < 0 gives up at once — a test hook that forces the
    SD_ROW_EXCHANGE_TIMEOUT path)."""
    check(lib.sd_set_poll_policy(1 if allow_poll else 0, int(spin_limit)), "sd_set_poll_policy")


def get_poll_policy():
    """(allow_poll, spin_limit) as the library holds them."""
    a, s = C.c_int32(), C.c_int32()
    check(lib.sd_get_poll_policy(C.byref(a), C.byref(s)), "sd_get_poll_policy")
    return bool(a.value), int(s.value)


def set_option(option: int, value: int) -> None:
    """sd_set_option: a process-wide dispatch switch (SD_OPT_*) between equivalent kernel paths."""
    check(lib.sd_set_option(int(option), int(value)), "sd_set_option")


def get_option(option: int) -> int:
    v = C.c_int32()
    check(lib.sd_get_option(int(option), C.byref(v)), "sd_get_option")
    return int(v.value)


class option:
    """Context manager: ``with option(SD_OPT_FUSED_VERIFY, 0): ...`` restores the old value after."""

    def __init__(self, opt: int, value: int):
        self.opt, self.value = opt, value

    def __enter__(self):
        self.old = get_option(self.opt)
        set_option(self.opt, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.opt, self.old)
        return False


def last_verify_path() -> int:
    """SD_PATH_* of this thread's last successful sd_verify (which kernels ran)."""
    return int(lib.sd_last_verify_path())


def last_sample_path() -> int:
    """SD_PATH_* of this thread's last successful sd_sample."""
    return int(lib.sd_last_sample_path())


class RowError(RuntimeError):
    """A row's outputs are unusable (SD_ROW_ERROR_MASK): where the reference's torch.multinomial
    raises (NaN / inf / all-zero probabilities, engine/infer_engine.py:246,321-325,
    sampling/speculative_decoding.py:171), or an in-launch exchange timed out, or the STREAM noise
    ran short.  The message is torch's for the invalid-distribution case."""


def raise_row_error(bits: int, where: str) -> None:
    """Raise RowError for the SD_ROW_ERROR_MASK bits of a row status / status_or word (no-op for 0)."""
    bits = int(bits) & SD_ROW_ERROR_MASK
    if not bits:
        return
    parts = []
    if bits & SD_ROW_EXCHANGE_TIMEOUT:
        parts.append("an in-launch exchange timed out (sd_set_poll_policy(allow_poll=False) selects the "
                     "counter exchanges when other work shares the GPU)")
    if bits & SD_ROW_NOISE_OVERRUN:
        parts.append("the STREAM noise buffer ran short")
    if bits & SD_ROW_INVALID_DIST and not bits & SD_ROW_EXCHANGE_TIMEOUT:
        parts.append("probability tensor contains either `inf`, `nan` or element < 0")
    raise RowError(f"{where}: " + "; ".join(parts) + f" (row status bits 0x{bits:x})")
