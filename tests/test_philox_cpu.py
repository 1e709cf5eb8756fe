"""The numpy Philox4x32-10 used to check the perf-mode kernels, pinned by the Random123
known-answer vectors (kat_vectors, philox4x32 R=10)."""
from philox_ref import philox4x32_10

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox4x32_10_known_answers():
    for ctr, key, want in KAT:
        got = tuple(int(v) for v in philox4x32_10(ctr, key))
        assert got == want, ([hex(g) for g in got], [hex(w) for w in want])
