"""Seeded synthetic corpora shaped like the reference's random_text.txt.

random_text.txt (reference, 1,048,576 B) is i.i.d.-looking bytes over the 95
printable ASCII values 32..126 with no NUL or newline.  The
reference file itself is not copied into this repository; benches and tests use
this counter-based generator instead:

    z_i    = mix64(seed + (i + 1) * 0x9E3779B97F4A7C15)      (splitmix64)
    byte_i = 32 + (((z_i >> 32) * 95) >> 32)

It is counter-based, so any slice [lo, hi) of a corpus can be produced
independently (multi-GPU shards generate their own slice) and the device-side
generator (bpe_gpu_synth in libbpe_amd) produces the identical bytes.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def synth_bytes(seed: int, n: int, lo: int = 0, chunk: int = 1 << 24) -> bytes:
    """Bytes lo..lo+n-1 of the corpus with the given seed."""
    out = np.empty(n, dtype=np.uint8)
    s = np.uint64(seed)
    with np.errstate(over="ignore"):
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            i = np.arange(lo + c0 + 1, lo + c1 + 1, dtype=np.uint64)
            z = _mix64(s + i * GOLDEN)
            hi = z >> np.uint64(32)
            out[c0:c1] = (np.uint64(32) + ((hi * np.uint64(95)) >> np.uint64(32))).astype(np.uint8)
    return out.tobytes()
