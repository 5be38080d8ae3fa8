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


def english_like(n: int, seed: int = 7) -> bytes:
    """n bytes of Zipf-distributed pseudo-words over English letter
    frequencies with spaces, commas, periods and newlines (no real text is
    shipped here): the skewed-pair workload of tools/init_skew.py and the
    batch engine's regression tests"""
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b"etaoinshrdlcumwfgypbvkjxqz", np.uint8)
    freq = np.array([12.7, 9.1, 8.2, 7.5, 7.0, 6.7, 6.3, 6.1, 6.0, 4.3, 4.0, 2.8, 2.8, 2.4, 2.4, 2.2, 2.0,
                     2.0, 1.9, 1.5, 1.0, 0.8, 0.15, 0.15, 0.1, 0.07])
    freq /= freq.sum()
    nw = 20000
    lens = np.clip(rng.geometric(0.22, nw), 1, 14)
    words = [bytes(rng.choice(letters, L, p=freq)) for L in lens]
    ranks = np.minimum(rng.zipf(1.15, n // 5 + 16) - 1, nw - 1)
    seps = rng.choice(np.frombuffer(b"    ,.\n", np.uint8), ranks.size, p=[0.8 / 4] * 4 + [0.1, 0.07, 0.03])
    bank = np.frombuffer(b"".join(words), np.uint8)
    woff = np.concatenate([[0], np.cumsum(lens)[:-1]])
    wl = lens[ranks] + 1  # the word and its separator
    ends = np.cumsum(wl)
    k = int(np.searchsorted(ends, n)) + 1
    ranks, seps, wl, ends = ranks[:k], seps[:k], wl[:k], ends[:k]
    starts = ends - wl
    # position j of the output: word t = the one whose span holds j, offset j - starts[t]
    t = np.repeat(np.arange(k), wl)
    off = np.arange(t.size) - starts[t]
    out = np.where(off < lens[ranks][t], bank[np.minimum(woff[ranks][t] + off, bank.size - 1)], seps[t]).astype(np.uint8)
    return out[:n].tobytes()
