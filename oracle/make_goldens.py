#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY: regenerate tests/golden/*.json from the
unmodified reference (oracle/_ref/bpe_ref, built by oracle/build_ref.sh from
/root/reference) -- run in the build container, never on the GPU box.

Each fixture holds the input (inline base64 for small inputs, or a synth
recipe seed/size for the generator in llmtokenizer_amd/synth.py), the merge cap
passed to the reference through BPE_REF_MAX_MERGES, and the reference's
outputs: the merge list and the final ids (inline when small, else length +
md5 of the little-endian u32 array).  Nothing from the reference's sources is
stored; only its outputs on our inputs.

usage: python3 oracle/make_goldens.py [--big] [--only NAME...]
"""
import argparse
import base64
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from llmtokenizer_amd.synth import synth_bytes  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "bpe_ref")
GOLD = os.path.join(ROOT, "tests", "golden")

PROSE = (
    "Byte pair encoding starts from single bytes and repeatedly fuses the most "
    "frequent adjacent pair into a new symbol. The trainer counts every pair, "
    "picks the winner, records it, and rewrites the text; the encoder replays "
    "the recorded merges in order. Ties are common: many pairs share the same "
    "count, so the order in which the counting table is walked decides which "
    "pair wins. A faithful port has to walk the same order, bucket by bucket, "
    "even when the table is rebuilt on a graphics processor with thousands of "
    "lanes counting at once. The quick brown fox jumps over the lazy dog; the "
    "lazy dog sleeps, the quick fox jumps again, and again, and again.\n"
).encode()


def cases(big: bool):
    c = []
    c.append(dict(name="prose", data=PROSE, max_merges=-1))
    # within-bucket tie KATs: X="!k" (33,107), Y="&?" (38,63)
    # collide modulo 65536, so the chain order decides the winner.
    X, Y = b"!k", b"&?"
    tail = b"abcdefghijlmnopqrstuvwxyz"
    c.append(dict(name="kat_tie_xy", data=X + b"0" + Y + b"1" + X + b"2" + Y + b"3" + X + b"4" + Y + b"5" + tail, max_merges=1))
    c.append(dict(name="kat_tie_yx", data=Y + b"0" + X + b"1" + Y + b"2" + X + b"3" + Y + b"4" + X + b"5" + tail, max_merges=1))
    c.append(dict(name="kat_tie_yyyxxx", data=Y + b"0" + Y + b"1" + Y + b"2" + tail + b"ABCDEFGHIJKLMNOPQRS" + X + b"3" + X + b"4" + X + b"5", max_merges=1))
    c.append(dict(name="kat_tie_xxxyyy", data=X + b"0" + X + b"1" + X + b"2" + tail + b"ABCDEFGHIJKLMNOPQRS" + Y + b"3" + Y + b"4" + Y + b"5", max_merges=1))
    # degenerate shapes
    c.append(dict(name="two_bytes", data=b"ab", max_merges=-1))
    c.append(dict(name="aaaa", data=b"aaaa", max_merges=-1))
    c.append(dict(name="run_a_1000", data=b"a" * 1000, max_merges=-1))
    c.append(dict(name="run_a_777_b", data=b"a" * 777 + b"b" + b"a" * 333, max_merges=-1))
    c.append(dict(name="abab_500", data=b"ab" * 500, max_merges=-1))
    c.append(dict(name="aab_runs", data=(b"aab" * 50 + b"aaab" * 40 + b"aaaaab" * 30) * 3, max_merges=-1))
    c.append(dict(name="nul_truncates", data=b"hello hello hello\x00world world world", max_merges=-1))
    rng = np.random.default_rng(5)
    c.append(dict(name="binary_5k", data=rng.integers(1, 256, 5000, dtype=np.uint8).tobytes(), max_merges=-1))
    c.append(dict(name="binary_skew_20k", data=np.minimum(rng.geometric(0.08, 20000), 255).astype(np.uint8).tobytes(), max_merges=400))
    # random_text.txt-shaped corpora (static split, chain ties appear late)
    c.append(dict(name="synth_s1_4k", seed=1, n=4096, max_merges=-1))
    for seed, n, m in ((101, 3000, 300), (103, 20000, 300), (118, 20000, 300),
                       (102, 70000, 120), (149, 3000, 300), (158, 3000, 300)):
        c.append(dict(name=f"synth_s{seed}_{n}", seed=seed, n=n, max_merges=m))
    c.append(dict(name="synth_s7_64k", seed=7, n=65536, max_merges=512))
    c.append(dict(name="synth_s3_300k", seed=3, n=300000, max_merges=256))
    # the reference's own corpora, committed as data fixtures
    # under tests/golden/: testing.txt to the stop rule (config 0's input) and
    # random_text.txt x 1024 merges (config 1's input; ~2 min of reference time)
    c.append(dict(name="ref_testing", file="testing.txt", max_merges=-1))
    if big:
        c.append(dict(name="ref_random_text", file="random_text.txt", max_merges=1024))
        # config 2 analog: 1 MiB (n == 2^20: iteration 0 is dynamic), 1024 merges
        c.append(dict(name="synth_s1_1m", seed=1, n=1 << 20, max_merges=1024))
        # dynamic but tracked (2^20 <= n < 2^21)
        c.append(dict(name="synth_s4_1500k", seed=4, n=1_500_000, max_merges=48))
        # 64 MiB, 16 merges; 1 GiB, 4 merges (seed 2 = the bench corpus)
        c.append(dict(name="synth_s2_64m", seed=2, n=64 << 20, max_merges=16))
        c.append(dict(name="synth_s2_1g", seed=2, n=1 << 30, max_merges=4))
    return c


# fixtures that also keep the reference's own dump_pairs file (bpe.c:243-278)
# and main.c's stdout (print_text of the encoding, bpe.c:182-196)
WITH_IO = ("prose", "synth_s1_4k", "aab_runs", "binary_5k", "nul_truncates", "ref_testing", "ref_random_text")


def run_ref(data: bytes, max_merges: int, with_io=False):
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.bin")
        with open(inp, "wb") as f:
            f.write(data)
        mo, io_, po = os.path.join(td, "m.txt"), os.path.join(td, "i.bin"), os.path.join(td, "p.bin")
        env = dict(os.environ, BPE_REF_MAX_MERGES=str(max_merges), BPE_REF_PRINT="1" if with_io else "0")
        t0 = time.time()
        p = subprocess.run([REF, inp, mo, io_] + ([po] if with_io else []), env=env, capture_output=True)
        dt = time.time() - t0
        if p.returncode != 0:
            return dict(error=True, stdout=p.stdout.decode(errors="replace"), seconds=dt)
        merges = []
        with open(mo) as f:
            for line in f:
                i, a, b = line.split()
                merges.append([int(a), int(b)])
        ids = np.fromfile(io_, dtype="<u4")
        out = dict(error=False, merges=merges, ids=ids, seconds=dt)
        if with_io:
            with open(po, "rb") as f:
                out["pairs_file"] = f.read()
            out["print_text"] = p.stdout
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit("oracle/_ref/bpe_ref missing: run oracle/build_ref.sh first")
    os.makedirs(GOLD, exist_ok=True)
    for c in cases(args.big):
        if args.only and c["name"] not in args.only:
            continue
        data = c.get("data")
        if "file" in c:
            with open(os.path.join(GOLD, c["file"]), "rb") as f:
                data = f.read()
        elif data is None:
            data = synth_bytes(c["seed"], c["n"])
        r = run_ref(data, c["max_merges"], with_io=c["name"] in WITH_IO)
        fx = dict(name=c["name"], max_merges=c["max_merges"], generator="oracle/make_goldens.py",
                  ref_seconds=round(r["seconds"], 3))
        if "file" in c:
            fx["input_file"] = c["file"]
            fx["input_sha256"] = hashlib.sha256(data).hexdigest()
        elif "data" in c:
            fx["input_b64"] = base64.b64encode(c["data"]).decode()
        else:
            fx["synth"] = dict(seed=c["seed"], n=c["n"])
        if r["error"]:
            fx["error"] = True
            fx["stdout"] = r["stdout"]
        else:
            ids = r["ids"]
            fx["merges"] = r["merges"]
            fx["ids_len"] = int(ids.size)
            fx["ids_md5"] = hashlib.md5(ids.astype("<u4").tobytes()).hexdigest()
            if ids.size <= 4096:
                fx["ids"] = ids.tolist()
            if "pairs_file" in r:
                fx["dump_pairs_b64"] = base64.b64encode(r["pairs_file"]).decode()
                fx["print_text_md5"] = hashlib.md5(r["print_text"]).hexdigest()
                fx["print_text_len"] = len(r["print_text"])
        with open(os.path.join(GOLD, c["name"] + ".json"), "w") as f:
            json.dump(fx, f, separators=(",", ":"))
        print(f"{c['name']}: merges={len(fx.get('merges', []))} ids_len={fx.get('ids_len')} "
              f"ref {r['seconds']:.2f}s", flush=True)


if __name__ == "__main__":
    main()
