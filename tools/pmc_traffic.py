#!/usr/bin/env python3
"""HBM traffic per launch of the engine's kernels from two rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

rocprofv3 reports both in KiB.  MI355X_MICROARCH.md (HBM): on gfx950
FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane) coalesced
streaming read, so k_pair_hist's fetch is doubled; for the random 4-byte
gathers of the per-merge kernels the counter is uncalibrated and reported raw.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import csv
import re
import json
import sys
from collections import defaultdict

WIDE_STREAM = {"k_pair_hist", "k_pair_hist_span", "k_pair_hist_v", "k_live_compact", "k_enc_win"}  # whole-line coalesced streaming reads: FETCH_SIZE x 2


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("bpeamd::", "")
            name = re.sub(r"<.*>", "", name.replace("void ", "")).strip()  # "void k_scan<false>" -> "k_scan"
            vals[name].append(float(r["Counter_Value"]))
    return vals


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 1024.0 * sum(f) / max(1, len(f))
        wb = 1024.0 * sum(w) / max(1, len(w))
        corr = 2.0 if k in WIDE_STREAM else 1.0
        out[k] = {"launches": max(len(f), len(w)), "fetch_bytes_raw": round(fb), "write_bytes": round(wb),
                  "fetch_correction": corr, "traffic_bytes_per_launch": round(fb * corr + wb)}
    with open(sys.argv[3], "w") as fo:
        json.dump(out, fo, indent=1)
    for k, v in out.items():
        print(k, v)


if __name__ == "__main__":
    main()
