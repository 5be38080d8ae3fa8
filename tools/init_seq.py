#!/usr/bin/env python3
"""The kernel sequence of the last training job's init from a rocprofv3
kernel_trace.csv: every launch from the last `start` kernel (default
k_pair_hist_v, the count pass) up to the first batch scan, with its duration
and the idle gap before it (host round trips show up as gaps).
usage: init_seq.py run_kernel_trace.csv [start_kernel] [stop_kernel]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    start = sys.argv[2] if len(sys.argv) > 2 else "k_presence"
    stop = sys.argv[3] if len(sys.argv) > 3 else "k_bscan"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("bpeamd::", "").strip()
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    # the last job: the last launch of `start` followed by a `stop`
    idx = [i for i, r in enumerate(rows) if r[2].startswith(start)]
    if not idx:
        print("no", start)
        return
    i0 = idx[-1]
    if not any(r[2].startswith(stop) for r in rows[i0:]) and len(idx) > 1:
        i0 = idx[-2]
    t0 = rows[i0][0]
    prev_end = t0
    busy = 0
    print(f"{'t_us':>9s} {'gap_us':>8s} {'dur_us':>8s}  kernel")
    for s, e, n in rows[i0:]:
        if n.startswith(stop):
            print(f"{(s - t0) / 1e3:9.1f} {(s - prev_end) / 1e3:8.1f} {'':>8s}  {n} (first)")
            break
        busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} {(s - prev_end) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {n}")
        prev_end = max(prev_end, e)
    print(f"kernels busy {busy / 1e3:.1f} us of {(prev_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
