#!/usr/bin/env python3
"""Per-kernel launches / total / average from a rocprofv3 kernel_trace.csv,
over all launches and over the launches longer than a threshold (the batch
engine's pipelined graphs queue kernels past a stop, which exit at once).
usage: prof_nonempty.py run_kernel_trace.csv [threshold_us=6] [kernels,...]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
    want = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    d = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("bpeamd::", "").strip()
            d[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':40s} {'launches':>8s} {'avg_us':>9s} | {'>= %g us' % thr:>9s} {'avg_us':>9s} {'total_ms':>9s}")
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        if want and not name.startswith(want):
            continue
        big = [x for x in v if x >= thr]
        print(f"{name[:40]:40s} {len(v):8d} {sum(v) / len(v):9.2f} | {len(big):9d} "
              f"{(sum(big) / len(big) if big else 0):9.2f} {sum(v) / 1e3:9.3f}")


if __name__ == "__main__":
    main()
