#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter collections (any counters),
optionally over the dispatches from index --from on (per kernel).
usage: pmc_latency.py [--from K] [--kernels k_a,k_b] <counter_collection.csv>..."""
import csv
import re
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    k0 = 0
    kern = ("k_rescan_spec", "k_fused")
    while args and args[0] in ("--from", "--kernels"):
        if args[0] == "--from":
            k0 = int(args[1])
        else:
            kern = tuple(args[1].split(","))
        args = args[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for path in args:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0].replace("bpeamd::", "").replace("void ", "")).strip()
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in sorted(vals.items()):
        if not name.startswith(kern):
            continue
        parts = []
        for c, v in sorted(cs.items()):
            v = v[k0:] if len(v) > k0 else v
            parts.append(f"{c}={sum(v) / max(1, len(v)):.0f}")
        print(name, len(next(iter(cs.values()))), " ".join(parts))


if __name__ == "__main__":
    main()
