#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (SQLite .db or kernel_stats.csv)
into a per-kernel table: launches, total ms, average us, max us."""
import csv
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    q = ("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3, max(end-start)/1e3 "
         "from kernels group by name order by sum(end-start) desc")
    return con.execute(q).fetchall()


def from_csv(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                         float(r["AverageNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    return sorted(rows, key=lambda x: -x[2])


def main():
    path = sys.argv[1]
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':58s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>10s} {'max_us':>10s} {'share':>6s}")
    for name, n, t, a, m in rows:
        print(f"{name[:58]:58s} {n:7d} {t:10.3f} {a:10.2f} {m:10.1f} {100 * t / tot:5.1f}%")
    print(f"{'TOTAL':58s} {'':7s} {tot:10.3f}")


if __name__ == "__main__":
    main()
