#!/usr/bin/env python3
"""Summarise a rocprofv3 run (rocpd SQLite output or *_kernel_stats.csv) as a
kernel table: name, calls, total/avg/min/max duration (us), share.
usage: prof_summary.py <run_results.db | kernel_stats.csv> [out.md]"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    if "rocprim" in name:
        m = re.search(r"(radix_sort_\w+|merge_sort_\w+|scan_\w+|transform_\w+|init_lookback\w+)", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    return name.replace("bpg::dev::", "")


def from_db(path):
    c = sqlite3.connect(path)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        r = rows.setdefault(short(name), [0, 0.0, float("inf"), 0.0])
        r[0] += 1
        r[1] += dur
        r[2] = min(r[2], dur)
        r[3] = max(r[3], dur)
    return rows


def from_csv(path):
    rows = {}
    for d in csv.DictReader(open(path)):
        k = short(d["Name"])
        r = rows.setdefault(k, [0, 0.0, float("inf"), 0.0])
        r[0] += int(d["Calls"])
        r[1] += float(d["TotalDurationNs"])
        r[2] = min(r[2], float(d["MinNs"]))
        r[3] = max(r[3], float(d["MaxNs"]))
    return rows


def main():
    src = sys.argv[1]
    rows = from_db(src) if src.endswith(".db") else from_csv(src)
    tot = sum(r[1] for r in rows.values()) or 1
    out = ["| kernel | calls | total ms | avg us | min us | max us | share |", "|---|---|---|---|---|---|---|"]
    for k, r in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        out.append("| %s | %d | %.2f | %.1f | %.1f | %.1f | %.1f%% |" %
                   (k, r[0], r[1] / 1e6, r[1] / r[0] / 1e3, r[2] / 1e3, r[3] / 1e3, 100 * r[1] / tot))
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
