#!/usr/bin/env python3
"""HBM bytes per launch from rocprofv3 PMC passes (scripts/pmc.sh): pass 0
FETCH_SIZE, pass 1 WRITE_SIZE, each in KB per dispatch. Per
MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE counts half the bytes of
16-B-per-lane reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.
usage: pmc_summary.py <prefix e.g. gpurun_out/r01g_pmc> <out.json>"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n).replace("bpg::dev::", "").replace("void ", "")
    return n.strip()


def load(path, counter):
    agg = defaultdict(lambda: [0, 0.0])
    for d in csv.DictReader(open(path)):
        if d["Counter_Name"] != counter:
            continue
        a = agg[short(d["Kernel_Name"])]
        a[0] += 1
        a[1] += float(d["Counter_Value"])
    return agg


pre, out = sys.argv[1], sys.argv[2]
fetch = load(pre + "0/run_counter_collection.csv", "FETCH_SIZE")
write = load(pre + "1/run_counter_collection.csv", "WRITE_SIZE")
res = {}
for k in set(fetch) | set(write):
    f, w = fetch.get(k, [0, 0.0]), write.get(k, [0, 0.0])
    fb = 2 * 1024 * f[1] / f[0] if f[0] else None
    wb = 1024 * w[1] / w[0] if w[0] else None
    res[k] = {"launches": max(f[0], w[0]), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
              "hbm_bytes_per_launch": (fb or 0) + (wb or 0)}
json.dump({"source": pre, "correction": "FETCH_SIZE x 2 (gfx950, 16-B/lane reads), WRITE_SIZE x 1; KB -> B",
           "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
    print("%-32s %6d launches  %.3g B/launch" % (k, v["launches"], v["hbm_bytes_per_launch"]))
