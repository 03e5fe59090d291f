#!/usr/bin/env python3
"""Reduce a rocprofv3 CSV on the GPU box (so gpurun_out/ stays small): per
kernel name, the dispatch count and the sum of every counter
(counter_collection.csv) or of the durations in ns (kernel_trace.csv).
usage: pmc_reduce.py <in.csv> <out.json>"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*", "", n).replace("bpg::dev::", "").replace("void ", "").strip()


src, out = sys.argv[1], sys.argv[2]
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in csv.DictReader(open(src)):
    k = short(d.get("Kernel_Name", "?"))
    if "Counter_Name" in d:
        agg[k][d["Counter_Name"]] += float(d["Counter_Value"])
        disp[k].add(d.get("Dispatch_Id") or d.get("Correlation_Id"))
    elif "Start_Timestamp" in d:
        agg[k]["duration_ns"] += float(d["End_Timestamp"]) - float(d["Start_Timestamp"])
        agg[k]["dispatches"] += 1
res = {k: dict(v, **({"dispatches": len(disp[k])} if disp[k] else {})) for k, v in agg.items()}
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
