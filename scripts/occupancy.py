#!/usr/bin/env python3
"""GPU occupancy from a rocprofv3 kernel trace (rocpd db): busy union,
mean concurrency, and per-kernel share of workgroup-time (duration x
min(1, workgroups / (CUs x slots))) — a proxy for the chip capacity each
kernel consumes when streams overlap.
usage: occupancy.py run_results.db [t0_fraction t1_fraction]"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
q = "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels"
try:
    rows = list(db.execute(q))
except sqlite3.Error:
    print(cols)
    raise
rows.sort(key=lambda r: r[1])
t0, t1 = rows[0][1], max(r[2] for r in rows)
if len(sys.argv) > 3:
    a, b = float(sys.argv[2]), float(sys.argv[3])
    lo, hi = t0 + a * (t1 - t0), t0 + b * (t1 - t0)
    rows = [r for r in rows if r[1] >= lo and r[2] <= hi]
    t0, t1 = lo, hi
ev = []
for r in rows:
    ev.append((r[1], 1)); ev.append((r[2], -1))
ev.sort()
busy = 0; conc = 0; last = ev[0][0]; area = 0
for t, d in ev:
    if conc > 0:
        busy += t - last; area += conc * (t - last)
    conc += d; last = t
print("window %.1f ms, GPU busy (any kernel) %.1f%%, mean concurrency while busy %.2f" %
      ((t1 - t0) / 1e6, 100 * busy / (t1 - t0), area / max(busy, 1)))
CU, SLOTS = 256, 8
agg = defaultdict(lambda: [0, 0.0, 0.0])
for name, s, e, gx, gy, gz, wx in rows:
    n = re.sub(r"\(.*", "", name).replace("bpg::dev::", "")
    if "rocprim" in n:
        n = "rocprim"
    wgs = max(1, (gx * gy * gz) // max(wx, 1))
    frac = min(1.0, wgs / (CU * SLOTS))
    a = agg[n]; a[0] += 1; a[1] += (e - s); a[2] += (e - s) * frac
tot = sum(a[2] for a in agg.values())
print("%-34s %6s %10s %12s %7s" % ("kernel", "calls", "dur ms", "CU-wt ms", "share"))
for n, a in sorted(agg.items(), key=lambda kv: -kv[1][2])[:22]:
    print("%-34s %6d %10.1f %12.1f %6.1f%%" % (n[:34], a[0], a[1] / 1e6, a[2] / 1e6, 100 * a[2] / tot))
print("sum CU-weighted %.1f ms over a %.1f ms window" % (tot / 1e6, (t1 - t0) / 1e6))
