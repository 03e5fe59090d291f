#!/usr/bin/env python3
"""Print the kernel sequence of the last MSM job(s) in a rocprofv3 trace."""
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, duration, start from kernels order by start"))
idx = [i for i, (n, d, s) in enumerate(rows) if "k_msm_digits" in n]
for j in [idx[int(a)] for a in (sys.argv[2:] or ["-1"])]:
    nxt = [i for i in idx if i > j]
    e = nxt[0] if nxt else len(rows)
    agg = {}
    for n, d, s in rows[j:e]:
        n2 = re.sub(r"\(.*", "", n).replace("bpg::dev::", "")[:50]
        a = agg.setdefault(n2, [0, 0]); a[0] += 1; a[1] += d
    tot = sum(a[1] for a in agg.values())
    for n2, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-50s x%-3d %9.1f us" % (n2, a[0], a[1] / 1e3))
    print("total %.1f us, span %.1f us\n" % (tot / 1e3, (rows[e - 1][2] + rows[e - 1][1] - rows[j][2]) / 1e3))
