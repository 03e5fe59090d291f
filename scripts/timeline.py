#!/usr/bin/env python3
"""GPU occupancy of a rocprofv3 kernel trace (rocpd SQLite output).

Prints the traced span, the union of kernel intervals (time the GPU had at
least one kernel resident), the mean number of concurrently resident kernels,
and per kernel: calls, summed duration, and its share of the busy union
(each instant of the union is split evenly over the kernels resident then).
Also: time with k kernels resident (k = 0, 1, 2, 3, 4+) and the time at
least one VALU-heavy kernel (MSM pass 1, comb/Straus folds) was resident.
usage: timeline.py <run_results.db> [t_from_frac] [out.md] [t_to_frac]
"""
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("bpg::dev::", "").replace("void ", "")


def main():
    db = sys.argv[1]
    frac0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    s_col = "start" if "start" in cols else [x for x in cols if "start" in x][0]
    e_col = "end" if "end" in cols else [x for x in cols if x.endswith("end")][0]
    ev = [(int(s), int(e), short(n)) for n, s, e in c.execute("select name, %s, %s from kernels" % (s_col, e_col))]
    ev.sort()
    t_lo, t_hi = ev[0][0], max(e for _, e, _ in ev)
    frac1 = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
    cut = t_lo + frac0 * (t_hi - t_lo)
    cut1 = t_lo + frac1 * (t_hi - t_lo)
    ev = [x for x in ev if x[0] >= cut and x[1] <= cut1]
    t_lo = ev[0][0]
    t_hi = max(e for _, e, _ in ev)
    heavy = ("k_rbk_pass<true", "k_ipp_comb_fold", "k_ipp_fold2", "k_ipp_fold3")
    hist = [0] * 5
    heavy_t = 0
    pts = []
    for i, (s, e, n) in enumerate(ev):
        pts.append((s, 1, i))
        pts.append((e, -1, i))
    pts.sort(key=lambda p: (p[0], p[1]))
    active = set()
    last = t_lo
    busy = 0
    conc = 0.0
    share = {}
    calls = {}
    dur = {}
    for s, e, n in ev:
        calls[n] = calls.get(n, 0) + 1
        dur[n] = dur.get(n, 0) + (e - s)
    for t, d, i in pts:
        if t > last:
            hist[min(len(active), 4)] += t - last
            if any(ev[j][2].startswith(heavy) for j in active):
                heavy_t += t - last
        if active and t > last:
            dt = t - last
            busy += dt
            conc += dt * len(active)
            w = dt / len(active)
            for j in active:
                share[ev[j][2]] = share.get(ev[j][2], 0) + w
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    span = t_hi - t_lo
    lines = ["span %.2f ms, busy union %.2f ms (%.1f%%), mean resident kernels while busy %.2f, kernels %d" %
             (span / 1e6, busy / 1e6, 100 * busy / span, conc / max(busy, 1), len(ev)),
             "time with 0/1/2/3/4+ kernels resident: " + " / ".join("%.1f%%" % (100 * h / span) for h in hist) +
             "; a VALU-heavy kernel resident %.1f%%" % (100 * heavy_t / span), "",
             "| kernel | calls | sum dur ms | avg us | share of busy ms | share % |", "|---|---|---|---|---|---|"]
    for n in sorted(share, key=lambda k: -share[k]):
        lines.append("| %s | %d | %.2f | %.1f | %.2f | %.1f%% |" % (n, calls[n], dur[n] / 1e6, dur[n] / calls[n] / 1e3,
                                                                 share[n] / 1e6, 100 * share[n] / busy))
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
