#!/usr/bin/env python3
"""Per-kernel roofline table from the reduced PMC passes of scripts/pmc_passes.sh
(pmc0 FETCH_SIZE, pmc1 WRITE_SIZE, pmc2 SQ issue/wait counters, pmc3
GRBM_GUI_ACTIVE), every pass a kernel-trace + one counter group. Counter
collection serialises the dispatches, so the durations are per-kernel
isolated times.

Per MI355X_MICROARCH.md: FETCH_SIZE (KB) counts half the bytes of 16-B-per-lane
reads on gfx950 (doubled here), WRITE_SIZE is exact for 16-B stores; SQ_*
cycle counters count quad-cycles; the effective clock is GRBM_GUI_ACTIVE / 8
(XCDs) / duration. MI355X: 256 CUs x 4 SIMDs.

usage: pmc_table.py <gpurun_out/r02c> [out.json]"""
import json
import sys

pre = sys.argv[1]
J = lambda i, f: json.load(open("%s_pmc%d/run_%s.json" % (pre, i, f)))  # noqa: E731
fetch, write, sq, grbm = J(0, "counter_collection"), J(1, "counter_collection"), J(2, "counter_collection"), \
    J(3, "counter_collection")
trace = J(2, "kernel_trace")
SIMDS = 1024
# the bench line the FETCH_SIZE pass printed: its live per-label table gives
# the algorithmic bytes per launch of each bracketed kernel in THIS run (same
# job mix as the counters), so hbm / alg is the kernel's over-fetch ratio
alg = {}
try:
    line = [ln for ln in open("%s_pmc0.json" % pre) if ln.startswith("{")][-1]
    for lab, r in ((json.loads(line).get("roofline") or {}).get("kernel_table") or {}).items():
        alg[r["rocprof_name"]] = dict(r, label=lab)
except (OSError, IndexError, ValueError):
    pass
rows = {}
for k, c in sq.items():
    t = trace.get(k, {})
    n = t.get("dispatches") or c.get("dispatches") or 1
    dur_s = t.get("duration_ns", 0) * 1e-9
    g = grbm.get(k, {})
    clk = g.get("GRBM_GUI_ACTIVE", 0) / 8 / dur_s if dur_s and "GRBM_GUI_ACTIVE" in g else 2.1e9
    cyc = dur_s * clk
    f = fetch.get(k, {}).get("FETCH_SIZE")
    w = write.get(k, {}).get("WRITE_SIZE")
    hbm = ((2 * f if f else 0) + (w or 0)) * 1024 / n
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    rows[k] = {
        "dispatches": n, "avg_us": dur_s / n * 1e6, "clock_ghz": clk / 1e9,
        "hbm_bytes_per_launch": hbm, "hbm_gbs": hbm * n / dur_s / 1e9 if dur_s else None,
        "valu_issue_share": 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / (SIMDS * cyc) if cyc else None,
        "avg_waves_per_simd": 4 * wc / (SIMDS * cyc) if cyc else None,
        "wave_active": c.get("SQ_ACTIVE_INST_ANY", 0) / wc, "wave_wait_mem": c.get("SQ_WAIT_ANY", 0) / wc,
        "wave_wait_issue": c.get("SQ_WAIT_INST_ANY", 0) / wc,
        "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1),
    }
    if k in alg:
        a = alg[k]["alg_bytes_per_launch"]
        rows[k].update(label=alg[k]["label"], alg_bytes_per_launch=a, bench_launches=alg[k]["launches"],
                       hbm_over_alg=hbm / a if a else None)
order = sorted(rows, key=lambda k: -rows[k]["avg_us"] * rows[k]["dispatches"])
print("| kernel | launches | avg us | GHz | HBM B/launch | alg B/launch | HBM/alg | HBM GB/s | VALU issue share | "
      "waves/SIMD | wave active | wait mem | wait issue |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
for k in order[:24]:
    r = rows[k]
    print("| %s | %d | %.1f | %.2f | %.3g | %s | %s | %.0f | %.3f | %.2f | %.2f | %.2f | %.2f |" % (
        k, r["dispatches"], r["avg_us"], r["clock_ghz"], r["hbm_bytes_per_launch"],
        "%.3g" % r["alg_bytes_per_launch"] if r.get("alg_bytes_per_launch") else "",
        "%.1f" % r["hbm_over_alg"] if r.get("hbm_over_alg") else "", r["hbm_gbs"] or 0,
        r["valu_issue_share"] or 0, r["avg_waves_per_simd"] or 0, r["wave_active"], r["wave_wait_mem"],
        r["wave_wait_issue"]))
if len(sys.argv) > 2:
    json.dump({"source": pre, "kernels": rows}, open(sys.argv[2], "w"), indent=1, sort_keys=True)
