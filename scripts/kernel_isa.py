#!/usr/bin/env python3
"""Per-kernel instruction counts of the gfx950 build of kernels.hip (device
assembly, static counts): total, VALU, v_mad_u64_u32. Used to check that a
formula change removes instructions before spending GPU time on it.
usage: kernel_isa.py [out.txt]   (compiles to /tmp/bpg_kernels.s)"""
import re
import subprocess
import sys
from collections import Counter

SRC = "bulletproof-gadgets_amd/csrc/device/kernels.hip"
ASM = "/tmp/bpg_kernels.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                       "-S", "-o", ASM, SRC])
kern, counts = None, {}
for line in open(ASM):
    m = re.match(r"^(_Z\w+):", line)
    if m:
        kern = m.group(1)
        counts[kern] = Counter()
        continue
    if kern and line.startswith("\t.section") or (kern and line.startswith("\t.end_amdhsa")):
        kern = None
        continue
    if kern:
        t = line.strip().split()
        if t and re.match(r"^[vsgdb][a-z_0-9]+$", t[0]) and not t[0].startswith("."):
            counts[kern][t[0]] += 1
out = []
for k, c in sorted(counts.items(), key=lambda kv: -sum(kv[1].values())):
    tot = sum(c.values())
    if tot < 200:
        continue
    valu = sum(v for i, v in c.items() if i.startswith("v_"))
    out.append("%6d total %6d valu %5d v_mad_u64_u32  %s" % (tot, valu, c["v_mad_u64_u32"], k[:110]))
txt = "\n".join(out) + "\n"
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(txt)
print(txt)
