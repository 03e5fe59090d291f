"""Extract DATA (no code) from the reference checkout into tests/golden/.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/extract_reference_data.py
Outputs:
  mimc_round_constants.hex  — the 486 MiMC-769 round constants as 32-byte LE hex,
                              one per line (src/mimc_hash/mimc_consts.rs:2)
  resources/<name>.{gadgets,inst,wtns} — the reference CLI fixtures
                              (tests/resources/*, example.*), copied verbatim
"""
import os
import re
import shutil

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = open(os.path.join(REF, "src/mimc_hash/mimc_consts.rs")).read()
    rows = re.findall(r"\[((?:\s*0x[0-9a-fA-F]{2},?){32})\s*\]", src)
    assert len(rows) == 486, len(rows)
    with open(os.path.join(HERE, "mimc_round_constants.hex"), "w") as f:
        for r in rows:
            f.write(bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", r)).hex() + "\n")
    dst = os.path.join(HERE, "resources")
    os.makedirs(dst, exist_ok=True)
    res = os.path.join(REF, "tests/resources")
    for fn in sorted(os.listdir(res)):
        shutil.copy(os.path.join(res, fn), os.path.join(dst, fn))
    for ext in ("gadgets", "inst", "wtns"):
        shutil.copy(os.path.join(REF, "example." + ext), os.path.join(dst, "example." + ext))


if __name__ == "__main__":
    main()
