#!/usr/bin/env python3
"""Extract the inputs and expected verdicts of the reference's round-trip
tests (the accept/reject matrix) into reference_cases.json.

Run in the CPU container, where /root/reference exists; the JSON is committed
and is all tests/test_reference_matrix.py and tests/test_gpu_reference_matrix.py
read. Extracted per `#[test] fn` (in file order): the byte literals
(`vec![0x.., ..]`, decimal too) in textual order, the 32-byte constant names
the body uses (`W8.to_vec()`, `VALUE1.to_vec()`) in order with the vector
they are pushed into, the same tokens grouped by the `let` statement that
binds them, `hash!` patterns, `let n = <int>` values, the
Transcript label and the expected verdict of the final `verify(...)`
assertion (is_ok / is_err) with its line. Named `[u8; 32]` constants are
extracted per file. Only data is written, no source text.

usage: python tests/golden/extract_reference_cases.py [/root/reference]
"""
import json
import os
import re
import sys

FILES = [
    "src/bounds_check/bounds_check_gadget.rs", "src/equality/equality_gadget.rs",
    "src/inequality/inequality_gadget.rs", "src/less_than/less_than_gadget.rs",
    "src/merkle_tree/merkle_tree_gadget.rs", "src/mimc_hash/mimc_hash_gadget.rs",
    "src/or/or_conjunction.rs", "src/set_membership/set_membership_gadget.rs", "src/utils.rs",
    "tests/combine_gadgets.rs",
]
NUM = r"(?:0x[0-9a-fA-F]+|\d+)"
BYTES_RE = re.compile(r"vec!\[\s*(" + NUM + r"(?:\s*,\s*" + NUM + r")*)\s*,?\s*\]")
TOKEN_RE = re.compile(r"\b((?:W|VALUE)\d+)\.to_vec\(\)|vec!\[\s*(" + NUM + r"(?:\s*,\s*" + NUM + r")*)\s*,?\s*\]")
CONST_RE = re.compile(r"const\s+(\w+)\s*:\s*\[u8;\s*32\]\s*=\s*\[([^\]]*)\]", re.S)


def strip_comments(s):
    return re.sub(r"//[^\n]*", "", s)


def to_bytes(body):
    return bytes(int(x, 0) for x in re.split(r"\s*,\s*", body.strip().rstrip(",")) if x)


def block_end(text, start):
    """index just past the brace block opening at text[start] == '{'."""
    depth = 0
    for i in range(start, len(text)):
        if text[i] == "{":
            depth += 1
        elif text[i] == "}":
            depth -= 1
            if depth == 0:
                return i + 1
    raise ValueError("unbalanced braces")


def extract(path):
    raw = open(path).read()
    text = strip_comments(raw)
    consts = {m.group(1): to_bytes(m.group(2)).hex() for m in CONST_RE.finditer(text)}
    tests = []
    for m in re.finditer(r"#\[test\]\s*(#\[ignore\]\s*)?fn\s+(\w+)\s*\(\s*\)\s*\{", text):
        a = m.end() - 1
        b = block_end(text, a)
        body = text[a:b]
        verdicts = re.findall(r"verify\([^;]*\)\s*\.(is_ok|is_err)\(\)", body)
        labels = re.findall(r'Transcript::new\(b"([^"]*)"\)', body)
        refs = [(mm.group(1), mm.group(2)) for mm in
                re.finditer(r"(?:(\w+)\.push\()?\b((?:W|VALUE)\d+)\.to_vec\(\)", body)]
        pats = [re.sub(r"\s+", "", p) for p in re.findall(r"Pattern\s*=\s*(hash!\(.*?\));", body, re.S)]
        ints = [int(x) for x in re.findall(r"let\s+n\s*=\s*(\d+)\s*;", body)]
        # line of the final verdict assertion in the original file
        line = None
        if verdicts:
            pos = raw.find("fn " + m.group(2) + "(")
            end = raw.find("\n    }\n", pos)
            seg = raw[pos:end if end > 0 else len(raw)]
            k = max(seg.rfind(".is_ok()"), seg.rfind(".is_err()"))
            line = raw[:pos + k].count("\n") + 1
        # let-bound values: name -> tokens in order, a token being a constant
        # name ("W8", "VALUE1") or the hex of a byte literal
        lets = {}
        for lm in re.finditer(r"let\s+(?:mut\s+)?(\w+)\s*(?::[^=;]*)?=\s*(.*?);", body, re.S):
            toks = []
            for t in TOKEN_RE.finditer(lm.group(2)):
                toks.append(t.group(1) if t.group(1) else to_bytes(t.group(2)).hex())
            if toks:
                lets[lm.group(1)] = toks
        tests.append({"fn": m.group(2), "ignored": bool(m.group(1)), "label": labels[0] if labels else None, "lets": lets,
                      "verdict": verdicts[-1][3:] if verdicts else None, "verdict_line": line,
                      "bytes": [to_bytes(x.group(1)).hex() for x in BYTES_RE.finditer(body)],
                      "refs": refs, "patterns": pats, "ints": ints})
    return {"consts": consts, "tests": tests}


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = {f: extract(os.path.join(ref, f)) for f in FILES}
    here = os.path.dirname(os.path.abspath(__file__))
    json.dump(out, open(os.path.join(here, "reference_cases.json"), "w"), indent=1, sort_keys=True)
    n = sum(len(v["tests"]) for v in out.values())
    ok = sum(1 for v in out.values() for t in v["tests"] if t["verdict"] == "ok")
    err = sum(1 for v in out.values() for t in v["tests"] if t["verdict"] == "err")
    print("%d tests: %d is_ok, %d is_err, %d without a verify verdict" % (n, ok, err, n - ok - err))


if __name__ == "__main__":
    main()
