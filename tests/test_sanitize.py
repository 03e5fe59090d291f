"""Host sanitizers: the statement layer, host crypto,
lockstep RNG and the device arithmetic compiled for the host, built with
AddressSanitizer + UndefinedBehaviorSanitizer (g++) and run over the
reference's fixtures, malformed statements and random operands
(tests/sanitize/driver.cpp). GPU code cannot be sanitized on this pool; the
host code around it can."""
import glob
import os
import subprocess

from conftest import ROOT

HOST = os.path.join(ROOT, "bulletproof-gadgets_amd", "csrc", "host")
OUT = os.path.join(ROOT, "tests", "sanitize", "_build", "driver")


def test_host_code_under_asan_ubsan():
    srcs = [os.path.join(ROOT, "tests", "sanitize", "driver.cpp")] + \
           [os.path.join(HOST, f) for f in ("statement.cpp", "hcrypto.cpp", "rng8.cpp")]
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(s) for s in srcs):
        subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-march=x86-64-v3", "-fsanitize=address,undefined",
                               "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-o", OUT] + srcs)
    bases = sorted(p[:-len(".gadgets")] for p in glob.glob(os.path.join(ROOT, "tests", "golden", "resources", "*.gadgets")))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([OUT] + bases, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "sanitize ok: %d fixtures" % len(bases) in r.stdout
