"""Process-level behaviour of the device context:

* the on-disk generator cache (bpg_gens_cache_dir): the first process
  derives and writes it, the next one loads it and proves the same bytes; a
  corrupted or group-writable file is not used, and the verifier re-derives
  the set rather than trusting the file;
* two circuit sizes proved concurrently from two host threads on a fresh
  context (the larger circuit grows the generator set while the smaller
  circuit's proofs hold their snapshot) give the same bytes as sequential
  proving;
* thread exit and process exit (round 4's SIGSEGV, DESIGN.md "Thread exit"):
  a worker exits right after joining its proving threads, and one exits with
  device workspaces still owned by its main thread and by a live thread, on
  the low-HBM path (no comb tables) -- both with this process still holding
  what earlier tests left cached (no trim first); a thread's exit parks its
  workspace, the next thread takes it over.
"""
import threading
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "robust_worker.py")


@pytest.fixture(scope="module")
def bpg():
    import workloads
    return workloads._bpg()


def run(*args, env=None):
    r = subprocess.run([sys.executable, WORKER] + list(args), capture_output=True, text=True, timeout=200, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "bpg: fatal signal" not in r.stderr, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_generator_disk_cache(tmp_path):
    a = run("cache", str(tmp_path))
    assert not a["gens_from_cache"]
    files = list(tmp_path.glob("bpg_gens_*.bin"))
    assert len(files) == 1
    b = run("cache", str(tmp_path))
    assert b["gens_from_cache"] and b["proof"] == a["proof"]
    # the verifier re-derived instead of trusting the file
    assert a["verified"] and b["verified"] and not b["from_cache_after_verify"]
    os.chmod(files[0], 0o664)                        # group-writable: never loaded
    d = run("cache", str(tmp_path))
    assert not d["gens_from_cache"] and d["proof"] == a["proof"]
    os.chmod(files[0], 0o644)
    raw = bytearray(files[0].read_bytes())
    raw[100000] ^= 1
    files[0].write_bytes(bytes(raw))
    c = run("cache", str(tmp_path))                 # checksum mismatch: derived again
    assert not c["gens_from_cache"] and c["proof"] == a["proof"]


def test_concurrent_circuit_sizes(bpg):
    import workloads as W
    conc = run("concurrent")
    ctx = bpg.Context(0)
    for k, stmt, reps in (("small", W.config2(), 6), ("large", W.config3(), 2)):
        bpg.set_seed(9)
        syn = bpg.Synth(*stmt)
        want = [ctx.r1cs_prove(b"conc", syn.view, bytes([r]) * 32)[0].hex() for r in range(reps)]
        assert conc[k] == want, k


def test_exit_with_live_workspaces():
    out = run("exit")
    assert all(len(out[k]) > 800 for k in ("main", "done", "live"))


def test_thread_exit_parks_workspace(bpg):
    """A proving thread's exit hands its device workspace to the next thread
    (no HIP call in thread exit); bpg_ctx_trim frees the parked ones."""
    import time
    import workloads as W
    ctx = bpg.Context(0)
    syn = bpg.Synth(*W.config2())

    def prove_on_new_thread():
        res = []
        t = threading.Thread(target=lambda: res.append(ctx.r1cs_prove(b"park", syn.view, bytes(32))[0]))
        t.start()
        t.join()
        return res[0]

    s0 = ctx.setup_stats()
    a = prove_on_new_thread()
    deadline = time.time() + 10   # the OS thread finishes its exit after join()
    while ctx.setup_stats()["workspace_parks"] == s0["workspace_parks"] and time.time() < deadline:
        time.sleep(0.01)
    s1 = ctx.setup_stats()
    assert s1["workspace_parks"] == s0["workspace_parks"] + 1 and s1["workspaces_parked"] >= 1
    b = prove_on_new_thread()     # takes the parked workspace over
    assert a == b
    assert ctx.trim() >= 0
    assert ctx.setup_stats()["workspaces_parked"] == 0


def test_batch_sizes_consumers_to_hw_queues():
    """Without GPU_MAX_HW_QUEUES (HIP's default 4 queues) a 14-thread batch
    runs at most 4 consumer streams and proves the same bytes as single
    proofs (the layout must not depend on bench.py's env)."""
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = run("queues", env=env)
    st = out["stats"]
    assert st["hw_queues"] == 4 and 1 <= st["consumers"] <= 4, st
    assert out["same"] and out["distinct"] == 40


def test_statements_layout_next_to_foreign_allocation(bpg):
    """bpg_set_statements_layout(12, 4) with 16 hardware queues
    next to a foreign 200 GB allocation (made by the worker process itself)
    completes, with device threads admitted by HBM -- never an aborted HSA
    queue. The proving kernels need no scratch memory (tests/test_host.py
    checks the code object), so no dispatch allocates device memory behind
    the admission's back. This process first hands back its cached tables
    and workspaces (bpg_ctx_trim): the pressure under test is the worker's
    200 GB, not what earlier tests left here."""
    bpg.Context(0).trim()
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    out = run("stmts_hbm", "200", env=env)
    st = out["stats"]
    assert out["foreign_gb"] >= 150, json.dumps(out)[:2000]
    assert out["error"] is None, json.dumps(out)[:2000]
    assert out["proved"] == out["count"] and out["verified_last"], json.dumps(out)[:2000]
    assert 1 <= st["consumers"] <= 12, st
    # the admission's estimate holds: no device thread had to retire on an
    # out-of-memory error
    assert st["oom_retired"] == 0, st
    # and no device thread's workspace outgrew the estimate it was admitted by
    assert 0 < st["ws_gb_max"] <= st["est_gb_per_device_thread"], st


def test_statements_device_thread_retires_on_oom():
    """a device thread whose proof fails with hipErrorOutOfMemory
    half way through (injected at IPP round 3 by BPG_TEST_INJECT_OOM) retires
    and hands its statements back; the other device threads prove them, and
    the bytes equal sequential proving (a half-finished lockstep step leaves
    the prepared statements and their TranscriptRng draws untouched)."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16", BPG_TEST_INJECT_OOM="3")
    out = run("stmts_oom", env=env)
    st = out["stats"]
    assert out["error"] is None, json.dumps(out)[:2000]
    assert st["oom_retired"] == 1 and st["consumers"] == 3, st
    assert out["proved"] == out["count"] and all(out["same"]) and len(out["same"]) == out["count"], out
