#!/usr/bin/env python3
"""R1CS prove throughput on MI355X (BASELINE.json metric).

A *step* is one pass of the hot path (`Prover::prove`, prove.rs:79) over one
batch of `--batch` independent proofs of the config-5 statement (2^20
generators: 256-leaf MiMC Merkle tree + 16-element set membership + 64-bit
bounds check), each proof with its own TranscriptRng entropy. The flattened
circuit (a_L/a_R/a_O, transposed constraints) and the generators are resident
in HBM before timing; inside the timed region every proof runs the full
protocol: serial TranscriptRng draws and Merlin transcript on the host,
commitment MSMs, flattened_constraints, t(x), and all lg N IPP rounds on the
device.

value = (proofs completed on all ranks) x q / max-over-ranks wall time, with
q = prover.num_constraints() (the count prove.rs:75 prints).

Multi-GPU: one process per GPU (torchrun), every rank proves its own batch
(independent proofs shard with no data-path collective) ->
"scaling": "weak". The barrier and the max-over-ranks timing use
torch.distributed (RCCL on ROCm).
"""
import argparse
import ctypes
import json
import os
import sys
import time

# HIP hardware queues per process (HIP's default is 4): each host consumer
# thread drives its own stream; with fewer queues than streams they serialise
# behind each other's kernels, with more than 16 the chip does worse again
# (profiles/r01h_sweep.txt, r01t_sweep.txt). The GPU boxes export the default
# (GPU_MAX_HW_QUEUES=4), so the bench raises it unless it was set to something
# else; the runtime reads it when HIP initialises, after this line.
HW_QUEUES = "16"
if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":
    os.environ["GPU_MAX_HW_QUEUES"] = HW_QUEUES

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of this run. Without a torchrun environment and N > 1 the bench starts "
                         "N rank processes itself (one per GPU, RCCL); under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="proofs per step (default: 24 x threads)")
    ap.add_argument("--threads", type=int, default=0,
                    help="host threads per GPU: the TranscriptRng producers plus the device consumers (one HIP "
                         "stream each, four proofs at a time, admitted by HBM: at most 24 proofs in flight at 2^20). "
                         "Default: producers + 8 (verify mode 24)")
    ap.add_argument("--producers", type=int, default=0,
                    help="TranscriptRng producer threads per GPU (default: one per CPU of the rank's share, at most 8)")
    ap.add_argument("--ipp-tail", type=int, default=-1,
                    help="IPP tail threshold in lanes (bpg_ctx_set_ipp_tail; -1: the default, 512)")
    ap.add_argument("--consumers", type=int, default=0,
                    help="statements mode: device threads (bpg_set_statements_layout; 0: min(5, threads / 2))")
    ap.add_argument("--stmt-lockstep", type=int, default=0,
                    help="statements mode: statements a device thread proves at once (1-4; 0: 4)")
    ap.add_argument("--max-inflight", type=int, default=0,
                    help="proofs in flight per GPU (bpg_ctx_set_pipeline max_inflight; 0: 24 at 2^20, and what HBM "
                         "admits)")
    ap.add_argument("--cpus", type=int, default=0,
                    help="pin this rank to its first N CPUs (emulates the per-rank CPU share of a multi-GPU node)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fold-tables", type=int, default=-1, choices=(-1, 0, 1),
                    help="IPP comb tables: 1 on, 0 off (the path a device without ~208 GB free takes), -1 default")
    ap.add_argument("--msm-tables", type=int, default=-1, choices=(-1, 0, 1),
                    help="fixed-base generator tables for the MSMs over the generators (13 windows of 20 bits, "
                         "~7 GB at 2^20): 1 on, 0 or -1 (the default) off")
    ap.add_argument("--isolated-proofs", type=int, default=64,
                    help="proofs of the isolated leg after the timed region (one consumer stream: the kernels' own "
                         "chip time, the roofline's basis); 0 skips it")
    ap.add_argument("--mode", choices=("prove", "verify", "verify-sharded", "latency", "statements", "isolated"),
                    default="prove",
                    help="verify: Verifier::verify throughput over a batch of proofs made before timing "
                         "(config 5's batch verification); latency: one proof at a time, sharded over all "
                         "ranks (bpg_prove_prepared); verify-sharded: one verification at a time, its mega-MSM "
                         "split over all ranks; statements: distinct statements end to end through c_prove "
                         "(parse + synthesis + upload + prove, prove.rs:37-82); isolated: only the isolated leg "
                         "(one consumer stream), for a rocprofv3 trace of the kernels' own chip time. Secondary "
                         "lines, not the headline metric")
    ap.add_argument("--cpu-leaves", type=int, default=16, help="leaves of the config-5-family CPU sample")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes of the all-core CPU leg (default: the CPUs this job may use: the cgroup CPU "
                         "quota, else the affinity mask)")
    return ap.parse_args()


# single kernels bracketed live (bpg name -> rocprofv3 kernel name); every
# label brackets exactly one kernel instantiation, so a label's launch count,
# average and bytes are that rocprof kernel's
KERNELS = {"msm_pass1_gens": "k_rbk_pass<true, 1, 2>", "msm_pass1_folded": "k_rbk_pass<true, 1, 0>",
           "msm_pass1_cached": "k_rbk_pass<true, 0, 0>", "msm_pass1_negc": "k_rbk_pass<true, 1, 1>",
           "ipp_fold_points": "k_ipp_fold_points<gec>", "ipp_fold_points_niels": "k_ipp_fold_points<gen>",
           "ipp_fold2_niels": "k_ipp_fold2<gen, 3>",
           "ipp_comb_fold": "k_ipp_comb_fold", "ipp_fold2": "k_ipp_fold2<gec, 3>", "ipp_fold3": "k_ipp_fold3<gen>",
           "ipp_fold3_cached": "k_ipp_fold3<gec>",
           "flatten": "k_flatten_short"}
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E (MI355X_MICROARCH.md)
FEMUL_PEAK_G = 261.5         # GF(2^255-19) multiplies/s x1e9, measured: profiles/r02d_valu_micro.log (fe_variants V2)


def pmc_row(kernel):
    """The committed rocprofv3 PMC row of `kernel` (profiles/*_pmc.json, the
    latest; scripts/pmc_table.py: FETCH_SIZE x 2 per the gfx950 correction +
    WRITE_SIZE, and the SQ issue counters, separate passes), or {}."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    if not files:
        return {}
    d = json.load(open(files[-1]))
    row = dict(d.get("kernels", {}).get(kernel) or {})
    if row:
        row["source"] = os.path.relpath(files[-1], ROOT)
    return row


def prof_row(kernel, kind="profdefault"):
    """The average duration (us) and launch count of `kernel` in the latest
    committed rocprofv3 --kernel-trace --stats table of the bench's default
    command (profiles/*_profdefault_kernels.md) or of `bench.py --mode
    isolated` (kind "isolated": profiles/*_isolated_kernels.md;
    scripts/prof_summary.py), or {}."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_%s_kernels.md" % kind)))
    if not files:
        return {}
    for line in open(files[-1]):
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) >= 4 and cells[0].replace("void ", "") == kernel:
            return {"avg_us": float(cells[3]), "calls": int(cells[1]), "source": os.path.relpath(files[-1], ROOT)}
    return {}


def _cpu_sample(leaves):
    """(constraints, seconds) of one warm single-thread oracle proof of the
    config-5 family with `leaves` Merkle leaves (also run as a child process
    by the all-core leg: `python bench.py --cpu-sample-child <leaves>`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import workloads as W
    bpg = W._bpg()
    inst, wit, gad = W.merkle_set_bound(1005, leaves)
    bpg.set_seed(1)
    syn = bpg.Synth(inst, wit, gad)
    L = O.lib()
    out = ctypes.create_string_buffer(417 + 64 * 31)
    plen = ctypes.c_size_t(0)
    V = ctypes.create_string_buffer(32 * max(syn.m, 1))
    view = ctypes.cast(ctypes.addressof(syn.view), ctypes.POINTER(O.R1csView))
    # cold call derives + caches generators; the timed call is warm
    L.oracle_r1cs_prove(b"bench", 5, view, b"\1" * 32, out, len(out), ctypes.byref(plen), V)
    t0 = time.perf_counter()
    L.oracle_r1cs_prove(b"bench", 5, view, b"\2" * 32, out, len(out), ctypes.byref(plen), V)
    return syn.q, time.perf_counter() - t0, syn.n


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs this job may use: the cgroup CPU quota (cgroup v2 cpu.max, v1
    cfs_quota_us / cfs_period_us) when one is set, else None. On the GPU
    boxes the affinity mask lists the whole machine while the job's cgroup is
    granted a share of it."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return float(q) / float(per)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0 and per > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def job_cpus():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cpu_quota()
    return max(1, min(aff, int(quota))) if quota else aff


FULL_CPU = os.path.join("profiles", "r02d_cpu_baseline_full.json")


def cpu_baseline(leaves, procs):
    """The CPU oracle (oracle/: a plain-C restatement of dalek/bulletproofs
    with dalek's algorithms on 5x51-bit limbs — not dalek's AVX2 backend,
    Cargo.toml:21; the reference prover is single-threaded, prove.rs:79)
    proving a bounded sample of the same workload family: the config-5
    statement with `leaves` Merkle leaves. Two legs: one core,
    and `procs` independent single-thread provers at once, `procs` = the CPUs
    this job may use (the host's all-core throughput on independent proofs;
    more processes than the job's CPU quota would only time-slice). The full
    config-5 size (N = 2^20) on one core takes ~150 s, so it is measured by
    scripts/cpu_baseline_full.py and reported here from its record."""
    import subprocess
    q, dt, n = _cpu_sample(leaves)
    N = 1
    while N < n:
        N *= 2
    t0 = time.perf_counter()
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-sample-child", str(leaves)],
                           stdout=subprocess.PIPE, text=True) for _ in range(procs)]
    res = [json.loads(p.communicate()[0]) for p in ps]
    wall = time.perf_counter() - t0
    allcore = sum(r["q"] / r["s"] for r in res)
    quota = cpu_quota()
    aff = len(os.sched_getaffinity(0))
    out = {"value": round(q / dt, 1), "unit": "constraints/s", "cores": 1, "kind": "port",
           "sample": "oracle/ plain-C restatement (dalek's algorithms, 5x51-bit limbs, not dalek's AVX2 backend; "
                     "1 thread like the reference prover) proving the config-5 family with %d Merkle leaves: n=%d, "
                     "N=2^%d, q=%d, warm generators, %.1f s" % (leaves, n, N.bit_length() - 1, q, dt),
           "all_cores": {"value": round(allcore, 1), "cores": procs, "wall_s": round(wall, 1),
                         "per_core": round(allcore / procs, 1),
                         "sample": "%d independent single-thread oracle provers of the same sample at once" % procs,
                         "cap": ("the job's cgroup CPU quota (%.1f CPUs) of the %d CPUs in the affinity mask: more "
                                 "provers than that only time-slice" % (quota, aff)) if quota and procs < aff else
                                "all CPUs in the affinity mask",
                         "whole_host_extrapolated": round(allcore / procs * (os.cpu_count() or procs), 1)},
           "host": {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota, "model": _cpu_model()}}
    try:
        full = json.load(open(os.path.join(ROOT, FULL_CPU)))
        out["full_size_single_core"] = {"value": full["constraints_per_s_warm"], "cold_value":
                                        full["constraints_per_s_cold"], "n": full["n"], "q": full["q"],
                                        "N": "2^20", "warm_s": full["warm_s"], "model": full["cpu_model"],
                                        "source": FULL_CPU + " (scripts/cpu_baseline_full.py on a GPU box)"}
    except (OSError, ValueError, KeyError):
        pass
    return out


def heartbeat(period=20.0):
    """A progress line on stderr every `period` seconds: the long timed
    region is one library call and prints nothing else."""
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(period)
            print("bench: running, %.0f s" % (time.perf_counter() - t0), file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


class GpuTelemetry:
    """GFX clock, socket power, hotspot temperature and GFX activity of this
    rank's GPU sampled by amdsmi every `period` s between start() and stop()
    (the timed region), so that a record carries the clock it ran at and
    round-over-round numbers from different boxes can be told apart from a
    box effect. Everything is optional: without amdsmi, or a metric the
    device does not report, the line says so instead of failing."""

    def __init__(self, torch, dev, period=0.25):
        import threading
        self.samples, self.err, self.h, self.period = [], None, None, period
        self.stop_ev = threading.Event()
        self.thread = None
        try:
            import amdsmi
            self.smi = amdsmi
            amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
            handles = amdsmi.amdsmi_get_processor_handles()
            bus = getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", None)
            for h in handles:   # the handle on this rank's PCI bus ("dddd:bb:dd.f")
                try:
                    if bus is not None and int(amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")[1], 16) == bus:
                        self.h = h
                        break
                except Exception:
                    pass
            if self.h is None and len(handles) == 1:
                self.h = handles[0]
            if self.h is None:
                self.err = "no amdsmi handle on PCI bus %r (%d handles)" % (bus, len(handles))
        except Exception as e:   # amdsmi absent or not permitted on this box
            self.err = "amdsmi: %s" % e

    @staticmethod
    def _num(v):
        return float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else None

    def sample(self):
        m = self.smi.amdsmi_get_gpu_metrics_info(self.h)
        clks = [self._num(c) for c in (m.get("current_gfxclks") or []) if self._num(c)]
        clk = (sum(clks) / len(clks)) if clks else (self._num(m.get("current_gfxclk")) or
                                                    self._num(m.get("average_gfxclk_frequency")))
        pw = self._num(m.get("current_socket_power")) or self._num(m.get("average_socket_power"))
        return {"t": time.perf_counter(), "sclk_mhz": clk, "power_w": pw,
                "temp_hotspot_c": self._num(m.get("temperature_hotspot")),
                "gfx_activity_pct": self._num(m.get("average_gfx_activity"))}

    def start(self):
        import threading
        if self.h is None:
            return

        def run():
            while not self.stop_ev.is_set():
                try:
                    self.samples.append(self.sample())
                except Exception as e:
                    self.err = "amdsmi sample: %s" % e
                    return
                self.stop_ev.wait(self.period)
        self.thread = threading.Thread(target=run, daemon=True)
        self.thread.start()

    def stop(self):
        self.stop_ev.set()
        if self.thread is not None:
            self.thread.join(timeout=5)
        out = {"samples": len(self.samples), "period_s": self.period, "source": "amdsmi gpu_metrics"}
        if self.err:
            out["error"] = self.err
        for k in ("sclk_mhz", "power_w", "temp_hotspot_c", "gfx_activity_pct"):
            vs = [s[k] for s in self.samples if s[k] is not None]
            if vs:
                out[k] = {"mean": round(sum(vs) / len(vs), 1), "min": round(min(vs), 1), "max": round(max(vs), 1)}
        return out


DIST_INFO = None


def dist_info(torch, dist, D, dev, world):
    """What the ranks saw: the process group's world size and backend, and
    every rank's HIP device index and PCI bus (gathered over the group)."""
    try:
        p = torch.cuda.get_device_properties(dev)
        bus = "%s" % getattr(p, "pci_bus_id", "?")
        name = p.name
    except Exception:
        bus, name = "?", "?"
    mine = ("%d:%s" % (dev, bus)).encode()[:30].ljust(30, b" ")
    ranks = [m.decode().strip() for m in D.all_gather_bytes(mine)] if dist is not None else [mine.decode().strip()]
    return {"world_size": dist.get_world_size() if dist is not None else 1,
            "backend": dist.get_backend() if dist is not None else "none (1 rank)",
            "rank_devices": ranks, "device_name": name,
            "launcher": "bench.py --gpus" if os.environ.get("BENCH_SPAWNED") else
                        ("torchrun" if world > 1 else "single process")}


def spawn_ranks(n):
    """`bench.py --gpus N` without a torchrun environment: start N rank
    processes (RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on 127.0.0.1), one
    per GPU, and exit with their status. This process has not touched HIP
    (nothing here imports torch), so no GPU state is forked or replaced."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in procs:   # a failed rank would leave the others in a collective
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-sample-child":
        q, dt, _ = _cpu_sample(int(sys.argv[2]))
        print(json.dumps({"q": q, "s": dt}))
        return
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(spawn_ranks(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is not None and a.gpus != world:
        sys.exit("bench: --gpus %d but the launcher started %d ranks (WORLD_SIZE)" % (a.gpus, world))
    if os.environ.get("BENCH_RANK_PROBE"):   # tests/test_host.py: the launcher's view of a rank, no GPU touched
        print(json.dumps({"rank": rank, "world": world, "local": local, "master": os.environ.get("MASTER_ADDR"),
                          "spawned": os.environ.get("BENCH_SPAWNED") == "1"}), flush=True)
        return
    if a.cpus:   # before anything starts a thread: the pool inherits the mask
        cpus = sorted(os.sched_getaffinity(0))[:a.cpus]
        os.sched_setaffinity(0, cpus)
    if rank == 0:
        heartbeat()
    import torch
    dist = None
    ndev = torch.cuda.device_count()
    dev = local % max(ndev, 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        # RCCL between GPUs; BENCH_DIST_BACKEND=gloo lets several ranks share
        # one GPU (RCCL refuses two ranks on one device)
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    import workloads as W
    bpg = W._bpg()
    sys.path.insert(0, os.path.join(ROOT, "bulletproof-gadgets_amd"))
    import dist as D
    bpg.lib().bpg_set_device(dev)
    global DIST_INFO
    DIST_INFO = dist_info(torch, dist, D, dev, world)
    ncpu = job_cpus()
    # the rank's CPU share: the job's CPUs (cgroup quota, else affinity)
    # divided among the ranks on this node
    per_rank = max(1, ncpu // max(world, 1)) if world > 1 else ncpu
    # producers draw the TranscriptRng streams (one keeps a core busy, ~20
    # proofs/s at 2^20): one per CPU of the rank's share, at most 8. Consumers
    # mostly sleep on the device (event polls); the library admits them by HBM
    # (six streams of four proofs at 2^20 next to the comb tables)
    producers = a.producers or max(1, min(8, per_rank))
    threads = a.threads or producers + 8
    if a.mode == "verify" and not a.threads:
        threads = max(1, min(24, per_rank * 3 // 2))   # one HIP stream per verifying thread
    threads = min(threads, 64)
    # 384 proofs per step at the default layout (24 per host thread at 16
    # threads); the timed steps run as one continuous pipeline (below), so the
    # end-of-batch drain is paid once
    batch = a.batch or 384

    if a.mode == "statements":
        return bench_statements(a, bpg, dist, D, rank, world, W)

    # every rank proves its own statement, except in latency mode, where the
    # ranks share ONE proof of one statement
    srank = 0 if a.mode in ("latency", "verify-sharded") else rank
    inst, wit, gad = W.CONFIGS[a.config]() if a.config != 5 else W.config5(1005 + 7919 * srank)
    bpg.set_seed(1000 + srank)
    syn = bpg.Synth(inst, wit, gad)
    ctx = bpg.Context(dev)
    if a.fold_tables >= 0 or a.msm_tables >= 0 or a.ipp_tail >= 0:
        ctx.set_strategy(fold_tables=a.fold_tables, ipp_tail=a.ipp_tail, msm_tables=a.msm_tables)
    ctx.set_pipeline(producers=min(producers, 8), max_inflight=a.max_inflight)
    if a.mode == "latency":
        return bench_latency(a, bpg, ctx, syn, D, dist, rank, world, W)
    # cold setup, outside the timed region: BulletproofGens::new (prove.rs:78,
    # derived on the device) and the circuit upload (the IPP comb tables are
    # built by the first warm-up batch, ~0.9 s)
    tp = time.perf_counter()
    prep = ctx.prepare(syn.view)
    prepare_ms = (time.perf_counter() - tp) * 1e3
    setup = ctx.setup_stats()
    q, n = syn.q, syn.n
    N = 1
    while N < n:
        N *= 2

    def entropies(step):
        return [((rank << 40) | (step << 20) | k).to_bytes(32, "little") for k in range(batch)]

    if a.mode == "verify":
        return bench_verify(a, bpg, ctx, syn, prep, D, dist, rank, world, threads, entropies, q, n, N, W)
    if a.mode == "verify-sharded":
        return bench_verify_sharded(a, bpg, ctx, syn, prep, D, dist, rank, world, q, n, N, W)
    L = bpg.lib()
    if a.mode == "isolated":
        return bench_isolated(a, prep, L, producers, rank, q, W)
    if a.warmup:
        prep.prove_batch(b"bench", sum((entropies(1000 + s) for s in range(a.warmup)), []), threads)
    L.bpg_profile_enable(0 if os.environ.get("BENCH_LIVE_TIMING") == "0" else 1)
    L.bpg_kernel_stats_reset()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    telem = GpuTelemetry(torch, dev)
    barrier()
    telem.start()
    c0 = os.times()
    t0 = time.perf_counter()
    # the K steps' batches go through the producer/consumer pipeline as one
    # stream of K x batch independent proofs (a serving prover does not
    # drain between batches); every proof is one full Prover::prove
    proofs = prep.prove_batch(b"bench", sum((entropies(s) for s in range(a.steps)), []), threads)
    barrier()
    dt = time.perf_counter() - t0
    c1 = os.times()
    gpu_telemetry = telem.stop()
    pipe = bpg.last_batch_stats()
    host_busy = ((c1.user - c0.user) + (c1.system - c0.system)) / dt   # host cores kept busy by this rank
    if os.environ.get("BENCH_THREAD_CPU"):   # diagnostic: per-thread CPU seconds (utime, stime)
        rows = []
        for tid in os.listdir("/proc/self/task"):
            try:
                st = open("/proc/self/task/%s/stat" % tid).read().rsplit(")", 1)[1].split()
                name = open("/proc/self/task/%s/comm" % tid).read().strip()
                rows.append((int(st[11]) / 100.0, int(st[12]) / 100.0, tid, name))
            except OSError:
                pass
        rows.sort(reverse=True)
        print("thread cpu (utime s, stime s, tid, comm), wall %.1f s:" % dt, file=sys.stderr)
        for r in rows[:48]:
            print("  %.2f %.2f %s %s" % r, file=sys.stderr)
    L.bpg_profile_enable(0)
    free_b, total_b = torch.cuda.mem_get_info(dev)   # HBM in use after the run (tables + workspaces)
    if dist is not None:
        dt = D.max_over_ranks(dt)

    # single-proof latency (one host thread), outside the timed region; the
    # first such proof may land on a pool thread whose device workspace was
    # never used (its one-time allocations then count as commit time), so
    # the second one is reported
    prep.prove_batch(b"bench", [b"\x08" * 32], 1)
    t1 = time.perf_counter()
    prep.prove_batch(b"bench", [b"\x09" * 32], 1)
    single_ms = (time.perf_counter() - t1) * 1e3
    # the consumer thread's device phases of that proof; its TranscriptRng
    # chain was drawn by a producer thread of the same call, attributed here
    # from the call's pipeline counters
    single_phases = dict(bpg.last_timings())
    one = bpg.last_batch_stats()
    single_phases["rng_ms"] = round(one["producer_draw_ms"], 1)
    single_phases["device_total_ms"] = single_phases.pop("total_ms", None)
    single_phases["note"] = ("rng_ms: the producer thread's draw of the proof's TranscriptRng chain; "
                             "device_total_ms: the consumer's part after the draws (commit, vectors, IPP)")
    # a timed proof must verify (device verifier, outside the timed region)
    sample = proofs[-1]
    ok = ctx.r1cs_verify(b"bench", syn.view, _commitments(ctx, syn), sample)
    if not ok:
        raise SystemExit("bench: a timed proof failed to verify")

    # roofline of the dominant kernel: live HIP-event timing of single kernel
    # launches on the stream they run on, inside the timed region (under six
    # streams' concurrency) and in the isolated leg below (one stream: the
    # kernel's own chip time)
    kernels, jobs = kernel_stats(L)
    try:   # outside the timed region; a failure here must not lose the measured line
        iso = isolated_leg(prep, L, producers, a.isolated_proofs, rank)
    except (Exception, SystemExit) as e:
        iso = None
        print("bench: isolated leg failed (%s); roofline on the concurrent basis" % e, file=sys.stderr)
    roof = roofline(kernels, jobs, iso, a.steps, dt / a.steps * 1e3)

    total_proofs = a.steps * batch * world
    value = total_proofs * q / dt
    out = {
        "metric": "R1CS prove constraints/sec (Ristretto MSM) at %d MI355X; bit-exact verify" % world,
        "value": round(value, 1),
        "unit": "constraints/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (255-bit integer field/scalar arithmetic)",
        "data": "synthetic: seeded config-%d statement (random leaves/witnesses, roots via MiMC)" % a.config,
        "config": {"workload": W.NAMES[a.config], "n_gates": n, "N": N, "q_constraints": q,
                   "proofs_per_step_per_gpu": batch, "host_threads_per_gpu": threads,
                   "parallelism": "independent proofs per GPU (%d ranks)" % world,
                   "pipeline": "the K steps' proofs stream through one producer/consumer pipeline",
                   "ipp_comb_tables": {-1: "default (on)", 0: "off", 1: "on"}[a.fold_tables],
                   "msm_fixed_base_tables": {-1: "default (off)", 0: "off", 1: "on"}[a.msm_tables],
                   "ipp_tail_lanes": a.ipp_tail if a.ipp_tail >= 0 else "default (512)"},
        "host_cores_busy": round(host_busy, 2),
        # the producer/consumer pipeline of the timed batch (bpg_last_batch_stats):
        # consumer time starved of ready proofs while producers were drawing
        # (after the pipeline fill) and host_bound when that exceeds a tenth
        "pipeline": pipeline_line(pipe, ncpu, per_rank, a.cpus, a.steps * batch),
        "hbm_used_gb": round((total_b - free_b) / 1e9, 1),
        "latency_ms_single_proof": round(single_ms, 1),
        "cold_setup_ms": round(prepare_ms, 1),
        "msm_table_gb": round(ctx.setup_stats()["msm_table_bytes"] / 1e9, 2),
        "cold_setup_breakdown_ms": {"generators": round(setup["gens_ms"], 1), "comb_tables": round(setup["comb_ms"], 1),
                                    "comb_tables_alloc": round(setup["comb_alloc_ms"], 1),
                                    "generators_from_disk_cache": setup["gens_from_cache"]},
        "device_phase_ms_single_proof": single_phases,
        "roofline": roof,
        # this rank's GPU over the timed region (amdsmi): the clock and power
        # a record ran at, so that box effects are visible
        "gpu_telemetry": gpu_telemetry,
        "dist": DIST_INFO,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_leaves, a.cpu_procs or job_cpus())
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def kernel_stats(L):
    """Every bracketed kernel label's (launches, summed ms, algorithmic bytes,
    fe_mul count) since the last bpg_kernel_stats_reset, and the two MSM job
    labels'."""
    L.bpg_kernel_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.bpg_kernel_femul.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]

    def stat(name):
        lc, ms, by, fm = ctypes.c_uint64(0), ctypes.c_double(0), ctypes.c_double(0), ctypes.c_double(0)
        if L.bpg_kernel_stats(name.encode(), ctypes.byref(lc), ctypes.byref(ms), ctypes.byref(by)) != 0:
            return None
        L.bpg_kernel_femul(name.encode(), ctypes.byref(fm))
        return (lc.value, ms.value, by.value, fm.value) if lc.value else None
    kernels = {k: stat(k) for k in KERNELS}
    jobs = {k: stat(k) for k in ("msm_commit", "msm_ipp")}
    return {k: v for k, v in kernels.items() if v}, {k: v for k, v in jobs.items() if v}


def isolated_leg(prep, L, producers, nproofs, rank):
    """The kernels' own chip time: `nproofs` more proofs of the same batch
    layout (four per lockstep step, so the same job mix per launch) through
    ONE consumer thread, i.e. one HIP stream, so each bracketed launch has the
    chip to itself (the producers only draw on the host and copy). Outside
    the timed region; the timed region's brackets also count the time a
    dispatch waits for CUs held by the other five streams' kernels."""
    if nproofs <= 0:
        return None
    ents = [((rank << 40) | (1 << 39) | k).to_bytes(32, "little") for k in range(nproofs)]
    # the library runs min(producers, groups of 8 proofs) producers: pool
    # threads 0..P-1 draw, thread P proves. With 8 groups or more, P is the
    # timed region's producer count and thread P its first consumer, whose
    # four-proof workspace exists already (a thread that was a producer
    # would allocate ~13 GB next to a full HBM)
    P = max(1, min(producers, 8, (nproofs + 7) // 8))
    L.bpg_kernel_stats_reset()
    L.bpg_profile_enable(1)
    t0 = time.perf_counter()
    prep.prove_batch(b"bench", ents, P + 1)
    wall = time.perf_counter() - t0
    L.bpg_profile_enable(0)
    import workloads as W
    pipe = W._bpg().last_batch_stats()
    if pipe["consumers"] != 1:
        raise SystemExit("bench: the isolated leg ran %d consumer streams" % pipe["consumers"])
    kernels, jobs = kernel_stats(L)
    return {"kernels": kernels, "jobs": jobs, "proofs": nproofs, "wall_s": wall,
            "consumers": pipe["consumers"], "lockstep": pipe["lockstep"]}


def roofline(kernels, jobs, iso, steps, ms_per_step):
    """The bench line's `roofline` object for the dominant kernel label (the
    most bracketed device time in the timed region). `frac` is on the
    kernel's own chip time (the isolated leg's average launch); the timed
    region's concurrency-stretched average is `frac_concurrent`, and
    `consistency` checks that launches per step x the average used fits in
    a step."""
    if not kernels:
        return None
    dom = max(kernels, key=lambda k: kernels[k][1])
    lc, ms, by, fm = kernels[dom]
    sec_c = ms / lc / 1e3                        # average launch under the bench's concurrency
    alg = by / lc                                # algorithmic bytes per launch (SURVEY §8d units)
    ik = (iso or {}).get("kernels", {}).get(dom)
    if ik:
        sec, alg_i, fm_i = ik[1] / ik[0] / 1e3, ik[2] / ik[0], ik[3] / ik[0]
        basis = ("exclusive: the isolated leg's live HIP-event average (%d launches on one stream, %d proofs, "
                 "%d proofs per step), the kernel alone on the chip" % (ik[0], iso["proofs"], iso["lockstep"]))
    else:
        sec, alg_i, fm_i = sec_c, alg, fm / lc
        basis = "concurrent: no isolated leg (--isolated-proofs 0)"
    achieved = alg_i / sec / 1e9
    pmc = pmc_row(KERNELS[dom])
    prof = prof_row(KERNELS[dom])
    iprof = prof_row(KERNELS[dom], "isolated")
    pmc_alg = pmc.get("alg_bytes_per_launch")
    per_step = lc / max(steps, 1)
    return {"kernel": dom, "rocprof_name": KERNELS[dom], "bound": "hbm",
            # the HBM fraction is the metric's; the kernel is limited by its
            # GF(p) multiply rate and gather latency, see "valu"
            "limiter": "valu+gather-latency", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
            "basis": basis, "avg_launch_ms": round(sec * 1e3, 4), "alg_bytes_per_launch": round(alg_i, 1),
            # the same kernel's launches in the timed region, each bracket
            # stretched by the other streams' kernels holding CUs
            "frac_concurrent": round(alg / sec_c / 1e9 / HBM_PEAK_GBS, 6),
            "avg_launch_ms_concurrent": round(sec_c * 1e3, 4), "launches": lc,
            "alg_bytes_per_launch_timed": round(alg, 1),
            "consistency": {"launches_per_step": round(per_step, 1), "ms_per_step": round(ms_per_step, 2),
                            "launches_x_avg_ms": round(per_step * sec * 1e3, 1),
                            "launches_x_avg_concurrent_ms": round(per_step * sec_c * 1e3, 1),
                            "ok": per_step * sec * 1e3 <= ms_per_step,
                            "share_of_step": round(per_step * sec * 1e3 / ms_per_step, 4)},
            "traffic": pmc.get("hbm_bytes_per_launch"),
            "traffic_source": {"pmc_alg_bytes_per_launch": pmc_alg,
                               "traffic_over_alg": round(pmc["hbm_bytes_per_launch"] / pmc_alg, 2)
                               if pmc_alg and pmc.get("hbm_bytes_per_launch") else None,
                               "pmc_avg_us": pmc.get("avg_us"),
                               "pmc_source": pmc.get("source")} if pmc else None,
            # the kernels are VALU-bound (255-bit field arithmetic): the same
            # launches against the measured GF(p) multiply peak
            "valu": {"unit": "G fe_mul/s", "achieved": round(fm_i / sec / 1e9, 2), "peak": FEMUL_PEAK_G,
                     "frac": round(fm_i / sec / 1e9 / FEMUL_PEAK_G, 4),
                     "frac_concurrent": round(fm / lc / sec_c / 1e9 / FEMUL_PEAK_G, 4)},
            # the same kernel in the committed PMC passes (which serialise
            # dispatches): SQ_ACTIVE_INST_VALU share of the SIMDs' cycles, HBM GB/s
            "pmc_isolated": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in pmc.items()
                             if k in ("avg_us", "valu_issue_share", "avg_waves_per_simd", "wave_wait_mem",
                                      "hbm_gbs", "clock_ghz", "source")} or None,
            # the committed rocprofv3 kernel traces of `bench.py --mode
            # isolated` (must agree with avg_launch_ms) and of the default
            # command (must agree with avg_launch_ms_concurrent)
            "rocprof_isolated_cmd": iprof or None,
            "rocprof_default_cmd": prof or None,
            "device_ms_by_kernel": {k: round(v[1], 2) for k, v in kernels.items()},
            # every bracketed kernel: launches, average launch (timed region and
            # isolated leg) and algorithmic bytes per launch
            "kernel_table": {k: {"rocprof_name": KERNELS[k], "launches": v[0],
                                 "avg_launch_ms": round(v[1] / v[0], 4),
                                 "avg_launch_ms_isolated": round(iso["kernels"][k][1] / iso["kernels"][k][0], 4)
                                 if iso and k in iso["kernels"] else None,
                                 "alg_bytes_per_launch": round(v[2] / v[0], 1)}
                             for k, v in kernels.items()},
            "device_ms_by_msm_job": {k: round(v[1], 2) for k, v in jobs.items()},
            "isolated_leg": {"proofs": iso["proofs"], "wall_s": round(iso["wall_s"], 2),
                             "consumers": iso["consumers"], "proofs_per_step": iso["lockstep"]} if iso else None}


def bench_isolated(a, prep, L, producers, rank, q, W):
    """`--mode isolated`: only the isolated leg (warm-up included: one
    consumer stream), for a rocprofv3 kernel trace whose per-kernel averages
    are the line's exclusive launch times (profiles/*_isolated_kernels.md)."""
    if a.warmup:   # the same layout once (comb tables, the consumer's workspace)
        isolated_leg(prep, L, producers, a.isolated_proofs, rank)
    iso = isolated_leg(prep, L, producers, a.isolated_proofs, rank)
    out = {"metric": "isolated leg: kernel launches on one stream (no concurrency)", "proofs": iso["proofs"],
           "wall_s": round(iso["wall_s"], 2), "constraints_per_s": round(iso["proofs"] * q / iso["wall_s"], 1),
           "kernel_table": {k: {"rocprof_name": KERNELS[k], "launches": v[0], "avg_launch_ms": round(v[1] / v[0], 4),
                                "alg_bytes_per_launch": round(v[2] / v[0], 1)} for k, v in iso["kernels"].items()},
           "config": {"workload": W.NAMES[a.config]}}
    if rank == 0:
        print(json.dumps(out), flush=True)


def pipeline_line(p, ncpu, per_rank, pinned, nproofs):
    span = max(1e-9, (p["wall_ms"] - p["fill_ms"]) * p["consumers"])
    return {"producers": p["producers"], "consumers": p["consumers"], "proofs_per_consumer_step": p["lockstep"],
            "proofs_in_flight": p["inflight"], "host_bound": p["host_bound"],
            "consumer_starved_frac": round(p["consumer_starved_ms"] / span, 4),
            "consumer_starved_ms": round(p["consumer_starved_ms"], 1), "fill_ms": round(p["fill_ms"], 1),
            "producer_slot_wait_frac": round(p["producer_slot_wait_ms"] / max(1e-9, p["wall_ms"] * p["producers"]), 4),
            "producer_draw_ms": round(p["producer_draw_ms"], 1),
            # proofs one producer draws per second of its busy time, and what
            # all producers could draw against what the device consumed
            "proofs_per_busy_s_per_producer": round(nproofs / (p["producer_draw_ms"] / 1e3), 2)
            if p["producer_draw_ms"] else None,
            "producer_capacity_proofs_per_s": round(p["producers"] * nproofs / (p["producer_draw_ms"] / 1e3), 1)
            if p["producer_draw_ms"] else None,
            "proofs_per_s": round(nproofs / (p["wall_ms"] / 1e3), 2),
            "consumers_by_threads": p["consumers_by_threads"], "consumers_by_hbm": p["consumers_by_hbm"],
            "hw_queues": p["hw_queues"],
            "est_gb_per_consumer": round(p["est_gb_per_consumer"], 2), "ws_gb_max": round(p.get("ws_gb_max", 0), 2),
            "hbm_free_gb_at_start": round(p["hbm_free_gb"], 1),
            "cpus": {"job": ncpu, "rank_share": per_rank, "process": p["process_cpus"], "pinned": pinned or None}}


def bench_verify(a, bpg, ctx, syn, prep, D, dist, rank, world, threads, entropies, q, n, N, W):
    """Verifier::verify (verify.rs:71) throughput: every rank verifies its own
    batch of proofs (made before timing) with `threads` host threads, one HIP
    stream each; a step = one pass over the batch. value = proofs verified
    on all ranks x q / max-over-ranks wall time."""
    import torch
    import time as _t
    batch = a.batch or 8 * threads
    # the proofs are made before timing on 4 threads: a consumer keeps its
    # prover workspace (four proofs' buffers and MSM scratch, ~12 GB) for
    # later batches, and the verifying threads need HBM of their own
    proofs = prep.prove_batch(b"bench", entropies(777), min(threads, 4))[:batch]
    while len(proofs) < batch:
        proofs += proofs[:batch - len(proofs)]
    V = _commitments(ctx, syn)
    prep = ctx.prepare(syn.view, verifier=True)
    for _ in range(a.warmup):
        if not all(prep.verify_batch(b"bench", V, proofs, threads)):
            raise SystemExit("bench: a valid proof was rejected")
    bad = bytearray(proofs[0])
    bad[-40] ^= 1
    if prep.verify_batch(b"bench", V, [bytes(bad)], 1)[0]:
        raise SystemExit("bench: a tampered proof was accepted")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = _t.perf_counter()
    ok = True
    for _ in range(a.steps):
        ok &= all(prep.verify_batch(b"bench", V, proofs, threads))
    barrier()
    dt = _t.perf_counter() - t0
    if not ok:
        raise SystemExit("bench: a valid proof was rejected in the timed region")
    if dist is not None:
        dt = D.max_over_ranks(dt)
    t1 = _t.perf_counter()
    prep.verify_batch(b"bench", V, proofs[:1], 1)
    single_ms = (_t.perf_counter() - t1) * 1e3
    total = a.steps * batch * world
    out = {
        "metric": "R1CS verify constraints/sec (Ristretto MSM) at %d MI355X" % world,
        "value": round(total * q / dt, 1), "unit": "constraints/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32 (255-bit integer field/scalar arithmetic)",
        "data": "synthetic: seeded config-%d statement; proofs made before timing" % a.config,
        "config": {"workload": W.NAMES[a.config], "n_gates": n, "N": N, "q_constraints": q,
                   "proofs_per_step_per_gpu": batch, "host_threads_per_gpu": threads,
                   "parallelism": "independent verifications per GPU (%d ranks)" % world},
        "proofs_per_s": round(total / dt, 2),
        "latency_ms_single_verify": round(single_ms, 2),
        "dist": DIST_INFO,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_verify_sharded(a, bpg, ctx, syn, prep, D, dist, rank, world, q, n, N, W):
    """Verifier::verify (verify.rs:71) one proof at a time with its mega-MSM
    split over all ranks (bpg_r1cs_verify_shard on every rank, one all-gather
    of 32-byte partial sums, dist.sharded_verify) — SURVEY §8e's second
    option for "batch verify across GPUs", next to --mode verify's
    independent proofs per rank. value = verifications x q / max-over-ranks
    seconds; scaling strong (the work per verification is fixed)."""
    import torch
    proof = prep.prove_batch(b"bench", [b"\x07" * 32], 1)[0]
    if dist is not None:   # every rank verifies rank 0's bytes
        proof = D.all_gather_bytes(proof)[0]
    V = _commitments(ctx, syn)
    # every rank prepares the circuit once (bpg_prepare_verifier); per proof:
    # transcript replay, this rank's slice of the mega-MSM, one 33-byte gather
    vprep = ctx.prepare(syn.view, verifier=True)

    def verify(p):   # one rank: the whole mega-MSM, no exchange
        if dist is None:
            return vprep.verify_one(b"bench", V, p)
        return D.sharded_verify_prepared(bpg, vprep, b"bench", V, p)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        if not verify(proof):
            raise SystemExit("bench: a valid proof was rejected")
    bad = bytearray(proof)
    bad[-40] ^= 1
    if verify(bytes(bad)):
        raise SystemExit("bench: a tampered proof was accepted")
    barrier()
    t0 = time.perf_counter()
    ok = all(verify(proof) for _ in range(a.steps))
    barrier()
    dt = time.perf_counter() - t0
    if not ok:
        raise SystemExit("bench: a valid proof was rejected in the timed region")
    if dist is not None:
        dt = D.max_over_ranks(dt)
    out = {
        "metric": "R1CS verify constraints/sec, one verification at a time sharded over %d MI355X" % world,
        "value": round(a.steps * q / dt, 1), "unit": "constraints/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (255-bit integer field/scalar arithmetic)",
        "data": "synthetic: seeded config-%d statement" % a.config,
        "config": {"workload": W.NAMES[a.config], "n_gates": n, "N": N, "q_constraints": q,
                   "parallelism": "one verification's mega-MSM split over %d ranks" % world},
        "latency_ms_verify": round(dt / a.steps * 1e3, 3),
        "dist": DIST_INFO,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_latency(a, bpg, ctx, syn, D, dist, rank, world, W):
    """Single-proof latency of Prover::prove (prove.rs:79) with ONE proof
    split over all ranks (bpg_prepare_shard + bpg_prove_prepared,
    cyclic lane layout, partial sums all-gathered over torch.distributed).
    A step = one proof; value = q / (max-over-ranks seconds per proof).
    The serial TranscriptRng chain (2n Keccak-f on one host core, run by
    every rank) is part of every proof and does not shrink with ranks."""
    import torch
    q, n = syn.q, syn.n
    N = 1
    while N < n:
        N *= 2
    tp = time.perf_counter()
    prep = ctx.prepare_shard(syn.view, rank, world)
    prepare_ms = (time.perf_counter() - tp) * 1e3
    ag = D.all_gather_bytes if world > 1 else None

    def ent(k):
        return (k + 1).to_bytes(32, "little")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for s in range(a.warmup):
        prep.prove_one(b"bench", ent(10000 + s), ag)
    barrier()
    t0 = time.perf_counter()
    proofs = [prep.prove_one(b"bench", ent(s), ag) for s in range(a.steps)]
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        dt = D.max_over_ranks(dt)
    phases = bpg.last_timings()
    if rank == 0 and not ctx.r1cs_verify(b"bench", syn.view, _commitments(ctx, syn), proofs[-1]):
        raise SystemExit("bench: a sharded proof failed to verify")
    out = {
        "metric": "R1CS single-proof latency constraints/sec at %d MI355X (one proof sharded over the ranks)" % world,
        "value": round(a.steps * q / dt, 1), "unit": "constraints/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (255-bit integer field/scalar arithmetic)",
        "data": "synthetic: seeded config-%d statement" % a.config,
        "config": {"workload": W.NAMES[a.config], "n_gates": n, "N": N, "q_constraints": q,
                   "parallelism": "one proof sharded over %d ranks (lanes i = j*%d + rank)" % (world, world)},
        "latency_ms": round(dt / a.steps * 1e3, 1), "phase_ms_last_proof_rank0": phases,
        "prepare_ms": round(prepare_ms, 1),
        "dist": DIST_INFO,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_statements(a, bpg, dist, D, rank, world, W):
    """The reference's prove() (prove.rs:37-82) for DISTINCT statements, end to
    end: every proof parses its own statement text, synthesises the circuit on
    the host, uploads it (flattened view, transposed constraints) and proves
    it, through the reference C-ABI (c_prove), on `threads` host threads at
    once (one HIP stream each; ctypes releases the GIL). The statement texts
    (config-5 family, seeded) are generated before timing. A step = `batch`
    statements; value = statements x q / wall time."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    threads = a.threads or max(2, min(64, job_cpus() // max(world, 1)))   # synthesis is host work: one per CPU
    # 8 statements per thread per step: every statement's latency (~0.5 s:
    # synthesis, upload, the serial TranscriptRng chain, device work) is paid
    # once per call as pipeline fill, so short batches understate the rate
    batch = a.batch or 8 * threads
    texts = [W.config5(50000 + 100003 * rank + i) for i in range(batch * (a.steps + a.warmup))]
    q = bpg.Synth(*texts[0]).q

    def one(t):
        return bpg.prove("bench", t[0], t[1], t[2])

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    if os.environ.get("BENCH_STATEMENTS_API") == "c_prove":   # one c_prove per statement per thread
        pool = ThreadPoolExecutor(threads)
        list(pool.map(one, texts[:batch * a.warmup]))
        barrier()
        t0 = time.perf_counter()
        outs = list(pool.map(one, texts[batch * a.warmup:]))
        barrier()
        dt = time.perf_counter() - t0
        # the worker threads (and their per-thread device workspaces) end
        # here, while the HIP runtime is certainly still up
        pool.shutdown(wait=True)
        api = "c_prove on %d threads" % threads
        stages = None
    else:   # bpg_prove_statements: lockstep RNG over distinct statements, device consumers
        bpg.set_statements_layout(a.consumers, a.stmt_lockstep)
        bpg.prove_statements("bench", texts[:batch * a.warmup], threads)
        barrier()
        t0 = time.perf_counter()
        outs = bpg.prove_statements("bench", texts[batch * a.warmup:], threads)
        barrier()
        dt = time.perf_counter() - t0
        stages = bpg.last_statements_stats()
        if any(o is None for o in outs):
            raise SystemExit("bench: a statement failed: %s" % bpg.last_error())
        api = "bpg_prove_statements, %d CPU workers + %d device threads of up to %d statements" % (
            threads, stages["consumers"] if stages else min(a.consumers or 5, max(1, a.consumers or threads // 2)),
            a.stmt_lockstep or 4)
    if dist is not None:
        dt = D.max_over_ranks(dt)
    last = texts[-1]
    if rank == 0 and not bpg.verify("bench", last[0], outs[-1][0], outs[-1][1], last[2]):
        raise SystemExit("bench: a statement's proof failed to verify")
    # where one statement's time goes, on one otherwise idle thread (outside
    # the timed region): synthesis, prepare (transpose + upload), prove
    t0 = time.perf_counter()
    syn = bpg.Synth(*last)
    t1 = time.perf_counter()
    ctx = bpg.Context(torch.cuda.current_device() if torch.cuda.is_available() else 0)
    prep = ctx.prepare_shard(syn.view, 0, 1)
    t2 = time.perf_counter()
    prep.prove_one(b"bench", b"\x03" * 32)
    t3 = time.perf_counter()
    phases = {"synthesis_ms": round((t1 - t0) * 1e3, 1), "prepare_ms": round((t2 - t1) * 1e3, 1),
              "prove_ms": round((t3 - t2) * 1e3, 1), "prove_phases_ms": bpg.last_timings()}
    n_st = batch * a.steps * world
    out = {
        "metric": "R1CS prove constraints/sec end to end over distinct statements (prove.rs:37-82: parse + "
                  "synthesis + upload + prove) at %d MI355X" % world,
        "value": round(n_st * q / dt, 1), "unit": "constraints/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32 (255-bit integer field/scalar arithmetic)",
        "data": "synthetic: %d distinct seeded config-5 statements per rank" % (batch * a.steps),
        "config": {"workload": W.NAMES[5], "q_constraints": q, "statements_per_step_per_gpu": batch,
                   "host_threads_per_gpu": threads, "api": api},
        "statements_per_s": round(n_st / dt, 2),
        # bpg_last_statements_stats: busy / idle ms per stage summed over
        # threads, and the stage that bounded the call
        "stages": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in stages.items()} if stages else None,
        "single_statement_ms": phases,
        "dist": DIST_INFO,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _commitments(ctx, syn):
    """V_i of the prepared statement, recomputed on the device."""
    return ctx.pedersen(syn.vec("v", syn.m), syn.vec("v_blinding", syn.m))


if __name__ == "__main__":
    main()
