// capi.cpp — the exported C ABI (include/bpg.h).
//   c_prove / c_verify / free_proof: interfaces/ios/src/lib.rs:20-66 over
//   src/prove.rs:37-82 and src/verify.rs:36-73. Errors never cross the ABI:
//   NULL / false plus bpg_last_error().
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <map>
#include <sched.h>
#include <stdio.h>

#include "r1cs_gpu.h"
#include "statement.h"

using namespace bpg;

static thread_local std::string g_err;
static thread_local uint64_t g_last_q = 0;
static thread_local int g_device = 0;

static void set_err(const std::string &s) { g_err = s; }

template <class F>
static auto guarded(F f, decltype(f()) fail) -> decltype(f()) {
    try {
        g_err.clear();
        return f();
    } catch (const dev::HipError &e) {
        set_err(std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr + " (" + e.file + ":" +
                std::to_string(e.line) + ")");
    } catch (const std::exception &e) {
        set_err(e.what());
    } catch (...) {
        set_err("unknown error");
    }
    return fail;
}

static void require_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        throw std::runtime_error("no HIP device available: libbpg computes the proof on the GPU only");
    if (g_device >= n) throw std::runtime_error("device index out of range");
}

static std::string hex32(const uint8_t *p) {
    static const char *d = "0123456789abcdef";
    std::string s;
    for (int i = 0; i < 32; i++) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}

extern "C" {

const char *bpg_last_error(void) { return g_err.c_str(); }
uint64_t bpg_last_num_constraints(void) { return g_last_q; }

void bpg_set_seed(uint64_t seed) {
    EntropySource &e = thread_entropy();
    e.seeded = true;
    e.cs.seed(seed);
}
void bpg_clear_seed(void) { thread_entropy().seeded = false; }
void bpg_gens_cache_dir(const char *dir) { set_gens_cache_dir(dir); }
int bpg_set_device(int device) {
    if (device < 0) return -1;
    g_device = device;
    return 0;
}

// prove.rs:37-82
struct ProofArtifacts *c_prove(const char *name, const char *instance, const char *witness, const char *gadgets) {
    return guarded([&]() -> ProofArtifacts * {
        if (!name || !instance || !witness || !gadgets) throw std::runtime_error("NULL argument");
        require_device();
        Synthesis syn = synthesize_prover(instance, witness, gadgets);
        bpg_r1cs_view v = syn.cs->view(true);
        g_last_q = v.q;
        std::unique_ptr<PreparedCS> P = prepare_cs(&v, g_device);
        std::string coms;
        for (size_t i = 0; i < syn.com_names.size(); i++)
            coms += syn.com_names[i] + " = 0x" + hex32(P->V.data() + 32 * i) + "\n";
        uint8_t entropy[32];
        thread_entropy().fill(entropy, 32);
        std::vector<uint8_t> proof = gpu_prove(*P, (const uint8_t *)name, strlen(name), entropy);
        ProofArtifacts *a = (ProofArtifacts *)malloc(sizeof(ProofArtifacts));
        char *c = (char *)malloc(coms.size() + 1);
        uint8_t *p = (uint8_t *)malloc(proof.size() ? proof.size() : 1);
        if (!a || !c || !p) { free(a); free(c); free(p); throw std::runtime_error("out of memory"); }
        memcpy(c, coms.c_str(), coms.size() + 1);
        memcpy(p, proof.data(), proof.size());
        a->commitments = c;
        a->proof = p;
        a->proof_len = proof.size();
        a->proof_cap = proof.size();
        return a;
    }, (ProofArtifacts *)nullptr);
}

// verify.rs:36-73
bool c_verify(const char *name, const char *instance, const char *gadgets, const char *commitments,
              const uint8_t *proof, size_t proof_len) {
    return guarded([&]() -> bool {
        if (!name || !instance || !gadgets || !commitments || (!proof && proof_len)) throw std::runtime_error("NULL argument");
        require_device();
        Synthesis syn = synthesize_verifier(instance, commitments, gadgets);
        bpg_r1cs_view v = syn.cs->view(false);
        std::unique_ptr<PreparedCS> P = prepare_cs(&v, g_device);
        uint8_t entropy[32];
        thread_entropy().fill(entropy, 32);
        int r = gpu_verify(*P, (const uint8_t *)name, strlen(name), syn.cs->V().data(), proof, proof_len, entropy);
        return r == 1;
    }, false);
}

void free_proof(struct ProofArtifacts *a) {
    if (!a) return;
    free((void *)a->commitments);
    free((void *)a->proof);
    free(a);
}

// Device bytes each pool thread's prover workspace held after its last batch
// (per device): the consumers of the next batch reuse them, so HBM admission
// counts them as available.
static std::mutex g_held_mu;
static std::map<int, std::vector<size_t>> g_held;

// ------------------------------------------------------------ inner ABI
// Batched-prover pipeline layout (bpg_ctx_set_pipeline; 0 = automatic)
struct Pipeline {
    uint32_t producers = 0, lockstep = 0, max_inflight = 0;
};
struct bpg_ctx {
    int device;
    Strategy strat;   // IPP fold strategy of the calls made through this handle
    Pipeline pipe;    // bpg_prove_batch layout of circuits prepared through it
};
bpg_ctx *bpg_ctx_create(int device) {
    return guarded([&]() -> bpg_ctx * {
        g_device = device;
        require_device();
        DeviceContext::get(device);
        return new bpg_ctx{device, Strategy(), Pipeline()};
    }, (bpg_ctx *)nullptr);
}
void bpg_ctx_destroy(bpg_ctx *ctx) { delete ctx; }
int bpg_ctx_set_fold_tables(bpg_ctx *ctx, int mode) {
    if (!ctx || mode < -1 || mode > 1) return -1;
    ctx->strat.fold_tables = mode;
    return 0;
}
int bpg_ctx_set_fold_pairs(bpg_ctx *ctx, int mode) {
    if (!ctx || mode < -1 || mode > 2) return -1;
    ctx->strat.fold_pairs = mode;
    return 0;
}
int bpg_ctx_set_msm_tables(bpg_ctx *ctx, int mode) {
    if (!ctx || mode < -1 || mode > 1) return -1;
    ctx->strat.msm_tables = mode;
    return 0;
}
int bpg_ctx_set_ipp_tail(bpg_ctx *ctx, int lanes) {
    if (!ctx || lanes < -1) return -1;
    ctx->strat.ipp_tail = lanes;
    return 0;
}
int bpg_ctx_set_pipeline(bpg_ctx *ctx, uint32_t producers, uint32_t lockstep, uint32_t max_inflight) {
    if (!ctx || producers > 8 || lockstep > 4) return -1;
    ctx->pipe = Pipeline{producers, lockstep, max_inflight};
    return 0;
}
int bpg_ctx_setup_stats(bpg_ctx *ctx, double *out, int n) {
    if (!ctx) return -1;
    DeviceContext &c = DeviceContext::get(ctx->device);
    std::lock_guard<std::mutex> lk(c.mu);
    double resident = 0, fb = 0;
    for (auto &e : c.combs) resident += (double)e.second->bytes;
    for (auto &e : c.fbs) fb += (double)e.second->bytes;
    const ParkStats ps = park_stats();
    const double v[10] = {c.gens_ms, c.comb_ms, c.gens_from_cache ? 1.0 : 0.0, c.comb_alloc_ms, resident, fb,
                          (double)ps.workspaces_parked, (double)ps.workspace_parks, (double)ps.stages_parked,
                          (double)ps.stage_parks};
    for (int i = 0; i < n && i < 10; i++) out[i] = v[i];
    return 0;
}
int bpg_gens_ensure(bpg_ctx *ctx, uint32_t capacity) {
    return guarded([&]() -> int {
        DeviceContext::get(ctx->device).gens(capacity);
        return 0;
    }, -1);
}

int bpg_pedersen_commit(bpg_ctx *ctx, const uint8_t *v, const uint8_t *vb, uint32_t count, uint8_t *V_out) {
    return guarded([&]() -> int {
        std::vector<Scalar> a(count), b(count);
        for (uint32_t i = 0; i < count; i++) { memcpy(a[i].v, v + 32 * (size_t)i, 32); memcpy(b[i].v, vb + 32 * (size_t)i, 32); }
        gpu_pedersen(ctx->device, a, b, V_out);
        return 0;
    }, -1);
}

int bpg_r1cs_prove(bpg_ctx *ctx, const uint8_t *label, size_t label_len, const bpg_r1cs_view *cs,
                   const uint8_t entropy[32], uint8_t *proof_out, size_t proof_cap, size_t *proof_len, uint8_t *V_out) {
    return guarded([&]() -> int {
        if (!cs->a_L) throw std::runtime_error("prover view without witness");
        std::unique_ptr<PreparedCS> P = prepare_cs(cs, ctx->device, ctx->strat);
        std::vector<uint8_t> proof = gpu_prove(*P, label, label_len, entropy);
        if (proof.size() > proof_cap) throw std::runtime_error("proof buffer too small");
        memcpy(proof_out, proof.data(), proof.size());
        *proof_len = proof.size();
        if (V_out && cs->m) memcpy(V_out, P->V.data(), (size_t)cs->m * 32);
        return 0;
    }, -1);
}

int bpg_r1cs_prove_sharded(bpg_ctx *ctx, const uint8_t *label, size_t label_len, const bpg_r1cs_view *cs,
                           const uint8_t entropy[32], uint32_t rank, uint32_t world, bpg_allgather_fn allgather,
                           void *user, uint8_t *proof_out, size_t proof_cap, size_t *proof_len, uint8_t *V_out) {
    return guarded([&]() -> int {
        if (!cs->a_L) throw std::runtime_error("prover view without witness");
        if (!allgather) throw std::runtime_error("NULL all-gather");
        std::unique_ptr<PreparedCS> P = prepare_cs(cs, ctx->device, ctx->strat, rank, world);
        AllGather ag = [&](const void *send, size_t bytes, void *recv) {
            if (allgather(user, send, bytes, recv) != 0) throw std::runtime_error("all-gather failed");
        };
        std::vector<uint8_t> proof = gpu_prove(*P, label, label_len, entropy, nullptr, &ag);
        if (proof.size() > proof_cap) throw std::runtime_error("proof buffer too small");
        memcpy(proof_out, proof.data(), proof.size());
        *proof_len = proof.size();
        if (V_out && cs->m) memcpy(V_out, P->V.data(), (size_t)cs->m * 32);
        return 0;
    }, -1);
}

int bpg_r1cs_verify(bpg_ctx *ctx, const uint8_t *label, size_t label_len, const bpg_r1cs_view *cs, const uint8_t *V,
                    const uint8_t *proof, size_t proof_len, const uint8_t entropy[32]) {
    return guarded([&]() -> int {
        bpg_r1cs_view v = *cs;
        v.a_L = v.a_R = v.a_O = v.v = v.v_blinding = nullptr;
        std::unique_ptr<PreparedCS> P = prepare_cs(&v, ctx->device);
        return gpu_verify(*P, label, label_len, V, proof, proof_len, entropy);
    }, -1);
}

int bpg_r1cs_verify_shard(bpg_ctx *ctx, const uint8_t *label, size_t label_len, const bpg_r1cs_view *cs,
                          const uint8_t *V, const uint8_t *proof, size_t proof_len, const uint8_t entropy[32],
                          uint32_t shard, uint32_t nshards, uint8_t partial[32]) {
    return guarded([&]() -> int {
        if (nshards < 2) throw std::runtime_error("nshards must be >= 2 (use bpg_r1cs_verify)");
        bpg_r1cs_view v = *cs;
        v.a_L = v.a_R = v.a_O = v.v = v.v_blinding = nullptr;
        std::unique_ptr<PreparedCS> P = prepare_cs(&v, ctx->device);
        return gpu_verify_shard(*P, label, label_len, V, proof, proof_len, entropy, shard, nshards, partial);
    }, -1);
}

// Host-only: sum of compressed Ristretto points (the verifier shards'
// partials); the identity encodes as 32 zero bytes.
int bpg_point_sum(const uint8_t *points, uint32_t count, uint8_t out[32]) {
    return guarded([&]() -> int {
        Point acc, p;
        pt_identity(acc);
        for (uint32_t i = 0; i < count; i++) {
            if (!ristretto_decompress(p, points + 32 * (size_t)i)) return -1;
            Point t; pt_add(t, acc, p); acc = t;
        }
        ristretto_compress(out, acc);
        return 0;
    }, -1);
}

struct bpg_prepared {
    std::unique_ptr<PreparedCS> p;
    Pipeline pipe;
};
bpg_prepared *bpg_prepare(bpg_ctx *ctx, const bpg_r1cs_view *cs) {
    return guarded([&]() -> bpg_prepared * {
        bpg_prepared *b = new bpg_prepared();
        b->p = prepare_cs(cs, ctx->device, ctx->strat);
        b->pipe = ctx->pipe;
        DeviceContext::get(ctx->device).gens(b->p->N);
        return b;
    }, (bpg_prepared *)nullptr);
}
bpg_prepared *bpg_prepare_verifier(bpg_ctx *ctx, const bpg_r1cs_view *cs) {
    bpg_r1cs_view v = *cs;
    v.a_L = v.a_R = v.a_O = v.v = v.v_blinding = nullptr;
    return bpg_prepare(ctx, &v);
}
void bpg_prepared_free(bpg_prepared *p) { delete p; }
int bpg_verify_prepared(bpg_prepared *p, const uint8_t *label, size_t label_len, const uint8_t *V, const uint8_t *proof,
                        size_t proof_len, const uint8_t entropy[32], uint32_t shard, uint32_t nshards,
                        uint8_t *partial) {
    return guarded([&]() -> int {
        if (!p || !label || !entropy || (!proof && proof_len)) throw std::runtime_error("NULL argument");
        const PreparedCS &cs = *p->p;
        if (cs.prover) throw std::runtime_error("circuit prepared for proving: use bpg_prepare_verifier");
        if (!V && cs.m) throw std::runtime_error("NULL commitments");
        if (nshards > 1 && !partial) throw std::runtime_error("NULL partial");
        return gpu_verify_shard(cs, label, label_len, V, proof, proof_len, entropy, shard, nshards, partial);
    }, -1);
}
bpg_prepared *bpg_prepare_shard(bpg_ctx *ctx, const bpg_r1cs_view *cs, uint32_t rank, uint32_t world) {
    return guarded([&]() -> bpg_prepared * {
        if (!cs->a_L) throw std::runtime_error("prover view without witness");
        bpg_prepared *b = new bpg_prepared();
        b->p = prepare_cs(cs, ctx->device, ctx->strat, rank, world);
        return b;
    }, (bpg_prepared *)nullptr);
}
int bpg_prove_prepared(bpg_prepared *p, const uint8_t *label, size_t label_len, const uint8_t entropy[32],
                       bpg_allgather_fn allgather, void *user, uint8_t *proof_out, size_t proof_cap,
                       size_t *proof_len) {
    return guarded([&]() -> int {
        const PreparedCS &cs = *p->p;
        if (!cs.prover) throw std::runtime_error("prepared circuit has no witness");
        if (cs.world > 1 && !allgather) throw std::runtime_error("sharded circuit without an all-gather");
        AllGather ag = [&](const void *send, size_t bytes, void *recv) {
            if (allgather(user, send, bytes, recv) != 0) throw std::runtime_error("all-gather failed");
        };
        std::vector<uint8_t> proof = gpu_prove(cs, label, label_len, entropy, nullptr, cs.world > 1 ? &ag : nullptr);
        if (proof.size() > proof_cap) throw std::runtime_error("proof buffer too small");
        memcpy(proof_out, proof.data(), proof.size());
        *proof_len = proof.size();
        return 0;
    }, -1);
}

// Persistent host worker pool: each worker owns its thread-local device
// workspace (stream + buffers), so repeated batches reuse HBM allocations.
namespace {
struct Pool {
    std::vector<std::thread> workers;
    std::mutex run_mu;   // one batch at a time: concurrent bpg_*_batch callers queue here
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::function<void(int)> job;
    uint64_t gen = 0;
    int active = 0, want = 0;
    bool stop = false;
    void ensure(int n) {
        while ((int)workers.size() < n) {
            int id = (int)workers.size();
            workers.emplace_back([this, id] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(int)> f;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return stop || (gen != seen && id < want); });
                        if (stop) return;
                        seen = gen;
                        f = job;
                    }
                    f(id);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--active == 0) done_cv.notify_all();
                }
            });
        }
    }
    int size() {
        std::lock_guard<std::mutex> serial(run_mu);
        return (int)workers.size();
    }
    void run(int n, std::function<void(int)> f) {
        std::lock_guard<std::mutex> serial(run_mu);
        ensure(n);
        std::unique_lock<std::mutex> lk(mu);
        job = std::move(f);
        want = n;
        active = n;
        gen++;
        cv.notify_all();
        done_cv.wait(lk, [&] { return active == 0; });
    }
    ~Pool() {
        { std::lock_guard<std::mutex> lk(mu); stop = true; }
        cv.notify_all();
        for (auto &t : workers) t.detach();
    }
};
}  // namespace
static Pool &pool() { static Pool *p = new Pool(); return *p; }

int64_t bpg_ctx_trim(bpg_ctx *ctx) {
    return guarded([&]() -> int64_t {
        if (!ctx) throw std::runtime_error("NULL context");
        DeviceContext &c = DeviceContext::get(ctx->device);
        int64_t freed = 0;
        {
            std::lock_guard<std::mutex> lk(c.mu);
            for (auto e = c.combs.begin(); e != c.combs.end();) {
                if (e->second.use_count() == 1) { freed += (int64_t)e->second->bytes; e = c.combs.erase(e); }
                else ++e;
            }
            for (auto e = c.slices.begin(); e != c.slices.end();) {
                if (e->second.use_count() == 1) e = c.slices.erase(e);
                else ++e;
            }
            for (auto e = c.fbs.begin(); e != c.fbs.end();) {
                if (e->second.use_count() == 1) { freed += (int64_t)e->second->bytes; e = c.fbs.erase(e); }
                else ++e;
            }
        }
        // the worker pool's per-thread workspaces (streams, MSM scratch, proof
        // buffers: ~12 GB per consumer of four 2^20 proofs) and the caller's
        const int dev = ctx->device;
        std::atomic<int64_t> ws(0);
        const int nw = pool().size();
        // (and the producer stages' pinned host buffers, which are not counted)
        if (nw) pool().run(nw, [&](int) { ws += (int64_t)release_thread_workspace(dev); release_producer_stage(dev); });
        ws += (int64_t)release_thread_workspace(dev);
        release_producer_stage(dev);
        {
            std::lock_guard<std::mutex> lk(g_held_mu);
            g_held.erase(dev);
        }
        return freed + ws.load();
    }, (int64_t)-1);
}

// CPUs this process may use: the affinity mask, capped by a cgroup CPU
// quota (cgroup v2 cpu.max). Producers are sized from it: each one keeps a
// core busy drawing TranscriptRng streams.
static uint32_t process_cpus() {
    cpu_set_t set;
    uint32_t n = 0;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (uint32_t)CPU_COUNT(&set);
    if (!n) n = std::max(1u, std::thread::hardware_concurrency());
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long per = 0;
        if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
            n = std::min<uint32_t>(n, std::max<uint32_t>(1, (uint32_t)(atol(q) / per)));
        fclose(f);
    }
    return n;
}
// Hardware queues HIP gives this process: GPU_MAX_HW_QUEUES as the runtime
// read it when it initialised (its default, 4, when unset). Each consumer
// thread drives its own HIP stream; streams beyond the queues share them in
// order and serialise behind each other's kernels (47.0 vs 51.9 M
// constraints/s with 8 streams on 4 queues, profiles/r01h_sweep.txt), so
// the batch layouts size their device streams to this.
static uint32_t hw_queues() {
    static const uint32_t q = [] {
        const char *e = getenv("GPU_MAX_HW_QUEUES");
        const long v = e ? atol(e) : 0;
        return (uint32_t)(v > 0 ? v : 4);
    }();
    return q;
}
static double since_ms(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}
namespace {
// The last bpg_prove_batch's layout and pipeline counters (bpg_last_batch_stats)
std::mutex g_bs_mu;
double g_bs[BPG_BATCH_STATS] = {0};
}  // namespace

// Batched proving as a two-stage pipeline: producer threads
// draw the TranscriptRng streams of 8 proofs at a time in lockstep (rng8)
// into device slots, consumer threads drive the device part of up to
// `lockstep` proofs at once on their own HIP stream. The RNG phase of later
// proofs overlaps the device phase of earlier ones instead of alternating
// with it. Consumers are admitted by HBM: what free memory (plus the
// workspaces the pool's consumers already hold) leaves after a reserve for a
// verifier context, at consumer_bytes_estimate() each.
int bpg_prove_batch(bpg_prepared *p, const uint8_t *label, size_t label_len, const uint8_t *entropy, uint32_t count,
                    uint32_t threads, uint8_t *proof_out, size_t proof_stride, size_t *lens) {
    return guarded([&]() -> int {
        if (!count) return 0;
        const PreparedCS &cs = *p->p;
        if (!cs.prover) throw std::runtime_error("prepared circuit has no witness");
        if (threads == 0) threads = 1;
        const auto t_start = std::chrono::steady_clock::now();
        const uint32_t groups = (count + 7) / 8;
        // proofs per consumer step (1 to 4; default 4: the proofs' IPP MSM
        // jobs merged, so the latency-bound launches after each job's first
        // pass run once per four proofs. Measured at 24 proofs in flight: 82.9
        // / 83.2 M constraints/s against 81.3 / 81.0 for two per step and 75.9
        // / 70.5 for one, profiles/r03k_ab_lockstep4.txt, r03h_ab_lockstep_consumers.txt)
        const uint32_t L = p->pipe.lockstep ? p->pipe.lockstep : 4;
        // producers: one lockstep group of 8 proofs each, at most 8, at most
        // half of the threads and at most one per CPU of the process (a
        // producer keeps a core busy; ~20 proofs/s each at 2^20)
        uint32_t P = p->pipe.producers;
        if (!P) P = std::max<uint32_t>(1, std::min<uint32_t>(threads / 2, process_cpus()));
        P = std::max<uint32_t>(1, std::min<uint32_t>(std::min<uint32_t>(P, 8), groups));
        if (P >= threads && threads > 1) P = threads - 1;
        const uint32_t C_req = std::max<uint32_t>(1, threads > P ? threads - P : 1);
        uint32_t C = std::min<uint32_t>(C_req, (count + L - 1) / L);
        C = std::min<uint32_t>(C, hw_queues());   // one hardware queue per consumer stream
        // proofs in flight: at most max_inflight (default 24 at N = 2^20,
        // scaled by 1/N: a proof in flight holds ~3.1 GB next to the 208 GB
        // of comb tables, profiles/r03u_bench.json hbm_used_gb), and what
        // HBM admits
        const uint64_t cap2p20 = p->pipe.max_inflight ? p->pipe.max_inflight : 24;
        const uint64_t inflight =
            p->pipe.max_inflight ? cap2p20 : std::max<uint64_t>(1, (cap2p20 << 20) / std::max<uint32_t>(cs.N, 1));
        C = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(C, inflight / L));
        BPG_HIP(hipSetDevice(cs.device));
        size_t free_b = 0, total_b = 0;
        BPG_HIP(hipMemGetInfo(&free_b, &total_b));
        const size_t slot_bytes = 2 * (size_t)cs.n * 64 + 64;
        // RNG slots (2n x 64 B each): every consumer's L proofs, plus groups
        // of 8 being drawn by at most four producers at a time (four draw
        // ~100 proofs/s at 2^20, above what the device proves; with 2C slots
        // for the consumers, as before, CPU-starved producers held slots that
        // consumers needed for full steps, profiles/r04d_cpus4.json)
        const uint32_t draw_slots = 8 * std::min<uint32_t>(P, 4);
        const size_t est_c = consumer_bytes_estimate(cs, (int)L);
        const size_t reserve = std::max<size_t>((size_t)2 << 30, total_b / 64) + verifier_bytes_estimate(cs);
        uint32_t C_hbm = 0;
        {
            size_t held = 0, have_slots;
            {
                std::lock_guard<std::mutex> lk(g_held_mu);
                const std::vector<size_t> &h = g_held[cs.device];
                for (uint32_t id = P; id < P + C && id < h.size(); id++) held += h[id];
            }
            {
                std::lock_guard<std::mutex> lk(cs.slot_mu);
                have_slots = cs.slot_bytes >= slot_bytes ? cs.slot_bufs.size() : 0;
            }
            for (C_hbm = C; C_hbm > 1; C_hbm--) {
                const size_t want_slots = std::min<size_t>(draw_slots + (size_t)L * C_hbm, 8 * (size_t)groups);
                const size_t new_slots = want_slots > have_slots ? (want_slots - have_slots) * slot_bytes : 0;
                if ((double)C_hbm * est_c + new_slots + reserve <= (double)free_b + held) break;
            }
        }
        C = std::min(C, C_hbm);
        const uint32_t nslots = std::min<uint32_t>(draw_slots + L * C, 8 * groups);
        std::vector<uint8_t *> slot = cs.slots(nslots, slot_bytes);
        std::mutex mu;
        std::condition_variable cv;
        std::vector<int> free_slots;
        for (uint32_t i = 0; i < nslots; i++) free_slots.push_back((int)i);
        std::vector<RngBlock> blocks(count);
        std::deque<uint32_t> ready;
        std::atomic<uint32_t> next_group(0);
        uint32_t producers_left = P;
        bool abort = false, any_ready = false;
        std::string err;
        // pipeline counters (ms, summed over threads): consumers waiting for
        // a ready proof while producers were still drawing (after the first
        // group: the pipeline fill is reported on its own), producers waiting
        // for a free slot (the device is behind), producers drawing,
        // consumers proving
        double fill_ms = 0, starve_ms = 0, slot_wait_ms = 0, draw_ms = 0, prove_ms = 0;
        auto fail = [&](const std::string &e) {
            std::lock_guard<std::mutex> lk(mu);
            if (err.empty()) err = e;
            abort = true;
            cv.notify_all();
        };
        std::vector<int> slot_of(count, -1);
        std::vector<ProveTimings> timings(count);
        std::vector<size_t> held_after(P + C, 0);
        pool().run((int)(P + C), [&](int id) {
            try {
                if ((uint32_t)id < P) {
                    for (;;) {
                        uint32_t g = next_group.fetch_add(1);
                        if (g >= groups) break;
                        uint32_t k0 = 8 * g, cnt = std::min<uint32_t>(8, count - k0);
                        {
                            std::unique_lock<std::mutex> lk(mu);
                            const auto tw = std::chrono::steady_clock::now();
                            cv.wait(lk, [&] { return abort || free_slots.size() >= cnt; });
                            slot_wait_ms += since_ms(tw);
                            if (abort) break;
                            for (uint32_t i = 0; i < cnt; i++) {
                                slot_of[k0 + i] = free_slots.back();
                                free_slots.pop_back();
                            }
                        }
                        const uint8_t *ent[8];
                        RngBlock *out[8];
                        for (uint32_t i = 0; i < cnt; i++) {
                            ent[i] = entropy + 32 * (size_t)(k0 + i);
                            blocks[k0 + i].wide = slot[slot_of[k0 + i]];
                            blocks[k0 + i].on_device = true;
                            out[i] = &blocks[k0 + i];
                        }
                        const auto td = std::chrono::steady_clock::now();
                        rng_draw_group(cs, label, label_len, ent, (int)cnt, out, true);
                        const double dms = since_ms(td);
                        std::lock_guard<std::mutex> lk(mu);
                        draw_ms += dms;
                        if (!any_ready) { any_ready = true; fill_ms = since_ms(t_start); }
                        for (uint32_t i = 0; i < cnt; i++) ready.push_back(k0 + i);
                        cv.notify_all();
                    }
                    std::lock_guard<std::mutex> lk(mu);
                    producers_left--;
                    cv.notify_all();
                } else {
                    // each consumer proves up to L ready proofs at once on its
                    // stream (gpu_prove_lockstep: one MSM job per step for all)
                    for (;;) {
                        uint32_t ks[4];
                        int nk = 0;
                        {
                            std::unique_lock<std::mutex> lk(mu);
                            const auto tw = std::chrono::steady_clock::now();
                            const bool filled = any_ready;
                            cv.wait(lk, [&] { return abort || !ready.empty() || producers_left == 0; });
                            if (filled && (!ready.empty() || producers_left > 0)) starve_ms += since_ms(tw);
                            if (abort || ready.empty()) break;
                            while (!ready.empty() && nk < (int)L) {
                                ks[nk++] = ready.front();
                                ready.pop_front();
                            }
                        }
                        const RngBlock *rbs[4];
                        ProveTimings tms[4];
                        for (int i = 0; i < nk; i++) rbs[i] = &blocks[ks[i]];
                        const auto tp = std::chrono::steady_clock::now();
                        std::vector<std::vector<uint8_t>> prs = gpu_prove_lockstep(cs, label, label_len, rbs, nk, tms);
                        const double pms = since_ms(tp);
                        for (int i = 0; i < nk; i++) {
                            if (prs[i].size() > proof_stride) throw std::runtime_error("proof stride too small");
                            memcpy(proof_out + proof_stride * (size_t)ks[i], prs[i].data(), prs[i].size());
                            lens[ks[i]] = prs[i].size();
                            timings[ks[i]] = tms[i];
                        }
                        std::lock_guard<std::mutex> lk(mu);
                        prove_ms += pms;
                        for (int i = 0; i < nk; i++) free_slots.push_back(slot_of[ks[i]]);
                        cv.notify_all();
                    }
                    held_after[id] = thread_workspace_bytes(cs.device);
                }
            } catch (const dev::HipError &e) {
                fail(std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr);
            } catch (const std::exception &e) {
                fail(e.what());
            }
        });
        size_t ws_max = 0;   // the largest consumer workspace after the call (vs est_c)
        {
            std::lock_guard<std::mutex> lk(g_held_mu);
            std::vector<size_t> &h = g_held[cs.device];
            if (h.size() < P + C) h.resize(P + C, 0);
            for (uint32_t id = P; id < P + C; id++) { h[id] = held_after[id]; ws_max = std::max(ws_max, held_after[id]); }
        }
        const double wall = since_ms(t_start);
        {
            // host-bound: the consumers spent more than a tenth of their time
            // after the pipeline fill waiting for producers
            const double span = std::max(1e-9, (wall - fill_ms) * C);
            std::lock_guard<std::mutex> lk(g_bs_mu);
            const double v[BPG_BATCH_STATS] = {(double)P, (double)C, (double)L, (double)(C * L), wall, fill_ms,
                                               starve_ms, slot_wait_ms, draw_ms, prove_ms,
                                               starve_ms / span > 0.10 ? 1.0 : 0.0, free_b / 1e9, est_c / 1e9,
                                               (double)C_req, (double)C_hbm, (double)process_cpus(),
                                               (double)hw_queues(), ws_max / 1e9};
            memcpy(g_bs, v, sizeof(v));
        }
        if (!err.empty()) throw std::runtime_error(err);
        last_timings() = timings[count - 1];   // the caller's thread reports the batch's last proof
        return 0;
    }, -1);
}
int bpg_last_batch_stats(double *out, int n) {
    std::lock_guard<std::mutex> lk(g_bs_mu);
    for (int i = 0; i < n && i < BPG_BATCH_STATS; i++) out[i] = g_bs[i];
    return 0;
}

// prove.rs:37-82 for `count` distinct statements (include/bpg.h): CPU
// workers synthesise and upload statements and draw the TranscriptRng
// streams of up to 8 of them in lockstep (rng_draw_multi); consumer threads
// (one HIP stream each, mostly asleep on the device) run the device part.
static ProofArtifacts *make_artifacts(const std::string &coms, const std::vector<uint8_t> &proof) {
    ProofArtifacts *a = (ProofArtifacts *)malloc(sizeof(ProofArtifacts));
    char *c = (char *)malloc(coms.size() + 1);
    uint8_t *p = (uint8_t *)malloc(proof.size() ? proof.size() : 1);
    if (!a || !c || !p) { free(a); free(c); free(p); throw std::runtime_error("out of memory"); }
    memcpy(c, coms.c_str(), coms.size() + 1);
    memcpy(p, proof.data(), proof.size());
    a->commitments = c;
    a->proof = p;
    a->proof_len = proof.size();
    a->proof_cap = proof.size();
    return a;
}
namespace {
std::atomic<uint32_t> g_stmt_consumers(0), g_stmt_lockstep(0);   // bpg_set_statements_layout (0: defaults)
std::mutex g_ss_mu;
double g_ss[18] = {0};   // bpg_last_statements_stats
}  // namespace
int bpg_prove_statements(const char *name, const char *const *instances, const char *const *witnesses,
                         const char *const *gadgets, const uint64_t *seeds, uint32_t count, uint32_t threads,
                         struct ProofArtifacts **out) {
    return guarded([&]() -> int {
        if (!name || (count && (!instances || !witnesses || !gadgets || !out))) throw std::runtime_error("NULL argument");
        require_device();
        if (!count) return 0;
        for (uint32_t k = 0; k < count; k++) out[k] = nullptr;
        const int device = g_device;
        const auto t_start = std::chrono::steady_clock::now();
        const uint32_t W = std::max<uint32_t>(1, threads);
        const uint32_t c_set = g_stmt_consumers.load();
        // device threads, each proving up to L ready statements of one shape
        // in lockstep (one MSM job per IPP round for all of them, as
        // bpg_prove_batch does for one circuit)
        const uint32_t l_set = g_stmt_lockstep.load();
        uint32_t L = l_set ? l_set : 4;   // lowered by the HBM admission if need be (under mu)
        // device threads: the layout's (default 5), at most one per hardware
        // queue, then admitted by HBM below
        const uint32_t C = std::min<uint32_t>(std::min<uint32_t>(c_set ? c_set : 5, hw_queues()),
                                              std::max<uint32_t>(1, c_set ? c_set : W / 2));
        const size_t label_len = strlen(name);
        const uint8_t *label = (const uint8_t *)name;
        struct Item {
            uint32_t k;
            std::unique_ptr<PreparedCS> cs;
            std::string coms;
            uint8_t entropy[32];
            RngBlock rb;
        };
        BPG_HIP(hipSetDevice(device));
        size_t free_b = 0, total_b = 0;
        BPG_HIP(hipMemGetInfo(&free_b, &total_b));
        size_t held = 0;
        {
            std::lock_guard<std::mutex> lk(g_held_mu);
            const std::vector<size_t> &h = g_held[device];
            for (uint32_t id = W; id < W + C && id < h.size(); id++) held += h[id];
        }
        std::mutex mu;
        std::condition_variable cv;
        std::deque<std::unique_ptr<Item>> prepared, ready;
        // prepared statements of finished proofs, recycled (device arrays and
        // RNG slot kept: no hipMalloc / hipFree per statement)
        std::vector<std::unique_ptr<PreparedCS>> spare;
        uint32_t next = 0, synth_busy = 0, inflight = 0, done = 0, proved = 0;
        uint32_t consumers_left = 0, oom_retired = 0;   // device threads still proving; retired on OOM
        // statements in flight (synthesised, prepared, drawn or being proved):
        // a statement spends ~0.5 s between its synthesis and the end of its
        // RNG group's draw (the group forms from eight prepared statements),
        // so by Little's law the in-flight count bounds the rate: W + 8 + 2C
        // (40 at 16 workers) held it to ~35 statements/s
        // (profiles/r04d_statements.json). At most 4W + 8 + 2C, and at most
        // what HBM holds next to the consumers' workspaces, sized once the
        // first statement is prepared (until then at most W)
        uint32_t limit = 4 * W + 8 + 2 * C, hbm_limit = 0, C_eff = C;
        double est_st = 0, adm_free_b = 0, per_c_est = 0;
        double synth_ms = 0, prep_ms = 0, rng_ms = 0, prove_ms = 0, widle_ms = 0, cidle_ms = 0;
        std::string first_err;
        bool fatal = false;
        auto note_err = [&](uint32_t k, const std::string &e, bool hip) {
            std::lock_guard<std::mutex> lk(mu);
            if (first_err.empty()) first_err = "statement " + std::to_string(k) + ": " + e;
            if (hip) fatal = true;
            cv.notify_all();
        };
        std::vector<size_t> held_after(W + C, 0);
        pool().run((int)(W + C), [&](int id) {
            const bool worker = (uint32_t)id < W;
            for (;;) {
                std::vector<std::unique_ptr<Item>> group;
                std::vector<std::unique_ptr<Item>> items;   // a consumer's lockstep step
                std::unique_ptr<PreparedCS> reuse;
                uint32_t k = 0;
                int what = 0;   // 1 synthesise k, 2 RNG group, 3 device
                {
                    std::unique_lock<std::mutex> lk(mu);
                    const auto tw = std::chrono::steady_clock::now();
                    cv.wait(lk, [&] {
                        if (fatal || done == count) return true;
                        if (!worker) return (uint32_t)id - W >= C_eff || !ready.empty();
                        const bool tail = next == count && synth_busy == 0;
                        if (prepared.size() >= 8 || (tail && !prepared.empty())) return true;
                        return next < count && inflight < (est_st > 0 ? limit : W);
                    });
                    if (!worker && (uint32_t)id - W >= C_eff) break;   // not admitted by HBM
                    (worker ? widle_ms : cidle_ms) += since_ms(tw);
                    if (fatal || done == count) break;
                    if (!worker) {
                        items.push_back(std::move(ready.front()));
                        ready.pop_front();
                        // up to L - 1 more ready statements of the same shape
                        const PreparedCS &c0 = *items[0]->cs;
                        for (auto it = ready.begin(); it != ready.end() && items.size() < L;) {
                            const PreparedCS &c = *(*it)->cs;
                            if (c.n == c0.n && c.m == c0.m && c.N == c0.N) {
                                items.push_back(std::move(*it));
                                it = ready.erase(it);
                            } else {
                                ++it;
                            }
                        }
                        what = 3;
                    } else if (prepared.size() >= 8 || (next == count && synth_busy == 0 && !prepared.empty())) {
                        while (!prepared.empty() && group.size() < 8) {
                            group.push_back(std::move(prepared.front()));
                            prepared.pop_front();
                        }
                        what = 2;
                    } else {
                        k = next++;
                        synth_busy++;
                        inflight++;
                        if (!spare.empty()) { reuse = std::move(spare.back()); spare.pop_back(); }
                        what = 1;
                    }
                }
                if (what == 1) {
                    std::unique_ptr<Item> it(new Item());
                    it->k = k;
                    bool ok = false;
                    double ms_s = 0, ms_p = 0;
                    try {
                        EntropySource &e = thread_entropy();
                        const EntropySource saved = e;
                        if (seeds) { e.seeded = true; e.cs.seed(seeds[k]); }
                        try {
                            const auto t0 = std::chrono::steady_clock::now();
                            Synthesis syn = synthesize_prover(instances[k], witnesses[k], gadgets[k]);
                            bpg_r1cs_view v = syn.cs->view(true);
                            ms_s = since_ms(t0);
                            const auto t1 = std::chrono::steady_clock::now();
                            it->cs = prepare_cs(&v, device, Strategy(), 0, 1, std::move(reuse));
                            for (size_t i = 0; i < syn.com_names.size(); i++)
                                it->coms += syn.com_names[i] + " = 0x" + hex32(it->cs->V.data() + 32 * i) + "\n";
                            e.fill(it->entropy, 32);
                            it->rb.wide = it->cs->slots(1, 2 * (size_t)it->cs->n * 64 + 64)[0];
                            it->rb.on_device = true;
                            ms_p = since_ms(t1);
                        } catch (...) {
                            e = saved;
                            throw;
                        }
                        e = saved;
                        ok = true;
                    } catch (const dev::HipError &e) {
                        note_err(k, std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr, true);
                    } catch (const std::exception &e) {
                        note_err(k, e.what(), false);
                    }
                    std::lock_guard<std::mutex> lk(mu);
                    synth_busy--;
                    synth_ms += ms_s;
                    prep_ms += ms_p;
                    if (ok && est_st == 0) {
                        // HBM budget, sized from the first prepared statement:
                        // free memory and the consumers' reusable workspaces,
                        // less a reserve, must hold C_eff consumer workspaces
                        // of L proofs and at least C_eff L + 8 statements in
                        // flight (the rest of it bounds the in-flight limit);
                        // consumers beyond C_eff stay idle. When not even one
                        // consumer of L fits, L is lowered (a consumer of one
                        // proof needs about a third of one of four); when one
                        // of one does not fit, the call fails here with an
                        // error, before any proof allocates.
                        est_st = (double)prepared_bytes(*it->cs);
                        const double reserve = std::max<double>(2.0 * (1 << 30), total_b / 64.0);
                        // free memory now: the first prepare built the comb
                        // tables (208 GB at 2^20) if no earlier call had;
                        // this statement's own bytes count as in flight
                        size_t free_now = 0, tot_now = 0;
                        BPG_HIP(hipMemGetInfo(&free_now, &tot_now));
                        adm_free_b = (double)free_now;
                        const double all = (double)free_now + (double)held + est_st - reserve;
                        double per_c = 0;
                        uint32_t c_fit = 0;
                        for (uint32_t l = L; l >= 1 && !c_fit; l--) {
                            per_c = (double)consumer_bytes_estimate(*it->cs, (int)l);
                            for (uint32_t c = C; c >= 1; c--)
                                if (c * per_c + (c * l + 8) * est_st <= all) { c_fit = c; L = l; break; }
                        }
                        if (!c_fit) {
                            char msg[256];
                            snprintf(msg, sizeof msg,
                                     "not enough free HBM for one device thread: %.1f GB free, %.1f GB needed "
                                     "(one proof's workspace and 9 statements in flight, %.1f GB reserve)",
                                     free_now / 1e9, (per_c + 9 * est_st + reserve) / 1e9, reserve / 1e9);
                            if (first_err.empty()) first_err = msg;
                            fatal = true;
                            c_fit = 1;
                        }
                        C_eff = c_fit;
                        per_c_est = per_c;
                        consumers_left = C_eff;
                        hbm_limit = (uint32_t)std::max<double>(std::min<double>(C_eff * L + 8, limit),
                                                               (all - C_eff * per_c) / est_st);
                        limit = std::min(limit, hbm_limit);
                    }
                    if (ok) prepared.push_back(std::move(it));
                    else { inflight--; done++; }
                    cv.notify_all();
                } else if (what == 2) {
                    const auto t0 = std::chrono::steady_clock::now();
                    try {
                        const PreparedCS *cs[8];
                        const uint8_t *ent[8];
                        RngBlock *rb[8];
                        for (size_t i = 0; i < group.size(); i++) {
                            cs[i] = group[i]->cs.get();
                            ent[i] = group[i]->entropy;
                            rb[i] = &group[i]->rb;
                        }
                        rng_draw_multi(cs, label, label_len, ent, (int)group.size(), rb);
                    } catch (const dev::HipError &e) {
                        note_err(group[0]->k, std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr,
                                 true);
                    } catch (const std::exception &e) {
                        note_err(group[0]->k, e.what(), true);
                    }
                    const double ms = since_ms(t0);
                    std::lock_guard<std::mutex> lk(mu);
                    rng_ms += ms;
                    for (auto &g : group) ready.push_back(std::move(g));
                    cv.notify_all();
                } else {
                    const auto t0 = std::chrono::steady_clock::now();
                    const int P = (int)items.size();
                    bool oom = false;
                    try {
                        const PreparedCS *csv[MAX_LOCKSTEP];
                        const RngBlock *rbs[MAX_LOCKSTEP];
                        for (int i = 0; i < P; i++) { csv[i] = items[i]->cs.get(); rbs[i] = &items[i]->rb; }
                        std::vector<std::vector<uint8_t>> prs = gpu_prove_lockstep(csv, label, label_len, rbs, P, nullptr);
                        for (int i = 0; i < P; i++) out[items[i]->k] = make_artifacts(items[i]->coms, prs[i]);
                        std::lock_guard<std::mutex> lk(mu);
                        proved += P;
                    } catch (const dev::HipError &e) {
                        // a device thread whose workspace could not grow (the
                        // admission's estimate was short): it hands its
                        // statements back, frees its workspace and retires,
                        // and the remaining device threads prove them (the
                        // draws are on the device; proving is deterministic).
                        // The last device thread does not retire: the error
                        // ends the call.
                        oom = e.err == hipErrorOutOfMemory;
                        if (oom) {
                            std::lock_guard<std::mutex> lk(mu);
                            oom = consumers_left > 1;
                            if (oom) consumers_left--;
                        }
                        if (!oom)
                            note_err(items[0]->k,
                                     std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr, true);
                    } catch (const std::exception &e) {
                        note_err(items[0]->k, e.what(), false);
                    }
                    if (oom) {
                        (void)hipGetLastError();
                        try {
                            release_thread_workspace(device);
                        } catch (...) {
                        }
                        std::lock_guard<std::mutex> lk(mu);
                        oom_retired++;
                        for (auto it = items.rbegin(); it != items.rend(); ++it) ready.push_front(std::move(*it));
                        items.clear();
                        cv.notify_all();
                        break;   // this device thread retires
                    }
                    const double ms = since_ms(t0);
                    std::lock_guard<std::mutex> lk(mu);
                    prove_ms += ms;
                    for (auto &it : items) spare.push_back(std::move(it->cs));   // recycled by the next statements
                    items.clear();
                    inflight -= P;
                    done += P;
                    cv.notify_all();
                }
            }
            if (!worker) held_after[id] = thread_workspace_bytes(device);
        });
        size_t ws_max = 0;   // the largest device-thread workspace after the call (vs the estimate)
        {
            std::lock_guard<std::mutex> lk(g_held_mu);
            std::vector<size_t> &h = g_held[device];
            if (h.size() < W + C) h.resize(W + C, 0);
            for (uint32_t id = W; id < W + C; id++) { h[id] = held_after[id]; ws_max = std::max(ws_max, held_after[id]); }
        }
        spare.clear();   // the recycled statements' device memory, freed once per call
        {
            // the bounding stage: the busier of the two (its threads' busy
            // share of the wall time; the workers' idle time includes each
            // call's fill and drain)
            const double wall = since_ms(t_start);
            const double wbusy = 1.0 - widle_ms / std::max(1e-9, wall * W);
            const double cbusy = 1.0 - cidle_ms / std::max(1e-9, wall * C_eff);
            const int bound = wbusy >= cbusy ? 1 : 2;
            const double v[18] = {(double)W, (double)C_eff, (double)limit, wall, synth_ms, prep_ms, rng_ms, prove_ms,
                                  widle_ms, cidle_ms, (double)bound, (double)hbm_limit, est_st / 1e9, (double)L,
                                  adm_free_b / 1e9, (double)oom_retired, per_c_est / 1e9, ws_max / 1e9};
            std::lock_guard<std::mutex> lk(g_ss_mu);
            memcpy(g_ss, v, sizeof(v));
        }
        if (fatal) {
            for (uint32_t k = 0; k < count; k++) { free_proof(out[k]); out[k] = nullptr; }
            throw std::runtime_error(first_err);
        }
        if (!first_err.empty()) set_err(first_err);
        const int n_ok = (int)proved;
        if (n_ok < (int)count) g_err = first_err;   // guarded() cleared it on entry; keep the reason
        return n_ok;
    }, -1);
}
int bpg_set_statements_layout(uint32_t consumers, uint32_t lockstep) {
    // no fixed cap on device threads: each call takes at most one per
    // hardware queue and what the HBM admission holds (round 4 capped them at
    // 12 after 16 aborted the process's HSA queues: a kernel's lazily
    // allocated scratch memory next to a full HBM; the prove path needs no
    // scratch now, tests/test_host.py)
    if (consumers > 64 || lockstep > (uint32_t)MAX_LOCKSTEP) return -1;
    g_stmt_consumers = consumers;
    g_stmt_lockstep = lockstep;
    return 0;
}
int bpg_last_statements_stats(double *out, int n) {
    std::lock_guard<std::mutex> lk(g_ss_mu);
    for (int i = 0; i < n && i < 18; i++) out[i] = g_ss[i];
    return 0;
}

// Verifier::verify (verify.rs:71) over `count` proofs of one prepared
// circuit: the proofs are cut into chunks of 8 to 64 (about six), and each
// worker thread checks a chunk at a time with one random-linear-
// combination MSM on its own HIP stream (gpu_verify_batch; a chunk that
// fails is re-verified proof by proof). results[k] = 1 accept, 0 reject.
int bpg_verify_batch(bpg_prepared *p, const uint8_t *label, size_t label_len, const uint8_t *V,
                     const uint8_t *proofs, size_t proof_stride, const size_t *lens, uint32_t count,
                     uint32_t threads, const uint8_t entropy[32], int *results) {
    return guarded([&]() -> int {
        if (!count) return 0;
        const PreparedCS &cs = *p->p;
        // the prover's layout drops the constant column the verifier needs
        if (cs.prover) throw std::runtime_error("circuit prepared for proving: use bpg_prepare_verifier");
        if (threads == 0) threads = 1;
        // chunks of 8-64 proofs, about six of them at once: a chunk's MSM
        // covers the 2N generators once however many proofs it holds, so
        // larger chunks amortise it better (192 proofs in chunks of 8 / 16 /
        // 32 / 64: 1,170 / 1,431 / 1,538 / 1,631 proofs/s,
        // profiles/r04y_verify_chunks.txt)
        const uint32_t chunk = std::min<uint32_t>(64, std::max<uint32_t>(8, (count + 5) / 6));
        const uint32_t nchunks = (count + chunk - 1) / chunk;
        threads = std::min<uint32_t>(threads, nchunks);
        std::atomic<uint32_t> next(0);
        std::mutex mu;
        std::string err;
        pool().run((int)threads, [&](int) {
            try {
                for (;;) {
                    const uint32_t c = next.fetch_add(1);
                    if (c >= nchunks) break;
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        if (!err.empty()) break;
                    }
                    const uint32_t k0 = c * chunk, k1 = std::min(count, k0 + chunk);
                    gpu_verify_batch(cs, label, label_len, V, proofs + proof_stride * (size_t)k0, proof_stride,
                                     lens + k0, k1 - k0, entropy, results + k0);
                }
            } catch (const dev::HipError &e) {
                std::lock_guard<std::mutex> lk(mu);
                if (err.empty()) err = std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr;
            } catch (const std::exception &e) {
                std::lock_guard<std::mutex> lk(mu);
                if (err.empty()) err = e.what();
            }
        });
        if (!err.empty()) throw std::runtime_error(err);
        return 0;
    }, -1);
}

// Diagnostics: lockstep RNG against the scalar TranscriptRng (0 = equal),
// and its draw rate (draws per second per thread for `lanes` proofs).
int bpg_rng_selftest(void) {
    return guarded([&]() -> int {
        // the permutations against the portable scalar Keccak-f[1600]
        uint64_t x = 0x9e3779b97f4a7c15ULL;
        for (int t = 0; t < 64; t++) {
            uint64_t a[25], b[25];
            for (int i = 0; i < 25; i++) {
                x = x * 6364136223846793005ULL + 1442695040888963407ULL;
                a[i] = b[i] = x;
            }
            keccakf_scalar(a);
            keccakf(b);   // the AVX-512 single-state form where available
            if (memcmp(a, b, sizeof(a))) return 20;
        }
        {
            // keccak8 lane k equals the scalar permutation of lane k's state
            alignas(64) uint64_t L[25][8];
            uint64_t ref[8][25];
            for (int i = 0; i < 25; i++)
                for (int k = 0; k < 8; k++) L[i][k] = ref[k][i] = 0x0123456789abcdefULL * (uint64_t)(i + 1) + (uint64_t)k * 0x1111;
            keccak8(L);
            for (int k = 0; k < 8; k++) {
                keccakf_scalar(ref[k]);
                for (int i = 0; i < 25; i++) if (L[i][k] != ref[k][i]) return 21;
            }
        }
        Transcript T((const uint8_t *)"selftest", 8);
        T.append_u64("m", 3);
        TranscriptRng base(T);
        base.rekey_with_witness_bytes("v_blinding", (const uint8_t *)"0123456789abcdef0123456789abcdef", 32);
        {
            // TranscriptRng::draw64 (constant-framing fast path) = fill_bytes
            TranscriptRng r1(base), r2(base);
            const uint8_t ent[32] = {7, 1, 2};
            r1.finalize(ent);
            r2.finalize(ent);
            uint8_t a[64], b[64];
            for (int d = 0; d < 300; d++) {
                r1.fill_bytes(a, d % 7 == 3 ? 32 : 64);
                if (d % 7 == 3) { r2.fill_bytes(b, 32); }
                else r2.draw64(b);
                if (memcmp(a, b, d % 7 == 3 ? 32 : 64)) return 22;
            }
        }
        for (int lanes = 1; lanes <= 8; lanes++) {
            uint8_t ent[8][32];
            const uint8_t *ep[8];
            for (int k = 0; k < 8; k++) { for (int i = 0; i < 32; i++) ent[k][i] = (uint8_t)(k * 31 + i * 7 + lanes); ep[k] = ent[k]; }
            Strobe8 S; S.from(base.s, lanes);
            S.meta_ad((const uint8_t *)"rng", 3);
            S.key_each(ep, 32);
            std::vector<TranscriptRng> ref;
            for (int k = 0; k < lanes; k++) { ref.push_back(base); ref.back().finalize(ent[k]); }
            uint8_t out[8][64], want[64];
            uint8_t *op[8];
            for (int k = 0; k < 8; k++) op[k] = out[k];
            for (int d = 0; d < 300; d++) {
                S.draw64(op);
                for (int k = 0; k < lanes; k++) {
                    ref[k].fill_bytes(want, 64);
                    if (memcmp(want, out[k], 64)) return 1 + lanes;
                }
            }
        }
        return 0;
    }, -1);
}
double bpg_rng_rate(uint32_t draws, int lanes) {
    return guarded([&]() -> double {
        Transcript T((const uint8_t *)"rate", 4);
        TranscriptRng base(T);
        Strobe8 S; S.from(base.s, lanes < 1 ? 1 : (lanes > 8 ? 8 : lanes));
        uint8_t ent[32] = {1};
        const uint8_t *ep[8] = {ent, ent, ent, ent, ent, ent, ent, ent};
        S.meta_ad((const uint8_t *)"rng", 3);
        S.key_each(ep, 32);
        std::vector<uint8_t> buf((size_t)8 * 64);
        uint8_t *op[8];
        for (int k = 0; k < 8; k++) op[k] = buf.data() + 64 * k;
        auto t0 = std::chrono::steady_clock::now();
        for (uint32_t d = 0; d < draws; d++) S.draw64(op);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return dt > 0 ? draws * (double)S.nstates / dt : 0.0;
    }, -1.0);
}

int bpg_last_timings(double *out, int n) {
    const ProveTimings &t = last_timings();
    double v[5] = {t.rng_ms, t.commit_ms, t.vec_ms, t.ipp_ms, t.total_ms};
    for (int i = 0; i < n && i < 5; i++) out[i] = v[i];
    return 0;
}

int bpg_msm(bpg_ctx *ctx, const uint8_t *scalars, const uint8_t *points, uint32_t count, uint8_t out[32]) {
    return guarded([&]() -> int { return gpu_msm(ctx->device, scalars, points, count, out); }, -2);
}

// Synthesis export (no device work; commitments are not computed here).
struct bpg_synth {
    Synthesis s;
    bpg_r1cs_view view;
    std::string names;
};
bpg_synth *bpg_synthesize(const char *instance, const char *witness, const char *gadgets) {
    return guarded([&]() -> bpg_synth * {
        bpg_synth *b = new bpg_synth();
        b->s = synthesize_prover(instance, witness, gadgets);
        b->view = b->s.cs->view(true);
        for (auto &n : b->s.com_names) b->names += n + "\n";
        return b;
    }, (bpg_synth *)nullptr);
}
bpg_synth *bpg_synthesize_verifier(const char *instance, const char *commitments, const char *gadgets) {
    return guarded([&]() -> bpg_synth * {
        bpg_synth *b = new bpg_synth();
        b->s = synthesize_verifier(instance, commitments, gadgets);
        b->view = b->s.cs->view(false);
        return b;
    }, (bpg_synth *)nullptr);
}
const bpg_r1cs_view *bpg_synth_view(const bpg_synth *s) { return &s->view; }
const char *bpg_synth_commitments(const bpg_synth *s) { return s->names.c_str(); }
const uint8_t *bpg_synth_V(const bpg_synth *s) { return s->s.cs->V().data(); }
void bpg_synth_free(bpg_synth *s) { delete s; }

// Gadget-API recorder (bulletproofs r1cs::ConstraintSystem as the
// reference's ProverBuffer / VerifierBuffer record it, cs_buffer.rs:22-199).
struct bpg_cs {
    ConstraintSystem cs;
    bpg_r1cs_view view;
    explicit bpg_cs(bool prover) : cs(prover), view() {}
};
static LC to_lc(const bpg_lc *l) {
    LC r;
    if (!l) return r;
    if (l->nterms && (!l->vars || !l->coeffs)) throw std::runtime_error("NULL linear combination");
    r.t.reserve(l->nterms);
    for (uint32_t k = 0; k < l->nterms; k++) {   // kept as given, like dalek's (possibly unreduced) Scalars
        Scalar c;
        memcpy(c.v, l->coeffs + 32 * (size_t)k, 32);
        r.t.push_back({l->vars[k], c});
    }
    return r;
}
static void check_lc_vars(const bpg_cs *c, const LC &lc) {
    for (auto &t : lc.t) {
        const uint32_t kind = BPG_VAR_KIND(t.first), idx = BPG_VAR_INDEX(t.first);
        const bool ok = kind == BPG_VAR_ONE ? idx == 0
                        : kind == BPG_VAR_V  ? idx < c->cs.m()
                        : (kind >= BPG_VAR_L && kind <= BPG_VAR_O) ? idx < c->cs.n() : false;
        if (!ok) throw std::runtime_error("linear combination names an unknown variable");
    }
}
bpg_cs *bpg_cs_create(int prover) {
    return guarded([&]() -> bpg_cs * { return new bpg_cs(prover != 0); }, (bpg_cs *)nullptr);
}
void bpg_cs_free(bpg_cs *c) { delete c; }
int64_t bpg_cs_commit(bpg_cs *c, const uint8_t v[32], const uint8_t v_blinding[32]) {
    return guarded([&]() -> int64_t {
        if (!c->cs.prover()) throw std::runtime_error("verifier-side recorder: use bpg_cs_commit_point");
        Scalar a, b;
        memcpy(a.v, v, 32);            // Scalar::from_bits: kept as given (prove.rs commits may be unreduced)
        memcpy(b.v, v_blinding, 32);
        return (int64_t)c->cs.commit_value(a, b);
    }, (int64_t)-1);
}
int64_t bpg_cs_commit_point(bpg_cs *c, const uint8_t V[32]) {
    return guarded([&]() -> int64_t {
        if (c->cs.prover()) throw std::runtime_error("prover-side recorder: use bpg_cs_commit");
        return (int64_t)c->cs.commit_point(V);
    }, (int64_t)-1);
}
int bpg_cs_multiply(bpg_cs *c, const bpg_lc *left, const bpg_lc *right, uint32_t out[3]) {
    return guarded([&]() -> int {
        LC l = to_lc(left), r = to_lc(right);
        check_lc_vars(c, l);
        check_lc_vars(c, r);
        ConstraintSystem::Triple t = c->cs.multiply(l, r);
        out[0] = t.l; out[1] = t.r; out[2] = t.o;
        return 0;
    }, -1);
}
int bpg_cs_allocate_multiplier(bpg_cs *c, const uint8_t *left, const uint8_t *right, uint32_t out[3]) {
    return guarded([&]() -> int {
        ConstraintSystem::Triple t;
        if (c->cs.prover()) {
            if (!left || !right) throw std::runtime_error("prover-side allocate_multiplier needs an assignment");
            Scalar l = Scalar::reduce(left), r = Scalar::reduce(right);
            t = c->cs.allocate_multiplier(&l, &r);
        } else {
            t = c->cs.allocate_multiplier(nullptr, nullptr);
        }
        out[0] = t.l; out[1] = t.r; out[2] = t.o;
        return 0;
    }, -1);
}
int bpg_cs_constrain(bpg_cs *c, const bpg_lc *lc) {
    return guarded([&]() -> int {
        LC l = to_lc(lc);
        check_lc_vars(c, l);
        c->cs.constrain(l);
        return 0;
    }, -1);
}
int bpg_cs_merkle_tree(bpg_cs *c, const bpg_lc *root, const bpg_lc *inst, uint32_t ninst, const bpg_lc *wit,
                       uint32_t nwit, const char *pattern) {
    return guarded([&]() -> int {
        if (!pattern) throw std::runtime_error("NULL pattern");
        std::vector<LC> i, w;
        for (uint32_t k = 0; k < ninst; k++) { i.push_back(to_lc(inst + k)); check_lc_vars(c, i.back()); }
        for (uint32_t k = 0; k < nwit; k++) { w.push_back(to_lc(wit + k)); check_lc_vars(c, w.back()); }
        LC r = to_lc(root);
        check_lc_vars(c, r);
        merkle_tree_assemble(c->cs, r, std::move(i), std::move(w), pattern);
        return 0;
    }, -1);
}
int bpg_cs_range_proof(bpg_cs *c, const bpg_lc *x, uint32_t bits, const uint8_t *x_assignment) {
    return guarded([&]() -> int {
        if (bits > 256) throw std::runtime_error("range proof wider than 256 bits");
        LC l = to_lc(x);
        check_lc_vars(c, l);
        Scalar a;
        if (x_assignment) memcpy(a.v, x_assignment, 32);
        if (c->cs.prover() && !x_assignment) throw std::runtime_error("prover-side range proof needs the assignment");
        range_proof_assemble(c->cs, l, bits, c->cs.prover() ? &a : nullptr);
        return 0;
    }, -1);
}
const bpg_r1cs_view *bpg_cs_view(bpg_cs *c) {
    c->view = c->cs.view(true);
    return &c->view;
}
const uint8_t *bpg_cs_V(const bpg_cs *c) { return c->cs.V().data(); }

int bpg_mimc_hash(const uint8_t *data, size_t len, uint8_t out[32]) {
    return guarded([&]() -> int {
        mimc_hash(std::vector<uint8_t>(data, data + len)).to_bytes(out);
        return 0;
    }, -1);
}
int bpg_mimc_sponge(const uint8_t *blocks, uint32_t count, uint8_t out[32]) {
    return guarded([&]() -> int {
        std::vector<Scalar> b(count);
        for (uint32_t i = 0; i < count; i++) b[i] = Scalar::from_bits(blocks + 32 * (size_t)i);
        mimc_sponge_native(b).to_bytes(out);
        return 0;
    }, -1);
}

int bpg_profile_enable(int on) { return set_kernel_profiling(on != 0); }
int bpg_kernel_stats(const char *name, uint64_t *launches, double *total_ms, double *alg_bytes) {
    KernelStat st;
    if (!get_kernel_stat(name, st)) return -1;
    *launches = st.launches;
    *total_ms = st.total_ms;
    *alg_bytes = st.alg_bytes;
    return 0;
}
int bpg_kernel_femul(const char *name, double *femul) {
    KernelStat st;
    if (!get_kernel_stat(name, st)) return -1;
    *femul = st.femul;
    return 0;
}
void bpg_kernel_stats_reset(void) { reset_kernel_stats(); }

}  // extern "C"
