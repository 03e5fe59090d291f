// capi.cpp — the exported C ABI (include/bpg.h).
//   c_prove / c_verify / free_proof: interfaces/ios/src/lib.rs:20-66 over
//   src/prove.rs:37-82 and src/verify.rs:36-73. Errors never cross the ABI:
//   NULL / false plus bpg_last_error().
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

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

// ------------------------------------------------------------ inner ABI
struct bpg_ctx { int device; };
bpg_ctx *bpg_ctx_create(int device) {
    return guarded([&]() -> bpg_ctx * {
        g_device = device;
        require_device();
        DeviceContext::get(device);
        return new bpg_ctx{device};
    }, (bpg_ctx *)nullptr);
}
void bpg_ctx_destroy(bpg_ctx *ctx) { delete ctx; }

int bpg_gens_ensure(bpg_ctx *ctx, uint32_t capacity) {
    return guarded([&]() -> int {
        DeviceContext::get(ctx->device).ensure_gens(capacity);
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
        std::unique_ptr<PreparedCS> P = prepare_cs(cs, ctx->device);
        std::vector<uint8_t> proof = gpu_prove(*P, label, label_len, entropy);
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

struct bpg_prepared { std::unique_ptr<PreparedCS> p; };
bpg_prepared *bpg_prepare(bpg_ctx *ctx, const bpg_r1cs_view *cs) {
    return guarded([&]() -> bpg_prepared * {
        bpg_prepared *b = new bpg_prepared();
        b->p = prepare_cs(cs, ctx->device);
        DeviceContext::get(ctx->device).ensure_gens(b->p->N);
        return b;
    }, (bpg_prepared *)nullptr);
}
void bpg_prepared_free(bpg_prepared *p) { delete p; }

// Persistent host worker pool: each worker owns its thread-local device
// workspace (stream + buffers), so repeated batches reuse HBM allocations.
namespace {
struct Pool {
    std::vector<std::thread> workers;
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
    void run(int n, std::function<void(int)> f) {
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
Pool &pool() { static Pool *p = new Pool(); return *p; }
}  // namespace

int bpg_prove_batch(bpg_prepared *p, const uint8_t *label, size_t label_len, const uint8_t *entropy, uint32_t count,
                    uint32_t threads, uint8_t *proof_out, size_t proof_stride, size_t *lens) {
    return guarded([&]() -> int {
        if (threads == 0) threads = 1;
        if (threads > count) threads = count ? count : 1;
        std::atomic<uint32_t> next(0);
        std::mutex emu;
        std::string err;
        pool().run((int)threads, [&](int) {
            try {
                for (;;) {
                    uint32_t k = next.fetch_add(1);
                    if (k >= count) break;
                    std::vector<uint8_t> pr = gpu_prove(*p->p, label, label_len, entropy + 32 * (size_t)k);
                    if (pr.size() > proof_stride) throw std::runtime_error("proof stride too small");
                    memcpy(proof_out + proof_stride * (size_t)k, pr.data(), pr.size());
                    lens[k] = pr.size();
                }
            } catch (const dev::HipError &e) {
                std::lock_guard<std::mutex> lk(emu);
                err = std::string("HIP error: ") + hipGetErrorString(e.err) + " in " + e.expr;
            } catch (const std::exception &e) {
                std::lock_guard<std::mutex> lk(emu);
                err = e.what();
            }
        });
        if (!err.empty()) throw std::runtime_error(err);
        return 0;
    }, -1);
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
void bpg_kernel_stats_reset(void) { reset_kernel_stats(); }

}  // extern "C"
