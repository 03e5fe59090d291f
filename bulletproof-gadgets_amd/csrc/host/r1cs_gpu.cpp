// r1cs_gpu.cpp — see r1cs_gpu.h.
// Protocol steps follow bulletproofs@2.1.0 src/r1cs/prover.rs `prove` and
// src/r1cs/verifier.rs `verify` (one-phase circuits: no deferred
// constraints), src/inner_product_proof.rs `create` / `verification_scalars`,
// and src/r1cs/proof.rs `to_bytes` / `from_bytes`.
#include "r1cs_gpu.h"

#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <map>
#include <stdexcept>

namespace bpg {
using namespace dev;

static inline ScD to_dev(const Scalar &s) { ScD d; memcpy(d.v, s.v, 32); return d; }
static inline Scalar from_dev(const ScD &d) { Scalar s; memcpy(s.v, d.v, 32); return s; }
static const Scalar R_MOD_L = {{0xd6ec31748d98951dULL, 0xc6ef5bf4737dcf70ULL, 0xfffffffffffffffeULL, 0x0fffffffffffffffULL}};
static inline ScD mont(const Scalar &s) { return to_dev(s * R_MOD_L); }
static uint32_t next_pow2(uint32_t n) { uint32_t p = 1; while (p < n) p <<= 1; return p; }
static uint32_t lg2u(uint32_t n) { uint32_t k = 0; while ((1u << k) < n) k++; return k; }
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------ context
// Fatal-signal report: a native backtrace on stderr before the default
// action (the round-4 exit-time SIGSEGV left no stack). Installed with the
// first device context, only for signals nobody else handles (an embedding
// runtime's own handler, e.g. Python's faulthandler, is left alone).
static void crash_report(int sig) {
    char msg[64] = "bpg: fatal signal ";
    size_t k = strlen(msg);
    if (sig >= 10) msg[k++] = (char)('0' + sig / 10);
    msg[k++] = (char)('0' + sig % 10);
    memcpy(msg + k, ", native backtrace:\n", 21);
    (void)!write(2, msg, strlen(msg));
    void *bt[64];
    const int n = backtrace(bt, 64);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
static void install_crash_report() {
    void *warm[2];
    (void)backtrace(warm, 2);   // loads the unwinder now, not inside the handler
    for (int sig : {SIGSEGV, SIGBUS, SIGILL, SIGFPE}) {
        struct sigaction cur;
        if (sigaction(sig, nullptr, &cur) != 0 || (cur.sa_flags & SA_SIGINFO) || cur.sa_handler != SIG_DFL) continue;
        struct sigaction sa;
        memset(&sa, 0, sizeof(sa));
        sa.sa_handler = crash_report;
        sigemptyset(&sa.sa_mask);
        sa.sa_flags = SA_RESETHAND | SA_NODEFER;
        sigaction(sig, &sa, nullptr);
    }
}
static std::mutex g_ctx_mu;
DeviceContext &DeviceContext::get(int device) {
    static std::map<int, std::unique_ptr<DeviceContext>> ctxs;
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto &p = ctxs[device];
    if (!p) {
        static bool hooked = false;
        if (!hooked) {   // runs before `ctxs` and the later statics are destroyed
            hooked = true;
            std::atexit(dev::mark_process_exiting);
            install_crash_report();
        }
        p.reset(new DeviceContext());
        p->device = device;
        BPG_HIP(hipSetDevice(device));
        // fixed-base tables for B and B_blinding: T[w][j] = (j+1) 16^w P
        std::vector<PtD> tab(2 * 512);
        for (int which = 0; which < 2; which++) {
            Point base = which ? basepoint_B_blinding() : basepoint_B();
            for (int w = 0; w < 64; w++) {
                Point acc = base;
                for (int j = 0; j < 8; j++) {
                    pt_to_dev(tab[which * 512 + 8 * w + j].v, acc);
                    Point t; pt_add(t, acc, base); acc = t;
                }
                for (int k = 0; k < 4; k++) pt_dbl(base, base);
            }
        }
        BPG_HIP(hipMalloc(&p->tabB, 1024 * sizeof(PtD)));
        p->tabBb = p->tabB + 512;
        BPG_HIP(hipMemcpy(p->tabB, tab.data(), 1024 * sizeof(PtD), hipMemcpyHostToDevice));
        PtD bb; pt_to_dev(bb.v, basepoint_B_blinding());
        BPG_HIP(hipMalloc(&p->Bb, sizeof(PtD)));
        BPG_HIP(hipMemcpy(p->Bb, &bb, sizeof(PtD), hipMemcpyHostToDevice));
    }
    return *p;
}

GenSet::~GenSet() {
    if (dev::process_exiting()) return;
    if (G || H) (void)hipSetDevice(device);
    if (G) (void)hipFree(G);
    if (H) (void)hipFree(H);
    if (GH) (void)hipFree(GH);
}
const dev::NielsD *gh_table(const GenSet &gs, hipStream_t st) {
    std::lock_guard<std::mutex> lk(gs.sums_mu);
    if (gs.GH) return gs.GH;
    BPG_HIP(hipSetDevice(gs.device));
    dev::NielsD *gh = nullptr;
    PtD *tmp = nullptr;
    BPG_HIP(hipMalloc(&gh, 2 * (size_t)gs.N * sizeof(dev::NielsD)));
    if (hipMalloc(&tmp, (size_t)gs.N * sizeof(PtD)) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(gh);
        throw HipError(hipErrorOutOfMemory, "hipMalloc(G + H staging)", __FILE__, __LINE__);
    }
    // prepare_cs builds it with no stream of its own: a private one
    hipStream_t own = nullptr;
    if (!st) BPG_HIP(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
    const hipStream_t s = st ? st : own;
    launch_gen_sum(gs.G, gs.H, tmp, gs.N, s);
    const PtD *in[1] = {tmp};
    dev::NielsD *out[1] = {gh};
    launch_cached_to_niels(in, out, 1, gs.N, s);
    launch_niels_neg(gh, gh + gs.N, gs.N, s);
    BPG_HIP(hipStreamSynchronize(s));
    if (own) (void)hipStreamDestroy(own);
    (void)hipFree(tmp);
    gs.GH = gh;
    return gh;
}
FbTables::~FbTables() {
    if (dev::process_exiting()) return;
    if (G || H) (void)hipSetDevice(device);
    if (G) (void)hipFree(G);
    if (H) (void)hipFree(H);
}
CombTables::~CombTables() {
    if (dev::process_exiting()) return;
    if (tabG || tabH) (void)hipSetDevice(device);
    if (tabG) (void)hipFree(tabG);
    if (tabH) (void)hipFree(tabH);
}
bool Strategy::tables() const { return fold_tables != 0; }
bool Strategy::pairs() const { return fold_pairs != 0; }
// 512 since round 6 (4096 before): at 2^20 the level-8 triple fold (4096 ->
// 512 lanes) replaces three tail rounds' 4-segment MSMs over 4096 lanes, and
// the tail's nine rounds run over 512: ~170 K fewer MSM points per proof, a
// few percent of the VALU work on a power-limited chip, +1.0% in three
// alternating runs (profiles/r06t_ab_tail512.txt; 2048 and 8192 were noise
// in rounds 2 and 4)
uint32_t Strategy::tail() const { return ipp_tail >= 0 ? (uint32_t)ipp_tail : 512u; }
int Strategy::group() const { return fold_pairs == 0 ? 1 : fold_pairs == 1 ? 2 : 3; }

static std::mutex g_cache_mu;
static std::string g_cache_dir;
static bool g_cache_dir_set = false;
void set_gens_cache_dir(const char *dir) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_cache_dir = dir ? dir : "";
    g_cache_dir_set = true;
}
static std::string gens_cache_dir() {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    if (g_cache_dir_set) return g_cache_dir;
    const char *e = getenv("BPG_GENS_CACHE");
    return e ? e : "";
}

// The 64-byte uniform strings of generator chain `tag` (G or H):
// SHAKE256("GeneratorsChain" || tag || u32le(0)) squeezed 64 bytes per point
// (generators.rs GeneratorsChain; one serial XOF per chain).
static void gens_uniform(char tag, uint8_t *out, size_t points) {
    uint8_t label[20];
    memcpy(label, "GeneratorsChain", 15);
    label[15] = (uint8_t)tag;
    label[16] = label[17] = label[18] = label[19] = 0;
    Shake256 xof;
    xof.init_absorb(label, 20);
    xof.squeeze(out, points * 64);
}

// On-disk cache file of a full set: magic, N, a checksum, then G and H as
// device affine Niels points. Validated on load by the checksum and by
// recomputing the first points of both chains on the host (a prefix of the
// XOF, so the check costs microseconds, not the chain).
static const uint64_t GENS_MAGIC = 0x32736e6567677062ULL;   // "bpggens2"
static std::string gens_cache_path(const std::string &dir, uint32_t N) {
    return dir + "/bpg_gens_" + std::to_string(N) + ".bin";
}
static uint64_t gens_checksum(const std::vector<dev::NielsD> &G, const std::vector<dev::NielsD> &H) {
    uint64_t h = 0x9e3779b97f4a7c15ULL;
    for (const std::vector<dev::NielsD> *v : {&G, &H}) {
        const uint64_t *w = reinterpret_cast<const uint64_t *>(v->data());
        const size_t nw = v->size() * sizeof(dev::NielsD) / 8;
        for (size_t i = 0; i < nw; i++) h = (h ^ w[i]) * 0x100000001b3ULL + (h >> 29);
    }
    return h;
}
static bool gens_cache_check(const std::vector<dev::NielsD> &G, const std::vector<dev::NielsD> &H) {
    const uint32_t K = (uint32_t)std::min<size_t>(4, G.size());
    uint8_t uni[64 * 4];
    for (int which = 0; which < 2; which++) {
        gens_uniform(which ? 'H' : 'G', uni, K);
        for (uint32_t k = 0; k < K; k++) {
            Point p;
            ristretto_from_uniform(p, uni + 64 * k);
            dev::NielsD want;
            pt_to_dev_niels(want.v, p);
            if (memcmp(&want, which ? &H[k] : &G[k], sizeof(want))) return false;
        }
    }
    return true;
}

// A cache file is read only if nobody but this user could have written it:
// a regular file owned by the effective uid, not writable by group or others,
// in a directory owned by this uid (or root) that group and others cannot
// write either. The verifier never uses a loaded set (DeviceContext::gens).
static bool gens_cache_trusted(const std::string &dir, int fd) {
    struct stat fs, ds;
    if (fstat(fd, &fs) != 0 || stat(dir.c_str(), &ds) != 0) return false;
    const uid_t me = geteuid();
    if (!S_ISREG(fs.st_mode) || fs.st_uid != me || (fs.st_mode & (S_IWGRP | S_IWOTH))) return false;
    if (!S_ISDIR(ds.st_mode) || (ds.st_uid != me && ds.st_uid != 0) || (ds.st_mode & (S_IWGRP | S_IWOTH))) return false;
    return true;
}

std::shared_ptr<const GenSet> DeviceContext::gens(uint32_t N, uint32_t rank, uint32_t world, bool verifier) {
    if (world < 1 || rank >= world || N % world) throw std::runtime_error("bad generator slice");
    std::lock_guard<std::mutex> lk(mu);
    BPG_HIP(hipSetDevice(device));
    // a set loaded from the on-disk cache is checked only by a checksum and
    // its first points: the verifier's soundness must not rest on a file, so
    // a verifier request re-derives it (once) from the SHAKE256 chains
    if (!full || full->N < N || (verifier && gens_from_cache)) {
        const double t0 = now_ms();
        const uint32_t cap = std::max<uint32_t>(std::max<uint32_t>(N, 64), full ? full->N : 0);
        std::shared_ptr<GenSet> gs(new GenSet());
        gs->device = device;
        gs->N = cap;
        BPG_HIP(hipMalloc(&gs->G, 2 * (size_t)cap * sizeof(dev::NielsD)));
        BPG_HIP(hipMalloc(&gs->H, 2 * (size_t)cap * sizeof(dev::NielsD)));
        const std::string dir = verifier ? std::string() : gens_cache_dir();
        bool loaded = false;
        if (!dir.empty()) {
            FILE *f = fopen(gens_cache_path(dir, cap).c_str(), "rb");
            if (f && !gens_cache_trusted(dir, fileno(f))) {
                fclose(f);
                f = nullptr;
            }
            if (f) {
                uint64_t hdr[3] = {0, 0, 0};
                std::vector<dev::NielsD> hG(cap), hH(cap);
                if (fread(hdr, 8, 3, f) == 3 && hdr[0] == GENS_MAGIC && hdr[1] == cap &&
                    fread(hG.data(), sizeof(dev::NielsD), cap, f) == cap &&
                    fread(hH.data(), sizeof(dev::NielsD), cap, f) == cap && hdr[2] == gens_checksum(hG, hH) &&
                    gens_cache_check(hG, hH)) {
                    BPG_HIP(hipMemcpy(gs->G, hG.data(), (size_t)cap * sizeof(dev::NielsD), hipMemcpyHostToDevice));
                    BPG_HIP(hipMemcpy(gs->H, hH.data(), (size_t)cap * sizeof(dev::NielsD), hipMemcpyHostToDevice));
                    loaded = true;
                }
                fclose(f);
            }
        }
        if (!loaded) {
            // host SHAKE chains, Elligator x2 + add on the device
            std::vector<uint8_t> uni((size_t)cap * 64);
            uint8_t *duni = nullptr;
            BPG_HIP(hipMalloc(&duni, uni.size()));
            for (int which = 0; which < 2; which++) {
                gens_uniform(which ? 'H' : 'G', uni.data(), cap);
                BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
                launch_gens_map(duni, which ? gs->H : gs->G, cap, 0);
            }
            BPG_HIP(hipDeviceSynchronize());
            (void)hipFree(duni);
            const std::string wdir = gens_cache_dir();
            if (!wdir.empty()) {   // write-then-rename: concurrent processes never read a partial file
                std::vector<dev::NielsD> hG(cap), hH(cap);
                BPG_HIP(hipMemcpy(hG.data(), gs->G, (size_t)cap * sizeof(dev::NielsD), hipMemcpyDeviceToHost));
                BPG_HIP(hipMemcpy(hH.data(), gs->H, (size_t)cap * sizeof(dev::NielsD), hipMemcpyDeviceToHost));
                const std::string path = gens_cache_path(wdir, cap);
                const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
                const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL, 0644);
                if (FILE *f = fd >= 0 ? fdopen(fd, "wb") : nullptr) {
                    const uint64_t hdr[3] = {GENS_MAGIC, cap, gens_checksum(hG, hH)};
                    bool ok = fwrite(hdr, 8, 3, f) == 3 && fwrite(hG.data(), sizeof(dev::NielsD), cap, f) == cap &&
                              fwrite(hH.data(), sizeof(dev::NielsD), cap, f) == cap;
                    ok = (fclose(f) == 0) && ok;
                    if (!ok || rename(tmp.c_str(), path.c_str()) != 0) remove(tmp.c_str());
                }
            }
        }
        launch_niels_neg(gs->G, gs->G + cap, cap, 0);
        launch_niels_neg(gs->H, gs->H + cap, cap, 0);
        BPG_HIP(hipDeviceSynchronize());
        if (full && gens_from_cache) {   // slices / tables of the loaded set: rebuilt from the derived one
            slices.clear();
            combs.clear();
        }
        full = gs;
        gens_from_cache = loaded;
        gens_ms += now_ms() - t0;
    }
    if (world == 1) return full;
    auto key = std::make_tuple(N, rank, world);
    auto it = slices.find(key);
    if (it != slices.end()) return it->second;
    std::shared_ptr<GenSet> sl(new GenSet());
    sl->device = device;
    sl->N = N / world;
    sl->rank = rank;
    sl->world = world;
    BPG_HIP(hipMalloc(&sl->G, 2 * (size_t)sl->N * sizeof(dev::NielsD)));
    BPG_HIP(hipMalloc(&sl->H, 2 * (size_t)sl->N * sizeof(dev::NielsD)));
    launch_gather_niels(full->G, sl->N, world, rank, sl->G, 0);
    launch_gather_niels(full->H, sl->N, world, rank, sl->H, 0);
    launch_niels_neg(sl->G, sl->G + sl->N, sl->N, 0);
    launch_niels_neg(sl->H, sl->H + sl->N, sl->N, 0);
    BPG_HIP(hipDeviceSynchronize());
    slices[key] = sl;
    return sl;
}

std::shared_ptr<CombTables> DeviceContext::comb(const std::shared_ptr<const GenSet> &gs, uint32_t N) {
    if (N < 8 || !gs || gs->N < N) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(N, gs->rank, gs->world);
    auto it = combs.find(key);
    if (it != combs.end()) return it->second;
    const double t0 = now_ms();
    const uint32_t h1 = N / 4, ntab = 3 * h1;
    const size_t bytes = (size_t)ntab * COMB_WIN * COMB_ENT * 96;   // per vector
    BPG_HIP(hipSetDevice(device));
    size_t free_b = 0, total_b = 0;
    BPG_HIP(hipMemGetInfo(&free_b, &total_b));
    const size_t reserve = std::max<size_t>((size_t)32 << 30, total_b / 8);   // per-thread workspaces
    if (2 * bytes + reserve > free_b) {
        // evict tables of other sizes that no proof is using
        for (auto e = combs.begin(); e != combs.end();) {
            if (e->second.use_count() == 1) e = combs.erase(e);
            else ++e;
        }
        BPG_HIP(hipMemGetInfo(&free_b, &total_b));
        if (2 * bytes + reserve > free_b) return nullptr;
    }
    std::shared_ptr<CombTables> t(new CombTables());
    t->device = device;
    t->N = N;
    t->bytes = 2 * bytes;
    if (hipMalloc(&t->tabG, bytes) != hipSuccess || hipMalloc(&t->tabH, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    comb_alloc_ms += now_ms() - t0;
    launch_comb_build(gs->G, h1, ntab, t->tabG, 0);
    launch_comb_build(gs->H, h1, ntab, t->tabH, 0);
    BPG_HIP(hipDeviceSynchronize());
    combs[key] = t;
    comb_ms += now_ms() - t0;
    return t;
}

std::shared_ptr<FbTables> DeviceContext::fb(const std::shared_ptr<const GenSet> &gs, uint32_t N) {
    if (!gs || gs->world != 1 || N < 2 || N > (1u << 20) || gs->N < N) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto it = fbs.find(N);
    if (it != fbs.end()) return it->second;
    const size_t bytes = (size_t)dev::FB_W * 2 * N * sizeof(dev::NielsD);   // per vector
    BPG_HIP(hipSetDevice(device));
    size_t free_b = 0, total_b = 0;
    BPG_HIP(hipMemGetInfo(&free_b, &total_b));
    if (2 * bytes + std::max<size_t>((size_t)8 << 30, total_b / 32) > free_b) return nullptr;
    std::shared_ptr<FbTables> t(new FbTables());
    t->device = device;
    t->N = N;
    t->bytes = 2 * bytes;
    if (hipMalloc(&t->G, bytes) != hipSuccess || hipMalloc(&t->H, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    launch_fb_build(gs->G, N, t->G, 0);
    launch_fb_build(gs->H, N, t->H, 0);
    BPG_HIP(hipDeviceSynchronize());
    fbs[N] = t;
    return t;
}

// ---------------------------------------------------------- instrumentation
static std::atomic<bool> g_prof(false);
static std::mutex g_prof_mu;
static std::map<std::string, KernelStat> g_prof_stats;
struct PendingEvent { const char *name; hipEvent_t a, b; double bytes, femul; };
int set_kernel_profiling(bool on) { g_prof = on; return 0; }
bool get_kernel_stat(const char *name, KernelStat &out) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    auto it = g_prof_stats.find(name);
    if (it == g_prof_stats.end()) return false;
    out = it->second;
    return true;
}
void reset_kernel_stats() { std::lock_guard<std::mutex> lk(g_prof_mu); g_prof_stats.clear(); }

// ---------------------------------------------------------------- workspace
// Per-proof device buffers of the prover: a workspace drives up to
// MAX_LOCKSTEP proofs of one circuit in lockstep (gpu_prove_lockstep).
static const size_t ROWS_HALF = 1024;   // pinned MSM row buffer: commitments [0, 1024), IPP L/R [1024, 2048)
struct ProofBufs {
    DBuf wide, sL, sR, w, wloc, l1, r0, r1, r3, ypm, yipm, zlo, zhi, ylo, yhi, tabs, a, b, mscal, partial, Gp[2], Hp[2],
        small, wG, wH, wconv, f3tab, eqsc, ytab;
    ScD *small_host = nullptr;   // pinned, 4096 scalars
    ScD *small_view = nullptr;   // its device view (kernels write c_L, c_R there)
    dev::ArgStage fold_stage, comb_stage, fold2_stage, fold3_stage;
    ~ProofBufs() {
        for (dev::ArgStage *a : {&fold_stage, &comb_stage, &fold2_stage, &fold3_stage}) {
            if (a->dev) (void)hipFree(a->dev);
            if (a->host) (void)hipHostFree(a->host);
            if (a->copied) (void)hipEventDestroy(a->copied);
        }
        if (small_host) (void)hipHostFree(small_host);
        DBuf *bufs[] = {&wide, &sL, &sR, &w, &wloc, &l1, &r0, &r1, &r3, &ypm, &yipm, &zlo, &zhi, &ylo, &yhi, &tabs,
                        &a, &b, &mscal, &partial, &Gp[0], &Gp[1], &Hp[0], &Hp[1], &small, &wG, &wH, &wconv, &f3tab,
                        &eqsc, &ytab};
        for (DBuf *d : bufs) if (d->p) (void)hipFree(d->p);
    }
};
struct Workspace : dev::ProfSink {
    ProofBufs pb[MAX_LOCKSTEP];      // the prover's per-proof buffers (the verifier uses the ones below)
    int device = 0;
    hipStream_t st = nullptr;
    std::unique_ptr<MsmEngine> msm;
    DBuf w, yipm, zlo, zhi, ylo, yhi, tabs, mscal, partial, small, gh, ynwR, pts, okflag, ghacc, vcomp, ones, vtab;
    PtD *rows_host = nullptr;        // pinned, 2 x ROWS_HALF window rows
    PtD *rows_view = nullptr;        // its device view (the row kernels write there)
    uint8_t *s_host = nullptr;       // pinned staging for s_L | s_R
    size_t s_host_cap = 0;
    ScD *small_host = nullptr;       // pinned small transfers (4096 scalars)
    hipEvent_t done_ev = nullptr;    // blocking-sync event: waiting threads sleep instead of spinning
    hipEvent_t stage_wiped = nullptr;   // s_host zeroed after its last proof
    void sync() {
        BPG_HIP(hipEventRecord(done_ev, st));
        event_wait(done_ev);
    }
    ~Workspace() {
        if (dev::process_exiting()) return;
        for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
        if (done_ev) (void)hipEventDestroy(done_ev);
        if (stage_wiped) (void)hipEventDestroy(stage_wiped);
        if (rows_host) (void)hipHostFree(rows_host);
        if (s_host) (void)hipHostFree(s_host);
        if (small_host) (void)hipHostFree(small_host);
        DBuf *bufs[] = {&w, &yipm, &zlo, &zhi, &ylo, &yhi, &tabs, &mscal, &partial, &small, &gh, &ynwR, &pts, &okflag,
                        &ghacc, &vcomp, &ones, &vtab};
        for (DBuf *d : bufs) if (d->p) (void)hipFree(d->p);
        msm.reset();
        if (st) (void)hipStreamDestroy(st);
    }
    std::vector<PendingEvent> pend;
    // timing events, created once per workspace and reused after every flush
    // (no hipEventCreate / hipEventDestroy per bracketed launch)
    std::vector<hipEvent_t> ev_pool;
    size_t ev_next = 0;
    hipEvent_t take_event() {
        if (ev_next == ev_pool.size()) {
            hipEvent_t e;
            BPG_HIP(hipEventCreate(&e));
            ev_pool.push_back(e);
        }
        return ev_pool[ev_next++];
    }
    // bracket the launches issued between begin() and end() on `st`
    int prof_begin(const char *name, double bytes, double femul = 0) {
        if (!g_prof) return -1;
        PendingEvent e{name, take_event(), take_event(), bytes, femul};
        BPG_HIP(hipEventRecord(e.a, st));
        pend.push_back(e);
        return (int)pend.size() - 1;
    }
    void prof_end(int h) { if (h >= 0) BPG_HIP(hipEventRecord(pend[h].b, st)); }
    int begin(const char *name, double bytes, double femul) override { return prof_begin(name, bytes, femul); }
    void end(int h) override { prof_end(h); }
    void prof_flush() {   // call after the stream is synchronised
        if (pend.empty()) return;
        std::lock_guard<std::mutex> lk(g_prof_mu);
        for (auto &e : pend) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
                KernelStat &k = g_prof_stats[e.name];
                k.launches++;
                k.total_ms += ms;
                k.alg_bytes += e.bytes;
                k.femul += e.femul;
            }
        }
        pend.clear();
        ev_next = 0;
    }
    void stage(size_t bytes) {
        if (bytes <= s_host_cap) return;
        if (s_host) BPG_HIP(hipHostFree(s_host));
        s_host_cap = bytes + bytes / 4 + 4096;
        BPG_HIP(hipHostMalloc((void **)&s_host, s_host_cap, hipHostMallocDefault));
    }
};

// Thread-owned device resources (workspaces, producer stages) and thread exit.
// A thread's exit never frees them: it parks them in a process-wide list
// (heap-allocated and never destroyed), and the next thread that needs one
// for the device takes it over. Freeing happens only in explicit calls
// (bpg_ctx_trim) while the process is live.
//
// Why (round-4 SIGSEGV, profiles/r04u_gpu_tests_exit_segv.log): a Python
// thread's join() returns when its interpreter state is released, BEFORE the
// OS thread runs its C++ thread_local destructors. The robustness worker
// joined its two proving threads, printed its results and exited while those
// threads were still in ~Workspace (hipFree of GBs, hipHostFree,
// hipStreamDestroy): glibc's exit() ran the HIP runtime's teardown
// concurrently with them, and the process died with SIGSEGV after its
// output. The exiting flag did not help: it is set by an atexit handler,
// i.e. after the race has begun (and the exiting thread's own TLS
// destructors run before atexit handlers anyway). With nothing done in
// thread exit but a list insertion under a mutex there is no race left.
template <class T>
struct Parked {
    std::mutex mu;
    std::multimap<int, T *> items;   // device -> resource
    uint64_t parked_total = 0;       // thread exits that parked one (diagnostics)
    void put(int device, T *t) {
        std::lock_guard<std::mutex> lk(mu);
        items.emplace(device, t);
        parked_total++;
    }
    T *take(int device) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = items.find(device);
        if (it == items.end()) return nullptr;
        T *t = it->second;
        items.erase(it);
        return t;
    }
    std::vector<T *> take_all(int device) {
        std::lock_guard<std::mutex> lk(mu);
        std::vector<T *> out;
        auto r = items.equal_range(device);
        for (auto it = r.first; it != r.second; ++it) out.push_back(it->second);
        items.erase(r.first, r.second);
        return out;
    }
};
template <class T>
static Parked<T> &parked() {
    static Parked<T> *p = new Parked<T>();   // never destroyed: outlives every thread
    return *p;
}
template <class T>
struct ThreadOwned {   // one thread's resources by device; parked on thread exit
    std::map<int, T *> m;
    ~ThreadOwned() {
        for (auto &e : m)
            if (e.second) parked<T>().put(e.first, e.second);
    }
};
static std::map<int, Workspace *> &thread_workspaces() {
    static thread_local ThreadOwned<Workspace> wss;
    return wss.m;
}
ParkStats park_stats() {
    ParkStats s;
    {
        Parked<Workspace> &p = parked<Workspace>();
        std::lock_guard<std::mutex> lk(p.mu);
        s.workspaces_parked = p.items.size();
        s.workspace_parks = p.parked_total;
    }
    {
        Parked<ProducerStage> &p = parked<ProducerStage>();
        std::lock_guard<std::mutex> lk(p.mu);
        s.stages_parked = p.items.size();
        s.stage_parks = p.parked_total;
    }
    return s;
}
Workspace &thread_workspace(int device) {
    auto &p = thread_workspaces()[device];
    if (!p && (p = parked<Workspace>().take(device))) {   // a finished thread's workspace
        BPG_HIP(hipSetDevice(device));
        BPG_HIP(hipStreamSynchronize(p->st));
        p->pend.clear();   // timing brackets its last owner never flushed
        p->ev_next = 0;
    }
    if (!p) {
        BPG_HIP(hipSetDevice(device));
        p = new Workspace();
        p->device = device;
        BPG_HIP(hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking));
        BPG_HIP(hipEventCreateWithFlags(&p->done_ev, hipEventBlockingSync | hipEventDisableTiming));
        p->msm.reset(new MsmEngine(p->st));
        BPG_HIP(hipHostMalloc((void **)&p->rows_host, 2 * ROWS_HALF * sizeof(PtD), hipHostMallocDefault));
        BPG_HIP(hipHostGetDevicePointer((void **)&p->rows_view, p->rows_host, 0));
        BPG_HIP(hipHostMalloc((void **)&p->small_host, 4096 * sizeof(ScD), hipHostMallocDefault));
    }
    dev::set_prof_sink(p);   // this thread's launches record on its own stream
    BPG_HIP(hipSetDevice(device));
    return *p;
}
static size_t workspace_bytes(const Workspace &ws);
size_t release_thread_workspace(int device) {
    auto &m = thread_workspaces();
    auto it = m.find(device);
    size_t b = 0;
    BPG_HIP(hipSetDevice(device));
    if (it != m.end() && it->second) {
        b += workspace_bytes(*it->second);
        BPG_HIP(hipStreamSynchronize(it->second->st));
        dev::set_prof_sink(nullptr);
        delete it->second;
    }
    if (it != m.end()) m.erase(it);
    // and the workspaces finished threads left behind
    for (Workspace *w : parked<Workspace>().take_all(device)) {
        b += workspace_bytes(*w);
        BPG_HIP(hipStreamSynchronize(w->st));
        delete w;
    }
    return b;
}
size_t thread_workspace_bytes(int device) {
    auto &m = thread_workspaces();
    auto it = m.find(device);
    if (it == m.end() || !it->second) return 0;
    return workspace_bytes(*it->second);
}
static size_t workspace_bytes(const Workspace &ws) {
    size_t b = ws.msm ? ws.msm->bytes() : 0;
    for (const DBuf *d : {&ws.w, &ws.yipm, &ws.zlo, &ws.zhi, &ws.ylo, &ws.yhi, &ws.tabs, &ws.mscal, &ws.partial,
                          &ws.small, &ws.gh, &ws.ynwR, &ws.pts, &ws.okflag, &ws.ghacc, &ws.vcomp, &ws.ones, &ws.vtab})
        b += d->cap;
    for (const ProofBufs &B : ws.pb)
        for (const DBuf *d : {&B.wide, &B.sL, &B.sR, &B.w, &B.wloc, &B.l1, &B.r0, &B.r1, &B.r3, &B.ypm, &B.yipm,
                              &B.zlo, &B.zhi, &B.ylo, &B.yhi, &B.tabs, &B.a, &B.b, &B.mscal, &B.partial, &B.Gp[0],
                              &B.Gp[1], &B.Hp[0], &B.Hp[1], &B.small, &B.wG, &B.wH, &B.wconv, &B.f3tab, &B.eqsc,
                              &B.ytab})
            b += d->cap;
    return b;
}
static size_t grown(size_t need) { return need + need / 4 + 256; }   // DBuf::grow's allocation
// What gpu_prove_lockstep grows a workspace to for P proofs of `cs` (the
// per-proof vectors, the IPP point buffers and the largest fold3 table, and
// the MSM scratch of the largest job: rounds 0 and 1 cover 2 Nl points per
// proof, the commitments 5 nl per proof in their own jobs).
size_t consumer_bytes_estimate(const PreparedCS &cs, int P) {
    const size_t S = sizeof(ScD), nl = cs.nl, Nl = cs.Nl;
    // the first triple fold's table: level 2 -> 5 (Nl / 32 output lanes)
    // after the comb pass, but level 0 -> 3 (Nl / 8, four times the table:
    // 1.2 GB per 2^20 proof) when this device holds no comb tables for the
    // circuit (e.g. next to a foreign allocation). Round 5's estimate always
    // assumed the former, so a statements call without tables admitted
    // device threads that ran out of HBM in their first fold
    bool comb = false;
    if (cs.strat.tables()) {
        DeviceContext &c = DeviceContext::get(cs.device);
        std::lock_guard<std::mutex> lk(c.mu);
        comb = c.combs.count(std::make_tuple(Nl, cs.rank, cs.world)) != 0;
    }
    const size_t hq = std::max<size_t>(comb ? Nl / 32 : Nl / 8, 64);
    const size_t per_proof = 6 * grown(nl * S + 64) + grown(cs.ncol * S + 64) + 4 * grown(Nl * S + 64) +
                             grown((2 * Nl + 2) * S + 64) + 4 * grown(Nl / 2 * sizeof(PtD)) +
                             grown(ipp_fold3_table_bytes((uint32_t)hq, COMB_MAXRANGE)) +
                             grown(2 * nl * S + 64) + ((size_t)8 << 20);
    // generator_range_sum's unit scalars (round 0's padding lanes, once per
    // generator set; at most Nl / 2 of them) in the workspace
    const size_t ones = grown(Nl / 2 * S + 64);
    const size_t msm = std::max(MsmEngine::job_bytes(2 * (uint64_t)Nl * P, 2 * P, MSM_NIELS),
                                MsmEngine::job_bytes(5 * (uint64_t)nl, 3, MSM_NIELS));
    return (size_t)P * per_proof + ones + msm;
}
// Verifier::verify of a circuit of cs's size on a fresh workspace: the
// mega-MSM over 2N generators and the flattened / y^-i / g-h vectors.
size_t verifier_bytes_estimate(const PreparedCS &cs) {
    const size_t S = sizeof(ScD), N = cs.N;
    return MsmEngine::job_bytes(2 * (uint64_t)N + 64, 1, MSM_NIELS) + grown(cs.ncol * S + 64) +
           2 * grown(N * S) + grown(2 * N * S + 64) + grown((size_t)cs.n * S + 64) + ((size_t)64 << 20);
}

ProveTimings &last_timings() { static thread_local ProveTimings t; return t; }

template <class T>
static T *as(DBuf &b) { return reinterpret_cast<T *>(b.p); }

// ------------------------------------------------------------------ prepare
std::vector<uint8_t *> PreparedCS::slots(size_t count, size_t bytes, bool host) const {
    std::lock_guard<std::mutex> lk(slot_mu);
    std::vector<uint8_t *> &bufs = host ? host_slot_bufs : slot_bufs;
    size_t &cap = host ? host_slot_bytes : slot_bytes;
    if (bytes > cap) {
        for (uint8_t *b : bufs) (void)(host ? hipHostFree(b) : hipFree(b));
        bufs.clear();
        cap = bytes;
    }
    BPG_HIP(hipSetDevice(device));
    while (bufs.size() < count) {
        uint8_t *b = nullptr;
        if (host) BPG_HIP(hipHostMalloc((void **)&b, cap, hipHostMallocDefault));
        else BPG_HIP(hipMalloc((void **)&b, cap));
        bufs.push_back(b);
    }
    return std::vector<uint8_t *>(bufs.begin(), bufs.begin() + count);
}

PreparedCS::~PreparedCS() {
    for (uint8_t *b : slot_bufs) (void)hipFree(b);
    // pinned RNG slots held raw blinding draws: zeroed before they go back
    for (uint8_t *b : host_slot_bufs) {
        memset(b, 0, host_slot_bytes);
        (void)hipHostFree(b);
    }
    DBuf *bufs[] = {&aL, &aR, &aO, &vb_dev, &col_ptr, &col_row, &col_coeff, &short_cols, &long_cols, &eqI, &dfI};
    for (DBuf *d : bufs) if (d->p) (void)hipFree(d->p);
}

std::unique_ptr<PreparedCS> prepare_cs(const bpg_r1cs_view *cs, int device, const Strategy &strat, uint32_t rank,
                                       uint32_t world, std::unique_ptr<PreparedCS> reuse) {
    // a recycled PreparedCS keeps its device arrays and RNG slots (grow-only):
    // no hipMalloc / hipFree per statement (a hipFree synchronises the device)
    std::unique_ptr<PreparedCS> P = reuse && reuse->device == device ? std::move(reuse)
                                                                      : std::unique_ptr<PreparedCS>(new PreparedCS());
    P->huge_cols.clear();
    BPG_HIP(hipSetDevice(device));
    P->device = device;
    P->n = cs->n; P->m = cs->m; P->q = cs->q;
    P->N = next_pow2(cs->n);
    P->lgN = lg2u(P->N);
    P->prover = cs->a_L != nullptr;
    P->strat = strat;
    const uint32_t n = cs->n, m = cs->m;
    if (n >= (1u << 28) || m >= (1u << 28)) throw std::runtime_error("circuit too large");
    if (world < 1 || (world & (world - 1)) || rank >= world) throw std::runtime_error("bad shard (world must be a power of two)");
    // the sharded prover keeps at least 8 lanes per rank (the IPP tail needs
    // a materialised level before the local rounds end)
    if (world > 1 && (!P->prover || P->N < 8 * world || n < world))
        throw std::runtime_error("circuit too small to shard over this many ranks");
    P->rank = rank; P->world = world;
    P->Nl = P->N / world;
    P->nl = n > rank ? (n - rank + world - 1) / world : 0;
    // constraint matrix, transposed to columns [L | R | O | V | One]
    const uint32_t ncol = 3 * n + m + 1;
    P->ncol = ncol;
    // transposition scratch, kept per thread across calls (c_prove prepares
    // every statement: ~170 MB at 2^20, otherwise reallocated and page-faulted
    // in each time)
    static thread_local std::vector<uint32_t> cnt, pos, rows;
    static thread_local std::vector<ScD> coef;
    cnt.assign(ncol + 1, 0);
    const uint32_t nnz = cs->row_ptr[cs->q];
    auto colof = [&](uint32_t var) -> uint32_t {
        uint32_t kind = BPG_VAR_KIND(var), idx = BPG_VAR_INDEX(var);
        switch (kind) {
            case BPG_VAR_ONE: return 3 * n + m;
            case BPG_VAR_L: if (idx >= n) throw std::runtime_error("bad variable"); return idx;
            case BPG_VAR_R: if (idx >= n) throw std::runtime_error("bad variable"); return n + idx;
            case BPG_VAR_O: if (idx >= n) throw std::runtime_error("bad variable"); return 2 * n + idx;
            case BPG_VAR_V: if (idx >= m) throw std::runtime_error("bad variable"); return 3 * n + idx;
        }
        throw std::runtime_error("bad variable kind");
    };
    for (uint32_t k = 0; k < nnz; k++) cnt[colof(cs->term_var[k]) + 1]++;
    for (uint32_t c = 0; c < ncol; c++) cnt[c + 1] += cnt[c];
    pos.assign(cnt.begin(), cnt.end() - 1);
    rows.resize(nnz ? nnz : 1);
    coef.resize(nnz ? nnz : 1);
    for (uint32_t q = 0; q < cs->q; q++)
        for (uint32_t k = cs->row_ptr[q]; k < cs->row_ptr[q + 1]; k++) {
            uint32_t c = colof(cs->term_var[k]);
            uint32_t at = pos[c]++;
            rows[at] = q;
            coef[at] = to_dev(Scalar::reduce(cs->term_coeff + 32 * (size_t)k));
        }
    // length classes: <= 16 terms -> one thread, <= 4096 -> one wave, larger
    // (the constant column, some commitments) -> grid-wide reduction
    std::vector<uint32_t> sc_, lc_;
    for (uint32_t c = 0; c < ncol; c++) {
        uint32_t len = cnt[c + 1] - cnt[c];
        if (P->prover && c == ncol - 1) continue;   // prover never needs wc (Variable::One)
        if (len > 4096) P->huge_cols.push_back(c);
        else ((len > 16) ? lc_ : sc_).push_back(c);
    }
    P->col_ptr_host = cnt;
    P->nshort = (uint32_t)sc_.size(); P->nlong = (uint32_t)lc_.size();
    auto up = [&](DBuf &d, const void *src, size_t bytes) {
        d.grow_first_exact(bytes ? bytes : 4);
        if (bytes) BPG_HIP(hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice));
    };
    up(P->col_ptr, cnt.data(), cnt.size() * 4);
    up(P->col_row, rows.data(), rows.size() * 4);
    up(P->col_coeff, coef.data(), coef.size() * sizeof(ScD));
    up(P->short_cols, sc_.data(), sc_.size() * 4);
    up(P->long_cols, lc_.data(), lc_.size() * 4);
    if (P->prover) {
        // a_L, a_R, a_O: this rank's lanes i = j * world + rank
        const uint32_t nl = P->nl;
        static thread_local std::vector<ScD> tL, tmp;
        static thread_local std::vector<uint32_t> iE, iD;
        tL.resize(nl ? nl : 1);
        tmp.resize(nl ? nl : 1);
        const uint8_t *src[3] = {cs->a_L, cs->a_R, cs->a_O};
        DBuf *dst[3] = {&P->aL, &P->aR, &P->aO};
        P->eq_split = false;
        for (int k = 0; k < 3; k++) {
            std::vector<ScD> &t = k == 0 ? tL : tmp;
            for (uint32_t j = 0; j < nl; j++)
                t[j] = to_dev(Scalar::reduce(src[k] + 32 * ((size_t)j * world + rank)));
            up(*dst[k], t.data(), (size_t)nl * sizeof(ScD));
            if (k == 1 && world == 1) {
                // lanes with a_L == a_R: one A_I1 term on G_i + H_i
                iE.clear(); iD.clear();
                iE.reserve(nl); iD.reserve(nl);
                for (uint32_t j = 0; j < nl; j++) (!memcmp(&tL[j], &t[j], sizeof(ScD)) ? iE : iD).push_back(j);
                if (!iE.empty()) {
                    // the lanes' scalars are gathered at commit time into
                    // the proving thread's workspace (commit_a_segments):
                    // a statement in flight holds only the lane indices
                    P->eq_split = true;
                    P->nE = (uint32_t)iE.size();
                    P->nD = (uint32_t)iD.size();
                    up(P->eqI, iE.data(), iE.size() * 4);
                    up(P->dfI, iD.data(), iD.size() * 4);
                }
            }
        }
        // the witness copies (and the equal-lane lists, which derive from
        // the witness): wiped (the barrier keeps the memset of a live
        // buffer), and kept for the thread's next statement only up to 32 MB
        // each, a 2^20 circuit's (several GB across a large pool
        // otherwise). Releasing them after every statement cost the
        // statements mode's CPU workers ~45 ms of page faults and zero fills
        // per config-5 statement (prepare 123 vs 78 ms, profiles/r06zz_statements.json)
        const size_t KEEP = (size_t)32 << 20;
        for (std::vector<ScD> *t : {&tL, &tmp}) {
            memset(t->data(), 0, t->size() * sizeof(ScD));
            __asm__ __volatile__("" : : "r"(t->data()) : "memory");
            if (t->capacity() * sizeof(ScD) > KEEP) std::vector<ScD>().swap(*t);
        }
        for (std::vector<uint32_t> *t : {&iE, &iD}) {
            memset(t->data(), 0, t->size() * sizeof(uint32_t));
            __asm__ __volatile__("" : : "r"(t->data()) : "memory");
            if (t->capacity() * sizeof(uint32_t) > KEEP) std::vector<uint32_t>().swap(*t);
        }
        P->v.resize(m); P->vb.resize(m);
        std::vector<ScD> vbd(m ? m : 1);
        for (uint32_t i = 0; i < m; i++) {
            P->v[i] = Scalar::from_bits(cs->v + 32 * (size_t)i);
            // keep raw bytes of v (Scalar::from_bits may differ only in bit 255)
            memcpy(P->v[i].v, cs->v + 32 * (size_t)i, 32);
            P->vb[i] = Scalar::reduce(cs->v_blinding + 32 * (size_t)i);
            memcpy(P->vb[i].v, cs->v_blinding + 32 * (size_t)i, 32);
            vbd[i] = to_dev(P->vb[i].reduced());
        }
        up(P->vb_dev, vbd.data(), (size_t)m * sizeof(ScD));
        P->V.resize((size_t)m * 32);
        if (m) gpu_pedersen(device, P->v, P->vb, P->V.data());
        // circuit-independent, outside any timed region
        DeviceContext &ctx = DeviceContext::get(device);
        std::shared_ptr<const GenSet> gs = ctx.gens(P->N, rank, world);
        // the A_I1 split's G_i + H_i table (256 MB at 2^20, 160 MB of staging
        // while it is built) now, before any caller's HBM admission reads the
        // free memory: never allocated mid-proof
        if (P->eq_split) gh_table(*gs, nullptr);
        if (strat.fixed_base()) ctx.fb(gs, P->N);
        if (strat.tables()) ctx.comb(gs, P->Nl);
    }
    return P;
}

size_t prepared_bytes(const PreparedCS &cs) {
    size_t b = 0;
    for (const DBuf *d : {&cs.aL, &cs.aR, &cs.aO, &cs.vb_dev, &cs.col_ptr, &cs.col_row, &cs.col_coeff, &cs.short_cols,
                          &cs.long_cols, &cs.eqI, &cs.dfI})
        b += d->cap;
    std::lock_guard<std::mutex> lk(cs.slot_mu);
    return b + cs.slot_bufs.size() * cs.slot_bytes;
}

void gpu_pedersen(int device, const std::vector<Scalar> &v, const std::vector<Scalar> &vb, uint8_t *out) {
    DeviceContext &ctx = DeviceContext::get(device);
    Workspace &ws = thread_workspace(device);
    const uint32_t m = (uint32_t)v.size();
    if (!m) return;
    std::vector<ScD> h(2 * (size_t)m);
    for (uint32_t i = 0; i < m; i++) { memcpy(h[i].v, v[i].v, 32); memcpy(h[m + i].v, vb[i].v, 32); }
    ws.small.grow(2 * (size_t)m * sizeof(ScD) + (size_t)m * 32);
    ScD *d = as<ScD>(ws.small);
    BPG_HIP(hipMemcpyAsync(d, h.data(), 2 * (size_t)m * sizeof(ScD), hipMemcpyHostToDevice, ws.st));
    uint32_t *outd = reinterpret_cast<uint32_t *>(d + 2 * (size_t)m);
    launch_pedersen(d, d + m, m, ctx.tabB, ctx.tabBb, outd, ws.st);
    BPG_HIP(hipMemcpyAsync(out, outd, (size_t)m * 32, hipMemcpyDeviceToHost, ws.st));
    ws.sync();
}

// -------------------------------------------------------------- MSM helpers
static void combine_rows(Point &out, const PtD *rows, int W, int c) {
    Point acc;
    pt_from_dev(acc, rows[W - 1].v);
    for (int w = W - 2; w >= 0; w--) {
        for (int k = 0; k < c; k++) pt_dbl(acc, acc);
        Point r; pt_from_dev(r, rows[w].v);
        Point t; pt_add(t, acc, r); acc = t;
    }
    out = acc;
}

int gpu_msm(int device, const uint8_t *scalars, const uint8_t *points, uint32_t n, uint8_t out[32]) {
    DeviceContext::get(device);
    Workspace &ws = thread_workspace(device);
    ws.small.grow((size_t)n * sizeof(ScD) + 64);
    ws.pts.grow(2 * (size_t)n * sizeof(NielsD) + 64);   // points, then their negations
    ws.okflag.grow(64);
    std::vector<ScD> s(n ? n : 1);
    for (uint32_t i = 0; i < n; i++) s[i] = to_dev(Scalar::reduce(scalars + 32 * (size_t)i));
    BPG_HIP(hipMemcpyAsync(ws.small.p, s.data(), (size_t)n * sizeof(ScD), hipMemcpyHostToDevice, ws.st));
    // compressed points -> device decompress
    ws.gh.grow((size_t)n * 32 + 64);
    BPG_HIP(hipMemcpyAsync(ws.gh.p, points, (size_t)n * 32, hipMemcpyHostToDevice, ws.st));
    int one = 1;
    BPG_HIP(hipMemcpyAsync(ws.okflag.p, &one, 4, hipMemcpyHostToDevice, ws.st));
    launch_decompress(as<uint32_t>(ws.gh), as<NielsD>(ws.pts), as<int>(ws.okflag), n, ws.st);
    launch_niels_neg(as<NielsD>(ws.pts), as<NielsD>(ws.pts) + n, n, ws.st);
    int ok = 0;
    BPG_HIP(hipMemcpyAsync(&ok, ws.okflag.p, 4, hipMemcpyDeviceToHost, ws.st));
    MsmSeg seg{as<ScD>(ws.small), ws.pts.p, n, 0, (int64_t)n};
    MsmPlan p = ws.msm->enqueue(&seg, 1, 1, ws.rows_host, MSM_NIELS);
    ws.sync();
    if (!ok) return -1;
    Point r;
    combine_rows(r, ws.rows_host, p.W, p.c);
    ristretto_compress(out, r);
    return 0;
}

// Upload base^(2^b) (b < 40) in Montgomery form through the pinned slot
// `slot` of small_host; returns the device pointer (in tabs).
static ScD *upload_base2(ScD *small_host, DBuf &tabs, hipStream_t st, int slot, const Scalar &base) {
    ScD *h = small_host + 40 * slot;
    Scalar cur = base;
    for (int b = 0; b < 40; b++) { h[b] = mont(cur); cur = cur * cur; }
    ScD *d = as<ScD>(tabs) + 40 * slot;
    BPG_HIP(hipMemcpyAsync(d, h, 40 * sizeof(ScD), hipMemcpyHostToDevice, st));
    return d;
}
// out[i] = mont(mult * base^i), i < count, via two 1024-ary levels
static void pow_vector(ScD *small_host, DBuf &tabs, hipStream_t st, int slot, const Scalar &base, uint32_t count,
                       DBuf &lo, DBuf &hi, ScD *out, const Scalar &mult = Scalar::one()) {
    uint32_t nhi = count / 1024 + 1;
    lo.grow(1024 * sizeof(ScD));
    hi.grow((size_t)nhi * sizeof(ScD));
    ScD *b2 = upload_base2(small_host, tabs, st, slot, base);
    ScD *b2h = upload_base2(small_host, tabs, st, slot + 1, sc_pow_u64(base, 1024));
    launch_pow_table(b2, 0, 1024, as<ScD>(lo), st);
    launch_pow_table(b2h, 0, nhi, as<ScD>(hi), st);
    if (out) launch_pow_expand(as<ScD>(lo), as<ScD>(hi), count, mont(mult), out, st);
}
static void pow_vector(Workspace &ws, int slot, const Scalar &base, uint32_t count, DBuf &lo, DBuf &hi, ScD *out,
                       const Scalar &mult = Scalar::one()) {
    pow_vector(ws.small_host, ws.tabs, ws.st, slot, base, count, lo, hi, out, mult);
}

// ------------------------------------------------------------------- prove
// Transcript::new(label) + Prover::new + commit(V_i) (prove.rs:45-72 order)
static Transcript prover_transcript(const PreparedCS &cs, const uint8_t *label, size_t label_len) {
    Transcript T(label, label_len);
    T.append_message("dom-sep", (const uint8_t *)"r1cs v1", 7);
    for (uint32_t i = 0; i < cs.m; i++) T.append_point("V", cs.V.data() + 32 * (size_t)i);
    T.append_u64("m", cs.m);
    return T;
}

// Every TranscriptRng draw of Prover::prove, in program order: i, o, s
// blindings, s_L[n], s_R[n], then the t_1, t_3..t_6 blindings. The RNG is
// forked from the transcript before any challenge, so all draws can be made
// before the device work starts. Up to 8 proofs run in lockstep (Strobe8).
// The producers' host-to-device copies (95 MB per 2^20 proof, a few GB/s in
// all) go to one stream per producer thread: one stream shared by all
// producers (fewer streams than hardware queues for the consumers) measured
// 62.3 / 62.4 vs 70.8 / 69.7 M constraints/s (profiles/r03a_ab_producer_streams.txt).
static std::map<int, ProducerStage *> &thread_stages() {
    static thread_local ThreadOwned<ProducerStage> m;   // parked on thread exit (see Parked)
    return m.m;
}
size_t release_producer_stage(int device) {
    auto &m = thread_stages();
    std::vector<ProducerStage *> all = parked<ProducerStage>().take_all(device);
    auto it = m.find(device);
    if (it != m.end()) {
        if (it->second) all.push_back(it->second);
        m.erase(it);
    }
    size_t b = 0;
    BPG_HIP(hipSetDevice(device));
    for (ProducerStage *s : all) {
        BPG_HIP(hipStreamSynchronize(s->st));
        b += 2 * (size_t)8 * ProducerStage::CHUNK * 64 + s->one_cap;
        delete s;
    }
    return b;
}
ProducerStage &producer_stage(int device) {
    auto &p = thread_stages()[device];
    if (!p && (p = parked<ProducerStage>().take(device))) {
        BPG_HIP(hipSetDevice(device));
        BPG_HIP(hipStreamSynchronize(p->st));
    }
    if (!p) {
        BPG_HIP(hipSetDevice(device));
        p = new ProducerStage();
        BPG_HIP(hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking));
        for (int b = 0; b < 2; b++) {
            BPG_HIP(hipHostMalloc((void **)&p->host[b], (size_t)8 * ProducerStage::CHUNK * 64, hipHostMallocDefault));
            BPG_HIP(hipEventCreateWithFlags(&p->ev[b], hipEventBlockingSync | hipEventDisableTiming));
            BPG_HIP(hipEventRecord(p->ev[b], p->st));
            BPG_HIP(hipEventCreateWithFlags(&p->drawn[b], hipEventDisableTiming));
        }
        BPG_HIP(hipEventCreateWithFlags(&p->wiped, hipEventBlockingSync | hipEventDisableTiming));
        BPG_HIP(hipEventRecord(p->wiped, p->st));
    }
    BPG_HIP(hipSetDevice(device));
    return *p;
}
ProducerStage::~ProducerStage() {
    if (dev::process_exiting()) return;
    for (int b = 0; b < 2; b++) {
        if (host[b]) (void)hipHostFree(host[b]);
        if (ev[b]) (void)hipEventDestroy(ev[b]);
        if (drawn[b]) (void)hipEventDestroy(drawn[b]);
    }
    if (wiped) (void)hipEventDestroy(wiped);
    if (one) (void)hipHostFree(one);
    if (st) (void)hipStreamDestroy(st);
}

void rng_draw_group(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *const *entropy,
                    int count, RngBlock *const *out, bool dev_out, const DrawProgress *progress) {
    if (count < 1 || count > 8) throw std::runtime_error("rng group size");
    Transcript T = prover_transcript(cs, label, label_len);
    TranscriptRng base(T);
    for (uint32_t i = 0; i < cs.m; i++) base.rekey_with_witness_bytes("v_blinding", (const uint8_t *)cs.vb[i].v, 32);
    // one proof (the latency path): the contiguous single-state STROBE with
    // its AVX-512 permutation; several: eight states in lockstep (Strobe8)
    TranscriptRng one(base);
    Strobe8 S;
    if (count == 1) {
        one.finalize(entropy[0]);                 // TranscriptRngBuilder::finalize
    } else {
        S.from(base.s, count);
        S.meta_ad((const uint8_t *)"rng", 3);
        S.key_each(entropy, 32);
    }
    auto draw = [&](uint8_t *const *wp) {
        if (count == 1) one.draw64(wp[0]);
        else S.draw64(wp);
    };
    uint8_t tmp[8][64];
    uint8_t *tp[8];
    for (int k = 0; k < 8; k++) tp[k] = tmp[k];
    auto draw_scalars = [&](Scalar RngBlock::*field) {
        draw(tp);
        for (int k = 0; k < count; k++) out[k]->*field = Scalar::from_wide(tmp[k]);
    };
    draw_scalars(&RngBlock::i_bl);
    draw_scalars(&RngBlock::o_bl);
    draw_scalars(&RngBlock::s_bl);
    const uint64_t nd = 2 * (uint64_t)cs.n;
    if (!dev_out) {
        uint8_t *wp[8];
        for (uint64_t i = 0; i < nd; i++) {
            for (int k = 0; k < count; k++) wp[k] = out[k]->wide + 64 * i;
            for (int k = count; k < 8; k++) wp[k] = tmp[k];
            draw(wp);
        }
    } else if (count == 1) {
        // one proof: draws straight into a pinned buffer of all of them
        // (the caller's, else this thread's), copied up 2 MB at a time while
        // the next ones are drawn (nothing waits on a copy); the s_L half
        // ends a chunk, so its copy is the progress point
        ProducerStage &ps = producer_stage(cs.device);
        const uint64_t BIG = 32768;
        uint8_t *h = out[0]->stage;
        const bool own = !h;
        if (own) {
            // the previous proof's copies out of this buffer, and its wipe,
            // are complete
            BPG_HIP(hipEventSynchronize(ps.wiped));
            if (ps.one_cap < 64 * nd) {
                if (ps.one) BPG_HIP(hipHostFree(ps.one));
                ps.one = nullptr;
                BPG_HIP(hipHostMalloc((void **)&ps.one, 64 * nd, hipHostMallocDefault));
                ps.one_cap = 64 * nd;
            }
            h = ps.one;
        }
        for (int v = 0; v < 2; v++) {
            const uint64_t a = v ? nd / 2 : 0, b = v ? nd : nd / 2;
            for (uint64_t i0 = a; i0 < b; i0 += BIG) {
                const uint64_t len = std::min<uint64_t>(BIG, b - i0);
                for (uint64_t i = 0; i < len; i++) one.draw64(h + 64 * (i0 + i));
                BPG_HIP(hipMemcpyAsync(out[0]->wide + 64 * i0, h + 64 * i0, (size_t)len * 64, hipMemcpyHostToDevice,
                                       ps.st));
            }
            if (progress) {
                BPG_HIP(hipEventRecord(ps.drawn[v], ps.st));
                (*progress)(v, ps.drawn[v]);
            }
        }
        if (!progress) {
            BPG_HIP(hipEventRecord(ps.drawn[1], ps.st));
            event_wait(ps.drawn[1]);
        }
        if (own) {   // behind the copies on the same stream (no draws left in pinned memory)
            BPG_HIP(hipMemsetAsync(h, 0, (size_t)64 * nd, ps.st));
            BPG_HIP(hipEventRecord(ps.wiped, ps.st));
        }
    } else {
        // stream chunks of draws through two pinned staging buffers into
        // the blocks' device buffers on the caller's stream
        ProducerStage &ps = producer_stage(cs.device);
        const uint32_t CH = ProducerStage::CHUNK;
        uint8_t *wp[8];
        int buf = 0;
        bool left_done = false;
        for (uint64_t i0 = 0; i0 < nd; i0 += CH, buf ^= 1) {
            const uint32_t len = (uint32_t)std::min<uint64_t>(CH, nd - i0);
            event_wait(ps.ev[buf]);
            uint8_t *stg = ps.host[buf];
            for (uint32_t i = 0; i < len; i++) {
                for (int k = 0; k < 8; k++) wp[k] = stg + ((size_t)k * CH + i) * 64;
                draw(wp);
            }
            for (int k = 0; k < count; k++)
                BPG_HIP(hipMemcpyAsync(out[k]->wide + 64 * i0, stg + (size_t)k * CH * 64, (size_t)len * 64,
                                       hipMemcpyHostToDevice, ps.st));
            BPG_HIP(hipEventRecord(ps.ev[buf], ps.st));
            if (progress && !left_done && i0 + len >= nd / 2) {   // all s_L draws are on their way
                left_done = true;
                BPG_HIP(hipEventRecord(ps.drawn[0], ps.st));
                (*progress)(0, ps.drawn[0]);
            }
        }
        if (progress) {
            BPG_HIP(hipEventRecord(ps.drawn[1], ps.st));
            (*progress)(1, ps.drawn[1]);
        }
        event_wait(ps.ev[0]);
        event_wait(ps.ev[1]);
        // the staging buffers' last chunks are blinding draws: zeroed behind
        // their copies; the next group's first chunk waits on ev[] as before
        for (int b = 0; b < 2; b++) {
            BPG_HIP(hipMemsetAsync(ps.host[b], 0, (size_t)8 * CH * 64, ps.st));
            BPG_HIP(hipEventRecord(ps.ev[b], ps.st));
        }
    }
    for (int j = 0; j < 5; j++) {
        draw(tp);
        for (int k = 0; k < count; k++) out[k]->tb[j] = Scalar::from_wide(tmp[k]);
    }
}

// The same for proofs of up to 8 DIFFERENT statements (bpg_prove_statements):
// each statement's TranscriptRng runs on its own until its first draw
// (i_bl), which leaves every STROBE state at byte 64 after a permutation, so
// the remaining draws run in lockstep although the transcripts differ. Lane
// k draws o_bl, s_bl, 2 n_k wide scalars (to out[k]->wide, a device buffer)
// and the five t blindings; lanes with fewer gates write their surplus
// draws to scratch.
void rng_draw_multi(const PreparedCS *const *cs, const uint8_t *label, size_t label_len,
                    const uint8_t *const *entropy, int count, RngBlock *const *out) {
    if (count < 1 || count > 8) throw std::runtime_error("rng group size");
    std::vector<TranscriptRng> rng;
    rng.reserve(count);
    uint8_t first[64];
    const Strobe128 *st[8];
    uint64_t D[8], maxD = 0;   // draws after i_bl: o_bl, s_bl, 2n wide, 5 t blindings
    for (int k = 0; k < count; k++) {
        Transcript T = prover_transcript(*cs[k], label, label_len);
        rng.emplace_back(T);
        for (uint32_t i = 0; i < cs[k]->m; i++)
            rng.back().rekey_with_witness_bytes("v_blinding", (const uint8_t *)cs[k]->vb[i].v, 32);
        rng.back().finalize(entropy[k]);
        rng.back().fill_bytes(first, 64);
        out[k]->i_bl = Scalar::from_wide(first);
        D[k] = 2 + 2 * (uint64_t)cs[k]->n + 5;
        maxD = std::max(maxD, D[k]);
    }
    for (int k = 0; k < count; k++) st[k] = &rng[k].s;
    Strobe8 S;
    if (!S.from_each(st, count)) throw std::runtime_error("rng lockstep: states out of step");
    uint8_t tmp[8][64], junk[64];
    uint8_t *wp[8];
    ProducerStage &ps = producer_stage(cs[0]->device);
    const uint32_t CH = ProducerStage::CHUNK;
    int buf = 0;
    for (uint64_t d0 = 0; d0 < maxD; d0 += CH, buf ^= 1) {
        const uint32_t len = (uint32_t)std::min<uint64_t>(CH, maxD - d0);
        event_wait(ps.ev[buf]);
        uint8_t *stg = ps.host[buf];   // lane k's draws d0 .. d0 + len at stg + k CH 64
        for (uint32_t i = 0; i < len; i++) {
            for (int k = 0; k < 8; k++) wp[k] = k < count ? stg + ((size_t)k * CH + i) * 64 : junk;
            S.draw64(wp);
        }
        for (int k = 0; k < count; k++) {
            const uint8_t *lane = stg + (size_t)k * CH * 64;
            const uint64_t w0 = 2, w1 = 2 + 2 * (uint64_t)cs[k]->n;   // the wide draws [w0, w1)
            for (uint64_t d = d0; d < d0 + len && d < D[k]; d++) {
                const uint8_t *x = lane + (d - d0) * 64;
                if (d == 0) out[k]->o_bl = Scalar::from_wide(x);
                else if (d == 1) out[k]->s_bl = Scalar::from_wide(x);
                else if (d >= w1) out[k]->tb[d - w1] = Scalar::from_wide(x);
            }
            const uint64_t a = std::max(d0, w0), b = std::min<uint64_t>(d0 + len, w1);
            if (a < b)
                BPG_HIP(hipMemcpyAsync(out[k]->wide + 64 * (a - w0), lane + (a - d0) * 64, (size_t)(b - a) * 64,
                                       hipMemcpyHostToDevice, ps.st));
        }
        BPG_HIP(hipEventRecord(ps.ev[buf], ps.st));
    }
    event_wait(ps.ev[0]);
    event_wait(ps.ev[1]);
    (void)tmp;
}

// One proof on the calling thread (c_prove, bpg_r1cs_prove, the sharded and
// prepared single-proof paths). Its latency is the serial TranscriptRng
// chain (2n + 8 permutations) plus what the device does after it, so the
// commitment MSMs run under the chain (SURVEY §7 hard part 1): A_I1 / A_O1
// need no draw and start first, <s_L, G> starts once the s_L half of the
// draws is on the device (streamed up in chunks as it is drawn) and only
// <s_R, H> is left when the last draw is made.
static void commit_a_segments(const PreparedCS &cp, const GenSet &gs, bool split_ok, const void *G0, const void *H0,
                              int64_t gneg, uint64_t gws, hipStream_t st, DBuf &eqsc, MsmSeg *sg, int &ns);
std::vector<uint8_t> gpu_prove(const PreparedCS &cs, const uint8_t *label, size_t label_len,
                               const uint8_t entropy[32], ProveTimings *tm, const AllGather *ag) {
    if (!cs.prover) throw std::runtime_error("prepared circuit has no witness");
    DeviceContext &ctx = DeviceContext::get(cs.device);
    std::shared_ptr<const GenSet> gs = ctx.gens(cs.N, cs.rank, cs.world);
    Workspace &ws = thread_workspace(cs.device);
    double t0 = now_ms();
    const uint32_t n = cs.n, nl = cs.nl;
    ProofBufs &B = ws.pb[0];
    B.wide.grow(2 * (size_t)n * 64 + 64);
    B.sL.grow((size_t)nl * sizeof(ScD) + 64);
    B.sR.grow((size_t)nl * sizeof(ScD) + 64);
    CommitPre pre;
    std::shared_ptr<FbTables> fbt = (cs.world == 1 && cs.strat.fixed_base()) ? ctx.fb(gs, cs.N) : nullptr;
    const void *G0 = fbt ? (const void *)fbt->G : (const void *)gs->G;
    const void *H0 = fbt ? (const void *)fbt->H : (const void *)gs->H;
    // generator jobs negate in registers (gather set G and H, 256 MB, not
    // with their negated copies, 512 MB: +0.8% under the power limit,
    // profiles/r06g_ab.txt); the fixed-base tables keep their negations
    const int64_t gneg = fbt ? (int64_t)fbt->N : 0;
    const uint64_t gws = fbt ? 2 * (uint64_t)fbt->N : 0;
    PtD *rows = ws.rows_host, *rows_dev = ws.rows_view;
    if (nl) {
        MsmSeg sa[4];
        int ns = 0;
        commit_a_segments(cs, *gs, !fbt, G0, H0, gneg, gws, ws.st, B.eqsc, sa, ns);
        sa[ns++] = {as<ScD>(const_cast<DBuf &>(cs.aO)), G0, nl, 1, gneg, gws};
        for (int i = 0; i < ns; i++) sa[i].gen = true;
        int ph = ws.prof_begin("msm_commit", 3.0 * nl * (64 + 32));
        pre.A = ws.msm->enqueue(sa, ns, 2, rows + CommitPre::ROWS_A, MSM_NIELS, rows_dev + CommitPre::ROWS_A);
        ws.prof_end(ph);
    }
    DrawProgress progress = [&](int v, hipEvent_t drawn) {
        if (!nl) return;
        BPG_HIP(hipStreamWaitEvent(ws.st, drawn, 0));
        ScD *s = as<ScD>(v ? B.sR : B.sL);
        launch_wide_reduce(as<uint8_t>(B.wide) + (size_t)v * 64 * n, nl, cs.world, cs.rank, s, ws.st);
        MsmSeg seg = {s, v ? H0 : G0, nl, 0, gneg, gws};
        seg.gen = true;
        const size_t off = v ? CommitPre::ROWS_S1 : CommitPre::ROWS_S0;
        int ph = ws.prof_begin("msm_commit", 1.0 * nl * (64 + 32));
        pre.S[v] = ws.msm->enqueue(&seg, 1, 1, rows + off, MSM_NIELS, rows_dev + off);
        ws.prof_end(ph);
    };
    if (ws.stage_wiped) BPG_HIP(hipEventSynchronize(ws.stage_wiped));   // the last proof's wipe of s_host
    ws.stage(2 * (size_t)n * 64 + 64);
    RngBlock rb;
    rb.wide = as<uint8_t>(B.wide);
    rb.on_device = true;
    rb.stage = ws.s_host;
    RngBlock *rbp = &rb;
    // s_host receives this proof's s_L / s_R draws. On success it is zeroed
    // on the stream that read them, waited for by the next proof
    // before it draws; when the draw or the device part throws, this guard
    // waits for both streams and zeroes it on the host
    struct WipeOnError {
        Workspace &ws;
        int device;
        size_t bytes;
        bool armed = true;
        ~WipeOnError() {
            if (!armed) return;
            // error path only: wait for every copy that may still read the
            // buffer (the draw copies run on this thread's producer stream),
            // allocating nothing and throwing nothing here
            (void)hipSetDevice(device);
            (void)hipDeviceSynchronize();
            (void)hipGetLastError();
            memset(ws.s_host, 0, bytes);
            __asm__ __volatile__("" : : "r"(ws.s_host) : "memory");
        }
    } wipe{ws, cs.device, 2 * (size_t)n * 64};
    rng_draw_group(cs, label, label_len, &entropy, 1, &rbp, true, &progress);
    double t1 = now_ms();
    ProveTimings t;
    const RngBlock *crb = &rb;
    std::vector<uint8_t> pr = gpu_prove_lockstep(cs, label, label_len, &crb, 1, &t, ag, &pre)[0];
    if (!ws.stage_wiped) BPG_HIP(hipEventCreateWithFlags(&ws.stage_wiped, hipEventBlockingSync | hipEventDisableTiming));
    BPG_HIP(hipMemsetAsync(ws.s_host, 0, 2 * (size_t)n * 64, ws.st));
    BPG_HIP(hipEventRecord(ws.stage_wiped, ws.st));
    wipe.armed = false;
    t.rng_ms = t1 - t0;
    t.total_ms += t1 - t0;
    last_timings() = t;
    if (tm) *tm = t;
    return pr;
}

// Sharded prover exchanges: every rank's partial points or
// scalars are all-gathered and summed identically on every rank (a Ristretto
// point sum is not an RCCL reduction op, so the sum happens on the host).
static std::vector<Point> allgather_point_sums(const AllGather &ag, const Point *p, int cnt, uint32_t world) {
    std::vector<uint8_t> send(32 * (size_t)cnt), recv(32 * (size_t)cnt * world);
    for (int c = 0; c < cnt; c++) ristretto_compress(send.data() + 32 * c, p[c]);
    ag(send.data(), send.size(), recv.data());
    std::vector<Point> out(cnt);
    for (int c = 0; c < cnt; c++) {
        pt_identity(out[c]);
        for (uint32_t r = 0; r < world; r++) {
            Point q, t;
            if (!ristretto_decompress(q, recv.data() + 32 * ((size_t)r * cnt + c)))
                throw std::runtime_error("sharded prove: a rank sent an invalid point");
            pt_add(t, out[c], q);
            out[c] = t;
        }
    }
    return out;
}
static std::vector<Scalar> allgather_scalar_sums(const AllGather &ag, const Scalar *s, int cnt, uint32_t world) {
    std::vector<uint8_t> send(32 * (size_t)cnt), recv(32 * (size_t)cnt * world);
    for (int c = 0; c < cnt; c++) s[c].to_bytes(send.data() + 32 * c);
    ag(send.data(), send.size(), recv.data());
    std::vector<Scalar> out(cnt, Scalar::zero());
    for (int c = 0; c < cnt; c++)
        for (uint32_t r = 0; r < world; r++) out[c] = out[c] + Scalar::reduce(recv.data() + 32 * ((size_t)r * cnt + c));
    return out;
}

// Prover::prove (prove.rs:79) after the RNG phase for P proofs of one
// prepared circuit in lockstep on this thread's stream (P = 1: the single
// proof; the sharded prover). The proofs share the circuit, so their control
// flow (round groups, tail, lane classes) is identical and only scalars,
// transcripts and buffers differ: every MSM job covers all P proofs (one
// digit/sort/run-reduction/bucket chain of latency-bound launches for P
// proofs, 2P or 3P MSMs), the other kernels run per proof (ProofBufs).
// The IPP's c_L Q and c_R Q terms are added on the host (Q = w B, so
// c Q = (c w) B by the fixed-base table): the L/R jobs hold only generator
// segments (at most 16 per proof, 32 per job).
// Proof p's circuit is csv[p]: one prepared circuit for the proofs of a
// batch, or distinct statements of one shape (n, m, N: the IPP and every
// MSM job depend only on those; a_L/a_R/a_O, the constraint matrix and the
// commitments are each proof's own).
// A_I1's segments, <a_L, G> + <a_R, H> (MSM 0 of a commitment job): with the
// prepared split (eq_split), lanes where a_L == a_R as ONE term a_L (G_i +
// H_i) and the others as two (a quarter fewer entries when half the lanes
// are equal, as in a MiMC circuit), else the plain two segments.
static void commit_a_segments(const PreparedCS &cp, const GenSet &gs, bool split_ok, const void *G0, const void *H0,
                              int64_t gneg, uint64_t gws, hipStream_t st, DBuf &eqsc, MsmSeg *sg, int &ns) {
    const uint32_t nl = cp.nl;
    if (cp.eq_split && split_ok && cp.world == 1) {
        const dev::NielsD *GH = gh_table(gs, st);
        // the split's scalars, gathered from a_L / a_R by the prepared lane
        // indices: a_L of the equal lanes, then a_L and a_R of the others
        eqsc.grow(((size_t)cp.nE + 2 * (size_t)cp.nD) * sizeof(ScD) + 64);
        ScD *eS = as<ScD>(eqsc), *dL = eS + cp.nE, *dR = dL + cp.nD;
        launch_eq_gather(as<ScD>(const_cast<DBuf &>(cp.aL)), as<ScD>(const_cast<DBuf &>(cp.aR)),
                         as<uint32_t>(const_cast<DBuf &>(cp.eqI)), cp.nE, as<uint32_t>(const_cast<DBuf &>(cp.dfI)),
                         cp.nD, eS, st);
        if (cp.nE) sg[ns++] = {eS, GH, cp.nE, 0, gneg, 0, as<uint32_t>(const_cast<DBuf &>(cp.eqI))};
        if (cp.nD) {
            sg[ns++] = {dL, G0, cp.nD, 0, gneg, 0, as<uint32_t>(const_cast<DBuf &>(cp.dfI))};
            sg[ns++] = {dR, H0, cp.nD, 0, gneg, 0, as<uint32_t>(const_cast<DBuf &>(cp.dfI))};
        }
        return;
    }
    sg[ns++] = {as<ScD>(const_cast<DBuf &>(cp.aL)), G0, nl, 0, gneg, gws};
    sg[ns++] = {as<ScD>(const_cast<DBuf &>(cp.aR)), H0, nl, 0, gneg, gws};
}

// sum_{j in [a, b)} H_j of a generator set (one MSM with unit scalars on the
// workspace's stream, once per range; rows land in the commitment half of the
// pinned row buffer, which is free once the commitments are combined).
// Test hook (tests/test_gpu_robustness.py): with BPG_TEST_INJECT_OOM=<k> the
// first proof of the process to reach IPP round k throws hipErrorOutOfMemory
// there, once, half way through gpu_prove_lockstep, as a workspace that
// cannot grow would (the statements path's device-thread retirement).
static uint32_t inject_oom_round() {
    static const uint32_t r = [] {
        const char *e = getenv("BPG_TEST_INJECT_OOM");
        return e && *e ? (uint32_t)atoi(e) : ~0u;
    }();
    return r;
}
static void inject_oom_once() {
    static std::atomic<bool> fired(false);
    if (!fired.exchange(true)) throw HipError(hipErrorOutOfMemory, "injected (BPG_TEST_INJECT_OOM)", __FILE__, __LINE__);
}

static Point generator_range_sum(Workspace &ws, const GenSet &gs, uint32_t a, uint32_t b) {
    {
        std::lock_guard<std::mutex> lk(gs.sums_mu);
        auto it = gs.h_sums.find({a, b});
        if (it != gs.h_sums.end()) return it->second;
    }
    Point S;
    pt_identity(S);
    if (b > a) {
        const uint32_t cnt = b - a;
        ws.ones.grow((size_t)cnt * sizeof(ScD) + 64);
        launch_fill_scalars(as<ScD>(ws.ones), to_dev(Scalar::one()), cnt, ws.st);
        const MsmSeg seg = {as<ScD>(ws.ones), gs.H + a, cnt, 0, (int64_t)gs.N};
        MsmPlan pl = ws.msm->enqueue(&seg, 1, 1, ws.rows_host, MSM_NIELS);
        ws.sync();
        combine_rows(S, ws.rows_host, pl.W, pl.c);
    }
    std::lock_guard<std::mutex> lk(gs.sums_mu);
    gs.h_sums[{a, b}] = S;
    return S;
}

std::vector<std::vector<uint8_t>> gpu_prove_lockstep(const PreparedCS &cs, const uint8_t *label, size_t label_len,
                                                     const RngBlock *const *rbs, int P, ProveTimings *tms,
                                                     const AllGather *ag, const CommitPre *pre) {
    const PreparedCS *csv[MAX_LOCKSTEP];
    for (int p = 0; p < MAX_LOCKSTEP; p++) csv[p] = &cs;
    return gpu_prove_lockstep(csv, label, label_len, rbs, P, tms, ag, pre);
}
std::vector<std::vector<uint8_t>> gpu_prove_lockstep(const PreparedCS *const *csv, const uint8_t *label,
                                                     size_t label_len, const RngBlock *const *rbs, int P,
                                                     ProveTimings *tms, const AllGather *ag, const CommitPre *pre) {
    if (P < 1 || P > MAX_LOCKSTEP) throw std::runtime_error("lockstep proof count");
    const PreparedCS &cs = *csv[0];
    for (int p = 0; p < P; p++) {
        const PreparedCS &c = *csv[p];
        if (!c.prover) throw std::runtime_error("prepared circuit has no witness");
        if (c.n != cs.n || c.m != cs.m || c.N != cs.N || c.world != cs.world || c.rank != cs.rank ||
            c.device != cs.device)
            throw std::runtime_error("lockstep proofs of different shapes");
    }
    static_assert(16 * MAX_LOCKSTEP <= MSM_MAX_SEGS, "an IPP job holds up to 16 segments per proof");
    DeviceContext &ctx = DeviceContext::get(cs.device);
    const uint32_t n = cs.n, m = cs.m, N = cs.N, lgN = cs.lgN;
    // this rank's slice: lanes i = j * world + rank, j < nl real, j < Nl padded
    const uint32_t world = cs.world, rank = cs.rank, nl = cs.nl, Nl = cs.Nl;
    const bool sharded = world > 1;
    if (sharded && !ag) throw std::runtime_error("sharded prove without an exchange");
    if (sharded && P != 1) throw std::runtime_error("the sharded prover proves one proof at a time");
    if (pre && P != 1) throw std::runtime_error("precomputed commitments are for one proof");
    std::shared_ptr<const GenSet> gs = ctx.gens(N, rank, world);
    Workspace &ws = thread_workspace(cs.device);
    hipStream_t st = ws.st;
    double t0 = now_ms();
    std::vector<Transcript> T;
    for (int p = 0; p < P; p++) {
        ProofBufs &B = ws.pb[p];
        B.tabs.grow(8 * 40 * sizeof(ScD));
        if (!B.small_host) {
            BPG_HIP(hipHostMalloc((void **)&B.small_host, 4096 * sizeof(ScD), hipHostMallocDefault));
            BPG_HIP(hipHostGetDevicePointer((void **)&B.small_view, B.small_host, 0));
        }
        T.push_back(prover_transcript(*csv[p], label, label_len));
    }

    // A_I1 = <a_L,G> + <a_R,H>, A_O1 = <a_O,G>, S1 = <s_L,G> + <s_R,H>
    // (blinding terms added on the host): one MSM job of 3 MSMs per proof
    PtD *rowsA = ws.rows_host, *rowsLR = ws.rows_host + ROWS_HALF;
    // zero copy: the MSM row kernels and the c_L / c_R reductions write into
    // the pinned buffers through their device views (no copy launch per job)
    PtD *rowsA_dev = ws.rows_view, *rowsLR_dev = ws.rows_view + ROWS_HALF;
    // level-0 generators (affine Niels) for the MSM jobs: the fixed-base
    // tables when this set has them (window 0 = the generators, negations
    // at + N, window w at + w 2N), else the set itself (negations at + N)
    std::shared_ptr<FbTables> fbt = (!sharded && cs.strat.fixed_base()) ? ctx.fb(gs, N) : nullptr;
    const void *G0 = fbt ? (const void *)fbt->G : (const void *)gs->G;
    const void *H0 = fbt ? (const void *)fbt->H : (const void *)gs->H;
    // generator jobs negate in registers (as gpu_prove: one 256 MB gather set)
    const int64_t gneg = fbt ? (int64_t)fbt->N : 0;
    const uint64_t gws = fbt ? 2 * (uint64_t)fbt->N : 0;   // MsmSeg::wstride of their segments
    // one commitment job per proof: a P-proof commitment job would be the
    // largest of the proof and size every workspace's MSM scratch (~7 GB at
    // P = 2 and 2^20), leaving HBM for fewer consumers
    const size_t ROWS_PER_PROOF = 192;   // 3 MSMs x at most 64 windows
    MsmPlan pA[MAX_LOCKSTEP] = {};
    if (!pre) {
        MsmSeg seg[MAX_LOCKSTEP][6];
        int nseg[MAX_LOCKSTEP] = {0};
        WideBatch WB{};   // s_L, s_R of every proof: one reduction launch
        int nwq = 0;
        for (int p = 0; p < P; p++) {
            ProofBufs &B = ws.pb[p];
            const RngBlock &rb = *rbs[p];
            // s_L | s_R: raw 64-byte draws -> device, reduced mod l there (this
            // rank's lanes only)
            B.sL.grow((size_t)nl * sizeof(ScD) + 64);
            B.sR.grow((size_t)nl * sizeof(ScD) + 64);
            if (!nl) continue;
            const uint8_t *wd = rb.wide;
            if (!rb.on_device) {
                B.wide.grow(2 * (size_t)n * 64 + 64);
                BPG_HIP(hipMemcpyAsync(B.wide.p, rb.wide, 2 * (size_t)n * 64, hipMemcpyHostToDevice, st));
                wd = as<uint8_t>(B.wide);
            }
            WB.wide[2 * nwq] = wd; WB.out[2 * nwq] = as<ScD>(B.sL);
            WB.wide[2 * nwq + 1] = wd + 64 * (size_t)n; WB.out[2 * nwq + 1] = as<ScD>(B.sR);
            nwq++;
            const PreparedCS &cp = *csv[p];
            MsmSeg *sg = seg[p];
            int &ns = nseg[p];
            commit_a_segments(cp, *gs, !fbt, G0, H0, gneg, gws, st, B.eqsc, sg, ns);
            sg[ns++] = {as<ScD>(const_cast<DBuf &>(cp.aO)), G0, nl, 1, gneg, gws};
            sg[ns++] = {as<ScD>(B.sL), G0, nl, 2, gneg, gws};
            sg[ns++] = {as<ScD>(B.sR), H0, nl, 2, gneg, gws};
            for (int i = 0; i < ns; i++) sg[i].gen = true;
        }
        if (nwq) launch_wide_reduce_batch(WB, 2 * nwq, nl, world, rank, st);
        for (int p = 0; p < P && nl; p++) {
            int ph = ws.prof_begin("msm_commit", 5.0 * nl * (64 + 32));
            pA[p] = ws.msm->enqueue(seg[p], nseg[p], 3, rowsA + ROWS_PER_PROOF * p, MSM_NIELS,
                                    rowsA_dev + ROWS_PER_PROOF * p);
            ws.prof_end(ph);
        }
    }
    ws.sync();
    std::vector<Scalar> y(P), z(P);
    std::vector<std::array<uint8_t, 96>> cA(P);   // compressed A_I1 | A_O1 | S1
    for (int p = 0; p < P; p++) {
        const RngBlock &rb = *rbs[p];
        Point AIS[3], tmp;
        if (nl && pre) {   // A_I1, A_O1 from one job; S1 = <s_L, G> + <s_R, H> from two
            combine_rows(AIS[0], rowsA + CommitPre::ROWS_A, pre->A.W, pre->A.c);
            combine_rows(AIS[1], rowsA + CommitPre::ROWS_A + pre->A.W, pre->A.W, pre->A.c);
            Point sl, sr;
            combine_rows(sl, rowsA + CommitPre::ROWS_S0, pre->S[0].W, pre->S[0].c);
            combine_rows(sr, rowsA + CommitPre::ROWS_S1, pre->S[1].W, pre->S[1].c);
            pt_add(AIS[2], sl, sr);
        } else if (nl) {
            const MsmPlan &pl = pA[p];
            const PtD *rows = rowsA + ROWS_PER_PROOF * p;
            for (int k = 0; k < 3; k++) combine_rows(AIS[k], rows + k * pl.W, pl.W, pl.c);
        } else {
            pt_identity(AIS[0]); pt_identity(AIS[1]); pt_identity(AIS[2]);
        }
        if (sharded) {
            std::vector<Point> sum = allgather_point_sums(*ag, AIS, 3, world);
            for (int k = 0; k < 3; k++) AIS[k] = sum[k];
        }
        mul_B_blinding(tmp, rb.i_bl); pt_add(AIS[0], AIS[0], tmp);
        mul_B_blinding(tmp, rb.o_bl); pt_add(AIS[1], AIS[1], tmp);
        mul_B_blinding(tmp, rb.s_bl); pt_add(AIS[2], AIS[2], tmp);
        uint8_t *c = cA[p].data();
        ristretto_compress(c, AIS[0]); ristretto_compress(c + 32, AIS[1]); ristretto_compress(c + 64, AIS[2]);
        T[p].append_point("A_I1", c);
        T[p].append_point("A_O1", c + 32);
        T[p].append_point("S1", c + 64);
        T[p].append_message("dom-sep", (const uint8_t *)"r1cs-1phase", 11);
        const uint8_t zero32[32] = {0};
        T[p].append_point("A_I2", zero32);
        T[p].append_point("A_O2", zero32);
        T[p].append_point("S2", zero32);
        y[p] = T[p].challenge_scalar("y");
        z[p] = T[p].challenge_scalar("z");
    }
    double t1 = now_ms();

    // vectors: powers, flattened_constraints(z), l(x)/r(x) coefficients, t(x)
    // (y^i and y^-i at this rank's lanes: (y^world)^j * y^rank)
    std::vector<Scalar> y_inv(P);
    {
        // y^i, y^-i (at this rank's lanes: (y^world)^j y^rank) and the z^q
        // tables of every proof of the step: one table launch and one
        // expansion launch, the doubling powers read from pinned memory (no
        // upload copies; 14 launches per proof before, round 5)
        PowBatch PT{};
        PowExpandBatch PE{};
        for (int p = 0; p < P; p++) {
            ProofBufs &B = ws.pb[p];
            const PreparedCS &cp = *csv[p];
            y_inv[p] = sc_invert(y[p]);
            const Scalar base[3] = {sharded ? sc_pow_u64(y[p], world) : y[p],
                                    sharded ? sc_pow_u64(y_inv[p], world) : y_inv[p], z[p]};
            const uint32_t cnt[3] = {Nl, Nl, cp.q + 2};
            for (int j = 0; j < 3; j++) {
                ScD *h = B.small_host + 80 * j;
                Scalar cur = base[j];
                for (int b = 0; b < 40; b++) { h[b] = mont(cur); cur = cur * cur; }
                cur = sc_pow_u64(base[j], 1024);
                for (int b = 0; b < 40; b++) { h[40 + b] = mont(cur); cur = cur * cur; }
                PT.nhi[p][j] = cnt[j] / 1024 + 1;
            }
            // lo | hi of y in ytab, of y^-1 in ylo / yhi, of z in zlo / zhi
            // (the flatten reads those); in the workspace, not freed per
            // proof: a hipFree synchronises the whole device
            B.ytab.grow((1024 + (size_t)PT.nhi[p][0]) * sizeof(ScD));
            B.ylo.grow(1024 * sizeof(ScD)); B.yhi.grow((size_t)PT.nhi[p][1] * sizeof(ScD));
            B.zlo.grow(1024 * sizeof(ScD)); B.zhi.grow((size_t)PT.nhi[p][2] * sizeof(ScD));
            B.ypm.grow((size_t)Nl * sizeof(ScD));
            B.yipm.grow((size_t)Nl * sizeof(ScD));
            PT.b2[p] = B.small_view;
            PT.lo[p][0] = as<ScD>(B.ytab); PT.hi[p][0] = as<ScD>(B.ytab) + 1024;
            PT.lo[p][1] = as<ScD>(B.ylo); PT.hi[p][1] = as<ScD>(B.yhi);
            PT.lo[p][2] = as<ScD>(B.zlo); PT.hi[p][2] = as<ScD>(B.zhi);
            for (int j = 0; j < 2; j++) { PE.lo[p][j] = PT.lo[p][j]; PE.hi[p][j] = PT.hi[p][j]; }
            PE.out[p][0] = as<ScD>(B.ypm); PE.out[p][1] = as<ScD>(B.yipm);
            PE.mult[p][0] = mont(sharded ? sc_pow_u64(y[p], rank) : Scalar::one());
            PE.mult[p][1] = mont(sharded ? sc_pow_u64(y_inv[p], rank) : Scalar::one());
        }
        launch_pow_tables(PT, P, 3, st);
        launch_pow_expand_batch(PE, P, 2, Nl, st);
    }
    for (int p = 0; p < P; p++) {
        ProofBufs &B = ws.pb[p];
        const PreparedCS &cp = *csv[p];
        CscDev csc{as<uint32_t>(const_cast<DBuf &>(cp.col_ptr)), as<uint32_t>(const_cast<DBuf &>(cp.col_row)),
                   as<ScD>(const_cast<DBuf &>(cp.col_coeff)), as<uint32_t>(const_cast<DBuf &>(cp.short_cols)),
                   as<uint32_t>(const_cast<DBuf &>(cp.long_cols)), cp.nshort, cp.nlong, cp.ncol, 3 * n};
        B.w.grow((size_t)cp.ncol * sizeof(ScD) + 64);
        int pfl = ws.prof_begin("flatten", (double)cp.ncol * 32);
        launch_flatten(csc, as<ScD>(B.zlo), as<ScD>(B.zhi), as<ScD>(B.w), st);
        grow_partial(B.partial, st);
        for (uint32_t col : cp.huge_cols)
            launch_flatten_huge(csc, col, cp.col_ptr_host[col], cp.col_ptr_host[col + 1], as<ScD>(B.zlo),
                                as<ScD>(B.zhi), as<ScD>(B.partial), as<ScD>(B.w), st);
        ws.prof_end(pfl);
        ScD *wfull = as<ScD>(B.w);
        ScD *wV = wfull + 3 * (size_t)n;
        ScD *wL = wfull, *wR = wfull + n, *wO = wfull + 2 * (size_t)n;
        if (sharded) {   // w_L, w_R, w_O at this rank's lanes
            B.wloc.grow(3 * (size_t)nl * sizeof(ScD) + 64);
            wL = as<ScD>(B.wloc); wR = wL + nl; wO = wL + 2 * (size_t)nl;
            launch_gather_scalars(wfull, nl, world, rank, wL, st);
            launch_gather_scalars(wfull + n, nl, world, rank, wR, st);
            launch_gather_scalars(wfull + 2 * (size_t)n, nl, world, rank, wO, st);
        }
        for (DBuf *d : {&B.l1, &B.r0, &B.r1, &B.r3}) d->grow((size_t)nl * sizeof(ScD) + 64);
        B.small.grow(64 * sizeof(ScD));
        ScD *dsmall = B.small_view + 1000;   // t_1..t_6, <w_V, v_blinding> (pinned, device view)
        if (nl) {
            launch_lr_build(as<ScD>(const_cast<DBuf &>(cp.aL)), as<ScD>(const_cast<DBuf &>(cp.aR)), as<ScD>(B.sR), wL,
                            wR, wO, as<ScD>(B.ypm), as<ScD>(B.yipm), nl, as<ScD>(B.l1), as<ScD>(B.r0), as<ScD>(B.r1),
                            as<ScD>(B.r3), st);
            launch_tpoly(as<ScD>(B.l1), as<ScD>(const_cast<DBuf &>(cp.aO)), as<ScD>(B.sL), as<ScD>(B.r0),
                         as<ScD>(B.r1), as<ScD>(B.r3), nl, as<ScD>(B.partial), dsmall, st);
        } else {
            BPG_HIP(hipMemsetAsync(dsmall, 0, 6 * sizeof(ScD), st));
        }
        if (m) launch_dot(wV, as<ScD>(const_cast<DBuf &>(cp.vb_dev)), m, as<ScD>(B.partial), dsmall + 6, st);
        else BPG_HIP(hipMemsetAsync(dsmall + 6, 0, sizeof(ScD), st));
    }
    ws.sync();
    std::vector<Scalar> u(P), x(P), t_x(P), t_xb(P), e_bl(P), wch(P);
    std::vector<std::array<uint8_t, 160>> cT(P);
    for (int p = 0; p < P; p++) {
        ProofBufs &B = ws.pb[p];
        const RngBlock &rb = *rbs[p];
        Scalar tp[6];
        for (int k = 0; k < 6; k++) tp[k] = from_dev(B.small_host[1000 + k]);
        if (sharded) {
            std::vector<Scalar> sum = allgather_scalar_sums(*ag, tp, 6, world);
            for (int k = 0; k < 6; k++) tp[k] = sum[k];
        }
        const Scalar tb2 = from_dev(B.small_host[1006]);   // <w_V, v_blinding>: every rank holds all of w_V
        const Scalar tb1 = rb.tb[0], tb3 = rb.tb[1], tb4 = rb.tb[2], tb5 = rb.tb[3], tb6 = rb.tb[4];
        uint8_t *c = cT[p].data();
        pedersen_commit(c, tp[0], tb1);
        pedersen_commit(c + 32, tp[2], tb3);
        pedersen_commit(c + 64, tp[3], tb4);
        pedersen_commit(c + 96, tp[4], tb5);
        pedersen_commit(c + 128, tp[5], tb6);
        T[p].append_point("T_1", c);
        T[p].append_point("T_3", c + 32);
        T[p].append_point("T_4", c + 64);
        T[p].append_point("T_5", c + 96);
        T[p].append_point("T_6", c + 128);
        u[p] = T[p].challenge_scalar("u");
        x[p] = T[p].challenge_scalar("x");
        const Scalar xx = x[p];
        auto eval6 = [&](const Scalar cc[6]) {
            Scalar acc = xx * cc[5];
            for (int k = 4; k >= 0; k--) acc = xx * (cc[k] + acc);
            return acc;
        };
        const Scalar tbs[6] = {tb1, tb2, tb3, tb4, tb5, tb6};
        t_x[p] = eval6(tp);
        t_xb[p] = eval6(tbs);
        e_bl[p] = xx * (rb.i_bl + xx * (rb.o_bl + xx * rb.s_bl));
        T[p].append_scalar("t_x", t_x[p]);
        T[p].append_scalar("t_x_blinding", t_xb[p]);
        T[p].append_scalar("e_blinding", e_bl[p]);
        wch[p] = T[p].challenge_scalar("w");
        B.a.grow((size_t)Nl * sizeof(ScD) + 64);
        B.b.grow((size_t)Nl * sizeof(ScD) + 64);
        launch_lr_eval(as<ScD>(B.l1), as<ScD>(const_cast<DBuf &>(csv[p]->aO)), as<ScD>(B.sL), as<ScD>(B.r0),
                       as<ScD>(B.r1), as<ScD>(B.r3), as<ScD>(B.ypm), nl, Nl, mont(xx), mont(xx * xx), as<ScD>(B.a),
                       as<ScD>(B.b), st);
    }
    double t2 = now_ms();

    // InnerProductProof::create with weighted single-scalar point folding
    // over this rank's Nl lanes (a round pairs lane i with i + h, h a
    // multiple of world, so every local round is rank-local: local half
    // h / world). With comb tables (Nl >= 8) rounds 0 and 1 leave the level-1
    // generators unmaterialised: round 1's MSM expands them into level-0
    // generators and level 2 is built in one table pass.
    for (int p = 0; p < P; p++) {
        T[p].append_message("dom-sep", (const uint8_t *)"ipp v1", 6);
        T[p].append_u64("n", N);
    }
    std::shared_ptr<CombTables> comb = cs.strat.tables() ? ctx.comb(gs, Nl) : nullptr;
    std::vector<std::vector<uint8_t>> LRc(P, std::vector<uint8_t>(64 * (size_t)lgN));
    std::vector<Scalar> lam(P, Scalar::one()), mu(P, Scalar::one());
    std::vector<const void *> Gh(P, gs->G), Hh(P, gs->H);
    int gfmt = MSM_NIELS;
    for (int p = 0; p < P; p++) {
        ProofBufs &B = ws.pb[p];
        B.mscal.grow((size_t)(2 * Nl + 2) * sizeof(ScD) + 64);
        if (Nl >= 2)
            for (int k = 0; k < 2; k++) {
                B.Gp[k].grow((size_t)(Nl / 2) * sizeof(PtD));
                B.Hp[k].grow((size_t)(Nl / 2) * sizeof(PtD));
            }
    }
    // Round groups: after round k the fold is left pending (Ghat stays at
    // level k); round k+d's MSM expands each level-(k+d) base into its 2^d
    // level-k points, and after the group's last round one pass builds the
    // next level from level k: comb tables from the level-0 generators (a
    // pair), else the three- (pair) or seven-scalar (triple) Straus fold.
    const int group_cfg = cs.strat.group();
    std::vector<std::array<std::array<Scalar, 4>, 2>> rho_h(P);   // pending rounds' fold scalars, oldest first
    int depth = 0;        // pending levels: Ghat at level k, this round at level k + depth
    int cur = -1;         // buffer holding Ghat/Hhat: -1 the generators, else Gp/Hp[cur]
    // Tail (DESIGN.md "IPP tail without folds"): once a materialised level is
    // short, the remaining rounds keep it and weight its points instead of
    // folding them (each fold there is a latency-bound launch). The sharded
    // prover always ends in the tail: its last local round's fold is needed
    // (as weights) for the final generator of each rank. Sharded, the
    // materialised levels are Nl/8^j (or /4^j, /2^j) after the first group,
    // so the last one of at least 2 lanes has at most 8 lanes: a threshold
    // of 8 or more always meets it.
    const uint32_t tail_len = sharded ? std::max<uint32_t>(cs.strat.tail(), 8u) : cs.strat.tail();
    bool tail = false;
    uint32_t M = 0;
    uint32_t len = Nl;
    // A level a fold group materialises (cached points in Gp/Hp[cur]) is
    // converted to affine Niels in the other buffer (k_cached_to_niels: one
    // inversion per 32 points, ~15M per point): every later MSM entry over it
    // is then a 7M madd in pass 1's three-wave kernel instead of an 8M cached
    // addition at two waves, and the folds read it as they read generators
    // (+0.9% in the bench, profiles/r04o_ab.txt).
    auto niels_level = [&](uint32_t cnt) {
        const int oth = cur == 0 ? 1 : 0;
        const PtD *vin[2 * MAX_LOCKSTEP];
        NielsD *vout[2 * MAX_LOCKSTEP];
        for (int p = 0; p < P; p++) {   // every proof's G and H level in one launch
            ProofBufs &B = ws.pb[p];
            vin[2 * p] = as<PtD>(B.Gp[cur]); vout[2 * p] = as<NielsD>(B.Gp[oth]);
            vin[2 * p + 1] = as<PtD>(B.Hp[cur]); vout[2 * p + 1] = as<NielsD>(B.Hp[oth]);
            Gh[p] = B.Gp[oth].p; Hh[p] = B.Hp[oth].p;
        }
        launch_cached_to_niels(vin, vout, 2 * P, cnt, st);
        cur = oth;
        gfmt = MSM_NIELS;
    };
    // a (= l(x), zero past the real lanes) is nonzero only on lanes < anz:
    // anz = nl, then min(anz, h) after each round's fold
    uint32_t anz = nl;
    uint32_t k = 0;
    for (; len != 1; k++) {
        const uint32_t h = len / 2;
        if (k == inject_oom_round()) inject_oom_once();
        if (!tail && depth == 0 && cur >= 0 && len <= tail_len && len >= (sharded ? 2u : 4u)) {
            tail = true;
            M = len;
            ScD *wq[2 * MAX_LOCKSTEP];
            for (int p = 0; p < P; p++) {
                ProofBufs &B = ws.pb[p];
                B.wG.grow((size_t)M * sizeof(ScD) + 64);
                B.wH.grow((size_t)M * sizeof(ScD) + 64);
                wq[2 * p] = as<ScD>(B.wG); wq[2 * p + 1] = as<ScD>(B.wH);
            }
            launch_fill_scalars_batch(wq, 2 * P, mont(Scalar::one()), M, st);
        }
        // MSM bases: the level-0 generators (affine Niels), else Ghat/Hhat (cached)
        const int mfmt = cur < 0 ? MSM_NIELS : gfmt;
        const size_t ps = mfmt == MSM_NIELS ? sizeof(NielsD) : sizeof(PtD);
        // jobs over the level-0 generators gather their negated copies for
        // negative digits (a converted level negates in registers)
        const int64_t gn = cur < 0 ? gneg : 0;
        auto at = [&](const void *b, size_t i) { return (const void *)((const uint8_t *)b + i * ps); };
        const bool lazy = depth == 1;
        const size_t hh = h;
        // round 0 over the level-0 generators with padding lanes: their L
        // terms on H_lo become one precomputed sum (below)
        const bool round0_pad = k == 0 && cur < 0 && depth == 0 && !tail && nl > h && nl < len;
        Point pad_sum;
        if (round0_pad)   // before the job: the sum's MSM uses the workspace's engine and row buffer
            pad_sum = generator_range_sum(ws, *gs, nl - h, h);
        MsmSeg seg[MSM_MAX_SEGS];
        int nseg = 0;
        PrepBatch PB{};   // the round preparation of every proof, one launch after the loop
        int prep_kind = PREP_PLAIN;
        for (int p = 0; p < P; p++) {
            ProofBufs &B = ws.pb[p];
            IppRoundArgs A;
            A.h = h; A.n = nl;
            A.lamG1 = mont(lam[p]); A.lamGu = mont(lam[p] * u[p]);
            A.muH1 = mont(mu[p]); A.muHu = mont(mu[p] * u[p]);
            ScD *ms = as<ScD>(B.mscal);
            ScD *cout = B.small_view + 1020;   // c_L, c_R (pinned, device view)
            PB.a[p] = as<ScD>(B.a); PB.b[p] = as<ScD>(B.b); PB.yipm[p] = as<ScD>(B.yipm);
            PB.out[p] = ms; PB.partial[p] = as<ScD>(B.partial); PB.c_out[p] = cout;
            PB.A[p] = A;
            const void *Gm = cur < 0 ? G0 : Gh[p], *Hm = cur < 0 ? H0 : Hh[p];
            const uint32_t L0 = 2 * (uint32_t)p, R0 = L0 + 1;   // this proof's L and R MSMs
            if (tail) {
                prep_kind = PREP_TAIL;
                PB.M = M; PB.wG[p] = as<ScD>(B.wG); PB.wH[p] = as<ScD>(B.wH);
                const size_t mm_ = M;
                seg[nseg++] = {ms, Gh[p], M, L0};
                seg[nseg++] = {ms + mm_, Hh[p], M, L0};
                seg[nseg++] = {ms + 2 * mm_, Gh[p], M, R0};
                seg[nseg++] = {ms + 3 * mm_, Hh[p], M, R0};
            } else if (lazy) {
                const uint32_t h0 = 2 * h;
                LazyArgs Z;
                Z.h0 = h0;
                Z.rGa = mont(rho_h[p][0][0]); Z.rGb = mont(rho_h[p][0][1]);
                Z.rHa = mont(rho_h[p][0][2]); Z.rHb = mont(rho_h[p][0][3]);
                prep_kind = PREP_LAZY;
                PB.lz[p] = Z;
                seg[nseg++] = {ms, at(Gm, h), h, L0, gn};
                seg[nseg++] = {ms + hh, at(Gm, h + h0), h, L0, gn};
                seg[nseg++] = {ms + 2 * hh, Hm, h, L0, gn};
                seg[nseg++] = {ms + 3 * hh, at(Hm, h0), h, L0, gn};
                seg[nseg++] = {ms + 4 * hh, Gm, h, R0, gn};
                seg[nseg++] = {ms + 5 * hh, at(Gm, h0), h, R0, gn};
                seg[nseg++] = {ms + 6 * hh, at(Hm, h), h, R0, gn};
                seg[nseg++] = {ms + 7 * hh, at(Hm, h + h0), h, R0, gn};
            } else if (depth == 2) {
                // bases at level k+2 expanded into level k: family f, term t at
                // out[(4f + t) h], point offset x0(f) + 2h t
                Deep2Args Z;
                for (int v = 0; v < 2; v++)
                    for (int c = 0; c < 2; c++) {
                        Z.r0[v][c] = mont(rho_h[p][0][2 * v + c]);
                        Z.r1[v][c] = mont(rho_h[p][1][2 * v + c]);
                    }
                prep_kind = PREP_DEEP2;
                PB.dz[p] = Z;
                for (int f = 0; f < 4; f++) {
                    const void *Bs = (f & 1) ? Hm : Gm;
                    const size_t x0 = (f == 0 || f == 3) ? hh : 0;
                    for (int t = 0; t < 4; t++)
                        seg[nseg++] = {ms + (size_t)(4 * f + t) * hh, at(Bs, x0 + 2 * hh * t), h,
                                       (uint32_t)(f >> 1) + L0, gn};
                }
            } else {
                prep_kind = PREP_PLAIN;
                // points whose a-scalar is zero (padding lanes) are left out of
                // the job: L's G part runs over a_lo, R's over a_hi. In round
                // 0 L's H part leaves out the padding lanes too: there
                // b_hi[j] * y^-j = -y^(j + h) y^-j = -y^h for every padding
                // lane (r(x) is -y^i past the real lanes, prover.rs pads it so),
                // so their terms are -y^h * sum H_j over a fixed range, added
                // on the host (pad_sum): 29% of round 0's L entries at 2^20
                const uint32_t nLG = std::min(h, anz), nRG = anz > h ? std::min(h, anz - h) : 0u;
                const uint32_t nLH = round0_pad ? nl - h : h;
                const MsmSeg sl[4] = {{ms, at(Gm, h), nLG, L0, gn}, {ms + hh, Hm, nLH, L0, gn},
                                      {ms + 2 * hh, Gm, nRG, R0, gn}, {ms + 3 * hh, at(Hm, h), h, R0, gn}};
                for (const MsmSeg &s : sl) if (s.count) seg[nseg++] = s;
            }
        }
        launch_ipp_prep(PB, prep_kind, P, st);
        if (cur < 0)   // level-0 generator segments (gathering from the fixed-base tables when on)
            for (int i = 0; i < nseg; i++) { seg[i].wstride = gws; seg[i].gen = true; }
        int ph = ws.prof_begin("msm_ipp", P * (tail ? 2.0 * M : (4.0 * h) * (1 << depth)) * (64 + 32));
        MsmPlan pl = ws.msm->enqueue(seg, nseg, 2 * P, rowsLR, mfmt, rowsLR_dev);
        ws.prof_end(ph);
        ws.sync();
        std::vector<std::array<Scalar, 4>> rnow(P);   // this round's fold scalars (G a/b, H a/b)
        ScD *fa[MAX_LOCKSTEP], *fb[MAX_LOCKSTEP], fu[MAX_LOCKSTEP], fui[MAX_LOCKSTEP];   // a, b folds
        for (int p = 0; p < P; p++) {
            ProofBufs &B = ws.pb[p];
            Point LR[2], cq;
            combine_rows(LR[0], rowsLR + (2 * p) * pl.W, pl.W, pl.c);
            combine_rows(LR[1], rowsLR + (2 * p + 1) * pl.W, pl.W, pl.c);
            if (round0_pad) {   // the padding lanes' L terms: -y^(h world) mu * sum H_j
                const Scalar spad = -(sc_pow_u64(y[p], (uint64_t)h * world) * mu[p]);
                Point t;
                mul_var(t, spad, pad_sum);
                pt_add(LR[0], LR[0], t);
            }
            // + c_L Q, + c_R Q (this rank's share of c_L, c_R when sharded)
            for (int s = 0; s < 2; s++) {
                mul_B(cq, from_dev(B.small_host[1020 + s]) * wch[p]);
                pt_add(LR[s], LR[s], cq);
            }
            if (sharded) {   // sum the ranks' partial L and R
                std::vector<Point> sum = allgather_point_sums(*ag, LR, 2, world);
                LR[0] = sum[0]; LR[1] = sum[1];
            }
            uint8_t *cl = LRc[p].data() + 64 * (size_t)k, *cr = cl + 32;
            ristretto_compress(cl, LR[0]);
            ristretto_compress(cr, LR[1]);
            T[p].append_point("L", cl);
            T[p].append_point("R", cr);
            const Scalar uk = T[p].challenge_scalar("u");
            const Scalar uinv = sc_invert(uk);
            fa[p] = as<ScD>(B.a); fb[p] = as<ScD>(B.b); fu[p] = mont(uk); fui[p] = mont(uinv);
            const Scalar u2 = uk * uk, ui2 = uinv * uinv;
            const Scalar yh = sc_pow_u64(y_inv[p], (uint64_t)h * world);   // the round's global half length
            rnow[p] = {u2, u2 * u[p], ui2 * yh, ui2 * yh * u[p]};
            lam[p] = lam[p] * uinv;
            mu[p] = mu[p] * uk;
        }
        launch_ipp_fold_scalars(fa, fb, fu, fui, P, h, st);   // the round's a, b folds of every proof
        const int nxt = cur == 0 ? 1 : 0;
        if (tail) {
            if (h > 1 || sharded) {
                ScD *wg[MAX_LOCKSTEP], *wh[MAX_LOCKSTEP], rw[MAX_LOCKSTEP][4];
                for (int p = 0; p < P; p++) {
                    wg[p] = as<ScD>(ws.pb[p].wG); wh[p] = as<ScD>(ws.pb[p].wH);
                    for (int q = 0; q < 4; q++) rw[p][q] = mont(rnow[p][q]);
                }
                launch_ipp_tail_weights(wg, wh, rw, P, M, h, nl, st);
            }
        } else if (h > 1) {
            const int group = (comb && cur < 0) ? 2 : group_cfg;
            if (depth + 1 < group) {   // level k + depth + 1 stays implicit
                for (int p = 0; p < P; p++) rho_h[p][depth] = rnow[p];
                depth++;
            } else if (depth == 0) {
                for (int p = 0; p < P; p++) {
                    ProofBufs &B = ws.pb[p];
                    PtD *Gn = as<PtD>(B.Gp[nxt]), *Hn = as<PtD>(B.Hp[nxt]);
                    launch_ipp_fold_points(Gh[p], Hh[p], gfmt, h, nl, to_dev(rnow[p][0]), to_dev(rnow[p][1]),
                                           to_dev(rnow[p][2]), to_dev(rnow[p][3]), Gn, Hn, B.fold_stage, st);
                    Gh[p] = Gn; Hh[p] = Hn;
                }
                cur = nxt;
                gfmt = MSM_CACHED;
                niels_level(h);
            } else if (depth == 1) {
                // level k+2 from level k: out_i = P_i + c1 P_{i+h1} + c2 P_{i+2h1} + c3 P_{i+3h1}
                const uint32_t h1 = h, h0 = 2 * h;
                std::vector<int64_t> cut = {0, (int64_t)h1, (int64_t)nl - h1, (int64_t)nl, (int64_t)nl - h0,
                                            (int64_t)nl - h0 - h1};
                std::vector<uint32_t> starts;
                for (int64_t c : cut) if (c >= 0 && c < (int64_t)h1) starts.push_back((uint32_t)c);
                std::sort(starts.begin(), starts.end());
                starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
                const bool table = comb && cur < 0;
                for (int p = 0; p < P; p++) {
                    ProofBufs &B = ws.pb[p];
                    const std::array<Scalar, 4> &rho_p = rho_h[p][0];
                    ScD coef[2][COMB_MAXRANGE][3];
                    CombArgs C{};
                    C.nrange = (uint32_t)starts.size();
                    for (uint32_t r = 0; r < C.nrange; r++) {
                        const uint64_t i = starts[r];
                        C.rstart[r] = (uint32_t)i;
                        const bool b1 = i < nl && i + h1 >= nl, b0 = i < nl && i + h0 >= nl,
                                   b0h = i + h1 < nl && i + h1 + h0 >= nl;
                        for (int v = 0; v < 2; v++) {
                            const Scalar c1 = rnow[p][2 * v + (b1 ? 1 : 0)];
                            const Scalar c2 = rho_p[2 * v + (b0 ? 1 : 0)];
                            const Scalar c3 = c1 * rho_p[2 * v + (b0h ? 1 : 0)];
                            if (table) {
                                uint8_t sb[3][32];
                                c1.reduced().to_bytes(sb[0]); c2.reduced().to_bytes(sb[1]); c3.reduced().to_bytes(sb[2]);
                                comb_digits(sb[0], C.dig[v][r][0]);
                                comb_digits(sb[1], C.dig[v][r][1]);
                                comb_digits(sb[2], C.dig[v][r][2]);
                            } else {
                                coef[v][r][0] = to_dev(c1); coef[v][r][1] = to_dev(c2); coef[v][r][2] = to_dev(c3);
                            }
                        }
                    }
                    if (table) {
                        C.gens[0] = gs->G; C.gens[1] = gs->H;
                        C.tab[0] = comb->tabG; C.tab[1] = comb->tabH;
                        C.out[0] = B.Gp[nxt].p; C.out[1] = B.Hp[nxt].p;
                        C.h1 = h1; C.ntab = 3 * h1;
                        launch_ipp_comb_fold(C, B.comb_stage, st);
                    } else {
                        launch_ipp_fold2(Gh[p], Hh[p], gfmt, h1, C.nrange, C.rstart, coef, as<PtD>(B.Gp[nxt]),
                                         as<PtD>(B.Hp[nxt]), B.fold2_stage, st);
                    }
                    Gh[p] = B.Gp[nxt].p; Hh[p] = B.Hp[nxt].p;
                }
                cur = nxt;
                gfmt = MSM_CACHED;
                niels_level(h);
                depth = 0;
            } else {
                // level k+3 from level k: out_i = sum_{t<8} c_t P_{i + t hq}, point
                // t = 4 b0 + 2 b1 + b2 reached through round k+2 (lane i), round
                // k+1 (lane i + b2 hq) and round k (lane i + b2 hq + 2 b1 hq);
                // each set bit contributes its round's scalar for that lane's class
                const uint32_t hq = h;
                std::vector<uint32_t> starts = {0};
                for (int j = 0; j <= 8; j++) {
                    const int64_t c = (int64_t)nl - (int64_t)j * hq;
                    if (c > 0 && c < (int64_t)hq) starts.push_back((uint32_t)c);
                }
                std::sort(starts.begin(), starts.end());
                starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
                if (starts.size() > COMB_MAXRANGE) throw std::runtime_error("fold3 ranges");
                auto cls = [&](uint64_t xx, uint64_t half) { return xx < nl && xx + half >= nl ? 1 : 0; };
                // every proof's fold in one launch (one argument upload), the
                // tables of all its blocks in proof 0's buffer
                ScD coefs[MAX_LOCKSTEP][2][COMB_MAXRANGE][7];
                const ScD (*cp3[MAX_LOCKSTEP])[COMB_MAXRANGE][7];
                const void *gin[MAX_LOCKSTEP], *hin[MAX_LOCKSTEP];
                PtD *gout[MAX_LOCKSTEP], *hout[MAX_LOCKSTEP];
                for (int p = 0; p < P; p++) {
                    ProofBufs &B = ws.pb[p];
                    const std::array<Scalar, 4> *rr[3] = {&rho_h[p][0], &rho_h[p][1], &rnow[p]};
                    ScD (&coef)[2][COMB_MAXRANGE][7] = coefs[p];
                    for (size_t r = 0; r < starts.size(); r++) {
                        const uint64_t i = starts[r];
                        for (int t = 1; t < 8; t++) {
                            const int b0 = (t >> 2) & 1, b1 = (t >> 1) & 1, b2 = t & 1;
                            const uint64_t x2 = i, x1 = i + (uint64_t)b2 * hq, x0 = x1 + (uint64_t)b1 * 2 * hq;
                            for (int v = 0; v < 2; v++) {
                                Scalar c = Scalar::one();
                                if (b2) c = c * (*rr[2])[2 * v + cls(x2, hq)];
                                if (b1) c = c * (*rr[1])[2 * v + cls(x1, 2 * (uint64_t)hq)];
                                if (b0) c = c * (*rr[0])[2 * v + cls(x0, 4 * (uint64_t)hq)];
                                coef[v][r][t - 1] = to_dev(c);
                            }
                        }
                    }
                    cp3[p] = coef;
                    gin[p] = Gh[p]; hin[p] = Hh[p];
                    gout[p] = as<PtD>(B.Gp[nxt]); hout[p] = as<PtD>(B.Hp[nxt]);
                    Gh[p] = B.Gp[nxt].p; Hh[p] = B.Hp[nxt].p;
                }
                ProofBufs &B0 = ws.pb[0];
                B0.f3tab.grow((size_t)P * ipp_fold3_table_bytes(hq, (uint32_t)starts.size()));
                launch_ipp_fold3(gin, hin, gfmt, hq, (uint32_t)starts.size(), starts.data(), cp3, gout, hout, P,
                                 B0.f3tab.p, B0.f3tab.cap, B0.fold3_stage, st);
                cur = nxt;
                gfmt = MSM_CACHED;
                niels_level(h);
                depth = 0;
            }
        }
        len = h;
        anz = std::min(anz, h);
    }
    for (int p = 0; p < P; p++) {
        ProofBufs &B = ws.pb[p];
        BPG_HIP(hipMemcpyAsync(B.small_host + 1010, B.a.p, sizeof(ScD), hipMemcpyDeviceToHost, st));
        BPG_HIP(hipMemcpyAsync(B.small_host + 1011, B.b.p, sizeof(ScD), hipMemcpyDeviceToHost, st));
    }
    Point Gfin, Hfin;   // sharded: this rank's last generator pair (weighted sum of the tail level)
    if (sharded) {
        if (!tail) throw std::runtime_error("sharded prove ended outside the IPP tail");
        ProofBufs &B = ws.pb[0];
        B.wconv.grow(2 * (size_t)M * sizeof(ScD) + 64);
        ScD *wc = as<ScD>(B.wconv);
        launch_from_mont(as<ScD>(B.wG), M, wc, st);
        launch_from_mont(as<ScD>(B.wH), M, wc + M, st);
        MsmSeg sl[2] = {{wc, Gh[0], M, 0}, {wc + M, Hh[0], M, 1}};
        MsmPlan pl = ws.msm->enqueue(sl, 2, 2, rowsLR, gfmt);
        ws.sync();
        combine_rows(Gfin, rowsLR, pl.W, pl.c);
        combine_rows(Hfin, rowsLR + pl.W, pl.W, pl.c);
    }
    ws.sync();
    std::vector<Scalar> fa(P), fb(P);
    for (int p = 0; p < P; p++) {
        fa[p] = from_dev(ws.pb[p].small_host[1010]);
        fb[p] = from_dev(ws.pb[p].small_host[1011]);
    }
    if (sharded) {
        // the last lg(world) rounds over one lane per rank (global lane i =
        // rank), dalek's InnerProductProof::create on the host: true
        // generators G_i = lam * Gf_i * Ghat_i, H_i = mu * y^-i * Gf_i * Hhat_i
        const Scalar gf = rank < n ? Scalar::one() : u[0];
        Point t;
        mul_var(t, lam[0] * gf, Gfin); Gfin = t;
        mul_var(t, mu[0] * sc_pow_u64(y_inv[0], rank) * gf, Hfin); Hfin = t;
        std::vector<uint8_t> send(128), recv(128 * (size_t)world);
        fa[0].to_bytes(send.data()); fb[0].to_bytes(send.data() + 32);
        ristretto_compress(send.data() + 64, Gfin);
        ristretto_compress(send.data() + 96, Hfin);
        (*ag)(send.data(), send.size(), recv.data());
        std::vector<Scalar> va(world), vb(world);
        std::vector<Point> vG(world), vH(world);
        for (uint32_t r = 0; r < world; r++) {
            const uint8_t *q = recv.data() + 128 * (size_t)r;
            va[r] = Scalar::reduce(q);
            vb[r] = Scalar::reduce(q + 32);
            if (!ristretto_decompress(vG[r], q + 64) || !ristretto_decompress(vH[r], q + 96))
                throw std::runtime_error("sharded prove: a rank sent an invalid generator");
        }
        Point Qp;
        mul_B(Qp, wch[0]);
        for (uint32_t L = world; L > 1; L /= 2, k++) {
            const uint32_t h = L / 2;
            Scalar cL = Scalar::zero(), cR = Scalar::zero();
            Point Lp, Rp;
            pt_identity(Lp); pt_identity(Rp);
            auto madd = [&](Point &acc, const Scalar &s, const Point &pt) { Point q, r; mul_var(q, s, pt); pt_add(r, acc, q); acc = r; };
            for (uint32_t i = 0; i < h; i++) {
                cL = cL + va[i] * vb[h + i];
                cR = cR + va[h + i] * vb[i];
                madd(Lp, va[i], vG[h + i]); madd(Lp, vb[h + i], vH[i]);
                madd(Rp, va[h + i], vG[i]); madd(Rp, vb[i], vH[h + i]);
            }
            madd(Lp, cL, Qp); madd(Rp, cR, Qp);
            uint8_t *cl = LRc[0].data() + 64 * (size_t)k, *cr = cl + 32;
            ristretto_compress(cl, Lp);
            ristretto_compress(cr, Rp);
            T[0].append_point("L", cl);
            T[0].append_point("R", cr);
            const Scalar uk = T[0].challenge_scalar("u"), uinv = sc_invert(uk);
            for (uint32_t i = 0; i < h; i++) {
                va[i] = va[i] * uk + va[h + i] * uinv;
                vb[i] = vb[i] * uinv + vb[h + i] * uk;
                Point g1, g2, h1, h2;
                mul_var(g1, uinv, vG[i]); mul_var(g2, uk, vG[h + i]); pt_add(vG[i], g1, g2);
                mul_var(h1, uk, vH[i]); mul_var(h2, uinv, vH[h + i]); pt_add(vH[i], h1, h2);
            }
        }
        fa[0] = va[0];
        fb[0] = vb[0];
    }
    ws.prof_flush();
    double t3 = now_ms();

    // R1CSProof::to_bytes (one-phase)
    std::vector<std::vector<uint8_t>> proofs(P);
    for (int p = 0; p < P; p++) {
        std::vector<uint8_t> &proof = proofs[p];
        proof.reserve(417 + 64 * (size_t)lgN);
        proof.push_back(0);
        auto put = [&](const uint8_t *q) { proof.insert(proof.end(), q, q + 32); };
        put(cA[p].data()); put(cA[p].data() + 32); put(cA[p].data() + 64);
        for (int i = 0; i < 5; i++) put(cT[p].data() + 32 * i);
        uint8_t b32[32];
        t_x[p].to_bytes(b32); put(b32);
        t_xb[p].to_bytes(b32); put(b32);
        e_bl[p].to_bytes(b32); put(b32);
        proof.insert(proof.end(), LRc[p].begin(), LRc[p].end());
        fa[p].to_bytes(b32); put(b32);
        fb[p].to_bytes(b32); put(b32);
        ProveTimings t;
        t.commit_ms = t1 - t0;
        t.vec_ms = t2 - t1;
        t.ipp_ms = t3 - t2;
        t.total_ms = t3 - t0;
        last_timings() = t;
        if (tms) tms[p] = t;
    }
    return proofs;
}

std::vector<uint8_t> gpu_prove_rng(const PreparedCS &cs, const uint8_t *label, size_t label_len, const RngBlock &rb,
                                   ProveTimings *tm, const AllGather *ag) {
    const RngBlock *rbp = &rb;
    return gpu_prove_lockstep(cs, label, label_len, &rbp, 1, tm, ag)[0];
}

// ------------------------------------------------------------------ verify
int gpu_verify(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V, const uint8_t *proof,
               size_t plen, const uint8_t entropy[32]) {
    return gpu_verify_shard(cs, label, label_len, V, proof, plen, entropy, 0, 1, nullptr);
}

// The per-proof part of Verifier::verify (verify.rs:71): parse the proof,
// replay the transcript, and build the verification scalars. The 2N
// generator scalars land in `gh` (device, canonical: g_0..g_{N-1}, then
// h_0..h_{N-1}); the proof's ns small points (A_I1, A_O1, S1, V_i, T_*,
// L_k, R_k) are decompressed to `pts` (an invalid encoding clears *ok_dev)
// and their scalars, with those of B and B_blinding, go to `vt`. Ends with
// the stream synchronised and *ok_host holding the decompression verdict.
// Returns 0 when a format or transcript check rejects the proof.
struct VerifyTerms {
    uint32_t ns = 0;
    std::vector<Scalar> ss;   // scalars of the small points
    Scalar sB, sBb;           // of B and B_blinding
};
// acc (batch verification): the g / h scalars weighted by rho are added into
// acc (written when first) instead of stored in gh, on the device and only if
// the proof's points decompressed (ok_dev)
static int verify_terms(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                        const uint8_t *proof, size_t plen, const uint8_t entropy[32], Workspace &ws, ScD *gh,
                        NielsD *pts, int *ok_dev, int *ok_host, VerifyTerms &vt, ScD *acc = nullptr,
                        const Scalar *rho = nullptr, bool first = false) {
    const uint32_t n = cs.n, m = cs.m, N = cs.N;
    hipStream_t st = ws.st;
    // R1CSProof::from_bytes
    if (plen < 1 || proof[0] != 0) return 0;
    const uint8_t *p = proof + 1;
    size_t rem = plen - 1;
    if (rem % 32 != 0 || rem < 11 * 32) return 0;
    const uint8_t *cAI = p, *cAO = p + 32, *cS = p + 64, *cT = p + 96;
    Scalar tx, txb, ebl, pa, pb;
    if (!Scalar::from_canonical(p + 256, tx) || !Scalar::from_canonical(p + 288, txb) ||
        !Scalar::from_canonical(p + 320, ebl))
        return 0;
    const uint8_t *ipp = p + 352;
    size_t ne = (rem - 352) / 32;
    if (ne < 2 || (ne - 2) % 2) return 0;
    uint32_t lgn = (uint32_t)((ne - 2) / 2);
    if (lgn >= 32) return 0;
    if (!Scalar::from_canonical(ipp + 64 * lgn, pa) || !Scalar::from_canonical(ipp + 64 * lgn + 32, pb)) return 0;
    if (N != (1u << lgn)) return 0;
    ws.tabs.grow(8 * 40 * sizeof(ScD));
    auto is_zero32 = [](const uint8_t *b) { uint8_t a = 0; for (int i = 0; i < 32; i++) a |= b[i]; return a == 0; };

    Transcript T(label, label_len);
    T.append_message("dom-sep", (const uint8_t *)"r1cs v1", 7);
    for (uint32_t i = 0; i < m; i++) T.append_point("V", V + 32 * (size_t)i);
    T.append_u64("m", m);
    if (is_zero32(cAI) || is_zero32(cAO) || is_zero32(cS)) return 0;
    T.append_point("A_I1", cAI);
    T.append_point("A_O1", cAO);
    T.append_point("S1", cS);
    T.append_message("dom-sep", (const uint8_t *)"r1cs-1phase", 11);
    const uint8_t zero32[32] = {0};
    T.append_point("A_I2", zero32);
    T.append_point("A_O2", zero32);
    T.append_point("S2", zero32);
    Scalar y = T.challenge_scalar("y"), z = T.challenge_scalar("z");
    static const char *TL[5] = {"T_1", "T_3", "T_4", "T_5", "T_6"};
    for (int i = 0; i < 5; i++) {
        if (is_zero32(cT + 32 * i)) return 0;
        T.append_point(TL[i], cT + 32 * i);
    }
    Scalar u = T.challenge_scalar("u"), x = T.challenge_scalar("x");
    T.append_message("t_x", p + 256, 32);
    T.append_message("t_x_blinding", p + 288, 32);
    T.append_message("e_blinding", p + 320, 32);
    Scalar w = T.challenge_scalar("w");
    // device: flattened_constraints(z), y^-i
    Scalar y_inv = sc_invert(y);
    ws.yipm.grow((size_t)N * sizeof(ScD));
    pow_vector(ws, 2, y_inv, N, ws.ylo, ws.yhi, as<ScD>(ws.yipm));
    pow_vector(ws, 4, z, cs.q + 2, ws.zlo, ws.zhi, nullptr);
    ws.sync();
    ws.w.grow((size_t)cs.ncol * sizeof(ScD) + 64);
    CscDev csc{as<uint32_t>(const_cast<DBuf &>(cs.col_ptr)), as<uint32_t>(const_cast<DBuf &>(cs.col_row)),
               as<ScD>(const_cast<DBuf &>(cs.col_coeff)), as<uint32_t>(const_cast<DBuf &>(cs.short_cols)),
               as<uint32_t>(const_cast<DBuf &>(cs.long_cols)), cs.nshort, cs.nlong, cs.ncol, 3 * n};
    launch_flatten(csc, as<ScD>(ws.zlo), as<ScD>(ws.zhi), as<ScD>(ws.w), st);
    grow_partial(ws.partial, st);
    for (uint32_t col : cs.huge_cols)
        launch_flatten_huge(csc, col, cs.col_ptr_host[col], cs.col_ptr_host[col + 1], as<ScD>(ws.zlo), as<ScD>(ws.zhi),
                            as<ScD>(ws.partial), as<ScD>(ws.w), st);
    // verification_scalars
    T.append_message("dom-sep", (const uint8_t *)"ipp v1", 6);
    T.append_u64("n", N);
    std::vector<Scalar> uc(lgn), ucinv;
    for (uint32_t k = 0; k < lgn; k++) {
        if (is_zero32(ipp + 64 * k) || is_zero32(ipp + 64 * k + 32)) return 0;
        T.append_point("L", ipp + 64 * k);
        T.append_point("R", ipp + 64 * k + 32);
        uc[k] = T.challenge_scalar("u");
    }
    ucinv = uc;
    sc_batch_invert(ucinv);
    Scalar allinv = Scalar::one();
    for (auto &v : ucinv) allinv = allinv * v;
    std::vector<Scalar> u2(lgn), ui2(lgn);
    for (uint32_t k = 0; k < lgn; k++) { u2[k] = uc[k] * uc[k]; ui2[k] = ucinv[k] * ucinv[k]; }
    TranscriptRng rng(T);
    rng.finalize(entropy);
    Scalar r = rng.random_scalar();
    Scalar xx = x * x, rxx = r * xx, xxx = x * xx;
    // g, h scalars on device
    ScD *u2h = ws.small_host + 2000;
    for (uint32_t k = 0; k < lgn; k++) u2h[k] = mont(u2[k]);
    ws.small.grow(64 * sizeof(ScD) + 4096 * sizeof(ScD));
    ScD *u2d = as<ScD>(ws.small);
    if (lgn) BPG_HIP(hipMemcpyAsync(u2d, u2h, lgn * sizeof(ScD), hipMemcpyHostToDevice, st));
    ws.ynwR.grow((size_t)(n ? n : 1) * sizeof(ScD) + 64);
    // small points: A_I1, A_O1, S1, V_i, T_*, L_k, R_k
    const uint32_t ns = 3 + m + 5 + 2 * lgn;
    std::vector<uint8_t> comp((size_t)ns * 32);
    memcpy(comp.data(), cAI, 32); memcpy(comp.data() + 32, cAO, 32); memcpy(comp.data() + 64, cS, 32);
    if (m) memcpy(comp.data() + 96, V, (size_t)m * 32);
    memcpy(comp.data() + 96 + 32 * (size_t)m, cT, 160);
    for (uint32_t k = 0; k < lgn; k++) {
        memcpy(comp.data() + (8 + m + k) * (size_t)32, ipp + 64 * k, 32);
        memcpy(comp.data() + (8 + m + lgn + k) * (size_t)32, ipp + 64 * k + 32, 32);
    }
    ws.vcomp.grow((size_t)ns * 32 + 64);
    uint32_t *compd = as<uint32_t>(ws.vcomp);
    BPG_HIP(hipMemcpyAsync(compd, comp.data(), comp.size(), hipMemcpyHostToDevice, st));
    launch_decompress(compd, pts, ok_dev, ns, st);
    // g, h (after the decompression: a batch's accumulation is skipped on
    // the device for a proof whose points do not decompress)
    ws.vtab.grow((size_t)(2048 + 64) * sizeof(ScD));   // 2^min(lgn,10) + 2^(lgn-10) <= 2048 for lgn < 21
    if (lgn > 20) ws.vtab.grow((size_t)((1u << 10) + (1u << (lgn - 10))) * sizeof(ScD));
    launch_verify_gh(as<ScD>(ws.w), as<ScD>(ws.yipm), u2d, to_dev(allinv), n, N, lgn, mont(x), mont(pa), mont(pb),
                     mont(u), as<ScD>(ws.vtab), gh, as<ScD>(ws.ynwR), acc, rho ? mont(*rho) : ScD{}, first, ok_dev, st);
    grow_partial(ws.partial, st);
    ScD *dsm = u2d + 40;
    if (n) launch_dot(as<ScD>(ws.ynwR), as<ScD>(ws.w), n, as<ScD>(ws.partial), dsm, st);
    else BPG_HIP(hipMemsetAsync(dsm, 0, sizeof(ScD), st));
    // wV and wc back to the host
    ScD *hsm = ws.small_host + 2100;
    BPG_HIP(hipMemcpyAsync(hsm, dsm, sizeof(ScD), hipMemcpyDeviceToHost, st));
    std::vector<ScD> wvh(m + 1);
    BPG_HIP(hipMemcpyAsync(wvh.data(), as<ScD>(ws.w) + 3 * (size_t)n, (size_t)(m + 1) * sizeof(ScD),
                           hipMemcpyDeviceToHost, st));
    BPG_HIP(hipMemcpyAsync(ok_host, ok_dev, 4, hipMemcpyDeviceToHost, st));
    ws.sync();
    Scalar delta = from_dev(hsm[0]);
    Scalar wc = from_dev(wvh[m]);
    vt.ns = ns;
    vt.ss.assign(ns, Scalar::zero());
    vt.ss[0] = x; vt.ss[1] = xx; vt.ss[2] = xxx;
    for (uint32_t i = 0; i < m; i++) vt.ss[3 + i] = from_dev(wvh[i]) * rxx;
    const Scalar Ts[5] = {r * x, rxx * x, rxx * xx, rxx * xxx, rxx * xx * xx};
    for (int i = 0; i < 5; i++) vt.ss[3 + m + i] = Ts[i];
    for (uint32_t k = 0; k < lgn; k++) { vt.ss[8 + m + k] = u2[k]; vt.ss[8 + m + lgn + k] = ui2[k]; }
    vt.sB = w * (tx - pa * pb) + r * (xx * (wc + delta) - tx);
    vt.sBb = -ebl - r * txb;
    return 1;
}

// One shard of Verifier::verify's mega-check. Every shard replays the
// transcript and the rejection checks; shard s of S sums the generator terms
// j in [s N/S, (s+1) N/S) of G and H, shard 0 also the proof/commitment
// points and the B, B_blinding terms. The shards' partial sums add up to the
// point that must be the identity; `partial` (32 B, compressed) receives this
// shard's part. Returns 1 (partial written, or accept when S == 1), 0 reject.
int gpu_verify_shard(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                     const uint8_t *proof, size_t plen, const uint8_t entropy[32], uint32_t shard, uint32_t nshards,
                     uint8_t *partial) {
    if (nshards < 1 || shard >= nshards) throw std::runtime_error("bad shard");
    DeviceContext &ctx = DeviceContext::get(cs.device);
    const uint32_t N = cs.N;
    if (plen < 1 || proof[0] != 0) return 0;
    std::shared_ptr<const GenSet> gs = ctx.gens(N, 0, 1, true);
    Workspace &ws = thread_workspace(cs.device);
    hipStream_t st = ws.st;
    ws.gh.grow((size_t)2 * N * sizeof(ScD) + 64);
    const uint32_t ns_max = 3 + cs.m + 5 + 2 * 32;
    ws.pts.grow(2 * (size_t)ns_max * sizeof(NielsD) + 64);   // points, then their negations
    ws.okflag.grow(64);
    int one = 1, ok = 0;
    BPG_HIP(hipMemcpyAsync(ws.okflag.p, &one, 4, hipMemcpyHostToDevice, st));
    VerifyTerms vt;
    if (!verify_terms(cs, label, label_len, V, proof, plen, entropy, ws, as<ScD>(ws.gh), as<NielsD>(ws.pts),
                      as<int>(ws.okflag), &ok, vt))
        return 0;
    if (!ok) return 0;
    const uint32_t ns = vt.ns;
    launch_niels_neg(as<NielsD>(ws.pts), as<NielsD>(ws.pts) + ns, ns, st);
    ws.mscal.grow((size_t)ns * sizeof(ScD) + 64);
    ScD *sscal = as<ScD>(ws.mscal);
    std::vector<ScD> ss(ns);
    for (uint32_t i = 0; i < ns; i++) ss[i] = to_dev(vt.ss[i]);
    BPG_HIP(hipMemcpyAsync(sscal, ss.data(), (size_t)ns * sizeof(ScD), hipMemcpyHostToDevice, st));
    const uint64_t j0 = (uint64_t)N * shard / nshards, j1 = (uint64_t)N * (shard + 1) / nshards;
    const uint32_t cnt = (uint32_t)(j1 - j0);
    const int64_t gneg = gs->N;   // negated generators follow each vector
    MsmSeg seg[3] = {{as<ScD>(ws.gh) + j0, gs->G + j0, cnt, 0, gneg}, {as<ScD>(ws.gh) + N + j0, gs->H + j0, cnt, 0, gneg},
                     {sscal, ws.pts.p, ns, 0, (int64_t)ns}};
    MsmPlan pl = ws.msm->enqueue(seg, shard == 0 ? 3 : 2, 1, ws.rows_host, MSM_NIELS);
    ws.sync();
    Point R;
    combine_rows(R, ws.rows_host, pl.W, pl.c);
    if (shard == 0) {   // B and B_blinding terms
        Point t1, t2;
        mul_B(t1, vt.sB); mul_B_blinding(t2, vt.sBb);
        pt_add(R, R, t1); pt_add(R, R, t2);
    }
    if (nshards == 1) return pt_is_identity(R) ? 1 : 0;
    ristretto_compress(partial, R);
    return 1;
}

// Verifier::verify for `count` proofs of one circuit with one MSM (SURVEY
// §8f "multi-proof batch verification"): proof j's verification equation
// (a point that must be the identity) is weighted by a random scalar rho_j,
// drawn from a transcript of every proof finalised with fresh entropy, and
// the weighted sum is checked at once: its 2N generator terms carry
// sum_j rho_j (g_j, h_j), accumulated on the device, and its small points
// are all proofs' points. The identity means every proof is valid (but for
// a ~1/l chance). Otherwise the set is split in halves, each checked the same
// way with fresh weights, down to pairs verified alone: one invalid proof in
// a chunk of 64 costs 1 + 2 lg 64 = 13 MSMs instead of 65 (a
// single bad proof must not buy 64 extra 2N-point MSMs). results[j] = 1
// accept, 0 reject.
static void verify_batch_set(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                             const uint8_t *proofs, size_t stride, const size_t *lens,
                             const std::vector<uint32_t> &idx, const uint8_t entropy[32], int *results) {
    if (idx.empty()) return;
    if (idx.size() <= 2) {
        for (uint32_t j : idx)
            results[j] = gpu_verify(cs, label, label_len, V, proofs + stride * (size_t)j, lens[j], entropy);
        return;
    }
    DeviceContext &ctx = DeviceContext::get(cs.device);
    const uint32_t N = cs.N;
    std::shared_ptr<const GenSet> gs = ctx.gens(N, 0, 1, true);
    Workspace &ws = thread_workspace(cs.device);
    hipStream_t st = ws.st;
    const uint32_t ns_max = 3 + cs.m + 5 + 2 * 32;
    const uint32_t count = (uint32_t)idx.size();
    ws.ghacc.grow((size_t)2 * N * sizeof(ScD) + 64);   // (verify_terms accumulates, gh is not written)
    ws.pts.grow(2 * (size_t)count * ns_max * sizeof(NielsD) + 64);
    ws.okflag.grow(64);
    // the weights: bound to every proof and to entropy the prover cannot know
    Transcript Tb((const uint8_t *)"bpg batch verify", 16);
    Tb.append_message("label", label, label_len);
    for (uint32_t j : idx) Tb.append_message("proof", proofs + stride * (size_t)j, lens[j]);
    TranscriptRng wr(Tb);
    uint8_t ent[32];
    thread_entropy().fill(ent, 32);
    for (int i = 0; i < 32; i++) ent[i] ^= entropy[i];
    wr.finalize(ent);
    std::vector<Scalar> ss_all;
    std::vector<uint32_t> in_batch;
    Scalar sB = Scalar::zero(), sBb = Scalar::zero();
    uint32_t off = 0;
    bool first = true;
    for (uint32_t j : idx) {
        const Scalar rho = wr.random_scalar();
        results[j] = 0;
        int one = 1, ok = 0;
        BPG_HIP(hipMemcpyAsync(ws.okflag.p, &one, 4, hipMemcpyHostToDevice, st));
        VerifyTerms vt;
        if (!verify_terms(cs, label, label_len, V, proofs + stride * (size_t)j, lens[j], entropy, ws,
                          as<ScD>(ws.gh), as<NielsD>(ws.pts) + off, as<int>(ws.okflag), &ok, vt, as<ScD>(ws.ghacc),
                          &rho, first) ||
            !ok)
            continue;   // rejected on its own (its g / h were not accumulated)
        first = false;
        for (uint32_t i = 0; i < vt.ns; i++) ss_all.push_back(vt.ss[i] * rho);
        sB = sB + vt.sB * rho;
        sBb = sBb + vt.sBb * rho;
        off += vt.ns;
        in_batch.push_back(j);
    }
    if (in_batch.empty()) return;
    // one MSM: the weighted generator terms and every proof's small points
    launch_niels_neg(as<NielsD>(ws.pts), as<NielsD>(ws.pts) + off, off, st);
    ws.mscal.grow((size_t)off * sizeof(ScD) + 64);
    ScD *sscal = as<ScD>(ws.mscal);
    std::vector<ScD> ss(off);
    for (uint32_t i = 0; i < off; i++) ss[i] = to_dev(ss_all[i]);
    BPG_HIP(hipMemcpyAsync(sscal, ss.data(), (size_t)off * sizeof(ScD), hipMemcpyHostToDevice, st));
    const int64_t gneg = gs->N;
    MsmSeg seg[3] = {{as<ScD>(ws.ghacc), gs->G, N, 0, gneg}, {as<ScD>(ws.ghacc) + N, gs->H, N, 0, gneg},
                     {sscal, ws.pts.p, off, 0, (int64_t)off}};
    MsmPlan pl = ws.msm->enqueue(seg, 3, 1, ws.rows_host, MSM_NIELS);
    ws.sync();
    Point R, t1, t2;
    combine_rows(R, ws.rows_host, pl.W, pl.c);
    mul_B(t1, sB); mul_B_blinding(t2, sBb);
    pt_add(R, R, t1); pt_add(R, R, t2);
    if (pt_is_identity(R)) {
        for (uint32_t j : in_batch) results[j] = 1;
        return;
    }
    // some proof is invalid: bisect, fresh weights per half
    const size_t h = in_batch.size() / 2;
    verify_batch_set(cs, label, label_len, V, proofs, stride, lens,
                     std::vector<uint32_t>(in_batch.begin(), in_batch.begin() + h), entropy, results);
    verify_batch_set(cs, label, label_len, V, proofs, stride, lens,
                     std::vector<uint32_t>(in_batch.begin() + h, in_batch.end()), entropy, results);
}
void gpu_verify_batch(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                      const uint8_t *proofs, size_t stride, const size_t *lens, uint32_t count,
                      const uint8_t entropy[32], int *results) {
    std::vector<uint32_t> idx;
    for (uint32_t j = 0; j < count; j++) {
        results[j] = 0;
        if (lens[j] <= stride) idx.push_back(j);   // a longer "proof" would read past its slot: rejected
    }
    verify_batch_set(cs, label, label_len, V, proofs, stride, lens, idx, entropy, results);
}

}  // namespace bpg
