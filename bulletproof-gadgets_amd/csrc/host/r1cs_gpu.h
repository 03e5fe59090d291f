// r1cs_gpu.h — host driver of the hot path: bulletproofs@2.1.0
// r1cs::Prover::prove (prove.rs:79) and r1cs::Verifier::verify (verify.rs:71)
// over a flattened constraint system, with every O(n) group / scalar-vector
// operation in HIP kernels (kernels.h) and the Merlin transcript + RNG on the
// host.
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/bpg.h"
#include "../device/kernels.h"
#include "hcrypto.h"
#include "rng8.h"

namespace bpg {

using dev::DBuf;
using dev::PtD;
using dev::ScD;

// Per-device state shared by all threads: generator cache in HBM
// (BulletproofGens::new(N,1) is circuit-independent, so derive once) and the
// fixed-base tables of PedersenGens.
// Comb tables of the generators for the IPP's first two rounds:
// j in [N/4, N) of G and of H, 512 packed affine-Niels entries each.
struct CombTables {
    int device = 0;
    uint32_t N = 0;
    void *tabG = nullptr, *tabH = nullptr;
    size_t bytes = 0;
    ~CombTables();
};
// Fixed-base window tables of G and H (DESIGN.md "Fixed-base MSMs"):
// [w * N + j] = 2^(16 w) P_j for w < 16, affine Niels, 4 GB at N = 2^20.
struct WinTables {
    int device = 0;
    uint32_t N = 0;
    dev::NielsD *G = nullptr, *H = nullptr;
    ~WinTables();
};
struct DeviceContext {
    int device = 0;
    std::mutex mu;
    uint32_t gens_cap = 0;
    dev::NielsD *G = nullptr, *H = nullptr;   // gens_cap points each, affine Niels
    dev::AffD *Ga = nullptr, *Ha = nullptr;   // the same points as affine (x, y): 64-B MSM gathers
    PtD *tabB = nullptr, *tabBb = nullptr;
    PtD *Bb = nullptr;                  // B_blinding as a device point
    std::shared_ptr<CombTables> comb;   // for one N at a time
    static DeviceContext &get(int device);
    void ensure_gens(uint32_t N);       // thread-safe; grows the cache
    // Tables for circuits of padded size N, built on first use; null when
    // disabled (bpg_set_fold_tables / BPG_FOLD_TABLES=0), N < 8, or when they
    // would not fit in free HBM with room left for workspaces.
    std::shared_ptr<CombTables> ensure_comb(uint32_t N);
    std::shared_ptr<WinTables> wtab;
    // Window tables for N generators (null when disabled by bpg_set_msm_fixed /
    // BPG_MSM_FIXED=0 or when they would not fit in free HBM)
    std::shared_ptr<WinTables> ensure_wtab(uint32_t N);
};
// -1 auto (env BPG_FOLD_TABLES, default on), 0 off, 1 on
void set_fold_tables(int mode);
// -1 auto (env BPG_FOLD_PAIRS, default on), 0 off, 1 on
void set_fold_pairs(int mode);
// MSM base format for the level-0 generators: -1 auto (env BPG_MSM_AFFINE,
// default off: measured no throughput gain, profiles/r01j_ab.txt), 0 affine
// Niels (128 B, 7M adds), 1 affine (64 B, 9M adds)
void set_msm_affine(int mode);
// level-0 MSMs over fixed-base window tables: -1 auto (env BPG_MSM_FIXED,
// default off: 11% slower, the 4 GB of tables defeat the cache reuse of the
// 256 MB of generators, profiles/r01l_ab.txt), 0 off, 1 on
void set_msm_fixed(int mode);

// Flattened circuit resident on the device (inputs in HBM before timing).
struct PreparedCS {
    int device = 0;
    uint32_t n = 0, m = 0, q = 0, N = 1, lgN = 0;
    std::vector<Scalar> v, vb;          // high-level witness + blindings
    std::vector<uint8_t> V;             // m x 32 compressed commitments
    bool prover = true;
    DBuf aL, aR, aO, vb_dev;            // ScD arrays
    DBuf col_ptr, col_row, col_coeff, short_cols, long_cols;
    uint32_t nshort = 0, nlong = 0, ncol = 0;
    std::vector<uint32_t> huge_cols, col_ptr_host;
    // pinned host buffers for batched RNG output (grow-only, reused)
    mutable std::mutex slot_mu;
    mutable std::vector<uint8_t *> slot_bufs;
    mutable size_t slot_bytes = 0;
    std::vector<uint8_t *> slots(size_t count, size_t bytes) const;
    ~PreparedCS();
};

// Build from a view. With cs->a_L == NULL the circuit is verifier-only.
std::unique_ptr<PreparedCS> prepare_cs(const bpg_r1cs_view *cs, int device);

// Per-thread workspace (stream + buffers), grown on demand.
struct Workspace;
Workspace &thread_workspace(int device);

struct ProveTimings { double rng_ms = 0, commit_ms = 0, vec_ms = 0, ipp_ms = 0, total_ms = 0; };

// All TranscriptRng draws of one proof (Prover::prove order).
struct RngBlock {
    Scalar i_bl, o_bl, s_bl;
    Scalar tb[5];                // t_1, t_3, t_4, t_5, t_6 blindings
    uint8_t *wide = nullptr;     // 2n x 64 raw bytes: s_L then s_R
    bool on_device = false;      // wide is a device buffer (batched path)
};
// Per-thread staging of RNG output into device buffers.
struct ProducerStage {
    static const uint32_t CHUNK = 2048;   // draws per staged chunk
    hipStream_t st = nullptr;
    uint8_t *host[2] = {nullptr, nullptr};   // pinned, 8 x CHUNK x 64 B each
    hipEvent_t ev[2] = {nullptr, nullptr};
    ~ProducerStage();
};
ProducerStage &producer_stage(int device);
// Draw the RNG streams of `count` (<= 8) proofs of `cs` in lockstep. With
// dev_out the s_L | s_R draws go to out[k]->wide as device buffers.
void rng_draw_group(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *const *entropy,
                    int count, RngBlock *const *out, bool dev_out);
// Prover::prove. Returns proof bytes (R1CSProof::to_bytes, one-phase layout).
std::vector<uint8_t> gpu_prove(const PreparedCS &cs, const uint8_t *label, size_t label_len,
                               const uint8_t entropy[32], ProveTimings *tm = nullptr);
// Prover::prove after the RNG phase (the device part and the transcript).
std::vector<uint8_t> gpu_prove_rng(const PreparedCS &cs, const uint8_t *label, size_t label_len, const RngBlock &rb,
                                   ProveTimings *tm = nullptr);
// Verifier::verify; returns 1 accept / 0 reject.
int gpu_verify(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
               const uint8_t *proof, size_t proof_len, const uint8_t entropy[32]);
// One shard of the verifier's mega-MSM (see r1cs_gpu.cpp); 1 = partial
// written to `partial` (32 B), 0 = rejected by the shared checks.
int gpu_verify_shard(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                     const uint8_t *proof, size_t proof_len, const uint8_t entropy[32], uint32_t shard,
                     uint32_t nshards, uint8_t *partial);
// Batched Pedersen commitments (V_i) on the device.
void gpu_pedersen(int device, const std::vector<Scalar> &v, const std::vector<Scalar> &vb, uint8_t *out);
// Generic MSM test hook.
int gpu_msm(int device, const uint8_t *scalars, const uint8_t *points, uint32_t n, uint8_t out[32]);

ProveTimings &last_timings();

// Live kernel instrumentation (bench.py roofline): HIP events around the hot
// launches on their own stream, resolved after the stream synchronises.
struct KernelStat { uint64_t launches = 0; double total_ms = 0, alg_bytes = 0, femul = 0; };
int set_kernel_profiling(bool on);
bool get_kernel_stat(const char *name, KernelStat &out);
void reset_kernel_stats();

}  // namespace bpg
