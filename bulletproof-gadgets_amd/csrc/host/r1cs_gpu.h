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

namespace bpg {

using dev::DBuf;
using dev::PtD;
using dev::ScD;

// Per-device state shared by all threads: generator cache in HBM
// (BulletproofGens::new(N,1) is circuit-independent, so derive once) and the
// fixed-base tables of PedersenGens.
struct DeviceContext {
    int device = 0;
    std::mutex mu;
    uint32_t gens_cap = 0;
    PtD *G = nullptr, *H = nullptr;     // gens_cap points each
    PtD *tabB = nullptr, *tabBb = nullptr;
    PtD *Bb = nullptr;                  // B_blinding as a device point
    static DeviceContext &get(int device);
    void ensure_gens(uint32_t N);       // thread-safe; grows the cache
};

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
    ~PreparedCS();
};

// Build from a view. With cs->a_L == NULL the circuit is verifier-only.
std::unique_ptr<PreparedCS> prepare_cs(const bpg_r1cs_view *cs, int device);

// Per-thread workspace (stream + buffers), grown on demand.
struct Workspace;
Workspace &thread_workspace(int device);

struct ProveTimings { double rng_ms = 0, commit_ms = 0, vec_ms = 0, ipp_ms = 0, total_ms = 0; };

// Prover::prove. Returns proof bytes (R1CSProof::to_bytes, one-phase layout).
std::vector<uint8_t> gpu_prove(const PreparedCS &cs, const uint8_t *label, size_t label_len,
                               const uint8_t entropy[32], ProveTimings *tm = nullptr);
// Verifier::verify; returns 1 accept / 0 reject.
int gpu_verify(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
               const uint8_t *proof, size_t proof_len, const uint8_t entropy[32]);
// Batched Pedersen commitments (V_i) on the device.
void gpu_pedersen(int device, const std::vector<Scalar> &v, const std::vector<Scalar> &vb, uint8_t *out);
// Generic MSM test hook.
int gpu_msm(int device, const uint8_t *scalars, const uint8_t *points, uint32_t n, uint8_t out[32]);

ProveTimings &last_timings();

// Live kernel instrumentation (bench.py roofline): HIP events around the hot
// launches on their own stream, resolved after the stream synchronises.
struct KernelStat { uint64_t launches = 0; double total_ms = 0, alg_bytes = 0; };
int set_kernel_profiling(bool on);
bool get_kernel_stat(const char *name, KernelStat &out);
void reset_kernel_stats();

}  // namespace bpg
