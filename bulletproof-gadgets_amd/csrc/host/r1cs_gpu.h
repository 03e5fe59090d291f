// r1cs_gpu.h — host driver of the hot path: bulletproofs@2.1.0
// r1cs::Prover::prove (prove.rs:79) and r1cs::Verifier::verify (verify.rs:71)
// over a flattened constraint system, with every O(n) group / scalar-vector
// operation in HIP kernels (kernels.h) and the Merlin transcript + RNG on the
// host.
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "../../../include/bpg.h"
#include "../device/kernels.h"
#include "hcrypto.h"
#include "rng8.h"

namespace bpg {

using dev::DBuf;
using dev::MsmPlan;
using dev::PtD;
using dev::ScD;

// BulletproofGens::new(N, 1) (generators.rs) resident in HBM as affine
// Niels points, or the slice of it one rank of the sharded prover holds
// (point j of the set = generator j * world + rank). Immutable once built and
// shared by reference count: a proof holds its snapshot, so a larger circuit
// arriving on another thread never frees generators still in use.
struct GenSet {
    int device = 0;
    uint32_t N = 0;                 // points per vector
    uint32_t rank = 0, world = 1;
    // G, H: N points each, followed in the same allocation by their negations
    // (G[N + i] = -G[i]): a negative MSM digit gathers -G_i (MsmSeg::negofs = N)
    dev::NielsD *G = nullptr, *H = nullptr;
    // sums of H over local index ranges [a, b) (the IPP's padding lanes in
    // round 0, gpu_prove_lockstep): computed once per range on first use
    mutable std::mutex sums_mu;
    mutable std::map<std::pair<uint32_t, uint32_t>, Point> h_sums;
    // G_i + H_i (affine Niels, followed by their negations like G and H),
    // built on first use (gh_table): A_I1's lanes with a_L == a_R
    mutable dev::NielsD *GH = nullptr;
    ~GenSet();
};
// Comb tables of a generator set for the IPP's first two rounds:
// points j in [N/4, N) of G and of H, COMB_WIN x COMB_ENT (43 x 32 at the
// default COMB_BITS 6) packed affine-Niels entries of 96 B each.
struct CombTables {
    int device = 0;
    uint32_t N = 0;
    void *tabG = nullptr, *tabH = nullptr;
    size_t bytes = 0;
    ~CombTables();
};
// Fixed-base tables of the first N generators of a full set (world 1):
// FB_W windows of 2^(FB_C w) G_i and H_i with their negations, affine Niels
// (dev::launch_fb_build): the commitment and IPP round-0/1 MSM jobs then put
// all 13 windows of a point into one bucket row, 13 additions per point
// instead of 16 (~7 GB at N = 2^20).
struct FbTables {
    int device = 0;
    uint32_t N = 0;
    dev::NielsD *G = nullptr, *H = nullptr;   // FB_W x 2N points each
    size_t bytes = 0;
    ~FbTables();
};
// IPP fold strategy, per context (bpg_ctx_set_fold_tables / _pairs / _ipp_tail):
// -1 default (tables on, round triples, tail at 512 lanes), 0 off, 1 on.
// Proof bytes are identical under every strategy.
struct Strategy {
    int fold_tables = -1, fold_pairs = -1;
    // fixed-base generator tables (bpg_ctx_set_msm_tables): 1 on; 0 and -1
    // (the default) off: 5.7% slower with them in the bench, whose sixth
    // consumer they crowd out of HBM (profiles/r04l_ab.txt)
    int msm_tables = -1;
    bool fixed_base() const { return msm_tables == 1; }
    int ipp_tail = -1;   // IPP tail threshold in lanes (-1: 512)
    uint32_t tail() const;
    bool tables() const;
    bool pairs() const;
    // rounds folded together after the comb pass: 1 (one fold per round),
    // 2 (pairs) or 3 (triples: fold_pairs 2, the default)
    int group() const;
};
// Per-device state shared by all threads: the generator sets and comb
// tables (circuit-independent, so derived once), the fixed-base tables of
// PedersenGens.
struct DeviceContext {
    int device = 0;
    std::mutex mu;
    std::shared_ptr<const GenSet> full;   // the largest full set derived so far
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::shared_ptr<const GenSet>> slices;   // (N, rank, world)
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::shared_ptr<CombTables>> combs;      // (N, rank, world)
    std::map<uint32_t, std::shared_ptr<FbTables>> fbs;                                          // N
    PtD *tabB = nullptr, *tabBb = nullptr;
    PtD *Bb = nullptr;                  // B_blinding as a device point
    double gens_ms = 0, comb_ms = 0;    // time spent deriving / building (cold-setup breakdown)
    double comb_alloc_ms = 0;           // of comb_ms: allocating the table memory
    bool gens_from_cache = false;
    static DeviceContext &get(int device);
    // Thread-safe. world == 1: a full set with at least N points (grown on
    // demand); else the N / world points of rank `rank` of BulletproofGens(N).
    // verifier: never a set loaded from the on-disk cache (re-derived once).
    std::shared_ptr<const GenSet> gens(uint32_t N, uint32_t rank = 0, uint32_t world = 1, bool verifier = false);
    // Comb tables over the first N points of `gs`, built on first use and
    // cached per (N, slice); null when N < 8 or when they would not fit in
    // free HBM (tables not in use are evicted first).
    std::shared_ptr<CombTables> comb(const std::shared_ptr<const GenSet> &gs, uint32_t N);
    // Fixed-base tables over the first N points of a full set, built on
    // first use; null when sharded, when N > 2^20 (an entry's 25-bit index
    // must reach window 12) or when they would not fit in free HBM.
    std::shared_ptr<FbTables> fb(const std::shared_ptr<const GenSet> &gs, uint32_t N);
};
// On-disk cache of the derived generators: directory from
// bpg_gens_cache_dir() or env BPG_GENS_CACHE; empty = off.
void set_gens_cache_dir(const char *dir);

// Flattened circuit resident on the device (inputs in HBM before timing).
struct PreparedCS {
    int device = 0;
    uint32_t n = 0, m = 0, q = 0, N = 1, lgN = 0;
    // Sharded prover: this rank holds lanes i = j * world + rank
    // of every length-N vector; nl real lanes (i < n) and Nl = N / world.
    uint32_t rank = 0, world = 1, nl = 0, Nl = 1;
    Strategy strat;
    std::vector<Scalar> v, vb;          // high-level witness + blindings
    std::vector<uint8_t> V;             // m x 32 compressed commitments
    bool prover = true;
    DBuf aL, aR, aO, vb_dev;            // ScD arrays
    // A_I1 = <a_L, G> + <a_R, H> as one term per lane on G_i + H_i where
    // a_L_i == a_R_i (half the gates of a MiMC circuit: x + k squared) and two
    // elsewhere (one rank only): compacted scalars and their lane indices
    bool eq_split = false;
    uint32_t nE = 0, nD = 0;
    DBuf eqI, dfI;   // lane indices of the A_I1 split (a_L == a_R, the others)
    DBuf col_ptr, col_row, col_coeff, short_cols, long_cols;
    uint32_t nshort = 0, nlong = 0, ncol = 0;
    std::vector<uint32_t> huge_cols, col_ptr_host;
    // buffers for batched RNG output (grow-only, reused): device memory, or
    // pinned host memory (host = true) that the consumer's stream copies up
    mutable std::mutex slot_mu;
    mutable std::vector<uint8_t *> slot_bufs, host_slot_bufs;
    mutable size_t slot_bytes = 0, host_slot_bytes = 0;
    std::vector<uint8_t *> slots(size_t count, size_t bytes, bool host = false) const;
    ~PreparedCS();
};

// Build from a view. With cs->a_L == NULL the circuit is verifier-only.
// world > 1: the prover's witness vectors are uploaded as this rank's slice.
// reuse: a PreparedCS of an earlier statement whose device buffers and RNG
// slots are recycled (grown if needed) instead of allocated anew.
std::unique_ptr<PreparedCS> prepare_cs(const bpg_r1cs_view *cs, int device, const Strategy &strat = Strategy(),
                                       uint32_t rank = 0, uint32_t world = 1,
                                       std::unique_ptr<PreparedCS> reuse = nullptr);
// Device bytes a prepared statement holds (its arrays and RNG slots).
size_t prepared_bytes(const PreparedCS &cs);
// G_i + H_i of a full generator set (with negations at + gs.N), built on the
// stream on first use and kept with the set.
const dev::NielsD *gh_table(const GenSet &gs, hipStream_t st);

// Per-thread workspace (stream + buffers), grown on demand.
struct Workspace;
Workspace &thread_workspace(int device);
// Device bytes held by the calling thread's workspace on `device` (0: none).
size_t thread_workspace_bytes(int device);
// Free the calling thread's workspace on `device` and those finished threads
// parked (bpg_ctx_trim); their bytes. A thread's exit frees nothing: it parks
// its workspaces / producer stages for the next thread (r1cs_gpu.cpp Parked).
size_t release_thread_workspace(int device);
struct ParkStats { uint64_t workspaces_parked = 0, workspace_parks = 0, stages_parked = 0, stage_parks = 0; };
ParkStats park_stats();
// HBM admission estimates: what a workspace proving P proofs of `cs` in
// lockstep grows to, and what one Verifier::verify of a circuit of its size
// needs on a fresh workspace.
size_t consumer_bytes_estimate(const PreparedCS &cs, int P);
size_t verifier_bytes_estimate(const PreparedCS &cs);

struct ProveTimings { double rng_ms = 0, commit_ms = 0, vec_ms = 0, ipp_ms = 0, total_ms = 0; };

// All TranscriptRng draws of one proof (Prover::prove order).
struct RngBlock {
    Scalar i_bl, o_bl, s_bl;
    Scalar tb[5];                // t_1, t_3, t_4, t_5, t_6 blindings
    uint8_t *wide = nullptr;     // 2n x 64 raw bytes: s_L then s_R
    bool on_device = false;      // wide is a device buffer (batched path)
    // single proof with a device `wide`: a pinned host buffer of all 2n draws,
    // copied up in large chunks as they are drawn (no staging round trips)
    uint8_t *stage = nullptr;
};
// Per-thread staging of RNG output into device buffers.
struct ProducerStage {
    // draws per staged chunk: 8 x 16384 x 64 B = 8 MB per staging buffer, so
    // a group of eight 2^20 proofs takes 91 chunks (728 per proof before:
    // the copy calls and event polls were ~10% of a producer's time)
    static const uint32_t CHUNK = 16384;
    hipStream_t st = nullptr;                 // this producer thread's copy stream
    uint8_t *host[2] = {nullptr, nullptr};   // pinned, 8 x CHUNK x 64 B each
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipEvent_t drawn[2] = {nullptr, nullptr};   // s_L / s_R copies complete (rng_draw_group's progress)
    uint8_t *one = nullptr;                  // pinned, all draws of a one-proof group (grown)
    size_t one_cap = 0;
    // the pinned buffers hold blinding draws (s_L, s_R): zeroed on the copy
    // stream once their copies have landed; the next writer waits for it
    hipEvent_t wiped = nullptr;
    ~ProducerStage();
};
ProducerStage &producer_stage(int device);
// Free the calling thread's producer stage on `device` and the parked ones
// (bpg_ctx_trim); their pinned bytes.
size_t release_producer_stage(int device);
// Draw the RNG streams of `count` (<= 8) proofs of `cs` in lockstep. With
// dev_out the s_L | s_R draws go to out[k]->wide as device buffers, and
// `progress(v, ev)` (if given, dev_out only) is called once all s_L (v = 0)
// and once all s_R (v = 1) draws have been copied up: `ev` completes when
// the copies have landed (a stream that waits on it may read them).
typedef std::function<void(int, hipEvent_t)> DrawProgress;
void rng_draw_group(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *const *entropy,
                    int count, RngBlock *const *out, bool dev_out, const DrawProgress *progress = nullptr);
// The same for up to 8 proofs of DIFFERENT prepared statements (lockstep
// after each statement's first draw); wide draws go to device buffers.
void rng_draw_multi(const PreparedCS *const *cs, const uint8_t *label, size_t label_len,
                    const uint8_t *const *entropy, int count, RngBlock *const *out);
// Collective of the sharded prover: every rank contributes `bytes` and
// receives world x bytes in rank order (an all-gather; the caller supplies
// it, e.g. torch.distributed over RCCL).
typedef std::function<void(const void *send, size_t bytes, void *recv)> AllGather;
// Prover::prove. Returns proof bytes (R1CSProof::to_bytes, one-phase layout).
std::vector<uint8_t> gpu_prove(const PreparedCS &cs, const uint8_t *label, size_t label_len,
                               const uint8_t entropy[32], ProveTimings *tm = nullptr, const AllGather *ag = nullptr);
// Prover::prove after the RNG phase (the device part and the transcript).
// With cs.world > 1 every rank runs this on its slice and `ag` exchanges the
// partial sums; all ranks return the same proof bytes.
std::vector<uint8_t> gpu_prove_rng(const PreparedCS &cs, const uint8_t *label, size_t label_len, const RngBlock &rb,
                                   ProveTimings *tm = nullptr, const AllGather *ag = nullptr);
// Commitment MSMs of a single proof enqueued while its TranscriptRng was
// still being drawn (gpu_prove): A_I1 / A_O1 (no RNG input) before the
// draws, <s_L, G> and <s_R, H> as soon as each half is on the device. Window
// rows in the calling thread's pinned row buffer at the offsets below.
struct CommitPre {
    MsmPlan A, S[2];
    static const size_t ROWS_A = 0, ROWS_S0 = 256, ROWS_S1 = 384;
};
static const int MAX_LOCKSTEP = 4;   // proofs per lockstep step
// The same for P (<= MAX_LOCKSTEP = 4) proofs of one circuit in lockstep on
// the calling thread's stream (one MSM job per IPP step for all of them);
// tms: P entries or null. P must be 1 when sharded. pre: P = 1 and the
// commitment jobs already enqueued on this thread's stream (s_L, s_R reduced
// into its proof buffers).
std::vector<std::vector<uint8_t>> gpu_prove_lockstep(const PreparedCS &cs, const uint8_t *label, size_t label_len,
                                                     const RngBlock *const *rbs, int P, ProveTimings *tms = nullptr,
                                                     const AllGather *ag = nullptr, const CommitPre *pre = nullptr);
// The same for proofs of distinct prepared circuits of one shape (n, m, N):
// proof p's circuit is csv[p] (distinct statements, bpg_prove_statements).
std::vector<std::vector<uint8_t>> gpu_prove_lockstep(const PreparedCS *const *csv, const uint8_t *label,
                                                     size_t label_len, const RngBlock *const *rbs, int P,
                                                     ProveTimings *tms, const AllGather *ag = nullptr,
                                                     const CommitPre *pre = nullptr);
// Verifier::verify; returns 1 accept / 0 reject.
int gpu_verify(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
               const uint8_t *proof, size_t proof_len, const uint8_t entropy[32]);
// Verifier::verify for `count` proofs of one circuit with one random-linear-
// combination MSM (falls back to single verifications when the batch fails);
// results[j] = 1 accept, 0 reject.
void gpu_verify_batch(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                      const uint8_t *proofs, size_t stride, const size_t *lens, uint32_t count,
                      const uint8_t entropy[32], int *results);
// One shard of the verifier's mega-MSM (see r1cs_gpu.cpp); 1 = partial
// written to `partial` (32 B), 0 = rejected by the shared checks.
int gpu_verify_shard(const PreparedCS &cs, const uint8_t *label, size_t label_len, const uint8_t *V,
                     const uint8_t *proof, size_t proof_len, const uint8_t entropy[32], uint32_t shard,
                     uint32_t nshards, uint8_t *partial);
// Batched Pedersen commitments (V_i) on the device.
void gpu_pedersen(int device, const std::vector<Scalar> &v, const std::vector<Scalar> &vb, uint8_t *out);
// Generic MSM test hook.
int gpu_msm(int device, const uint8_t *scalars, const uint8_t *points, uint32_t n, uint8_t out[32]);

ProveTimings &last_timings();   // the calling thread's last proof

// Live kernel instrumentation (bench.py roofline): HIP events around the hot
// launches on their own stream, resolved after the stream synchronises.
struct KernelStat { uint64_t launches = 0; double total_ms = 0, alg_bytes = 0, femul = 0; };
int set_kernel_profiling(bool on);
bool get_kernel_stat(const char *name, KernelStat &out);
void reset_kernel_stats();

}  // namespace bpg
