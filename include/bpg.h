/*
 * bpg.h — C ABI of the MI355X-native Bulletproofs R1CS prover/verifier
 * (drop-in for FairAds/bulletproof-gadgets @ 2025-02-02).
 *
 * Two layers are exported by libbpg.so:
 *
 *  1. The UPWARD drop-in ABI (what the reference's FFI binds):
 *       c_prove / c_verify / free_proof  — interfaces/ios/src/lib.rs:10-66,
 *       header interfaces/ios/src/bulletproofs_ios.h:4-13.
 *     Behaviour follows src/prove.rs:37-82 and src/verify.rs:36-73 (statement
 *     text in, `.coms` text + `.proof` bytes out). The reference panics on bad
 *     input (UB across `extern fn`); here errors return NULL / false and the
 *     reason is available from bpg_last_error().
 *     NOTE: the reference header declares `int proof_len` but the Rust struct
 *     uses `usize`; this header uses size_t (what the Rust side really passes).
 *
 *  2. The INNER operator ABI at the hot-path cut (`Prover::prove`,
 *     src/prove.rs:79, and `Verifier::verify`, src/verify.rs:71): a flattened
 *     constraint system (bpg_r1cs_view) goes in, proof bytes come out. The
 *     transcript and RNG stay on the host, all group arithmetic (MSM, IPP
 *     folding, commitments, point (de)compression) and the bulk scalar-vector
 *     work run in HIP kernels on gfx950.
 *
 * All scalars cross the ABI as 32-byte little-endian strings, all points as
 * 32-byte compressed Ristretto255 encodings. Every entry point returns a
 * status (>= 0 success, < 0 error) and never throws across the boundary.
 */
#ifndef BPG_H
#define BPG_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* 1. Upward drop-in ABI (interfaces/ios/src/lib.rs:10-66)                   */
/* ------------------------------------------------------------------------ */

/* interfaces/ios/src/lib.rs:10-18 (#[repr(C)] struct ProofArtifacts). */
struct ProofArtifacts {
    const char *commitments;   /* NUL-terminated `.coms` text            */
    const uint8_t *proof;      /* proof bytes (417 + 64*lg(N))           */
    size_t proof_len;
    size_t proof_cap;
};

/* interfaces/ios/src/lib.rs:20-42 -> src/prove.rs:37 `prove`.
 * Returns NULL on any error (bpg_last_error() tells why). */
struct ProofArtifacts *c_prove(const char *name, const char *instance,
                               const char *witness, const char *gadgets);

/* interfaces/ios/src/lib.rs:44-52 -> src/verify.rs:36 `verify`.
 * true iff the proof verifies; false on rejection or on any error. */
bool c_verify(const char *name, const char *instance, const char *gadgets,
              const char *commitments, const uint8_t *proof, size_t proof_len);

/* interfaces/ios/src/lib.rs:54-66. Accepts NULL. */
void free_proof(struct ProofArtifacts *artifacts);

/* Added: thread-local description of the last error ("" if none). */
const char *bpg_last_error(void);

/* Added: prove.rs:37-82 for `count` DISTINCT statements at once (a serving
 * prover's batch). Statement k is parsed, synthesised and proved exactly as
 * c_prove(name, instances[k], witnesses[k], gadgets[k]) on a thread whose
 * thread_rng stream is seeded with seeds[k] (bpg_set_seed semantics;
 * seeds == NULL: OS entropy), and out[k] receives what that c_prove returns
 * (release with free_proof), or NULL if statement k failed. `threads` CPU
 * workers synthesise and upload statements and draw the TranscriptRng
 * streams of up to 8 statements in lockstep; min(5, threads / 2) more
 * threads (bpg_set_statements_layout overrides) drive the device, one HIP
 * stream each, proving up to four ready statements of one shape (n, m, N)
 * at once (their IPP MSM jobs merged, as in bpg_prove_batch). Statements in
 * flight are
 * capped by HBM (free memory next to the device threads' workspaces, at the
 * footprint of the first prepared statement), and finished statements' device
 * arrays are recycled for the next ones. Returns the number of
 * statements proved (bpg_last_error() names the first failure), < 0 on a
 * device error (then every out[k] is NULL). */
int bpg_prove_statements(const char *name, const char *const *instances,
                         const char *const *witnesses, const char *const *gadgets,
                         const uint64_t *seeds, uint32_t count, uint32_t threads,
                         struct ProofArtifacts **out);

/* Added: layout of later bpg_prove_statements calls of the process: device
 * threads (1-64; 0, the default: min(5, threads / 2); each call takes at
 * most one per hardware queue HIP gives the process, and fewer if HBM does not
 * hold them) and statements each proves at once (1-4; 0, the default: 4).
 * -1 if out of range. */
int bpg_set_statements_layout(uint32_t consumers, uint32_t lockstep);

/* Added: the last bpg_prove_statements of the process, per stage (ms summed
 * over threads; out[i], i < n <= 16): [0] CPU workers, [1] device consumers,
 * [2] statements in flight allowed, [3] wall ms, [4] synthesis ms, [5]
 * prepare ms (transpose + upload + commitments), [6] TranscriptRng ms, [7]
 * device prove ms, [8] worker idle ms, [9] consumer idle ms, [10] the
 * bounding stage, the one whose threads were busy the larger share of the
 * wall time (1 CPU workers, 2 device consumers), [11] statements in flight
 * HBM admits (sized from the first prepared statement), [12] GB one prepared
 * statement holds, [13] statements a device thread proved at once (the
 * layout's lockstep, lowered when HBM does not hold one device thread of
 * that many), [14] free HBM (GB) when the admission was made, [15] device
 * threads that retired because their workspace could not grow (their
 * statements were proved by the others), [16] the admission's estimate of a
 * device thread's workspace (GB), [17] the largest device-thread workspace
 * after the call (GB). A call whose free HBM does not hold one device thread
 * of one statement fails before proving with an error saying so (out[k] all
 * NULL). (n <= 18) */
int bpg_last_statements_stats(double *out, int n);

/* Added: `prover.num_constraints()` of the last c_prove on this thread
 * (the reference prints it from prove.rs:75; the CLI prints it here). */
uint64_t bpg_last_num_constraints(void);

/* Added: deterministic mode. Every `thread_rng()` draw of the reference
 * (commitment blindings gadget.rs:32, commitments.rs:28,40 and the 32-byte
 * TranscriptRng finalize entropy inside Prover::prove / Verifier::verify)
 * comes from one ChaCha20 stream keyed by `seed`, consumed in program order.
 * Applies to calls made on the calling thread after this call.
 * bpg_clear_seed() returns to OS entropy. */
void bpg_set_seed(uint64_t seed);
void bpg_clear_seed(void);

/* Added: select the HIP device used by the calling thread (default 0). */
int bpg_set_device(int device);

/* Added: on-disk cache of the derived generators (BulletproofGens::new,
 * prove.rs:78 / verify.rs:70). The SHAKE256 generator
 * chains are serial host work (~1-2 s at N = 2^20); with a cache directory
 * set, the first process derives and writes `bpg_gens_<N>.bin` there and
 * later processes load it (checked by a checksum and by recomputing the
 * first points of both chains). NULL or "" turns the cache off; default:
 * env BPG_GENS_CACHE, else off. The directory must be TRUSTED: a file is
 * loaded only if owned by the effective uid and not group/other-writable,
 * in a directory owned by that uid (or root) that group/others cannot
 * write; and only provers use a loaded set — every verifier entry point
 * re-derives the generators, since a planted set with known discrete-log
 * relations would make forged proofs verify. */
void bpg_gens_cache_dir(const char *dir);

/* ------------------------------------------------------------------------ */
/* 2. Inner operator ABI: the flattened constraint system                     */
/* ------------------------------------------------------------------------ */

/* Variable encoding inside a linear-combination term (bulletproofs r1cs
 * `Variable`): kind in the top 4 bits, index in the low 28 bits. */
#define BPG_VAR_ONE 0u        /* Variable::One()                      */
#define BPG_VAR_L 1u          /* Variable::MultiplierLeft(i)          */
#define BPG_VAR_R 2u          /* Variable::MultiplierRight(i)         */
#define BPG_VAR_O 3u          /* Variable::MultiplierOutput(i)        */
#define BPG_VAR_V 4u          /* Variable::Committed(i)               */
#define BPG_VAR(kind, idx) (((uint32_t)(kind) << 28) | ((uint32_t)(idx) & 0x0FFFFFFFu))
#define BPG_VAR_KIND(v) ((uint32_t)(v) >> 28)
#define BPG_VAR_INDEX(v) ((uint32_t)(v) & 0x0FFFFFFFu)

/* The state `Prover::prove` consumes (bulletproofs r1cs::Prover fields
 * `secrets {a_L,a_R,a_O,v,v_blinding}` and `constraints`). The verifier side
 * uses the same struct with the secret arrays set to NULL. */
typedef struct bpg_r1cs_view {
    uint32_t n;               /* multiplication gates (a_L.len())        */
    uint32_t m;               /* high-level commitments (v.len())         */
    uint32_t q;               /* linear constraints (constraints.len())  */
    uint32_t nnz;             /* total terms over all constraints        */
    const uint8_t *a_L;       /* n x 32 (prover only)                    */
    const uint8_t *a_R;       /* n x 32 (prover only)                    */
    const uint8_t *a_O;       /* n x 32 (prover only)                    */
    const uint8_t *v;         /* m x 32 raw scalars (prover only; may be
                                 non-canonical, Scalar::from_bits)        */
    const uint8_t *v_blinding;/* m x 32 (prover only)                    */
    const uint32_t *row_ptr;  /* q + 1 offsets into the term arrays      */
    const uint32_t *term_var; /* nnz encoded variables                   */
    const uint8_t *term_coeff;/* nnz x 32 coefficients (raw scalars)     */
} bpg_r1cs_view;

/* Maximum proof length for lg(N) <= 31: 417 + 64*31. */
#define BPG_MAX_PROOF_LEN (417u + 64u * 31u)

/* Opaque device context: owns the HBM-resident generator cache
 * (BulletproofGens::new, prove.rs:78) and per-call streams/workspaces. */
typedef struct bpg_ctx bpg_ctx;

bpg_ctx *bpg_ctx_create(int device);
void bpg_ctx_destroy(bpg_ctx *ctx);

/* IPP fold strategy of the calls made through `ctx` (bpg_r1cs_prove,
 * bpg_prepare; a prepared circuit keeps the strategy it was prepared with).
 * Proof bytes are identical under every strategy.
 *   fold_tables 1: comb tables of the generators fold IPP rounds 0-1 in one
 *     table pass; 0: per-round variable-base fold; -1 (default): on
 *     (tables are skipped when they do not fit in free HBM). Footprint (default build, COMB_BITS 6): generators j in [N/4, N)
 *     of G and of H, COMB_WIN (43) windows x COMB_ENT (32) entries x 96 B
 *     each, i.e. 0.75 x 43 x 32 x 96 x 2 B = ~198 KB x N per device
 *     (208 GB at N = 2^20; a sharded rank holds the tables of its N/world
 *     generators).
 *   fold_pairs 2: after the comb pass, rounds k, k+1, k+2 fold together
 *     (level k+3 from level k by a seven-scalar Straus pass; rounds k+1, k+2
 *     expand their bases into level-k points); 1: rounds fold in pairs
 *     (three-scalar Straus pass); 0: one fold per round; -1 (default): 2.
 *     The sharded prover uses the same grouping. */
int bpg_ctx_set_fold_tables(bpg_ctx *ctx, int mode);
int bpg_ctx_set_fold_pairs(bpg_ctx *ctx, int mode);
/* Fixed-base generator tables for the MSMs over the generators (the
 * commitments A_I1, A_O1, S1 and IPP rounds 0-1) of `ctx`'s calls: 13 windows
 * of 20 bits with 2^(20w) G_i, 2^(20w) H_i precomputed (and negated) for
 * the first N generators, so all windows of a point share one bucket row:
 * 13 additions per point instead of 16-17. 1 on (one rank, N <= 2^20, when
 * HBM holds them: ~7 GB at N = 2^20), 0 or -1 (the default) off: with them
 * the bench proves 5.7% slower, as the tables crowd a consumer out of HBM and
 * their gathers miss the cache the 256 MB generator set stays in. Proof bytes
 * are identical either way. */
int bpg_ctx_set_msm_tables(bpg_ctx *ctx, int mode);
/* IPP tail threshold of `ctx`'s calls: once a materialised generator level
 * has at most `lanes` points, the remaining rounds weight its points instead
 * of folding them (-1, the default: 512). Proof bytes
 * are identical for every threshold; small values exercise the fold passes on
 * small circuits. The sharded prover must end its local rounds in the tail
 * and uses max(lanes, 8). */
int bpg_ctx_set_ipp_tail(bpg_ctx *ctx, int lanes);

/* Cold-setup breakdown of the device `ctx` is on: out[0] ms spent deriving
 * (or loading) generators, out[1] ms building comb tables, out[2] 1 if the
 * generators came from the on-disk cache, out[3] ms of out[1] spent
 * allocating the tables' memory, out[4] bytes of comb tables resident,
 * out[5] bytes of fixed-base MSM tables resident, out[6] / out[7] device
 * workspaces parked now / parked in all by exiting threads, out[8] / out[9]
 * the same for producer stages (n <= 10). A thread that proved and exits
 * frees nothing (no HIP call runs in a thread's exit, where it could race
 * the process's own teardown): its workspace waits for the next thread. */
int bpg_ctx_setup_stats(bpg_ctx *ctx, double *out, int n);
/* Release the device's cached comb tables and sharded generator slices that
 * no proof in flight holds, and the batch worker pool's (and the caller's)
 * per-thread device workspaces and those exited threads parked (they are
 * rebuilt on next use): lets another process or circuit size on the same GPU
 * have the HBM. Call it between batches. Returns the bytes released, < 0 on
 * error. */
int64_t bpg_ctx_trim(bpg_ctx *ctx);

/* Ensure G_i, H_i for i < capacity are resident (BulletproofGens::new(cap,1),
 * bulletproofs@2.1.0 generators.rs). */
int bpg_gens_ensure(bpg_ctx *ctx, uint32_t capacity);

/* Pedersen commitments V_i = v_i*B + vb_i*B_blinding (PedersenGens::commit,
 * used by Prover::commit at commitments.rs:28,40 and gadget.rs:32). */
int bpg_pedersen_commit(bpg_ctx *ctx, const uint8_t *v, const uint8_t *vb,
                        uint32_t count, uint8_t *V_out);

/* Hot path: bulletproofs r1cs::Prover::prove (prove.rs:79) for a one-phase
 * circuit, preceded by the transcript prefix Transcript::new(label),
 * r1cs_domain_sep and one append_point("V") per commitment (V computed on
 * device from v/v_blinding and returned in V_out, m x 32).
 * `entropy` is the 32-byte input of TranscriptRngBuilder::finalize.
 * Writes proof bytes (R1CSProof::to_bytes, prove.rs:81). */
int bpg_r1cs_prove(bpg_ctx *ctx, const uint8_t *label, size_t label_len,
                   const bpg_r1cs_view *cs, const uint8_t entropy[32],
                   uint8_t *proof_out, size_t proof_cap, size_t *proof_len,
                   uint8_t *V_out);

/* Hot path: bulletproofs r1cs::Verifier::verify (verify.rs:71). `V` holds
 * the m compressed commitments in commit order. Returns 1 = accept,
 * 0 = reject, < 0 = error. */
int bpg_r1cs_verify(bpg_ctx *ctx, const uint8_t *label, size_t label_len,
                    const bpg_r1cs_view *cs, const uint8_t *V,
                    const uint8_t *proof, size_t proof_len,
                    const uint8_t entropy[32]);

/* Multi-GPU proving of ONE proof (north_star "the MSM shards
 * by scalar/point slice across the GPUs"): call on every rank r < world
 * (world a power of two, N >= 8 * world) with the same arguments. Rank r
 * holds lanes i = j * world + r of every length-N vector (a_L, a_R, a_O,
 * s_L, s_R, the generators, l(x), r(x)); an IPP round pairs lane i with
 * i + N/2^(k+1), a multiple of world, so the commitment MSMs, t(x) and the
 * first lg(N / world) IPP rounds are rank-local. Exchanges, all 32-byte
 * values gathered from every rank and summed on the host (a Ristretto sum is
 * not an RCCL reduction op): the commitment partials (A_I1, A_O1, S1), the
 * t(x) partials, per IPP round the partial L and R, and once the last
 * lane's (a, b, G, H); the final lg(world) rounds run on the host. Every
 * rank runs the transcript and the TranscriptRng itself, so no broadcast is
 * needed; all ranks return the same proof, byte-identical to
 * bpg_r1cs_prove's. `allgather(user, send, bytes, recv)` must place every
 * rank's `bytes` in rank order into recv (world * bytes) and return 0. */
typedef int (*bpg_allgather_fn)(void *user, const void *send, size_t bytes,
                                void *recv);
int bpg_r1cs_prove_sharded(bpg_ctx *ctx, const uint8_t *label, size_t label_len,
                           const bpg_r1cs_view *cs, const uint8_t entropy[32],
                           uint32_t rank, uint32_t world,
                           bpg_allgather_fn allgather, void *user,
                           uint8_t *proof_out, size_t proof_cap,
                           size_t *proof_len, uint8_t *V_out);

/* Multi-GPU verification: shard `shard` of `nshards` of
 * Verifier::verify's single mega-MSM. Every shard replays the transcript and
 * the rejection checks; shard s sums the generator terms of its slice of G
 * and H (shard 0 also the proof/commitment points and the B, B_blinding
 * terms) and writes its partial sum, compressed, to `partial`. The proof is
 * valid iff every shard returns 1 and the partials add up to the identity
 * (bpg_point_sum -> 32 zero bytes). The exchange between GPUs is one
 * all-gather of 32-byte partials (RCCL has no elliptic-curve reduction).
 * Returns 1 partial written, 0 rejected, < 0 error. */
int bpg_r1cs_verify_shard(bpg_ctx *ctx, const uint8_t *label, size_t label_len,
                          const bpg_r1cs_view *cs, const uint8_t *V,
                          const uint8_t *proof, size_t proof_len,
                          const uint8_t entropy[32], uint32_t shard,
                          uint32_t nshards, uint8_t partial[32]);

/* Host-only: out = sum of `count` compressed Ristretto points (identity =
 * 32 zero bytes). Returns 0, or -1 if an input does not decompress. */
int bpg_point_sum(const uint8_t *points, uint32_t count, uint8_t out[32]);

/* Verifier::verify (verify.rs:71) of one proof against a circuit prepared by
 * bpg_prepare_verifier (constraint matrix already resident: no per-call
 * transposition or upload), on the calling thread. nshards == 1: returns
 * 1 accept / 0 reject (`partial` may be NULL). nshards > 1: shard `shard` of
 * the mega-MSM exactly as bpg_r1cs_verify_shard (1 partial written, 0
 * rejected). < 0 on error. Every rank of a sharded verification prepares the
 * whole circuit once and then exchanges one 32-byte partial per proof. */
typedef struct bpg_prepared bpg_prepared;
int bpg_verify_prepared(bpg_prepared *p, const uint8_t *label, size_t label_len,
                        const uint8_t *V, const uint8_t *proof, size_t proof_len,
                        const uint8_t entropy[32], uint32_t shard, uint32_t nshards,
                        uint8_t *partial);

/* Prepared (HBM-resident) circuit for repeated proving: uploads a_L/a_R/a_O
 * and the transposed constraint matrix once. */
bpg_prepared *bpg_prepare(bpg_ctx *ctx, const bpg_r1cs_view *cs);
void bpg_prepared_free(bpg_prepared *p);
/* The same for verification only (witness fields of `cs` ignored): the
 * handle bpg_verify_batch takes (the prover's layout omits the constant
 * column, Variable::One, that Verifier::verify flattens). */
bpg_prepared *bpg_prepare_verifier(bpg_ctx *ctx, const bpg_r1cs_view *cs);

/* bpg_r1cs_prove_sharded with the circuit prepared once (HBM-resident) for
 * repeated single-proof proving: bpg_prepare_shard uploads this rank's slice
 * (world == 1: the whole circuit), bpg_prove_prepared proves one proof on the
 * calling thread (TranscriptRng included); `allgather` may be NULL when
 * world == 1. */
bpg_prepared *bpg_prepare_shard(bpg_ctx *ctx, const bpg_r1cs_view *cs, uint32_t rank, uint32_t world);
int bpg_prove_prepared(bpg_prepared *p, const uint8_t *label, size_t label_len,
                       const uint8_t entropy[32], bpg_allgather_fn allgather, void *user,
                       uint8_t *proof_out, size_t proof_cap, size_t *proof_len);

/* Prove `count` independent proofs of one prepared circuit (proof k uses
 * entropy + 32*k and writes proof_out + k*proof_stride) with `threads`
 * host threads sharing the device. lens[k] receives each proof length.
 * Producer threads draw the TranscriptRng streams, 8 proofs at a time (by
 * default half of the threads, at most 8 and at most one per CPU the process
 * may use: the affinity mask capped by a cgroup CPU quota); each of the
 * other threads (consumers) proves up to four proofs at once on its own HIP
 * stream, their IPP MSM jobs merged. Consumers are admitted by HBM: free
 * device memory plus what the pool's consumer workspaces already hold, minus
 * a reserve for a verifier context, at an estimated ~12 GB per consumer of
 * four proofs at N = 2^20; and at most 24 * 2^20 / N proofs are in flight
 * unless bpg_ctx_set_pipeline says otherwise. Extra threads stay idle. Proof
 * bytes do not depend on any of this. bpg_last_batch_stats reports the
 * layout used and whether the producers kept up.
 * Batch calls (this and bpg_verify_batch) run on one process-wide worker
 * pool: concurrent calls from several threads are safe and run one after
 * the other. */
int bpg_prove_batch(bpg_prepared *p, const uint8_t *label, size_t label_len,
                    const uint8_t *entropy, uint32_t count, uint32_t threads,
                    uint8_t *proof_out, size_t proof_stride, size_t *lens);

/* Pipeline layout of bpg_prove_batch on circuits prepared through `ctx`
 * afterwards (0 = automatic): `producers` TranscriptRng threads (1..8),
 * `lockstep` proofs per consumer step (1..4, default 4), `max_inflight`
 * proofs in flight (default 24 * 2^20 / N; HBM admission still applies).
 * Returns 0, -1 on an out-of-range value. */
int bpg_ctx_set_pipeline(bpg_ctx *ctx, uint32_t producers, uint32_t lockstep,
                         uint32_t max_inflight);

/* The last bpg_prove_batch of the process (out[i], i < n <= BPG_BATCH_STATS):
 * [0] producers, [1] consumers, [2] proofs per consumer step, [3] proofs in
 * flight, [4] wall ms, [5] ms until the first group of draws was ready (the
 * pipeline fill), [6] consumer ms spent waiting for a ready proof while
 * producers were still drawing (after the fill), [7] producer ms spent
 * waiting for a free slot (the device was behind), [8] producer ms drawing,
 * [9] consumer ms proving, [10] 1 if host-bound (consumers waited more than
 * a tenth of their time after the fill), [11] free HBM at the start (GB),
 * [12] estimated GB per consumer, [13] consumers the threads allowed,
 * [14] consumers HBM admitted, [15] CPUs the process may use, [16] the
 * hardware queues HIP gives the process (GPU_MAX_HW_QUEUES when HIP
 * initialised, else HIP's default 4): consumers are at most that many, one
 * stream per queue. Export GPU_MAX_HW_QUEUES=16 before anything initialises
 * HIP for the full layout. [17] the largest consumer
 * workspace after the call (GB; [12] is the admission's estimate of it). */
#define BPG_BATCH_STATS 18
int bpg_last_batch_stats(double *out, int n);

/* Verifier::verify (src/verify.rs:71) over `count` proofs of one circuit
 * prepared by bpg_prepare_verifier with `threads` host threads, each on its own HIP stream (config 5's
 * batch verification; independent proofs, so no cross-GPU exchange). Proof k
 * is proofs + k*proof_stride, lens[k] bytes; V holds the m compressed
 * commitments. results[k] = 1 accept, 0 reject. Returns 0, or < 0 on error. */
int bpg_verify_batch(bpg_prepared *p, const uint8_t *label, size_t label_len,
                     const uint8_t *V, const uint8_t *proofs, size_t proof_stride,
                     const size_t *lens, uint32_t count, uint32_t threads,
                     const uint8_t entropy[32], int *results);

/* Per-phase wall-clock timers of the last prove on this thread (ms):
 * [0] transcript+rng, [1] commit MSMs, [2] vectors, [3] IPP, [4] total.
 * After bpg_prove_batch: the batch's last proof. */
int bpg_last_timings(double *out, int n);

/* Generic device MSM: out = sum scalars[i] * points[i] (compressed in/out).
 * Test hook for the Pippenger kernel. Returns <0 if a point fails to
 * decompress. */
int bpg_msm(bpg_ctx *ctx, const uint8_t *scalars, const uint8_t *points,
            uint32_t count, uint8_t out[32]);

/* Statement synthesis only (no device work): runs the prover-side driver of
 * prove.rs:37-75 (commitment blindings drawn from the calling thread's
 * entropy source, so bpg_set_seed first for reproducible output) and exports
 * the flattened system. bpg_synth_commitments returns the `.coms` NAMES in
 * commit order, one per line (the points themselves need the device:
 * bpg_pedersen_commit). Buffers are owned by the returned handle. */
typedef struct bpg_synth bpg_synth;
bpg_synth *bpg_synthesize(const char *instance, const char *witness,
                          const char *gadgets);
/* Verifier side (verify.rs:36-69): commitments parsed from `.coms` text. */
bpg_synth *bpg_synthesize_verifier(const char *instance, const char *commitments,
                                   const char *gadgets);
const bpg_r1cs_view *bpg_synth_view(const bpg_synth *s);
const char *bpg_synth_commitments(const bpg_synth *s);
/* Verifier-side commitments (m x 32 bytes, commit order). */
const uint8_t *bpg_synth_V(const bpg_synth *s);
void bpg_synth_free(bpg_synth *s);

/* Gadget-API recorder: the r1cs::ConstraintSystem operations the reference's
 * Gadget trait callers (src/gadget.rs:7-60, tests/combine_gadgets.rs) issue,
 * recorded the way ProverBuffer / VerifierBuffer record them
 * (src/cs_buffer.rs:22-199) and flattened into a bpg_r1cs_view for
 * bpg_r1cs_prove / bpg_r1cs_verify / bpg_prepare. A Rust caller replays its
 * buffer (or implements ConstraintSystem over these calls), see
 * INTEGRATION.md. Variables are BPG_VAR encodings; a linear combination is
 * `nterms` (variable, 32-byte LE coefficient) pairs; coefficients are kept
 * as given (LinearCombination's Scalars may be unreduced, e.g. be_to_scalar
 * of 32 bytes) and reduced where the prover uses them, as dalek does. */
typedef struct bpg_lc {
    uint32_t nterms;
    const uint32_t *vars;
    const uint8_t *coeffs;   /* nterms x 32 */
} bpg_lc;
typedef struct bpg_cs bpg_cs;
/* prover != 0: r1cs::Prover semantics (assignments evaluated eagerly);
 * else r1cs::Verifier (variables only, commitments as points). */
bpg_cs *bpg_cs_create(int prover);
void bpg_cs_free(bpg_cs *cs);
/* Prover::commit(v, v_blinding) (v kept as given, Scalar::from_bits) /
 * Verifier::commit(V): the committed Variable, or < 0 on error. */
int64_t bpg_cs_commit(bpg_cs *cs, const uint8_t v[32], const uint8_t v_blinding[32]);
int64_t bpg_cs_commit_point(bpg_cs *cs, const uint8_t V[32]);
/* ConstraintSystem::multiply / allocate_multiplier (assignment NULL on the
 * verifier) / constrain. out = (left, right, output) variables. */
int bpg_cs_multiply(bpg_cs *cs, const bpg_lc *left, const bpg_lc *right, uint32_t out[3]);
int bpg_cs_allocate_multiplier(bpg_cs *cs, const uint8_t *left, const uint8_t *right, uint32_t out[3]);
int bpg_cs_constrain(bpg_cs *cs, const bpg_lc *lc);
/* The crate's gadgets as Gadget-API building blocks on a recorder:
 * MerkleTree256::assemble (merkle_tree_gadget.rs:44-56; `pattern` in the
 * reference's Display form, e.g. "H(H(W W) I)") and utils.rs:5 range_proof
 * (x_assignment NULL on the verifier). */
int bpg_cs_merkle_tree(bpg_cs *cs, const bpg_lc *root, const bpg_lc *inst, uint32_t ninst,
                       const bpg_lc *wit, uint32_t nwit, const char *pattern);
int bpg_cs_range_proof(bpg_cs *cs, const bpg_lc *x, uint32_t bits, const uint8_t *x_assignment);
/* The flattened system so far (owned by `cs`, valid until the next call on
 * it); verifier side: bpg_cs_V holds the m committed points. */
const bpg_r1cs_view *bpg_cs_view(bpg_cs *cs);
const uint8_t *bpg_cs_V(const bpg_cs *cs);

/* Native MiMC (src/mimc_hash/mimc.rs:61) and the unpadded node sponge
 * (merkle_tree_gadget.rs:106) for building statements (instances/roots). */
int bpg_mimc_hash(const uint8_t *data, size_t len, uint8_t out[32]);
int bpg_mimc_sponge(const uint8_t *blocks, uint32_t count, uint8_t out[32]);

/* Kernel instrumentation: when enabled, launches of the hot kernels are
 * bracketed by HIP events on their stream; stats accumulate per kernel name
 * ("ipp_fold_points", "msm_bucket_acc", ...) with the algorithmic HBM bytes
 * of each launch. */
int bpg_profile_enable(int on);
int bpg_kernel_stats(const char *name, uint64_t *launches, double *total_ms,
                     double *alg_bytes);
void bpg_kernel_stats_reset(void);
/* Field multiplications (GF(2^255-19), squarings included) the recorded
 * launches of `name` performed, for the VALU-side roofline. */
int bpg_kernel_femul(const char *name, double *femul);

/* Diagnostics for the batched RNG (lockstep STROBE / TranscriptRng for up
 * to 8 proofs, AVX-512 when available): self-test against the scalar
 * TranscriptRng (0 = identical output), and draws per second of one thread
 * driving `lanes` proofs. */
int bpg_rng_selftest(void);
double bpg_rng_rate(uint32_t draws, int lanes);

#ifdef __cplusplus
}
#endif
#endif /* BPG_H */
