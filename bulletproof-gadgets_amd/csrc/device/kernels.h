// kernels.h — host-callable launch wrappers for the gfx950 kernels of the
// Bulletproofs R1CS hot path (bulletproofs@2.1.0 Prover::prove /
// Verifier::verify, InnerProductProof::create). Only plain pointers cross this
// boundary; device buffers are owned by the caller (Workspace / Context).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bpg {
namespace dev {

// Device layouts (must match dev_field.h): 32 B scalars, 160 B extended
// points (X, Y, Z, T; each 10 limbs of 26/25 bits).
struct ScD { uint32_t v[8]; };
struct PtD { uint32_t v[40]; };
// affine Niels (y+x, y-x, 2dxy), Z = 1: 3 x 10 limbs + 2 pad words = 128 B
struct NielsD { uint32_t v[32]; };

#define BPG_HIP(x)                                                                 \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) throw ::bpg::dev::HipError(e_, #x, __FILE__, __LINE__); \
    } while (0)

struct HipError {
    hipError_t err;
    const char *expr, *file;
    int line;
    HipError(hipError_t e, const char *x, const char *f, int l) : err(e), expr(x), file(f), line(l) {}
};

// Live kernel timing (bench.py roofline): the calling thread's sink brackets
// single kernel launches with HIP events on their stream.
struct ProfSink {
    // alg_bytes: algorithmic HBM bytes of the launch; femul:
    // GF(p) multiplications it performs (squarings counted as multiplies)
    virtual int begin(const char *name, double alg_bytes, double femul) = 0;   // < 0: not recording
    virtual void end(int handle) = 0;
    virtual ~ProfSink() {}
};
void set_prof_sink(ProfSink *s);   // thread-local
// Wait for `ev` by polling with short sleeps. hipEventSynchronize busy-waits
// (even on hipEventBlockingSync events, measured: a host thread per stream at
// ~100% CPU), and with a 16-core CPU share the spinning threads got the whole
// process throttled while the GPU idled.
void event_wait(hipEvent_t ev);
// Set once the process has begun to exit (an atexit handler registered with
// the first device context): the destructors of process-lifetime device
// objects then leave their memory to the OS instead of calling into a HIP
// runtime that may already be tearing down.
bool process_exiting();
void mark_process_exiting();
ProfSink *prof_sink();

// -------------------------------------------------------------- points
// Generators and decompressed inputs live in HBM as affine Niels points
// (128 B, one line per random gather); folded generators are cached points
// (160 B); MSM window rows returned to the host are extended.
// out[i] = -in[i] (affine Niels: swap y+x / y-x, negate 2dxy)
// out_i = G_i + H_i as cached points (count points; affine Niels inputs)
void launch_gen_sum(const NielsD *G, const NielsD *H, PtD *out, uint32_t count, hipStream_t st);
void launch_niels_neg(const NielsD *in, NielsD *out, uint32_t count, hipStream_t st);
// out[i] = in[i] as affine Niels (cached in; one inversion per 32 points)
// cached -> affine Niels for nvec <= 8 vectors of `count` points each, one launch
void launch_cached_to_niels(const PtD *const *in, NielsD *const *out, int nvec, uint32_t count, hipStream_t st);
// out[i] = from_uniform_bytes(uniform[64*i .. 64*i+64))
void launch_gens_map(const uint8_t *uniform, NielsD *out, uint32_t count, hipStream_t st);
// out[i] = v[i]*B + vb[i]*B_blinding using fixed-base tables (64 x 8 points each)
void launch_pedersen(const ScD *v, const ScD *vb, uint32_t count, const PtD *tabB, const PtD *tabBb,
                     uint32_t *out_compressed, hipStream_t st);
void launch_compress(const PtD *in, uint32_t *out, uint32_t count, hipStream_t st);     // cached in
void launch_compress(const NielsD *in, uint32_t *out, uint32_t count, hipStream_t st);  // Niels in
void launch_decompress(const uint32_t *in, NielsD *out, int *ok, uint32_t count, hipStream_t st);

// -------------------------------------------------------------- MSM
#ifndef MSM_MAX_SEGS
#define MSM_MAX_SEGS 64   // segments per MSM job (four lockstep proofs of a round-triple IPP job: 4 x 16); the 6-bit segment field of an entry holds 0..63
#endif
#define MSM_CACHED 0   // bases are cached points (PtD)
#define MSM_NIELS 1    // bases are affine Niels points (NielsD)
struct MsmSeg {
    const ScD *scal;   // canonical scalars (< l)
    const void *base;  // PtD (cached) or NielsD, per the job's format
    uint32_t count;    // < 2^26
    uint32_t msm;      // which MSM of the job this segment contributes to
    // points from base + negofs on are the negatives of the segment's points
    // (0: no such copy). When every segment of a Niels job has one, a
    // negative digit gathers the negated base instead of negating it.
    int64_t negofs = 0;
    // fixed-base job (every segment of a Niels job sets it): the bases are
    // generator tables, window w's multiple 2^(FB_C w) P_i at base + w
    // wstride + i (and its negation at + negofs); digits of all FB_W windows
    // go to one bucket row per MSM (0: an ordinary job)
    uint64_t wstride = 0;
    // point indices of the segment's scalars (scal[k] multiplies base[idx[k]],
    // idx[k] < 2^25); null: scal[k] multiplies base[k]
    const uint32_t *idx = nullptr;
    // the bases are a generator set (or G_i + H_i): a job whose every
    // segment says so and that gathers no negated copies runs as its own
    // kernel instantiation (k_rbk_pass<true, 1, 2>, label msm_pass1_gens)
    bool gen = false;
};
// Fixed-base generator tables (DESIGN.md "Fixed-base windows"): 20-bit
// signed windows, 13 of them cover a canonical scalar.
static const int FB_C = 20, FB_W = 13;
// tab[w * 2N + i] = 2^(FB_C w) gens[i], tab[w * 2N + N + i] its negation,
// w < FB_W (affine Niels)
void launch_fb_build(const NielsD *gens, uint32_t N, NielsD *tab, hipStream_t st);
struct MsmPlan {
    int c, W, nmsm, rows, half;   // W: digit windows per scalar = rows per MSM
    uint64_t total;         // points in the job
    uint64_t E0;            // W * total
    uint32_t T;             // chunk size of the reduce-by-key passes
    int passes;
    uint64_t capE;          // capacity after the first pass
    uint32_t key_bits;
    size_t sort_tmp, scan_tmp;
    int nseg_per_row, seglen;
};
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    void grow(size_t need);
    // exactly `need` bytes on the first allocation (buffers whose size repeats,
    // e.g. a recycled prepared statement's: no 25% slack counted against the
    // HBM admission), as grow() after that
    void grow_first_exact(size_t need);
};
// Partial-sum buffer of the reducing kernels (dot products, t(x), c_L / c_R,
// huge flatten columns): 8192 scalars, the launch's reduction ticket at
// scalar RED_TICKET_WORD zeroed when (re)allocated (kernels.hip
// block_reduce_final).
static const unsigned RED_TICKET_WORD = 1024 * 6;
void grow_partial(DBuf &d, hipStream_t st);
class MsmEngine {
  public:
    explicit MsmEngine(hipStream_t st) : st_(st) {}
    ~MsmEngine();
    // Enqueue a multi-MSM job on the stream; window-row sums land in
    // `rows_host` (pinned, nmsm * W points) once the stream reaches this point.
    // rows_direct: the device view of rows_host (hipHostGetDevicePointer);
    // when given, the row kernel writes there and no copy is enqueued.
    // Returns the plan (window width c and count W are needed by the host
    // combine). Segments: at most MSM_MAX_SEGS, all bases in format `fmt`.
    MsmPlan enqueue(const MsmSeg *segs, int nseg, int nmsm, PtD *rows_host, int fmt, PtD *rows_direct = nullptr);
    // device bytes the engine holds now
    size_t bytes() const;
    // device bytes the scratch of a job of `total` points in `nmsm` MSMs grows
    // to (what enqueue reserves; HBM admission of the batched prover)
    static size_t job_bytes(uint64_t total, int nmsm, int fmt);
  private:
    void reserve(const MsmPlan &p);
    hipStream_t st_;
    DBuf keys_, vals_, keys2_, vals2_, sort_tmp_, rk_a_, rk_b_, rp_a_, rp_b_, buckets_,
        bflag_, segacc_, rows_dev_, tiles_, dhist_;
    uint32_t *tiles_host_ = nullptr;     // pinned staging of the sort tile table
    hipEvent_t tiles_ev_ = nullptr;      // its upload has completed
};

// -------------------------------------------------------------- scalar vectors
// out[j] = from_bytes_mod_order_wide(draw j * stride + offset) (canonical);
// draw i = wide[64 i .. 64 i + 64)
void launch_wide_reduce(const uint8_t *wide, uint32_t count, uint32_t stride, uint32_t offset, ScD *out,
                        hipStream_t st);
// out[i] = base^(start + i) for i < count, given base2[b] = base^(2^b), b < 32
void launch_pow_table(const ScD *base2, uint64_t start, uint32_t count, ScD *out, hipStream_t st);
// out[i] = lo[i & 1023] * hi[i >> 10] * mult (Montgomery)
void launch_pow_expand(const ScD *lo, const ScD *hi, uint32_t count, ScD mult, ScD *out, hipStream_t st);
// The power tables of a lockstep step in ONE launch (blockIdx.y = proof,
// blockIdx.z = base): lo[p][j][i] = mont(base^i), i < 1024, and
// hi[p][j][i] = mont(base^(1024 i)), i < nhi[p][j], from the Montgomery
// scalars base^(2^b) at b2[p] + 80 j + b and (base^1024)^(2^b) at
// b2[p] + 80 j + 40 + b (b < 40) that the host wrote to pinned memory: the
// kernel reads them through its device view, so no upload copy is launched.
struct PowBatch {
    const ScD *b2[4];
    ScD *lo[4][3], *hi[4][3];
    uint32_t nhi[4][3];
};
void launch_pow_tables(const PowBatch &A, int P, int nbase, hipStream_t st);
// out[p][j][i] = lo[p][j][i & 1023] * hi[p][j][i >> 10] * mult[p][j] for
// i < count (Montgomery), j < nvec, every proof's vectors in one launch
struct PowExpandBatch {
    const ScD *lo[4][2], *hi[4][2];
    ScD *out[4][2];
    ScD mult[4][2];
};
void launch_pow_expand_batch(const PowExpandBatch &A, int P, int nvec, uint32_t count, hipStream_t st);
// wide_reduce of the 2 P draw halves of a lockstep step in one launch:
// out[q][j] = draw j * stride + offset of wide[q] (q = 2 p + half)
struct WideBatch {
    const uint8_t *wide[8];
    ScD *out[8];
};
void launch_wide_reduce_batch(const WideBatch &A, int nq, uint32_t count, uint32_t stride, uint32_t offset,
                              hipStream_t st);
// flattened_constraints: columns in CSC form; out[col] = sgn * sum coeff * z^(q+1)
struct CscDev {
    const uint32_t *col_ptr;   // ncol + 1
    const uint32_t *row;       // nnz, constraint index q
    const ScD *coeff;          // nnz, canonical
    const uint32_t *short_cols, *long_cols;  // column ids by length class
    uint32_t nshort, nlong, ncol;
    uint32_t neg_from;         // columns >= neg_from are negated (V and One)
};
void launch_flatten(const CscDev &csc, const ScD *zlo, const ScD *zhi, ScD *out, hipStream_t st);
// one very long column (terms [k0, k1)) by a grid-wide reduction; partial >= 1024 scalars
void launch_flatten_huge(const CscDev &csc, uint32_t col, uint32_t k0, uint32_t k1, const ScD *zlo, const ScD *zhi,
                         ScD *partial, ScD *out, hipStream_t st);
// l(x)/r(x) coefficient vectors (VecPoly3, prover.rs)
void launch_lr_build(const ScD *aL, const ScD *aR, const ScD *sR, const ScD *wL, const ScD *wR,
                     const ScD *wO, const ScD *yp, const ScD *yip, uint32_t n, ScD *l1, ScD *r0, ScD *r1,
                     ScD *r3, hipStream_t st);
// t1..t6 of special_inner_product -> out[6]; partial is scratch (>= 6 * 1024)
void launch_tpoly(const ScD *l1, const ScD *l2, const ScD *l3, const ScD *r0, const ScD *r1, const ScD *r3,
                  uint32_t n, ScD *partial, ScD *out6, hipStream_t st);
// out = sum a[i] * b[i] (i < n)
void launch_dot(const ScD *a, const ScD *b, uint32_t n, ScD *partial, ScD *out, hipStream_t st);
// l_vec, r_vec at x (padded to N; r_vec[i] = -y^i for i >= n)
// xm, x2m: x and x^2 in Montgomery form (x * 2^256 mod l)
void launch_lr_eval(const ScD *l1, const ScD *l2, const ScD *l3, const ScD *r0, const ScD *r1, const ScD *r3,
                    const ScD *yp, uint32_t n, uint32_t N, ScD xm, ScD x2m, ScD *a, ScD *b, hipStream_t st);

// -------------------------------------------------------------- IPP
struct IppRoundArgs {
    uint32_t h, n;            // half length, number of real gates
    ScD lamG1, lamGu;         // lambda_k * Gf[i] for i < n / i >= n
    ScD muH1, muHu;           // mu_k * Gf[i] for i < n / i >= n  (times y^-i in-kernel)
};
// msm_scal[0..4h) = [aL*lamGf_R | bR*muHf_L | aR*lamGf_L | bL*muHf_R]; c_L -> msm_scal[4h],
// c_R -> msm_scal[4h+1]
// c_out: c_L, c_R (2 scalars; may be a device view of pinned host memory)
// acc = (first ? 0 : acc) + x * rho mod l (rho in Montgomery form)
// a' = a_lo u + a_hi u^-1, b' = b_lo u^-1 + b_hi u (Montgomery u, u^-1) for
// the P <= 4 proofs of a lockstep step in one launch
void launch_ipp_fold_scalars(ScD *const *a, ScD *const *b, const ScD *u, const ScD *uinv, int P, uint32_t h,
                             hipStream_t st);
// Ghat' = Ghat_L + rho * Ghat_R (rho = rho_a except lanes i < n <= h+i, which use rho_b)
// Kernel-argument block staged through pinned host memory to a device buffer
// (one per stream; the host side is rewritten only after the stream has
// passed the previous use).
struct ArgStage {
    void *dev = nullptr, *host = nullptr; hipEvent_t copied = nullptr;
};
// Gin/Hin: NielsD (in_fmt = MSM_NIELS, the generators) or PtD (MSM_CACHED)
void launch_ipp_fold_points(const void *Gin, const void *Hin, int in_fmt, uint32_t h, uint32_t n, ScD rhoG_a,
                            ScD rhoG_b, ScD rhoH_a, ScD rhoH_b, PtD *Gout, PtD *Hout, ArgStage &stage,
                            hipStream_t st);
// Two-round table fold: G2_i = G_i + c1 G_{i+h1} + c2 G_{i+2h1} + c3 G_{i+3h1}
// from comb tables of the level-0 generators j in [h1, 4h1) (likewise H).
// Table entry (w, d) of table index jj = (d+1) 2^(COMB_BITS w) P_{h1+jj},
// packed affine Niels, 96 B, at byte offset ((w*COMB_ENT+d)*ntab + jj)*96.
#define COMB_MAXRANGE 8
// Comb radix 2^COMB_BITS: signed digits in [-COMB_ENT, COMB_ENT), so a
// window keeps the COMB_ENT multiples 1..COMB_ENT of its power; COMB_WIN
// windows cover a canonical scalar (< 2^253) with its final carry.
#ifndef COMB_BITS
#define COMB_BITS 6
#endif
#define COMB_ENT (1 << (COMB_BITS - 1))
#define COMB_WIN ((253 + COMB_BITS) / COMB_BITS)
static_assert(COMB_WIN <= 64, "comb windows");
// signed radix-2^COMB_BITS digits of a canonical scalar (32 LE bytes), e[64]
// zero-filled past COMB_WIN
void comb_digits(const uint8_t s[32], int8_t e[64]);
struct CombArgs {
    const void *gens[2];       // G, H (NielsD), level 0
    const void *tab[2];        // comb tables of G, H over [h1, 4 h1)
    void *out[2];              // PtD (cached) outputs, h1 each
    uint32_t h1, ntab;         // ntab = 3 h1
    uint32_t nrange;           // lanes [rstart[r], rstart[r+1]) share digits
    uint32_t rstart[COMB_MAXRANGE];
    int8_t dig[2][COMB_MAXRANGE][3][64];   // comb_digits of c1, c2, c3
};
void launch_comb_build(const NielsD *gens, uint32_t j0, uint32_t ntab, void *tab, hipStream_t st);
void launch_ipp_comb_fold(const CombArgs &args, ArgStage &stage, hipStream_t st);
// Two-round Straus fold (no tables) from level-k generators (NielsD at level
// 0, else PtD cached): out_i = P_i + c1 P_{i+h1} + c2 P_{i+2h1} + c3 P_{i+3h1},
// i < h1, the three scalar multiples sharing one doubling chain. coef[v][r][t]
// (canonical, not Montgomery) is c_{t+1} of vector v (0 = G, 1 = H) for lanes
// [rstart[r], rstart[r+1]).
void launch_ipp_fold2(const void *Gin, const void *Hin, int in_fmt, uint32_t h1, uint32_t nrange,
                      const uint32_t *rstart, const ScD (*coef)[COMB_MAXRANGE][3], PtD *Gout, PtD *Hout,
                      ArgStage &stage, hipStream_t st);
// Round 1 of the lazy schedule: level-1 generators expanded into level 0.
struct LazyArgs {
    uint32_t h0;              // round-0 half length (pairs j, j + h0)
    ScD rGa, rGb, rHa, rHb;   // round-0 fold scalars (Montgomery), per class
};
// msm_scal[0..8h) (layout in kernels.hip), c_L -> [8h], c_R -> [8h+1]
// Round k+2 of a round triple (levels k+1, k+2 unmaterialised): each base
// expanded into four level-k points. r1/r0: rounds k+1 / k fold scalars
// (Montgomery) per vector (0 = G, 1 = H) and class (1: the pair straddles n).
struct Deep2Args {
    ScD r1[2][2], r0[2][2];
};
// msm_scal[0..16h) (layout in kernels.hip), c_L -> [16h], c_R -> [16h+1]
// The IPP round preparation of the P <= 4 proofs of a lockstep step, one
// launch: kind PREP_PLAIN (msm_scal[0..4h) = [aL*lamGf_R | bR*muHf_L |
// aR*lamGf_L | bL*muHf_R]), PREP_LAZY (8h scalars, bases one level above the
// materialised one), PREP_DEEP2 (16h, two levels above), PREP_TAIL (4M, the
// tail's weighted bases); per proof c_L -> c_out[0], c_R -> c_out[1] (may be
// a device view of pinned host memory). h (A[p].h) and M are the same for
// every proof of the step.
enum { PREP_PLAIN = 0, PREP_LAZY = 1, PREP_DEEP2 = 2, PREP_TAIL = 3 };
struct PrepBatch {
    const ScD *a[4], *b[4], *yipm[4];
    ScD *out[4], *partial[4], *c_out[4];
    IppRoundArgs A[4];
    LazyArgs lz[4];
    Deep2Args dz[4];
    const ScD *wG[4], *wH[4];
    uint32_t M;
};
void launch_ipp_prep(const PrepBatch &B, int kind, int P, hipStream_t st);
// Three-round Straus fold from level k (NielsD at level 0, else PtD):
// out_i = P_i + sum_{t=1..7} c_t P_{i + t hq}, i < hq; coef[v][r][t-1] canonical
// for lanes [rstart[r], rstart[r+1]). `tab`: odd-multiple tables,
// ipp_fold3_table_bytes(hq, nrange) bytes per proof.
size_t ipp_fold3_table_bytes(uint32_t hq, uint32_t nrange);
// P (<= 4) proofs of a lockstep step in one launch: proof p folds Gin[p],
// Hin[p] into Gout[p], Hout[p] with coef[p]; the same hq and lane ranges for
// all of them; `tab` holds P x ipp_fold3_table_bytes(hq, nrange).
void launch_ipp_fold3(const void *const *Gin, const void *const *Hin, int in_fmt, uint32_t hq, uint32_t nrange,
                      const uint32_t *rstart, const ScD (*const *coef)[COMB_MAXRANGE][7], PtD *const *Gout,
                      PtD *const *Hout, int P, void *tab, size_t tab_bytes, ArgStage &stage, hipStream_t st);
// IPP tail (DESIGN.md "IPP tail without folds"): below a few thousand lanes
// the generators stay at the last materialised level (M points each) with a
// per-point weight w_j (Montgomery form), so the round-k base i is
// sum over j = i mod 2h of w_j P_j. The round's L/R job is 4 segments of M
// scalars over that level: out = [sLG | sLH | sRG | sRH] (a point not in a
// segment's half gets 0), c_L -> out[4M], c_R -> out[4M + 1].
// after round k: w_j *= rho (Montgomery) for the upper half (j mod 2h >= h),
// rho_b for the lanes whose pair straddles n
// r[p] = {rGa, rGb, rHa, rHb} of proof p (P <= 4 proofs, one launch)
void launch_ipp_tail_weights(ScD *const *wG, ScD *const *wH, const ScD (*r)[4], int P, uint32_t M, uint32_t h,
                             uint32_t n, hipStream_t st);
// verifier helpers
// the verifier's g / h scalars (tables: scratch of 2^min(lgn,10) + 2^(lgn-10)
// scalars) into out[0..2N), or, with acc, added into acc weighted by rho
// (written when first) if *ok (the proof's points decompressed)
void launch_verify_gh(const ScD *w, const ScD *yipm, const ScD *u2m, ScD allinv, uint32_t n, uint32_t N, uint32_t lgn,
                      ScD xm, ScD am, ScD bm, ScD um, ScD *tables, ScD *out, ScD *ynwR, ScD *acc, ScD rho_mont,
                      bool first, const int *ok, hipStream_t st);
void launch_fill_scalars(ScD *dst, ScD val, uint32_t count, hipStream_t st);
// dst[q][i] = val for q < nq, i < count, in one launch (the IPP tail weights)
void launch_fill_scalars_batch(ScD *const *dst, int nq, ScD val, uint32_t count, hipStream_t st);
// sharded prover: dst[j] = src[j * stride + offset]
void launch_gather_scalars(const ScD *src, uint32_t count, uint32_t stride, uint32_t offset, ScD *dst, hipStream_t st);
// A_I1's split scalars: out = aL[eqI[0..nE)] | aL[dfI[0..nD)] | aR[dfI[0..nD)]
void launch_eq_gather(const ScD *aL, const ScD *aR, const uint32_t *eqI, uint32_t nE, const uint32_t *dfI, uint32_t nD,
                      ScD *out, hipStream_t st);
void launch_gather_niels(const NielsD *src, uint32_t count, uint32_t stride, uint32_t offset, NielsD *dst,
                         hipStream_t st);
// Montgomery -> canonical
void launch_from_mont(const ScD *src, uint32_t count, ScD *dst, hipStream_t st);

}  // namespace dev
}  // namespace bpg
