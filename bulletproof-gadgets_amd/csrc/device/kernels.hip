// kernels.hip — gfx950 kernels for the Bulletproofs R1CS hot path.
//
// Reference semantics (un-vendored crates pinned in Cargo.lock):
//   bulletproofs@2.1.0  r1cs/prover.rs Prover::prove, r1cs/verifier.rs,
//                       inner_product_proof.rs InnerProductProof::create,
//                       generators.rs BulletproofGens/PedersenGens
//   curve25519-dalek@3.2.0  Straus/Pippenger MSM, Ristretto encode/decode
// Design (MI355X-first, not a port): one thread per point/scalar lane,
// 64-wide waves, sort-based signed-window Pippenger (look-back-free radix
// sort + fixed-chunk reduce-by-key passes, no point atomics), Montgomery scalar
// vectors, and a weighted single-scalar IPP point fold.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "dev_field.h"
#include "kernels.h"
#include <time.h>

namespace bpg {
namespace dev {

static_assert(sizeof(ScD) == sizeof(sc), "scalar layout");
static_assert(sizeof(PtD) == sizeof(ge) && sizeof(PtD) == sizeof(gec), "point layout");
static_assert(sizeof(NielsD) == sizeof(gen) && sizeof(gen) == 128, "niels layout");

#define AS_SC(p) reinterpret_cast<sc *>(p)
#define AS_CSC(p) reinterpret_cast<const sc *>(p)
#define AS_GE(p) reinterpret_cast<ge *>(p)
#define AS_CGE(p) reinterpret_cast<const ge *>(p)
#define AS_GEC(p) reinterpret_cast<gec *>(p)
#define AS_CGEC(p) reinterpret_cast<const gec *>(p)
#define AS_GEN(p) reinterpret_cast<gen *>(p)
#define AS_CGEN(p) reinterpret_cast<const gen *>(p)

static inline unsigned nblk(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// Wave priorities (s_setprio, 0-3; 0 = the hardware default). Under the
// bench's concurrency a latency-bound kernel (window-row reduction, run
// merges, final run sums) runs ~10x its isolated time because the SIMDs'
// issue arbiter serves the VALU-bound waves of other streams first, and it
// holds its registers (225 VGPRs per row-reduction wave) and LDS all that
// time; the memory-bound sort kernels likewise. Raising their waves'
// priority lets them issue whenever they are ready and leave sooner; the
// VALU-bound kernels lose no work, only the order of issue.
//   BPG_LAT_PRIO:  row reduction, bucket segments, run merges, final run sums
//   BPG_SORT_PRIO: digit extraction and the radix-sort kernels
//   BPG_FOLD_PRIO: the Straus triple fold (one wave per SIMD, 332 VGPRs)
// Default 2 / 3 / 0: 84.45 / 84.39 vs 83.91 / 83.56 M constraints/s
// (profiles/r03r_ab_priority_stop.txt; tail 2 + sort 1: 84.14 / 84.09, sort
// 1 alone 83.99 / 83.84; the fold at 1 gave nothing more,
// r03q_ab_wave_priority.txt).
static constexpr int BPG_LAT_PRIO = 2;
static constexpr int BPG_SORT_PRIO = 3;
static constexpr int BPG_FOLD_PRIO = 0;
//   BPG_MISC_PRIO: the scalar-vector kernels between a proof's MSM jobs (IPP
//   round preparation and scalar folds, flatten, t(x), powers, draws)
//   BPG_CACHED_PRIO: MSM pass 1 over folded (cached) bases
//   BPG_COMB_PRIO: the comb-table fold (rounds 0-1)
// MSM pass 1 over the generators, the bulk of the VALU work, stays at 0: the
// throughput filler under everything on a proof's critical path. Misc 2 and
// cached 1 on top of tail 2 / sort 3: 85.28 / 85.21 vs 84.54 / 84.56 M
// (profiles/r03s_ab_priority.txt; misc 2 alone 85.14 / 84.72).
static constexpr int BPG_MISC_PRIO = 2;
static constexpr int BPG_CACHED_PRIO = 1;
static constexpr int BPG_COMB_PRIO = 0;
#define WAVE_PRIO(p) do { if constexpr ((p) > 0) __builtin_amdgcn_s_setprio((p)); } while (0)

static thread_local ProfSink *tl_sink = nullptr;
void set_prof_sink(ProfSink *s) { tl_sink = s; }
static std::atomic<bool> g_exiting(false);
bool process_exiting() { return g_exiting.load(); }
void mark_process_exiting() { g_exiting = true; }
void event_wait(hipEvent_t ev) {
    const long spin_us = 50;
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) BPG_HIP(e);
        struct timespec ts{0, spin_us * 1000};
        nanosleep(&ts, nullptr);
    }
}
ProfSink *prof_sink() { return tl_sink; }
struct ProfScope {   // brackets the launches issued while it lives
    int h = -1;
    ProfScope(const char *name, double bytes, double femul) {
        if (tl_sink && name) h = tl_sink->begin(name, bytes, femul);
    }
    ~ProfScope() { if (tl_sink && h >= 0) tl_sink->end(h); }
};

// ===========================================================================
// point kernels
// ===========================================================================
__global__ __launch_bounds__(64) void k_gens_map(const uint32_t *__restrict__ uni, gen *__restrict__ out, uint32_t count) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t *w = uni + 16 * (size_t)i;
    fe r1, r2;
    uint32_t a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { a[k] = w[k]; b[k] = w[8 + k]; }
    fe_fromw(r1, a);
    fe_fromw(r2, b);
    ge p1, p2, p;
    ristretto_elligator(p1, r1);
    ristretto_elligator(p2, r2);
    ge_add(p, p1, p2);
    gen c; ge_to_niels(c, p);
    gen_store(out + i, c);
}
void launch_gens_map(const uint8_t *uniform, NielsD *out, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_gens_map, dim3(nblk(count, 64)), dim3(64), 0, st, (const uint32_t *)uniform, AS_GEN(out), count);
    BPG_HIP(hipGetLastError());
}

// signed radix-16 digit `w` of a canonical scalar (Scalar::to_radix_16).
// Fully unrolled over the 64 nibbles with the lane's digit selected at its
// step: a lane-dependent loop bound or word index would put s in scratch.
DEVI int radix16_digit(const sc &s, int w) {
    int carry = 0, d = 0;
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const int nib = (s.v[i >> 3] >> (4 * (i & 7))) & 15;
        const int x = nib + carry;
        carry = (x + 8) >> 4;
        d = i == w ? x - (carry << 4) : d;
        if (i == 63 && w == 63) d += carry << 4;   // top digit is not recentred
    }
    return d;
}

// one wave per commitment: lane w adds the window-w table entries, then an
// LDS tree reduction (6 levels) instead of a 64-step serial chain.
__global__ __launch_bounds__(64) void k_pedersen(const sc *__restrict__ v, const sc *__restrict__ vb, uint32_t count,
                                                 const ge *__restrict__ tB, const ge *__restrict__ tBb,
                                                 uint32_t *__restrict__ out) {
    __shared__ ge sh[64];
    uint32_t idx = blockIdx.x, lane = threadIdx.x;
    if (idx >= count) return;
    sc s1, s2, t;
    sc_load(t, v + idx); sc_reduce(s1, t);
    sc_load(t, vb + idx); sc_reduce(s2, t);
    int d1 = radix16_digit(s1, lane), d2 = radix16_digit(s2, lane);
    ge acc, q;
    ge_identity(acc);
    if (d1) { ge_load(q, tB + 8 * lane + (d1 > 0 ? d1 : -d1) - 1); if (d1 < 0) ge_neg(q, q); acc = q; }
    if (d2) { ge_load(q, tBb + 8 * lane + (d2 > 0 ? d2 : -d2) - 1); if (d2 < 0) ge_neg(q, q); ge_add(acc, acc, q); }
    ge_store(&sh[lane], acc);
    for (int s = 32; s >= 1; s >>= 1) {
        __syncthreads();
        if (lane < (uint32_t)s) {
            ge a, b;
            ge_load(a, &sh[lane]); ge_load(b, &sh[lane + s]);
            ge_add(a, a, b);
            ge_store(&sh[lane], a);
        }
    }
    if (lane == 0) {
        ge r; ge_load(r, &sh[0]);
        ristretto_encode(out + 8 * (size_t)idx, r);
    }
}
void launch_pedersen(const ScD *v, const ScD *vb, uint32_t count, const PtD *tabB, const PtD *tabBb,
                     uint32_t *out_compressed, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_pedersen, dim3(count), dim3(64), 0, st, AS_CSC(v), AS_CSC(vb), count, AS_CGE(tabB),
                       AS_CGE(tabBb), out_compressed);
    BPG_HIP(hipGetLastError());
}

DEVI void load_as_cached(gec &c, const gec *p) { gec_load(c, p); }
DEVI void load_as_cached(gec &c, const gen *p) { gen q; gen_load(q, p); gen_to_cached(c, q); }
template <class P>
__global__ __launch_bounds__(64) void k_compress(const P *__restrict__ in, uint32_t *__restrict__ out, uint32_t count) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    gec c; load_as_cached(c, in + i);
    ge p; ge_from_cached(p, c);
    ristretto_encode(out + 8 * (size_t)i, p);
}
void launch_compress(const PtD *in, uint32_t *out, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_compress<gec>, dim3(nblk(count, 64)), dim3(64), 0, st, AS_CGEC(in), out, count);
    BPG_HIP(hipGetLastError());
}
void launch_compress(const NielsD *in, uint32_t *out, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_compress<gen>, dim3(nblk(count, 64)), dim3(64), 0, st, AS_CGEN(in), out, count);
    BPG_HIP(hipGetLastError());
}
__global__ __launch_bounds__(64) void k_decompress(const uint32_t *__restrict__ in, gen *__restrict__ out, int *ok, uint32_t count) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = in[8 * (size_t)i + k];
    ge p;
    bool good = ristretto_decode(p, w);
    if (!good) { ge_identity(p); atomicAnd(ok, 0); }
    // decoded points have Z = 1: affine Niels without an inversion
    gen c;
    fe_add(c.YpX, p.Y, p.X); fe_sub(c.YmX, p.Y, p.X); fe_mul(c.T2d, p.T, FE_D2);
    c.pad[0] = c.pad[1] = 0;
    gen_store(out + i, c);
}
void launch_decompress(const uint32_t *in, NielsD *out, int *ok, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_decompress, dim3(nblk(count, 64)), dim3(64), 0, st, in, AS_GEN(out), ok, count);
    BPG_HIP(hipGetLastError());
}


// ===========================================================================
// Pippenger MSM
//
// Bases are affine Niels (generators, decompressed points) or cached points
// (folded generators), one format per job. One job = up to 12 (scalar, base)
// segments feeding up to 2 MSMs. Signed c-bit windows give W digits per scalar; an entry
// (key = row * half + |d| - 1, val = point | sign) per nonzero digit is
// radix-sorted by key (k_rs_*), so each bucket is a contiguous run. Runs are
// summed by fixed chunks of RBK_T entries per thread with keys/vals staged
// through LDS (coalesced); a run that lies wholly inside one thread's chunk
// goes straight to its bucket, runs that straddle chunks leave pieces in
// two fixed slots per chunk, which the next pass reduces the same way. Buckets then fold into window rows (running sums per segment of
// buckets + a weighted correction, then a block reduction per row); the host
// combines rows with c doublings each.
// ===========================================================================
static constexpr uint32_t RBK_T = 16;        // entries per thread chunk of the run reduction
static constexpr uint32_t RBK_BLOCK = 256;
static constexpr uint32_t RBK_CHUNK = RBK_T * RBK_BLOCK;
#define MSM_MAXSEG MSM_MAX_SEGS
struct SegTab {
    const sc *scal[MSM_MAXSEG];
    const void *base[MSM_MAXSEG];
    const void *neg[MSM_MAXSEG];    // negated copies (NEGC jobs), else = base
    uint32_t gofs[MSM_MAXSEG + 1];
    uint32_t row0[MSM_MAXSEG];
    const uint32_t *idx[MSM_MAXSEG];   // point indices of the scalars (MsmSeg::idx), or null
    int n;
};
// val = sign << 31 | segment << 25 | point index within the segment: the
// digit kernel resolves the segment once per point, so the run reduction
// gathers from a per-block pointer table in LDS without searching segments
#define MSM_SEG_SHIFT 25
#define MSM_LOC_MASK ((1u << MSM_SEG_SHIFT) - 1)
static_assert(MSM_MAXSEG <= 64, "an entry's segment field is 6 bits");
// the segment holding point g: the last k < n with gofs[k] <= g (gofs[0] = 0;
// gofs staged in LDS by the caller)
DEVI int seg_of(const uint32_t *gofs, int n, uint32_t g) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (g >= gofs[mid]) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Signed c-bit windows. Entry of (point g, window w): key = row << c | slot,
// slot = |d| - 1 (< half) or half for a zero digit (a trash slot whose run is
// skipped), val = point | sign << 31. Rows are numbered window-major (row =
// w * nmsm + msm), so
// with the entries laid out [w][g] and segments ordered by MSM, the key array
// is already grouped by row: the sort only orders each row by slot.
// The same launch also clears the job's bucket flags and writes the sort's
// tile table (5 words per tile: start, end, first tile of the row, one past
// its last, row start; then each row's first tile), computed from the job's
// geometry instead of being built on the host and copied up per job.
#define TILEGEO_MAXMSM 8   // MSMs of a job whose tile table the digit launch writes (4 lockstep proofs' L and R)
struct TileGeo {
    uint32_t nt, rows, tile, TW;      // tiles, rows, entries per tile, tiles per window
    uint32_t moff[TILEGEO_MAXMSM], mtot[TILEGEO_MAXMSM], tpr[TILEGEO_MAXMSM], cum[TILEGEO_MAXMSM];
    // fixed-base jobs: MSM m's points [pmoff[m], pmoff[m] + pmtot[m]); its
    // one row holds their W windows' entries [w][point] from W pmoff[m]
    uint32_t pmoff[TILEGEO_MAXMSM], pmtot[TILEGEO_MAXMSM];
    uint8_t *bflag;                   // cleared: bflag_bytes (multiple of 16)
    uint64_t bflag_bytes;
    uint32_t *tiles;                  // null: the host wrote the table
    // the sort's first-pass histogram, counted here (null: k_rs_hist counts
    // it): block = (point tile b, part s of S); hist[d nt + w TW + b] for
    // digit d = key & (hbins - 1); parts of a tile hand their counts to the
    // tile's last part through hpart / htick (S > 1)
    uint32_t *hist, *hpart, *htick;
    uint32_t hbins, S, sub;           // bins; parts per tile; points per part
};
__global__ void k_msm_digits(SegTab T, uint32_t total, int c, int W, uint32_t nmsm, uint32_t half,
                             uint32_t *__restrict__ keys, uint32_t *__restrict__ vals, TileGeo G, uint32_t wstride) {
    WAVE_PRIO(BPG_SORT_PRIO);
    // the segment table in LDS: a per-lane (runtime) index into the kernel
    // argument struct would copy it to scratch
    __shared__ uint32_t gofs[MSM_MAXSEG + 1], srow0[MSM_MAXSEG];
    __shared__ const sc *sscal[MSM_MAXSEG];
    __shared__ const uint32_t *sidx[MSM_MAXSEG];
    uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t stride = gridDim.x * blockDim.x;
    if (threadIdx.x <= (uint32_t)T.n) gofs[threadIdx.x] = T.gofs[threadIdx.x];
    if (threadIdx.x < (uint32_t)T.n) {
        srow0[threadIdx.x] = T.row0[threadIdx.x];
        sscal[threadIdx.x] = T.scal[threadIdx.x];
        sidx[threadIdx.x] = T.idx[threadIdx.x];
    }
    __syncthreads();
    for (uint64_t q = g; q < G.bflag_bytes / 16; q += stride) reinterpret_cast<uint4 *>(G.bflag)[q] = uint4{0, 0, 0, 0};
    if (G.tiles) {
        for (uint32_t x = g; x < G.nt + G.rows; x += stride) {
            if (x < G.nt) {
                const uint32_t w = x / G.TW, rem = x % G.TW;
                uint32_t m = 0;
                while (m + 1 < nmsm && rem >= G.cum[m + 1]) m++;
                const uint32_t j = rem - G.cum[m];
                const uint32_t rs = w * total + G.moff[m];
                const uint32_t first = w * G.TW + G.cum[m];
                uint32_t *e = G.tiles + 5 * (size_t)x;
                e[0] = rs + j * G.tile;
                e[1] = rs + min(G.mtot[m], (j + 1) * G.tile);
                e[2] = first;
                e[3] = first + G.tpr[m];
                e[4] = rs;
            } else {
                const uint32_t r = x - G.nt;
                G.tiles[5 * (size_t)G.nt + r] = (r / nmsm) * G.TW + G.cum[r % nmsm];
            }
        }
    }
    extern __shared__ uint32_t lh[];   // fused histogram: [w][hbins]
    const uint32_t hmask = G.hbins - 1;
    auto point = [&](uint32_t g, bool count) {
    int si = seg_of(gofs, T.n, g);
    sc k;
    sc_load(k, sscal[si] + (g - gofs[si]));
    uint32_t carry = 0, mask = (1u << c) - 1, full = 1u << c;
    const uint32_t m = srow0[si];
    const uint32_t *ix = sidx[si];
    const uint32_t loc = (uint32_t)si << MSM_SEG_SHIFT | (ix ? ix[g - gofs[si]] : g - gofs[si]);
    for (int w = 0; w < W; w++) {
        int bit = w * c;
        int lo = bit >> 5, sh = bit & 31;
        // words lo and lo + 1 by selects (no runtime index into k.v: scratch)
        uint32_t x0 = 0, x1 = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            x0 = lo == j ? k.v[j] : x0;
            x1 = lo + 1 == j ? k.v[j] : x1;
        }
        const uint64_t x = (uint64_t)x0 | (uint64_t)x1 << 32;
        uint32_t d = (uint32_t)(x >> sh) & mask;
        d += carry;
        // rows window-major (row = w nmsm + m), or one per MSM for a
        // fixed-base job, whose entry of window w gathers table w
        const uint32_t row = wstride ? m : (uint32_t)w * nmsm + m;
        uint32_t slot = half, val = wstride ? loc + (uint32_t)w * wstride : loc;
        if (d > half) {
            uint32_t mag = full - d;
            carry = 1;
            if (mag) { slot = mag - 1; val |= 0x80000000u; }
        } else {
            carry = 0;
            if (d) slot = d - 1;
        }
        // rows contiguous: [w][g], one row per window and MSM; fixed-base:
        // [m][w][point of m]
        const size_t pos = wstride ? (size_t)W * G.pmoff[m] + (size_t)w * G.pmtot[m] + (g - G.pmoff[m])
                                   : (size_t)w * total + g;
        const uint32_t key = row << c | slot;
        keys[pos] = key;
        vals[pos] = val;
        if (count) atomicAdd(&lh[w * G.hbins + (key & hmask)], 1u);
    }
    };
    if (!G.hist) {
        if (g < total) point(g, false);
        return;
    }
    // fused first-pass histogram (window-major jobs with a device tile table)
    const uint32_t nw = (uint32_t)W * G.hbins, tid = threadIdx.x;
    for (uint32_t i = tid; i < nw; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x / G.S, part = blockIdx.x % G.S;
    uint32_t mm_ = 0;
    while (mm_ + 1 < nmsm && b >= G.cum[mm_ + 1]) mm_++;
    const uint32_t j = b - G.cum[mm_];
    const uint32_t p1 = G.moff[mm_] + min(G.mtot[mm_], (j + 1) * G.tile);
    const uint32_t q0 = G.moff[mm_] + j * G.tile + part * G.sub, q1 = min(p1, q0 + G.sub);
    for (uint32_t q = q0 + tid; q < q1; q += blockDim.x) point(q, true);
    __syncthreads();
    if (G.S == 1) {
        for (uint32_t i = tid; i < nw; i += blockDim.x)
            G.hist[(size_t)(i & hmask) * G.nt + (i / G.hbins) * G.TW + b] = lh[i];
        return;
    }
    // hand-off to the tile's last part: written-through partial stores
    // drained before the ticket add (as block_reduce_final)
    uint32_t *mine = G.hpart + (size_t)blockIdx.x * nw;
    for (uint32_t i = tid; i < nw; i += blockDim.x)
        __hip_atomic_store(mine + i, lh[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ uint32_t last;
    __syncthreads();
    if (tid == 0) {
        const uint32_t t = __hip_atomic_fetch_add(G.htick + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == G.S - 1 ? 1u : 0u;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;
    const uint32_t *parts = G.hpart + (size_t)b * G.S * nw;
    for (uint32_t i = tid; i < nw; i += blockDim.x) {
        uint32_t v = lh[i];
        for (uint32_t s2 = 0; s2 < G.S; s2++)
            if (s2 != part) v += parts[(size_t)s2 * nw + i];
        G.hist[(size_t)(i & hmask) * G.nt + (i / G.hbins) * G.TW + b] = v;
    }
    if (tid == 0) __hip_atomic_store(G.htick + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next job
}

// ---------------------------------------------------------------------------
// LSD radix sort of (key, value) pairs, 7-bit digits, written for sharing the
// chip with other streams: per-block histograms, one single-workgroup scan,
// then a stable per-block scatter — no decoupled look-back, so no block ever
// spins waiting for a block that other streams' kernels keep off the CUs.
// Stable ranking inside a wave: 7 ballots give each lane the mask of lanes
// holding its digit; rank = popcount of that mask below the lane.
// ---------------------------------------------------------------------------
// Digits are RS_BITS = 7 or 8 bits wide (8 when it saves a pass).
#define RS_MAXBINS 256
#define RS_MAXTILES (2048 + 4096)   // tiles of a job: <= 2048 full ones + one partial per row
#define RS_BLOCK 256
#define RS_ROUNDS 8
#define RS_ITER (RS_BLOCK * RS_ROUNDS)
template <int RS_BITS>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_hist(const uint32_t *__restrict__ keys, int shift,
                                                      const uint32_t *__restrict__ tiles, uint32_t nb,
                                                      uint32_t *__restrict__ hist) {
    constexpr uint32_t RS_BINS = 1u << RS_BITS;
    WAVE_PRIO(BPG_SORT_PRIO);
    __shared__ uint32_t h[RS_BINS];
    if (threadIdx.x < RS_BINS) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t t0 = tiles[5 * blockIdx.x], t1 = tiles[5 * blockIdx.x + 1];
    for (uint64_t i = t0 + threadIdx.x; i < t1; i += RS_BLOCK) atomicAdd(&h[(keys[i] >> shift) & (RS_BINS - 1)], 1u);
    __syncthreads();
    if (threadIdx.x < RS_BINS) hist[threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}
// per digit d (one block each): exclusive scan of hist[d][0..nb) in place,
// total[d] = the digit's count. 2048 counts per step, loaded up front
// (coalesced, 8 per thread), then scanned 256 at a time: wave shuffles inside
// each wave, the four waves' totals through LDS (double-buffered: one barrier
// per 256 counts).
#define RS_SCAN_K 8
__global__ __launch_bounds__(256) void k_rs_colscan(uint32_t *__restrict__ hist, uint32_t nb,
                                                    uint32_t *__restrict__ total) {
    __shared__ uint32_t wsum[2][4];
    WAVE_PRIO(BPG_SORT_PRIO);
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t *h = hist + (size_t)blockIdx.x * nb;
    uint32_t carry = 0, par = 0;
    for (uint32_t r0 = 0; r0 < nb; r0 += 256 * RS_SCAN_K) {
        uint32_t v[RS_SCAN_K];
#pragma unroll
        for (int k = 0; k < RS_SCAN_K; k++) {
            const uint32_t i = r0 + k * 256 + t;
            v[k] = i < nb ? h[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < RS_SCAN_K; k++) {
            if (r0 + k * 256 >= nb) break;   // uniform
            uint32_t x = v[k];   // inclusive scan over the wave
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                x += lane >= (uint32_t)d ? y : 0u;
            }
            if (lane == 63) wsum[par][wave] = x;
            __syncthreads();
            uint32_t before = 0, all = 0;
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t ws = wsum[par][q];
                before += q < wave ? ws : 0u;
                all += ws;
            }
            const uint32_t i = r0 + k * 256 + t;
            if (i < nb) h[i] = carry + before + x - v[k];
            carry += all;
            par ^= 1u;
        }
    }
    if (t == 0) total[blockIdx.x] = carry;
}
// Stable scatter of one block's tile, 2048 keys per iteration: wave ballots
// rank keys within their digit, the iteration is reordered by digit in LDS,
// then written out so that lanes with consecutive LDS slots of one digit
// write consecutive addresses.
// STABLE = false (the first pass of an LSD sort: it has no earlier order to
// keep, and equal keys are interchangeable in the MSM): keys are ranked
// within their digit by LDS atomics instead of the wave ballots. Every later
// pass must keep the order of the passes before it.
// Exclusive scan of one value per thread over a 256-thread block, in thread
// order: wave shuffles, then the four wave totals through `ws` (LDS, 4
// words); two barriers (the second lets the caller reuse `ws`).
DEVI uint32_t blk256_exscan(uint32_t v, uint32_t *ws) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t)d ? y : 0u;
    }
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    uint32_t before = 0;
#pragma unroll
    for (uint32_t q = 0; q < 3; q++) before += q < wave ? ws[q] : 0u;
    __syncthreads();
    return before + x - v;
}
template <int RS_BITS, bool STABLE>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_scatter(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                         int shift, const uint32_t *__restrict__ tiles, uint32_t nb,
                                                         const uint32_t *__restrict__ hist,
                                                         const uint32_t *__restrict__ total,
                                                         uint32_t *__restrict__ kout, uint32_t *__restrict__ vout) {
    constexpr uint32_t RS_BINS = 1u << RS_BITS;
    WAVE_PRIO(BPG_SORT_PRIO);
    __shared__ uint32_t base[RS_BINS], lstart[RS_BINS], tot[RS_BINS], ws[4];
    // ballot ranking only: per (round, wave) digit counts (<= 64), scanned in
    // place into offsets within the iteration (< RS_ITER): 16 bits each
    __shared__ uint16_t cnt[STABLE ? RS_ROUNDS : 1][RS_BLOCK / 64][RS_BINS];
    __shared__ uint32_t lk[RS_ITER], lv[RS_ITER];
    static_assert(RS_BLOCK == 256 && RS_BINS <= 256 && RS_ITER < 65536, "blk256_exscan, 16-bit offsets");
    const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint64_t below = (lane ? (~0ull >> (64 - lane)) : 0ull);
    // Segmented by row: this tile's row occupies tiles [r0, r1) and elements
    // from rstart; digit offsets = rstart + exclusive scan of the row's digit
    // counts + the count of the digit in the row's earlier tiles (hist holds
    // the exclusive prefix over all tiles per digit).
    const uint32_t *TL = tiles + 5 * blockIdx.x;
    const uint32_t r0 = TL[2], r1 = TL[3], rstart = TL[4];
    uint32_t p0 = 0, cr = 0;
    if (t < RS_BINS) {
        p0 = hist[t * nb + r0];
        cr = (r1 < nb ? hist[t * nb + r1] : total[t]) - p0;
    }
    const uint32_t rowpre = blk256_exscan(cr, ws);   // the row's digits before t
    if (t < RS_BINS) base[t] = rstart + rowpre + (hist[t * nb + blockIdx.x] - p0);
    const uint64_t t0 = TL[0], t1 = TL[1];
    for (uint64_t it = t0; it < t1; it += RS_ITER) {
        uint32_t kk[RS_ROUNDS], vv[RS_ROUNDS], dd[RS_ROUNDS], rk[RS_ROUNDS];
        if constexpr (!STABLE) {
            if (t < RS_BINS) tot[t] = 0;
            __syncthreads();
#pragma unroll
            for (int r = 0; r < RS_ROUNDS; r++) {
                const uint64_t idx = it + (uint64_t)r * RS_BLOCK + t;
                const bool ok = idx < t1;
                kk[r] = ok ? kin[idx] : 0u;
                vv[r] = ok ? vin[idx] : 0u;
                const uint32_t d = (kk[r] >> shift) & (RS_BINS - 1);
                dd[r] = ok ? d : 0xffffffffu;
                rk[r] = ok ? atomicAdd(&tot[d], 1u) : 0u;
            }
            __syncthreads();
            const uint32_t ex = blk256_exscan(t < RS_BINS ? tot[t] : 0u, ws);   // exclusive starts
            if (t < RS_BINS) lstart[t] = ex;
            __syncthreads();
#pragma unroll
            for (int r = 0; r < RS_ROUNDS; r++) {
                if (dd[r] != 0xffffffffu) {
                    const uint32_t pos = lstart[dd[r]] + rk[r];
                    lk[pos] = kk[r];
                    lv[pos] = vv[r];
                }
            }
            __syncthreads();
        } else {
        uint32_t *cz = reinterpret_cast<uint32_t *>(&cnt[0][0][0]);
        for (uint32_t j = t; j < RS_ROUNDS * (RS_BLOCK / 64) * RS_BINS / 2; j += RS_BLOCK) cz[j] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RS_ROUNDS; r++) {
            const uint64_t idx = it + (uint64_t)r * RS_BLOCK + t;
            const bool ok = idx < t1;
            kk[r] = ok ? kin[idx] : 0u;
            vv[r] = ok ? vin[idx] : 0u;
            const uint32_t d = (kk[r] >> shift) & (RS_BINS - 1);
            dd[r] = ok ? d : 0xffffffffu;
            uint64_t m = __ballot(ok);
#pragma unroll
            for (int b = 0; b < RS_BITS; b++) {
                const uint64_t bb = __ballot(ok && ((d >> b) & 1));
                m &= ((d >> b) & 1) ? bb : ~bb;
            }
            rk[r] = (uint32_t)__popcll(m & below);
            if (ok && rk[r] == 0) cnt[r][wave][d] = (uint16_t)__popcll(m);
        }
        __syncthreads();
        uint32_t run = 0;
        if (t < RS_BINS) {   // offsets within the iteration, (round, wave) order
            for (int r = 0; r < RS_ROUNDS; r++)
                for (int w = 0; w < RS_BLOCK / 64; w++) { const uint32_t c = cnt[r][w][t]; cnt[r][w][t] = (uint16_t)run; run += c; }
            tot[t] = run;
        }
        const uint32_t ex = blk256_exscan(run, ws);   // exclusive starts (its barriers publish cnt, tot)
        if (t < RS_BINS) lstart[t] = ex;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RS_ROUNDS; r++) {
            if (dd[r] != 0xffffffffu) {
                const uint32_t pos = lstart[dd[r]] + cnt[r][wave][dd[r]] + rk[r];
                lk[pos] = kk[r];
                lv[pos] = vv[r];
            }
        }
        __syncthreads();
        }
        const uint32_t n_it = (uint32_t)((t1 - it) < RS_ITER ? (t1 - it) : RS_ITER);
        for (uint32_t i = t; i < n_it; i += RS_BLOCK) {
            const uint32_t key = lk[i];
            const uint32_t d = (key >> shift) & (RS_BINS - 1);
            const uint32_t g = base[d] + (i - lstart[d]);
            kout[g] = key;
            vout[g] = lv[i];
        }
        __syncthreads();
        if (t < RS_BINS) base[t] += tot[t];
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// Run reduction over the sorted entries, by fixed chunks of RBK_T entries per
// thread (keys/values staged through LDS with one pad word per RBK_T, so
// thread t's entries t*T..t*T+T-1 sit at t*(T+1)+i, conflict-free). A run
// wholly inside one chunk goes straight to its bucket. Every chunk writes
// exactly two slots for the next pass — the piece of a run that began before
// it (head) and of one that continues after it (tail) — and a filler (key |
// RBK_FILL, no point) where it has none, so the next pass's input is still
// sorted and its size is known on the host: no count, no scan, one launch
// per pass. A run made only of fillers writes nothing.
// ---------------------------------------------------------------------------
#define RBK_FILL 0x80000000u
#define RBK_KEY(x) ((x) & 0x7fffffffu)
// bucket of key row << c | slot (slot < half = 2^(c-1); slot == half: trash)
DEVI uint32_t rbk_bucket(uint32_t key, int c) { return (key >> c) * (1u << (c - 1)) + (key & ((1u << (c - 1)) - 1)); }
DEVI bool rbk_trash(uint32_t key, int c) { return (key >> (c - 1)) & 1u; }
DEVI uint32_t rbk_lds(uint32_t j) { return j + j / RBK_T; }
DEVI void rbk_stage(uint32_t *sk, const uint32_t *__restrict__ keys, uint64_t base, uint64_t E, uint32_t invalid) {
    for (uint32_t k = threadIdx.x; k < RBK_CHUNK; k += RBK_BLOCK) {
        uint64_t idx = base + k;
        sk[rbk_lds(k)] = idx < E ? keys[idx] : invalid;
    }
}
// Base gathers by the job's base format: cached (160 B) or affine Niels
// (128 B, one line, 7M madd). The block's segment pointers sit in LDS:
// sptr[seg] the bases, sptr[MSM_MAXSEG + seg] their negated copies (NEGC) —
// a negative digit then gathers -P and adds it as is.
template <int FMT> struct BaseOf { typedef gec T; };
template <> struct BaseOf<MSM_NIELS> { typedef gen T; };
// pt_load from a pointer known to be global memory (the LDS table hides the
// address space; a generic pointer would compile to flat loads)
template <class P>
DEVI void pt_load_global(P &p, uint64_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(1))) const uint4 g4;
#else
    typedef const uint4 g4;   // host pass: the function is never called there
#endif
    constexpr int NQ = sizeof(P) / 16;
    const g4 *s = reinterpret_cast<const g4 *>(addr);
    uint32_t *d = reinterpret_cast<uint32_t *>(&p);
#pragma unroll
    for (int i = 0; i < NQ; i++) { const uint4 q = s[i]; d[4 * i] = q.x; d[4 * i + 1] = q.y; d[4 * i + 2] = q.z; d[4 * i + 3] = q.w; }
}
template <int FMT, bool NEGC>
DEVI void msm_load_base(typename BaseOf<FMT>::T &p, const uint64_t *sptr, uint32_t v) {
    const uint32_t si = (v >> MSM_SEG_SHIFT) & 63u;
    const uint32_t sel = NEGC ? (v >> 31) * MSM_MAXSEG + si : si;
    pt_load_global(p, sptr[sel] + (uint64_t)(v & MSM_LOC_MASK) * sizeof(typename BaseOf<FMT>::T));
}
template <bool NEGC> DEVI void msm_add_loaded(ge &acc, gen &p, bool neg) {
    if (!NEGC) gen_cneg(p, neg);
    ge_madd(acc, acc, p);
}
template <bool NEGC> DEVI void msm_add_loaded(ge &acc, gec &p, bool neg) {
    if (!NEGC) gec_cneg(p, neg);
    ge_add_c(acc, acc, p);
}
// the same into an accumulator that holds the identity: a conversion (1M)
template <bool NEGC> DEVI void msm_init_loaded(ge &acc, gen &p, bool neg) {
    if (!NEGC) gen_cneg(p, neg);
    ge_from_niels(acc, p);
}
template <bool NEGC> DEVI void msm_init_loaded(ge &acc, gec &p, bool neg) {
    if (!NEGC) gec_cneg(p, neg);
    ge_from_cached_t(acc, p);
}

// FIRST: entries are (key, signed base index) and the gather of entry i+1 is
// issued before entry i's addition; otherwise entries are slots (key or
// key|RBK_FILL, extended point at the same index) of the previous pass. A
// run's first point is converted or copied instead of being added to the
// identity (pass-1 entry 0 at 1M instead of 7M / 8M).
// Waves per SIMD each pass is compiled for: pass 1 over affine Niels bases 3
// (155 VGPRs; 4 spills 88 B per lane and measured slower,
// profiles/r02zz_ab_pass1_w4.txt), over cached bases 2, the latency-bound
// merge passes and final run sums 1 (capping them at 4 waves measured no
// gain, profiles/r02s_ab_latwaves.txt).
static constexpr int RBK_WAVES = 3, RBK_CWAVES = 2, RBK_LAT_WAVES = 1;
// KIND: 0 bases negated in registers (folded levels, cached bases, the
// merge passes), 1 negative digits gather pre-negated copies (the
// verifier's generator jobs), 2 generator jobs of the prover negated in
// registers -- the same code as 0, a kernel of its own so that its launches
// are one rocprof row and one bench label (round 6: gathering from G and H
// alone, 256 MB, instead of with their negations, 512 MB, measured +0.8% at
// a 0.5% higher clock under the chip's power limit, profiles/r06g_ab.txt)
template <bool FIRST, int FMT, int KIND>
__global__ __launch_bounds__(RBK_BLOCK, !FIRST ? RBK_LAT_WAVES : FMT == MSM_CACHED ? RBK_CWAVES : RBK_WAVES) void k_rbk_pass(const uint32_t *__restrict__ keys,
                                                        const uint32_t *__restrict__ vals,
                                                        const ge *__restrict__ pin, SegTab T, uint64_t E,
                                                        uint32_t invalid, int cw, uint32_t *__restrict__ kout,
                                                        ge *__restrict__ pout, ge *__restrict__ buckets,
                                                        uint8_t *__restrict__ bflag) {
    constexpr bool NEGC = KIND == 1;
    __shared__ uint32_t sk[RBK_CHUNK + RBK_BLOCK];
    if constexpr (!FIRST) WAVE_PRIO(BPG_LAT_PRIO);
    if constexpr (FIRST && FMT == MSM_CACHED) WAVE_PRIO(BPG_CACHED_PRIO);
    __shared__ uint32_t sv[FIRST ? RBK_CHUNK + RBK_BLOCK : 1];
    __shared__ uint64_t sptr[FIRST ? 2 * MSM_MAXSEG : 1];
    const uint32_t t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * RBK_CHUNK;
    rbk_stage(sk, keys, base, E, invalid);
    if (FIRST) {
        for (uint32_t k = t; k < RBK_CHUNK; k += RBK_BLOCK) {
            uint64_t idx = base + k;
            sv[rbk_lds(k)] = idx < E ? vals[idx] : 0;
        }
        if (t < MSM_MAXSEG) {
            sptr[t] = reinterpret_cast<uint64_t>(T.base[t]);
            sptr[MSM_MAXSEG + t] = reinterpret_cast<uint64_t>(T.neg[t]);
        }
    }
    __syncthreads();
    const uint64_t c = (uint64_t)blockIdx.x * RBK_BLOCK + t;
    uint32_t *ko = kout + 2 * c;
    ge *po = pout + 2 * c;
    const uint64_t gs = base + (uint64_t)t * RBK_T;
    const uint32_t first = RBK_KEY(sk[rbk_lds(t * RBK_T)]);
    if (gs >= E || first == invalid) { ko[0] = invalid; ko[1] = invalid; return; }
    const uint32_t pk = gs == 0 ? invalid : RBK_KEY(t ? sk[rbk_lds(t * RBK_T - 1)] : keys[gs - 1]);
    const uint64_t gn = gs + RBK_T;
    const uint32_t nk = gn >= E ? invalid : RBK_KEY((t + 1 < RBK_BLOCK) ? sk[rbk_lds((t + 1) * RBK_T)] : keys[gn]);
    const bool open_start = pk == first;
    bool head_done = false, real = false;
    uint32_t cur = first;
    ge acc;
    ge_identity(acc);
    // a new key closes the current run: the head piece goes to the next pass
    // (or its bucket when the run began in this chunk), later runs to buckets
    auto close_run = [&](uint32_t k) {
        if (!head_done) {
            if (open_start) { ko[0] = cur | (real ? 0u : RBK_FILL); if (real) ge_store(po, acc); }
            else { if (real) { ge_store(buckets + rbk_bucket(cur, cw), acc); bflag[rbk_bucket(cur, cw)] = 1; } ko[0] = cur | RBK_FILL; }
            head_done = true;
        } else if (real) {
            ge_store(buckets + rbk_bucket(cur, cw), acc); bflag[rbk_bucket(cur, cw)] = 1;
        }
        cur = k; real = false;
        ge_identity(acc);
    };
    if constexpr (FIRST) {
        typedef typename BaseOf<FMT>::T BT;
        typedef typename BaseOf<FMT>::T BT;
        BT pa;
        const uint32_t *skt = sk + rbk_lds(t * RBK_T), *svt = sv + rbk_lds(t * RBK_T);   // chunk has no pad inside
        if (!rbk_trash(first, cw)) msm_load_base<FMT, NEGC>(pa, sptr, svt[0]);
        // entry i: its base is in `use`; entry i+1's gather goes to `fill`.
        // Returns false at the chunk's end (padding key).
        auto step = [&](uint32_t i, BT &use, BT &fill) -> bool {
            const uint32_t k = RBK_KEY(skt[i]);
            if (k == invalid) return false;
            if (k != cur) close_run(k);
            const uint32_t v = svt[i];
            if (i + 1 < RBK_T) {
                const uint32_t kn = RBK_KEY(skt[i + 1]);
                if (kn != invalid && !rbk_trash(kn, cw)) msm_load_base<FMT, NEGC>(fill, sptr, svt[i + 1]);
            }
            // zero digits (trash, sorted to the end of their row) are never added
            if (!rbk_trash(k, cw)) { msm_add_loaded<NEGC>(acc, use, v >> 31); real = true; }
            return true;
        };
        // entry 0 starts every lane's chunk from the identity (its own run or
        // the open head), the same step for the whole wave: its base is
        // converted, not added
        {
            BT use = pa;
            const uint32_t kn = RBK_KEY(skt[1]);
            if (kn != invalid && !rbk_trash(kn, cw)) msm_load_base<FMT, NEGC>(pa, sptr, svt[1]);
            if (!rbk_trash(first, cw)) { msm_init_loaded<NEGC>(acc, use, svt[0] >> 31); real = true; }
        }
        for (uint32_t i = 1; i < RBK_T; i++) {
            BT use = pa;
            if (!step(i, use, pa)) break;
        }
    } else {
        for (uint32_t i = 0; i < RBK_T; i++) {
            const uint32_t x = sk[rbk_lds(t * RBK_T + i)];
            const uint32_t k = RBK_KEY(x);
            if (k == invalid) break;
            if (k != cur) close_run(k);
            if (!(x & RBK_FILL)) {
                ge p; ge_load(p, pin + gs + i);
                if (real) ge_add(acc, acc, p);
                else acc = p;              // the run's first piece: acc is the identity
                real = true;
            }
        }
    }
    const bool tail_open = nk == cur;
    if (!head_done) {            // one run in the chunk
        if (open_start || tail_open) { ko[0] = cur | (real ? 0u : RBK_FILL); if (real) ge_store(po, acc); }
        else { if (real) { ge_store(buckets + rbk_bucket(cur, cw), acc); bflag[rbk_bucket(cur, cw)] = 1; } ko[0] = cur | RBK_FILL; }
        ko[1] = cur | RBK_FILL;
    } else if (tail_open) {
        ko[1] = cur | (real ? 0u : RBK_FILL);
        if (real) ge_store(po + 1, acc);
    } else {
        if (real) { ge_store(buckets + rbk_bucket(cur, cw), acc); bflag[rbk_bucket(cur, cw)] = 1; }
        ko[1] = cur | RBK_FILL;
    }
}
// After the last pass: the head slot of each run sums the run's real pieces
// and owns the bucket (serial; long only for giant runs of structured digits).
__global__ __launch_bounds__(64, RBK_LAT_WAVES) void k_rbk_final(const uint32_t *__restrict__ keys, const ge *__restrict__ pts,
                                                  uint64_t E, uint32_t invalid, int cw, ge *__restrict__ buckets,
                                                  uint8_t *__restrict__ bflag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    WAVE_PRIO(BPG_LAT_PRIO);
    if (i >= E) return;
    const uint32_t k = RBK_KEY(keys[i]);
    if (k == invalid || (i > 0 && RBK_KEY(keys[i - 1]) == k)) return;
    ge acc, p;
    ge_identity(acc);
    bool real = false;
    for (uint64_t j = i; j < E && RBK_KEY(keys[j]) == k; j++) {
        if (keys[j] & RBK_FILL) continue;
        ge_load(p, pts + j);
        if (real) ge_add(acc, acc, p);
        else acc = p;
        real = true;
    }
    if (real) { ge_store(buckets + rbk_bucket(k, cw), acc); bflag[rbk_bucket(k, cw)] = 1; }
}
// Window rows from buckets: R_row = sum_b (b+1) S_b over the half buckets.
// Level 1 (thread per segment of L buckets): A_s = sum_j (j+1) S_{sL+j} and
// T_s = sum_j S_{sL+j} by the backward running sum (2L additions, no
// per-thread scalar multiple). Then R = sum_s A_s + L * sum_s s T_s.
DEVI void bucket_load(ge &p, const ge *__restrict__ B, const uint8_t *__restrict__ F, size_t i) {
    if (F[i]) ge_load(p, B + i); else ge_identity(p);
}
// Registers of the bucket-row kernels: they hold CUs next to the VALU-bound
// kernels of other streams for up to a millisecond, so every register they do
// not need is room for another wave of those (ROW_WAVES / BSEG_WAVES: waves
// per SIMD compiled for).
static constexpr int BSEG_WAVES = 3, ROW_WAVES = 2;
__global__ __launch_bounds__(64, BSEG_WAVES) void k_bucket_seg(const ge *__restrict__ buckets, const uint8_t *__restrict__ bflag,
                                                   uint32_t rows, uint32_t half, uint32_t seglen, uint32_t nseg,
                                                   ge *__restrict__ segA, ge *__restrict__ segT) {
    WAVE_PRIO(BPG_LAT_PRIO);
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * nseg) return;
    uint32_t row = t / nseg, sgi = t % nseg;
    const size_t b0 = (size_t)row * half + (size_t)sgi * seglen;
    ge run, acc, p;
    bucket_load(run, buckets, bflag, b0 + seglen - 1);
    acc = run;
    for (int b = (int)seglen - 2; b >= 0; b--) {
        bucket_load(p, buckets, bflag, b0 + b);
        ge_add(run, run, p);
        ge_add(acc, acc, run);
    }
    ge_store(segA + t, acc);
    ge_store(segT + t, run);
}
DEVI void ge_dbl_n(ge &r, int n) {
    for (int i = 1; i < n; i++) ge_dbl_t<false>(r, r);
    if (n > 0) ge_dbl_t<true>(r, r);
}
// p + q with q read from memory (global or LDS) one coordinate at a time,
// right before its products: 10 live registers for q instead of 40 (ge_add's
// formula and bounds)
DEVI void ge_add_mem(ge &r, const ge &p, const ge *q) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(q);
    fe a, b, c, d, u, v;
#pragma unroll
    for (int k = 0; k < 10; k++) { u.v[k] = w[10 + k]; v.v[k] = w[k]; }   // q.Y, q.X
    fe t;
    fe_sub_nc(t, u, v);                                   // 3T
    fe_add_nc(v, u, v);                                   // 2T
    fe_sub_nc(a, p.Y, p.X); fe_mul(a, a, t);
    fe_add_nc(b, p.Y, p.X); fe_mul(b, b, v);
#pragma unroll
    for (int k = 0; k < 10; k++) u.v[k] = w[30 + k];      // q.T
    fe_mul(c, p.T, u); fe_mul(c, c, FE_D2);
#pragma unroll
    for (int k = 0; k < 10; k++) u.v[k] = w[20 + k];      // q.Z
    fe_add_nc(u, u, u); fe_mul(d, p.Z, u);
    fe e, f, g, h;
    fe_sub_nc(e, b, a); fe_sub_nc(f, d, c); fe_add_nc(g, d, c); fe_add_nc(h, b, a);
    fe_mul(r.X, e, f); fe_mul(r.Y, g, h); fe_mul(r.T, e, h); fe_mul(r.Z, g, f);
}
// Level 2, one block per row; thread t owns segments [tK, tK + K):
//   sum_s s T_s = sum_t (acc_t - run_t) + K * sum_t t run_t,
//   sum_t t run_t = sum_{k>=1} suffix_k (suffix scan in LDS).
// The row is sum A_s + L * (that). L and K are powers of two.
// Rows are numbered window-major (row = w * nmsm + msm); results land at
// msm * W + w, the layout the host combine reads.
// Registers: every second operand is read from memory coordinate by
// coordinate (ge_add_mem), and acc / run wait out the LDS scan in the
// thread's own (consumed) segT slots, so at most two points are live: the
// kernel then fits on a SIMD next to two waves of MSM pass 1 (it held 225
// registers, and under the bench's concurrency waited ~10x its isolated time
// for a SIMD with that much room, profiles/r03w_pmc_table.md).
DEVI uint32_t row_perm(uint32_t row, uint32_t nmsm, uint32_t W) { return (row % nmsm) * W + row / nmsm; }
// FUSED (rows of at most 256 segments, the small jobs of the IPP tail):
// thread t first sums its own bucket segment t of the row, as k_bucket_seg
// does, into the same segA / segT slots it reads back below, so the job
// needs no k_bucket_seg launch (round 6).
template <bool FUSED>
__global__ __launch_bounds__(256, ROW_WAVES) void k_row_reduce(const ge *__restrict__ segA, ge *__restrict__ segT,
                                                    uint32_t nseg, int lgL, uint32_t nmsm, uint32_t W,
                                                    ge *__restrict__ rows_out, const ge *__restrict__ buckets,
                                                    const uint8_t *__restrict__ bflag, uint32_t half,
                                                    uint32_t seglen) {
    __shared__ ge sh[256];
    const uint32_t row = blockIdx.x, t = threadIdx.x;
    WAVE_PRIO(BPG_LAT_PRIO);
    if constexpr (FUSED) {
        if (t < nseg) {
            // two points live (each bucket read coordinate by coordinate
            // into its addition), as in the row phase below: 174 VGPRs, not
            // the 210 a third live point costs
            const size_t b0 = (size_t)row * half + (size_t)t * seglen;
            ge run, acc;
            bucket_load(run, buckets, bflag, b0 + seglen - 1);
            acc = run;
            for (int b = (int)seglen - 2; b >= 0; b--) {
                if (bflag[b0 + b]) ge_add_mem(run, run, buckets + b0 + b);
                ge_add(acc, acc, run);
            }
            ge_store(const_cast<ge *>(segA) + (size_t)row * nseg + t, acc);
            ge_store(segT + (size_t)row * nseg + t, run);
        }
    }
    const uint32_t K = (nseg + 255) / 256;
    int lgK = 0;
    while ((1u << lgK) < K) lgK++;
    const ge *A = segA + (size_t)row * nseg;
    ge *T = segT + (size_t)row * nseg;
    // sum_s A_s is added at the end (three points live at most, not four)
    ge run, acc;
    ge_identity(run); ge_identity(acc);
    for (int k = (int)K - 1; k >= 0; k--) {
        uint32_t s = t * K + k;
        if (s >= nseg) continue;
        ge_add_mem(run, run, T + s);
        ge_add(acc, acc, run);
    }
    // run and acc wait out the scan in this thread's first two segT slots
    // (their T_s are consumed); with one segment (K = 1, or the row's last
    // thread) acc = run, with none both are the identity. Slot s0 + 1 is
    // this thread's only when K >= 2.
    const uint32_t s0 = t * K;
    const bool has = s0 < nseg, two = has && K >= 2 && s0 + 1 < nseg;
    if (has) ge_store(T + s0, run);
    if (two) ge_store(T + s0 + 1, acc);
    // inclusive suffix scan of run over threads
    ge_store(&sh[t], run);
    for (uint32_t d = 1; d < 256; d <<= 1) {
        __syncthreads();
        ge a;
        const bool act = t + d < 256;
        if (act) { ge_load(a, &sh[t]); ge_add_mem(a, a, &sh[t + d]); }
        __syncthreads();
        if (act) ge_store(&sh[t], a);
    }
    __syncthreads();
    ge q, suf;
    ge_load(suf, &sh[t]);
    if (t == 0) ge_identity(suf);
    ge_dbl_n(suf, lgK);                    // K * suffix_t
    if (has) ge_load(run, T + s0); else ge_identity(run);
    if (two) ge_load(acc, T + s0 + 1); else acc = run;
    ge_sub(q, acc, run);
    ge_add(q, q, suf);
    ge_dbl_n(q, lgL);                      // L * (...)
    for (uint32_t k = 0; k < K; k++) {     // + this thread's A_s
        uint32_t s = t * K + k;
        if (s >= nseg) break;
        ge_add_mem(q, q, A + s);
    }
    __syncthreads();
    ge_store(&sh[t], q);
    for (int w = 128; w >= 1; w >>= 1) {
        __syncthreads();
        if (t < (uint32_t)w) {
            ge a;
            ge_load(a, &sh[t]);
            ge_add_mem(a, a, &sh[t + w]);
            ge_store(&sh[t], a);
        }
    }
    if (t == 0) {
        ge r; ge_load(r, &sh[0]);
        ge_store(rows_out + row_perm(row, nmsm, W), r);
    }
}

// Window width: lg(points) - 3 (measured best, profiles/r01 MSM window
// sweeps), or another width in [4, 16] when a GF(p)-multiply count of the
// job says it needs 3% fewer: W entries per point (7M Niels / 8M cached madd)
// against 2 nmsm W 2^(c-1) bucket additions (9M each). Widths above 16 would
// add a third sort pass. E.g. the IPP's 2^19-point jobs of rounds 2-4 take
// c = 15 (17 windows of 16384 buckets) instead of 16 (16 of 32768).
static int msm_window(uint64_t total, int nmsm, int fmt) {
    int lg = 0;
    while ((1ULL << (lg + 1)) <= total) lg++;
    int c = lg - 3;
    if (c < 4) c = 4;
    if (c > 16) c = 16;
    const double madd = fmt == MSM_NIELS ? 7.0 : 8.0;
    auto cost = [&](int w) {
        const double W = (254 + w - 1) / w;
        return W * (double)total * madd + 2.0 * nmsm * W * (double)(1u << (w - 1)) * 9.0;
    };
    // Jobs hold four proofs' MSMs (nmsm = 8 for the IPP rounds, so the bucket
    // term weighs 4x more): 82.7 / 83.1 vs 81.6 / 82.0 M constraints/s with
    // lg - 3 only (profiles/r03o_ab_rowreduce_window_model.txt); at one proof
    // per job it was neutral (r03d_ab_window_model_threads.txt).
    int best = c;
    for (int w = 4; w <= 16; w++)
        if (cost(w) < cost(best)) best = w;
    return cost(best) < 0.97 * cost(c) ? best : c;
}

MsmEngine::~MsmEngine() {
    if (process_exiting()) return;
    if (tiles_ev_) (void)hipEventDestroy(tiles_ev_);
    if (tiles_host_) (void)hipHostFree(tiles_host_);
    DBuf *bufs[] = {&keys_, &vals_, &keys2_, &vals2_, &sort_tmp_, &tiles_,
                    &rk_a_, &rk_b_, &rp_a_, &rp_b_, &buckets_, &bflag_, &segacc_, &rows_dev_, &dhist_};
    for (DBuf *b : bufs)
        if (b->p) (void)hipFree(b->p);
}

void grow_partial(DBuf &d, hipStream_t st) {
    const size_t before = d.cap;
    d.grow(1024 * 8 * sizeof(sc));
    static_assert(RED_TICKET_WORD < 1024 * 8, "ticket inside the partial buffer");
    if (d.cap != before) BPG_HIP(hipMemsetAsync(static_cast<sc *>(d.p) + RED_TICKET_WORD, 0, sizeof(sc), st));
}
void DBuf::grow(size_t need) {
    if (need <= cap) return;
    if (p) BPG_HIP(hipFree(p));
    p = nullptr;
    size_t n = need + need / 4 + 256;
    BPG_HIP(hipMalloc(&p, n));
    cap = n;
}

void DBuf::grow_first_exact(size_t need) {
    if (p) { grow(need); return; }
    BPG_HIP(hipMalloc(&p, need));
    cap = need;
}
static size_t grown(size_t need) { return need + need / 4 + 256; }   // DBuf::grow's allocation
// the digit launch's histogram hand-off: RS_MAXTILES tickets, then at most
// DHIST_PARTS parts' counts of 256 bins
#define DHIST_PARTS 16384
#define DHIST_BYTES ((size_t)(RS_MAXTILES + (size_t)DHIST_PARTS * RS_MAXBINS) * 4)
#define DIG_LDS_WORDS 8192   // fused histogram in LDS: windows x bins
// fused launch: ~2048 blocks of 256 threads (1024-thread blocks, fewer parts
// per tile, measured 1.6% slower in the bench: profiles/r05k_ab.txt)
#define DIG_FUSED_THREADS 256
#define DIG_FUSED_BLOCKS 2048
size_t MsmEngine::bytes() const {
    size_t b = 0;
    for (const DBuf *d : {&keys_, &vals_, &keys2_, &vals2_, &sort_tmp_, &tiles_, &rk_a_, &rk_b_, &rp_a_, &rp_b_,
                          &buckets_, &bflag_, &segacc_, &rows_dev_, &dhist_})
        b += d->cap;
    return b;
}
size_t MsmEngine::job_bytes(uint64_t total, int nmsm, int fmt) {
    if (!total) return 0;
    const int c = msm_window(total, nmsm, fmt), W = (254 + c - 1) / c;
    const uint64_t rows = (uint64_t)nmsm * W, half = 1ull << (c - 1), E0 = (uint64_t)W * total;
    const uint64_t capE = 2 * ((E0 + RBK_CHUNK - 1) / RBK_CHUNK) * RBK_BLOCK;
    const uint64_t nseg = half <= 2048 ? std::min<uint64_t>(half, 256) : half / 8;
    return 4 * grown(E0 * 4) + grown((size_t)RS_MAXBINS * (RS_MAXTILES + 1) * 4 + 256) + grown((size_t)6 * RS_MAXTILES * 4) +
           grown(capE * 4) + grown(capE * sizeof(ge)) + grown(capE + 1024) + grown((capE / 4 + 256) * sizeof(ge)) +
           grown(rows * half * sizeof(ge)) + grown(rows * half) + grown(2 * rows * nseg * sizeof(ge)) +
           grown(rows * sizeof(ge)) + grown(DHIST_BYTES);
}
void MsmEngine::reserve(const MsmPlan &p) {
    size_t kb = p.E0 * 4;
    keys_.grow(kb); vals_.grow(kb); keys2_.grow(kb); vals2_.grow(kb);
    // radix-sort tile histograms + totals
    sort_tmp_.grow((size_t)RS_MAXBINS * (RS_MAXTILES + 1) * 4 + 256);
    rk_a_.grow(p.capE * 4); rp_a_.grow(p.capE * sizeof(ge));
    rk_b_.grow(p.capE * 4 / 4 + 1024); rp_b_.grow((p.capE / 4 + 256) * sizeof(ge));
    buckets_.grow((size_t)p.rows * p.half * sizeof(ge));
    bflag_.grow((size_t)p.rows * p.half);
    segacc_.grow((size_t)2 * p.rows * p.nseg_per_row * sizeof(ge));
    rows_dev_.grow((size_t)p.rows * sizeof(ge));
}

// Sort (keys, vals) by the low key_bits within each row (tiles never straddle
// a row; tiles_dev: nt x {start, end, first tile of the row, one past its last
// tile, row start}); swaps the buffer pointers to the sorted pair.
// 8-bit digits only where they save a pass (their scatter costs more LDS)
static int rs_bits(int key_bits) { return (key_bits + 7) / 8 < (key_bits + 6) / 7 ? 8 : 7; }
// first_counted: the digit launch already wrote the first pass's histogram
static void radix_sort(uint32_t *&k, uint32_t *&v, uint32_t *&k2, uint32_t *&v2, int key_bits, const uint32_t *tiles,
                       uint32_t nt, uint32_t *hist, bool first_counted, hipStream_t st) {
    if (!nt || key_bits < 1) return;
    const int bits = rs_bits(key_bits);
    const uint32_t bins = 1u << bits;
    uint32_t *total = hist + (size_t)bins * nt;
    for (int shift = 0; shift < key_bits; shift += bits) {
        // every pass after the first keeps the order of equal digits (the
        // three-pass sorts of 20-bit fixed-base keys need the middle one too)
        const bool stable = shift > 0;
        if (shift == 0 && first_counted)
            ;
        else if (bits == 8)
            hipLaunchKernelGGL(k_rs_hist<8>, dim3(nt), dim3(RS_BLOCK), 0, st, k, shift, tiles, nt, hist);
        else
            hipLaunchKernelGGL(k_rs_hist<7>, dim3(nt), dim3(RS_BLOCK), 0, st, k, shift, tiles, nt, hist);
        hipLaunchKernelGGL(k_rs_colscan, dim3(bins), dim3(256), 0, st, hist, nt, total);
        if (bits == 8 && stable)
            hipLaunchKernelGGL((k_rs_scatter<8, true>), dim3(nt), dim3(RS_BLOCK), 0, st, k, v, shift, tiles, nt, hist,
                               total, k2, v2);
        else if (bits == 8)
            hipLaunchKernelGGL((k_rs_scatter<8, false>), dim3(nt), dim3(RS_BLOCK), 0, st, k, v, shift, tiles, nt, hist,
                               total, k2, v2);
        else if (stable)
            hipLaunchKernelGGL((k_rs_scatter<7, true>), dim3(nt), dim3(RS_BLOCK), 0, st, k, v, shift, tiles, nt, hist,
                               total, k2, v2);
        else
            hipLaunchKernelGGL((k_rs_scatter<7, false>), dim3(nt), dim3(RS_BLOCK), 0, st, k, v, shift, tiles, nt, hist,
                               total, k2, v2);
        std::swap(k, k2);
        std::swap(v, v2);
    }
    BPG_HIP(hipGetLastError());
}

MsmPlan MsmEngine::enqueue(const MsmSeg *segs, int nseg, int nmsm, PtD *rows_host, int fmt, PtD *rows_direct) {
    if (nseg < 1 || nseg > MSM_MAXSEG) throw HipError(hipErrorInvalidValue, "nseg", __FILE__, __LINE__);
    if (fmt != MSM_NIELS && fmt != MSM_CACHED)
        throw HipError(hipErrorInvalidValue, "fmt", __FILE__, __LINE__);
    MsmPlan p{};
    SegTab T{};
    uint64_t total = 0;
    T.n = nseg;
    for (int i = 0; i < nseg; i++) {
        T.gofs[i] = (uint32_t)total;
        total += segs[i].count;
    }
    if (total > 0x7fffffffu) throw HipError(hipErrorInvalidValue, "msm job too large", __FILE__, __LINE__);
    T.gofs[nseg] = (uint32_t)total;
    p.total = total;
    // fixed-base job: every segment gathers from generator tables (wstride):
    // FB_C-bit windows, all of a point's windows in its MSM's one row
    const uint64_t wstride = segs[0].wstride;
    const bool fb = wstride != 0;
    for (int i = 0; i < nseg; i++)
        if (segs[i].wstride != wstride) throw HipError(hipErrorInvalidValue, "mixed fixed-base job", __FILE__, __LINE__);
    if (fb && (fmt != MSM_NIELS || nmsm > TILEGEO_MAXMSM))
        throw HipError(hipErrorInvalidValue, "fixed-base job", __FILE__, __LINE__);
    p.c = fb ? FB_C : msm_window(total, nmsm, fmt);
    const int Wd = (254 + p.c - 1) / p.c;   // digit windows
    if (fb && Wd != FB_W) throw HipError(hipErrorInvalidValue, "fixed-base windows", __FILE__, __LINE__);
    p.W = fb ? 1 : Wd;                       // window rows per MSM (what the host combines)
    p.nmsm = nmsm;
    p.rows = nmsm * p.W;
    p.half = 1 << (p.c - 1);
    // segments grouped by MSM (msm indices non-decreasing): MSM m owns points
    // [moff[m], moff[m] + mtot[m])
    uint32_t moff[64] = {0}, mtot[64] = {0};
    if (nmsm < 1 || nmsm > 64) throw HipError(hipErrorInvalidValue, "nmsm", __FILE__, __LINE__);
    for (int i = 0; i < nseg; i++) {
        const uint32_t m = segs[i].msm;
        if ((int)m >= nmsm || (i && m < segs[i - 1].msm))
            throw HipError(hipErrorInvalidValue, "segments not grouped by msm", __FILE__, __LINE__);
        if (!mtot[m]) moff[m] = T.gofs[i];
        mtot[m] += segs[i].count;
    }
    // negated copies: used when every segment of a Niels job has one
    bool negc = fmt == MSM_NIELS;
    bool gens = fmt == MSM_NIELS;   // every segment over a generator set (MsmSeg::gen)
    const size_t psz = fmt == MSM_NIELS ? sizeof(NielsD) : sizeof(PtD);
    for (int i = 0; i < nseg; i++) {
        if (segs[i].count > MSM_LOC_MASK || (fb && (uint64_t)(Wd - 1) * wstride + segs[i].count > MSM_LOC_MASK))
            throw HipError(hipErrorInvalidValue, "msm segment too large", __FILE__, __LINE__);
        T.scal[i] = AS_CSC(segs[i].scal);
        T.base[i] = segs[i].base;
        T.neg[i] = segs[i].negofs ? (const void *)((const uint8_t *)segs[i].base + segs[i].negofs * (int64_t)psz)
                                  : segs[i].base;
        negc = negc && segs[i].negofs != 0;
        gens = gens && segs[i].gen;
        T.row0[i] = segs[i].msm;
        T.idx[i] = segs[i].idx;
        if (segs[i].idx && fb) throw HipError(hipErrorInvalidValue, "indexed fixed-base segment", __FILE__, __LINE__);
    }
    p.E0 = (uint64_t)Wd * total;
    p.T = RBK_T;
    // keys: row << c | slot (slot <= half, half = trash); padding key = rows << c
    const uint64_t D = (uint64_t)p.rows * p.half;
    const uint32_t invalid = (uint32_t)p.rows << p.c;
    p.key_bits = (uint32_t)p.c;   // the sort orders slots within rows
    // slots after pass 1: two per thread chunk, padded to whole blocks
    p.capE = 2 * ((p.E0 + RBK_CHUNK - 1) / RBK_CHUNK) * RBK_BLOCK;
    // buckets per first-level segment (k_bucket_seg): a row of `half`
    // buckets leaves half / seglen segments for the one-block row reduction,
    // whose serial part is 3 additions per segment per thread (16 or 32
    // measured 0.5-2% slower, profiles/r03j_ab_tskip_seglen.txt); the 2^19
    // buckets of a fixed-base row take 64 per segment (8192 segments)
    const uint32_t seg_cfg = std::max<uint32_t>(8, (uint32_t)p.half / 8192);
    p.seglen = p.half < seg_cfg ? p.half : seg_cfg;
    // rows of at most 2048 buckets (the small jobs of the IPP tail): the row
    // kernel sums the segments itself, one per thread, so they are spread
    // over its 256 threads (2 buckets each at c = 10) instead of leaving
    // three quarters of the block idle
    if (p.half <= 2048) p.seglen = std::max<uint32_t>(1, (uint32_t)p.half / 256);
    p.nseg_per_row = p.half / p.seglen;
    if (total == 0) {
        for (int r = 0; r < p.rows; r++) {
            uint32_t *w = reinterpret_cast<uint32_t *>(&rows_host[r]);
            memset(w, 0, sizeof(PtD)); w[10] = 1; w[20] = 1;
        }
        return p;
    }
    reserve(p);
    // sort tiles: each row's contiguous entries cut into tiles of at most `tile`
    uint64_t tile = (p.E0 + 2047) / 2048;
    tile = std::max<uint64_t>(RS_ITER, (tile + RS_ITER - 1) / RS_ITER * RS_ITER);
    tiles_.grow((size_t)6 * RS_MAXTILES * 4);
    uint8_t *bflag = (uint8_t *)bflag_.p;
    TileGeo geo{};
    geo.rows = (uint32_t)p.rows;
    geo.tile = (uint32_t)tile;
    geo.bflag = bflag;
    geo.bflag_bytes = (D + 15) / 16 * 16;   // bflag_ holds D + D/4 + 256 bytes
    uint32_t nt = 0;
    if (nmsm <= TILEGEO_MAXMSM) {   // the digit launch writes the tile table
        // (a fixed-base job is tiled as one window whose MSM m holds Wd
        // entries per point)
        const uint32_t scale = fb ? (uint32_t)Wd : 1u;
        for (int m = 0; m < nmsm; m++) {
            geo.moff[m] = scale * moff[m];
            geo.mtot[m] = scale * mtot[m];
            geo.pmoff[m] = moff[m];
            geo.pmtot[m] = mtot[m];
            geo.tpr[m] = (uint32_t)((geo.mtot[m] + tile - 1) / tile);
            geo.cum[m] = geo.TW;
            geo.TW += geo.tpr[m];
        }
        nt = (uint32_t)p.W * geo.TW;
        geo.nt = nt;
        geo.tiles = (uint32_t *)tiles_.p;
        if (nt + p.rows > RS_MAXTILES) throw HipError(hipErrorInvalidValue, "sort tiles", __FILE__, __LINE__);
    } else {
        if (!tiles_ev_) {
            BPG_HIP(hipEventCreateWithFlags(&tiles_ev_, hipEventDisableTiming));
            // tile table (5 words per tile), then each row's first tile
            BPG_HIP(hipHostMalloc((void **)&tiles_host_, (size_t)6 * RS_MAXTILES * 4, hipHostMallocDefault));
        } else {
            event_wait(tiles_ev_);   // the previous job's upload has left the staging buffer
        }
        std::vector<uint32_t> rowfirst(p.rows);
        for (int r = 0; r < p.rows; r++) {
            const uint32_t m = (uint32_t)r % nmsm, w = (uint32_t)r / nmsm;
            const uint64_t rs = (uint64_t)w * total + moff[m];
            const uint64_t rn = mtot[m];
            const uint32_t t0 = nt;
            for (uint64_t a = 0; a < rn; a += tile) {
                if (nt >= RS_MAXTILES) throw HipError(hipErrorInvalidValue, "sort tiles", __FILE__, __LINE__);
                uint32_t *e = tiles_host_ + 5 * nt++;
                e[0] = (uint32_t)(rs + a); e[1] = (uint32_t)(rs + std::min<uint64_t>(rn, a + tile));
                e[4] = (uint32_t)rs;
            }
            for (uint32_t k = t0; k < nt; k++) { tiles_host_[5 * k + 2] = t0; tiles_host_[5 * k + 3] = nt; }
            rowfirst[r] = t0;
        }
        if (nt + p.rows > RS_MAXTILES) throw HipError(hipErrorInvalidValue, "sort tiles", __FILE__, __LINE__);
        memcpy(tiles_host_ + 5 * nt, rowfirst.data(), (size_t)p.rows * 4);
        BPG_HIP(hipMemcpyAsync(tiles_.p, tiles_host_, (size_t)(5 * nt + p.rows) * 4, hipMemcpyHostToDevice, st_));
        BPG_HIP(hipEventRecord(tiles_ev_, st_));
    }
    uint32_t *keys = (uint32_t *)keys_.p, *vals = (uint32_t *)vals_.p, *keys2 = (uint32_t *)keys2_.p, *vals2 = (uint32_t *)vals2_.p;
    ge *buckets = AS_GE(buckets_.p);
    // the first sort pass's histogram in the digit launch: one block per
    // part of a tile of points (S parts, ~2048 blocks in all), each counting
    // its W windows' keys in LDS
    const uint32_t hbins = 1u << rs_bits((int)p.key_bits);
    const bool fused = geo.tiles && !fb && (uint64_t)Wd * hbins <= DIG_LDS_WORDS;
    uint32_t nblocks = nblk(total, 256);
    size_t lds = 0;
    if (fused) {
        if (!dhist_.p) {
            dhist_.grow(DHIST_BYTES);
            BPG_HIP(hipMemsetAsync(dhist_.p, 0, (size_t)RS_MAXTILES * 4, st_));   // tickets
        }
        uint32_t S = std::min<uint32_t>(16, std::max<uint32_t>(1, (DIG_FUSED_BLOCKS + geo.TW - 1) / geo.TW));
        while (S > 1 && (uint64_t)geo.TW * S * Wd > DHIST_PARTS) S--;
        geo.hist = (uint32_t *)sort_tmp_.p;
        geo.htick = (uint32_t *)dhist_.p;
        geo.hpart = geo.htick + RS_MAXTILES;
        geo.hbins = hbins;
        geo.S = S;
        geo.sub = (uint32_t)((tile + S - 1) / S + 63) / 64 * 64;
        nblocks = geo.TW * S;
        lds = (size_t)Wd * hbins * 4;
    }
    hipLaunchKernelGGL(k_msm_digits, dim3(nblocks), dim3(fused ? DIG_FUSED_THREADS : 256), lds, st_, T, (uint32_t)total, p.c, Wd,
                       (uint32_t)nmsm, (uint32_t)p.half, keys, vals, geo, (uint32_t)wstride);
    BPG_HIP(hipGetLastError());
    radix_sort(keys, vals, keys2, vals2, (int)p.key_bits, (const uint32_t *)tiles_.p, nt, (uint32_t *)sort_tmp_.p,
               fused, st_);
    // reduce passes: E shrinks 8x per pass (2 slots per 16 entries)
    uint64_t E = p.E0;
    const uint32_t *kin = keys;
    const ge *pin = nullptr;
    uint32_t *kout = (uint32_t *)rk_a_.p;
    ge *pout = AS_GE(rp_a_.p);
    p.passes = 0;
    for (;;) {
        const uint32_t nblocks = (uint32_t)std::max<uint64_t>(1, (E + RBK_CHUNK - 1) / RBK_CHUNK);
        // pass 1 consumes the job's operands: 64-B point + 32-B scalar each
        // (SURVEY §8d). One label per kernel instantiation, so a label's
        // launches are exactly one rocprof kernel: the prover's generator
        // jobs (Niels, negated in registers, k_rbk_pass<true, 1, 2>), jobs
        // gathering pre-negated generators (<true, 1, 1>: the verifier's),
        // folded IPP levels (Niels, negated in registers, <true, 1, 0>) and
        // cached bases (<true, 0, 0>).
        ProfScope ps(p.passes ? nullptr
                              : (fmt == MSM_CACHED ? "msm_pass1_cached"
                                 : negc            ? "msm_pass1_negc"
                                 : gens            ? "msm_pass1_gens"
                                                   : "msm_pass1_folded"),
                     96.0 * (double)total,   // one addition per entry: 8M cached, 7M Niels;
                     // each lane's first entry is a 1M conversion
                     (fmt == MSM_CACHED ? 8.0 : 7.0) * (double)p.E0 -
                         (fmt == MSM_CACHED ? 7.0 : 6.0) * (double)((p.E0 + RBK_T - 1) / RBK_T));
        if (p.passes == 0 && fmt == MSM_NIELS && negc)
            hipLaunchKernelGGL((k_rbk_pass<true, MSM_NIELS, 1>), dim3(nblocks), dim3(RBK_BLOCK), 0, st_, kin, vals,
                               pin, T, E, invalid, p.c, kout, pout, buckets, bflag);
        else if (p.passes == 0 && fmt == MSM_NIELS && gens)
            hipLaunchKernelGGL((k_rbk_pass<true, MSM_NIELS, 2>), dim3(nblocks), dim3(RBK_BLOCK), 0, st_, kin, vals,
                               pin, T, E, invalid, p.c, kout, pout, buckets, bflag);
        else if (p.passes == 0 && fmt == MSM_NIELS)
            hipLaunchKernelGGL((k_rbk_pass<true, MSM_NIELS, 0>), dim3(nblocks), dim3(RBK_BLOCK), 0, st_, kin, vals,
                               pin, T, E, invalid, p.c, kout, pout, buckets, bflag);
        else if (p.passes == 0)
            hipLaunchKernelGGL((k_rbk_pass<true, MSM_CACHED, 0>), dim3(nblocks), dim3(RBK_BLOCK), 0, st_, kin, vals,
                               pin, T, E, invalid, p.c, kout, pout, buckets, bflag);
        else
            hipLaunchKernelGGL((k_rbk_pass<false, MSM_CACHED, 0>), dim3(nblocks), dim3(RBK_BLOCK), 0, st_, kin,
                               vals, pin, T, E, invalid, p.c, kout, pout, buckets, bflag);
        BPG_HIP(hipGetLastError());
        p.passes++;
        E = 2 * (uint64_t)nblocks * RBK_BLOCK;
        kin = kout;
        pin = pout;
        // (handing the runs to the final sums after two passes once <= 2^18
        // slots remain measured 0.4% slower: profiles/r03r_ab_priority_stop.txt)
        if (E <= 8192 || p.passes >= 5) break;
        const bool a = kout == (uint32_t *)rk_a_.p;
        kout = a ? (uint32_t *)rk_b_.p : (uint32_t *)rk_a_.p;
        pout = a ? AS_GE(rp_b_.p) : AS_GE(rp_a_.p);
    }
    hipLaunchKernelGGL(k_rbk_final, dim3(nblk(E, 64)), dim3(64), 0, st_, kin, pin, E, invalid, p.c, buckets, bflag);
    // the row kernel writes the window rows straight into the caller's pinned
    // buffer when it gives a device view of it (no copy launch per job)
    ge *rows_out = rows_direct ? reinterpret_cast<ge *>(rows_direct) : AS_GE(rows_dev_.p);
    uint32_t nthr = (uint32_t)p.rows * p.nseg_per_row;
    ge *segA = AS_GE(segacc_.p), *segT = segA + (size_t)p.rows * p.nseg_per_row;
    int lgL = 0;
    while ((1 << lgL) < p.seglen) lgL++;
    if (p.nseg_per_row <= 256) {   // one segment per row thread: summed by the row kernel itself
        hipLaunchKernelGGL(k_row_reduce<true>, dim3(p.rows), dim3(256), 0, st_, (const ge *)segA, segT,
                           (uint32_t)p.nseg_per_row, lgL, (uint32_t)nmsm, (uint32_t)p.W, AS_GE(rows_out),
                           AS_CGE(buckets_.p), (const uint8_t *)bflag, (uint32_t)p.half, (uint32_t)p.seglen);
    } else {
        hipLaunchKernelGGL(k_bucket_seg, dim3(nblk(nthr, 64)), dim3(64), 0, st_, AS_CGE(buckets_.p), bflag,
                           (uint32_t)p.rows, (uint32_t)p.half, (uint32_t)p.seglen, (uint32_t)p.nseg_per_row, segA, segT);
        hipLaunchKernelGGL(k_row_reduce<false>, dim3(p.rows), dim3(256), 0, st_, (const ge *)segA, segT,
                           (uint32_t)p.nseg_per_row, lgL, (uint32_t)nmsm, (uint32_t)p.W, AS_GE(rows_out),
                           (const ge *)nullptr, (const uint8_t *)nullptr, 0u, 0u);
    }
    BPG_HIP(hipGetLastError());
    if (!rows_direct)
        BPG_HIP(hipMemcpyAsync(rows_host, rows_dev_.p, (size_t)p.rows * sizeof(ge), hipMemcpyDeviceToHost, st_));
    return p;
}

// ===========================================================================
// scalar-vector kernels (Montgomery domain noted per kernel)
// ===========================================================================
DEVI void mm(sc &r, const sc &a, const sc &b) { sc_montmul(r, a, b); }
DEVI sc sc_one_raw() { sc o; sc_zero(o); o.v[0] = 1; return o; }

// Scalar::from_bytes_mod_order_wide of raw 64-byte TranscriptRng draws:
// lo + hi * 2^256 mod l, with hi * 2^256 = montmul(hi, R^2).
// Draw j * stride + offset -> out[j] (a rank of the sharded prover reduces
// only its own lanes).
__global__ void k_wide_reduce(const uint32_t *__restrict__ wide, uint32_t count, uint32_t stride, uint32_t offset,
                              sc *__restrict__ out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint4 *w = reinterpret_cast<const uint4 *>(wide + 16 * ((size_t)i * stride + offset));
    uint4 q0 = w[0], q1 = w[1], q2 = w[2], q3 = w[3];
    sc lo, hi, r2, a, b;
    lo.v[0] = q0.x; lo.v[1] = q0.y; lo.v[2] = q0.z; lo.v[3] = q0.w; lo.v[4] = q1.x; lo.v[5] = q1.y; lo.v[6] = q1.z; lo.v[7] = q1.w;
    hi.v[0] = q2.x; hi.v[1] = q2.y; hi.v[2] = q2.z; hi.v[3] = q2.w; hi.v[4] = q3.x; hi.v[5] = q3.y; hi.v[6] = q3.z; hi.v[7] = q3.w;
#pragma unroll
    for (int k = 0; k < 8; k++) r2.v[k] = SC_R2[k];
    sc_reduce(a, lo);
    sc_montmul(b, hi, r2);
    sc_add(a, a, b);
    sc_store(out + i, a);
}
void launch_wide_reduce(const uint8_t *wide, uint32_t count, uint32_t stride, uint32_t offset, ScD *out,
                        hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_wide_reduce, dim3(nblk(count, 256)), dim3(256), 0, st, (const uint32_t *)wide, count, stride,
                       offset, AS_SC(out));
    BPG_HIP(hipGetLastError());
}

// out[i] = mont(base^(start+i)); base2[b] = mont(base^(2^b))
__global__ void k_pow_table(const sc *__restrict__ base2, uint64_t start, uint32_t count, sc *__restrict__ out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint64_t e = start + i;
    // mont(1) = R mod l
    sc acc;
    acc.v[0] = 0x8d98951du; acc.v[1] = 0xd6ec3174u; acc.v[2] = 0x737dcf70u; acc.v[3] = 0xc6ef5bf4u;
    acc.v[4] = 0xfffffffeu; acc.v[5] = 0xffffffffu; acc.v[6] = 0xffffffffu; acc.v[7] = 0x0fffffffu;
    for (int b = 0; b < 40 && e; b++, e >>= 1) {
        if (e & 1) { sc t; sc_load(t, base2 + b); mm(acc, acc, t); }
    }
    sc_store(out + i, acc);
}
void launch_pow_table(const ScD *base2, uint64_t start, uint32_t count, ScD *out, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_pow_table, dim3(nblk(count, 128)), dim3(128), 0, st, AS_CSC(base2), start, count, AS_SC(out));
    BPG_HIP(hipGetLastError());
}
__global__ void k_pow_expand(const sc *__restrict__ lo, const sc *__restrict__ hi, uint32_t count, sc mult,
                             sc *__restrict__ out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    sc a, b, r;
    sc_load(a, lo + (i & 1023)); sc_load(b, hi + (i >> 10));
    mm(r, a, b);
    mm(r, r, mult);
    sc_store(out + i, r);
}
void launch_pow_expand(const ScD *lo, const ScD *hi, uint32_t count, ScD mult, ScD *out, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_pow_expand, dim3(nblk(count, 256)), dim3(256), 0, st, AS_CSC(lo), AS_CSC(hi), count,
                       *reinterpret_cast<sc *>(&mult), AS_SC(out));
    BPG_HIP(hipGetLastError());
}

// Batched power tables (PowBatch): block (x, p, j) covers entries
// [256 x, 256 x + 256) of the concatenation lo (1024) | hi (nhi) of base j of
// proof p. The block's 40 doubling powers come from pinned host memory (the
// host wrote them before the launch; fine-grained, read once per block into
// LDS, one 32-B scalar per thread of the first 40).
__global__ __launch_bounds__(256) void k_pow_tables(PowBatch A) {
    WAVE_PRIO(BPG_MISC_PRIO);
    const uint32_t p = blockIdx.y, j = blockIdx.z;
    const uint32_t i0 = blockIdx.x * 256, nhi = A.nhi[p][j];
    if (i0 >= 1024 + nhi) return;
    const bool hi = i0 >= 1024;
    __shared__ sc b2[40];
    if (threadIdx.x < 40) sc_load(b2[threadIdx.x], AS_CSC(A.b2[p]) + 80 * j + (hi ? 40 : 0) + threadIdx.x);
    __syncthreads();
    const uint32_t i = i0 + threadIdx.x;
    if (i >= 1024 + nhi) return;
    uint64_t e = hi ? i - 1024 : i;
    sc acc;   // mont(1) = R mod l
    acc.v[0] = 0x8d98951du; acc.v[1] = 0xd6ec3174u; acc.v[2] = 0x737dcf70u; acc.v[3] = 0xc6ef5bf4u;
    acc.v[4] = 0xfffffffeu; acc.v[5] = 0xffffffffu; acc.v[6] = 0xffffffffu; acc.v[7] = 0x0fffffffu;
    for (int b = 0; b < 40 && e; b++, e >>= 1)
        if (e & 1) { sc t = b2[b]; mm(acc, acc, t); }
    sc_store(hi ? AS_SC(A.hi[p][j]) + (i - 1024) : AS_SC(A.lo[p][j]) + i, acc);
}
void launch_pow_tables(const PowBatch &A, int P, int nbase, hipStream_t st) {
    if (P < 1 || P > 4 || nbase < 1 || nbase > 3) throw HipError(hipErrorInvalidValue, "pow tables", __FILE__, __LINE__);
    uint32_t mx = 0;
    for (int p = 0; p < P; p++)
        for (int j = 0; j < nbase; j++) mx = std::max(mx, A.nhi[p][j]);
    hipLaunchKernelGGL(k_pow_tables, dim3(nblk(1024 + mx, 256), P, nbase), dim3(256), 0, st, A);
    BPG_HIP(hipGetLastError());
}
__global__ void k_pow_expand_batch(PowExpandBatch A, uint32_t count) {
    WAVE_PRIO(BPG_MISC_PRIO);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, p = blockIdx.y, j = blockIdx.z;
    if (i >= count) return;
    sc a, b, r, m = *reinterpret_cast<const sc *>(&A.mult[p][j]);
    sc_load(a, AS_CSC(A.lo[p][j]) + (i & 1023)); sc_load(b, AS_CSC(A.hi[p][j]) + (i >> 10));
    mm(r, a, b);
    mm(r, r, m);
    sc_store(AS_SC(A.out[p][j]) + i, r);
}
void launch_pow_expand_batch(const PowExpandBatch &A, int P, int nvec, uint32_t count, hipStream_t st) {
    if (!count) return;
    if (P < 1 || P > 4 || nvec < 1 || nvec > 2) throw HipError(hipErrorInvalidValue, "pow expand", __FILE__, __LINE__);
    hipLaunchKernelGGL(k_pow_expand_batch, dim3(nblk(count, 256), P, nvec), dim3(256), 0, st, A, count);
    BPG_HIP(hipGetLastError());
}
__global__ void k_wide_reduce_batch(WideBatch A, uint32_t count, uint32_t stride, uint32_t offset) {
    WAVE_PRIO(BPG_MISC_PRIO);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, q = blockIdx.y;
    if (i >= count) return;
    const uint4 *w = reinterpret_cast<const uint4 *>(A.wide[q] + 64 * ((size_t)i * stride + offset));
    uint4 q0 = w[0], q1 = w[1], q2 = w[2], q3 = w[3];
    sc lo, hi, r2, a, b;
    lo.v[0] = q0.x; lo.v[1] = q0.y; lo.v[2] = q0.z; lo.v[3] = q0.w; lo.v[4] = q1.x; lo.v[5] = q1.y; lo.v[6] = q1.z; lo.v[7] = q1.w;
    hi.v[0] = q2.x; hi.v[1] = q2.y; hi.v[2] = q2.z; hi.v[3] = q2.w; hi.v[4] = q3.x; hi.v[5] = q3.y; hi.v[6] = q3.z; hi.v[7] = q3.w;
#pragma unroll
    for (int k = 0; k < 8; k++) r2.v[k] = SC_R2[k];
    sc_reduce(a, lo);
    sc_montmul(b, hi, r2);
    sc_add(a, a, b);
    sc_store(AS_SC(A.out[q]) + i, a);
}
void launch_wide_reduce_batch(const WideBatch &A, int nq, uint32_t count, uint32_t stride, uint32_t offset,
                              hipStream_t st) {
    if (!count) return;
    if (nq < 1 || nq > 8) throw HipError(hipErrorInvalidValue, "wide reduce batch", __FILE__, __LINE__);
    hipLaunchKernelGGL(k_wide_reduce_batch, dim3(nblk(count, 256), nq), dim3(256), 0, st, A, count, stride, offset);
    BPG_HIP(hipGetLastError());
}

// flatten: z tables are Montgomery; result normal form
DEVI void flat_term(sc &acc, uint32_t q, const sc &coeff, const sc *zlo, const sc *zhi) {
    uint32_t e = q + 1;
    sc a, b, zm, t;
    sc_load(a, zlo + (e & 1023)); sc_load(b, zhi + (e >> 10));
    mm(zm, a, b);
    mm(t, coeff, zm);
    sc_add(acc, acc, t);
}
__global__ void k_flatten_short(CscDev c, const sc *__restrict__ zlo, const sc *__restrict__ zhi, sc *__restrict__ out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c.nshort) return;
    uint32_t col = c.short_cols[t];
    sc acc; sc_zero(acc);
    for (uint32_t k = c.col_ptr[col]; k < c.col_ptr[col + 1]; k++) {
        sc co; sc_load(co, AS_CSC(c.coeff) + k);
        flat_term(acc, c.row[k], co, zlo, zhi);
    }
    if (col >= c.neg_from) sc_neg(acc, acc);
    sc_store(out + col, acc);
}
__global__ __launch_bounds__(64) void k_flatten_long(CscDev c, const sc *__restrict__ zlo, const sc *__restrict__ zhi,
                                                     sc *__restrict__ out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    __shared__ sc sh[64];
    uint32_t t = blockIdx.x, lane = threadIdx.x;
    if (t >= c.nlong) return;
    uint32_t col = c.long_cols[t];
    sc acc; sc_zero(acc);
    for (uint32_t k = c.col_ptr[col] + lane; k < c.col_ptr[col + 1]; k += 64) {
        sc co; sc_load(co, AS_CSC(c.coeff) + k);
        flat_term(acc, c.row[k], co, zlo, zhi);
    }
    sc_store(&sh[lane], acc);
    for (int s = 32; s >= 1; s >>= 1) {
        __syncthreads();
        if (lane < (uint32_t)s) { sc a, b; sc_load(a, &sh[lane]); sc_load(b, &sh[lane + s]); sc_add(a, a, b); sc_store(&sh[lane], a); }
    }
    if (lane == 0) {
        sc r; sc_load(r, &sh[0]);
        if (col >= c.neg_from) sc_neg(r, r);
        sc_store(out + col, r);
    }
}
void launch_flatten(const CscDev &csc, const ScD *zlo, const ScD *zhi, ScD *out, hipStream_t st) {
    if (csc.nshort)
        hipLaunchKernelGGL(k_flatten_short, dim3(nblk(csc.nshort, 128)), dim3(128), 0, st, csc, AS_CSC(zlo), AS_CSC(zhi), AS_SC(out));
    if (csc.nlong)
        hipLaunchKernelGGL(k_flatten_long, dim3(csc.nlong), dim3(64), 0, st, csc, AS_CSC(zlo), AS_CSC(zhi), AS_SC(out));
    BPG_HIP(hipGetLastError());
}

__global__ void k_lr_build(const sc *__restrict__ aL, const sc *__restrict__ aR, const sc *__restrict__ sR,
                           const sc *__restrict__ wL, const sc *__restrict__ wR, const sc *__restrict__ wO,
                           const sc *__restrict__ ypm, const sc *__restrict__ yipm, uint32_t n, sc *__restrict__ l1,
                           sc *__restrict__ r0, sc *__restrict__ r1, sc *__restrict__ r3) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc a, b, y, t, u;
    sc_load(y, ypm + i);
    sc_load(t, yipm + i); sc_load(b, wR + i); mm(u, t, b); sc_load(a, aL + i); sc_add(u, a, u); sc_store(l1 + i, u);
    sc one = sc_one_raw(), yn;
    mm(yn, y, one);
    sc_load(a, wO + i); sc_sub(u, a, yn); sc_store(r0 + i, u);
    sc_load(a, aR + i); mm(u, y, a); sc_load(b, wL + i); sc_add(u, u, b); sc_store(r1 + i, u);
    sc_load(a, sR + i); mm(u, y, a); sc_store(r3 + i, u);
}
void launch_lr_build(const ScD *aL, const ScD *aR, const ScD *sR, const ScD *wL, const ScD *wR, const ScD *wO,
                     const ScD *yp, const ScD *yip, uint32_t n, ScD *l1, ScD *r0, ScD *r1, ScD *r3, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_lr_build, dim3(nblk(n, 128)), dim3(128), 0, st, AS_CSC(aL), AS_CSC(aR), AS_CSC(sR), AS_CSC(wL),
                       AS_CSC(wR), AS_CSC(wO), AS_CSC(yp), AS_CSC(yip), n, AS_SC(l1), AS_SC(r0), AS_SC(r1), AS_SC(r3));
    BPG_HIP(hipGetLastError());
}

// block reduction of K scalars per thread into partial[block*K + k]
template <int K>
DEVI void block_reduce_store(sc (&v)[K], sc *__restrict__ partial) {
    __shared__ sc sh[256];
    uint32_t tid = threadIdx.x;
    // unrolled: v[] stays in registers (a runtime index put it in scratch)
#pragma unroll
    for (int k = 0; k < K; k++) {
        sc_store(&sh[tid], v[k]);
        for (int s = 128; s >= 1; s >>= 1) {
            __syncthreads();
            if (tid < (uint32_t)s) { sc a, b; sc_load(a, &sh[tid]); sc_load(b, &sh[tid + s]); sc_add(a, a, b); sc_store(&sh[tid], a); }
        }
        __syncthreads();
        if (tid == 0) { sc r; sc_load(r, &sh[0]); sc_store(partial + blockIdx.x * K + k, r); }
        __syncthreads();
    }
}
// LDS tree over the block: on return thread 0's v[k] hold the block's sums
template <int K>
DEVI void block_reduce_lds(sc (&v)[K]) {
    __shared__ sc sh[256];
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; k++) {
        sc_store(&sh[tid], v[k]);
        for (int s = 128; s >= 1; s >>= 1) {
            __syncthreads();
            if (tid < (uint32_t)s) { sc a, b; sc_load(a, &sh[tid]); sc_load(b, &sh[tid + s]); sc_add(a, a, b); sc_store(&sh[tid], a); }
        }
        __syncthreads();
        if (tid == 0) sc_load(v[k], &sh[0]);
        __syncthreads();
    }
}
#define RED_BLOCKS 1024
// The launch's reduction ticket: a word after the partials (K <= 6 columns of
// at most RED_BLOCKS blocks) of the caller's partial buffer, zeroed when the
// buffer is allocated (grow_partial) and reset by each launch's last block.
#define RED_TICKET RED_TICKET_WORD
// Per-block partials, then the LAST block of the launch to finish sums them
// column by column into out[k] (mode 0: Montgomery-scaled partials, times R;
// 1: as is; 2: negated) -- one launch instead of the kernel plus a
// k_reduce_cols launch. Hand-off per cdna_hip_programming.md Guideline 16
// (counter form, write-through variant): each block's partial is stored
// sc1 (agent-scope relaxed atomic stores, written through to memory) and
// drained before the block's relaxed ticket add, so no release fence (a
// release writes back the whole L2 of the XCD, which the other streams'
// kernels keep full of dirty lines); the last block acquires before reading
// the partials.
template <int K>
DEVI void block_reduce_final(sc (&v)[K], sc *__restrict__ partial, sc *__restrict__ out, int mode) {
    block_reduce_lds<K>(v);   // thread 0 holds the block's sums
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            uint64_t *dst = reinterpret_cast<uint64_t *>(partial + blockIdx.x * K + k);
#pragma unroll
            for (int q = 0; q < 4; q++)
                __hip_atomic_store(dst + q, (uint64_t)v[k].v[2 * q] | (uint64_t)v[k].v[2 * q + 1] << 32,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __shared__ sc sh[256];
    __shared__ uint32_t last;
    const uint32_t tid = threadIdx.x, nb = gridDim.x;
    uint32_t *ticket = reinterpret_cast<uint32_t *>(partial + RED_TICKET);
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the partial's sc1 stores have landed
        const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == nb - 1 ? 1u : 0u;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;
#pragma unroll
    for (int k = 0; k < K; k++) {
        sc acc;
        sc_zero(acc);
        for (uint32_t b = tid; b < nb; b += blockDim.x) { sc t; sc_load(t, partial + (size_t)b * K + k); sc_add(acc, acc, t); }
        sc_store(&sh[tid], acc);
        for (int s = 128; s >= 1; s >>= 1) {
            __syncthreads();
            if (tid < (uint32_t)s) { sc x, y; sc_load(x, &sh[tid]); sc_load(y, &sh[tid + s]); sc_add(x, x, y); sc_store(&sh[tid], x); }
        }
        if (tid == 0) {
            sc r;
            sc_load(r, &sh[0]);
            if (mode == 0) {   // Montgomery-scaled partials: multiply back by R
                sc r2;
                for (int i = 0; i < 8; i++) r2.v[i] = SC_R2[i];
                mm(r, r, r2);
            } else if (mode == 2) {
                sc_neg(r, r);
            }
            sc_store(out + k, r);
        }
        __syncthreads();
    }
    if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // for the next launch
}
// Montgomery-scaled sums (sum a*b/R); the final reduce multiplies by R^2/R
__global__ __launch_bounds__(256) void k_tpoly(const sc *__restrict__ l1, const sc *__restrict__ l2,
                                               const sc *__restrict__ l3, const sc *__restrict__ r0,
                                               const sc *__restrict__ r1, const sc *__restrict__ r3, uint32_t n,
                                               sc *__restrict__ partial, sc *__restrict__ red_out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[6];
    for (int k = 0; k < 6; k++) sc_zero(acc[k]);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        sc a1, a2, a3, b0, b1, b3, t;
        sc_load(a1, l1 + i); sc_load(a2, l2 + i); sc_load(a3, l3 + i);
        sc_load(b0, r0 + i); sc_load(b1, r1 + i); sc_load(b3, r3 + i);
        mm(t, a1, b0); sc_add(acc[0], acc[0], t);                                   // t1 = l1.r0
        mm(t, a1, b1); sc_add(acc[1], acc[1], t); mm(t, a2, b0); sc_add(acc[1], acc[1], t);  // t2
        mm(t, a2, b1); sc_add(acc[2], acc[2], t); mm(t, a3, b0); sc_add(acc[2], acc[2], t);  // t3
        mm(t, a1, b3); sc_add(acc[3], acc[3], t); mm(t, a3, b1); sc_add(acc[3], acc[3], t);  // t4
        mm(t, a2, b3); sc_add(acc[4], acc[4], t);                                   // t5
        mm(t, a3, b3); sc_add(acc[5], acc[5], t);                                   // t6
    }
    block_reduce_final<6>(acc, partial, red_out, 0);
}
void launch_tpoly(const ScD *l1, const ScD *l2, const ScD *l3, const ScD *r0, const ScD *r1, const ScD *r3,
                  uint32_t n, ScD *partial, ScD *out6, hipStream_t st) {
    uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(RED_BLOCKS, nblk(n, 256)));
    hipLaunchKernelGGL(k_tpoly, dim3(nb), dim3(256), 0, st, AS_CSC(l1), AS_CSC(l2), AS_CSC(l3), AS_CSC(r0),
                       AS_CSC(r1), AS_CSC(r3), n, AS_SC(partial), AS_SC(out6));
    BPG_HIP(hipGetLastError());
}
__global__ __launch_bounds__(256) void k_flatten_range(const sc *__restrict__ coeff, const uint32_t *__restrict__ row,
                                                       uint32_t k0, uint32_t k1, const sc *__restrict__ zlo,
                                                       const sc *__restrict__ zhi, sc *__restrict__ partial, sc *__restrict__ red_out, int red_mode) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[1];
    sc_zero(acc[0]);
    for (uint32_t k = k0 + blockIdx.x * blockDim.x + threadIdx.x; k < k1; k += gridDim.x * blockDim.x) {
        sc co; sc_load(co, coeff + k);
        flat_term(acc[0], row[k], co, zlo, zhi);
    }
    block_reduce_final<1>(acc, partial, red_out, red_mode);
}
void launch_flatten_huge(const CscDev &csc, uint32_t col, uint32_t k0, uint32_t k1, const ScD *zlo, const ScD *zhi,
                         ScD *partial, ScD *out, hipStream_t st) {
    uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(RED_BLOCKS, nblk(k1 - k0, 256)));
    hipLaunchKernelGGL(k_flatten_range, dim3(nb), dim3(256), 0, st, AS_CSC(csc.coeff), csc.row, k0, k1, AS_CSC(zlo),
                       AS_CSC(zhi), AS_SC(partial), AS_SC(out + col), col >= csc.neg_from ? 2 : 1);
    BPG_HIP(hipGetLastError());
}
__global__ __launch_bounds__(256) void k_dot(const sc *__restrict__ a, const sc *__restrict__ b, uint32_t n,
                                             sc *__restrict__ partial, sc *__restrict__ red_out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[1];
    sc_zero(acc[0]);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        sc x, y, t;
        sc_load(x, a + i); sc_load(y, b + i);
        mm(t, x, y); sc_add(acc[0], acc[0], t);
    }
    block_reduce_final<1>(acc, partial, red_out, 0);
}
void launch_dot(const ScD *a, const ScD *b, uint32_t n, ScD *partial, ScD *out, hipStream_t st) {
    uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(RED_BLOCKS, nblk(n, 256)));
    hipLaunchKernelGGL(k_dot, dim3(nb), dim3(256), 0, st, AS_CSC(a), AS_CSC(b), n, AS_SC(partial), AS_SC(out));
    BPG_HIP(hipGetLastError());
}

// x given in Montgomery form (x*R); l2 = a_O, l3 = s_L
__global__ void k_lr_eval(const sc *__restrict__ l1, const sc *__restrict__ l2, const sc *__restrict__ l3,
                          const sc *__restrict__ r0, const sc *__restrict__ r1, const sc *__restrict__ r3,
                          const sc *__restrict__ ypm, uint32_t n, uint32_t N, sc xm, sc x2m, sc *__restrict__ a,
                          sc *__restrict__ b) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    sc ra, rb;
    if (i < n) {
        sc p, q, t;
        sc_load(p, l3 + i); mm(t, p, xm); sc_load(q, l2 + i); sc_add(t, t, q); mm(t, t, xm);
        sc_load(q, l1 + i); sc_add(t, t, q); mm(ra, t, xm);
        sc_load(p, r3 + i); mm(t, p, x2m); sc_load(q, r1 + i); sc_add(t, t, q); mm(t, t, xm);
        sc_load(q, r0 + i); sc_add(rb, t, q);
    } else {
        sc y, one = sc_one_raw();
        sc_load(y, ypm + i); mm(y, y, one);
        sc_zero(ra);
        sc_neg(rb, y);
    }
    sc_store(a + i, ra);
    sc_store(b + i, rb);
}
void launch_lr_eval(const ScD *l1, const ScD *l2, const ScD *l3, const ScD *r0, const ScD *r1, const ScD *r3,
                    const ScD *yp, uint32_t n, uint32_t N, ScD xm, ScD x2m, ScD *a, ScD *b, hipStream_t st) {
    hipLaunchKernelGGL(k_lr_eval, dim3(nblk(N, 128)), dim3(128), 0, st, AS_CSC(l1), AS_CSC(l2), AS_CSC(l3), AS_CSC(r0),
                       AS_CSC(r1), AS_CSC(r3), AS_CSC(yp), n, N, *reinterpret_cast<sc *>(&xm),
                       *reinterpret_cast<sc *>(&x2m), AS_SC(a), AS_SC(b));
    BPG_HIP(hipGetLastError());
}

// ===========================================================================
// IPP
// ===========================================================================
DEVI void ipp_prep_body(const sc *__restrict__ a, const sc *__restrict__ b,
                                                  const sc *__restrict__ yipm, const IppRoundArgs &A, sc *__restrict__ out,
                                                  sc *__restrict__ partial, sc *__restrict__ red_out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[2];
    sc_zero(acc[0]); sc_zero(acc[1]);
    const uint32_t h = A.h;
    const sc lamG1 = *reinterpret_cast<const sc *>(&A.lamG1), lamGu = *reinterpret_cast<const sc *>(&A.lamGu);
    const sc muH1 = *reinterpret_cast<const sc *>(&A.muH1), muHu = *reinterpret_cast<const sc *>(&A.muHu);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < h; i += gridDim.x * blockDim.x) {
        sc aL, aR, bL, bR, t, y;
        sc_load(aL, a + i); sc_load(aR, a + h + i); sc_load(bL, b + i); sc_load(bR, b + h + i);
        mm(t, aL, bR); sc_add(acc[0], acc[0], t);
        mm(t, aR, bL); sc_add(acc[1], acc[1], t);
        bool lo_real = i < A.n, hi_real = (h + i) < A.n;
        // L: aL * lam*Gf[h+i] (base Ghat_R), bR * mu*Gf[i]*y^-i (base Hhat_L)
        mm(t, aL, hi_real ? lamG1 : lamGu); sc_store(out + i, t);
        sc_load(y, yipm + i); mm(t, bR, y); mm(t, t, lo_real ? muH1 : muHu); sc_store(out + h + i, t);
        // R: aR * lam*Gf[i] (base Ghat_L), bL * mu*Gf[h+i]*y^-(h+i) (base Hhat_R)
        mm(t, aR, lo_real ? lamG1 : lamGu); sc_store(out + 2 * h + i, t);
        sc_load(y, yipm + h + i); mm(t, bL, y); mm(t, t, hi_real ? muH1 : muHu); sc_store(out + 3 * h + i, t);
    }
    block_reduce_final<2>(acc, partial, red_out, 0);
}
// u, uinv in Montgomery form
struct FoldScalarsArgs { sc *a[4], *b[4]; sc um[4], uim[4]; };
// a' = a_lo u + a_hi u^-1, b' = b_lo u^-1 + b_hi u for the P proofs of a
// lockstep step (blockIdx.y = proof): one launch per round, not one per proof
__global__ void k_ipp_fold_scalars(FoldScalarsArgs A, uint32_t h) {
    WAVE_PRIO(BPG_MISC_PRIO);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, p = blockIdx.y;
    if (i >= h) return;
    sc *a = A.a[p], *b = A.b[p];
    const sc um = A.um[p], uim = A.uim[p];
    sc x, y, t1, t2;
    sc_load(x, a + i); sc_load(y, a + h + i); mm(t1, x, um); mm(t2, y, uim); sc_add(t1, t1, t2); sc_store(a + i, t1);
    sc_load(x, b + i); sc_load(y, b + h + i); mm(t1, x, uim); mm(t2, y, um); sc_add(t1, t1, t2); sc_store(b + i, t1);
}
void launch_ipp_fold_scalars(ScD *const *a, ScD *const *b, const ScD *u, const ScD *uinv, int P, uint32_t h,
                             hipStream_t st) {
    if (P < 1 || P > 4) throw HipError(hipErrorInvalidValue, "fold scalars proofs", __FILE__, __LINE__);
    FoldScalarsArgs A{};
    for (int p = 0; p < P; p++) {
        A.a[p] = AS_SC(a[p]); A.b[p] = AS_SC(b[p]);
        A.um[p] = *reinterpret_cast<const sc *>(&u[p]); A.uim[p] = *reinterpret_cast<const sc *>(&uinv[p]);
    }
    hipLaunchKernelGGL(k_ipp_fold_scalars, dim3(nblk(h, 256), P), dim3(256), 0, st, A, h);
    BPG_HIP(hipGetLastError());
}
// Point fold: out_i = P_L,i + rho * P_R,i with one rho per lane class. rho is
// uniform across a block, so its width-4 wNAF schedule (digits in +-{1,3,5,7},
// top digit first, with the doubling count before each digit) is computed on
// the host and read from kernel arguments (scalar loads, no divergence). The
// odd multiples P, 3P, 5P, 7P of each lane's P_R live in registers as cached
// points; doublings that feed another doubling skip T (3M + 4S).
struct FoldSched {
    uint32_t ndig, tail;      // nonzero digits; doublings after the last one
    int8_t dig[64];           // signed odd digits, most significant first
    uint8_t gap[64];          // doublings before dig[k] (gap[0] unused)
};
struct FoldArgs {
    const void *in[2];
    gec *out[2];
    uint32_t h, nseg;
    uint32_t start[6], end[6], blk0[7];
    uint32_t vec[6], sched[6];
    FoldSched sc[4];
};
static void wnaf4_schedule(const ScD &k, FoldSched &s) {
    // LSB-first width-4 NAF of the canonical scalar
    int8_t d[260] = {0};
    uint32_t x[9];
    for (int i = 0; i < 8; i++) x[i] = k.v[i];
    x[8] = 0;
    int len = 0;
    auto nz = [&]() { for (int i = 0; i < 9; i++) if (x[i]) return true; return false; };
    while (nz() && len < 260) {
        int di = 0;
        if (x[0] & 1) {
            di = (int)(x[0] & 15);
            if (di >= 8) di -= 16;
            // x -= di
            if (di > 0) {
                uint64_t bw = (uint64_t)di;
                for (int i = 0; i < 9 && bw; i++) { uint64_t t = (uint64_t)x[i] - bw; x[i] = (uint32_t)t; bw = (t >> 63) & 1; }
            } else {
                uint64_t c = (uint64_t)(-di);
                for (int i = 0; i < 9 && c; i++) { c += x[i]; x[i] = (uint32_t)c; c >>= 32; }
            }
        }
        d[len++] = (int8_t)di;
        for (int i = 0; i < 8; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
        x[8] >>= 1;
    }
    s.ndig = 0; s.tail = 0;
    int last = -1;
    for (int pos = len - 1; pos >= 0; pos--) {
        if (!d[pos]) continue;
        if (s.ndig >= 64) throw HipError(hipErrorInvalidValue, "wnaf length", __FILE__, __LINE__);
        s.dig[s.ndig] = d[pos];
        s.gap[s.ndig] = (uint8_t)(last < 0 ? 0 : last - pos);
        s.ndig++;
        last = pos;
    }
    s.tail = last < 0 ? 0 : (uint32_t)last;
}
DEVI void fold_pick(gec &t, const gec &t1, const gec &t3, const gec &t5, const gec &t7, int d) {
    int m = d < 0 ? -d : d;
    if (m == 1) t = t1; else if (m == 3) t = t3; else if (m == 5) t = t5; else t = t7;
}
static constexpr int BPG_FOLD_WAVES = 2;
// P: input point type (gen = affine Niels generators in round 0 of the
// table-less path, gec = folded generators); the output is always cached.
template <class P>
__global__ __launch_bounds__(64, BPG_FOLD_WAVES) void k_ipp_fold_points(const FoldArgs *__restrict__ Ap) {
    const FoldArgs &A = *Ap;
    uint32_t b = blockIdx.x, sg = 0;
#pragma unroll
    for (int k = 1; k < 6; k++) if (k < (int)A.nseg && b >= A.blk0[k]) sg = k;
    const uint32_t i = A.start[sg] + (b - A.blk0[sg]) * 64 + threadIdx.x;
    if (i >= A.end[sg]) return;
    const uint32_t v = A.vec[sg];
    const FoldSched &S = A.sc[A.sched[sg]];
    const P *Pin = reinterpret_cast<const P *>(A.in[v]);
    gec PL;
    if (S.ndig == 0) {
        load_as_cached(PL, Pin + i);
        gec_store(A.out[v] + i, PL);
        return;
    }
    gec t1, t3, t5, t7;
    {
        load_as_cached(t1, Pin + A.h + i);
        ge pr, p2, q;
        fe_sub(pr.X, t1.YpX, t1.YmX);            // projective (2X : 2Y : 2Z), enough to double
        fe_add(pr.Y, t1.YpX, t1.YmX);
        pr.Z = t1.Z2;
        ge_dbl(p2, pr);
        gec c2; ge_to_cached(c2, p2);
        ge_add_c(q, p2, t1); ge_to_cached(t3, q);
        ge_add_c(q, q, c2); ge_to_cached(t5, q);
        ge_add_c(q, q, c2); ge_to_cached(t7, q);
    }
    ge acc;
    {
        gec t; fold_pick(t, t1, t3, t5, t7, S.dig[0]);
        if (S.dig[0] < 0) gec_neg(t, t);
        ge_from_cached(acc, t);
    }
    for (uint32_t k = 1; k < S.ndig; k++) {
        const uint32_t g = S.gap[k];
        for (uint32_t j = 1; j < g; j++) ge_dbl_t<false>(acc, acc);
        ge_dbl_t<true>(acc, acc);
        const int dk = S.dig[k];
        gec t; fold_pick(t, t1, t3, t5, t7, dk);
        // NAF digits are at least one doubling apart: T only for the last
        // addition when no doubling follows it
        if (k + 1 == S.ndig && S.tail == 0) {
            if (dk > 0) ge_add_c_t<true>(acc, acc, t); else ge_sub_c_t<true>(acc, acc, t);
        } else {
            if (dk > 0) ge_add_c_t<false>(acc, acc, t); else ge_sub_c_t<false>(acc, acc, t);
        }
    }
    if (S.tail) {
        for (uint32_t j = 1; j < S.tail; j++) ge_dbl_t<false>(acc, acc);
        ge_dbl_t<true>(acc, acc);
    }
    load_as_cached(PL, Pin + i);
    ge r; ge_add_c(r, acc, PL);
    gec out; ge_to_cached(out, r);
    gec_store(A.out[v] + i, out);
}
void launch_ipp_fold_points(const void *Gin, const void *Hin, int in_fmt, uint32_t h, uint32_t n, ScD rhoG_a,
                            ScD rhoG_b, ScD rhoH_a, ScD rhoH_b, PtD *Gout, PtD *Hout, ArgStage &stage,
                            hipStream_t st) {
    if (!stage.dev) {
        BPG_HIP(hipMalloc(&stage.dev, sizeof(FoldArgs)));
        BPG_HIP(hipHostMalloc(&stage.host, sizeof(FoldArgs), hipHostMallocDefault));
        BPG_HIP(hipEventCreateWithFlags(&stage.copied, hipEventBlockingSync | hipEventDisableTiming));
    } else {
        event_wait(stage.copied);   // previous upload has left the host buffer
    }
    FoldArgs &A = *reinterpret_cast<FoldArgs *>(stage.host);
    A = FoldArgs{};
    A.in[0] = Gin; A.in[1] = Hin;
    A.out[0] = AS_GEC(Gout); A.out[1] = AS_GEC(Hout);
    A.h = h;
    wnaf4_schedule(rhoG_a, A.sc[0]); wnaf4_schedule(rhoG_b, A.sc[1]);
    wnaf4_schedule(rhoH_a, A.sc[2]); wnaf4_schedule(rhoH_b, A.sc[3]);
    // lanes i < n <= h + i pair a real gate with padding and use rho_b
    const uint32_t a = n > h ? std::min(n - h, h) : 0, bnd = std::min(n, h);
    uint32_t blocks = 0;
    for (uint32_t v = 0; v < 2; v++) {
        const uint32_t lo[3] = {0, a, bnd}, hi[3] = {a, bnd, h}, cls[3] = {0, 1, 0};
        for (int c = 0; c < 3; c++) {
            if (hi[c] <= lo[c]) continue;
            uint32_t k = A.nseg++;
            A.start[k] = lo[c]; A.end[k] = hi[c]; A.vec[k] = v; A.sched[k] = 2 * v + cls[c];
            A.blk0[k] = blocks;
            blocks += nblk(hi[c] - lo[c], 64);
        }
    }
    A.blk0[A.nseg] = blocks;
    if (!blocks) return;
    BPG_HIP(hipMemcpyAsync(stage.dev, stage.host, sizeof(FoldArgs), hipMemcpyHostToDevice, st));
    BPG_HIP(hipEventRecord(stage.copied, st));
    // reads P_L, P_R of G and H, writes G', H': 6 x 64 B per lane pair;
    // per lane: doublings (3M+4S), digit additions (8M), odd multiples, final add
    double fem = 0;
    for (uint32_t k = 0; k < A.nseg; k++) {
        const FoldSched &S = A.sc[A.sched[k]];
        uint32_t dbl = S.tail;
        for (uint32_t d = 1; d < S.ndig; d++) dbl += S.gap[d];
        fem += (double)(A.end[k] - A.start[k]) * (7.0 * dbl + 8.0 * S.ndig + 40.0);
    }
    ProfScope ps(in_fmt == MSM_NIELS ? "ipp_fold_points_niels" : "ipp_fold_points", 6.0 * h * 64, fem);
    if (in_fmt == MSM_NIELS)
        hipLaunchKernelGGL(k_ipp_fold_points<gen>, dim3(blocks), dim3(64), 0, st, reinterpret_cast<const FoldArgs *>(stage.dev));
    else
        hipLaunchKernelGGL(k_ipp_fold_points<gec>, dim3(blocks), dim3(64), 0, st, reinterpret_cast<const FoldArgs *>(stage.dev));
    BPG_HIP(hipGetLastError());
}
// ---------------------------------------------------------------------------
// Two-round Straus fold (DESIGN.md "IPP fold in round pairs"). Lane i of the
// output (level k+2) is P_i + c1 P_{i+h1} + c2 P_{i+2h1} + c3 P_{i+3h1} over
// the level-k points: one shared chain of ~252 doublings with the width-WN
// NAF digits of the three scalars interleaved, instead of three single-scalar
// folds (~3 x 252 doublings over 1.5x the lanes). The scalars are uniform per
// lane range, so the merged op list (doublings before each addition, which
// point, which odd multiple, sign) is built on the host and read with scalar
// loads; blocks never straddle a range.
// ---------------------------------------------------------------------------
static constexpr int BPG_FOLD2_WNAF = 3;   // odd multiples P, 3P of the three points in registers
#define FOLD2_MAXSEG (2 * COMB_MAXRANGE)
#define FOLD2_MAXOPS 400
struct Fold2Args {
    const void *in[2];
    gec *out[2];
    uint32_t h1, nseg;
    uint32_t start[FOLD2_MAXSEG], end[FOLD2_MAXSEG], blk0[FOLD2_MAXSEG + 1], vec[FOLD2_MAXSEG];
    uint32_t nops[FOLD2_MAXSEG], tail[FOLD2_MAXSEG];
    // op: gap (doublings before it, 8 bits) | t << 8 (point 0..2) | (m >> 1) << 10 (odd multiple m) | neg << 15
    uint16_t ops[FOLD2_MAXSEG][FOLD2_MAXOPS];
};
// op k of a segment's list, read as a 32-bit word: the index is uniform, so
// this is a scalar load (a 16-bit read is a vector load plus a full vmcnt
// wait per op)
DEVI uint32_t fold2_op(const uint16_t *ops, uint32_t k) {
    const uint32_t w = reinterpret_cast<const uint32_t *>(ops)[k >> 1];
    return (k & 1) ? w >> 16 : w & 0xffffu;
}
// LSB-first width-w NAF of a canonical scalar; returns the digit count
static int wnaf_digits(const ScD &k, int w, int8_t d[264]) {
    uint32_t x[9];
    for (int i = 0; i < 8; i++) x[i] = k.v[i];
    x[8] = 0;
    const int full = 1 << w, half = full >> 1;
    int len = 0;
    auto nz = [&]() { for (int i = 0; i < 9; i++) if (x[i]) return true; return false; };
    while (nz()) {
        if (len >= 264) throw HipError(hipErrorInvalidValue, "wnaf length", __FILE__, __LINE__);
        int di = 0;
        if (x[0] & 1) {
            di = (int)(x[0] & (uint32_t)(full - 1));
            if (di >= half) di -= full;
            if (di > 0) {
                uint64_t bw = (uint64_t)di;
                for (int i = 0; i < 9 && bw; i++) { uint64_t t = (uint64_t)x[i] - bw; x[i] = (uint32_t)t; bw = (t >> 63) & 1; }
            } else {
                uint64_t c = (uint64_t)(-di);
                for (int i = 0; i < 9 && c; i++) { c += x[i]; x[i] = (uint32_t)c; c >>= 32; }
            }
        }
        d[len++] = (int8_t)di;
        for (int i = 0; i < 8; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
        x[8] >>= 1;
    }
    return len;
}
// selects the cached multiple m (1 or 3) of point t; uniform branches
template <int WN>
DEVI void fold2_pick(gec &r, const gec (&tp)[3][WN == 3 ? 2 : 1], uint32_t t, uint32_t mi) {
    if constexpr (WN == 3) {
        if (t == 0) r = mi ? tp[0][1] : tp[0][0];
        else if (t == 1) r = mi ? tp[1][1] : tp[1][0];
        else r = mi ? tp[2][1] : tp[2][0];
    } else {
        (void)mi;
        if (t == 0) r = tp[0][0]; else if (t == 1) r = tp[1][0]; else r = tp[2][0];
    }
}
// WN = 3: odd multiples P, 3P of the three points in registers (one wave per
// SIMD); WN = 2: P only (NAF, two waves per SIMD)
template <class P, int WN>
__global__ __launch_bounds__(64, WN == 3 ? 1 : 2) void k_ipp_fold2(const Fold2Args *__restrict__ Ap) {
    const Fold2Args &A = *Ap;
    uint32_t b = blockIdx.x, sg = 0;
    for (uint32_t k = 1; k < A.nseg; k++) if (b >= A.blk0[k]) sg = k;
    const uint32_t i = A.start[sg] + (b - A.blk0[sg]) * 64 + threadIdx.x;
    if (i >= A.end[sg]) return;
    const uint32_t v = A.vec[sg], nops = A.nops[sg];
    const P *Pin = reinterpret_cast<const P *>(A.in[v]);
    const uint16_t *ops = A.ops[sg];
    const uint32_t h1 = A.h1;
    gec P0;
    if (nops == 0) {
        load_as_cached(P0, Pin + i);
        gec_store(A.out[v] + i, P0);
        return;
    }
    gec tp[3][WN == 3 ? 2 : 1];
#pragma unroll
    for (int t = 0; t < 3; t++) {
        load_as_cached(tp[t][0], Pin + (size_t)(t + 1) * h1 + i);
        if constexpr (WN == 3) {
        ge pr, p2, q;
        fe_sub(pr.X, tp[t][0].YpX, tp[t][0].YmX);   // projective (2X : 2Y : 2Z), enough to double
        fe_add(pr.Y, tp[t][0].YpX, tp[t][0].YmX);
        pr.Z = tp[t][0].Z2;
        ge_dbl(p2, pr);
        ge_add_c(q, p2, tp[t][0]);
        ge_to_cached(tp[t][1], q);
        }
    }
    ge acc;
    {
        const uint32_t op = fold2_op(ops, 0);
        gec c;
        fold2_pick<WN>(c, tp, (op >> 8) & 3, (op >> 10) & 31);
        if (op >> 15) gec_neg(c, c);
        ge_from_cached(acc, c);
    }
    for (uint32_t k = 1; k < nops; k++) {
        const uint32_t op = fold2_op(ops, k);
        const uint32_t g = op & 255;
        if (g) {
            for (uint32_t j = 1; j < g; j++) ge_dbl_t<false>(acc, acc);
            ge_dbl_t<true>(acc, acc);
        }
        gec c;
        fold2_pick<WN>(c, tp, (op >> 8) & 3, (op >> 10) & 31);
        // T only when another addition follows directly (wave-uniform)
        if ((k + 1 < nops ? (fold2_op(ops, k + 1) & 255) : A.tail[sg]) == 0) {
            if (op >> 15) ge_sub_c_t<true>(acc, acc, c); else ge_add_c_t<true>(acc, acc, c);
        } else {
            if (op >> 15) ge_sub_c_t<false>(acc, acc, c); else ge_add_c_t<false>(acc, acc, c);
        }
    }
    const uint32_t tail = A.tail[sg];
    if (tail) {
        for (uint32_t j = 1; j < tail; j++) ge_dbl_t<false>(acc, acc);
        ge_dbl_t<true>(acc, acc);
    }
    load_as_cached(P0, Pin + i);
    ge r;
    ge_add_c(r, acc, P0);
    gec out;
    ge_to_cached(out, r);
    gec_store(A.out[v] + i, out);
}
void launch_ipp_fold2(const void *Gin, const void *Hin, int in_fmt, uint32_t h1, uint32_t nrange,
                      const uint32_t *rstart, const ScD (*coef)[COMB_MAXRANGE][3], PtD *Gout, PtD *Hout,
                      ArgStage &stage, hipStream_t st) {
    if (!h1) return;
    if (nrange < 1 || nrange > COMB_MAXRANGE) throw HipError(hipErrorInvalidValue, "fold2 ranges", __FILE__, __LINE__);
    if (!stage.dev) {
        BPG_HIP(hipMalloc(&stage.dev, sizeof(Fold2Args)));
        BPG_HIP(hipHostMalloc(&stage.host, sizeof(Fold2Args), hipHostMallocDefault));
        BPG_HIP(hipEventCreateWithFlags(&stage.copied, hipEventBlockingSync | hipEventDisableTiming));
    } else {
        event_wait(stage.copied);   // previous upload has left the host buffer
    }
    Fold2Args &A = *reinterpret_cast<Fold2Args *>(stage.host);
    A.in[0] = Gin; A.in[1] = Hin;
    A.out[0] = AS_GEC(Gout); A.out[1] = AS_GEC(Hout);
    A.h1 = h1;
    A.nseg = 0;
    uint32_t blocks = 0;
    double fem = 0;
    constexpr int WN = BPG_FOLD2_WNAF;
    for (uint32_t v = 0; v < 2; v++)
        for (uint32_t r = 0; r < nrange; r++) {
            const uint32_t lo = rstart[r], hi = r + 1 < nrange ? rstart[r + 1] : h1;
            if (hi <= lo) continue;
            const uint32_t s = A.nseg++;
            A.start[s] = lo; A.end[s] = hi; A.vec[s] = v; A.blk0[s] = blocks;
            blocks += nblk(hi - lo, 64);
            int8_t d[3][264];
            int len[3], top = -1;
            for (int t = 0; t < 3; t++) {
                len[t] = wnaf_digits(coef[v][r][t], WN, d[t]);
                top = std::max(top, len[t] - 1);
            }
            uint32_t n = 0, dbl = 0;
            int last = -1;
            for (int pos = top; pos >= 0; pos--)
                for (int t = 0; t < 3; t++) {
                    if (pos >= len[t] || !d[t][pos]) continue;
                    if (n >= FOLD2_MAXOPS) throw HipError(hipErrorInvalidValue, "fold2 ops", __FILE__, __LINE__);
                    const int dg = d[t][pos], m = dg < 0 ? -dg : dg;
                    const uint32_t gap = last < 0 ? 0u : (uint32_t)(last - pos);
                    if (gap > 255) throw HipError(hipErrorInvalidValue, "fold2 gap", __FILE__, __LINE__);
                    A.ops[s][n++] = (uint16_t)(gap | ((uint32_t)t << 8) | ((uint32_t)(m >> 1) << 10) |
                                               ((dg < 0 ? 1u : 0u) << 15));
                    dbl += gap;
                    last = pos;
                }
            A.nops[s] = n;
            A.tail[s] = last < 0 ? 0u : (uint32_t)last;
            dbl += A.tail[s];
            fem += (double)(hi - lo) * (7.0 * dbl + 8.0 * n + (WN == 3 ? 3 * 17.0 : 0.0) + 12.0);
        }
    A.blk0[A.nseg] = blocks;
    if (!blocks) return;
    BPG_HIP(hipMemcpyAsync(stage.dev, stage.host, sizeof(Fold2Args), hipMemcpyHostToDevice, st));
    BPG_HIP(hipEventRecord(stage.copied, st));
    // reads 4 points, writes 1 per output lane, G and H (SURVEY §8d accounting)
    ProfScope ps(in_fmt == MSM_NIELS ? "ipp_fold2_niels" : "ipp_fold2", 2.0 * h1 * 5 * 64, fem);
    const Fold2Args *dA = reinterpret_cast<const Fold2Args *>(stage.dev);
    if (in_fmt == MSM_NIELS) hipLaunchKernelGGL((k_ipp_fold2<gen, WN>), dim3(blocks), dim3(64), 0, st, dA);
    else hipLaunchKernelGGL((k_ipp_fold2<gec, WN>), dim3(blocks), dim3(64), 0, st, dA);
    BPG_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Three-round Straus fold (DESIGN.md "IPP fold in round triples"): lane i of
// level k+3 is sum_{t<8} c_t P_{i + t hq} over the level-k points (c_0 = 1):
// seven scalar multiples sharing one chain of ~252 doublings. The odd
// multiples P, 3P (WN = 3) or P..7P (WN = 4) of the seven points sit in a
// per-block global table, word-major (lane-contiguous, so every table read
// is coalesced); the next op's entry is loaded before the doublings.
// ---------------------------------------------------------------------------
// NAF width 4 (odd multiples P..7P); width 5 measured no better (fewer
// additions, twice the table, profiles/r02w_ab_fold3_w5.txt)
static constexpr int BPG_FOLD3_WNAF = 4;
// segments: (proof, vector, lane range); every proof of a lockstep step in
// one launch (round 6: one launch and one argument upload per step instead
// of one of each per proof)
#define FOLDN_MAXSEG (2 * COMB_MAXRANGE * 4)
#define FOLDN_MAXOPS 640
static constexpr int FOLDN_K = 7;
static constexpr int FOLDN_MULT = 1 << (BPG_FOLD3_WNAF - 2);           // odd multiples per point
static constexpr uint32_t FOLDN_TABW = FOLDN_K * FOLDN_MULT * 40 * 64;  // table words per block
struct FoldNArgs {
    uint32_t *tab;             // blocks x FOLDN_TABW words
    uint32_t hq, nseg;
    const void *in[FOLDN_MAXSEG];   // the segment's level (its proof's G or H)
    gec *out[FOLDN_MAXSEG];
    uint32_t start[FOLDN_MAXSEG], end[FOLDN_MAXSEG], blk0[FOLDN_MAXSEG + 1];
    uint32_t nops[FOLDN_MAXSEG], tail[FOLDN_MAXSEG];
    // op: gap (8 bits) | point t - 1 << 8 (3 bits) | (m >> 1) << 11 (3 bits) | neg << 15
    // (uploaded up to the last segment's list only)
    uint16_t ops[FOLDN_MAXSEG][FOLDN_MAXOPS];
};
DEVI void foldn_put(uint32_t *tb, const gec &c) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&c);
#pragma unroll
    for (int k = 0; k < 40; k++) tb[k * 64] = w[k];
}
DEVI void foldn_get(gec &c, const uint32_t *tb) {
    uint32_t *w = reinterpret_cast<uint32_t *>(&c);
#pragma unroll
    for (int k = 0; k < 40; k++) w[k] = tb[k * 64];
}
// waves per SIMD the triple fold is compiled for (332 VGPRs; at 2 waves
// it spilled and measured slower, profiles/r03c_ab_commitjob_fold3_smallmsm.txt;
// a 2-wave form loading each table operand coordinate by coordinate fit
// without spills but measured 1.2% slower, profiles/r04l_ab.txt)
static constexpr int FOLD3_WAVES = 1;
// the lane's odd multiples P, 3P, .. of the seven points into the block's
// word-major table
template <class P>
DEVI void foldn_build(const P *Pin, uint32_t hq, uint32_t i, uint32_t *tb) {
    for (int t = 0; t < FOLDN_K; t++) {
        gec c1;
        load_as_cached(c1, Pin + (size_t)(t + 1) * hq + i);
        foldn_put(tb + (t * FOLDN_MULT) * 40 * 64, c1);
        ge pr, p2, q;
        fe_sub(pr.X, c1.YpX, c1.YmX);   // projective (2X : 2Y : 2Z), enough to double
        fe_add(pr.Y, c1.YpX, c1.YmX);
        pr.Z = c1.Z2;
        ge_dbl(p2, pr);
        ge_add_c(q, p2, c1);             // 3P
        gec c;
        ge_to_cached(c, q);
        foldn_put(tb + (t * FOLDN_MULT + 1) * 40 * 64, c);
        if constexpr (FOLDN_MULT > 2) {
            gec d2;
            ge_to_cached(d2, p2);
            for (int m = 2; m < FOLDN_MULT; m++) {   // (2m+1)P = (2m-1)P + 2P
                ge_add_c(q, q, d2);
                ge_to_cached(c, q);
                foldn_put(tb + (t * FOLDN_MULT + m) * 40 * 64, c);
            }
        }
    }
}
DEVI const uint32_t *foldn_entry(const uint32_t *tb, uint32_t op) {
    return tb + (((op >> 8) & 7) * FOLDN_MULT + ((op >> 11) & 7)) * 40 * 64;
}
// The Straus chain over a built table, then + P_i, out as a cached point.
template <class P>
DEVI void foldn_chain(const FoldNArgs &A, uint32_t sg, const P *Pin, uint32_t i, const uint32_t *tb) {
    const uint32_t nops = A.nops[sg];
    const uint16_t *ops = A.ops[sg];
    ge acc;
    {
        const uint32_t op = fold2_op(ops, 0);
        gec c;
        foldn_get(c, foldn_entry(tb, op));
        if (op >> 15) gec_neg(c, c);
        ge_from_cached(acc, c);
    }
    // the next op's table entry is loaded before the doublings
    gec c;
    if (nops > 1) foldn_get(c, foldn_entry(tb, fold2_op(ops, 1)));
    for (uint32_t k = 1; k < nops; k++) {
        const uint32_t op = fold2_op(ops, k);
        const uint32_t g = op & 255;
        gec cn;
        if (k + 1 < nops) foldn_get(cn, foldn_entry(tb, fold2_op(ops, k + 1)));
        if (g) {
            for (uint32_t j = 1; j < g; j++) ge_dbl_t<false>(acc, acc);
            ge_dbl_t<true>(acc, acc);
        }
        // (skipping T before a doubling, as k_ipp_fold2 does, measured 4%
        // slower here: 7.6 vs 7.3 s of bracketed fold time per step,
        // profiles/r03j_ab_tskip_seglen.txt)
        if (op >> 15) ge_sub_c(acc, acc, c); else ge_add_c(acc, acc, c);
        c = cn;
    }
    const uint32_t tail = A.tail[sg];
    if (tail) {
        for (uint32_t j = 1; j < tail; j++) ge_dbl_t<false>(acc, acc);
        ge_dbl_t<true>(acc, acc);
    }
    gec P0;
    load_as_cached(P0, Pin + i);
    ge r;
    ge_add_c(r, acc, P0);
    gec out;
    ge_to_cached(out, r);
    gec_store(A.out[sg] + i, out);
}
DEVI bool foldn_lane(const FoldNArgs &A, uint32_t &sg, uint32_t &i) {
    const uint32_t b = blockIdx.x;
    sg = 0;
    for (uint32_t k = 1; k < A.nseg; k++) if (b >= A.blk0[k]) sg = k;
    i = A.start[sg] + (b - A.blk0[sg]) * 64 + threadIdx.x;
    return i < A.end[sg];
}
template <class P>
__global__ __launch_bounds__(64, FOLD3_WAVES) void k_ipp_fold3(const FoldNArgs *__restrict__ Ap) {
    WAVE_PRIO(BPG_FOLD_PRIO);
    const FoldNArgs &A = *Ap;
    uint32_t sg, i;
    if (!foldn_lane(A, sg, i)) return;
    const P *Pin = reinterpret_cast<const P *>(A.in[sg]);
    if (A.nops[sg] == 0) {
        gec P0;
        load_as_cached(P0, Pin + i);
        gec_store(A.out[sg] + i, P0);
        return;
    }
    uint32_t *tb = A.tab + (size_t)blockIdx.x * FOLDN_TABW + threadIdx.x;
    foldn_build(Pin, A.hq, i, tb);
    foldn_chain(A, sg, Pin, i, tb);
}
size_t ipp_fold3_table_bytes(uint32_t hq, uint32_t nrange) {
    // blocks: per vector and range, whole 64-lane blocks (one proof's)
    return ((size_t)2 * (hq / 64 + nrange + 1)) * FOLDN_TABW * 4;
}
void launch_ipp_fold3(const void *const *Gin, const void *const *Hin, int in_fmt, uint32_t hq, uint32_t nrange,
                      const uint32_t *rstart, const ScD (*const *coef)[COMB_MAXRANGE][7], PtD *const *Gout,
                      PtD *const *Hout, int P, void *tab, size_t tab_bytes, ArgStage &stage, hipStream_t st) {
    if (!hq) return;
    if (nrange < 1 || nrange > COMB_MAXRANGE) throw HipError(hipErrorInvalidValue, "fold3 ranges", __FILE__, __LINE__);
    if (P < 1 || P > 4) throw HipError(hipErrorInvalidValue, "fold3 proofs", __FILE__, __LINE__);
    if (!stage.dev) {
        BPG_HIP(hipMalloc(&stage.dev, sizeof(FoldNArgs)));
        BPG_HIP(hipHostMalloc(&stage.host, sizeof(FoldNArgs), hipHostMallocDefault));
        BPG_HIP(hipEventCreateWithFlags(&stage.copied, hipEventBlockingSync | hipEventDisableTiming));
    } else {
        event_wait(stage.copied);
    }
    FoldNArgs &A = *reinterpret_cast<FoldNArgs *>(stage.host);
    A.tab = reinterpret_cast<uint32_t *>(tab);
    A.hq = hq;
    A.nseg = 0;
    uint32_t blocks = 0;
    double fem = 0;
    constexpr int WN = BPG_FOLD3_WNAF;
    for (int p = 0; p < P; p++)
    for (uint32_t v = 0; v < 2; v++)
        for (uint32_t r = 0; r < nrange; r++) {
            const uint32_t lo = rstart[r], hi = r + 1 < nrange ? rstart[r + 1] : hq;
            if (hi <= lo) continue;
            const uint32_t s = A.nseg++;
            A.start[s] = lo; A.end[s] = hi; A.blk0[s] = blocks;
            A.in[s] = v ? Hin[p] : Gin[p];
            A.out[s] = AS_GEC(v ? Hout[p] : Gout[p]);
            blocks += nblk(hi - lo, 64);
            int8_t d[FOLDN_K][264];
            int len[FOLDN_K], top = -1;
            for (int t = 0; t < FOLDN_K; t++) {
                len[t] = wnaf_digits(coef[p][v][r][t], WN, d[t]);
                top = std::max(top, len[t] - 1);
            }
            uint32_t n = 0, dbl = 0;
            int last = -1;
            for (int pos = top; pos >= 0; pos--)
                for (int t = 0; t < FOLDN_K; t++) {
                    if (pos >= len[t] || !d[t][pos]) continue;
                    if (n >= FOLDN_MAXOPS) throw HipError(hipErrorInvalidValue, "fold3 ops", __FILE__, __LINE__);
                    const int dg = d[t][pos], m = dg < 0 ? -dg : dg;
                    const uint32_t gap = last < 0 ? 0u : (uint32_t)(last - pos);
                    if (gap > 255) throw HipError(hipErrorInvalidValue, "fold3 gap", __FILE__, __LINE__);
                    A.ops[s][n++] = (uint16_t)(gap | ((uint32_t)t << 8) | ((uint32_t)(m >> 1) << 11) |
                                               ((dg < 0 ? 1u : 0u) << 15));
                    dbl += gap;
                    last = pos;
                }
            A.nops[s] = n;
            A.tail[s] = last < 0 ? 0u : (uint32_t)last;
            dbl += A.tail[s];
            fem += (double)(hi - lo) * (7.0 * dbl + 8.0 * n + FOLDN_K * (7.0 + 9.0 * (FOLDN_MULT - 1)) + 12.0);
        }
    A.blk0[A.nseg] = blocks;
    if (!blocks) return;
    if ((size_t)blocks * FOLDN_TABW * 4 > tab_bytes) throw HipError(hipErrorInvalidValue, "fold3 table", __FILE__, __LINE__);
    // the used segments' op lists only (ops is the struct's last member)
    const size_t bytes = offsetof(FoldNArgs, ops) + (size_t)A.nseg * sizeof(A.ops[0]);
    BPG_HIP(hipMemcpyAsync(stage.dev, stage.host, bytes, hipMemcpyHostToDevice, st));
    BPG_HIP(hipEventRecord(stage.copied, st));
    // reads 8 points, writes 1 per output lane, G and H, every proof (SURVEY §8d accounting)
    ProfScope ps(in_fmt == MSM_NIELS ? "ipp_fold3" : "ipp_fold3_cached", 2.0 * P * hq * 9 * 64, fem);   // one label per kernel
    const FoldNArgs *dA = reinterpret_cast<const FoldNArgs *>(stage.dev);
    if (in_fmt == MSM_NIELS) hipLaunchKernelGGL(k_ipp_fold3<gen>, dim3(blocks), dim3(64), 0, st, dA);
    else hipLaunchKernelGGL(k_ipp_fold3<gec>, dim3(blocks), dim3(64), 0, st, dA);
    BPG_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Comb tables and the two-round table fold (DESIGN.md "IPP rounds 0-1").
// For generator j = j0 + jj (jj < ntab): entry (w, d) = (d+1) R^w P_j,
// R = 2^COMB_BITS, for w < COMB_WIN, d < COMB_ENT, packed affine Niels (96 B)
// at 16-byte unit ((w*COMB_ENT + d) * ntab + jj) * 6 — entry-major, so lanes
// that read the same entry of consecutive generators read one contiguous span.
void comb_digits(const uint8_t s[32], int8_t e[64]) {
    int v[64] = {0};
    for (int i = 0; i < COMB_WIN; i++) {
        const int bit = COMB_BITS * i;
        uint32_t x = 0;
        for (int b = 0; b < COMB_BITS; b++) {
            const int p = bit + b;
            if (p < 256) x |= (uint32_t)((s[p >> 3] >> (p & 7)) & 1) << b;
        }
        v[i] = (int)x;
    }
    for (int i = 0; i + 1 < COMB_WIN; i++) {   // recentre into [-COMB_ENT, COMB_ENT)
        const int c = (v[i] + COMB_ENT) >> COMB_BITS;
        v[i] -= c << COMB_BITS;
        v[i + 1] += c;
    }
    for (int i = 0; i < 64; i++) e[i] = (int8_t)(i < COMB_WIN ? v[i] : 0);
}
// ---------------------------------------------------------------------------
// One generator per lane. Entries go out as affine Niels, so each needs
// 1/Z: the entries of a chunk of COMB_BATCH consecutive multiples are first
// parked in their own slots as packed (X, Y, Z) with the running product of
// the Z's in registers, then one inversion and a backward walk give every
// 1/Z (Montgomery's trick: 3M per entry instead of an inversion each).
#define COMB_BATCH (COMB_ENT < 16 ? COMB_ENT : 16)
__global__ __launch_bounds__(64) void k_comb_build(const gen *__restrict__ gens, uint32_t j0, uint32_t ntab,
                                                   uint4 *__restrict__ tab) {
    const uint32_t jj = blockIdx.x * blockDim.x + threadIdx.x;
    if (jj >= ntab) return;
    gen g;
    gen_load(g, gens + j0 + jj);
    gec c;
    gen_to_cached(c, g);
    ge pw;
    ge_from_cached(pw, c);
    for (int w = 0; w < COMB_WIN; w++) {
        gec pc;
        ge_to_cached(pc, pw);
        ge q = pw;
        for (int d0 = 0; d0 < COMB_ENT; d0 += COMB_BATCH) {
            fe pre[COMB_BATCH];
#pragma unroll
            for (int b = 0; b < COMB_BATCH; b++) {
                const int d = d0 + b;
                if (d) ge_add_c(q, q, pc);
                uint32_t xw[24];
                fe_tow(xw, q.X); fe_tow(xw + 8, q.Y); fe_tow(xw + 16, q.Z);
                uint4 *slot = tab + ((size_t)(w * COMB_ENT + d) * ntab + jj) * 6;
#pragma unroll
                for (int k = 0; k < 6; k++) slot[k] = make_uint4(xw[4 * k], xw[4 * k + 1], xw[4 * k + 2], xw[4 * k + 3]);
                if (b) fe_mul(pre[b], pre[b - 1], q.Z); else pre[b] = q.Z;
            }
            fe inv;
            fe_invert(inv, pre[COMB_BATCH - 1]);
#pragma unroll
            for (int b = COMB_BATCH - 1; b >= 0; b--) {
                uint4 *slot = tab + ((size_t)(w * COMB_ENT + d0 + b) * ntab + jj) * 6;
                uint4 s6[6];
#pragma unroll
                for (int k = 0; k < 6; k++) s6[k] = slot[k];
                fe X = fe_from_words(s6[0].x, s6[0].y, s6[0].z, s6[0].w, s6[1].x, s6[1].y, s6[1].z, s6[1].w);
                fe Y = fe_from_words(s6[2].x, s6[2].y, s6[2].z, s6[2].w, s6[3].x, s6[3].y, s6[3].z, s6[3].w);
                fe zi, x, y, t;
                if (b) {
                    fe Z = fe_from_words(s6[4].x, s6[4].y, s6[4].z, s6[4].w, s6[5].x, s6[5].y, s6[5].z, s6[5].w);
                    fe_mul(zi, inv, pre[b - 1]);
                    fe_mul(inv, inv, Z);
                } else {
                    zi = inv;
                }
                fe_mul(x, X, zi); fe_mul(y, Y, zi);
                gen e;
                fe_add(e.YpX, y, x); fe_sub(e.YmX, y, x);
                fe_mul(t, x, y); fe_mul(e.T2d, t, FE_D2);
                e.pad[0] = e.pad[1] = 0;
                genp_store(slot, e);
            }
        }
        ge_dbl(pw, q);   // R^(w+1) P = 2 (COMB_ENT R^w P)
    }
}
void launch_comb_build(const NielsD *gens, uint32_t j0, uint32_t ntab, void *tab, hipStream_t st) {
    if (!ntab) return;
    hipLaunchKernelGGL(k_comb_build, dim3(nblk(ntab, 64)), dim3(64), 0, st, AS_CGEN(gens), j0, ntab,
                       reinterpret_cast<uint4 *>(tab));
    BPG_HIP(hipGetLastError());
}

// Output lane i < h1 of vector v (0 = G, 1 = H):
//   out_i = P_i + sum_{t<3} c_t * P_{i + (t+1) h1}
// with per-lane-range coefficient digits (signed radix 2^COMB_BITS, LSB
// first); no doublings: every nonzero digit is one table read and one 7M madd.
// The arguments (3.2 KB with the digit lists) travel by value in the
// kernel-argument segment: no staged upload, i.e. no copy launch per fold
// (round 6; they were a __amd_rocclr_copyBuffer dispatch before each fold)
__global__ __launch_bounds__(64, 2) void k_ipp_comb_fold(const CombArgs A) {
    WAVE_PRIO(BPG_COMB_PRIO);
    const uint32_t nb = (A.h1 + 63) / 64;
    const uint32_t v = blockIdx.x >= nb ? 1 : 0;
    const uint32_t i = (blockIdx.x - v * nb) * 64 + threadIdx.x;
    if (i >= A.h1) return;
    uint32_t r = 0;
#pragma unroll
    for (int k = 1; k < COMB_MAXRANGE; k++) if (k < (int)A.nrange && i >= A.rstart[k]) r = k;
    const uint4 *tab = reinterpret_cast<const uint4 *>(A.tab[v]);
    ge acc;
    {
        gen p;
        gen_load(p, reinterpret_cast<const gen *>(A.gens[v]) + i);
        ge_from_niels(acc, p);   // identity + P_i (1M)
    }
    for (int t = 0; t < 3; t++) {
        const uint32_t jj = i + (uint32_t)t * A.h1;
        const uint32_t *dw = reinterpret_cast<const uint32_t *>(A.dig[v][r][t]);
        for (int w4 = 0; w4 < (COMB_WIN + 3) / 4; w4++) {
            const uint32_t packed = dw[w4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int d = (int)(int8_t)(packed >> (8 * k));
                if (d == 0) continue;
                const int w = 4 * w4 + k;
                const int m = d < 0 ? -d : d;
                const uint4 *e = tab + ((size_t)(w * COMB_ENT + m - 1) * A.ntab + jj) * 6;
                uint4 q[6];
#pragma unroll
                for (int u = 0; u < 6; u++) q[u] = e[u];
                gen p;
                genp_unpack(p, q);
                gen_cneg(p, d < 0);
                ge_madd(acc, acc, p);
            }
        }
    }
    gec out;
    ge_to_cached(out, acc);
    gec_store(reinterpret_cast<gec *>(A.out[v]) + i, out);
}
void launch_ipp_comb_fold(const CombArgs &args, ArgStage &stage, hipStream_t st) {
    if (!args.h1) return;
    (void)stage;
    static_assert(sizeof(CombArgs) <= 4096, "comb fold arguments must fit the kernel-argument segment");
    const uint32_t nb = (args.h1 + 63) / 64;
    // reads 4 level-0 points, writes 1 level-2 point per lane, G and H;
    // one 7M madd per nonzero digit (+ the base term and the cached output)
    double fem = 0;
    for (uint32_t v = 0; v < 2; v++)
        for (uint32_t r = 0; r < args.nrange; r++) {
            const uint32_t lo = args.rstart[r], hi = r + 1 < args.nrange ? args.rstart[r + 1] : args.h1;
            uint32_t nz = 0;
            for (int t = 0; t < 3; t++) for (int w = 0; w < 64; w++) nz += args.dig[v][r][t][w] != 0;
            fem += (double)(hi - lo) * (7.0 * (nz + 1) + 1.0);
        }
    ProfScope ps("ipp_comb_fold", 2.0 * args.h1 * (4 * 64 + 64), fem);
    hipLaunchKernelGGL(k_ipp_comb_fold, dim3(2 * nb), dim3(64), 0, st, args);
    BPG_HIP(hipGetLastError());
}

// IPP round 1 with the level-1 generators left unmaterialised: each base of
// the round, G1_j = G_j + rho0(j) G_{j+h0} (likewise H), is expanded into its
// two level-0 generators, so the round's MSM scalars double (8h of them).
// Layout: [L: G_A | G_B | H_A | H_B | R: G_A | G_B | H_A | H_B], c_L at 8h,
// c_R at 8h+1. rho0 classes as in the fold (pair straddles n -> *_b).
DEVI void ipp_prep_lazy_body(const sc *__restrict__ a, const sc *__restrict__ b,
                                                       const sc *__restrict__ yipm, const IppRoundArgs &A, const LazyArgs &Z,
                                                       sc *__restrict__ out, sc *__restrict__ partial, sc *__restrict__ red_out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[2];
    sc_zero(acc[0]); sc_zero(acc[1]);
    const uint32_t h = A.h, h0 = Z.h0, n = A.n;
    const sc lamG1 = *reinterpret_cast<const sc *>(&A.lamG1), lamGu = *reinterpret_cast<const sc *>(&A.lamGu);
    const sc muH1 = *reinterpret_cast<const sc *>(&A.muH1), muHu = *reinterpret_cast<const sc *>(&A.muHu);
    const sc rGa = *reinterpret_cast<const sc *>(&Z.rGa), rGb = *reinterpret_cast<const sc *>(&Z.rGb);
    const sc rHa = *reinterpret_cast<const sc *>(&Z.rHa), rHb = *reinterpret_cast<const sc *>(&Z.rHb);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < h; i += gridDim.x * blockDim.x) {
        sc aL, aR, bL, bR, t, u, y;
        sc_load(aL, a + i); sc_load(aR, a + h + i); sc_load(bL, b + i); sc_load(bR, b + h + i);
        mm(t, aL, bR); sc_add(acc[0], acc[0], t);
        mm(t, aR, bL); sc_add(acc[1], acc[1], t);
        const uint32_t lo = i, hi = h + i;
        const bool lo_real = lo < n, hi_real = hi < n;
        const bool lo_b = lo < n && lo + h0 >= n, hi_b = hi < n && hi + h0 >= n;
        // L, G part: base G1_{h+i}
        mm(t, aL, hi_real ? lamG1 : lamGu); sc_store(out + i, t);
        mm(u, t, hi_b ? rGb : rGa); sc_store(out + h + i, u);
        // L, H part: base H1_i
        sc_load(y, yipm + lo); mm(t, bR, y); mm(t, t, lo_real ? muH1 : muHu); sc_store(out + 2 * h + i, t);
        mm(u, t, lo_b ? rHb : rHa); sc_store(out + 3 * h + i, u);
        // R, G part: base G1_i
        mm(t, aR, lo_real ? lamG1 : lamGu); sc_store(out + 4 * h + i, t);
        mm(u, t, lo_b ? rGb : rGa); sc_store(out + 5 * h + i, u);
        // R, H part: base H1_{h+i}
        sc_load(y, yipm + hi); mm(t, bL, y); mm(t, t, hi_real ? muH1 : muHu); sc_store(out + 6 * h + i, t);
        mm(u, t, hi_b ? rHb : rHa); sc_store(out + 7 * h + i, u);
    }
    block_reduce_final<2>(acc, partial, red_out, 0);
}

// IPP tail round over the materialised level (M points per vector).
// Round k+2 of a round triple: each level-(k+2) base x (2h of them per
// vector) expanded into its four level-k points x + 2h t, t < 4, with
// coefficients (1, r1(x), r0(x), r1(x) r0(x + 2h)), r1 the round-(k+1) fold
// scalar (class: x < n <= x + 2h), r0 the round-k one (class: y < n <= y + 4h).
// Layout: family f in [L: G_hi, H_lo | R: G_lo, H_hi], term t:
// out[(4 f + t) h + i]; c_L -> out[16h], c_R -> out[16h + 1].
DEVI void ipp_prep_deep2_body(const sc *__restrict__ a, const sc *__restrict__ b,
                                                        const sc *__restrict__ yipm, const IppRoundArgs &A, const Deep2Args &Z,
                                                        sc *__restrict__ out, sc *__restrict__ partial, sc *__restrict__ red_out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[2];
    sc_zero(acc[0]); sc_zero(acc[1]);
    const uint32_t h = A.h, n = A.n;
    const sc lamG1 = *reinterpret_cast<const sc *>(&A.lamG1), lamGu = *reinterpret_cast<const sc *>(&A.lamGu);
    const sc muH1 = *reinterpret_cast<const sc *>(&A.muH1), muHu = *reinterpret_cast<const sc *>(&A.muHu);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < h; i += gridDim.x * blockDim.x) {
        sc aL, aR, bL, bR, t, s, y;
        sc_load(aL, a + i); sc_load(aR, a + h + i); sc_load(bL, b + i); sc_load(bR, b + h + i);
        mm(t, aL, bR); sc_add(acc[0], acc[0], t);
        mm(t, aR, bL); sc_add(acc[1], acc[1], t);
        const uint32_t lo = i, hi = h + i;
        const bool lo_real = lo < n, hi_real = hi < n;
        // family scalar and its level-(k+2) lane x, per family
#pragma unroll
        for (int f = 0; f < 4; f++) {
            const bool G = (f & 1) == 0;          // 0: L G_hi, 1: L H_lo, 2: R G_lo, 3: R H_hi
            const uint32_t x = (f == 0 || f == 3) ? hi : lo;
            const bool real = x < n;
            if (f == 0) mm(s, aL, real ? lamG1 : lamGu);
            else if (f == 2) mm(s, aR, real ? lamG1 : lamGu);
            else {
                sc_load(y, yipm + x);
                mm(t, f == 1 ? bR : bL, y);
                mm(s, t, real ? muH1 : muHu);
            }
            const int v = G ? 0 : 1;
            const bool c1b = x < n && x + 2 * h >= n, c0b = x < n && x + 4 * h >= n;
            const bool c3b = x + 2 * h < n && x + 6 * h >= n;
            sc *o = out + (size_t)(4 * f) * h + i;
            sc_store(o, s);
            sc u;
            const sc r1a = *reinterpret_cast<const sc *>(&Z.r1[v][0]), r1b = *reinterpret_cast<const sc *>(&Z.r1[v][1]);
            const sc r0a = *reinterpret_cast<const sc *>(&Z.r0[v][0]), r0b = *reinterpret_cast<const sc *>(&Z.r0[v][1]);
            const sc r1 = c1b ? r1b : r1a, r0x = c0b ? r0b : r0a, r0y = c3b ? r0b : r0a;
            mm(u, s, r1); sc_store(o + h, u);
            mm(t, u, r0y); sc_store(o + 3 * (size_t)h, t);
            mm(u, s, r0x); sc_store(o + 2 * (size_t)h, u);
        }
    }
    block_reduce_final<2>(acc, partial, red_out, 0);
}
DEVI void ipp_prep_tail_body(const sc *__restrict__ a, const sc *__restrict__ b,
                                                       const sc *__restrict__ yipm, const IppRoundArgs &A, uint32_t M,
                                                       const sc *__restrict__ wG, const sc *__restrict__ wH,
                                                       sc *__restrict__ out, sc *__restrict__ partial, sc *__restrict__ red_out) {
    WAVE_PRIO(BPG_MISC_PRIO);
    sc acc[2];
    sc_zero(acc[0]); sc_zero(acc[1]);
    const uint32_t h = A.h, n = A.n;
    const sc lamG1 = *reinterpret_cast<const sc *>(&A.lamG1), lamGu = *reinterpret_cast<const sc *>(&A.lamGu);
    const sc muH1 = *reinterpret_cast<const sc *>(&A.muH1), muHu = *reinterpret_cast<const sc *>(&A.muHu);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < M; j += gridDim.x * blockDim.x) {
        sc t, u, y, z;
        sc_zero(z);
        const uint32_t i = j % (2 * h);
        const bool upper = i >= h;
        const uint32_t il = upper ? i - h : i;          // lane of the round's pair (il, h + il)
        const bool lo_real = il < n, hi_real = h + il < n;
        if (j < h) {                                    // c_L, c_R over the round's lanes
            sc aL, aR, bL, bR;
            sc_load(aL, a + j); sc_load(aR, a + h + j); sc_load(bL, b + j); sc_load(bR, b + h + j);
            mm(t, aL, bR); sc_add(acc[0], acc[0], t);
            mm(t, aR, bL); sc_add(acc[1], acc[1], t);
        }
        sc w;
        sc_load(w, wG + j);
        if (upper) {                                    // base G_{h+il}: L gets aL * lam
            sc_load(t, a + il); mm(t, t, hi_real ? lamG1 : lamGu); mm(u, t, w);
            sc_store(out + j, u); sc_store(out + 2 * (size_t)M + j, z);
        } else {                                        // base G_il: R gets aR * lam
            sc_load(t, a + h + il); mm(t, t, lo_real ? lamG1 : lamGu); mm(u, t, w);
            sc_store(out + j, z); sc_store(out + 2 * (size_t)M + j, u);
        }
        sc_load(w, wH + j);
        if (!upper) {                                   // base H_il: L gets bR * y^-il * mu
            sc_load(t, b + h + il); sc_load(y, yipm + il); mm(t, t, y); mm(t, t, lo_real ? muH1 : muHu); mm(u, t, w);
            sc_store(out + (size_t)M + j, u); sc_store(out + 3 * (size_t)M + j, z);
        } else {                                        // base H_{h+il}: R gets bL * y^-(h+il) * mu
            sc_load(t, b + il); sc_load(y, yipm + h + il); mm(t, t, y); mm(t, t, hi_real ? muH1 : muHu); mm(u, t, w);
            sc_store(out + (size_t)M + j, z); sc_store(out + 3 * (size_t)M + j, u);
        }
    }
    block_reduce_final<2>(acc, partial, red_out, 0);
}
// One launch per IPP round for the P <= 4 proofs of a lockstep step
// (blockIdx.y = proof): the round preparation's scalars and its c_L / c_R
// (each proof's reduction finished by the last of its blocks).
__global__ __launch_bounds__(256) void k_ipp_prep(PrepBatch B) {
    const uint32_t p = blockIdx.y;
    ipp_prep_body(AS_CSC(B.a[p]), AS_CSC(B.b[p]), AS_CSC(B.yipm[p]), B.A[p], AS_SC(B.out[p]), AS_SC(B.partial[p]),
                  AS_SC(B.c_out[p]));
}
__global__ __launch_bounds__(256) void k_ipp_prep_lazy(PrepBatch B) {
    const uint32_t p = blockIdx.y;
    ipp_prep_lazy_body(AS_CSC(B.a[p]), AS_CSC(B.b[p]), AS_CSC(B.yipm[p]), B.A[p], B.lz[p], AS_SC(B.out[p]),
                       AS_SC(B.partial[p]), AS_SC(B.c_out[p]));
}
__global__ __launch_bounds__(256) void k_ipp_prep_deep2(PrepBatch B) {
    const uint32_t p = blockIdx.y;
    ipp_prep_deep2_body(AS_CSC(B.a[p]), AS_CSC(B.b[p]), AS_CSC(B.yipm[p]), B.A[p], B.dz[p], AS_SC(B.out[p]),
                        AS_SC(B.partial[p]), AS_SC(B.c_out[p]));
}
__global__ __launch_bounds__(256) void k_ipp_prep_tail(PrepBatch B) {
    const uint32_t p = blockIdx.y;
    ipp_prep_tail_body(AS_CSC(B.a[p]), AS_CSC(B.b[p]), AS_CSC(B.yipm[p]), B.A[p], B.M, AS_CSC(B.wG[p]),
                       AS_CSC(B.wH[p]), AS_SC(B.out[p]), AS_SC(B.partial[p]), AS_SC(B.c_out[p]));
}
void launch_ipp_prep(const PrepBatch &B, int kind, int P, hipStream_t st) {
    if (P < 1 || P > 4) throw HipError(hipErrorInvalidValue, "prep proofs", __FILE__, __LINE__);
    const uint32_t len = kind == PREP_TAIL ? B.M : B.A[0].h;
    const dim3 grid(std::max<uint32_t>(1, std::min<uint32_t>(RED_BLOCKS, nblk(len, 256))), (uint32_t)P);
    switch (kind) {
    case PREP_PLAIN: hipLaunchKernelGGL(k_ipp_prep, grid, dim3(256), 0, st, B); break;
    case PREP_LAZY: hipLaunchKernelGGL(k_ipp_prep_lazy, grid, dim3(256), 0, st, B); break;
    case PREP_DEEP2: hipLaunchKernelGGL(k_ipp_prep_deep2, grid, dim3(256), 0, st, B); break;
    default: hipLaunchKernelGGL(k_ipp_prep_tail, grid, dim3(256), 0, st, B); break;
    }
    BPG_HIP(hipGetLastError());
}
struct TailWeightArgs { sc *wG[4], *wH[4]; sc r[4][4]; };   // per proof: rGa, rGb, rHa, rHb
__global__ void k_ipp_tail_weights(TailWeightArgs A, uint32_t M, uint32_t h, uint32_t n) {
    WAVE_PRIO(BPG_MISC_PRIO);
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x, p = blockIdx.y;
    if (j >= M) return;
    const uint32_t i = j % (2 * h);
    if (i < h) return;
    const uint32_t il = i - h;
    const bool bcls = il < n && il + h >= n;
    sc *wG = A.wG[p], *wH = A.wH[p];
    sc w;
    sc_load(w, wG + j); mm(w, w, A.r[p][bcls ? 1 : 0]); sc_store(wG + j, w);
    sc_load(w, wH + j); mm(w, w, A.r[p][bcls ? 3 : 2]); sc_store(wH + j, w);
}
void launch_ipp_tail_weights(ScD *const *wG, ScD *const *wH, const ScD (*r)[4], int P, uint32_t M, uint32_t h,
                             uint32_t n, hipStream_t st) {
    if (P < 1 || P > 4) throw HipError(hipErrorInvalidValue, "tail weights proofs", __FILE__, __LINE__);
    TailWeightArgs A{};
    for (int p = 0; p < P; p++) {
        A.wG[p] = AS_SC(wG[p]); A.wH[p] = AS_SC(wH[p]);
        for (int k = 0; k < 4; k++) A.r[p][k] = *reinterpret_cast<const sc *>(&r[p][k]);
    }
    hipLaunchKernelGGL(k_ipp_tail_weights, dim3(nblk(M, 256), P), dim3(256), 0, st, A, M, h, n);
    BPG_HIP(hipGetLastError());
}

__global__ void k_fill_scalars(sc *dst, sc val, uint32_t count) {
    WAVE_PRIO(BPG_MISC_PRIO);
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) sc_store(dst + i, val);
}
struct FillBatch { sc *dst[8]; };
__global__ void k_fill_scalars_batch(FillBatch A, sc val, uint32_t count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) sc_store(A.dst[blockIdx.y] + i, val);
}
void launch_fill_scalars_batch(ScD *const *dst, int nq, ScD val, uint32_t count, hipStream_t st) {
    if (!count) return;
    if (nq < 1 || nq > 8) throw HipError(hipErrorInvalidValue, "fill batch", __FILE__, __LINE__);
    FillBatch A{};
    for (int q = 0; q < nq; q++) A.dst[q] = AS_SC(dst[q]);
    hipLaunchKernelGGL(k_fill_scalars_batch, dim3(nblk(count, 256), nq), dim3(256), 0, st, A,
                       *reinterpret_cast<sc *>(&val), count);
    BPG_HIP(hipGetLastError());
}
void launch_fill_scalars(ScD *dst, ScD val, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_fill_scalars, dim3(nblk(count, 256)), dim3(256), 0, st, AS_SC(dst), *reinterpret_cast<sc *>(&val), count);
    BPG_HIP(hipGetLastError());
}
// Strided slices for the sharded prover: dst[j] = src[j * stride + offset].
__global__ void k_gather_scalars(const sc *__restrict__ src, uint32_t count, uint32_t stride, uint32_t offset,
                                 sc *__restrict__ dst) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count) return;
    sc a;
    sc_load(a, src + (size_t)j * stride + offset);
    sc_store(dst + j, a);
}
// A_I1's split scalars: out = aL[eqI[0..nE)] | aL[dfI[0..nD)] | aR[dfI[0..nD)]
__global__ void k_eq_gather(const sc *__restrict__ aL, const sc *__restrict__ aR, const uint32_t *__restrict__ eqI,
                            uint32_t nE, const uint32_t *__restrict__ dfI, uint32_t nD, sc *__restrict__ out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nE + 2 * nD) return;
    const sc *src = j < nE + nD ? aL : aR;
    const uint32_t i = j < nE ? eqI[j] : dfI[j < nE + nD ? j - nE : j - nE - nD];
    sc v;
    sc_load(v, src + i);
    sc_store(out + j, v);
}
void launch_eq_gather(const ScD *aL, const ScD *aR, const uint32_t *eqI, uint32_t nE, const uint32_t *dfI, uint32_t nD,
                      ScD *out, hipStream_t st) {
    const uint32_t count = nE + 2 * nD;
    if (!count) return;
    hipLaunchKernelGGL(k_eq_gather, dim3(nblk(count, 256)), dim3(256), 0, st, AS_CSC(aL), AS_CSC(aR), eqI, nE, dfI, nD,
                       AS_SC(out));
    BPG_HIP(hipGetLastError());
}
void launch_gather_scalars(const ScD *src, uint32_t count, uint32_t stride, uint32_t offset, ScD *dst, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_gather_scalars, dim3(nblk(count, 256)), dim3(256), 0, st, AS_CSC(src), count, stride, offset,
                       AS_SC(dst));
    BPG_HIP(hipGetLastError());
}
__global__ void k_gather_niels(const gen *__restrict__ src, uint32_t count, uint32_t stride, uint32_t offset,
                               gen *__restrict__ dst) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count) return;
    gen p;
    gen_load(p, src + (size_t)j * stride + offset);
    gen_store(dst + j, p);
}
void launch_gather_niels(const NielsD *src, uint32_t count, uint32_t stride, uint32_t offset, NielsD *dst,
                         hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_gather_niels, dim3(nblk(count, 64)), dim3(64), 0, st, AS_CGEN(src), count, stride, offset,
                       AS_GEN(dst));
    BPG_HIP(hipGetLastError());
}
__global__ __launch_bounds__(64) void k_niels_neg(const gen *__restrict__ in, gen *__restrict__ out, uint32_t count) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count) return;
    gen p;
    gen_load(p, in + j);
    gen_cneg(p, true);
    gen_store(out + j, p);
}
// Fixed-base tables: one generator per lane, window w = 2^(FB_C w) P by
// FB_C doublings from window w - 1, made affine (one inversion each: a
// one-time build, ~2 ms for both 2^20 vectors)
__global__ __launch_bounds__(64) void k_fb_build(const gen *__restrict__ gens, uint32_t N, gen *__restrict__ tab) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const size_t S = 2 * (size_t)N;
    gen g, e;
    gen_load(g, gens + i);
    gen_store(tab + i, g);
    e = g; gen_cneg(e, true); gen_store(tab + N + i, e);
    ge p;
    ge_from_niels(p, g);   // (2X : 2Y : 2 : 2T)
    for (int w = 1; w < FB_W; w++) {
        for (int k = 0; k < FB_C; k++) ge_dbl_t<false>(p, p);
        ge_to_niels(e, p);
        gen_store(tab + w * S + i, e);
        gen_cneg(e, true);
        gen_store(tab + w * S + N + i, e);
    }
}
void launch_fb_build(const NielsD *gens, uint32_t N, NielsD *tab, hipStream_t st) {
    if (!N) return;
    hipLaunchKernelGGL(k_fb_build, dim3(nblk(N, 64)), dim3(64), 0, st, AS_CGEN(gens), N, AS_GEN(tab));
    BPG_HIP(hipGetLastError());
}
// Cached points -> affine Niels with ONE field inversion per wave of 64
// threads x CTN_K points (Montgomery's trick across the wave): a
// materialised IPP level kept as Niels makes the MSM jobs over it 7M madds
// at pass 1's three waves per SIMD, instead of 8M cached additions at two.
// From (Y+X, Y-X, 2Z, 2dT): with zi = 2 / (2Z), y+x = (Y+X) zi, y-x =
// (Y-X) zi, 2dxy = 2dT zi.
// Each thread multiplies its CTN_K denominators (prefix products kept in
// registers); the lanes' products are scanned across the wave -- prefix and
// suffix products by lane shuffles -- so that 1 / (lane product) =
// (1 / wave product) x (product of the lanes before) x (product of the lanes
// after); the whole wave inverts its product (the same issue slots one
// lane's inversion would take, no barrier), then every thread walks back
// through its four points. Per point about 9M + 204M / 256, every lane busy
// (round 4's kernel ran one serial 32-point chain per thread: 0.05 waves per
// SIMD, profiles/r04q_pmc_table.md; a block-wide version with one inversion
// per 1,024 points kept three waves idle at a barrier while the fourth
// inverted).
static constexpr uint32_t CTN_T = 256, CTN_K = 4, CTN_B = CTN_T * CTN_K;
DEVI void fe_load_g(fe &r, const uint32_t *w) {
#pragma unroll
    for (int k = 0; k < 10; k++) r.v[k] = w[k];
}
DEVI void fe_store_g(uint32_t *w, const fe &a) {
#pragma unroll
    for (int k = 0; k < 10; k++) w[k] = a.v[k];
}
DEVI void fe_shfl_up(fe &r, const fe &a, int d) {
#pragma unroll
    for (int k = 0; k < 10; k++) r.v[k] = (uint32_t)__shfl_up((int)a.v[k], d, 64);
}
// keep a wave-uniform field element in vector registers (else the compiler
// runs its arithmetic on the scalar unit and spills SGPRs to scratch)
DEVI void fe_in_vgprs(fe &r) {
#pragma unroll
    for (int k = 0; k < 10; k++) asm volatile("" : "+v"(r.v[k]));
}
DEVI void fe_shfl_down(fe &r, const fe &a, int d) {
#pragma unroll
    for (int k = 0; k < 10; k++) r.v[k] = (uint32_t)__shfl_down((int)a.v[k], d, 64);
}
// up to 8 vectors per launch (the G and H levels of a lockstep step's
// proofs; blockIdx.y = vector)
struct CtnArgs { const gec *in[8]; gen *out[8]; };
__global__ __launch_bounds__(CTN_T) void k_cached_to_niels(CtnArgs V, uint32_t count) {
    WAVE_PRIO(BPG_MISC_PRIO);
    const gec *__restrict__ in = V.in[blockIdx.y];
    gen *__restrict__ out = V.out[blockIdx.y];
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint64_t base = (uint64_t)blockIdx.x * CTN_B;
    constexpr int SW = sizeof(gec) / 4;
    // this thread's points: base + k CTN_T + t (coalesced across the block);
    // q_k = product of its denominators 0..k (past the end: 1). Named
    // registers, not an array: the compiler put a q[] array in scratch.
    static_assert(CTN_K == 4, "the walk below is written out for four points");
    auto den = [&](int k, fe &z) {
        const uint64_t i = base + (uint64_t)k * CTN_T + t;
        if (i < count) fe_load_g(z, reinterpret_cast<const uint32_t *>(in + i) + 20);
        else fe_one(z);
    };
    fe q0, q1, q2, z;
    den(0, q0);
    den(1, z); fe_mul(q1, q0, z);
    den(2, z); fe_mul(q2, q1, z);
    den(3, z);
    fe p;
    fe_mul(p, q2, z);

    // inclusive prefix (pre) and suffix (suf) products of p within the wave
    fe pre = p, suf = p, o;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        fe_shfl_up(o, pre, d);
        fe_mul(o, o, pre);
        if (lane >= (uint32_t)d) pre = o;
        fe_shfl_down(o, suf, d);
        fe_mul(o, o, suf);
        if (lane + d < 64) suf = o;
    }
    // products of the lanes before (ex_pre) and after (ex_suf) this one;
    // the wave's product (lane 63's prefix) is inverted by the whole wave:
    // one inversion per 256 points costs every lane the same issue slots as
    // one lane's would, and no wave waits at a barrier for another's
    fe ex_pre, ex_suf, tot;
    fe_shfl_up(ex_pre, pre, 1);
    fe_shfl_down(ex_suf, suf, 1);
    if (lane == 0) fe_one(ex_pre);
    if (lane == 63) fe_one(ex_suf);
#pragma unroll
    for (int k = 0; k < 10; k++) tot.v[k] = (uint32_t)__shfl((int)pre.v[k], 63, 64);
    fe inv;   // 1 / p
    fe_invert(inv, tot);
    fe_mul(inv, inv, ex_pre);
    fe_mul(inv, inv, ex_suf);
    // walk back through the thread's own points: 1 / (2Z_k) = inv_k q_(k-1),
    // inv_(k-1) = inv_k 2Z_k
    auto emit = [&](int k, fe zi) {   // zi = 1 / (2Z_k)
        const uint64_t i = base + (uint64_t)k * CTN_T + t;
        if (i >= count) return;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(in + i);
        fe_add(zi, zi, zi);                       // 1 / Z_k
        gen g;
        fe tt;
        fe_load_g(tt, src);      fe_mul(g.YpX, tt, zi);
        fe_load_g(tt, src + 10); fe_mul(g.YmX, tt, zi);
        fe_load_g(tt, src + 30); fe_mul(g.T2d, tt, zi);
        g.pad[0] = g.pad[1] = 0;
        gen_store(out + i, g);
    };
    fe zi;
    fe_mul(zi, inv, q2); emit(3, zi); den(3, z); fe_mul(inv, inv, z);
    fe_mul(zi, inv, q1); emit(2, zi); den(2, z); fe_mul(inv, inv, z);
    fe_mul(zi, inv, q0); emit(1, zi); den(1, z); fe_mul(inv, inv, z);
    emit(0, inv);
}
void launch_cached_to_niels(const PtD *const *in, NielsD *const *out, int nvec, uint32_t count, hipStream_t st) {
    if (!count || nvec < 1) return;
    if (nvec > 8) throw HipError(hipErrorInvalidValue, "niels vectors", __FILE__, __LINE__);
    CtnArgs V{};
    for (int v = 0; v < nvec; v++) { V.in[v] = AS_CGEC(in[v]); V.out[v] = AS_GEN(out[v]); }
    hipLaunchKernelGGL(k_cached_to_niels, dim3((count + CTN_B - 1) / CTN_B, (uint32_t)nvec), dim3(CTN_T), 0, st, V,
                       count);
    BPG_HIP(hipGetLastError());
}
__global__ __launch_bounds__(64) void k_gen_sum(const gen *__restrict__ G, const gen *__restrict__ H, gec *__restrict__ out, uint32_t count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    gen g, h;
    gen_load(g, G + i);
    gen_load(h, H + i);
    ge a;
    ge_from_niels(a, g);
    ge_madd(a, a, h);
    gec c;
    ge_to_cached(c, a);
    gec_store(out + i, c);
}
void launch_gen_sum(const NielsD *G, const NielsD *H, PtD *out, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_gen_sum, dim3(nblk(count, 64)), dim3(64), 0, st, AS_CGEN(G), AS_CGEN(H), AS_GEC(out), count);
    BPG_HIP(hipGetLastError());
}
void launch_niels_neg(const NielsD *in, NielsD *out, uint32_t count, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_niels_neg, dim3(nblk(count, 64)), dim3(64), 0, st, AS_CGEN(in), AS_GEN(out), count);
    BPG_HIP(hipGetLastError());
}
// Montgomery form -> canonical (MSM scalars from the IPP tail weights)
__global__ void k_from_mont(const sc *__restrict__ src, uint32_t count, sc *__restrict__ dst) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= count) return;
    sc a, r, one = sc_one_raw();
    sc_load(a, src + j);
    mm(r, a, one);
    sc_store(dst + j, r);
}
void launch_from_mont(const ScD *src, uint32_t count, ScD *dst, hipStream_t st) {
    if (!count) return;
    hipLaunchKernelGGL(k_from_mont, dim3(nblk(count, 256)), dim3(256), 0, st, AS_CSC(src), count, AS_SC(dst));
    BPG_HIP(hipGetLastError());
}

// Verifier::verify g/h scalars (bulletproofs r1cs/verifier.rs, IPP
// verification_scalars): s_i = allinv * prod_{bit j of i} u_{lgn-1-j}^2.
// w = flatten output [wL | wR | wO | ...]; u2m = Montgomery(u_k^2);
// xm, am, bm, um Montgomery forms of x, ipp.a, ipp.b, r1cs u.
// s_i = allinv * prod_{bit j of i} u_{lgn-1-j}^2 from two tables: tlo[k]
// (Montgomery form) over the low `lo` bits of i, thi[k] (times allinv) over
// the others, so s_i = thi[i >> lo] tlo[i mod 2^lo] is ONE product per
// element instead of a product per bit of i (lgn of them; the low bits made
// the lanes of a wave diverge, ~26 products per element at 2^20), and the
// s for h, the complement bits, is s_(N-1-i) the same way.
__global__ void k_verify_tables(const sc *__restrict__ u2m, uint32_t lgn, uint32_t lo, sc allinv,
                                sc *__restrict__ tlo, sc *__restrict__ thi) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nlo = 1u << lo, nhi = 1u << (lgn - lo);
    if (k < nlo) {
        sc t, r2, one = sc_one_raw();
        for (int q = 0; q < 8; q++) r2.v[q] = SC_R2[q];
        mm(t, one, r2);   // 1 in Montgomery form (R mod l)
        for (uint32_t j = 0; j < lo; j++)
            if ((k >> j) & 1) { sc u; sc_load(u, u2m + (lgn - 1 - j)); mm(t, t, u); }
        sc_store(tlo + k, t);
    } else if (k - nlo < nhi) {
        const uint32_t kk = k - nlo;
        sc t = allinv;
        for (uint32_t j = lo; j < lgn; j++)
            if ((kk >> (j - lo)) & 1) { sc u; sc_load(u, u2m + (lgn - 1 - j)); mm(t, t, u); }
        sc_store(thi + kk, t);
    }
}
__global__ void k_verify_gh(const sc *__restrict__ w, const sc *__restrict__ yipm, const sc *__restrict__ tlo,
                            const sc *__restrict__ thi, uint32_t lo, uint32_t n, uint32_t N, sc xm, sc am, sc bm,
                            sc um, sc *__restrict__ out, sc *__restrict__ ynwR, sc *__restrict__ acc, sc rhom,
                            int first, const int *__restrict__ ok) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint32_t mlo = (1u << lo) - 1, ic = N - 1 - i;
    sc si, sv, p, q;
    sc_load(p, thi + (i >> lo)); sc_load(q, tlo + (i & mlo)); mm(si, p, q);
    sc_load(p, thi + (ic >> lo)); sc_load(q, tlo + (ic & mlo)); mm(sv, p, q);   // bits of N-1-i: the complement of i's
    sc yi; sc_load(yi, yipm + i);
    sc wL, wR, wO;
    if (i < n) { sc_load(wL, w + i); sc_load(wR, w + n + i); sc_load(wO, w + 2 * n + i); }
    else { sc_zero(wL); sc_zero(wR); sc_zero(wO); }
    sc yn; mm(yn, wR, yi);
    if (i < n) sc_store(ynwR + i, yn);
    sc g, a;
    mm(g, yn, xm); mm(a, si, am); sc_sub(g, g, a);
    if (i >= n) mm(g, g, um);
    sc h;
    mm(h, wL, xm); sc_add(h, h, wO); mm(a, sv, bm); sc_sub(h, h, a);
    mm(h, h, yi);
    sc one = sc_one_raw();
    sc_sub(h, h, one);
    if (i >= n) mm(h, h, um);
    if (!acc) {
        sc_store(out + i, g);
        sc_store(out + N + i, h);
        return;
    }
    // batch verification: acc += rho (g, h), only for a proof whose points
    // decompressed (the previous kernel on this stream set *ok)
    if (!*ok) return;
    mm(g, g, rhom);
    mm(h, h, rhom);
    if (!first) {
        sc_load(a, acc + i); sc_add(g, g, a);
        sc_load(a, acc + N + i); sc_add(h, h, a);
    }
    sc_store(acc + i, g);
    sc_store(acc + N + i, h);
}
void launch_verify_gh(const ScD *w, const ScD *yipm, const ScD *u2m, ScD allinv, uint32_t n, uint32_t N, uint32_t lgn,
                      ScD xm, ScD am, ScD bm, ScD um, ScD *tables, ScD *out, ScD *ynwR, ScD *acc, ScD rho_mont,
                      bool first, const int *ok, hipStream_t st) {
    const uint32_t lo = lgn < 10 ? lgn : 10, nlo = 1u << lo, nhi = 1u << (lgn - lo);
    ScD *tlo = tables, *thi = tables + nlo;
    hipLaunchKernelGGL(k_verify_tables, dim3(nblk(nlo + nhi, 128)), dim3(128), 0, st, AS_CSC(u2m), lgn, lo,
                       *reinterpret_cast<sc *>(&allinv), AS_SC(tlo), AS_SC(thi));
    hipLaunchKernelGGL(k_verify_gh, dim3(nblk(N, 128)), dim3(128), 0, st, AS_CSC(w), AS_CSC(yipm), AS_CSC(tlo),
                       AS_CSC(thi), lo, n, N, *reinterpret_cast<sc *>(&xm), *reinterpret_cast<sc *>(&am),
                       *reinterpret_cast<sc *>(&bm), *reinterpret_cast<sc *>(&um), AS_SC(out), AS_SC(ynwR),
                       AS_SC(acc), *reinterpret_cast<sc *>(&rho_mont), first ? 1 : 0, ok);
    BPG_HIP(hipGetLastError());
}

}  // namespace dev
}  // namespace bpg
