/*
 * bpg_oracle.c — CPU restatement of the Bulletproofs R1CS hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity oracle and the CPU
 * baseline ("port") for bench.py. Nothing in the product (libbpg.so) links,
 * loads or calls it; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do.
 *
 * The reference (FairAds/bulletproof-gadgets) holds no arithmetic of its own
 * on this path: `prover.prove(&bp_gens)` (src/prove.rs:79) and
 * `verifier.verify(..)` (src/verify.rs:71) live in un-vendored crates, pinned
 * in /root/reference/Cargo.lock:
 *     bulletproofs 2.1.0 (FairAds fork, git 3c00b01e)   Cargo.lock:77-95
 *     curve25519-dalek 3.2.0                            Cargo.lock:155-168
 *     merlin 2.0.1 (+ keccak 0.1.0)                     Cargo.lock:402-412,314
 *     sha3 0.9.1                                        Cargo.lock:679
 * None of them is in this container; this file restates their published
 * algorithms (named per function below). It is pinned by:
 *   - libsodium 1.0.18 ristretto255 (from_hash, add, scalarmult, encodings)
 *   - hashlib sha3_512 / shake_256
 *   - the merlin 2.0.1 conformance vector
 *   - B_blinding KAT 8c9240b4...48871134
 *   - the reference's own accept/reject tests and MiMC fixtures (tests/).
 * Proof BYTES versus the real fork binary stay unpinned (no fixture holds
 * them; blindings are random in the reference, .gitignore:9-10).
 *
 * Algorithms follow dalek's choices so the CPU timing is representative:
 * 5x51-bit field limbs (u64 backend), constant-time-style Straus radix 16
 * for the commitment MSMs, Straus/Pippenger (w=6..8) vartime MSMs for the
 * IPP and the verifier, two-point Straus for the IPP generator fold.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include "../include/bpg.h"

typedef unsigned __int128 u128;

/* ========================================================================= */
/* GF(2^255-19), radix 2^51 (curve25519-dalek backend/serial/u64/field.rs)    */
/* ========================================================================= */
typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL << 51) - 1)

static const fe FE_ZERO = {{0, 0, 0, 0, 0}};
static const fe FE_ONE = {{1, 0, 0, 0, 0}};
static const fe FE_D = {{0x34dca135978a3ULL, 0x1a8283b156ebdULL, 0x5e7a26001c029ULL, 0x739c663a03cbbULL, 0x52036cee2b6ffULL}};
static const fe FE_D2 = {{0x69b9426b2f159ULL, 0x35050762add7aULL, 0x3cf44c0038052ULL, 0x6738cc7407977ULL, 0x2406d9dc56dffULL}};
static const fe FE_SQRT_M1 = {{0x61b274a0ea0b0ULL, 0x0d5a5fc8f189dULL, 0x7ef5e9cbd0c60ULL, 0x78595a6804c9eULL, 0x2b8324804fc1dULL}};
static const fe FE_SQRT_AD_MINUS_ONE = {{0x7f6a0497b2e1bULL, 0x1836f0a97afd2ULL, 0x7d747f6be7638ULL, 0x456079e7e6498ULL, 0x376931bf2b834ULL}};
static const fe FE_INVSQRT_A_MINUS_D = {{0x0fdaa805d40eaULL, 0x2eb482e57d339ULL, 0x007610274bc58ULL, 0x6510b613dc8ffULL, 0x786c8905cfaffULL}};
static const fe FE_ONE_MINUS_D_SQ = {{0x409c1945fc176ULL, 0x719abc6a1fc4fULL, 0x1c37f90b20684ULL, 0x06bccca55eedfULL, 0x029072a8b2b3eULL}};
static const fe FE_D_MINUS_ONE_SQ = {{0x55aaa44ed4d20ULL, 0x59603c3332635ULL, 0x26d3baf4a7928ULL, 0x120a66e6997a9ULL, 0x5968b37af66c2ULL}};

static inline void fe_carry(fe *r) {
    uint64_t c;
    c = r->v[0] >> 51; r->v[0] &= M51; r->v[1] += c;
    c = r->v[1] >> 51; r->v[1] &= M51; r->v[2] += c;
    c = r->v[2] >> 51; r->v[2] &= M51; r->v[3] += c;
    c = r->v[3] >> 51; r->v[3] &= M51; r->v[4] += c;
    c = r->v[4] >> 51; r->v[4] &= M51; r->v[0] += c * 19;
}
static inline void fe_add(fe *r, const fe *a, const fe *b) {
    for (int i = 0; i < 5; i++) r->v[i] = a->v[i] + b->v[i];
    fe_carry(r);
}
static inline void fe_sub(fe *r, const fe *a, const fe *b) {
    /* a + 16p - b, as dalek's FieldElement51::sub */
    r->v[0] = (a->v[0] + 36028797018963664ULL) - b->v[0];
    r->v[1] = (a->v[1] + 36028797018963952ULL) - b->v[1];
    r->v[2] = (a->v[2] + 36028797018963952ULL) - b->v[2];
    r->v[3] = (a->v[3] + 36028797018963952ULL) - b->v[3];
    r->v[4] = (a->v[4] + 36028797018963952ULL) - b->v[4];
    fe_carry(r);
}
static inline void fe_neg(fe *r, const fe *a) { fe_sub(r, &FE_ZERO, a); }
static inline void fe_mul(fe *r, const fe *a, const fe *b) {
    const uint64_t a0 = a->v[0], a1 = a->v[1], a2 = a->v[2], a3 = a->v[3], a4 = a->v[4];
    const uint64_t b0 = b->v[0], b1 = b->v[1], b2 = b->v[2], b3 = b->v[3], b4 = b->v[4];
    const uint64_t b1_19 = b1 * 19, b2_19 = b2 * 19, b3_19 = b3 * 19, b4_19 = b4 * 19;
    u128 t0 = (u128)a0 * b0 + (u128)a1 * b4_19 + (u128)a2 * b3_19 + (u128)a3 * b2_19 + (u128)a4 * b1_19;
    u128 t1 = (u128)a0 * b1 + (u128)a1 * b0 + (u128)a2 * b4_19 + (u128)a3 * b3_19 + (u128)a4 * b2_19;
    u128 t2 = (u128)a0 * b2 + (u128)a1 * b1 + (u128)a2 * b0 + (u128)a3 * b4_19 + (u128)a4 * b3_19;
    u128 t3 = (u128)a0 * b3 + (u128)a1 * b2 + (u128)a2 * b1 + (u128)a3 * b0 + (u128)a4 * b4_19;
    u128 t4 = (u128)a0 * b4 + (u128)a1 * b3 + (u128)a2 * b2 + (u128)a3 * b1 + (u128)a4 * b0;
    uint64_t r0, r1, r2, r3, r4, c;
    r0 = (uint64_t)t0 & M51; t1 += (uint64_t)(t0 >> 51);
    r1 = (uint64_t)t1 & M51; t2 += (uint64_t)(t1 >> 51);
    r2 = (uint64_t)t2 & M51; t3 += (uint64_t)(t2 >> 51);
    r3 = (uint64_t)t3 & M51; t4 += (uint64_t)(t3 >> 51);
    r4 = (uint64_t)t4 & M51; c = (uint64_t)(t4 >> 51);
    r0 += c * 19;
    r1 += r0 >> 51; r0 &= M51;
    r->v[0] = r0; r->v[1] = r1; r->v[2] = r2; r->v[3] = r3; r->v[4] = r4;
}
static inline void fe_sq(fe *r, const fe *a) { fe_mul(r, a, a); }
static void fe_sqn(fe *r, const fe *a, int n) {
    fe_sq(r, a);
    for (int i = 1; i < n; i++) fe_sq(r, r);
}
static void fe_tobytes(uint8_t s[32], const fe *a) {
    fe t = *a;
    fe_carry(&t);
    fe_carry(&t);
    uint64_t q = (t.v[0] + 19) >> 51;
    q = (t.v[1] + q) >> 51;
    q = (t.v[2] + q) >> 51;
    q = (t.v[3] + q) >> 51;
    q = (t.v[4] + q) >> 51;
    t.v[0] += 19 * q;
    t.v[1] += t.v[0] >> 51; t.v[0] &= M51;
    t.v[2] += t.v[1] >> 51; t.v[1] &= M51;
    t.v[3] += t.v[2] >> 51; t.v[2] &= M51;
    t.v[4] += t.v[3] >> 51; t.v[3] &= M51;
    t.v[4] &= M51;
    uint64_t w[4];
    w[0] = t.v[0] | (t.v[1] << 51);
    w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
    w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
    w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
static inline uint64_t load64(const uint8_t *p) {
    uint64_t r = 0;
    for (int i = 0; i < 8; i++) r |= (uint64_t)p[i] << (8 * i);
    return r;
}
/* FieldElement51::from_bytes: ignores bit 255, may be non-canonical. */
static void fe_frombytes(fe *r, const uint8_t s[32]) {
    r->v[0] = load64(s) & M51;
    r->v[1] = (load64(s + 6) >> 3) & M51;
    r->v[2] = (load64(s + 12) >> 6) & M51;
    r->v[3] = (load64(s + 19) >> 1) & M51;
    r->v[4] = (load64(s + 24) >> 12) & M51;
}
static int fe_isneg(const fe *a) { uint8_t s[32]; fe_tobytes(s, a); return s[0] & 1; }
static int fe_iszero(const fe *a) {
    uint8_t s[32]; fe_tobytes(s, a);
    uint8_t acc = 0;
    for (int i = 0; i < 32; i++) acc |= s[i];
    return acc == 0;
}
static int fe_eq(const fe *a, const fe *b) {
    uint8_t x[32], y[32]; fe_tobytes(x, a); fe_tobytes(y, b);
    return memcmp(x, y, 32) == 0;
}
static void fe_cneg(fe *a, int c) { if (c) fe_neg(a, a); }
/* z^(2^250-1) and z^11 (the shared prefix of invert and pow_p58). */
static void fe_pow22501(fe *t19, fe *t3, const fe *z) {
    fe t0, t1, t2, t4;
    fe_sq(&t0, z);
    fe_sqn(&t1, &t0, 2);
    fe_mul(&t1, z, &t1);            /* z^9 */
    fe_mul(&t0, &t0, &t1);          /* z^11 */
    *t3 = t0;
    fe_sq(&t2, &t0);                /* z^22 */
    fe_mul(&t1, &t1, &t2);          /* z^31 = 2^5-1 */
    fe_sqn(&t2, &t1, 5);
    fe_mul(&t1, &t2, &t1);          /* 2^10-1 */
    fe_sqn(&t2, &t1, 10);
    fe_mul(&t2, &t2, &t1);          /* 2^20-1 */
    fe_sqn(&t4, &t2, 20);
    fe_mul(&t2, &t4, &t2);          /* 2^40-1 */
    fe_sqn(&t2, &t2, 10);
    fe_mul(&t1, &t2, &t1);          /* 2^50-1 */
    fe_sqn(&t2, &t1, 50);
    fe_mul(&t2, &t2, &t1);          /* 2^100-1 */
    fe_sqn(&t4, &t2, 100);
    fe_mul(&t2, &t4, &t2);          /* 2^200-1 */
    fe_sqn(&t2, &t2, 50);
    fe_mul(t19, &t2, &t1);          /* 2^250-1 */
}
static void fe_invert(fe *r, const fe *z) {
    fe t19, t3;
    fe_pow22501(&t19, &t3, z);
    fe_sqn(&t19, &t19, 5);
    fe_mul(r, &t19, &t3);
}
static void fe_pow_p58(fe *r, const fe *z) {
    fe t19, t3;
    fe_pow22501(&t19, &t3, z);
    fe_sqn(&t19, &t19, 2);
    fe_mul(r, &t19, z);
}
/* FieldElement::sqrt_ratio_i (curve25519-dalek field.rs). */
static int fe_sqrt_ratio_i(fe *r, const fe *u, const fe *v) {
    fe v3, v7, t, check, neg_u, neg_u_i, r_prime;
    fe_sq(&v3, v); fe_mul(&v3, &v3, v);
    fe_sq(&v7, &v3); fe_mul(&v7, &v7, v);
    fe_mul(&t, u, &v7);
    fe_pow_p58(&t, &t);
    fe_mul(r, u, &v3);
    fe_mul(r, r, &t);
    fe_sq(&check, r); fe_mul(&check, &check, v);
    fe_neg(&neg_u, u);
    fe_mul(&neg_u_i, &neg_u, &FE_SQRT_M1);
    int correct = fe_eq(&check, u);
    int flipped = fe_eq(&check, &neg_u);
    int flipped_i = fe_eq(&check, &neg_u_i);
    fe_mul(&r_prime, r, &FE_SQRT_M1);
    if (flipped || flipped_i) *r = r_prime;
    fe_cneg(r, fe_isneg(r));
    return correct || flipped;
}

/* ========================================================================= */
/* Scalars mod l (curve25519-dalek scalar.rs semantics: every arithmetic op  */
/* returns the canonical residue; from_bits values only appear as inputs)    */
/* 4 x 64-bit Montgomery (R = 2^256).                                          */
/* ========================================================================= */
typedef struct { uint64_t v[4]; } sc;
static const uint64_t SC_L[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
static uint64_t SC_NP;          /* -l^-1 mod 2^64 */
static sc SC_R2;                /* 2^512 mod l     */
static sc SC_RR;                /* 2^256 mod l     */
static int g_sc_init = 0;

static int sc_geq_l(const uint64_t t[4]) {
    for (int i = 3; i >= 0; i--) {
        if (t[i] > SC_L[i]) return 1;
        if (t[i] < SC_L[i]) return 0;
    }
    return 1;
}
static void sc_sub_l(uint64_t t[4]) {
    u128 b = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)t[i] - SC_L[i] - b;
        t[i] = (uint64_t)d;
        b = (d >> 64) & 1;
    }
}
static void sc_add(sc *r, const sc *a, const sc *b) {
    uint64_t t[4]; u128 c = 0;
    for (int i = 0; i < 4; i++) { c += (u128)a->v[i] + b->v[i]; t[i] = (uint64_t)c; c >>= 64; }
    if (sc_geq_l(t)) sc_sub_l(t);
    memcpy(r->v, t, 32);
}
static void sc_sub(sc *r, const sc *a, const sc *b) {
    uint64_t t[4]; u128 bw = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a->v[i] - b->v[i] - bw;
        t[i] = (uint64_t)d; bw = (d >> 64) & 1;
    }
    if (bw) { u128 c = 0; for (int i = 0; i < 4; i++) { c += (u128)t[i] + SC_L[i]; t[i] = (uint64_t)c; c >>= 64; } }
    memcpy(r->v, t, 32);
}
static void sc_neg(sc *r, const sc *a) { sc z = {{0, 0, 0, 0}}; sc_sub(r, &z, a); }
/* CIOS Montgomery product; inputs < l, output < l. */
static void sc_montmul(sc *r, const sc *a, const sc *b) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) { c += (u128)t[j] + (u128)a->v[j] * b->v[i]; t[j] = (uint64_t)c; c >>= 64; }
        c += t[4]; t[4] = (uint64_t)c; t[5] = (uint64_t)(c >> 64);
        uint64_t mm = t[0] * SC_NP;
        c = (u128)t[0] + (u128)mm * SC_L[0]; c >>= 64;
        for (int j = 1; j < 4; j++) { c += (u128)t[j] + (u128)mm * SC_L[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
        c += t[4]; t[3] = (uint64_t)c; c >>= 64;
        t[4] = t[5] + (uint64_t)c;
    }
    if (t[4] || sc_geq_l(t)) sc_sub_l(t);
    memcpy(r->v, t, 32);
}
static void sc_init(void) {
    if (g_sc_init) return;
    uint64_t inv = 1;
    for (int i = 0; i < 7; i++) inv *= 2 - SC_L[0] * inv;
    SC_NP = (uint64_t)0 - inv;
    sc x = {{1, 0, 0, 0}};
    for (int i = 0; i < 512; i++) {
        sc_add(&x, &x, &x);
        if (i == 255) SC_RR = x;
    }
    SC_R2 = x;
    g_sc_init = 1;
}
/* Reduce any 256-bit integer mod l. */
static void sc_reduce256(sc *r, const uint8_t s[32]) {
    uint64_t t[4];
    for (int i = 0; i < 4; i++) t[i] = load64(s + 8 * i);
    while (sc_geq_l(t)) {
        /* subtract q*l with q = t >> 252 (at most 16), then fix up */
        uint64_t q = t[3] >> 60;
        if (q <= 1) { sc_sub_l(t); continue; }
        q -= 1;
        u128 bw = 0;
        uint64_t ql[4]; u128 c = 0;
        for (int i = 0; i < 4; i++) { c += (u128)SC_L[i] * q; ql[i] = (uint64_t)c; c >>= 64; }
        for (int i = 0; i < 4; i++) { u128 d = (u128)t[i] - ql[i] - bw; t[i] = (uint64_t)d; bw = (d >> 64) & 1; }
    }
    memcpy(r->v, t, 32);
}
static void sc_frombytes_wide(sc *r, const uint8_t s[64]) {
    sc lo, hi;
    sc_reduce256(&lo, s);
    sc_reduce256(&hi, s + 32);
    sc_montmul(&hi, &hi, &SC_R2);   /* hi * 2^256 */
    sc_add(r, &lo, &hi);
}
static void sc_tobytes(uint8_t s[32], const sc *a) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(a->v[i] >> (8 * j));
}
static void sc_mul(sc *r, const sc *a, const sc *b) {
    sc t; sc_montmul(&t, a, b); sc_montmul(r, &t, &SC_R2);
}
static const sc SC_ZERO = {{0, 0, 0, 0}};
static const sc SC_ONE = {{1, 0, 0, 0}};
static int sc_iszero(const sc *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
/* Scalar::invert (a^(l-2)); invert(0) = 0. */
static void sc_invert(sc *r, const sc *a) {
    static const uint64_t E[4] = {0x5812631a5cf5d3ebULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
    sc am, acc;
    sc_montmul(&am, a, &SC_R2);     /* to Montgomery */
    acc = SC_RR;                    /* 1 in Montgomery */
    for (int i = 255; i >= 0; i--) {
        sc_montmul(&acc, &acc, &acc);
        if ((E[i / 64] >> (i % 64)) & 1) sc_montmul(&acc, &acc, &am);
    }
    sc one = {{1, 0, 0, 0}};
    sc_montmul(r, &acc, &one);       /* from Montgomery */
}
static void sc_load(sc *r, const uint8_t s[32]) { sc_reduce256(r, s); }

/* ========================================================================= */
/* Edwards points, extended coordinates (X:Y:Z:T)                            */
/* ========================================================================= */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_identity(ge *p) { p->X = FE_ZERO; p->Y = FE_ONE; p->Z = FE_ONE; p->T = FE_ZERO; }
/* add-2008-hwcd-3 (a = -1, k = 2d) */
static void ge_add(ge *r, const ge *p, const ge *q) {
    fe a, b, c, d, e, f, g, h, t;
    fe_sub(&a, &p->Y, &p->X); fe_sub(&t, &q->Y, &q->X); fe_mul(&a, &a, &t);
    fe_add(&b, &p->Y, &p->X); fe_add(&t, &q->Y, &q->X); fe_mul(&b, &b, &t);
    fe_mul(&c, &p->T, &q->T); fe_mul(&c, &c, &FE_D2);
    fe_mul(&d, &p->Z, &q->Z); fe_add(&d, &d, &d);
    fe_sub(&e, &b, &a); fe_sub(&f, &d, &c); fe_add(&g, &d, &c); fe_add(&h, &b, &a);
    fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}
static void ge_neg(ge *r, const ge *p) { fe_neg(&r->X, &p->X); r->Y = p->Y; r->Z = p->Z; fe_neg(&r->T, &p->T); }
static void ge_sub(ge *r, const ge *p, const ge *q) { ge nq; ge_neg(&nq, q); ge_add(r, p, &nq); }
/* dalek ProjectivePoint::double -> CompletedPoint -> extended */
static void ge_dbl(ge *r, const ge *p) {
    fe xx, yy, zz2, xpy2, ypx, ymx, ex, tc;
    fe_sq(&xx, &p->X); fe_sq(&yy, &p->Y); fe_sq(&zz2, &p->Z); fe_add(&zz2, &zz2, &zz2);
    fe_add(&xpy2, &p->X, &p->Y); fe_sq(&xpy2, &xpy2);
    fe_add(&ypx, &yy, &xx); fe_sub(&ymx, &yy, &xx);
    fe_sub(&ex, &xpy2, &ypx); fe_sub(&tc, &zz2, &ymx);
    fe_mul(&r->X, &ex, &tc); fe_mul(&r->Y, &ypx, &ymx); fe_mul(&r->Z, &ymx, &tc); fe_mul(&r->T, &ex, &ypx);
}
/* Ristretto equality / identity (ristretto.rs ct_eq). */
static int ge_is_identity(const ge *p) { return fe_iszero(&p->X) || fe_iszero(&p->Y); }

/* RistrettoPoint::compress */
static void ristretto_encode(uint8_t s[32], const ge *p) {
    fe u1, u2, t, invsqrt, i1, i2, z_inv, den_inv, iX, iY, ench, X, Y, tmp, sv;
    fe_add(&u1, &p->Z, &p->Y); fe_sub(&t, &p->Z, &p->Y); fe_mul(&u1, &u1, &t);
    fe_mul(&u2, &p->X, &p->Y);
    fe_sq(&t, &u2); fe_mul(&t, &t, &u1);
    fe_sqrt_ratio_i(&invsqrt, &FE_ONE, &t);
    fe_mul(&i1, &invsqrt, &u1); fe_mul(&i2, &invsqrt, &u2);
    fe_mul(&z_inv, &i2, &p->T); fe_mul(&z_inv, &z_inv, &i1);
    den_inv = i2;
    fe_mul(&iX, &p->X, &FE_SQRT_M1); fe_mul(&iY, &p->Y, &FE_SQRT_M1);
    fe_mul(&ench, &i1, &FE_INVSQRT_A_MINUS_D);
    fe_mul(&tmp, &p->T, &z_inv);
    int rotate = fe_isneg(&tmp);
    X = rotate ? iY : p->X;
    Y = rotate ? iX : p->Y;
    if (rotate) den_inv = ench;
    fe_mul(&tmp, &X, &z_inv);
    fe_cneg(&Y, fe_isneg(&tmp));
    fe_sub(&sv, &p->Z, &Y); fe_mul(&sv, &den_inv, &sv);
    fe_cneg(&sv, fe_isneg(&sv));
    fe_tobytes(s, &sv);
}
/* CompressedRistretto::decompress; returns 0 on failure. */
static int ristretto_decode(ge *p, const uint8_t s_in[32]) {
    fe s, ss, u1, u2, u2sq, v, t, I, Dx, Dy, x, y;
    uint8_t chk[32];
    fe_frombytes(&s, s_in);
    fe_tobytes(chk, &s);
    if (memcmp(chk, s_in, 32) != 0 || fe_isneg(&s)) return 0;
    fe_sq(&ss, &s);
    fe_sub(&u1, &FE_ONE, &ss);
    fe_add(&u2, &FE_ONE, &ss);
    fe_sq(&u2sq, &u2);
    fe_sq(&t, &u1); fe_mul(&t, &t, &FE_D); fe_neg(&t, &t); fe_sub(&v, &t, &u2sq);
    fe_mul(&t, &v, &u2sq);
    int ok = fe_sqrt_ratio_i(&I, &FE_ONE, &t);
    fe_mul(&Dx, &I, &u2);
    fe_mul(&Dy, &Dx, &v); fe_mul(&Dy, &I, &Dy);
    fe_add(&x, &s, &s); fe_mul(&x, &x, &Dx); fe_cneg(&x, fe_isneg(&x));
    fe_mul(&y, &u1, &Dy);
    fe_mul(&t, &x, &y);
    if (!ok || fe_isneg(&t) || fe_iszero(&y)) return 0;
    p->X = x; p->Y = y; p->Z = FE_ONE; p->T = t;
    return 1;
}
/* RistrettoPoint::elligator_ristretto_flavor */
static void ristretto_elligator(ge *p, const fe *r0) {
    fe r, Ns, Dd, s, sp, c, Nt, ssq, t, w0, w1, w2, w3;
    fe_sq(&r, r0); fe_mul(&r, &r, &FE_SQRT_M1);
    fe_add(&Ns, &r, &FE_ONE); fe_mul(&Ns, &Ns, &FE_ONE_MINUS_D_SQ);
    fe minus_one; fe_neg(&minus_one, &FE_ONE);
    c = minus_one;
    fe_mul(&t, &FE_D, &r); fe_sub(&Dd, &c, &t);
    fe_add(&t, &r, &FE_D); fe_mul(&Dd, &Dd, &t);
    int sq = fe_sqrt_ratio_i(&s, &Ns, &Dd);
    fe_mul(&sp, &s, r0);
    fe_cneg(&sp, !fe_isneg(&sp));
    if (!sq) { s = sp; c = r; }
    fe_sub(&t, &r, &FE_ONE); fe_mul(&Nt, &c, &t); fe_mul(&Nt, &Nt, &FE_D_MINUS_ONE_SQ); fe_sub(&Nt, &Nt, &Dd);
    fe_sq(&ssq, &s);
    fe_add(&w0, &s, &s); fe_mul(&w0, &w0, &Dd);
    fe_mul(&w1, &Nt, &FE_SQRT_AD_MINUS_ONE);
    fe_sub(&w2, &FE_ONE, &ssq);
    fe_add(&w3, &FE_ONE, &ssq);
    fe_mul(&p->X, &w0, &w3); fe_mul(&p->Y, &w2, &w1); fe_mul(&p->Z, &w1, &w3); fe_mul(&p->T, &w0, &w2);
}
/* RistrettoPoint::from_uniform_bytes */
static void ristretto_from_uniform(ge *p, const uint8_t b[64]) {
    fe r1, r2; ge p1, p2;
    fe_frombytes(&r1, b); fe_frombytes(&r2, b + 32);
    ristretto_elligator(&p1, &r1);
    ristretto_elligator(&p2, &r2);
    ge_add(p, &p1, &p2);
}

/* ========================================================================= */
/* Keccak-f[1600], SHA3-512, SHAKE256 (keccak@0.1.0, sha3@0.9.1)              */
/* ========================================================================= */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static inline uint64_t rol64(uint64_t x, int s) { return s ? (x << s) | (x >> (64 - s)) : x; }
void oracle_keccakf(uint64_t st[25]) {
    for (int round = 0; round < 24; round++) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; x++) C[x] = st[x] ^ st[x + 5] ^ st[x + 10] ^ st[x + 15] ^ st[x + 20];
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rol64(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) st[i] ^= D[i % 5];
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(st[x + 5 * y], KROT[x + 5 * y]);
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) st[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        st[0] ^= KRC[round];
    }
}
static inline void keccak_bytes_perm(uint8_t st[200]) {
    uint64_t w[25];
    for (int i = 0; i < 25; i++) w[i] = load64(st + 8 * i);
    oracle_keccakf(w);
    for (int i = 0; i < 25; i++)
        for (int j = 0; j < 8; j++) st[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
typedef struct { uint8_t st[200]; unsigned rate, pos; } sponge;
static void sponge_init(sponge *s, unsigned rate) { memset(s->st, 0, 200); s->rate = rate; s->pos = 0; }
static void sponge_absorb(sponge *s, const uint8_t *in, size_t len) {
    for (size_t i = 0; i < len; i++) {
        s->st[s->pos++] ^= in[i];
        if (s->pos == s->rate) { keccak_bytes_perm(s->st); s->pos = 0; }
    }
}
static void sponge_finish(sponge *s, uint8_t dsbyte) {
    s->st[s->pos] ^= dsbyte;
    s->st[s->rate - 1] ^= 0x80;
    keccak_bytes_perm(s->st);
    s->pos = 0;
}
static void sponge_squeeze(sponge *s, uint8_t *out, size_t len) {
    for (size_t i = 0; i < len; i++) {
        if (s->pos == s->rate) { keccak_bytes_perm(s->st); s->pos = 0; }
        out[i] = s->st[s->pos++];
    }
}
void oracle_sha3_512(uint8_t out[64], const uint8_t *in, size_t len) {
    sponge s; sponge_init(&s, 72); sponge_absorb(&s, in, len); sponge_finish(&s, 0x06); sponge_squeeze(&s, out, 64);
}

/* ========================================================================= */
/* STROBE-128 / Merlin transcript (merlin@2.0.1 strobe.rs, transcript.rs)     */
/* ========================================================================= */
#define STROBE_R 166
#define FLAG_I 1
#define FLAG_A 2
#define FLAG_C 4
#define FLAG_M 16
typedef struct { uint8_t st[200]; uint8_t pos, pos_begin, cur_flags; } strobe;

static void strobe_runf(strobe *s) {
    s->st[s->pos] ^= s->pos_begin;
    s->st[s->pos + 1] ^= 0x04;
    s->st[STROBE_R + 1] ^= 0x80;
    keccak_bytes_perm(s->st);
    s->pos = 0; s->pos_begin = 0;
}
static void strobe_absorb(strobe *s, const uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) { s->st[s->pos++] ^= d[i]; if (s->pos == STROBE_R) strobe_runf(s); }
}
static void strobe_overwrite(strobe *s, const uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) { s->st[s->pos++] = d[i]; if (s->pos == STROBE_R) strobe_runf(s); }
}
static void strobe_squeeze(strobe *s, uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) { d[i] = s->st[s->pos]; s->st[s->pos] = 0; s->pos++; if (s->pos == STROBE_R) strobe_runf(s); }
}
static void strobe_begin(strobe *s, uint8_t flags, int more) {
    if (more) return;
    uint8_t old = s->pos_begin;
    s->pos_begin = s->pos + 1;
    s->cur_flags = flags;
    uint8_t b[2] = {old, flags};
    strobe_absorb(s, b, 2);
    if ((flags & (FLAG_C | 32)) && s->pos != 0) strobe_runf(s);
}
static void strobe_meta_ad(strobe *s, const uint8_t *d, size_t n, int more) { strobe_begin(s, FLAG_M | FLAG_A, more); strobe_absorb(s, d, n); }
static void strobe_ad(strobe *s, const uint8_t *d, size_t n, int more) { strobe_begin(s, FLAG_A, more); strobe_absorb(s, d, n); }
static void strobe_prf(strobe *s, uint8_t *d, size_t n, int more) { strobe_begin(s, FLAG_I | FLAG_A | FLAG_C, more); strobe_squeeze(s, d, n); }
static void strobe_key(strobe *s, const uint8_t *d, size_t n, int more) { strobe_begin(s, FLAG_A | FLAG_C, more); strobe_overwrite(s, d, n); }
static void strobe_init(strobe *s, const uint8_t *label, size_t n) {
    memset(s->st, 0, 200);
    const uint8_t hdr[6] = {1, STROBE_R + 2, 1, 0, 1, 96};
    memcpy(s->st, hdr, 6);
    memcpy(s->st + 6, "STROBEv1.0.2", 12);
    keccak_bytes_perm(s->st);
    s->pos = 0; s->pos_begin = 0; s->cur_flags = 0;
    strobe_meta_ad(s, label, n, 0);
}
typedef struct { strobe s; } transcript;
static void u32le(uint8_t b[4], uint32_t x) { for (int i = 0; i < 4; i++) b[i] = (uint8_t)(x >> (8 * i)); }
static void tr_append(transcript *t, const char *label, const uint8_t *msg, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    strobe_meta_ad(&t->s, (const uint8_t *)label, strlen(label), 0);
    strobe_meta_ad(&t->s, len, 4, 1);
    strobe_ad(&t->s, msg, n, 0);
}
static void tr_new(transcript *t, const uint8_t *label, size_t n) {
    strobe_init(&t->s, (const uint8_t *)"Merlin v1.0", 11);
    tr_append(t, "dom-sep", label, n);
}
static void tr_append_u64(transcript *t, const char *label, uint64_t x) {
    uint8_t b[8]; for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
    tr_append(t, label, b, 8);
}
static void tr_challenge(transcript *t, const char *label, uint8_t *out, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    strobe_meta_ad(&t->s, (const uint8_t *)label, strlen(label), 0);
    strobe_meta_ad(&t->s, len, 4, 1);
    strobe_prf(&t->s, out, n, 0);
}
static void tr_challenge_scalar(transcript *t, const char *label, sc *out) {
    uint8_t b[64]; tr_challenge(t, label, b, 64); sc_frombytes_wide(out, b);
}
/* TranscriptRngBuilder / TranscriptRng */
static void rng_rekey(strobe *s, const char *label, const uint8_t *w, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    strobe_meta_ad(s, (const uint8_t *)label, strlen(label), 0);
    strobe_meta_ad(s, len, 4, 1);
    strobe_key(s, w, n, 0);
}
static void rng_finalize(strobe *s, const uint8_t entropy[32]) {
    strobe_meta_ad(s, (const uint8_t *)"rng", 3, 0);
    strobe_key(s, entropy, 32, 0);
}
static void rng_fill(strobe *s, uint8_t *d, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    strobe_meta_ad(s, len, 4, 0);
    strobe_prf(s, d, n, 0);
}
static void rng_scalar(strobe *s, sc *out) { uint8_t b[64]; rng_fill(s, b, 64); sc_frombytes_wide(out, b); }

/* ========================================================================= */
/* ChaCha20 stream for deterministic mode (stand-in for thread_rng())         */
/* key = u64le(seed) || 0^24, nonce = 0^12, block counter from 0              */
/* ========================================================================= */
#define QR(a, b, c, d) \
    a += b; d ^= a; d = (d << 16) | (d >> 16); c += d; b ^= c; b = (b << 12) | (b >> 20); \
    a += b; d ^= a; d = (d << 8) | (d >> 24);  c += d; b ^= c; b = (b << 7) | (b >> 25);
void oracle_chacha20_block(uint8_t out[64], const uint8_t key[32], uint32_t counter) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) s[4 + i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
    s[12] = counter; s[13] = 0; s[14] = 0; s[15] = 0;
    memcpy(x, s, 64);
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; i++) { uint32_t v = x[i] + s[i]; u32le(out + 4 * i, v); }
}
/* Bytes [offset, offset+len) of the deterministic stream for `seed`. */
void oracle_seed_stream(uint64_t seed, uint64_t offset, uint8_t *out, size_t len) {
    uint8_t key[32] = {0}, blk[64];
    for (int i = 0; i < 8; i++) key[i] = (uint8_t)(seed >> (8 * i));
    while (len) {
        uint32_t b = (uint32_t)(offset / 64); unsigned o = (unsigned)(offset % 64);
        oracle_chacha20_block(blk, key, b);
        size_t take = 64 - o; if (take > len) take = len;
        memcpy(out, blk + o, take); out += take; len -= take; offset += take;
    }
}

/* ========================================================================= */
/* Generators (bulletproofs@2.1.0 generators.rs)                             */
/* ========================================================================= */
static const uint8_t RISTRETTO_BASEPOINT_COMPRESSED[32] = {
    0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
    0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
static ge g_B, g_Bb;            /* PedersenGens::default(): B, B_blinding */
static int g_pc_init = 0;
static void pc_init(void) {
    if (g_pc_init) return;
    sc_init();
    ristretto_decode(&g_B, RISTRETTO_BASEPOINT_COMPRESSED);
    uint8_t h[64];
    oracle_sha3_512(h, RISTRETTO_BASEPOINT_COMPRESSED, 32);
    ristretto_from_uniform(&g_Bb, h);
    g_pc_init = 1;
}
/* GeneratorsChain(label = tag || u32le(party=0)), n points. */
static void gens_chain(ge *out, char tag, uint32_t n) {
    sponge s; sponge_init(&s, 136);
    uint8_t lbl[5] = {(uint8_t)tag, 0, 0, 0, 0};
    sponge_absorb(&s, (const uint8_t *)"GeneratorsChain", 15);
    sponge_absorb(&s, lbl, 5);
    sponge_finish(&s, 0x1f);
    for (uint32_t i = 0; i < n; i++) {
        uint8_t b[64]; sponge_squeeze(&s, b, 64);
        ristretto_from_uniform(&out[i], b);
    }
}
/* A tiny cache so repeated prove/verify calls at one size pay once
 * ("warm" timing excludes generator derivation). */
static ge *g_G = NULL, *g_H = NULL;
static uint32_t g_gcap = 0;
static int gens_ensure(uint32_t n) {
    if (n <= g_gcap) return 0;
    ge *G = (ge *)malloc(sizeof(ge) * n), *H = (ge *)malloc(sizeof(ge) * n);
    if (!G || !H) { free(G); free(H); return -1; }
    gens_chain(G, 'G', n); gens_chain(H, 'H', n);
    free(g_G); free(g_H); g_G = G; g_H = H; g_gcap = n;
    return 0;
}

/* ========================================================================= */
/* Multiscalar multiplication                                                */
/* ========================================================================= */
/* Scalar::to_radix_16 (requires bit 255 clear). */
static void to_radix16(int8_t e[64], const uint8_t s[32]) {
    for (int i = 0; i < 32; i++) { e[2 * i] = s[i] & 15; e[2 * i + 1] = (s[i] >> 4) & 15; }
    for (int i = 0; i < 63; i++) { int8_t c = (int8_t)((e[i] + 8) >> 4); e[i] -= (int8_t)(c << 4); e[i + 1] += c; }
}
/* Straus radix-16 (dalek backend/serial/scalar_mul/straus.rs, multiscalar_mul). */
static void msm_straus(ge *out, const uint8_t (*scal)[32], const ge *pts, size_t n) {
    ge *tab = (ge *)malloc(sizeof(ge) * 8 * (n ? n : 1));
    int8_t *dig = (int8_t *)malloc(64 * (n ? n : 1));
    for (size_t i = 0; i < n; i++) {
        tab[8 * i] = pts[i];
        for (int j = 1; j < 8; j++) ge_add(&tab[8 * i + j], &tab[8 * i + j - 1], &pts[i]);
        to_radix16(dig + 64 * i, scal[i]);
    }
    ge q; ge_identity(&q);
    for (int w = 63; w >= 0; w--) {
        for (int k = 0; k < 4; k++) ge_dbl(&q, &q);
        for (size_t i = 0; i < n; i++) {
            int d = dig[64 * i + w];
            if (d > 0) ge_add(&q, &q, &tab[8 * i + d - 1]);
            else if (d < 0) ge_sub(&q, &q, &tab[8 * i - d - 1]);
        }
    }
    *out = q;
    free(tab); free(dig);
}
/* Signed radix-2^w digits (Scalar::as_radix_2w): ceil(256/w) digits. */
static int to_radix2w(int16_t *e, const uint8_t s[32], int w) {
    uint64_t limbs[5] = {load64(s), load64(s + 8), load64(s + 16), load64(s + 24), 0};
    int nd = (256 + w - 1) / w;
    uint64_t radix = 1ULL << w, mask = radix - 1;
    int64_t carry = 0;
    for (int i = 0; i < nd; i++) {
        int bit = i * w, idx = bit / 64, off = bit % 64;
        uint64_t bits = limbs[idx] >> off;
        if (off + w > 64 && idx + 1 < 5) bits |= limbs[idx + 1] << (64 - off);
        int64_t coef = (int64_t)(bits & mask) + carry;
        carry = (coef + (int64_t)(radix / 2)) >> w;
        e[i] = (int16_t)(coef - (carry << w));
    }
    e[nd] = (int16_t)carry;
    return nd + 1;
}
/* Pippenger (dalek backend/serial/scalar_mul/pippenger.rs) */
static void msm_pippenger(ge *out, const uint8_t (*scal)[32], const ge *pts, size_t n) {
    int w = n < 500 ? 6 : (n < 800 ? 7 : 8);
    int nd = (256 + w - 1) / w + 1;
    int nb = 1 << (w - 1);
    int16_t *dig = (int16_t *)malloc(sizeof(int16_t) * nd * (n ? n : 1));
    for (size_t i = 0; i < n; i++) to_radix2w(dig + (size_t)nd * i, scal[i], w);
    ge *bk = (ge *)malloc(sizeof(ge) * nb);
    ge total; ge_identity(&total);
    for (int di = nd - 1; di >= 0; di--) {
        for (int k = 0; k < w && di != nd - 1; k++) ge_dbl(&total, &total);
        for (int b = 0; b < nb; b++) ge_identity(&bk[b]);
        for (size_t i = 0; i < n; i++) {
            int d = dig[(size_t)nd * i + di];
            if (d > 0) ge_add(&bk[d - 1], &bk[d - 1], &pts[i]);
            else if (d < 0) ge_sub(&bk[-d - 1], &bk[-d - 1], &pts[i]);
        }
        ge run = bk[nb - 1], sum = bk[nb - 1];
        for (int b = nb - 2; b >= 0; b--) { ge_add(&run, &run, &bk[b]); ge_add(&sum, &sum, &run); }
        ge_add(&total, &total, &sum);
    }
    *out = total;
    free(bk); free(dig);
}
static void msm_vartime(ge *out, const uint8_t (*scal)[32], const ge *pts, size_t n) {
    if (n < 190) msm_straus(out, scal, pts, n);
    else msm_pippenger(out, scal, pts, n);
}

/* ========================================================================= */
/* R1CS proof (bulletproofs@2.1.0 src/r1cs/prover.rs, verifier.rs,            */
/* inner_product_proof.rs, util.rs)                                          */
/* ========================================================================= */
static uint32_t next_pow2(uint32_t n) { uint32_t p = 1; while (p < n) p <<= 1; return p; }
static int lg2(uint32_t n) { int k = 0; while ((1u << k) < n) k++; return k; }

typedef struct { sc *wL, *wR, *wO, *wV; sc wc; } flat;
/* Prover/Verifier::flattened_constraints(z): constraint q weighs z^(q+1). */
static void flatten(flat *f, const bpg_r1cs_view *cs, const sc *z) {
    f->wL = (sc *)calloc(cs->n ? cs->n : 1, sizeof(sc));
    f->wR = (sc *)calloc(cs->n ? cs->n : 1, sizeof(sc));
    f->wO = (sc *)calloc(cs->n ? cs->n : 1, sizeof(sc));
    f->wV = (sc *)calloc(cs->m ? cs->m : 1, sizeof(sc));
    f->wc = SC_ZERO;
    sc ez = *z;
    for (uint32_t q = 0; q < cs->q; q++) {
        for (uint32_t k = cs->row_ptr[q]; k < cs->row_ptr[q + 1]; k++) {
            uint32_t var = cs->term_var[k], kind = BPG_VAR_KIND(var), idx = BPG_VAR_INDEX(var);
            sc coeff, t;
            sc_load(&coeff, cs->term_coeff + 32 * (size_t)k);
            sc_mul(&t, &ez, &coeff);
            switch (kind) {
                case BPG_VAR_L: sc_add(&f->wL[idx], &f->wL[idx], &t); break;
                case BPG_VAR_R: sc_add(&f->wR[idx], &f->wR[idx], &t); break;
                case BPG_VAR_O: sc_add(&f->wO[idx], &f->wO[idx], &t); break;
                case BPG_VAR_V: sc_sub(&f->wV[idx], &f->wV[idx], &t); break;
                default: sc_sub(&f->wc, &f->wc, &t); break;
            }
        }
        sc_mul(&ez, &ez, z);
    }
}
static void flat_free(flat *f) { free(f->wL); free(f->wR); free(f->wO); free(f->wV); }
static int check_view(const bpg_r1cs_view *cs) {
    for (uint32_t q = 0; q < cs->q; q++)
        for (uint32_t k = cs->row_ptr[q]; k < cs->row_ptr[q + 1]; k++) {
            uint32_t var = cs->term_var[k], kind = BPG_VAR_KIND(var), idx = BPG_VAR_INDEX(var);
            if (kind > 4) return -1;
            if ((kind >= 1 && kind <= 3 && idx >= cs->n) || (kind == 4 && idx >= cs->m)) return -1;
        }
    return 0;
}
static void pedersen(ge *out, const sc *v, const sc *vb) {
    uint8_t s[2][32]; ge P[2] = {g_B, g_Bb};
    sc_tobytes(s[0], v); sc_tobytes(s[1], vb);
    msm_straus(out, (const uint8_t(*)[32])s, P, 2);
}
static void compress_to(uint8_t out[32], const ge *p) { ristretto_encode(out, p); }

/* Prefix shared by prover and verifier (prove.rs:45-47 + Prover::commit). */
static void r1cs_transcript_prefix(transcript *t, const uint8_t *label, size_t label_len) {
    tr_new(t, label, label_len);
    tr_append(t, "dom-sep", (const uint8_t *)"r1cs v1", 7);
}

int oracle_pedersen_commit(const uint8_t v[32], const uint8_t vb[32], uint8_t out[32]) {
    pc_init();
    sc a, b; ge P;
    sc_load(&a, v); sc_load(&b, vb);
    pedersen(&P, &a, &b);
    compress_to(out, &P);
    return 0;
}

/* Prover::prove, one-phase (no deferred constraints). */
int oracle_r1cs_prove(const uint8_t *label, size_t label_len, const bpg_r1cs_view *cs,
                      const uint8_t entropy[32], uint8_t *proof, size_t cap, size_t *plen,
                      uint8_t *V_out) {
    pc_init();
    if (check_view(cs)) return -2;
    const uint32_t n = cs->n, m = cs->m;
    const uint32_t N = next_pow2(n), lgN = (uint32_t)lg2(N);
    const size_t need = 417 + 64 * (size_t)lgN;
    if (cap < need) return -3;
    if (gens_ensure(N)) return -4;
    transcript T; r1cs_transcript_prefix(&T, label, label_len);
    for (uint32_t i = 0; i < m; i++) {
        sc v, vb; ge P; uint8_t c[32];
        sc_load(&v, cs->v + 32 * (size_t)i); sc_load(&vb, cs->v_blinding + 32 * (size_t)i);
        pedersen(&P, &v, &vb); compress_to(c, &P);
        if (V_out) memcpy(V_out + 32 * (size_t)i, c, 32);
        tr_append(&T, "V", c, 32);
    }
    tr_append_u64(&T, "m", m);
    /* TranscriptRng: rekey with each v_blinding, finalize with entropy. */
    strobe rng = T.s;
    for (uint32_t i = 0; i < m; i++) rng_rekey(&rng, "v_blinding", cs->v_blinding + 32 * (size_t)i, 32);
    rng_finalize(&rng, entropy);
    sc i_bl, o_bl, s_bl;
    rng_scalar(&rng, &i_bl); rng_scalar(&rng, &o_bl); rng_scalar(&rng, &s_bl);
    sc *sL = (sc *)malloc(sizeof(sc) * (n ? n : 1)), *sR = (sc *)malloc(sizeof(sc) * (n ? n : 1));
    for (uint32_t i = 0; i < n; i++) rng_scalar(&rng, &sL[i]);
    for (uint32_t i = 0; i < n; i++) rng_scalar(&rng, &sR[i]);
    /* A_I1, A_O1, S1: constant-time Straus in dalek (multiscalar_mul). */
    size_t np = 2 * (size_t)n + 1;
    uint8_t (*sb)[32] = (uint8_t(*)[32])malloc(32 * np);
    ge *pb = (ge *)malloc(sizeof(ge) * np);
    ge AI, AO, S;
    uint8_t cAI[32], cAO[32], cS[32];
    sc_tobytes(sb[0], &i_bl); pb[0] = g_Bb;
    for (uint32_t i = 0; i < n; i++) {
        sc t; sc_load(&t, cs->a_L + 32 * (size_t)i); sc_tobytes(sb[1 + i], &t); pb[1 + i] = g_G[i];
        sc_load(&t, cs->a_R + 32 * (size_t)i); sc_tobytes(sb[1 + n + i], &t); pb[1 + n + i] = g_H[i];
    }
    msm_straus(&AI, (const uint8_t(*)[32])sb, pb, np);
    sc_tobytes(sb[0], &o_bl);
    for (uint32_t i = 0; i < n; i++) { sc t; sc_load(&t, cs->a_O + 32 * (size_t)i); sc_tobytes(sb[1 + i], &t); }
    msm_straus(&AO, (const uint8_t(*)[32])sb, pb, (size_t)n + 1);
    sc_tobytes(sb[0], &s_bl);
    for (uint32_t i = 0; i < n; i++) { sc_tobytes(sb[1 + i], &sL[i]); sc_tobytes(sb[1 + n + i], &sR[i]); }
    msm_straus(&S, (const uint8_t(*)[32])sb, pb, np);
    free(sb); free(pb);
    compress_to(cAI, &AI); compress_to(cAO, &AO); compress_to(cS, &S);
    tr_append(&T, "A_I1", cAI, 32);
    tr_append(&T, "A_O1", cAO, 32);
    tr_append(&T, "S1", cS, 32);
    tr_append(&T, "dom-sep", (const uint8_t *)"r1cs-1phase", 11);
    uint8_t zero32[32] = {0};
    tr_append(&T, "A_I2", zero32, 32);
    tr_append(&T, "A_O2", zero32, 32);
    tr_append(&T, "S2", zero32, 32);
    sc y, z;
    tr_challenge_scalar(&T, "y", &y);
    tr_challenge_scalar(&T, "z", &z);
    flat f; flatten(&f, cs, &z);
    /* l(x), r(x) (VecPoly3) */
    sc *l1 = (sc *)malloc(sizeof(sc) * (n ? n : 1)), *l2 = (sc *)malloc(sizeof(sc) * (n ? n : 1)), *l3 = sL;
    sc *r0 = (sc *)malloc(sizeof(sc) * (n ? n : 1)), *r1 = (sc *)malloc(sizeof(sc) * (n ? n : 1)), *r3 = (sc *)malloc(sizeof(sc) * (n ? n : 1));
    sc y_inv; sc_invert(&y_inv, &y);
    sc *eyi = (sc *)malloc(sizeof(sc) * N);
    eyi[0] = SC_ONE;
    for (uint32_t i = 1; i < N; i++) sc_mul(&eyi[i], &eyi[i - 1], &y_inv);
    sc ey = SC_ONE;
    for (uint32_t i = 0; i < n; i++) {
        sc aL, aR, aO, t;
        sc_load(&aL, cs->a_L + 32 * (size_t)i); sc_load(&aR, cs->a_R + 32 * (size_t)i); sc_load(&aO, cs->a_O + 32 * (size_t)i);
        sc_mul(&t, &eyi[i], &f.wR[i]); sc_add(&l1[i], &aL, &t);
        l2[i] = aO;
        sc_sub(&r0[i], &f.wO[i], &ey);
        sc_mul(&t, &ey, &aR); sc_add(&r1[i], &t, &f.wL[i]);
        sc_mul(&r3[i], &ey, &sR[i]);
        sc_mul(&ey, &ey, &y);
    }
    /* special_inner_product */
    sc t1 = SC_ZERO, t2 = SC_ZERO, t3 = SC_ZERO, t4 = SC_ZERO, t5 = SC_ZERO, t6 = SC_ZERO, tmp;
#define IP(acc, A, B) for (uint32_t i = 0; i < n; i++) { sc_mul(&tmp, &A[i], &B[i]); sc_add(&acc, &acc, &tmp); }
    IP(t1, l1, r0);
    IP(t2, l1, r1); IP(t2, l2, r0);
    IP(t3, l2, r1); IP(t3, l3, r0);
    IP(t4, l1, r3); IP(t4, l3, r1);
    IP(t5, l2, r3);
    IP(t6, l3, r3);
#undef IP
    sc tb1, tb3, tb4, tb5, tb6;
    rng_scalar(&rng, &tb1); rng_scalar(&rng, &tb3); rng_scalar(&rng, &tb4); rng_scalar(&rng, &tb5); rng_scalar(&rng, &tb6);
    uint8_t cT[5][32];
    { ge P; pedersen(&P, &t1, &tb1); compress_to(cT[0], &P); }
    { ge P; pedersen(&P, &t3, &tb3); compress_to(cT[1], &P); }
    { ge P; pedersen(&P, &t4, &tb4); compress_to(cT[2], &P); }
    { ge P; pedersen(&P, &t5, &tb5); compress_to(cT[3], &P); }
    { ge P; pedersen(&P, &t6, &tb6); compress_to(cT[4], &P); }
    tr_append(&T, "T_1", cT[0], 32);
    tr_append(&T, "T_3", cT[1], 32);
    tr_append(&T, "T_4", cT[2], 32);
    tr_append(&T, "T_5", cT[3], 32);
    tr_append(&T, "T_6", cT[4], 32);
    sc u, x;
    tr_challenge_scalar(&T, "u", &u);
    tr_challenge_scalar(&T, "x", &x);
    sc tb2 = SC_ZERO;
    for (uint32_t i = 0; i < m; i++) { sc vb; sc_load(&vb, cs->v_blinding + 32 * (size_t)i); sc_mul(&tmp, &f.wV[i], &vb); sc_add(&tb2, &tb2, &tmp); }
    /* Poly6::eval: x*(t1 + x*(t2 + x*(t3 + x*(t4 + x*(t5 + x*t6))))) */
    sc tx, txb;
#define EVAL6(out, a1, a2, a3, a4, a5, a6) do { sc acc; sc_mul(&acc, &x, &a6); sc_add(&acc, &acc, &a5); sc_mul(&acc, &acc, &x); \
        sc_add(&acc, &acc, &a4); sc_mul(&acc, &acc, &x); sc_add(&acc, &acc, &a3); sc_mul(&acc, &acc, &x); sc_add(&acc, &acc, &a2); \
        sc_mul(&acc, &acc, &x); sc_add(&acc, &acc, &a1); sc_mul(&out, &acc, &x); } while (0)
    EVAL6(tx, t1, t2, t3, t4, t5, t6);
    EVAL6(txb, tb1, tb2, tb3, tb4, tb5, tb6);
#undef EVAL6
    /* l_vec = l(x), r_vec = r(x), padded; r_vec[i] = -y^i for i >= n */
    sc *a = (sc *)malloc(sizeof(sc) * N), *b = (sc *)malloc(sizeof(sc) * N);
    for (uint32_t i = 0; i < n; i++) {
        /* VecPoly3::eval: l0 + x*(l1 + x*(l2 + x*l3)) with l0 = 0 */
        sc acc; sc_mul(&acc, &l3[i], &x); sc_add(&acc, &acc, &l2[i]); sc_mul(&acc, &acc, &x); sc_add(&acc, &acc, &l1[i]); sc_mul(&a[i], &acc, &x);
        /* r0 + x*(r1 + x*(r2 + x*r3)) with r2 = 0 */
        sc_mul(&acc, &r3[i], &x); sc_mul(&acc, &acc, &x); sc_add(&acc, &acc, &r1[i]); sc_mul(&acc, &acc, &x); sc_add(&b[i], &acc, &r0[i]);
    }
    for (uint32_t i = n; i < N; i++) { a[i] = SC_ZERO; sc_neg(&b[i], &ey); sc_mul(&ey, &ey, &y); }
    sc e_bl;
    { sc acc; sc_mul(&acc, &x, &s_bl); sc_add(&acc, &acc, &o_bl); sc_mul(&acc, &acc, &x); sc_add(&acc, &acc, &i_bl); sc_mul(&e_bl, &acc, &x); }
    uint8_t btx[32], btxb[32], bebl[32];
    sc_tobytes(btx, &tx); sc_tobytes(btxb, &txb); sc_tobytes(bebl, &e_bl);
    tr_append(&T, "t_x", btx, 32);
    tr_append(&T, "t_x_blinding", btxb, 32);
    tr_append(&T, "e_blinding", bebl, 32);
    sc w; tr_challenge_scalar(&T, "w", &w);
    ge Q; { uint8_t ws[32]; sc_tobytes(ws, &w); msm_straus(&Q, (const uint8_t(*)[32])ws, &g_B, 1); }
    /* G_factors: 1 for i < n, u for n <= i < N; H_factors = y^-i * G_factors */
    sc *Gf = (sc *)malloc(sizeof(sc) * N), *Hf = (sc *)malloc(sizeof(sc) * N);
    for (uint32_t i = 0; i < N; i++) { Gf[i] = i < n ? SC_ONE : u; sc_mul(&Hf[i], &eyi[i], &Gf[i]); }
    /* InnerProductProof::create */
    tr_append(&T, "dom-sep", (const uint8_t *)"ipp v1", 6);
    tr_append_u64(&T, "n", N);
    ge *G = (ge *)malloc(sizeof(ge) * N), *H = (ge *)malloc(sizeof(ge) * N);
    memcpy(G, g_G, sizeof(ge) * N); memcpy(H, g_H, sizeof(ge) * N);
    uint8_t (*LR)[32] = (uint8_t(*)[32])malloc(64 * (lgN ? lgN : 1));
    uint32_t len = N;
    size_t msz = N + 1;
    uint8_t (*ms)[32] = (uint8_t(*)[32])malloc(32 * msz);
    ge *mp = (ge *)malloc(sizeof(ge) * msz);
    for (uint32_t k = 0; len != 1; k++) {
        uint32_t h = len / 2;
        sc cL = SC_ZERO, cR = SC_ZERO;
        for (uint32_t i = 0; i < h; i++) { sc_mul(&tmp, &a[i], &b[h + i]); sc_add(&cL, &cL, &tmp); sc_mul(&tmp, &a[h + i], &b[i]); sc_add(&cR, &cR, &tmp); }
        ge Lp, Rp;
        for (uint32_t i = 0; i < h; i++) {
            sc t;
            if (k == 0) { sc_mul(&t, &a[i], &Gf[h + i]); } else t = a[i];
            sc_tobytes(ms[i], &t); mp[i] = G[h + i];
            if (k == 0) { sc_mul(&t, &b[h + i], &Hf[i]); } else t = b[h + i];
            sc_tobytes(ms[h + i], &t); mp[h + i] = H[i];
        }
        sc_tobytes(ms[2 * h], &cL); mp[2 * h] = Q;
        msm_vartime(&Lp, (const uint8_t(*)[32])ms, mp, 2 * (size_t)h + 1);
        for (uint32_t i = 0; i < h; i++) {
            sc t;
            if (k == 0) { sc_mul(&t, &a[h + i], &Gf[i]); } else t = a[h + i];
            sc_tobytes(ms[i], &t); mp[i] = G[i];
            if (k == 0) { sc_mul(&t, &b[i], &Hf[h + i]); } else t = b[i];
            sc_tobytes(ms[h + i], &t); mp[h + i] = H[h + i];
        }
        sc_tobytes(ms[2 * h], &cR); mp[2 * h] = Q;
        msm_vartime(&Rp, (const uint8_t(*)[32])ms, mp, 2 * (size_t)h + 1);
        compress_to(LR[2 * k], &Lp); compress_to(LR[2 * k + 1], &Rp);
        tr_append(&T, "L", LR[2 * k], 32);
        tr_append(&T, "R", LR[2 * k + 1], 32);
        sc uk, uinv; tr_challenge_scalar(&T, "u", &uk); sc_invert(&uinv, &uk);
        for (uint32_t i = 0; i < h; i++) {
            sc t0, t1b;
            sc_mul(&t0, &a[i], &uk); sc_mul(&t1b, &uinv, &a[h + i]); sc_add(&a[i], &t0, &t1b);
            sc_mul(&t0, &b[i], &uinv); sc_mul(&t1b, &uk, &b[h + i]); sc_add(&b[i], &t0, &t1b);
            uint8_t s2[2][32]; ge P2[2];
            if (k == 0) { sc_mul(&t0, &uinv, &Gf[i]); sc_mul(&t1b, &uk, &Gf[h + i]); } else { t0 = uinv; t1b = uk; }
            sc_tobytes(s2[0], &t0); sc_tobytes(s2[1], &t1b); P2[0] = G[i]; P2[1] = G[h + i];
            msm_straus(&G[i], (const uint8_t(*)[32])s2, P2, 2);
            if (k == 0) { sc_mul(&t0, &uk, &Hf[i]); sc_mul(&t1b, &uinv, &Hf[h + i]); } else { t0 = uk; t1b = uinv; }
            sc_tobytes(s2[0], &t0); sc_tobytes(s2[1], &t1b); P2[0] = H[i]; P2[1] = H[h + i];
            msm_straus(&H[i], (const uint8_t(*)[32])s2, P2, 2);
        }
        len = h;
    }
    /* R1CSProof::to_bytes, one-phase */
    uint8_t *o = proof;
    *o++ = 0;
    memcpy(o, cAI, 32); o += 32; memcpy(o, cAO, 32); o += 32; memcpy(o, cS, 32); o += 32;
    for (int i = 0; i < 5; i++) { memcpy(o, cT[i], 32); o += 32; }
    memcpy(o, btx, 32); o += 32; memcpy(o, btxb, 32); o += 32; memcpy(o, bebl, 32); o += 32;
    for (uint32_t k = 0; k < lgN; k++) { memcpy(o, LR[2 * k], 32); o += 32; memcpy(o, LR[2 * k + 1], 32); o += 32; }
    sc_tobytes(o, &a[0]); o += 32; sc_tobytes(o, &b[0]); o += 32;
    *plen = (size_t)(o - proof);
    free(ms); free(mp); free(G); free(H); free(LR); free(Gf); free(Hf); free(a); free(b); free(eyi);
    free(l1); free(l2); free(r0); free(r1); free(r3); free(sL); free(sR); flat_free(&f);
    return 0;
}

static int is_zero32(const uint8_t *p) { uint8_t acc = 0; for (int i = 0; i < 32; i++) acc |= p[i]; return acc == 0; }
static int sc_from_canonical(sc *r, const uint8_t s[32]) {
    if (s[31] >> 7) return 0;
    sc t; sc_reduce256(&t, s);
    uint8_t c[32]; sc_tobytes(c, &t);
    if (memcmp(c, s, 32) != 0) return 0;
    *r = t; return 1;
}

/* Verifier::verify (+ R1CSProof::from_bytes, verification_scalars).
 * 1 accept, 0 reject, <0 malformed input. */
int oracle_r1cs_verify(const uint8_t *label, size_t label_len, const bpg_r1cs_view *cs,
                       const uint8_t *V, const uint8_t *proof, size_t plen, const uint8_t entropy[32]) {
    pc_init();
    if (check_view(cs)) return -2;
    const uint32_t n = cs->n, m = cs->m;
    /* from_bytes */
    if (plen < 1 || proof[0] != 0) return 0;          /* only one-phase proofs are produced */
    const uint8_t *p = proof + 1; size_t rem = plen - 1;
    if (rem % 32 != 0 || rem < 11 * 32) return 0;
    const uint8_t *cAI = p, *cAO = p + 32, *cS = p + 64, *cT = p + 96;
    sc tx, txb, ebl;
    if (!sc_from_canonical(&tx, p + 256) || !sc_from_canonical(&txb, p + 288) || !sc_from_canonical(&ebl, p + 320)) return 0;
    const uint8_t *ipp = p + 352; size_t ib = rem - 352;
    size_t ne = ib / 32;
    if (ne < 2 || (ne - 2) % 2) return 0;
    uint32_t lgn = (uint32_t)((ne - 2) / 2);
    if (lgn >= 32) return 0;
    sc pa, pb;
    if (!sc_from_canonical(&pa, ipp + 64 * lgn) || !sc_from_canonical(&pb, ipp + 64 * lgn + 32)) return 0;
    const uint32_t N = next_pow2(n);
    if (N != (1u << lgn)) return 0;
    if (gens_ensure(N)) return -4;
    transcript T; r1cs_transcript_prefix(&T, label, label_len);
    for (uint32_t i = 0; i < m; i++) tr_append(&T, "V", V + 32 * (size_t)i, 32);
    tr_append_u64(&T, "m", m);
    if (is_zero32(cAI) || is_zero32(cAO) || is_zero32(cS)) return 0;
    tr_append(&T, "A_I1", cAI, 32);
    tr_append(&T, "A_O1", cAO, 32);
    tr_append(&T, "S1", cS, 32);
    tr_append(&T, "dom-sep", (const uint8_t *)"r1cs-1phase", 11);
    uint8_t zero32[32] = {0};
    tr_append(&T, "A_I2", zero32, 32);
    tr_append(&T, "A_O2", zero32, 32);
    tr_append(&T, "S2", zero32, 32);
    sc y, z; tr_challenge_scalar(&T, "y", &y); tr_challenge_scalar(&T, "z", &z);
    static const char *TL[5] = {"T_1", "T_3", "T_4", "T_5", "T_6"};
    for (int i = 0; i < 5; i++) { if (is_zero32(cT + 32 * i)) return 0; tr_append(&T, TL[i], cT + 32 * i, 32); }
    sc u, x; tr_challenge_scalar(&T, "u", &u); tr_challenge_scalar(&T, "x", &x);
    tr_append(&T, "t_x", p + 256, 32);
    tr_append(&T, "t_x_blinding", p + 288, 32);
    tr_append(&T, "e_blinding", p + 320, 32);
    sc w; tr_challenge_scalar(&T, "w", &w);
    flat f; flatten(&f, cs, &z);
    /* verification_scalars */
    tr_append(&T, "dom-sep", (const uint8_t *)"ipp v1", 6);
    tr_append_u64(&T, "n", N);
    sc *uch = (sc *)malloc(sizeof(sc) * (lgn ? lgn : 1)), *uinv = (sc *)malloc(sizeof(sc) * (lgn ? lgn : 1));
    int bad = 0;
    for (uint32_t k = 0; k < lgn; k++) {
        if (is_zero32(ipp + 64 * k) || is_zero32(ipp + 64 * k + 32)) { bad = 1; break; }
        tr_append(&T, "L", ipp + 64 * k, 32);
        tr_append(&T, "R", ipp + 64 * k + 32, 32);
        tr_challenge_scalar(&T, "u", &uch[k]);
    }
    if (bad) { free(uch); free(uinv); flat_free(&f); return 0; }
    sc allinv = SC_ONE;
    for (uint32_t k = 0; k < lgn; k++) { sc_invert(&uinv[k], &uch[k]); sc_mul(&allinv, &allinv, &uinv[k]); }
    for (uint32_t k = 0; k < lgn; k++) { sc_mul(&uch[k], &uch[k], &uch[k]); sc_mul(&uinv[k], &uinv[k], &uinv[k]); }
    sc *s = (sc *)malloc(sizeof(sc) * N);
    s[0] = allinv;
    for (uint32_t i = 1; i < N; i++) {
        int lgi = 31 - __builtin_clz(i);
        uint32_t kk = 1u << lgi;
        sc_mul(&s[i], &s[i - kk], &uch[lgn - 1 - lgi]);
    }
    sc y_inv; sc_invert(&y_inv, &y);
    sc *yiv = (sc *)malloc(sizeof(sc) * N);
    yiv[0] = SC_ONE; for (uint32_t i = 1; i < N; i++) sc_mul(&yiv[i], &yiv[i - 1], &y_inv);
    sc delta = SC_ZERO, tmp;
    sc *ynwR = (sc *)malloc(sizeof(sc) * N);
    for (uint32_t i = 0; i < N; i++) { if (i < n) sc_mul(&ynwR[i], &f.wR[i], &yiv[i]); else ynwR[i] = SC_ZERO; }
    for (uint32_t i = 0; i < n; i++) { sc_mul(&tmp, &ynwR[i], &f.wL[i]); sc_add(&delta, &delta, &tmp); }
    sc r; { strobe rng = T.s; rng_finalize(&rng, entropy); rng_scalar(&rng, &r); }
    sc xx, rxx, xxx;
    sc_mul(&xx, &x, &x); sc_mul(&rxx, &r, &xx); sc_mul(&xxx, &x, &xx);
    size_t tot = 6 + (size_t)m + 5 + 2 + 2 * (size_t)N + 2 * (size_t)lgn;
    uint8_t (*ms)[32] = (uint8_t(*)[32])malloc(32 * tot);
    ge *mp = (ge *)malloc(sizeof(ge) * tot);
    size_t c = 0;
    int ok = 1;
#define PUSH(sv, cptr) do { sc_tobytes(ms[c], &(sv)); if (!ristretto_decode(&mp[c], (cptr))) ok = 0; c++; } while (0)
#define PUSHP(sv, P) do { sc_tobytes(ms[c], &(sv)); mp[c] = (P); c++; } while (0)
    sc ux, uxx, uxxx; sc_mul(&ux, &u, &x); sc_mul(&uxx, &u, &xx); sc_mul(&uxxx, &u, &xxx);
    PUSH(x, cAI); PUSH(xx, cAO); PUSH(xxx, cS);
    { ge I; ge_identity(&I); PUSHP(ux, I); PUSHP(uxx, I); PUSHP(uxxx, I); }
    for (uint32_t i = 0; i < m; i++) { sc t; sc_mul(&t, &f.wV[i], &rxx); PUSH(t, V + 32 * (size_t)i); }
    sc Ts[5];
    sc_mul(&Ts[0], &r, &x); sc_mul(&Ts[1], &rxx, &x); sc_mul(&Ts[2], &rxx, &xx); sc_mul(&Ts[3], &rxx, &xxx);
    sc_mul(&Ts[4], &rxx, &xx); sc_mul(&Ts[4], &Ts[4], &xx);
    for (int i = 0; i < 5; i++) PUSH(Ts[i], cT + 32 * i);
    {   /* B: w*(t_x - a*b) + r*(xx*(wc + delta) - t_x) */
        sc ab, t1, t2;
        sc_mul(&ab, &pa, &pb); sc_sub(&t1, &tx, &ab); sc_mul(&t1, &w, &t1);
        sc_add(&t2, &f.wc, &delta); sc_mul(&t2, &xx, &t2); sc_sub(&t2, &t2, &tx); sc_mul(&t2, &r, &t2);
        sc_add(&t1, &t1, &t2); PUSHP(t1, g_B);
        /* B_blinding: -e_blinding - r*t_x_blinding */
        sc_mul(&t2, &r, &txb); sc_neg(&t1, &ebl); sc_sub(&t1, &t1, &t2); PUSHP(t1, g_Bb);
    }
    for (uint32_t i = 0; i < N; i++) {
        /* u_or_1 * (x * yneg_wR_i - a * s_i) */
        sc uo = i < n ? SC_ONE : u, t1, t2;
        sc_mul(&t1, &x, &ynwR[i]); sc_mul(&t2, &pa, &s[i]); sc_sub(&t1, &t1, &t2); sc_mul(&t1, &uo, &t1);
        PUSHP(t1, g_G[i]);
    }
    for (uint32_t i = 0; i < N; i++) {
        /* u_or_1 * (y_inv_i * (x*wL_i + wO_i - b*s_inv_i) - 1), s_inv_i = s[N-1-i] */
        sc uo = i < n ? SC_ONE : u, t1, t2;
        sc wLi = i < n ? f.wL[i] : SC_ZERO, wOi = i < n ? f.wO[i] : SC_ZERO;
        sc_mul(&t1, &x, &wLi); sc_add(&t1, &t1, &wOi); sc_mul(&t2, &pb, &s[N - 1 - i]); sc_sub(&t1, &t1, &t2);
        sc_mul(&t1, &yiv[i], &t1); sc_sub(&t1, &t1, &SC_ONE); sc_mul(&t1, &uo, &t1);
        PUSHP(t1, g_H[i]);
    }
    for (uint32_t k = 0; k < lgn; k++) PUSH(uch[k], ipp + 64 * k);
    for (uint32_t k = 0; k < lgn; k++) PUSH(uinv[k], ipp + 64 * k + 32);
#undef PUSH
#undef PUSHP
    int result = 0;
    if (ok) { ge R; msm_vartime(&R, (const uint8_t(*)[32])ms, mp, c); result = ge_is_identity(&R); }
    free(ms); free(mp); free(s); free(yiv); free(ynwR); free(uch); free(uinv); flat_free(&f);
    return result;
}

/* ========================================================================= */
/* Exports for tests (ctypes)                                                */
/* ========================================================================= */
int oracle_from_uniform(const uint8_t b[64], uint8_t out[32]) { pc_init(); ge p; ristretto_from_uniform(&p, b); compress_to(out, &p); return 0; }
int oracle_decompress_ok(const uint8_t in[32]) { ge p; return ristretto_decode(&p, in); }
int oracle_point_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    ge P, Q, R; if (!ristretto_decode(&P, a) || !ristretto_decode(&Q, b)) return -1;
    ge_add(&R, &P, &Q); compress_to(out, &R); return 0;
}
int oracle_point_mul(const uint8_t s[32], const uint8_t a[32], uint8_t out[32]) {
    pc_init(); ge P, R; sc t; uint8_t b[32];
    if (!ristretto_decode(&P, a)) return -1;
    sc_load(&t, s); sc_tobytes(b, &t);
    msm_straus(&R, (const uint8_t(*)[32])b, &P, 1); compress_to(out, &R); return 0;
}
int oracle_msm(const uint8_t *scal, const uint8_t *pts, uint32_t n, uint8_t out[32]) {
    pc_init();
    ge *P = (ge *)malloc(sizeof(ge) * (n ? n : 1));
    uint8_t (*s)[32] = (uint8_t(*)[32])malloc(32 * (size_t)(n ? n : 1));
    for (uint32_t i = 0; i < n; i++) {
        sc t; sc_load(&t, scal + 32 * (size_t)i); sc_tobytes(s[i], &t);
        if (!ristretto_decode(&P[i], pts + 32 * (size_t)i)) { free(P); free(s); return -1; }
    }
    ge R; msm_vartime(&R, (const uint8_t(*)[32])s, P, n); compress_to(out, &R);
    free(P); free(s); return 0;
}
int oracle_generators(uint32_t n, uint8_t *G_out, uint8_t *H_out) {
    pc_init(); if (gens_ensure(n)) return -1;
    for (uint32_t i = 0; i < n; i++) { compress_to(G_out + 32 * (size_t)i, &g_G[i]); compress_to(H_out + 32 * (size_t)i, &g_H[i]); }
    return 0;
}
int oracle_pedersen_gens(uint8_t B_out[32], uint8_t Bb_out[32]) { pc_init(); compress_to(B_out, &g_B); compress_to(Bb_out, &g_Bb); return 0; }
void oracle_sc_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) { sc_init(); sc x, y, r; sc_load(&x, a); sc_load(&y, b); sc_mul(&r, &x, &y); sc_tobytes(out, &r); }
void oracle_sc_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) { sc_init(); sc x, y, r; sc_load(&x, a); sc_load(&y, b); sc_add(&r, &x, &y); sc_tobytes(out, &r); }
void oracle_sc_invert(const uint8_t a[32], uint8_t out[32]) { sc_init(); sc x, r; sc_load(&x, a); sc_invert(&r, &x); sc_tobytes(out, &r); }
void oracle_sc_wide(const uint8_t a[64], uint8_t out[32]) { sc_init(); sc r; sc_frombytes_wide(&r, a); sc_tobytes(out, &r); }
/* Merlin conformance helper: Transcript(label); append(l1, m1); challenge(l2, n). */
void oracle_merlin_test(const uint8_t *proto, size_t pn, const char *l1, const uint8_t *m1, size_t mn,
                        const char *l2, uint8_t *out, size_t on) {
    transcript t; tr_new(&t, proto, pn); tr_append(&t, l1, m1, mn); tr_challenge(&t, l2, out, on);
}
void oracle_shake256(const uint8_t *in, size_t len, uint8_t *out, size_t olen) {
    sponge s; sponge_init(&s, 136); sponge_absorb(&s, in, len); sponge_finish(&s, 0x1f); sponge_squeeze(&s, out, olen);
}
