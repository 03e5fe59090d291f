// dev_field.h — GF(2^255-19), scalars mod l and Ristretto255 points on gfx950.
//
// Replaces the curve25519-dalek 3.2.0 serial/u64 + avx2 backends (field.rs,
// scalar.rs, ristretto.rs, edwards.rs) for the device side of the hot path.
// Representation is chosen for CDNA4's VALU, not translated from dalek:
//   * field elements: 8 x 32-bit limbs, radix 2^32, any value < 2^256 that is
//     congruent mod p ("weakly reduced"); products use v_mad_u64_u32 chains and
//     fold with 2^256 == 38 (mod p). Canonical form only at encode/compare.
//   * scalars: 8 x 32-bit limbs, canonical (< l); products by 32-bit CIOS
//     Montgomery (R = 2^256), no MFMA — this is 255-bit integer work.
//   * points: extended twisted-Edwards (X:Y:Z:T), a = -1, 128 bytes.
#pragma once
#include <stdint.h>
#ifdef BPG_HOST_SIM
// Host emulation build (tests/devsim): the same arithmetic compiled for the
// CPU so it can be checked against Python big integers without a GPU.
#define DEVI static inline
#define __device__
#define __constant__
struct uint4 { uint32_t x, y, z, w; };
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
#else
#include <hip/hip_runtime.h>
#define DEVI __device__ __forceinline__
#endif

struct fe { uint32_t v[8]; };
struct sc { uint32_t v[8]; };
struct ge { fe X, Y, Z, T; };

// ---------------------------------------------------------------------------
// constants (derivation: oracle/gen_consts.py; values per RFC 9496 §4.1)
// ---------------------------------------------------------------------------
#define FE_C(name, a0, a1, a2, a3, a4, a5, a6, a7) \
    static __device__ __constant__ const fe name = {{a0, a1, a2, a3, a4, a5, a6, a7}};
FE_C(FE_D, 0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu)
FE_C(FE_D2, 0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au, 0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu)
FE_C(FE_SQRT_M1, 0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u)
FE_C(FE_SQRT_AD_MINUS_ONE, 0x497b2e1bu, 0x7e97f6a0u, 0x1b7854bdu, 0xaf9d8e0cu, 0x31f5d1fdu, 0x0f3cfcc9u, 0x2b8348acu, 0x376931bfu)
FE_C(FE_INVSQRT_A_MINUS_D, 0x805d40eau, 0x99c8fdaau, 0x5a4172beu, 0x9d2f1617u, 0xfe01d840u, 0x16c27b91u, 0xcfaffca2u, 0x786c8905u)
FE_C(FE_ONE_MINUS_D_SQ, 0x945fc176u, 0xe27c09c1u, 0xcd5e350fu, 0x2c81a138u, 0xbe70dfe4u, 0x9994abddu, 0xb2b3e0d7u, 0x029072a8u)
FE_C(FE_D_MINUS_ONE_SQ, 0x44ed4d20u, 0x31ad5aaau, 0xb01e1999u, 0xd29e4a2cu, 0x529b4eebu, 0x4cdcd32fu, 0xf66c2241u, 0x5968b37au)
#undef FE_C

static __device__ __constant__ const uint32_t SC_L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
static __device__ __constant__ const uint32_t SC_R2[8] = {0x449c0f01u, 0xa40611e3u, 0x68859347u, 0xd00e1ba7u, 0x17f5be65u, 0xceec73d2u, 0x7c309a3du, 0x0399411bu};
#define SC_NP32 0x12547e1bu

// ---------------------------------------------------------------------------
// field arithmetic mod p = 2^255 - 19
// ---------------------------------------------------------------------------
DEVI void fe_zero(fe &r) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
}
DEVI void fe_one(fe &r) { fe_zero(r); r.v[0] = 1; }

DEVI void fe_add(fe &r, const fe &a, const fe &b) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (uint64_t)a.v[i] + b.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    c *= 38;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += r.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[0] += (uint32_t)c * 38;
}

DEVI void fe_sub(fe &r, const fe &a, const fe &b) {
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (int64_t)a.v[i] - (int64_t)b.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    // c in {-1, 0}: a wrap by 2^256 == +38, take it back
    c *= 38;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += r.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[0] += (uint32_t)((int32_t)c * 38);
}

DEVI void fe_neg(fe &r, const fe &a) { fe z; fe_zero(z); fe_sub(r, z, a); }

// 16-limb product -> fold with 38
DEVI void fe_reduce16(fe &r, const uint32_t t[16]) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (uint64_t)t[8 + i] * 38u + t[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    c *= 38;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += r.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[0] += (uint32_t)c * 38;
}

DEVI void fe_mul(fe &r, const fe &a, const fe &b) {
    uint32_t t[16];
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) { c += (uint64_t)a.v[0] * b.v[j]; t[j] = (uint32_t)c; c >>= 32; }
    t[8] = (uint32_t)c;
#pragma unroll
    for (int i = 1; i < 8; i++) {
        c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) { c += (uint64_t)a.v[i] * b.v[j] + t[i + j]; t[i + j] = (uint32_t)c; c >>= 32; }
        t[i + 8] = (uint32_t)c;
    }
    fe_reduce16(r, t);
}

DEVI void fe_sq(fe &r, const fe &a) {
    uint32_t t[16];
    // off-diagonal products a_i a_j (i < j)
#pragma unroll
    for (int i = 0; i < 16; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = i + 1; j < 8; j++) { c += (uint64_t)a.v[i] * a.v[j] + t[i + j]; t[i + j] = (uint32_t)c; c >>= 32; }
        t[i + 8] = (uint32_t)c;
    }
    // double
    uint32_t hi = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) { uint32_t x = t[i]; t[i] = (x << 1) | hi; hi = x >> 31; }
    // add squares
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t s = (uint64_t)a.v[i] * a.v[i];
        c += (uint64_t)t[2 * i] + (uint32_t)s; t[2 * i] = (uint32_t)c; c >>= 32;
        c += (uint64_t)t[2 * i + 1] + (uint32_t)(s >> 32); t[2 * i + 1] = (uint32_t)c; c >>= 32;
    }
    fe_reduce16(r, t);
}

DEVI void fe_sqn(fe &r, const fe &a, int n) {
    fe_sq(r, a);
    for (int i = 1; i < n; i++) fe_sq(r, r);
}

// Fully reduce to [0, p).
DEVI void fe_canon(fe &r, const fe &a) {
    r = a;
    // fold bit 255 (2^255 == 19): r < 2^255 + 19
    uint64_t c = (uint64_t)(r.v[7] >> 31) * 19;
    r.v[7] &= 0x7fffffffu;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += r.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    // r >= p  <=>  t = r + 19 has bit 255 set; then r - p = t - 2^255
    uint32_t t[8];
    c = 19;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += r.v[i]; t[i] = (uint32_t)c; c >>= 32; }
    if (t[7] >> 31) {
        t[7] &= 0x7fffffffu;
#pragma unroll
        for (int i = 0; i < 8; i++) r.v[i] = t[i];
    }
}

DEVI void fe_tobytes(uint8_t s[32], const fe &a) {
    fe c; fe_canon(c, a);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        s[4 * i] = (uint8_t)c.v[i]; s[4 * i + 1] = (uint8_t)(c.v[i] >> 8);
        s[4 * i + 2] = (uint8_t)(c.v[i] >> 16); s[4 * i + 3] = (uint8_t)(c.v[i] >> 24);
    }
}
DEVI void fe_tow(uint32_t w[8], const fe &a) { fe c; fe_canon(c, a); for (int i = 0; i < 8; i++) w[i] = c.v[i]; }
// FieldElement::from_bytes: bit 255 ignored.
DEVI void fe_fromw(fe &r, const uint32_t w[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = w[i];
    r.v[7] &= 0x7fffffffu;
}
DEVI bool fe_iszero(const fe &a) {
    fe c; fe_canon(c, a);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= c.v[i];
    return acc == 0;
}
DEVI bool fe_isneg(const fe &a) { fe c; fe_canon(c, a); return c.v[0] & 1; }
DEVI bool fe_eq(const fe &a, const fe &b) { fe d; fe_sub(d, a, b); return fe_iszero(d); }
DEVI void fe_cneg(fe &a, bool c) { if (c) fe_neg(a, a); }

DEVI void fe_pow22501(fe &t19, fe &t3, const fe &z) {
    fe t0, t1, t2, t4;
    fe_sq(t0, z);
    fe_sqn(t1, t0, 2);
    fe_mul(t1, z, t1);
    fe_mul(t0, t0, t1);
    t3 = t0;
    fe_sq(t2, t0);
    fe_mul(t1, t1, t2);
    fe_sqn(t2, t1, 5);
    fe_mul(t1, t2, t1);
    fe_sqn(t2, t1, 10);
    fe_mul(t2, t2, t1);
    fe_sqn(t4, t2, 20);
    fe_mul(t2, t4, t2);
    fe_sqn(t2, t2, 10);
    fe_mul(t1, t2, t1);
    fe_sqn(t2, t1, 50);
    fe_mul(t2, t2, t1);
    fe_sqn(t4, t2, 100);
    fe_mul(t2, t4, t2);
    fe_sqn(t2, t2, 50);
    fe_mul(t19, t2, t1);
}
DEVI void fe_invert(fe &r, const fe &z) {
    fe t19, t3;
    fe_pow22501(t19, t3, z);
    fe_sqn(t19, t19, 5);
    fe_mul(r, t19, t3);
}
DEVI void fe_pow_p58(fe &r, const fe &z) {
    fe t19, t3;
    fe_pow22501(t19, t3, z);
    fe_sqn(t19, t19, 2);
    fe_mul(r, t19, z);
}
// FieldElement::sqrt_ratio_i
DEVI bool fe_sqrt_ratio_i(fe &r, const fe &u, const fe &v) {
    fe v3, v7, t, check, nu, nui, rp;
    fe_sq(v3, v); fe_mul(v3, v3, v);
    fe_sq(v7, v3); fe_mul(v7, v7, v);
    fe_mul(t, u, v7);
    fe_pow_p58(t, t);
    fe_mul(r, u, v3);
    fe_mul(r, r, t);
    fe_sq(check, r); fe_mul(check, check, v);
    fe_neg(nu, u);
    fe_mul(nui, nu, FE_SQRT_M1);
    bool correct = fe_eq(check, u), flipped = fe_eq(check, nu), flipped_i = fe_eq(check, nui);
    fe_mul(rp, r, FE_SQRT_M1);
    if (flipped || flipped_i) r = rp;
    fe_cneg(r, fe_isneg(r));
    return correct || flipped;
}

// ---------------------------------------------------------------------------
// scalars mod l
// ---------------------------------------------------------------------------
DEVI void sc_zero(sc &r) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
}
DEVI bool sc_geq_l(const uint32_t t[8]) {
    // lexicographic compare from the top limb
    bool gt = false, lt = false;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
        bool g = t[i] > SC_L[i], l = t[i] < SC_L[i];
        gt = gt || (!lt && g);
        lt = lt || (!gt && l);
    }
    return !lt;
}
DEVI void sc_sub_l(uint32_t t[8]) {
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (int64_t)t[i] - (int64_t)SC_L[i]; t[i] = (uint32_t)c; c >>= 32; }
}
DEVI void sc_add(sc &r, const sc &a, const sc &b) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (uint64_t)a.v[i] + b.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    if (sc_geq_l(r.v)) sc_sub_l(r.v);
}
DEVI void sc_sub(sc &r, const sc &a, const sc &b) {
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (int64_t)a.v[i] - (int64_t)b.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    if (c) {
        uint64_t d = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) { d += (uint64_t)r.v[i] + SC_L[i]; r.v[i] = (uint32_t)d; d >>= 32; }
    }
}
DEVI void sc_neg(sc &r, const sc &a) { sc z; sc_zero(z); sc_sub(r, z, a); }
// Montgomery product a*b/2^256 mod l; a < 2^256, b < l -> result < l.
DEVI void sc_montmul(sc &r, const sc &a, const sc &b) {
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) { c += (uint64_t)a.v[j] * b.v[i] + t[j]; t[j] = (uint32_t)c; c >>= 32; }
        c += t[8]; t[8] = (uint32_t)c; t[9] = (uint32_t)(c >> 32);
        uint32_t m = t[0] * SC_NP32;
        c = (uint64_t)m * SC_L[0] + t[0]; c >>= 32;
#pragma unroll
        for (int j = 1; j < 8; j++) { c += (uint64_t)m * SC_L[j] + t[j]; t[j - 1] = (uint32_t)c; c >>= 32; }
        c += t[8]; t[7] = (uint32_t)c; c >>= 32;
        t[8] = t[9] + (uint32_t)c;
    }
    if (t[8] || sc_geq_l(t)) sc_sub_l(t);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = t[i];
}
DEVI void sc_mul(sc &r, const sc &a, const sc &b) {
    sc t, r2;
#pragma unroll
    for (int i = 0; i < 8; i++) r2.v[i] = SC_R2[i];
    sc_montmul(t, a, b);
    sc_montmul(r, t, r2);
}
// Reduce a raw 256-bit value mod l.
DEVI void sc_reduce(sc &r, const sc &a) {
    r = a;
    for (int k = 0; k < 20 && sc_geq_l(r.v); k++) {
        uint32_t q = r.v[7] >> 28;   // value >> 252
        if (q <= 1) { sc_sub_l(r.v); continue; }
        q -= 1;
        uint64_t c = 0; int64_t bw = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            c += (uint64_t)SC_L[i] * q;
            bw += (int64_t)r.v[i] - (int64_t)(uint32_t)c;
            c >>= 32;
            r.v[i] = (uint32_t)bw; bw >>= 32;
        }
    }
}
DEVI bool sc_iszero(const sc &a) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= a.v[i];
    return acc == 0;
}

// ---------------------------------------------------------------------------
// Edwards points, extended coordinates
// ---------------------------------------------------------------------------
DEVI void ge_identity(ge &p) { fe_zero(p.X); fe_one(p.Y); fe_one(p.Z); fe_zero(p.T); }
// add-2008-hwcd-3, a = -1
DEVI void ge_add(ge &r, const ge &p, const ge &q) {
    fe a, b, c, d, e, f, g, h, t;
    fe_sub(a, p.Y, p.X); fe_sub(t, q.Y, q.X); fe_mul(a, a, t);
    fe_add(b, p.Y, p.X); fe_add(t, q.Y, q.X); fe_mul(b, b, t);
    fe_mul(c, p.T, q.T); fe_mul(c, c, FE_D2);
    fe_mul(d, p.Z, q.Z); fe_add(d, d, d);
    fe_sub(e, b, a); fe_sub(f, d, c); fe_add(g, d, c); fe_add(h, b, a);
    fe_mul(r.X, e, f); fe_mul(r.Y, g, h); fe_mul(r.T, e, h); fe_mul(r.Z, f, g);
}
DEVI void ge_neg(ge &r, const ge &p) { fe_neg(r.X, p.X); r.Y = p.Y; r.Z = p.Z; fe_neg(r.T, p.T); }
DEVI void ge_sub(ge &r, const ge &p, const ge &q) { ge n; ge_neg(n, q); ge_add(r, p, n); }
// dbl-2008-hwcd (a = -1), 4M + 4S
DEVI void ge_dbl(ge &r, const ge &p) {
    fe xx, yy, zz2, xpy2, ypx, ymx, ex, tc;
    fe_sq(xx, p.X); fe_sq(yy, p.Y); fe_sq(zz2, p.Z); fe_add(zz2, zz2, zz2);
    fe_add(xpy2, p.X, p.Y); fe_sq(xpy2, xpy2);
    fe_add(ypx, yy, xx); fe_sub(ymx, yy, xx);
    fe_sub(ex, xpy2, ypx); fe_sub(tc, zz2, ymx);
    fe_mul(r.X, ex, tc); fe_mul(r.Y, ypx, ymx); fe_mul(r.Z, ymx, tc); fe_mul(r.T, ex, ypx);
}
DEVI bool ge_is_identity(const ge &p) { return fe_iszero(p.X) || fe_iszero(p.Y); }

// RistrettoPoint::compress -> 8 canonical words
DEVI void ristretto_encode(uint32_t out[8], const ge &p) {
    fe u1, u2, t, invsqrt, i1, i2, z_inv, den_inv, iX, iY, ench, X, Y, tmp, s, one;
    fe_one(one);
    fe_add(u1, p.Z, p.Y); fe_sub(t, p.Z, p.Y); fe_mul(u1, u1, t);
    fe_mul(u2, p.X, p.Y);
    fe_sq(t, u2); fe_mul(t, t, u1);
    fe_sqrt_ratio_i(invsqrt, one, t);
    fe_mul(i1, invsqrt, u1); fe_mul(i2, invsqrt, u2);
    fe_mul(z_inv, i2, p.T); fe_mul(z_inv, z_inv, i1);
    den_inv = i2;
    fe_mul(iX, p.X, FE_SQRT_M1); fe_mul(iY, p.Y, FE_SQRT_M1);
    fe_mul(ench, i1, FE_INVSQRT_A_MINUS_D);
    fe_mul(tmp, p.T, z_inv);
    bool rotate = fe_isneg(tmp);
    X = rotate ? iY : p.X;
    Y = rotate ? iX : p.Y;
    if (rotate) den_inv = ench;
    fe_mul(tmp, X, z_inv);
    fe_cneg(Y, fe_isneg(tmp));
    fe_sub(s, p.Z, Y); fe_mul(s, den_inv, s);
    fe_cneg(s, fe_isneg(s));
    fe_tow(out, s);
}
// CompressedRistretto::decompress; false on invalid encodings.
DEVI bool ristretto_decode(ge &p, const uint32_t in[8]) {
    fe s, ss, u1, u2, u2sq, v, t, I, Dx, Dy, x, y, one;
    fe_one(one);
    if (in[7] >> 31) return false;
    fe_fromw(s, in);
    uint32_t chk[8]; fe_tow(chk, s);
    bool canon = true;
    for (int i = 0; i < 8; i++) canon = canon && (chk[i] == in[i]);
    if (!canon || (in[0] & 1)) return false;
    fe_sq(ss, s);
    fe_sub(u1, one, ss);
    fe_add(u2, one, ss);
    fe_sq(u2sq, u2);
    fe_sq(t, u1); fe_mul(t, t, FE_D); fe_neg(t, t); fe_sub(v, t, u2sq);
    fe_mul(t, v, u2sq);
    bool ok = fe_sqrt_ratio_i(I, one, t);
    fe_mul(Dx, I, u2);
    fe_mul(Dy, Dx, v); fe_mul(Dy, I, Dy);
    fe_add(x, s, s); fe_mul(x, x, Dx); fe_cneg(x, fe_isneg(x));
    fe_mul(y, u1, Dy);
    fe_mul(t, x, y);
    if (!ok || fe_isneg(t) || fe_iszero(y)) return false;
    p.X = x; p.Y = y; p.Z = one; p.T = t;
    return true;
}
// RistrettoPoint::elligator_ristretto_flavor
DEVI void ristretto_elligator(ge &p, const fe &r0) {
    fe r, Ns, Dd, s, sp, c, Nt, ssq, t, w0, w1, w2, w3, one;
    fe_one(one);
    fe_sq(r, r0); fe_mul(r, r, FE_SQRT_M1);
    fe_add(Ns, r, one); fe_mul(Ns, Ns, FE_ONE_MINUS_D_SQ);
    fe_neg(c, one);
    fe_mul(t, FE_D, r); fe_sub(Dd, c, t);
    fe_add(t, r, FE_D); fe_mul(Dd, Dd, t);
    bool sq = fe_sqrt_ratio_i(s, Ns, Dd);
    fe_mul(sp, s, r0);
    fe_cneg(sp, !fe_isneg(sp));
    if (!sq) { s = sp; c = r; }
    fe_sub(t, r, one); fe_mul(Nt, c, t); fe_mul(Nt, Nt, FE_D_MINUS_ONE_SQ); fe_sub(Nt, Nt, Dd);
    fe_sq(ssq, s);
    fe_add(w0, s, s); fe_mul(w0, w0, Dd);
    fe_mul(w1, Nt, FE_SQRT_AD_MINUS_ONE);
    fe_sub(w2, one, ssq);
    fe_add(w3, one, ssq);
    fe_mul(p.X, w0, w3); fe_mul(p.Y, w2, w1); fe_mul(p.Z, w1, w3); fe_mul(p.T, w0, w2);
}

// ---------------------------------------------------------------------------
// memory helpers: points are 128 B (X,Y,Z,T), loaded as 8 x uint4
// ---------------------------------------------------------------------------
DEVI void ge_load(ge &p, const ge *src) {
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 q[8];
#pragma unroll
    for (int i = 0; i < 8; i++) q[i] = s[i];
    uint32_t *d = reinterpret_cast<uint32_t *>(&p);
#pragma unroll
    for (int i = 0; i < 8; i++) { d[4 * i] = q[i].x; d[4 * i + 1] = q[i].y; d[4 * i + 2] = q[i].z; d[4 * i + 3] = q[i].w; }
}
DEVI void ge_store(ge *dst, const ge &p) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    const uint32_t *s = reinterpret_cast<const uint32_t *>(&p);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = make_uint4(s[4 * i], s[4 * i + 1], s[4 * i + 2], s[4 * i + 3]);
}
DEVI void sc_load(sc &r, const sc *src) {
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 a = s[0], b = s[1];
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
}
DEVI void sc_store(sc *dst, const sc &a) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
