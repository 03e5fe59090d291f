// hcrypto.cpp — see hcrypto.h. Algorithms: curve25519-dalek 3.2.0 (scalar.rs
// semantics, ristretto.rs encode/decode/elligator), merlin 2.0.1 (strobe.rs,
// transcript.rs), FIPS 202 Keccak, RFC 8439 ChaCha20.
#include "hcrypto.h"

#include <chrono>

#include <stdio.h>
#include <stdlib.h>
#include <sys/random.h>

namespace bpg {
typedef unsigned __int128 u128;

static inline uint64_t ld64(const uint8_t *p) { uint64_t r; memcpy(&r, p, 8); return r; }
static inline void st64(uint8_t *p, uint64_t x) { memcpy(p, &x, 8); }

// ============================================================== scalars
static const uint64_t LL[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
// Montgomery constants of l (R = 2^256): np = -l^-1 mod 2^64, r1 = R mod l,
// r2 = R^2 mod l (the statement layer multiplies millions of scalars, so
// these are plain constants rather than computed on first use behind a
// thread-safe static guard)
struct ScConsts {
    uint64_t np;
    uint64_t r2[4];
    uint64_t r1[4];
};
static const ScConsts SCC = {0xd2b51da312547e1bULL,
                             {0xa40611e3449c0f01ULL, 0xd00e1ba768859347ULL, 0xceec73d217f5be65ULL, 0x0399411b7c309a3dULL},
                             {0xd6ec31748d98951dULL, 0xc6ef5bf4737dcf70ULL, 0xfffffffffffffffeULL, 0x0fffffffffffffffULL}};
static inline const ScConsts &scc() { return SCC; }

static inline bool geq_l(const uint64_t t[4]) {
    for (int i = 3; i >= 0; i--) { if (t[i] != LL[i]) return t[i] > LL[i]; }
    return true;
}
static inline void sub_l(uint64_t t[4]) {
    u128 b = 0;
    for (int i = 0; i < 4; i++) { u128 d = (u128)t[i] - LL[i] - b; t[i] = (uint64_t)d; b = (d >> 64) & 1; }
}
static void reduce256_slow(uint64_t t[4]) {
    while (geq_l(t)) {
        uint64_t q = t[3] >> 60;
        if (q <= 1) { sub_l(t); continue; }
        q -= 1;
        uint64_t ql[4]; u128 c = 0;
        for (int i = 0; i < 4; i++) { c += (u128)LL[i] * q; ql[i] = (uint64_t)c; c >>= 64; }
        u128 b = 0;
        for (int i = 0; i < 4; i++) { u128 d = (u128)t[i] - ql[i] - b; t[i] = (uint64_t)d; b = (d >> 64) & 1; }
    }
}
// t < l whenever its top limb is below l's (l >= 2^252): the common case
static inline void reduce256(uint64_t t[4]) {
    if (t[3] < LL[3]) return;
    reduce256_slow(t);
}
// CIOS Montgomery; a < 2^256, b < l -> result < l
static inline void montmul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    const uint64_t np = scc().np;
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) { c += (u128)t[j] + (u128)a[j] * b[i]; t[j] = (uint64_t)c; c >>= 64; }
        c += t[4]; t[4] = (uint64_t)c; t[5] = (uint64_t)(c >> 64);
        uint64_t m = t[0] * np;
        c = (u128)t[0] + (u128)m * LL[0]; c >>= 64;
        for (int j = 1; j < 4; j++) { c += (u128)t[j] + (u128)m * LL[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
        c += t[4]; t[3] = (uint64_t)c; c >>= 64;
        t[4] = t[5] + (uint64_t)c;
    }
    if (t[4] || geq_l(t)) sub_l(t);
    memcpy(r, t, 32);
}

Scalar Scalar::from_bits(const uint8_t b[32]) {
    Scalar s;
    for (int i = 0; i < 4; i++) s.v[i] = ld64(b + 8 * i);
    s.v[3] &= 0x7fffffffffffffffULL;
    return s;
}
Scalar Scalar::reduce(const uint8_t b[32]) {
    Scalar s;
    for (int i = 0; i < 4; i++) s.v[i] = ld64(b + 8 * i);
    reduce256(s.v);
    return s;
}
Scalar Scalar::reduced() const { Scalar s = *this; reduce256(s.v); return s; }
Scalar Scalar::from_wide(const uint8_t b[64]) {
    Scalar lo = reduce(b), hi = reduce(b + 32);
    montmul(hi.v, hi.v, scc().r2);
    return lo + hi;
}
bool Scalar::from_canonical(const uint8_t b[32], Scalar &out) {
    if (b[31] >> 7) return false;
    Scalar s = reduce(b);
    uint8_t c[32]; s.to_bytes(c);
    if (memcmp(c, b, 32) != 0) return false;
    out = s;
    return true;
}
void Scalar::to_bytes(uint8_t out[32]) const { for (int i = 0; i < 4; i++) st64(out + 8 * i, v[i]); }

Scalar operator+(const Scalar &a0, const Scalar &b0) {
    Scalar a = a0.reduced(), b = b0.reduced(), r;
    u128 c = 0;
    for (int i = 0; i < 4; i++) { c += (u128)a.v[i] + b.v[i]; r.v[i] = (uint64_t)c; c >>= 64; }
    if (geq_l(r.v)) sub_l(r.v);
    return r;
}
Scalar operator-(const Scalar &a0, const Scalar &b0) {
    Scalar a = a0.reduced(), b = b0.reduced(), r;
    u128 bw = 0;
    for (int i = 0; i < 4; i++) { u128 d = (u128)a.v[i] - b.v[i] - bw; r.v[i] = (uint64_t)d; bw = (d >> 64) & 1; }
    if (bw) { u128 c = 0; for (int i = 0; i < 4; i++) { c += (u128)r.v[i] + LL[i]; r.v[i] = (uint64_t)c; c >>= 64; } }
    return r;
}
Scalar operator-(const Scalar &a) { return Scalar::zero() - a; }
static inline bool is_one(const Scalar &x) { return x.v[0] == 1 && !x.v[1] && !x.v[2] && !x.v[3]; }
Scalar operator*(const Scalar &a, const Scalar &b0) {
    // unit coefficients are common in the statement layer's linear combinations
    if (is_one(b0)) return a.reduced();
    if (is_one(a)) return b0.reduced();
    Scalar b = b0.reduced(), t, r;
    montmul(t.v, a.v, b.v);
    montmul(r.v, t.v, scc().r2);
    return r;
}
Scalar sc_invert(const Scalar &a0) {
    static const uint64_t E[4] = {0x5812631a5cf5d3ebULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
    Scalar a = a0.reduced(), am, acc;
    montmul(am.v, a.v, scc().r2);
    memcpy(acc.v, scc().r1, 32);
    for (int i = 252; i >= 0; i--) {
        montmul(acc.v, acc.v, acc.v);
        if ((E[i / 64] >> (i % 64)) & 1) montmul(acc.v, acc.v, am.v);
    }
    Scalar one = Scalar::one(), r;
    montmul(r.v, acc.v, one.v);
    return r;
}
void sc_batch_invert(std::vector<Scalar> &xs) {
    // Montgomery's trick (dalek Scalar::batch_invert semantics for nonzero inputs)
    if (xs.empty()) return;
    std::vector<Scalar> pre(xs.size());
    Scalar acc = Scalar::one();
    for (size_t i = 0; i < xs.size(); i++) { pre[i] = acc; acc = acc * xs[i]; }
    Scalar inv = sc_invert(acc);
    for (size_t i = xs.size(); i-- > 0;) { Scalar t = inv * xs[i]; xs[i] = inv * pre[i]; inv = t; }
}
Scalar sc_pow_u64(const Scalar &a, uint64_t e) {
    Scalar r = Scalar::one(), b = a.reduced();
    while (e) { if (e & 1) r = r * b; b = b * b; e >>= 1; }
    return r;
}

// ============================================================== field 2^255-19
static const uint64_t M51 = (1ULL << 51) - 1;
static const Fe FE0 = {{0, 0, 0, 0, 0}};
static const Fe FE1 = {{1, 0, 0, 0, 0}};
static const Fe FD = {{0x34dca135978a3ULL, 0x1a8283b156ebdULL, 0x5e7a26001c029ULL, 0x739c663a03cbbULL, 0x52036cee2b6ffULL}};
static const Fe FD2 = {{0x69b9426b2f159ULL, 0x35050762add7aULL, 0x3cf44c0038052ULL, 0x6738cc7407977ULL, 0x2406d9dc56dffULL}};
static const Fe FSQRTM1 = {{0x61b274a0ea0b0ULL, 0x0d5a5fc8f189dULL, 0x7ef5e9cbd0c60ULL, 0x78595a6804c9eULL, 0x2b8324804fc1dULL}};
static const Fe FSQRTADM1 = {{0x7f6a0497b2e1bULL, 0x1836f0a97afd2ULL, 0x7d747f6be7638ULL, 0x456079e7e6498ULL, 0x376931bf2b834ULL}};
static const Fe FINVSQRTAMD = {{0x0fdaa805d40eaULL, 0x2eb482e57d339ULL, 0x007610274bc58ULL, 0x6510b613dc8ffULL, 0x786c8905cfaffULL}};
static const Fe F1MDSQ = {{0x409c1945fc176ULL, 0x719abc6a1fc4fULL, 0x1c37f90b20684ULL, 0x06bccca55eedfULL, 0x029072a8b2b3eULL}};
static const Fe FDM1SQ = {{0x55aaa44ed4d20ULL, 0x59603c3332635ULL, 0x26d3baf4a7928ULL, 0x120a66e6997a9ULL, 0x5968b37af66c2ULL}};

static inline void fcarry(Fe &r) {
    uint64_t c;
    c = r.v[0] >> 51; r.v[0] &= M51; r.v[1] += c;
    c = r.v[1] >> 51; r.v[1] &= M51; r.v[2] += c;
    c = r.v[2] >> 51; r.v[2] &= M51; r.v[3] += c;
    c = r.v[3] >> 51; r.v[3] &= M51; r.v[4] += c;
    c = r.v[4] >> 51; r.v[4] &= M51; r.v[0] += c * 19;
}
static inline void fadd(Fe &r, const Fe &a, const Fe &b) { for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i]; fcarry(r); }
static inline void fsub(Fe &r, const Fe &a, const Fe &b) {
    r.v[0] = (a.v[0] + 36028797018963664ULL) - b.v[0];
    for (int i = 1; i < 5; i++) r.v[i] = (a.v[i] + 36028797018963952ULL) - b.v[i];
    fcarry(r);
}
static inline void fneg(Fe &r, const Fe &a) { fsub(r, FE0, a); }
static void fmul(Fe &r, const Fe &a, const Fe &b) {
    const uint64_t b1 = b.v[1] * 19, b2 = b.v[2] * 19, b3 = b.v[3] * 19, b4 = b.v[4] * 19;
    u128 t0 = (u128)a.v[0] * b.v[0] + (u128)a.v[1] * b4 + (u128)a.v[2] * b3 + (u128)a.v[3] * b2 + (u128)a.v[4] * b1;
    u128 t1 = (u128)a.v[0] * b.v[1] + (u128)a.v[1] * b.v[0] + (u128)a.v[2] * b4 + (u128)a.v[3] * b3 + (u128)a.v[4] * b2;
    u128 t2 = (u128)a.v[0] * b.v[2] + (u128)a.v[1] * b.v[1] + (u128)a.v[2] * b.v[0] + (u128)a.v[3] * b4 + (u128)a.v[4] * b3;
    u128 t3 = (u128)a.v[0] * b.v[3] + (u128)a.v[1] * b.v[2] + (u128)a.v[2] * b.v[1] + (u128)a.v[3] * b.v[0] + (u128)a.v[4] * b4;
    u128 t4 = (u128)a.v[0] * b.v[4] + (u128)a.v[1] * b.v[3] + (u128)a.v[2] * b.v[2] + (u128)a.v[3] * b.v[1] + (u128)a.v[4] * b.v[0];
    uint64_t r0, r1, r2, r3, r4;
    r0 = (uint64_t)t0 & M51; t1 += (uint64_t)(t0 >> 51);
    r1 = (uint64_t)t1 & M51; t2 += (uint64_t)(t1 >> 51);
    r2 = (uint64_t)t2 & M51; t3 += (uint64_t)(t2 >> 51);
    r3 = (uint64_t)t3 & M51; t4 += (uint64_t)(t3 >> 51);
    r4 = (uint64_t)t4 & M51;
    r0 += (uint64_t)(t4 >> 51) * 19;
    r1 += r0 >> 51; r0 &= M51;
    r.v[0] = r0; r.v[1] = r1; r.v[2] = r2; r.v[3] = r3; r.v[4] = r4;
}
static inline void fsq(Fe &r, const Fe &a) { fmul(r, a, a); }
static void fsqn(Fe &r, const Fe &a, int n) { fsq(r, a); for (int i = 1; i < n; i++) fsq(r, r); }
static void ftobytes(uint8_t s[32], const Fe &a) {
    Fe t = a; fcarry(t); fcarry(t);
    uint64_t q = (t.v[0] + 19) >> 51;
    for (int i = 1; i < 5; i++) q = (t.v[i] + q) >> 51;
    t.v[0] += 19 * q;
    for (int i = 0; i < 4; i++) { t.v[i + 1] += t.v[i] >> 51; t.v[i] &= M51; }
    t.v[4] &= M51;
    st64(s, t.v[0] | (t.v[1] << 51));
    st64(s + 8, (t.v[1] >> 13) | (t.v[2] << 38));
    st64(s + 16, (t.v[2] >> 26) | (t.v[3] << 25));
    st64(s + 24, (t.v[3] >> 39) | (t.v[4] << 12));
}
static void ffrombytes(Fe &r, const uint8_t s[32]) {
    r.v[0] = ld64(s) & M51;
    r.v[1] = (ld64(s + 6) >> 3) & M51;
    r.v[2] = (ld64(s + 12) >> 6) & M51;
    r.v[3] = (ld64(s + 19) >> 1) & M51;
    r.v[4] = (ld64(s + 24) >> 12) & M51;
}
static bool fisneg(const Fe &a) { uint8_t s[32]; ftobytes(s, a); return s[0] & 1; }
static bool fiszero(const Fe &a) { uint8_t s[32]; ftobytes(s, a); uint8_t x = 0; for (int i = 0; i < 32; i++) x |= s[i]; return x == 0; }
static bool feq(const Fe &a, const Fe &b) { uint8_t x[32], y[32]; ftobytes(x, a); ftobytes(y, b); return memcmp(x, y, 32) == 0; }
static void fpow22501(Fe &t19, Fe &t3, const Fe &z) {
    Fe t0, t1, t2, t4;
    fsq(t0, z); fsqn(t1, t0, 2); fmul(t1, z, t1); fmul(t0, t0, t1); t3 = t0;
    fsq(t2, t0); fmul(t1, t1, t2);
    fsqn(t2, t1, 5); fmul(t1, t2, t1);
    fsqn(t2, t1, 10); fmul(t2, t2, t1);
    fsqn(t4, t2, 20); fmul(t2, t4, t2);
    fsqn(t2, t2, 10); fmul(t1, t2, t1);
    fsqn(t2, t1, 50); fmul(t2, t2, t1);
    fsqn(t4, t2, 100); fmul(t2, t4, t2);
    fsqn(t2, t2, 50); fmul(t19, t2, t1);
}
static void fpowp58(Fe &r, const Fe &z) { Fe a, b; fpow22501(a, b, z); fsqn(a, a, 2); fmul(r, a, z); }
static bool fsqrt_ratio_i(Fe &r, const Fe &u, const Fe &v) {
    Fe v3, v7, t, check, nu, nui, rp;
    fsq(v3, v); fmul(v3, v3, v);
    fsq(v7, v3); fmul(v7, v7, v);
    fmul(t, u, v7); fpowp58(t, t);
    fmul(r, u, v3); fmul(r, r, t);
    fsq(check, r); fmul(check, check, v);
    fneg(nu, u); fmul(nui, nu, FSQRTM1);
    bool correct = feq(check, u), flipped = feq(check, nu), flipped_i = feq(check, nui);
    fmul(rp, r, FSQRTM1);
    if (flipped || flipped_i) r = rp;
    if (fisneg(r)) fneg(r, r);
    return correct || flipped;
}

void pt_identity(Point &p) { p.X = FE0; p.Y = FE1; p.Z = FE1; p.T = FE0; }
void pt_add(Point &r, const Point &p, const Point &q) {
    Fe a, b, c, d, e, f, g, h, t;
    fsub(a, p.Y, p.X); fsub(t, q.Y, q.X); fmul(a, a, t);
    fadd(b, p.Y, p.X); fadd(t, q.Y, q.X); fmul(b, b, t);
    fmul(c, p.T, q.T); fmul(c, c, FD2);
    fmul(d, p.Z, q.Z); fadd(d, d, d);
    fsub(e, b, a); fsub(f, d, c); fadd(g, d, c); fadd(h, b, a);
    fmul(r.X, e, f); fmul(r.Y, g, h); fmul(r.T, e, h); fmul(r.Z, f, g);
}
void pt_neg(Point &r, const Point &p) { fneg(r.X, p.X); r.Y = p.Y; r.Z = p.Z; fneg(r.T, p.T); }
void pt_dbl(Point &r, const Point &p) {
    Fe xx, yy, zz2, xpy2, ypx, ymx, ex, tc;
    fsq(xx, p.X); fsq(yy, p.Y); fsq(zz2, p.Z); fadd(zz2, zz2, zz2);
    fadd(xpy2, p.X, p.Y); fsq(xpy2, xpy2);
    fadd(ypx, yy, xx); fsub(ymx, yy, xx);
    fsub(ex, xpy2, ypx); fsub(tc, zz2, ymx);
    fmul(r.X, ex, tc); fmul(r.Y, ypx, ymx); fmul(r.Z, ymx, tc); fmul(r.T, ex, ypx);
}
bool pt_is_identity(const Point &p) { return fiszero(p.X) || fiszero(p.Y); }

void ristretto_compress(uint8_t out[32], const Point &p) {
    Fe u1, u2, t, invsqrt, i1, i2, z_inv, den_inv, iX, iY, ench, X, Y, tmp, s;
    fadd(u1, p.Z, p.Y); fsub(t, p.Z, p.Y); fmul(u1, u1, t);
    fmul(u2, p.X, p.Y);
    fsq(t, u2); fmul(t, t, u1);
    fsqrt_ratio_i(invsqrt, FE1, t);
    fmul(i1, invsqrt, u1); fmul(i2, invsqrt, u2);
    fmul(z_inv, i2, p.T); fmul(z_inv, z_inv, i1);
    den_inv = i2;
    fmul(iX, p.X, FSQRTM1); fmul(iY, p.Y, FSQRTM1);
    fmul(ench, i1, FINVSQRTAMD);
    fmul(tmp, p.T, z_inv);
    bool rotate = fisneg(tmp);
    X = rotate ? iY : p.X;
    Y = rotate ? iX : p.Y;
    if (rotate) den_inv = ench;
    fmul(tmp, X, z_inv);
    if (fisneg(tmp)) fneg(Y, Y);
    fsub(s, p.Z, Y); fmul(s, den_inv, s);
    if (fisneg(s)) fneg(s, s);
    ftobytes(out, s);
}
bool ristretto_decompress(Point &p, const uint8_t in[32]) {
    Fe s, ss, u1, u2, u2sq, v, t, I, Dx, Dy, x, y;
    uint8_t chk[32];
    ffrombytes(s, in); ftobytes(chk, s);
    if (memcmp(chk, in, 32) != 0 || fisneg(s)) return false;
    fsq(ss, s); fsub(u1, FE1, ss); fadd(u2, FE1, ss); fsq(u2sq, u2);
    fsq(t, u1); fmul(t, t, FD); fneg(t, t); fsub(v, t, u2sq);
    fmul(t, v, u2sq);
    bool ok = fsqrt_ratio_i(I, FE1, t);
    fmul(Dx, I, u2); fmul(Dy, Dx, v); fmul(Dy, I, Dy);
    fadd(x, s, s); fmul(x, x, Dx); if (fisneg(x)) fneg(x, x);
    fmul(y, u1, Dy); fmul(t, x, y);
    if (!ok || fisneg(t) || fiszero(y)) return false;
    p.X = x; p.Y = y; p.Z = FE1; p.T = t;
    return true;
}
static void elligator(Point &p, const Fe &r0) {
    Fe r, Ns, Dd, s, sp, c, Nt, ssq, t, w0, w1, w2, w3;
    fsq(r, r0); fmul(r, r, FSQRTM1);
    fadd(Ns, r, FE1); fmul(Ns, Ns, F1MDSQ);
    fneg(c, FE1);
    fmul(t, FD, r); fsub(Dd, c, t); fadd(t, r, FD); fmul(Dd, Dd, t);
    bool sq = fsqrt_ratio_i(s, Ns, Dd);
    fmul(sp, s, r0); if (!fisneg(sp)) fneg(sp, sp);
    if (!sq) { s = sp; c = r; }
    fsub(t, r, FE1); fmul(Nt, c, t); fmul(Nt, Nt, FDM1SQ); fsub(Nt, Nt, Dd);
    fsq(ssq, s);
    fadd(w0, s, s); fmul(w0, w0, Dd); fmul(w1, Nt, FSQRTADM1); fsub(w2, FE1, ssq); fadd(w3, FE1, ssq);
    fmul(p.X, w0, w3); fmul(p.Y, w2, w1); fmul(p.Z, w1, w3); fmul(p.T, w0, w2);
}
void ristretto_from_uniform(Point &p, const uint8_t b[64]) {
    Fe r1, r2; Point p1, p2;
    ffrombytes(r1, b); ffrombytes(r2, b + 32);
    elligator(p1, r1); elligator(p2, r2);
    pt_add(p, p1, p2);
}

// Device field elements are 10 limbs of 26/25 bits (dev_field.h): limbs 2k
// and 2k+1 are the low 26 and high 25 bits of radix-2^51 limb k. Device
// limbs may carry a few bits over their width; fcarry absorbs that.
static void fe_from_w(Fe &r, const uint32_t w[10]) {
    for (int k = 0; k < 5; k++) r.v[k] = (uint64_t)w[2 * k] + ((uint64_t)w[2 * k + 1] << 26);
    fcarry(r);
}
static void fe_to_w(uint32_t w[10], const Fe &a) {
    Fe t = a;
    fcarry(t);
    for (int k = 0; k < 5; k++) { w[2 * k] = (uint32_t)(t.v[k] & 0x3ffffff); w[2 * k + 1] = (uint32_t)(t.v[k] >> 26); }
}
void pt_from_dev(Point &p, const uint32_t w[40]) { fe_from_w(p.X, w); fe_from_w(p.Y, w + 10); fe_from_w(p.Z, w + 20); fe_from_w(p.T, w + 30); }
void pt_to_dev(uint32_t w[40], const Point &p) { fe_to_w(w, p.X); fe_to_w(w + 10, p.Y); fe_to_w(w + 20, p.Z); fe_to_w(w + 30, p.T); }
void pt_to_dev_cached(uint32_t w[40], const Point &p) {
    Fe ypx, ymx, z2, t2d;
    fadd(ypx, p.Y, p.X); fsub(ymx, p.Y, p.X); fadd(z2, p.Z, p.Z); fmul(t2d, p.T, FD2);
    fe_to_w(w, ypx); fe_to_w(w + 10, ymx); fe_to_w(w + 20, z2); fe_to_w(w + 30, t2d);
}

void pt_to_dev_niels(uint32_t w[32], const Point &p) {
    Fe t19, t3, zi, x, y, t, ypx, ymx, t2d;
    fpow22501(t19, t3, p.Z); fsqn(t19, t19, 5); fmul(zi, t19, t3);   // Z^(p-2)
    fmul(x, p.X, zi); fmul(y, p.Y, zi);
    fadd(ypx, y, x); fsub(ymx, y, x); fmul(t, x, y); fmul(t2d, t, FD2);
    fe_to_w(w, ypx); fe_to_w(w + 10, ymx); fe_to_w(w + 20, t2d);
    w[30] = w[31] = 0;
}
void pt_to_dev_affine(uint32_t w[16], const Point &p) {
    Fe t19, t3, zi, x, y;
    fpow22501(t19, t3, p.Z); fsqn(t19, t19, 5); fmul(zi, t19, t3);   // Z^(p-2)
    fmul(x, p.X, zi); fmul(y, p.Y, zi);
    uint8_t b[32];
    ftobytes(b, x); memcpy(w, b, 32);
    ftobytes(b, y); memcpy(w + 8, b, 32);
}
void pt_from_dev_niels(Point &p, const uint32_t w[32]) {
    Fe ypx, ymx, two, t;
    fe_from_w(ypx, w); fe_from_w(ymx, w + 10);
    // (2x : 2y : 2 : ...) -> extended (X Z : Y Z : Z^2 : X Y) with Z = 2
    Fe x2, y2;
    fsub(x2, ypx, ymx); fadd(y2, ypx, ymx);
    two = FE1; fadd(two, two, two);
    fmul(p.X, x2, two); fmul(p.Y, y2, two); fmul(p.Z, two, two); fmul(p.T, x2, y2);
    (void)t;
}
void radix16_digits(const Scalar &s0, int8_t e[64]) {
    Scalar s = s0.reduced();
    uint8_t b[32]; s.to_bytes(b);
    for (int i = 0; i < 32; i++) { e[2 * i] = b[i] & 15; e[2 * i + 1] = (b[i] >> 4) & 15; }
    for (int i = 0; i < 63; i++) { int8_t c = (e[i] + 8) >> 4; e[i] -= c << 4; e[i + 1] += c; }
}

static const uint8_t BASEPOINT_COMPRESSED[32] = {
    0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
    0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};

// Fixed-base table: T[w][j] = (j+1) * 16^w * P, w < 64, j < 8 (signed radix 16).
struct FixedTable {
    Point P;
    std::vector<Point> T;
    void build(const Point &p) {
        P = p; T.resize(64 * 8);
        Point base = p;
        for (int w = 0; w < 64; w++) {
            T[8 * w] = base;
            for (int j = 1; j < 8; j++) pt_add(T[8 * w + j], T[8 * w + j - 1], base);
            for (int k = 0; k < 4; k++) pt_dbl(base, base);
        }
    }
    void mul(Point &r, const Scalar &s0) const {
        Scalar s = s0.reduced();
        uint8_t b[32]; s.to_bytes(b);
        int8_t e[64];
        for (int i = 0; i < 32; i++) { e[2 * i] = b[i] & 15; e[2 * i + 1] = (b[i] >> 4) & 15; }
        for (int i = 0; i < 63; i++) { int8_t c = (e[i] + 8) >> 4; e[i] -= c << 4; e[i + 1] += c; }
        pt_identity(r);
        for (int w = 0; w < 64; w++) {
            if (e[w] > 0) pt_add(r, r, T[8 * w + e[w] - 1]);
            else if (e[w] < 0) { Point n; pt_neg(n, T[8 * w - e[w] - 1]); pt_add(r, r, n); }
        }
    }
};
struct PedersenTables {
    FixedTable B, Bb;
    PedersenTables() {
        Point b; ristretto_decompress(b, BASEPOINT_COMPRESSED);
        uint8_t h[64]; sha3_512(h, BASEPOINT_COMPRESSED, 32);
        Point bb; ristretto_from_uniform(bb, h);
        B.build(b); Bb.build(bb);
    }
};
static const PedersenTables &ptab() { static PedersenTables t; return t; }
const Point &basepoint_B() { return ptab().B.P; }
const Point &basepoint_B_blinding() { return ptab().Bb.P; }
void mul_B(Point &r, const Scalar &s) { ptab().B.mul(r, s); }
void mul_B_blinding(Point &r, const Scalar &s) { ptab().Bb.mul(r, s); }
void pedersen_commit(uint8_t out[32], const Scalar &v, const Scalar &vb) {
    Point a, b, c; mul_B(a, v); mul_B_blinding(b, vb); pt_add(c, a, b); ristretto_compress(out, c);
}
void mul_var(Point &r, const Scalar &s0, const Point &p) {
    Scalar s = s0.reduced();
    uint8_t b[32]; s.to_bytes(b);
    pt_identity(r);
    for (int i = 255; i >= 0; i--) {
        pt_dbl(r, r);
        if ((b[i / 8] >> (i % 8)) & 1) pt_add(r, r, p);
    }
}

// ============================================================== keccak
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
#define ROL(x, s) (((x) << (s)) | ((x) >> (64 - (s))))
// Keccak-f[1600], fully unrolled theta/rho/pi/chi/iota on 25 named lanes.
void keccakf_scalar(uint64_t s[25]) {
    uint64_t a00 = s[0], a01 = s[1], a02 = s[2], a03 = s[3], a04 = s[4];
    uint64_t a05 = s[5], a06 = s[6], a07 = s[7], a08 = s[8], a09 = s[9];
    uint64_t a10 = s[10], a11 = s[11], a12 = s[12], a13 = s[13], a14 = s[14];
    uint64_t a15 = s[15], a16 = s[16], a17 = s[17], a18 = s[18], a19 = s[19];
    uint64_t a20 = s[20], a21 = s[21], a22 = s[22], a23 = s[23], a24 = s[24];
    for (int r = 0; r < 24; r++) {
        uint64_t c0 = a00 ^ a05 ^ a10 ^ a15 ^ a20, c1 = a01 ^ a06 ^ a11 ^ a16 ^ a21;
        uint64_t c2 = a02 ^ a07 ^ a12 ^ a17 ^ a22, c3 = a03 ^ a08 ^ a13 ^ a18 ^ a23;
        uint64_t c4 = a04 ^ a09 ^ a14 ^ a19 ^ a24;
        uint64_t d0 = c4 ^ ROL(c1, 1), d1 = c0 ^ ROL(c2, 1), d2 = c1 ^ ROL(c3, 1), d3 = c2 ^ ROL(c4, 1), d4 = c3 ^ ROL(c0, 1);
        // theta + rho + pi: b[y][2x+3y] = rot(a[x][y] ^ d[x])
        uint64_t b00 = a00 ^ d0;
        uint64_t b10 = ROL(a01 ^ d1, 1), b20 = ROL(a02 ^ d2, 62), b05 = ROL(a03 ^ d3, 28), b15 = ROL(a04 ^ d4, 27);
        uint64_t b16 = ROL(a05 ^ d0, 36), b01 = ROL(a06 ^ d1, 44), b11 = ROL(a07 ^ d2, 6), b21 = ROL(a08 ^ d3, 55), b06 = ROL(a09 ^ d4, 20);
        uint64_t b07 = ROL(a10 ^ d0, 3), b17 = ROL(a11 ^ d1, 10), b02 = ROL(a12 ^ d2, 43), b12 = ROL(a13 ^ d3, 25), b22 = ROL(a14 ^ d4, 39);
        uint64_t b23 = ROL(a15 ^ d0, 41), b08 = ROL(a16 ^ d1, 45), b18 = ROL(a17 ^ d2, 15), b03 = ROL(a18 ^ d3, 21), b13 = ROL(a19 ^ d4, 8);
        uint64_t b14 = ROL(a20 ^ d0, 18), b24 = ROL(a21 ^ d1, 2), b09 = ROL(a22 ^ d2, 61), b19 = ROL(a23 ^ d3, 56), b04 = ROL(a24 ^ d4, 14);
        a00 = b00 ^ (~b01 & b02) ^ RC[r]; a01 = b01 ^ (~b02 & b03); a02 = b02 ^ (~b03 & b04); a03 = b03 ^ (~b04 & b00); a04 = b04 ^ (~b00 & b01);
        a05 = b05 ^ (~b06 & b07); a06 = b06 ^ (~b07 & b08); a07 = b07 ^ (~b08 & b09); a08 = b08 ^ (~b09 & b05); a09 = b09 ^ (~b05 & b06);
        a10 = b10 ^ (~b11 & b12); a11 = b11 ^ (~b12 & b13); a12 = b12 ^ (~b13 & b14); a13 = b13 ^ (~b14 & b10); a14 = b14 ^ (~b10 & b11);
        a15 = b15 ^ (~b16 & b17); a16 = b16 ^ (~b17 & b18); a17 = b17 ^ (~b18 & b19); a18 = b18 ^ (~b19 & b15); a19 = b19 ^ (~b15 & b16);
        a20 = b20 ^ (~b21 & b22); a21 = b21 ^ (~b22 & b23); a22 = b22 ^ (~b23 & b24); a23 = b23 ^ (~b24 & b20); a24 = b24 ^ (~b20 & b21);
    }
    s[0] = a00; s[1] = a01; s[2] = a02; s[3] = a03; s[4] = a04;
    s[5] = a05; s[6] = a06; s[7] = a07; s[8] = a08; s[9] = a09;
    s[10] = a10; s[11] = a11; s[12] = a12; s[13] = a13; s[14] = a14;
    s[15] = a15; s[16] = a16; s[17] = a17; s[18] = a18; s[19] = a19;
    s[20] = a20; s[21] = a21; s[22] = a22; s[23] = a23; s[24] = a24;
}
#undef ROL
// One state: the AVX-512 form or the scalar one, whichever is faster on
// this CPU, measured once (the single-proof TranscriptRng chain is ~1.5 M
// serial permutations). The two differ by CPU: on the Intel host of the
// build container the AVX-512 form takes 464 vs 690 ns, on the GPU box's
// EPYC 9575F 244 vs 191 ns (profiles/r04d_rng_bench.txt).
static bool pick_avx512_x1() {
    if (!have_avx512()) return false;
    uint64_t a[25] = {1}, b[25] = {1};
    auto time = [](void (*f)(uint64_t *), uint64_t *st) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 4000; i++) f(st);
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    time(keccakf_scalar, a);
    time(keccakf_x1_avx512, b);
    return time(keccakf_x1_avx512, b) < time(keccakf_scalar, a);
}
void keccakf(uint64_t s[25]) {
    static const bool avx = pick_avx512_x1();
    if (avx) keccakf_x1_avx512(s);
    else keccakf_scalar(s);
}
static inline void perm_bytes(uint8_t st[200]) {
    uint64_t w[25];
    memcpy(w, st, 200);   // little-endian host
    keccakf(w);
    memcpy(st, w, 200);
}
static void sponge_hash(uint8_t *out, size_t olen, const uint8_t *in, size_t len, unsigned rate, uint8_t ds) {
    uint8_t st[200] = {0};
    size_t pos = 0;
    for (size_t i = 0; i < len; i++) { st[pos++] ^= in[i]; if (pos == rate) { perm_bytes(st); pos = 0; } }
    st[pos] ^= ds; st[rate - 1] ^= 0x80; perm_bytes(st); pos = 0;
    for (size_t i = 0; i < olen; i++) { if (pos == rate) { perm_bytes(st); pos = 0; } out[i] = st[pos++]; }
}
void sha3_512(uint8_t out[64], const uint8_t *in, size_t len) { sponge_hash(out, 64, in, len, 72, 0x06); }
void Shake256::init_absorb(const uint8_t *in, size_t len) {
    uint8_t st8[200] = {0};
    size_t p = 0;
    for (size_t i = 0; i < len; i++) { st8[p++] ^= in[i]; if (p == 136) { perm_bytes(st8); p = 0; } }
    st8[p] ^= 0x1f; st8[135] ^= 0x80; perm_bytes(st8);
    memcpy(st, st8, 200);
    pos = 0;
}
void Shake256::squeeze(uint8_t *out, size_t len) {
    uint8_t *b = reinterpret_cast<uint8_t *>(st);
    while (len) {
        if (pos == 136) { keccakf(st); pos = 0; }
        size_t take = 136 - pos; if (take > len) take = len;
        memcpy(out, b + pos, take); out += take; len -= take; pos += (unsigned)take;
    }
}

// ============================================================== strobe / merlin
enum { F_I = 1, F_A = 2, F_C = 4, F_M = 16, F_K = 32, STROBE_R = 166 };
void Strobe128::run_f() {
    st[pos] ^= pos_begin; st[pos + 1] ^= 0x04; st[STROBE_R + 1] ^= 0x80;
    perm_bytes(st); pos = 0; pos_begin = 0;
}
void Strobe128::absorb(const uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) { st[pos++] ^= d[i]; if (pos == STROBE_R) run_f(); }
}
void Strobe128::begin_op(uint8_t flags, bool more) {
    if (more) return;
    uint8_t old = pos_begin;
    pos_begin = pos + 1; cur_flags = flags;
    uint8_t b[2] = {old, flags};
    absorb(b, 2);
    if ((flags & (F_C | F_K)) && pos != 0) run_f();
}
void Strobe128::init(const uint8_t *label, size_t n) {
    memset(st, 0, 200);
    const uint8_t hdr[6] = {1, STROBE_R + 2, 1, 0, 1, 96};
    memcpy(st, hdr, 6); memcpy(st + 6, "STROBEv1.0.2", 12);
    perm_bytes(st); pos = pos_begin = cur_flags = 0;
    meta_ad(label, n, false);
}
void Strobe128::meta_ad(const uint8_t *d, size_t n, bool more) { begin_op(F_M | F_A, more); absorb(d, n); }
void Strobe128::ad(const uint8_t *d, size_t n, bool more) { begin_op(F_A, more); absorb(d, n); }
void Strobe128::prf(uint8_t *d, size_t n, bool more) {
    begin_op(F_I | F_A | F_C, more);
    for (size_t i = 0; i < n; i++) { d[i] = st[pos]; st[pos] = 0; pos++; if (pos == STROBE_R) run_f(); }
}
void Strobe128::key(const uint8_t *d, size_t n, bool more) {
    begin_op(F_A | F_C, more);
    for (size_t i = 0; i < n; i++) { st[pos++] = d[i]; if (pos == STROBE_R) run_f(); }
}
static inline void u32le(uint8_t b[4], uint32_t x) { b[0] = x; b[1] = x >> 8; b[2] = x >> 16; b[3] = x >> 24; }
Transcript::Transcript(const uint8_t *label, size_t n) {
    s.init((const uint8_t *)"Merlin v1.0", 11);
    append_message("dom-sep", label, n);
}
void Transcript::append_message(const char *label, const uint8_t *msg, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    s.meta_ad((const uint8_t *)label, strlen(label), false);
    s.meta_ad(len, 4, true);
    s.ad(msg, n, false);
}
void Transcript::append_u64(const char *label, uint64_t x) { uint8_t b[8]; st64(b, x); append_message(label, b, 8); }
void Transcript::challenge_bytes(const char *label, uint8_t *out, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    s.meta_ad((const uint8_t *)label, strlen(label), false);
    s.meta_ad(len, 4, true);
    s.prf(out, n, false);
}
Scalar Transcript::challenge_scalar(const char *label) { uint8_t b[64]; challenge_bytes(label, b, 64); return Scalar::from_wide(b); }
void TranscriptRng::rekey_with_witness_bytes(const char *label, const uint8_t *w, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    s.meta_ad((const uint8_t *)label, strlen(label), false);
    s.meta_ad(len, 4, true);
    s.key(w, n, false);
}
void TranscriptRng::finalize(const uint8_t entropy[32]) {
    s.meta_ad((const uint8_t *)"rng", 3, false);
    s.key(entropy, 32, false);
}
void TranscriptRng::fill_bytes(uint8_t *d, size_t n) {
    uint8_t len[4]; u32le(len, (uint32_t)n);
    s.meta_ad(len, 4, false);
    s.prf(d, n, false);
}
// fill_bytes(d, 64) after another 64-byte draw (STROBE at pos 64, pos_begin
// 0): meta_ad(len) + begin_op(I|A|C) + run_f only xor constant framing
// bytes into words 8, 9 and 20 (DRAW64_W*), then the permutation, and the
// 64 output bytes are read and zeroed. Identical to fill_bytes
// (bpg_rng_selftest); any other state takes the general path.
void TranscriptRng::draw64(uint8_t d[64]) {
    if (s.pos != 64 || s.pos_begin != 0) { fill_bytes(d, 64); return; }
    uint64_t *w = reinterpret_cast<uint64_t *>(s.st);
    w[8] ^= DRAW64_W8;
    w[9] ^= DRAW64_W9;
    w[20] ^= DRAW64_W20;
    keccakf(w);
    memcpy(d, w, 64);
    memset(w, 0, 64);
    s.pos = 64;
    s.pos_begin = 0;
    s.cur_flags = F_I | F_A | F_C;
}

// ============================================================== chacha20
static void chacha_block(uint8_t out[64], const uint8_t key[32], uint32_t counter) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) { uint32_t k; memcpy(&k, key + 4 * i, 4); s[4 + i] = k; }
    s[12] = counter; s[13] = s[14] = s[15] = 0;
    memcpy(x, s, 64);
#define QR(a, b, c, d) a += b; d ^= a; d = (d << 16) | (d >> 16); c += d; b ^= c; b = (b << 12) | (b >> 20); \
    a += b; d ^= a; d = (d << 8) | (d >> 24); c += d; b ^= c; b = (b << 7) | (b >> 25);
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
#undef QR
    for (int i = 0; i < 16; i++) { uint32_t v = x[i] + s[i]; memcpy(out + 4 * i, &v, 4); }
}
void ChaChaStream::seed(uint64_t sd) {
    memset(key, 0, 32); st64(key, sd);
    offset = 0; block_idx = (uint64_t)-1;
}
void ChaChaStream::fill(uint8_t *out, size_t n) {
    while (n) {
        uint64_t b = offset / 64; unsigned o = offset % 64;
        if (b != block_idx) { chacha_block(block, key, (uint32_t)b); block_idx = b; }
        size_t take = 64 - o; if (take > n) take = n;
        memcpy(out, block + o, take); out += take; n -= take; offset += take;
    }
}
void EntropySource::fill(uint8_t *out, size_t n) {
    if (seeded) { cs.fill(out, n); return; }
    size_t got = 0;
    while (got < n) {
        ssize_t r = getrandom(out + got, n - got, 0);
        if (r <= 0) { fprintf(stderr, "bpg: getrandom failed\n"); abort(); }
        got += (size_t)r;
    }
}
EntropySource &thread_entropy() { static thread_local EntropySource e; return e; }

}  // namespace bpg
