// dev_field.h — GF(2^255-19), scalars mod l and Ristretto255 points on gfx950.
//
// Replaces the curve25519-dalek 3.2.0 serial/u64 + avx2 backends (field.rs,
// scalar.rs, ristretto.rs, edwards.rs) for the device side of the hot path.
// Representation is chosen for CDNA4's VALU, not translated from dalek:
//   * field elements: 10 limbs of 26/25 bits (radix 2^25.5), carry-free
//     64-bit column sums (v_mad_u64_u32), 2^255 == 19 folding; canonical
//     form only at encode/compare (details and bounds below).
//   * scalars: 8 x 32-bit limbs, canonical (< l); products by 32-bit CIOS
//     Montgomery (R = 2^256), no MFMA — this is 255-bit integer work.
//   * points: extended twisted-Edwards (X:Y:Z:T), a = -1, 160 bytes; cached
//     (Y+X, Y-X, 2Z, 2dT) right operands for 8M additions.
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

// Field elements: 10 limbs, radix 2^25.5 (widths 26,25,26,...; limb i sits
// at bit ceil(25.5 i)). Measured on gfx950 (csrc/bench/fe_variants.hip):
// v_mad_u64_u32 issues at full rate, and 100 carry-free 64-bit
// multiply-accumulates into column sums plus one carry pass beat an 8x32-bit
// schoolbook product by 1.6x (the 32-bit carry chains cost more in moves
// and 64-bit adds than the extra multiplies).
//
// Bounds. "T" (tight) = each limb <= mask + 2^17; every fe_mul / fe_sq /
// fe_carry output and every stored coordinate is T. Unreduced sums are
// allowed where the bound is tracked (tests/test_devsim.py checks the worst
// cases):
//   fe_add_nc(T,T) <= 2T;  fe_sub_nc(a, T) <= a + 2T;  fe_sub4_nc(a, <=3T) <= a + 4T
//   fe_mul(f, g): f <= 5T (6T if g <= 2T), g <= 3T   (column sums < 2^64,
//   19 g_j < 2^32);  fe_sq(f): f <= 3T.
// fe_add / fe_sub / fe_neg (no suffix) carry and return T.
struct fe { uint32_t v[10]; };
struct sc { uint32_t v[8]; };
struct ge { fe X, Y, Z, T; };           // extended twisted Edwards, a = -1
struct gec { fe YpX, YmX, Z2, T2d; };   // cached: (Y+X, Y-X, 2Z, 2dT)
// affine Niels (Z = 1): (y+x, y-x, 2dxy), padded to 128 B so a random gather
// is exactly one 128-B line (generators, decompressed inputs)
struct gen { fe YpX, YmX, T2d; uint32_t pad[2]; };

#define FE_M26 0x3ffffffu
#define FE_M25 0x1ffffffu
DEVI constexpr int fe_width(int i) { return (i & 1) ? 25 : 26; }
DEVI constexpr int fe_pos(int i) { return (i >> 1) * 51 + ((i & 1) ? 26 : 0); }

// 8 little-endian 32-bit words (bit 255 ignored) -> limbs
DEVI constexpr fe fe_from_words(const uint32_t w0, const uint32_t w1, const uint32_t w2, const uint32_t w3,
                                const uint32_t w4, const uint32_t w5, const uint32_t w6, const uint32_t w7) {
    fe r{};
    const uint32_t w[9] = {w0, w1, w2, w3, w4, w5, w6, w7, 0};
    for (int i = 0; i < 10; i++) {
        int p = fe_pos(i), wi = p >> 5, sh = p & 31;
        uint64_t x = ((uint64_t)w[wi] | ((uint64_t)w[wi + 1] << 32)) >> sh;
        r.v[i] = (uint32_t)x & ((1u << fe_width(i)) - 1);
    }
    return r;
}

// ---------------------------------------------------------------------------
// constants (derivation: oracle/gen_consts.py; values per RFC 9496 §4.1)
// ---------------------------------------------------------------------------
#define FE_C(name, a0, a1, a2, a3, a4, a5, a6, a7) \
    static __device__ __constant__ const fe name = fe_from_words(a0, a1, a2, a3, a4, a5, a6, a7);
FE_C(FE_D, 0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu)
FE_C(FE_D_INV, 0xcdc9f843u, 0x25e0f276u, 0x4279542eu, 0x0b5dd698u, 0xcdb9cf66u, 0x2b162114u, 0x14d5ce43u, 0x40907ed2u)   // 1/d
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
    for (int i = 0; i < 10; i++) r.v[i] = 0;
}
DEVI void fe_one(fe &r) { fe_zero(r); r.v[0] = 1; }

// weak reduction to T: every limb to its width plus the incoming carry
DEVI void fe_carry(fe &r, const fe &a) {
    uint32_t c[10];
#pragma unroll
    for (int i = 0; i < 10; i++) c[i] = a.v[i] >> fe_width(i);
    r.v[0] = (a.v[0] & FE_M26) + 19 * c[9];
#pragma unroll
    for (int i = 1; i < 10; i++) r.v[i] = (a.v[i] & ((i & 1) ? FE_M25 : FE_M26)) + c[i - 1];
}
DEVI void fe_add_nc(fe &r, const fe &a, const fe &b) {
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + b.v[i];
}
// a - b + 2p (b <= T)
DEVI void fe_sub_nc(fe &r, const fe &a, const fe &b) {
    r.v[0] = a.v[0] + 0x7ffffdau - b.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) r.v[i] = a.v[i] + ((i & 1) ? 0x3fffffeu : 0x7fffffeu) - b.v[i];
}
// a - b + 4p (b <= 3T)
DEVI void fe_sub4_nc(fe &r, const fe &a, const fe &b) {
    r.v[0] = a.v[0] + 0xfffffb4u - b.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) r.v[i] = a.v[i] + ((i & 1) ? 0x7fffffcu : 0xffffffcu) - b.v[i];
}
DEVI void fe_add(fe &r, const fe &a, const fe &b) { fe t; fe_add_nc(t, a, b); fe_carry(r, t); }
DEVI void fe_sub(fe &r, const fe &a, const fe &b) { fe t; fe_sub4_nc(t, a, b); fe_carry(r, t); }
DEVI void fe_neg(fe &r, const fe &a) { fe z; fe_zero(z); fe_sub(r, z, a); }

DEVI uint64_t fe_m64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

// column sums -> T (carry order keeps every intermediate < 2^64)
DEVI void fe_carry_cols(fe &r, uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3, uint64_t h4, uint64_t h5,
                        uint64_t h6, uint64_t h7, uint64_t h8, uint64_t h9) {
    uint64_t c;
    c = h0 >> 26; h1 += c; h0 &= FE_M26;
    c = h4 >> 26; h5 += c; h4 &= FE_M26;
    c = h1 >> 25; h2 += c; h1 &= FE_M25;
    c = h5 >> 25; h6 += c; h5 &= FE_M25;
    c = h2 >> 26; h3 += c; h2 &= FE_M26;
    c = h6 >> 26; h7 += c; h6 &= FE_M26;
    c = h3 >> 25; h4 += c; h3 &= FE_M25;
    c = h7 >> 25; h8 += c; h7 &= FE_M25;
    c = h4 >> 26; h5 += c; h4 &= FE_M26;
    c = h8 >> 26; h9 += c; h8 &= FE_M26;
    c = h9 >> 25; h0 += c * 19; h9 &= FE_M25;
    c = h0 >> 26; h1 += c; h0 &= FE_M26;
    r.v[0] = (uint32_t)h0; r.v[1] = (uint32_t)h1; r.v[2] = (uint32_t)h2; r.v[3] = (uint32_t)h3;
    r.v[4] = (uint32_t)h4; r.v[5] = (uint32_t)h5; r.v[6] = (uint32_t)h6; r.v[7] = (uint32_t)h7;
    r.v[8] = (uint32_t)h8; r.v[9] = (uint32_t)h9;
}

DEVI void fe_mul(fe &h, const fe &f, const fe &g) {
    const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4], f5 = f.v[5], f6 = f.v[6],
                   f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
    const uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4], g5 = g.v[5], g6 = g.v[6],
                   g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
    const uint32_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4, g5_19 = 19 * g5,
                   g6_19 = 19 * g6, g7_19 = 19 * g7, g8_19 = 19 * g8, g9_19 = 19 * g9;
    const uint32_t f1_2 = 2 * f1, f3_2 = 2 * f3, f5_2 = 2 * f5, f7_2 = 2 * f7, f9_2 = 2 * f9;
    uint64_t h0 = fe_m64(f0, g0) + fe_m64(f1_2, g9_19) + fe_m64(f2, g8_19) + fe_m64(f3_2, g7_19) +
                  fe_m64(f4, g6_19) + fe_m64(f5_2, g5_19) + fe_m64(f6, g4_19) + fe_m64(f7_2, g3_19) +
                  fe_m64(f8, g2_19) + fe_m64(f9_2, g1_19);
    uint64_t h1 = fe_m64(f0, g1) + fe_m64(f1, g0) + fe_m64(f2, g9_19) + fe_m64(f3, g8_19) + fe_m64(f4, g7_19) +
                  fe_m64(f5, g6_19) + fe_m64(f6, g5_19) + fe_m64(f7, g4_19) + fe_m64(f8, g3_19) + fe_m64(f9, g2_19);
    uint64_t h2 = fe_m64(f0, g2) + fe_m64(f1_2, g1) + fe_m64(f2, g0) + fe_m64(f3_2, g9_19) + fe_m64(f4, g8_19) +
                  fe_m64(f5_2, g7_19) + fe_m64(f6, g6_19) + fe_m64(f7_2, g5_19) + fe_m64(f8, g4_19) +
                  fe_m64(f9_2, g3_19);
    uint64_t h3 = fe_m64(f0, g3) + fe_m64(f1, g2) + fe_m64(f2, g1) + fe_m64(f3, g0) + fe_m64(f4, g9_19) +
                  fe_m64(f5, g8_19) + fe_m64(f6, g7_19) + fe_m64(f7, g6_19) + fe_m64(f8, g5_19) + fe_m64(f9, g4_19);
    uint64_t h4 = fe_m64(f0, g4) + fe_m64(f1_2, g3) + fe_m64(f2, g2) + fe_m64(f3_2, g1) + fe_m64(f4, g0) +
                  fe_m64(f5_2, g9_19) + fe_m64(f6, g8_19) + fe_m64(f7_2, g7_19) + fe_m64(f8, g6_19) +
                  fe_m64(f9_2, g5_19);
    uint64_t h5 = fe_m64(f0, g5) + fe_m64(f1, g4) + fe_m64(f2, g3) + fe_m64(f3, g2) + fe_m64(f4, g1) +
                  fe_m64(f5, g0) + fe_m64(f6, g9_19) + fe_m64(f7, g8_19) + fe_m64(f8, g7_19) + fe_m64(f9, g6_19);
    uint64_t h6 = fe_m64(f0, g6) + fe_m64(f1_2, g5) + fe_m64(f2, g4) + fe_m64(f3_2, g3) + fe_m64(f4, g2) +
                  fe_m64(f5_2, g1) + fe_m64(f6, g0) + fe_m64(f7_2, g9_19) + fe_m64(f8, g8_19) + fe_m64(f9_2, g7_19);
    uint64_t h7 = fe_m64(f0, g7) + fe_m64(f1, g6) + fe_m64(f2, g5) + fe_m64(f3, g4) + fe_m64(f4, g3) +
                  fe_m64(f5, g2) + fe_m64(f6, g1) + fe_m64(f7, g0) + fe_m64(f8, g9_19) + fe_m64(f9, g8_19);
    uint64_t h8 = fe_m64(f0, g8) + fe_m64(f1_2, g7) + fe_m64(f2, g6) + fe_m64(f3_2, g5) + fe_m64(f4, g4) +
                  fe_m64(f5_2, g3) + fe_m64(f6, g2) + fe_m64(f7_2, g1) + fe_m64(f8, g0) + fe_m64(f9_2, g9_19);
    uint64_t h9 = fe_m64(f0, g9) + fe_m64(f1, g8) + fe_m64(f2, g7) + fe_m64(f3, g6) + fe_m64(f4, g5) +
                  fe_m64(f5, g4) + fe_m64(f6, g3) + fe_m64(f7, g2) + fe_m64(f8, g1) + fe_m64(f9, g0);
    fe_carry_cols(h, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);
}

// 55 products (symmetric terms doubled up front)
DEVI void fe_sq(fe &h, const fe &f) {
    const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4], f5 = f.v[5], f6 = f.v[6],
                   f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
    const uint32_t f0_2 = 2 * f0, f1_2 = 2 * f1, f2_2 = 2 * f2, f3_2 = 2 * f3, f4_2 = 2 * f4, f5_2 = 2 * f5,
                   f6_2 = 2 * f6, f7_2 = 2 * f7;
    const uint32_t f5_38 = 38 * f5, f6_19 = 19 * f6, f7_38 = 38 * f7, f8_19 = 19 * f8, f9_38 = 38 * f9;
    uint64_t h0 = fe_m64(f0, f0) + fe_m64(f1_2, f9_38) + fe_m64(f2_2, f8_19) + fe_m64(f3_2, f7_38) +
                  fe_m64(f4_2, f6_19) + fe_m64(f5, f5_38);
    uint64_t h1 = fe_m64(f0_2, f1) + fe_m64(f2, f9_38) + fe_m64(f3_2, f8_19) + fe_m64(f4, f7_38) +
                  fe_m64(f5_2, f6_19);
    uint64_t h2 = fe_m64(f0_2, f2) + fe_m64(f1_2, f1) + fe_m64(f3_2, f9_38) + fe_m64(f4_2, f8_19) +
                  fe_m64(f5_2, f7_38) + fe_m64(f6, f6_19);
    uint64_t h3 = fe_m64(f0_2, f3) + fe_m64(f1_2, f2) + fe_m64(f4, f9_38) + fe_m64(f5_2, f8_19) +
                  fe_m64(f6, f7_38);
    uint64_t h4 = fe_m64(f0_2, f4) + fe_m64(f1_2, f3_2) + fe_m64(f2, f2) + fe_m64(f5_2, f9_38) +
                  fe_m64(f6_2, f8_19) + fe_m64(f7, f7_38);
    uint64_t h5 = fe_m64(f0_2, f5) + fe_m64(f1_2, f4) + fe_m64(f2_2, f3) + fe_m64(f6, f9_38) +
                  fe_m64(f7_2, f8_19);
    uint64_t h6 = fe_m64(f0_2, f6) + fe_m64(f1_2, f5_2) + fe_m64(f2_2, f4) + fe_m64(f3_2, f3) +
                  fe_m64(f7_2, f9_38) + fe_m64(f8, f8_19);
    uint64_t h7 = fe_m64(f0_2, f7) + fe_m64(f1_2, f6) + fe_m64(f2_2, f5) + fe_m64(f3_2, f4) + fe_m64(f8, f9_38);
    uint64_t h8 = fe_m64(f0_2, f8) + fe_m64(f1_2, f7_2) + fe_m64(f2_2, f6) + fe_m64(f3_2, f5_2) +
                  fe_m64(f4, f4) + fe_m64(f9, f9_38);
    uint64_t h9 = fe_m64(f0_2, f9) + fe_m64(f1_2, f8) + fe_m64(f2_2, f7) + fe_m64(f3_2, f6) + fe_m64(f4_2, f5);
    fe_carry_cols(h, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);
}

DEVI void fe_sqn(fe &r, const fe &a, int n) {
    fe_sq(r, a);
    for (int i = 1; i < n; i++) fe_sq(r, r);
}

// Fully reduce to the canonical representative in [0, p), limbs at width.
DEVI void fe_canon(fe &r, const fe &a) {
    uint32_t h[10];
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = a.v[i];
    // two sequential carry passes: value < 2^255 + small, limbs at width
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
#pragma unroll
        for (int i = 0; i < 9; i++) { h[i + 1] += h[i] >> fe_width(i); h[i] &= (i & 1) ? FE_M25 : FE_M26; }
        h[0] += 19 * (h[9] >> 25); h[9] &= FE_M25;
    }
    // h >= p  <=>  h + 19 >= 2^255
    uint32_t q = (h[0] + 19) >> 26;
#pragma unroll
    for (int i = 1; i < 10; i++) q = (h[i] + q) >> fe_width(i);
    h[0] += 19 * q;
#pragma unroll
    for (int i = 0; i < 9; i++) { h[i + 1] += h[i] >> fe_width(i); h[i] &= (i & 1) ? FE_M25 : FE_M26; }
    h[9] &= FE_M25;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = h[i];
}

// canonical 8 x 32-bit words
DEVI void fe_tow(uint32_t w[8], const fe &a) {
    fe c; fe_canon(c, a);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const int p = fe_pos(i), wi = p >> 5, sh = p & 31;
        w[wi] |= c.v[i] << sh;
        if (sh + fe_width(i) > 32 && wi + 1 < 8) w[wi + 1] |= c.v[i] >> (32 - sh);
    }
}
DEVI void fe_tobytes(uint8_t s[32], const fe &a) {
    uint32_t w[8]; fe_tow(w, a);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        s[4 * i] = (uint8_t)w[i]; s[4 * i + 1] = (uint8_t)(w[i] >> 8);
        s[4 * i + 2] = (uint8_t)(w[i] >> 16); s[4 * i + 3] = (uint8_t)(w[i] >> 24);
    }
}
// FieldElement::from_bytes: bit 255 ignored.
DEVI void fe_fromw(fe &r, const uint32_t w[8]) { r = fe_from_words(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]); }
DEVI bool fe_iszero(const fe &a) {
    fe c; fe_canon(c, a);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) acc |= c.v[i];
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
// Edwards points. Extended (X:Y:Z:T), T = XY/Z; cached (Y+X, Y-X, 2Z, 2dT)
// for the right operand of additions. All coordinates T on output.
// ---------------------------------------------------------------------------
DEVI void ge_identity(ge &p) { fe_zero(p.X); fe_one(p.Y); fe_one(p.Z); fe_zero(p.T); }
DEVI void gec_identity(gec &c) { fe_one(c.YpX); fe_one(c.YmX); fe_zero(c.Z2); c.Z2.v[0] = 2; fe_zero(c.T2d); }
DEVI void ge_to_cached(gec &c, const ge &p) {
    fe_add(c.YpX, p.Y, p.X);
    fe_sub(c.YmX, p.Y, p.X);
    fe_add(c.Z2, p.Z, p.Z);
    fe_mul(c.T2d, p.T, FE_D2);
}
// -c: swap Y+X / Y-X and negate 2dT
DEVI void gec_neg(gec &r, const gec &c) { r.YpX = c.YmX; r.YmX = c.YpX; r.Z2 = c.Z2; fe_neg(r.T2d, c.T2d); }
DEVI void gec_cneg(gec &c, bool neg) {
    if (neg) { fe t = c.YpX; c.YpX = c.YmX; c.YmX = t; fe_neg(c.T2d, c.T2d); }
}
// Operand roles in the four output products: fe_mul(h, f, g) doubles the odd
// limbs of f and multiplies g by 19, so the formulas pair the outputs'
// factors as two sets, one always first and one always second (X = e f,
// Y = g h, T = e h, Z = g f): each set's premultiplied limbs are computed
// once and shared by its two products (14 fewer instructions per addition),
// with the g side within 3T as fe_mul requires.
// add-2008-hwcd-3 (a = -1) with a cached right operand: 8M; with_t = false
// skips T (7M) for an addition followed by a doubling (T is not an input of
// doubling), as ge_dbl_t does.
template <bool with_t>
DEVI void ge_add_c_t(ge &r, const ge &p, const gec &q) {
    fe a, b, c, d, e, f, g, h;
    fe_sub_nc(a, p.Y, p.X); fe_mul(a, a, q.YmX);       // 3T x T
    fe_add_nc(b, p.Y, p.X); fe_mul(b, b, q.YpX);       // 2T x T
    fe_mul(c, p.T, q.T2d);
    fe_mul(d, p.Z, q.Z2);
    fe_sub_nc(e, b, a);                                 // 3T
    fe_sub_nc(f, d, c);                                 // 3T
    fe_add_nc(g, d, c);                                 // 2T
    fe_add_nc(h, b, a);                                 // 2T
    fe_mul(r.X, e, f); fe_mul(r.Y, g, h); if (with_t) fe_mul(r.T, e, h); fe_mul(r.Z, g, f);
}
template <bool with_t>
DEVI void ge_sub_c_t(ge &r, const ge &p, const gec &q) {
    fe a, b, c, d, e, f, g, h;
    fe_sub_nc(a, p.Y, p.X); fe_mul(a, a, q.YpX);
    fe_add_nc(b, p.Y, p.X); fe_mul(b, b, q.YmX);
    fe_mul(c, p.T, q.T2d);
    fe_mul(d, p.Z, q.Z2);
    fe_sub_nc(e, b, a);
    fe_add_nc(f, d, c);                                 // D + C for -q
    fe_sub_nc(g, d, c);
    fe_add_nc(h, b, a);
    fe_mul(r.X, e, f); fe_mul(r.Y, g, h); if (with_t) fe_mul(r.T, e, h); fe_mul(r.Z, g, f);
}
DEVI void ge_add_c(ge &r, const ge &p, const gec &q) { ge_add_c_t<true>(r, p, q); }
DEVI void ge_sub_c(ge &r, const ge &p, const gec &q) { ge_sub_c_t<true>(r, p, q); }
// madd-2008-hwcd-3 (a = -1) with an affine Niels right operand: 7M.
// D = 2 Z1 unreduced (2T): F = D - C <= 4T, G = D + C <= 3T, E <= 3T,
// H <= 2T, so every product below keeps fe_mul's argument bounds.
DEVI void ge_madd(ge &r, const ge &p, const gen &q) {
    fe a, b, c, d, e, f, g, h;
    fe_sub_nc(a, p.Y, p.X); fe_mul(a, a, q.YmX);
    fe_add_nc(b, p.Y, p.X); fe_mul(b, b, q.YpX);
    fe_mul(c, p.T, q.T2d);
    fe_add_nc(d, p.Z, p.Z);
    fe_sub_nc(e, b, a);
    fe_sub_nc(f, d, c);
    fe_add_nc(g, d, c);
    fe_add_nc(h, b, a);
    fe_mul(r.X, f, e); fe_mul(r.Y, h, g); fe_mul(r.T, h, e); fe_mul(r.Z, f, g);
}
DEVI void gen_cneg(gen &c, bool neg) {
    if (neg) { fe t = c.YpX; c.YpX = c.YmX; c.YmX = t; fe_neg(c.T2d, c.T2d); }
}
// identity + q without the addition (a run's first entry): from Y+X, Y-X
// and 2dT, (Y+X)-(Y-X) = 2X, (Y+X)+(Y-X) = 2Y and (2dT)/d = 2T give
// (2X : 2Y : 2Z : 2T), with Z = 1 for an affine Niels point: 1M instead of
// the 7M madd / 8M cached addition into the identity.
DEVI void ge_from_niels(ge &r, const gen &q) {
    fe_sub(r.X, q.YpX, q.YmX); fe_add(r.Y, q.YpX, q.YmX);
    fe_zero(r.Z); r.Z.v[0] = 2;
    fe_mul(r.T, q.T2d, FE_D_INV);
}
DEVI void ge_from_cached_t(ge &r, const gec &q) {   // uses 2dT (ge_from_cached below does not)
    fe_sub(r.X, q.YpX, q.YmX); fe_add(r.Y, q.YpX, q.YmX);
    r.Z = q.Z2;
    fe_mul(r.T, q.T2d, FE_D_INV);
}
DEVI void gen_identity(gen &c) { fe_one(c.YpX); fe_one(c.YmX); fe_zero(c.T2d); c.pad[0] = c.pad[1] = 0; }
// affine Niels as a cached point (2Z = 2)
DEVI void gen_to_cached(gec &r, const gen &q) { r.YpX = q.YpX; r.YmX = q.YmX; fe_zero(r.Z2); r.Z2.v[0] = 2; r.T2d = q.T2d; }
// extended -> affine Niels (one inversion)
DEVI void ge_to_niels(gen &n, const ge &p) {
    fe zi, x, y, t;
    fe_invert(zi, p.Z);
    fe_mul(x, p.X, zi); fe_mul(y, p.Y, zi);
    fe_add(n.YpX, y, x); fe_sub(n.YmX, y, x);
    fe_mul(t, x, y); fe_mul(n.T2d, t, FE_D2);
    n.pad[0] = n.pad[1] = 0;
}
// extended + extended (cached form of q built on the fly, unreduced): 9M
DEVI void ge_add(ge &r, const ge &p, const ge &q) {
    fe a, b, c, d, e, f, g, h, t;
    fe_sub_nc(a, p.Y, p.X); fe_sub_nc(t, q.Y, q.X); fe_mul(a, a, t);   // 3T x 3T
    fe_add_nc(b, p.Y, p.X); fe_add_nc(t, q.Y, q.X); fe_mul(b, b, t);   // 2T x 2T
    fe_mul(c, p.T, q.T); fe_mul(c, c, FE_D2);
    fe_add_nc(t, q.Z, q.Z); fe_mul(d, p.Z, t);                         // T x 2T
    fe_sub_nc(e, b, a);
    fe_sub_nc(f, d, c);
    fe_add_nc(g, d, c);
    fe_add_nc(h, b, a);
    fe_mul(r.X, e, f); fe_mul(r.Y, g, h); fe_mul(r.T, e, h); fe_mul(r.Z, g, f);
}
DEVI void ge_neg(ge &r, const ge &p) { fe_neg(r.X, p.X); r.Y = p.Y; r.Z = p.Z; fe_neg(r.T, p.T); }
DEVI void ge_sub(ge &r, const ge &p, const ge &q) { ge n; ge_neg(n, q); ge_add(r, p, n); }
// dbl-2008-hwcd (a = -1): 4M + 4S; with_t = false skips T (3M + 4S), for
// doublings followed by another doubling (T is not an input of doubling).
template <bool with_t>
DEVI void ge_dbl_t(ge &r, const ge &p) {
    fe xx, yy, zz2, xpy2, ypx, ymx, ex, tc;
    fe_sq(xx, p.X); fe_sq(yy, p.Y); fe_sq(zz2, p.Z);
    fe_add_nc(zz2, zz2, zz2);                           // 2T
    fe_add_nc(xpy2, p.X, p.Y); fe_sq(xpy2, xpy2);       // sq(2T)
    fe_add_nc(ypx, yy, xx);                             // 2T
    fe_sub_nc(ymx, yy, xx);                             // 3T
    fe_sub4_nc(ex, xpy2, ypx);                          // 5T
    fe_sub4_nc(tc, zz2, ymx); fe_carry(tc, tc);         // 6T -> T
    fe_mul(r.X, ex, tc); fe_mul(r.Y, ymx, ypx); fe_mul(r.Z, ymx, tc);
    if (with_t) fe_mul(r.T, ex, ypx);
}
DEVI void ge_dbl(ge &r, const ge &p) { ge_dbl_t<true>(r, p); }
DEVI bool ge_is_identity(const ge &p) { return fe_iszero(p.X) || fe_iszero(p.Y); }
// cached -> extended: (Y+X)-(Y-X) = 2X etc. give the projective (2X:2Y:2Z);
// extend with (X'Z' : Y'Z' : Z'^2 : X'Y')  (3M + 1S)
DEVI void ge_from_cached(ge &r, const gec &c) {
    fe x, y;
    fe_sub(x, c.YpX, c.YmX);
    fe_add(y, c.YpX, c.YmX);
    fe_mul(r.T, x, y);
    fe_mul(r.X, x, c.Z2);
    fe_mul(r.Y, y, c.Z2);
    fe_sq(r.Z, c.Z2);
}

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
// memory helpers: points move as 16-byte vectors (160 B extended/cached,
// 128 B affine Niels)
// ---------------------------------------------------------------------------
template <class P>
DEVI void pt_load(P &p, const P *src) {
    static_assert(sizeof(P) % 16 == 0, "point layout");
    constexpr int NQ = sizeof(P) / 16;
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 q[NQ];
#pragma unroll
    for (int i = 0; i < NQ; i++) q[i] = s[i];
    uint32_t *d = reinterpret_cast<uint32_t *>(&p);
#pragma unroll
    for (int i = 0; i < NQ; i++) { d[4 * i] = q[i].x; d[4 * i + 1] = q[i].y; d[4 * i + 2] = q[i].z; d[4 * i + 3] = q[i].w; }
}
template <class P>
DEVI void pt_store(P *dst, const P &p) {
    constexpr int NQ = sizeof(P) / 16;
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    const uint32_t *s = reinterpret_cast<const uint32_t *>(&p);
#pragma unroll
    for (int i = 0; i < NQ; i++) d[i] = make_uint4(s[4 * i], s[4 * i + 1], s[4 * i + 2], s[4 * i + 3]);
}
DEVI void ge_load(ge &p, const ge *src) { pt_load(p, src); }
DEVI void ge_store(ge *dst, const ge &p) { pt_store(dst, p); }
DEVI void gec_load(gec &p, const gec *src) { pt_load(p, src); }
DEVI void gec_store(gec *dst, const gec &p) { pt_store(dst, p); }
DEVI void gen_load(gen &p, const gen *src) { pt_load(p, src); }
DEVI void gen_store(gen *dst, const gen &p) { pt_store(dst, p); }
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

// Packed affine Niels (comb tables): three canonical field elements as
// 8 little-endian words each, 96 B = 6 x uint4.
DEVI void genp_store(uint4 *dst, const gen &q) {
    uint32_t w[24];
    fe_tow(w, q.YpX); fe_tow(w + 8, q.YmX); fe_tow(w + 16, q.T2d);
#pragma unroll
    for (int i = 0; i < 6; i++) dst[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}
DEVI void genp_unpack(gen &q, const uint4 (&s)[6]) {
    q.YpX = fe_from_words(s[0].x, s[0].y, s[0].z, s[0].w, s[1].x, s[1].y, s[1].z, s[1].w);
    q.YmX = fe_from_words(s[2].x, s[2].y, s[2].z, s[2].w, s[3].x, s[3].y, s[3].z, s[3].w);
    q.T2d = fe_from_words(s[4].x, s[4].y, s[4].z, s[4].w, s[5].x, s[5].y, s[5].z, s[5].w);
}
