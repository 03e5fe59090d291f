// hcrypto.h — host-side primitives that stay on the CPU by design:
//   * Scalar mod l (exact residues; curve25519-dalek 3.2.0 Scalar semantics:
//     Add/Sub/Mul/Neg return canonical values for any 256-bit input,
//     equality and byte access use the raw 32 bytes).
//   * a small Edwards/Ristretto point library for O(1)/O(log N) serial tails
//     (window combination of device MSM partials, T_k / Q fixed-base products,
//     encoding a handful of points). All O(N) group work runs in HIP kernels.
//   * Keccak-f[1600] / SHAKE256 / SHA3-512, STROBE-128 + Merlin transcript and
//     TranscriptRng (merlin@2.0.1), ChaCha20 (deterministic thread_rng).
#pragma once
#include <stdint.h>
#include <string.h>
#include <string>
#include <vector>

namespace bpg {

// ------------------------------------------------------------------- scalars
struct Scalar {
    uint64_t v[4];  // little-endian limbs; canonical unless built by from_bits
    static Scalar zero() { return Scalar{{0, 0, 0, 0}}; }
    static Scalar one() { return Scalar{{1, 0, 0, 0}}; }
    static Scalar from_u64(uint64_t x) { return Scalar{{x, 0, 0, 0}}; }
    // Scalar::from_bits: raw bytes with bit 255 cleared, no reduction.
    static Scalar from_bits(const uint8_t b[32]);
    // Scalar::from_bytes_mod_order_wide
    static Scalar from_wide(const uint8_t b[64]);
    static Scalar reduce(const uint8_t b[32]);          // any 256-bit -> mod l
    static bool from_canonical(const uint8_t b[32], Scalar &out);
    void to_bytes(uint8_t out[32]) const;
    std::string bytes() const { uint8_t b[32]; to_bytes(b); return std::string((const char *)b, 32); }
    Scalar reduced() const;
    bool is_zero_raw() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
    bool operator==(const Scalar &o) const { return memcmp(v, o.v, 32) == 0; }  // raw bytes, as dalek
    bool operator!=(const Scalar &o) const { return !(*this == o); }
};
Scalar operator+(const Scalar &a, const Scalar &b);
Scalar operator-(const Scalar &a, const Scalar &b);
Scalar operator*(const Scalar &a, const Scalar &b);
Scalar operator-(const Scalar &a);
Scalar sc_invert(const Scalar &a);      // Scalar::invert, invert(0) = 0
void sc_batch_invert(std::vector<Scalar> &xs);
Scalar sc_pow_u64(const Scalar &a, uint64_t e);

// ------------------------------------------------------- points (host tails)
struct Fe { uint64_t v[5]; };             // radix 2^51
struct Point { Fe X, Y, Z, T; };          // extended Edwards coordinates
void pt_identity(Point &p);
void pt_add(Point &r, const Point &p, const Point &q);
void pt_dbl(Point &r, const Point &p);
void pt_neg(Point &r, const Point &p);
bool pt_is_identity(const Point &p);
void ristretto_compress(uint8_t out[32], const Point &p);
bool ristretto_decompress(Point &p, const uint8_t in[32]);
void ristretto_from_uniform(Point &p, const uint8_t b[64]);
// conversion from/to the device layout (8 x 32-bit limbs per coordinate)
void pt_from_dev(Point &p, const uint32_t w[40]);   // device layout, dev_field.h
void pt_to_dev(uint32_t w[40], const Point &p);
void pt_to_dev_cached(uint32_t w[40], const Point &p);   // (Y+X, Y-X, 2Z, 2dT)
void pt_to_dev_niels(uint32_t w[32], const Point &p);    // affine (y+x, y-x, 2dxy)
void pt_to_dev_affine(uint32_t w[16], const Point &p);   // affine (x, y), canonical words
void pt_from_dev_niels(Point &p, const uint32_t w[32]);
// signed radix-16 digits of the reduced scalar, LSB first, |e[i]| <= 8
// (curve25519-dalek Scalar::to_radix_16)
void radix16_digits(const Scalar &s, int8_t e[64]);
// PedersenGens::default() with fixed-base tables
const Point &basepoint_B();
const Point &basepoint_B_blinding();
void mul_B(Point &r, const Scalar &s);            // s * B
void mul_B_blinding(Point &r, const Scalar &s);   // s * B_blinding
void pedersen_commit(uint8_t out[32], const Scalar &v, const Scalar &vb);
void mul_var(Point &r, const Scalar &s, const Point &p);

// -------------------------------------------------------- keccak / merlin
void keccakf(uint64_t st[25]);          // AVX-512 single-state form when available
void keccakf_scalar(uint64_t st[25]);   // the portable 64-bit form (reference for the self-test)
// Framing of a 64-byte TranscriptRng draw that follows another one (STROBE
// pos 64, pos_begin 0): bytes 64..73 = 0, M|A, 64, 0, 0, 0, 65, I|A|C (the
// meta_ad of the length and both begin_ops), 71, 0x04 (run_f's pos_begin and
// padding) and 0x80 at byte 167, as little-endian words 8, 9 and 20.
static const uint64_t DRAW64_W8 = 0x0741000000401200ULL, DRAW64_W9 = 0x0000000000000447ULL,
                      DRAW64_W20 = 0x8000000000000000ULL;
bool have_avx512();
void keccakf_x1_avx512(uint64_t s[25]);
void sha3_512(uint8_t out[64], const uint8_t *in, size_t len);

struct Shake256 {
    uint64_t st[25];
    unsigned pos;
    void init_absorb(const uint8_t *in, size_t len);   // absorb + finalize
    void squeeze(uint8_t *out, size_t len);
};

struct Strobe128 {
    uint8_t st[200];
    uint8_t pos, pos_begin, cur_flags;
    void init(const uint8_t *label, size_t n);
    void meta_ad(const uint8_t *d, size_t n, bool more);
    void ad(const uint8_t *d, size_t n, bool more);
    void prf(uint8_t *d, size_t n, bool more);
    void key(const uint8_t *d, size_t n, bool more);
  private:
    void run_f();
    void begin_op(uint8_t flags, bool more);
    void absorb(const uint8_t *d, size_t n);
};

struct Transcript {
    Strobe128 s;
    Transcript(const uint8_t *label, size_t n);
    void append_message(const char *label, const uint8_t *msg, size_t n);
    void append_u64(const char *label, uint64_t x);
    void challenge_bytes(const char *label, uint8_t *out, size_t n);
    Scalar challenge_scalar(const char *label);
    void append_point(const char *label, const uint8_t p[32]) { append_message(label, p, 32); }
    void append_scalar(const char *label, const Scalar &s) { uint8_t b[32]; s.to_bytes(b); append_message(label, b, 32); }
};

struct TranscriptRng {
    Strobe128 s;
    explicit TranscriptRng(const Transcript &t) : s(t.s) {}
    void rekey_with_witness_bytes(const char *label, const uint8_t *w, size_t n);
    void finalize(const uint8_t entropy[32]);
    void fill_bytes(uint8_t *d, size_t n);
    void draw64(uint8_t d[64]);   // fill_bytes(d, 64), constant-framing fast path
    Scalar random_scalar() { uint8_t b[64]; fill_bytes(b, 64); return Scalar::from_wide(b); }
};

// --------------------------------------------------------------- ChaCha20
// Deterministic stand-in for rand::thread_rng(): key = u64le(seed) || 0^24,
// nonce 0, counter from 0; bytes consumed in program order.
struct ChaChaStream {
    uint8_t key[32];
    uint64_t offset;
    uint8_t block[64];
    uint64_t block_idx;
    void seed(uint64_t s);
    void fill(uint8_t *out, size_t n);
    Scalar random_scalar() { uint8_t b[64]; fill(b, 64); return Scalar::from_wide(b); }
};
// Per-thread entropy source: seeded stream (bpg_set_seed) or OS entropy.
struct EntropySource {
    bool seeded = false;
    ChaChaStream cs;
    void fill(uint8_t *out, size_t n);
    Scalar random_scalar() { uint8_t b[64]; fill(b, 64); return Scalar::from_wide(b); }
};
EntropySource &thread_entropy();

}  // namespace bpg
