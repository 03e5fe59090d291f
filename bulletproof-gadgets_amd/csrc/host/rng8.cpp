// rng8.cpp — lockstep STROBE-128 / TranscriptRng for 8 proofs (see rng8.h).
#include "rng8.h"

#include <immintrin.h>
#include <string.h>

namespace bpg {

static const uint64_t RC8[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

bool have_avx512() {
    static const bool ok = __builtin_cpu_supports("avx512f");
    return ok;
}

// theta / rho / pi / chi / iota on 8 states at once; lane (x, y) = A[x + 5y]
__attribute__((target("avx512f"))) static void keccak8_avx512(uint64_t L[25][8]) {
    __m512i A[25];
    for (int i = 0; i < 25; i++) A[i] = _mm512_load_si512(reinterpret_cast<const void *>(L[i]));
#define XOR3(a, b, c) _mm512_ternarylogic_epi64(a, b, c, 0x96)
#define CHI(a, b, c) _mm512_ternarylogic_epi64(a, b, c, 0xD2)   // a ^ (~b & c)
#define ROL(x, s) _mm512_rol_epi64(x, s)
    for (int r = 0; r < 24; r++) {
        __m512i C0 = XOR3(A[0], A[5], XOR3(A[10], A[15], A[20]));
        __m512i C1 = XOR3(A[1], A[6], XOR3(A[11], A[16], A[21]));
        __m512i C2 = XOR3(A[2], A[7], XOR3(A[12], A[17], A[22]));
        __m512i C3 = XOR3(A[3], A[8], XOR3(A[13], A[18], A[23]));
        __m512i C4 = XOR3(A[4], A[9], XOR3(A[14], A[19], A[24]));
        __m512i D0 = _mm512_xor_si512(C4, ROL(C1, 1)), D1 = _mm512_xor_si512(C0, ROL(C2, 1));
        __m512i D2 = _mm512_xor_si512(C1, ROL(C3, 1)), D3 = _mm512_xor_si512(C2, ROL(C4, 1));
        __m512i D4 = _mm512_xor_si512(C3, ROL(C0, 1));
        __m512i B00 = _mm512_xor_si512(A[0], D0);
        __m512i B10 = ROL(_mm512_xor_si512(A[1], D1), 1), B20 = ROL(_mm512_xor_si512(A[2], D2), 62);
        __m512i B05 = ROL(_mm512_xor_si512(A[3], D3), 28), B15 = ROL(_mm512_xor_si512(A[4], D4), 27);
        __m512i B16 = ROL(_mm512_xor_si512(A[5], D0), 36), B01 = ROL(_mm512_xor_si512(A[6], D1), 44);
        __m512i B11 = ROL(_mm512_xor_si512(A[7], D2), 6), B21 = ROL(_mm512_xor_si512(A[8], D3), 55);
        __m512i B06 = ROL(_mm512_xor_si512(A[9], D4), 20);
        __m512i B07 = ROL(_mm512_xor_si512(A[10], D0), 3), B17 = ROL(_mm512_xor_si512(A[11], D1), 10);
        __m512i B02 = ROL(_mm512_xor_si512(A[12], D2), 43), B12 = ROL(_mm512_xor_si512(A[13], D3), 25);
        __m512i B22 = ROL(_mm512_xor_si512(A[14], D4), 39);
        __m512i B23 = ROL(_mm512_xor_si512(A[15], D0), 41), B08 = ROL(_mm512_xor_si512(A[16], D1), 45);
        __m512i B18 = ROL(_mm512_xor_si512(A[17], D2), 15), B03 = ROL(_mm512_xor_si512(A[18], D3), 21);
        __m512i B13 = ROL(_mm512_xor_si512(A[19], D4), 8);
        __m512i B14 = ROL(_mm512_xor_si512(A[20], D0), 18), B24 = ROL(_mm512_xor_si512(A[21], D1), 2);
        __m512i B09 = ROL(_mm512_xor_si512(A[22], D2), 61), B19 = ROL(_mm512_xor_si512(A[23], D3), 56);
        __m512i B04 = ROL(_mm512_xor_si512(A[24], D4), 14);
        A[0] = _mm512_xor_si512(CHI(B00, B01, B02), _mm512_set1_epi64((long long)RC8[r]));
        A[1] = CHI(B01, B02, B03); A[2] = CHI(B02, B03, B04); A[3] = CHI(B03, B04, B00); A[4] = CHI(B04, B00, B01);
        A[5] = CHI(B05, B06, B07); A[6] = CHI(B06, B07, B08); A[7] = CHI(B07, B08, B09); A[8] = CHI(B08, B09, B05);
        A[9] = CHI(B09, B05, B06);
        A[10] = CHI(B10, B11, B12); A[11] = CHI(B11, B12, B13); A[12] = CHI(B12, B13, B14); A[13] = CHI(B13, B14, B10);
        A[14] = CHI(B14, B10, B11);
        A[15] = CHI(B15, B16, B17); A[16] = CHI(B16, B17, B18); A[17] = CHI(B17, B18, B19); A[18] = CHI(B18, B19, B15);
        A[19] = CHI(B19, B15, B16);
        A[20] = CHI(B20, B21, B22); A[21] = CHI(B21, B22, B23); A[22] = CHI(B22, B23, B24); A[23] = CHI(B23, B24, B20);
        A[24] = CHI(B24, B20, B21);
    }
#undef XOR3
#undef CHI
#undef ROL
    for (int i = 0; i < 25; i++) _mm512_store_si512(reinterpret_cast<void *>(L[i]), A[i]);
}

void keccak8(uint64_t L[25][8]) {
    if (have_avx512()) { keccak8_avx512(L); return; }
    for (int s = 0; s < 8; s++) {
        uint64_t st[25];
        for (int i = 0; i < 25; i++) st[i] = L[i][s];
        keccakf(st);
        for (int i = 0; i < 25; i++) L[i][s] = st[i];
    }
}

enum { S8_I = 1, S8_A = 2, S8_C = 4, S8_M = 16, S8_K = 32, S8_R = 166 };

void Strobe8::from(const Strobe128 &s, int n) {
    nstates = n;
    uint64_t w[25];
    memcpy(w, s.st, 200);
    for (int i = 0; i < 25; i++)
        for (int k = 0; k < 8; k++) L[i][k] = w[i];
    pos = s.pos; pos_begin = s.pos_begin; cur_flags = s.cur_flags;
}
bool Strobe8::from_each(const Strobe128 *const *s, int n) {
    if (n < 1 || n > 8) return false;
    for (int k = 1; k < n; k++)
        if (s[k]->pos != s[0]->pos || s[k]->pos_begin != s[0]->pos_begin || s[k]->cur_flags != s[0]->cur_flags)
            return false;
    nstates = n;
    for (int k = 0; k < 8; k++) {
        uint64_t w[25];
        memcpy(w, s[k < n ? k : 0]->st, 200);
        for (int i = 0; i < 25; i++) L[i][k] = w[i];
    }
    pos = s[0]->pos; pos_begin = s[0]->pos_begin; cur_flags = s[0]->cur_flags;
    return true;
}
void Strobe8::run_f() {
    for (int s = 0; s < 8; s++) { byte(s, pos) ^= pos_begin; byte(s, pos + 1) ^= 0x04; byte(s, S8_R + 1) ^= 0x80; }
    if (nstates == 1) {   // single proof (latency path): the scalar permutation is faster
        uint64_t st[25];
        for (int i = 0; i < 25; i++) st[i] = L[i][0];
        keccakf(st);
        for (int i = 0; i < 25; i++) L[i][0] = st[i];
    } else {
        keccak8(L);
    }
    pos = 0; pos_begin = 0;
}
void Strobe8::absorb_same(const uint8_t *d, size_t len) {
    for (size_t i = 0; i < len; i++) {
        for (int s = 0; s < 8; s++) byte(s, pos) ^= d[i];
        if (++pos == S8_R) run_f();
    }
}
void Strobe8::begin_op(uint8_t flags) {
    uint8_t old = pos_begin;
    pos_begin = pos + 1; cur_flags = flags;
    const uint8_t b[2] = {old, flags};
    absorb_same(b, 2);
    if ((flags & (S8_C | S8_K)) && pos != 0) run_f();
}
void Strobe8::meta_ad(const uint8_t *d, size_t len) { begin_op(S8_M | S8_A); absorb_same(d, len); }
void Strobe8::key_each(const uint8_t *const *d, size_t len) {
    begin_op(S8_A | S8_C);
    for (size_t i = 0; i < len; i++) {
        for (int s = 0; s < 8; s++) byte(s, pos) = d[s < nstates ? s : 0][i];
        if (++pos == S8_R) run_f();
    }
}
void Strobe8::draw64(uint8_t *const *out) {
    static const uint8_t len64[4] = {64, 0, 0, 0};
    meta_ad(len64, 4);
    begin_op(S8_I | S8_A | S8_C);   // C forces a permutation: pos is now 0
    if (pos == 0) {
        for (int s = 0; s < nstates; s++) {
            uint64_t *o = reinterpret_cast<uint64_t *>(out[s]);
            for (int k = 0; k < 8; k++) o[k] = L[k][s];
        }
        for (int k = 0; k < 8; k++)
            for (int s = 0; s < 8; s++) L[k][s] = 0;
        pos = 64;
    } else {
        for (int i = 0; i < 64; i++) {
            for (int s = 0; s < 8; s++) {
                if (s < nstates) out[s][i] = byte(s, pos);
                byte(s, pos) = 0;
            }
            if (++pos == S8_R) run_f();
        }
    }
}

}  // namespace bpg
