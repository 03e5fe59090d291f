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
        // rho + pi + chi one output plane at a time (B[x, y'] for the five x
        // of plane y' come from five input planes), so that at most one
        // plane of B is live next to the old state: the 25-wide B of the
        // unordered form did not fit in 32 zmm registers and spilled
        {
            __m512i B00 = _mm512_xor_si512(A[0], D0), B01 = ROL(_mm512_xor_si512(A[6], D1), 44);
            __m512i B02 = ROL(_mm512_xor_si512(A[12], D2), 43), B03 = ROL(_mm512_xor_si512(A[18], D3), 21);
            __m512i B04 = ROL(_mm512_xor_si512(A[24], D4), 14);
            __m512i B05 = ROL(_mm512_xor_si512(A[3], D3), 28), B06 = ROL(_mm512_xor_si512(A[9], D4), 20);
            __m512i B07 = ROL(_mm512_xor_si512(A[10], D0), 3), B08 = ROL(_mm512_xor_si512(A[16], D1), 45);
            __m512i B09 = ROL(_mm512_xor_si512(A[22], D2), 61);
            __m512i B10 = ROL(_mm512_xor_si512(A[1], D1), 1), B11 = ROL(_mm512_xor_si512(A[7], D2), 6);
            __m512i B12 = ROL(_mm512_xor_si512(A[13], D3), 25), B13 = ROL(_mm512_xor_si512(A[19], D4), 8);
            __m512i B14 = ROL(_mm512_xor_si512(A[20], D0), 18);
            __m512i B15 = ROL(_mm512_xor_si512(A[4], D4), 27), B16 = ROL(_mm512_xor_si512(A[5], D0), 36);
            __m512i B17 = ROL(_mm512_xor_si512(A[11], D1), 10), B18 = ROL(_mm512_xor_si512(A[17], D2), 15);
            __m512i B19 = ROL(_mm512_xor_si512(A[23], D3), 56);
            __m512i B20 = ROL(_mm512_xor_si512(A[2], D2), 62), B21 = ROL(_mm512_xor_si512(A[8], D3), 55);
            __m512i B22 = ROL(_mm512_xor_si512(A[14], D4), 39), B23 = ROL(_mm512_xor_si512(A[15], D0), 41);
            __m512i B24 = ROL(_mm512_xor_si512(A[21], D1), 2);
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
    }
#undef XOR3
#undef CHI
#undef ROL
    for (int i = 0; i < 25; i++) _mm512_store_si512(reinterpret_cast<void *>(L[i]), A[i]);
}

// One state (the single-proof TranscriptRng chain: 2n + 8 serial
// permutations per proof, ~1.5 M at 2^20, so its latency is the proof's
// latency floor). The five planes y (lanes x = 0..4 of A[x + 5y]) sit in
// five zmm registers; theta and chi permute lanes within a plane, and pi
// (A[x, y] -> B[y, 2x + 3y]: output plane Y, lane X = input plane X, lane
// (X + 3Y) mod 5) is a skewed 5 x 5 transpose done by two levels of
// two-source permutes and a blend. About 45 vector ops per round on a ~20
// cycle dependency chain, against ~130 scalar ops (and register spills) for
// the unrolled 64-bit version.
__attribute__((target("avx512f"))) void keccakf_x1_avx512(uint64_t s[25]) {
    __m512i P0 = _mm512_maskz_loadu_epi64(0x1f, s), P1 = _mm512_maskz_loadu_epi64(0x1f, s + 5);
    __m512i P2 = _mm512_maskz_loadu_epi64(0x1f, s + 10), P3 = _mm512_maskz_loadu_epi64(0x1f, s + 15);
    __m512i P4 = _mm512_maskz_loadu_epi64(0x1f, s + 20);
    const __m512i M1 = _mm512_setr_epi64(4, 0, 1, 2, 3, 5, 6, 7);   // lane x <- x - 1
    const __m512i P1i = _mm512_setr_epi64(1, 2, 3, 4, 0, 5, 6, 7);  // lane x <- x + 1
    const __m512i P2i = _mm512_setr_epi64(2, 3, 4, 0, 1, 5, 6, 7);  // lane x <- x + 2
    // rho offsets of the lanes of each plane
    const __m512i R0 = _mm512_setr_epi64(0, 1, 62, 28, 27, 0, 0, 0), R1 = _mm512_setr_epi64(36, 44, 6, 55, 20, 0, 0, 0);
    const __m512i R2 = _mm512_setr_epi64(3, 10, 43, 25, 39, 0, 0, 0), R3 = _mm512_setr_epi64(41, 45, 15, 21, 8, 0, 0, 0);
    const __m512i R4 = _mm512_setr_epi64(18, 2, 61, 56, 14, 0, 0, 0);
    // pi: Q_X[k] = P_X[(k + X) mod 5]; output plane Y = column 3Y mod 5 of Q.
    // E01 = (Q0[k], Q1[k]) for k < 4, F01 the k = 4 pair (b-source lanes + 8)
    const __m512i IE01 = _mm512_setr_epi64(0, 9, 1, 10, 2, 11, 3, 12), IF01 = _mm512_setr_epi64(4, 8, 0, 0, 0, 0, 0, 0);
    const __m512i IE23 = _mm512_setr_epi64(2, 11, 3, 12, 4, 8, 0, 9), IF23 = _mm512_setr_epi64(1, 10, 0, 0, 0, 0, 0, 0);
    const __m512i IO0 = _mm512_setr_epi64(0, 1, 8, 9, 0, 0, 0, 0), IO1 = _mm512_setr_epi64(2, 3, 10, 11, 0, 0, 0, 0);
    const __m512i IO2 = _mm512_setr_epi64(4, 5, 12, 13, 0, 0, 0, 0), IO3 = _mm512_setr_epi64(6, 7, 14, 15, 0, 0, 0, 0);
    // lane 4 of column k: Q4[k] = P4[(k + 4) mod 5]
    const __m512i IQ0 = _mm512_set1_epi64(4), IQ1 = _mm512_set1_epi64(0), IQ2 = _mm512_set1_epi64(1);
    const __m512i IQ3 = _mm512_set1_epi64(2), IQ4 = _mm512_set1_epi64(3);
    for (int r = 0; r < 24; r++) {
        // theta
        __m512i C = _mm512_ternarylogic_epi64(P0, P1, P2, 0x96);
        C = _mm512_ternarylogic_epi64(C, P3, P4, 0x96);
        const __m512i Cm = _mm512_permutexvar_epi64(M1, C);
        const __m512i Cr = _mm512_rol_epi64(_mm512_permutexvar_epi64(P1i, C), 1);
        // theta's D, then rho
        P0 = _mm512_rolv_epi64(_mm512_ternarylogic_epi64(P0, Cm, Cr, 0x96), R0);
        P1 = _mm512_rolv_epi64(_mm512_ternarylogic_epi64(P1, Cm, Cr, 0x96), R1);
        P2 = _mm512_rolv_epi64(_mm512_ternarylogic_epi64(P2, Cm, Cr, 0x96), R2);
        P3 = _mm512_rolv_epi64(_mm512_ternarylogic_epi64(P3, Cm, Cr, 0x96), R3);
        P4 = _mm512_rolv_epi64(_mm512_ternarylogic_epi64(P4, Cm, Cr, 0x96), R4);
        // pi
        const __m512i E01 = _mm512_permutex2var_epi64(P0, IE01, P1), F01 = _mm512_permutex2var_epi64(P0, IF01, P1);
        const __m512i E23 = _mm512_permutex2var_epi64(P2, IE23, P3), F23 = _mm512_permutex2var_epi64(P2, IF23, P3);
        const __m512i O0 = _mm512_mask_blend_epi64(0x10, _mm512_permutex2var_epi64(E01, IO0, E23), _mm512_permutexvar_epi64(IQ0, P4));
        const __m512i O1 = _mm512_mask_blend_epi64(0x10, _mm512_permutex2var_epi64(E01, IO1, E23), _mm512_permutexvar_epi64(IQ1, P4));
        const __m512i O2 = _mm512_mask_blend_epi64(0x10, _mm512_permutex2var_epi64(E01, IO2, E23), _mm512_permutexvar_epi64(IQ2, P4));
        const __m512i O3 = _mm512_mask_blend_epi64(0x10, _mm512_permutex2var_epi64(E01, IO3, E23), _mm512_permutexvar_epi64(IQ3, P4));
        const __m512i O4 = _mm512_mask_blend_epi64(0x10, _mm512_permutex2var_epi64(F01, IO0, F23), _mm512_permutexvar_epi64(IQ4, P4));
        // B_Y = O_{3Y mod 5}, then chi: A[x] = B[x] ^ (~B[x+1] & B[x+2]), iota
        P0 = _mm512_ternarylogic_epi64(O0, _mm512_permutexvar_epi64(P1i, O0), _mm512_permutexvar_epi64(P2i, O0), 0xD2);
        P1 = _mm512_ternarylogic_epi64(O3, _mm512_permutexvar_epi64(P1i, O3), _mm512_permutexvar_epi64(P2i, O3), 0xD2);
        P2 = _mm512_ternarylogic_epi64(O1, _mm512_permutexvar_epi64(P1i, O1), _mm512_permutexvar_epi64(P2i, O1), 0xD2);
        P3 = _mm512_ternarylogic_epi64(O4, _mm512_permutexvar_epi64(P1i, O4), _mm512_permutexvar_epi64(P2i, O4), 0xD2);
        P4 = _mm512_ternarylogic_epi64(O2, _mm512_permutexvar_epi64(P1i, O2), _mm512_permutexvar_epi64(P2i, O2), 0xD2);
        P0 = _mm512_xor_si512(P0, _mm512_maskz_set1_epi64(1, (long long)RC8[r]));
    }
    _mm512_mask_storeu_epi64(s, 0x1f, P0);
    _mm512_mask_storeu_epi64(s + 5, 0x1f, P1);
    _mm512_mask_storeu_epi64(s + 10, 0x1f, P2);
    _mm512_mask_storeu_epi64(s + 15, 0x1f, P3);
    _mm512_mask_storeu_epi64(s + 20, 0x1f, P4);
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
    if (nstates == 1) {   // single proof (latency path): one state, not eight
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
    if (pos == 64 && pos_begin == 0) {
        // after another 64-byte draw the framing is constant
        // (TranscriptRng::draw64): three words of every state, the
        // permutation, then the 64 output bytes out and zeroed
        for (int s = 0; s < 8; s++) { L[8][s] ^= DRAW64_W8; L[9][s] ^= DRAW64_W9; L[20][s] ^= DRAW64_W20; }
        if (nstates == 1) {
            uint64_t st[25];
            for (int i = 0; i < 25; i++) st[i] = L[i][0];
            keccakf(st);
            for (int i = 0; i < 25; i++) L[i][0] = st[i];
        } else {
            keccak8(L);
        }
        for (int s = 0; s < nstates; s++) {
            uint64_t *o = reinterpret_cast<uint64_t *>(out[s]);
            for (int k = 0; k < 8; k++) o[k] = L[k][s];
        }
        memset(L, 0, 8 * sizeof(L[0]));
        cur_flags = S8_I | S8_A | S8_C;
        return;
    }
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
