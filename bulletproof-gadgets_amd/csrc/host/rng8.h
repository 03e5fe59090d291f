// rng8.h — TranscriptRng (merlin@2.0.1 transcript.rs TranscriptRng, STROBE-128
// prf draws) for up to 8 proofs of the same statement in lockstep.
//
// Proofs of one prepared circuit share the transcript prefix and the
// witness rekeying, so their STROBE states differ only in the finalize
// entropy and every state sits at the same byte position at every step.
// The 8 Keccak-f[1600] states are stored lane-interleaved (L[lane][state])
// and permuted together with AVX-512 (vprolq / vpternlogq); without
// AVX-512 the same layout is permuted state by state. Each draw is exactly
// what TranscriptRng::fill_bytes(64) does per state: meta_ad(u32le(64)),
// prf(64) -> one permutation, 64 bytes out.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "hcrypto.h"

namespace bpg {

struct Strobe8 {
    alignas(64) uint64_t L[25][8];
    uint8_t pos, pos_begin, cur_flags;
    int nstates;
    void from(const Strobe128 &s, int n);              // n copies of one state
    // n distinct states (proofs of different statements) that sit at the same
    // byte position and operation (true after any draw: its prf permutes
    // first, so every state ends at pos 64); false if they do not
    bool from_each(const Strobe128 *const *s, int n);
    void meta_ad(const uint8_t *d, size_t len);        // same data for every state
    void key_each(const uint8_t *const *d, size_t len);  // per-state key material
    // TranscriptRng::fill_bytes(64) on every state; out[s] receives 64 bytes
    void draw64(uint8_t *const *out);
  private:
    void run_f();
    void begin_op(uint8_t flags);
    void absorb_same(const uint8_t *d, size_t len);
    uint8_t &byte(int s, unsigned p) { return reinterpret_cast<uint8_t *>(&L[p >> 3][s])[p & 7]; }
};

void keccak8(uint64_t L[25][8]);
// Keccak-f[1600] of one state with AVX-512 (call only when have_avx512())
void keccakf_x1_avx512(uint64_t s[25]);
bool have_avx512();

}  // namespace bpg
