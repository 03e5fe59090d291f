// rng_bench.cpp — host RNG rates on the machine it runs on (the GPU box's
// CPU decides single-proof latency and producer throughput): Keccak-f[1600]
// scalar vs the AVX-512 single-state form, the eight-state form, and the
// TranscriptRng / Strobe8 64-byte draws built on them.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../host/hcrypto.h"
#include "../host/rng8.h"

using namespace bpg;
template <class F> static double ns_per(int n, F f) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) f();
    return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / n;
}
int main() {
    const int N = 1000000;
    uint64_t a[25] = {1}, b[25] = {1};
    alignas(64) static uint64_t L[25][8];
    printf("avx512: %d\n", (int)have_avx512());
    printf("keccakf scalar      %7.1f ns\n", ns_per(N, [&] { keccakf_scalar(a); }));
    if (have_avx512()) printf("keccakf avx512 x1   %7.1f ns\n", ns_per(N, [&] { keccakf_x1_avx512(b); }));
    printf("keccak8 (8 states)  %7.1f ns\n", ns_per(N / 4, [&] { keccak8(L); }));
    Transcript T((const uint8_t *)"rate", 4);
    TranscriptRng base(T);
    uint8_t ent[32] = {1}, out[8][64];
    TranscriptRng r(base);
    r.finalize(ent);
    printf("TranscriptRng fill_bytes(64) %7.1f ns\n", ns_per(N, [&] { r.fill_bytes(out[0], 64); }));
    printf("TranscriptRng draw64         %7.1f ns\n", ns_per(N, [&] { r.draw64(out[0]); }));
    for (int lanes : {1, 8}) {
        Strobe8 S;
        S.from(base.s, lanes);
        const uint8_t *ep[8] = {ent, ent, ent, ent, ent, ent, ent, ent};
        S.meta_ad((const uint8_t *)"rng", 3);
        S.key_each(ep, 32);
        uint8_t *op[8];
        for (int k = 0; k < 8; k++) op[k] = out[k];
        printf("Strobe8 draw64, %d lanes       %7.1f ns per step\n", lanes, ns_per(N / 4, [&] { S.draw64(op); }));
    }
    return 0;
}
