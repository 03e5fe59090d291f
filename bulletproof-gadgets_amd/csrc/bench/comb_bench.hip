// comb_bench.hip — the table fold of IPP rounds 0-1 (k_comb_build +
// k_ipp_comb_fold) in isolation: build tables for generators [h1, 4 h1),
// fold with random coefficients in two lane ranges, check sampled lanes
// against host arithmetic, time per launch.
#include "../device/kernels.hip"
#include "../host/hcrypto.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
using namespace bpg::dev;
int main(int argc, char **argv) {
    uint32_t h1 = argc > 1 ? atoi(argv[1]) : (1u << 17);
    const uint32_t N = 4 * h1, ntab = 3 * h1;
    std::vector<uint8_t> uni((size_t)N * 64);
    srand(3);
    for (auto &b : uni) b = rand() & 255;
    uint8_t *duni; NielsD *G; PtD *Go, *Ho;
    BPG_HIP(hipMalloc(&duni, uni.size()));
    BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
    BPG_HIP(hipMalloc(&G, (size_t)N * sizeof(NielsD)));
    BPG_HIP(hipMalloc(&Go, (size_t)h1 * sizeof(PtD))); BPG_HIP(hipMalloc(&Ho, (size_t)h1 * sizeof(PtD)));
    launch_gens_map(duni, G, N, 0);
    void *tab;
    const size_t tbytes = (size_t)ntab * COMB_WIN * COMB_ENT * 96;
    BPG_HIP(hipMalloc(&tab, tbytes));
    hipEvent_t e0, e1; BPG_HIP(hipEventCreate(&e0)); BPG_HIP(hipEventCreate(&e1));
    BPG_HIP(hipDeviceSynchronize());
    BPG_HIP(hipEventRecord(e0, 0));
    launch_comb_build(G, h1, ntab, tab, 0);
    BPG_HIP(hipEventRecord(e1, 0));
    BPG_HIP(hipEventSynchronize(e1));
    float ms;
    BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
    printf("comb build: %u generators, %.2f GB, %.1f ms (%.1f GB/s)\n", ntab, tbytes / 1e9, ms, tbytes / ms / 1e6);
    // coefficients: two ranges per vector (G and H use the same points here)
    bpg::Scalar co[2][2][3];
    for (auto &a : co) for (auto &b : a) for (auto &c : b) {
        uint8_t w[64]; for (auto &x : w) x = rand() & 255; c = bpg::Scalar::from_wide(w);
    }
    CombArgs C{};
    C.gens[0] = G; C.gens[1] = G; C.tab[0] = tab; C.tab[1] = tab; C.out[0] = Go; C.out[1] = Ho;
    C.h1 = h1; C.ntab = ntab; C.nrange = 2; C.rstart[0] = 0; C.rstart[1] = h1 / 3;
    for (int v = 0; v < 2; v++) for (int r = 0; r < 2; r++) for (int t = 0; t < 3; t++) { uint8_t sb[32]; co[v][r][t].reduced().to_bytes(sb); comb_digits(sb, C.dig[v][r][t]); }
    ArgStage stage;
    hipStream_t st; BPG_HIP(hipStreamCreate(&st));
    launch_ipp_comb_fold(C, stage, st);
    BPG_HIP(hipStreamSynchronize(st));
    const int reps = 3;
    BPG_HIP(hipEventRecord(e0, st));
    for (int k = 0; k < reps; k++) launch_ipp_comb_fold(C, stage, st);
    BPG_HIP(hipEventRecord(e1, st));
    BPG_HIP(hipEventSynchronize(e1));
    BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
    double per = ms / reps;
    double bytes = 2.0 * h1 * (4 * 64 + 64);
    printf("comb fold h1=%u: %.3f ms per launch (%.2f ns/lane, %.1f GB/s algorithmic, %.1f GB/s table reads)\n", h1, per,
           per * 1e6 / (2.0 * h1), bytes / per / 1e6, 2.0 * h1 * 3 * 60 * 96 / per / 1e6);
    // check
    std::vector<uint32_t> cin((size_t)N * 8), cout_((size_t)2 * h1 * 8);
    uint32_t *dcin, *dcout;
    BPG_HIP(hipMalloc(&dcin, cin.size() * 4)); BPG_HIP(hipMalloc(&dcout, cout_.size() * 4));
    launch_compress(G, dcin, N, st);
    launch_compress(Go, dcout, h1, st); launch_compress(Ho, dcout + (size_t)8 * h1, h1, st);
    BPG_HIP(hipMemcpyAsync(cin.data(), dcin, cin.size() * 4, hipMemcpyDeviceToHost, st));
    BPG_HIP(hipMemcpyAsync(cout_.data(), dcout, cout_.size() * 4, hipMemcpyDeviceToHost, st));
    BPG_HIP(hipStreamSynchronize(st));
    int bad = 0, checked = 0;
    uint32_t lanes[] = {0, 1, 63, 64, h1 / 3 - 1, h1 / 3, h1 / 2, h1 - 1};
    for (int v = 0; v < 2; v++)
        for (uint32_t i : lanes) {
            int r = i >= h1 / 3 ? 1 : 0;
            bpg::Point acc, P, t;
            bpg::ristretto_decompress(acc, (const uint8_t *)&cin[(size_t)i * 8]);
            for (int k = 0; k < 3; k++) {
                bpg::ristretto_decompress(P, (const uint8_t *)&cin[(size_t)(i + (k + 1) * h1) * 8]);
                bpg::mul_var(t, co[v][r][k], P);
                bpg::pt_add(acc, acc, t);
            }
            uint8_t wb[32]; bpg::ristretto_compress(wb, acc);
            checked++;
            if (memcmp(wb, &cout_[((size_t)v * h1 + i) * 8], 32)) bad++;
        }
    printf("comb fold check: %d/%d lanes bad\n", bad, checked);
    return bad ? 1 : 0;
}
