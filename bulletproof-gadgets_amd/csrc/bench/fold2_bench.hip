// fold2_bench.hip — isolated timing of the two-round Straus fold
// (k_ipp_fold2) at the config-5 level-2 -> level-4 size (h1 = 2^16 output
// lanes per vector), level-0 (Niels) and cached inputs, with sampled lanes
// checked against host arithmetic: out_i = P_i + c1 P_{i+h1} + c2 P_{i+2h1}
// + c3 P_{i+3h1}.
#include "../device/kernels.hip"
#include "../host/hcrypto.h"
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
using namespace bpg::dev;

static int check(const std::vector<uint32_t> &cin, const std::vector<uint32_t> &cout_, uint32_t h1,
                 const ScD (*coef)[COMB_MAXRANGE][3]) {
    int bad = 0;
    uint32_t lanes[] = {0, 1, 63, 64, 65, h1 / 3, h1 / 2 + 7, h1 - 1};
    for (int v = 0; v < 2; v++)
        for (uint32_t i : lanes) {
            bpg::Point acc, P, t;
            const uint8_t *p0 = (const uint8_t *)&cin[((size_t)v * 4 * h1 + i) * 8];
            bpg::ristretto_decompress(acc, p0);
            for (int k = 1; k < 4; k++) {
                bpg::ristretto_decompress(P, (const uint8_t *)&cin[((size_t)v * 4 * h1 + k * h1 + i) * 8]);
                bpg::Scalar s; memcpy(s.v, coef[v][0][k - 1].v, 32);
                bpg::mul_var(t, s, P);
                bpg::pt_add(acc, acc, t);
            }
            uint8_t wb[32];
            bpg::ristretto_compress(wb, acc);
            if (memcmp(wb, &cout_[((size_t)v * h1 + i) * 8], 32)) bad++;
        }
    return bad;
}

int main(int argc, char **argv) {
    const uint32_t h1 = argc > 1 ? atoi(argv[1]) : (1u << 16);
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<uint8_t> uni((size_t)4 * h1 * 64);
    srand(7);
    for (auto &b : uni) b = rand() & 255;
    uint8_t *duni; NielsD *G, *H; PtD *Gc, *Hc, *Go, *Ho;
    BPG_HIP(hipMalloc(&duni, uni.size()));
    BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
    BPG_HIP(hipMalloc(&G, (size_t)4 * h1 * sizeof(NielsD))); BPG_HIP(hipMalloc(&H, (size_t)4 * h1 * sizeof(NielsD)));
    BPG_HIP(hipMalloc(&Gc, (size_t)4 * h1 * sizeof(PtD))); BPG_HIP(hipMalloc(&Hc, (size_t)4 * h1 * sizeof(PtD)));
    BPG_HIP(hipMalloc(&Go, (size_t)h1 * sizeof(PtD))); BPG_HIP(hipMalloc(&Ho, (size_t)h1 * sizeof(PtD)));
    launch_gens_map(duni, G, 4 * h1, 0);
    for (auto &b : uni) b = rand() & 255;
    BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
    launch_gens_map(duni, H, 4 * h1, 0);
    BPG_HIP(hipDeviceSynchronize());
    hipStream_t st; BPG_HIP(hipStreamCreate(&st));
    ScD coef[2][COMB_MAXRANGE][3];
    for (int v = 0; v < 2; v++)
        for (int t = 0; t < 3; t++) {
            for (int i = 0; i < 8; i++) coef[v][0][t].v[i] = rand() * 2654435761u + rand();
            coef[v][0][t].v[7] &= 0x0fffffff;
        }
    const uint32_t rstart[1] = {0};
    ArgStage stage;
    // cached inputs: the identity-weighted fold of the Niels inputs (c = 0 -> P)
    ScD zero[2][COMB_MAXRANGE][3] = {};
    launch_ipp_fold2(G, H, MSM_NIELS, 4 * h1, 1, rstart, zero, Gc, Hc, stage, st);
    std::vector<uint32_t> cin((size_t)8 * h1 * 8), cout_((size_t)2 * h1 * 8);
    uint32_t *dcin, *dcout;
    BPG_HIP(hipMalloc(&dcin, cin.size() * 4)); BPG_HIP(hipMalloc(&dcout, cout_.size() * 4));
    launch_compress(G, dcin, 4 * h1, st); launch_compress(H, dcin + (size_t)32 * h1, 4 * h1, st);
    BPG_HIP(hipMemcpyAsync(cin.data(), dcin, cin.size() * 4, hipMemcpyDeviceToHost, st));
    BPG_HIP(hipStreamSynchronize(st));
    hipEvent_t e0, e1; BPG_HIP(hipEventCreate(&e0)); BPG_HIP(hipEventCreate(&e1));
    for (int fmt = 0; fmt < 2; fmt++) {
        const void *gi = fmt ? (const void *)G : (const void *)Gc, *hi = fmt ? (const void *)H : (const void *)Hc;
        const int in_fmt = fmt ? MSM_NIELS : MSM_CACHED;
        launch_ipp_fold2(gi, hi, in_fmt, h1, 1, rstart, coef, Go, Ho, stage, st);
        BPG_HIP(hipStreamSynchronize(st));
        BPG_HIP(hipEventRecord(e0, st));
        for (int k = 0; k < reps; k++) launch_ipp_fold2(gi, hi, in_fmt, h1, 1, rstart, coef, Go, Ho, stage, st);
        BPG_HIP(hipEventRecord(e1, st));
        BPG_HIP(hipEventSynchronize(e1));
        float ms;
        BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
        launch_compress(Go, dcout, h1, st); launch_compress(Ho, dcout + (size_t)8 * h1, h1, st);
        BPG_HIP(hipMemcpyAsync(cout_.data(), dcout, cout_.size() * 4, hipMemcpyDeviceToHost, st));
        BPG_HIP(hipStreamSynchronize(st));
        const int bad = check(cin, cout_, h1, coef);
        printf("fold2 %s inputs h1=%u: %.3f ms per launch (%.2f ns per output lane); check: %d of 16 lanes bad\n",
               fmt ? "niels" : "cached", h1, ms / reps, ms / reps * 1e6 / (2.0 * h1), bad);
    }
    return 0;
}
