// fold3_bench.hip — isolated timing of the three-round Straus fold
// (k_ipp_fold3) at the config-5 level-2 -> level-5 size (hq = 2^15 output
// lanes per vector), cached inputs, with sampled lanes checked against host
// arithmetic: out_i = P_i + sum_{t=1..7} c_t P_{i + t hq}.
#include "../device/kernels.hip"
#include "../host/hcrypto.h"
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
using namespace bpg::dev;

static int check(const std::vector<uint32_t> &cin, const std::vector<uint32_t> &cout_, uint32_t hq,
                 const ScD (*coef)[COMB_MAXRANGE][7]) {
    int bad = 0;
    uint32_t lanes[] = {0, 1, 63, 64, 65, hq / 3, hq / 2 + 7, hq - 1};
    for (int v = 0; v < 2; v++)
        for (uint32_t i : lanes) {
            bpg::Point acc, P, t;
            bpg::ristretto_decompress(acc, (const uint8_t *)&cin[((size_t)v * 8 * hq + i) * 8]);
            for (int k = 1; k < 8; k++) {
                bpg::ristretto_decompress(P, (const uint8_t *)&cin[((size_t)v * 8 * hq + k * hq + i) * 8]);
                bpg::Scalar s; memcpy(s.v, coef[v][0][k - 1].v, 32);
                bpg::mul_var(t, s, P);
                bpg::pt_add(acc, acc, t);
            }
            uint8_t wb[32];
            bpg::ristretto_compress(wb, acc);
            if (memcmp(wb, &cout_[((size_t)v * hq + i) * 8], 32)) bad++;
        }
    return bad;
}

int main(int argc, char **argv) {
    const uint32_t hq = argc > 1 ? atoi(argv[1]) : (1u << 15);
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<uint8_t> uni((size_t)8 * hq * 64);
    srand(11);
    for (auto &b : uni) b = rand() & 255;
    uint8_t *duni; NielsD *G, *H; PtD *Gc, *Hc, *Go, *Ho;
    BPG_HIP(hipMalloc(&duni, uni.size()));
    BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
    BPG_HIP(hipMalloc(&G, (size_t)8 * hq * sizeof(NielsD))); BPG_HIP(hipMalloc(&H, (size_t)8 * hq * sizeof(NielsD)));
    BPG_HIP(hipMalloc(&Gc, (size_t)8 * hq * sizeof(PtD))); BPG_HIP(hipMalloc(&Hc, (size_t)8 * hq * sizeof(PtD)));
    BPG_HIP(hipMalloc(&Go, (size_t)hq * sizeof(PtD))); BPG_HIP(hipMalloc(&Ho, (size_t)hq * sizeof(PtD)));
    launch_gens_map(duni, G, 8 * hq, 0);
    for (auto &b : uni) b = rand() & 255;
    BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
    launch_gens_map(duni, H, 8 * hq, 0);
    BPG_HIP(hipDeviceSynchronize());
    hipStream_t st; BPG_HIP(hipStreamCreate(&st));
    ScD coef[2][COMB_MAXRANGE][7];
    for (int v = 0; v < 2; v++)
        for (int t = 0; t < 7; t++) {
            for (int i = 0; i < 8; i++) coef[v][0][t].v[i] = rand() * 2654435761u + rand();
            coef[v][0][t].v[7] &= 0x0fffffff;
        }
    const uint32_t rstart[1] = {0};
    ArgStage stage, stage3;
    ScD zero[2][COMB_MAXRANGE][3] = {};
    launch_ipp_fold2(G, H, MSM_NIELS, 8 * hq, 1, rstart, zero, Gc, Hc, stage, st);   // cached copies
    std::vector<uint32_t> cin((size_t)16 * hq * 8), cout_((size_t)2 * hq * 8);
    uint32_t *dcin, *dcout;
    BPG_HIP(hipMalloc(&dcin, cin.size() * 4)); BPG_HIP(hipMalloc(&dcout, cout_.size() * 4));
    launch_compress(G, dcin, 8 * hq, st); launch_compress(H, dcin + (size_t)64 * hq, 8 * hq, st);
    BPG_HIP(hipMemcpyAsync(cin.data(), dcin, cin.size() * 4, hipMemcpyDeviceToHost, st));
    BPG_HIP(hipStreamSynchronize(st));
    const size_t tb = ipp_fold3_table_bytes(hq, 1);
    void *tab; BPG_HIP(hipMalloc(&tab, tb));
    hipEvent_t e0, e1; BPG_HIP(hipEventCreate(&e0)); BPG_HIP(hipEventCreate(&e1));
    const void *gin[1] = {Gc}, *hin[1] = {Hc};
    PtD *gout[1] = {Go}, *hout[1] = {Ho};
    const ScD (*cp[1])[COMB_MAXRANGE][7] = {coef};
    launch_ipp_fold3(gin, hin, MSM_CACHED, hq, 1, rstart, cp, gout, hout, 1, tab, tb, stage3, st);
    BPG_HIP(hipStreamSynchronize(st));
    BPG_HIP(hipEventRecord(e0, st));
    for (int k = 0; k < reps; k++) launch_ipp_fold3(gin, hin, MSM_CACHED, hq, 1, rstart, cp, gout, hout, 1, tab, tb, stage3, st);
    BPG_HIP(hipEventRecord(e1, st));
    BPG_HIP(hipEventSynchronize(e1));
    float ms;
    BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
    launch_compress(Go, dcout, hq, st); launch_compress(Ho, dcout + (size_t)8 * hq, hq, st);
    BPG_HIP(hipMemcpyAsync(cout_.data(), dcout, cout_.size() * 4, hipMemcpyDeviceToHost, st));
    BPG_HIP(hipStreamSynchronize(st));
    const int bad = check(cin, cout_, hq, coef);
    printf("fold3 cached inputs hq=%u: %.3f ms per launch (%.2f ns per output lane); check: %d of 16 lanes bad\n", hq,
           ms / reps, ms / reps * 1e6 / (2.0 * hq), bad);
    return bad ? 1 : 0;
}
