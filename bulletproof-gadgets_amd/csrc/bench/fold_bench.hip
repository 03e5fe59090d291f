// fold_bench.hip — isolated timing of the IPP point fold (k_ipp_fold_points)
// and one MSM job at the config-5 round-0 size, for occupancy/variant
// experiments. Points come from the generator map on random bytes.
#include "../device/kernels.hip"
#include "../host/hcrypto.h"
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
using namespace bpg::dev;
int main(int argc, char **argv) {
    uint32_t h = argc > 1 ? atoi(argv[1]) : (1u << 19);
    uint32_t n = argc > 2 ? atoi(argv[2]) : 744712 / 2;
    std::vector<uint8_t> uni((size_t)2 * h * 64);
    srand(1);
    for (auto &b : uni) b = rand() & 255;
    uint8_t *duni; NielsD *G, *H; PtD *Go, *Ho;
    BPG_HIP(hipMalloc(&duni, uni.size()));
    BPG_HIP(hipMemcpy(duni, uni.data(), uni.size(), hipMemcpyHostToDevice));
    BPG_HIP(hipMalloc(&G, (size_t)2 * h * sizeof(NielsD))); BPG_HIP(hipMalloc(&H, (size_t)2 * h * sizeof(NielsD)));
    BPG_HIP(hipMalloc(&Go, (size_t)h * sizeof(PtD))); BPG_HIP(hipMalloc(&Ho, (size_t)h * sizeof(PtD)));
    launch_gens_map(duni, G, 2 * h, 0);
    launch_gens_map(duni, H, 2 * h, 0);
    BPG_HIP(hipDeviceSynchronize());
    ScD r[4];
    for (int k = 0; k < 4; k++) { for (int i = 0; i < 8; i++) r[k].v[i] = rand() * 2654435761u; r[k].v[7] &= 0x0fffffff; }
    ArgStage stage;
    hipStream_t st; BPG_HIP(hipStreamCreate(&st));
    hipEvent_t e0, e1; BPG_HIP(hipEventCreate(&e0)); BPG_HIP(hipEventCreate(&e1));
    const int reps = 3;
    float ms;
    std::vector<uint32_t> cin((size_t)4 * h * 8), cout_((size_t)2 * h * 8);
    uint32_t *dcin, *dcout;
    BPG_HIP(hipMalloc(&dcin, cin.size() * 4)); BPG_HIP(hipMalloc(&dcout, cout_.size() * 4));
    launch_compress(G, dcin, 2 * h, st); launch_compress(H, dcin + (size_t)16 * h, 2 * h, st);
    BPG_HIP(hipMemcpyAsync(cin.data(), dcin, cin.size() * 4, hipMemcpyDeviceToHost, st));
    BPG_HIP(hipStreamSynchronize(st));
    uint32_t ns[4] = {n, 744712, h, 2 * h};
    for (uint32_t nn : ns) {
        launch_ipp_fold_points(G, H, MSM_NIELS, h, nn, r[0], r[1], r[2], r[3], Go, Ho, stage, st);
        BPG_HIP(hipStreamSynchronize(st));
        BPG_HIP(hipEventRecord(e0, st));
        for (int k = 0; k < reps; k++) launch_ipp_fold_points(G, H, MSM_NIELS, h, nn, r[0], r[1], r[2], r[3], Go, Ho, stage, st);
        BPG_HIP(hipEventRecord(e1, st));
        BPG_HIP(hipEventSynchronize(e1));
        BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
        // check sampled lanes against host arithmetic
        launch_compress(Go, dcout, h, st); launch_compress(Ho, dcout + (size_t)8 * h, h, st);
        BPG_HIP(hipMemcpyAsync(cout_.data(), dcout, cout_.size() * 4, hipMemcpyDeviceToHost, st));
        BPG_HIP(hipStreamSynchronize(st));
        int bad = 0, checked = 0;
        const uint32_t a = nn > h ? std::min(nn - h, h) : 0, bnd = std::min(nn, h);
        uint32_t lanes[] = {0, 1, 63, 64, a ? a - 1 : 0, a, a + 1, bnd ? bnd - 1 : 0, bnd < h ? bnd : 0, h - 1, h / 3};
        for (int v = 0; v < 2; v++)
            for (uint32_t i : lanes) {
                if (i >= h) continue;
                bool special = i >= a && i < bnd;
                const ScD &rho = r[2 * v + (special ? 1 : 0)];
                bpg::Point PL, PR, t, want;
                const uint8_t *pl = (const uint8_t *)&cin[((size_t)v * 2 * h + i) * 8];
                const uint8_t *pr = (const uint8_t *)&cin[((size_t)v * 2 * h + h + i) * 8];
                bpg::ristretto_decompress(PL, pl); bpg::ristretto_decompress(PR, pr);
                bpg::Scalar sr; memcpy(sr.v, rho.v, 32);
                bpg::mul_var(t, sr, PR); bpg::pt_add(want, PL, t);
                uint8_t wb[32]; bpg::ristretto_compress(wb, want);
                checked++;
                if (memcmp(wb, &cout_[((size_t)v * h + i) * 8], 32)) bad++;
            }
        printf("fold h=%u n=%u: %.3f ms per launch (%.2f ns/lane); check %d/%d lanes bad\n", h, nn, ms / reps,
               ms / reps * 1e6 / (2.0 * h), bad, checked);
    }
    // one MSM job: 4 segments of h points (round-0 L/R shape)
    std::vector<ScD> sc((size_t)4 * h);
    for (auto &s : sc) { for (int i = 0; i < 8; i++) s.v[i] = rand() * 2654435761u + rand(); s.v[7] &= 0x0fffffff; }
    ScD *dsc; BPG_HIP(hipMalloc(&dsc, sc.size() * sizeof(ScD)));
    BPG_HIP(hipMemcpy(dsc, sc.data(), sc.size() * sizeof(ScD), hipMemcpyHostToDevice));
    MsmEngine eng(st);
    PtD *rows; BPG_HIP(hipHostMalloc((void **)&rows, 128 * sizeof(PtD), hipHostMallocDefault));
    MsmSeg seg[4] = {{dsc, G + h, h, 0}, {dsc + h, H, h, 0}, {dsc + 2 * (size_t)h, G, h, 1}, {dsc + 3 * (size_t)h, H + h, h, 1}};
    eng.enqueue(seg, 4, 2, rows, MSM_NIELS);
    BPG_HIP(hipStreamSynchronize(st));
    BPG_HIP(hipEventRecord(e0, st));
    for (int k = 0; k < reps; k++) eng.enqueue(seg, 4, 2, rows, MSM_NIELS);
    BPG_HIP(hipEventRecord(e1, st));
    BPG_HIP(hipEventSynchronize(e1));
    BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
    printf("msm job 4h=%u points (Niels bases): %.3f ms per job\n", 4 * h, ms / reps);
    // cached bases (folded generators), round-2 shape: 4 x h/4 points
    const uint32_t q = h / 4;
    MsmSeg segc[4] = {{dsc, Go + q, q, 0}, {dsc + q, Ho, q, 0}, {dsc + 2 * (size_t)q, Go, q, 1}, {dsc + 3 * (size_t)q, Ho + q, q, 1}};
    eng.enqueue(segc, 4, 2, rows, MSM_CACHED);
    BPG_HIP(hipStreamSynchronize(st));
    BPG_HIP(hipEventRecord(e0, st));
    for (int k = 0; k < reps; k++) eng.enqueue(segc, 4, 2, rows, MSM_CACHED);
    BPG_HIP(hipEventRecord(e1, st));
    BPG_HIP(hipEventSynchronize(e1));
    BPG_HIP(hipEventElapsedTime(&ms, e0, e1));
    printf("msm job 4q=%u points (cached bases): %.3f ms per job\n", 4 * q, ms / reps);
    return 0;
}
