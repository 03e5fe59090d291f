// affine_bench.hip — does batch-affine bucket accumulation pay on gfx950?
// (MSM pass 1 adds every entry to its bucket with the 7M
// mixed Edwards addition, ge_madd.)
//
// Batch-affine accumulation (affine Montgomery / short-Weierstrass
// coordinates: lambda = (y2 - y1) / (x2 - x1), x3 = lambda^2 - A - x1 - x2,
// y3 = lambda (x1 - x3) - y1) costs 2M + 1S per addition plus the inversion,
// which Montgomery's trick shares over a batch of B INDEPENDENT additions
// (3M each: prefix product, and two on the way back) -- on a SIMD machine per
// lane: every lane pays its own inversion, so the batch must be B additions
// of one lane, B different buckets, with B prefix products and B bucket
// states live at once.
//
// This program measures, on the whole chip:
//   madd   ge_madd into a register accumulator, the point read from HBM
//          (what pass 1 does per entry)
//   mul/sq fe_mul, fe_sq chains (the unit costs)
//   inv    fe_invert
//   aff<B> batch-affine additions, B buckets per lane: bucket states
//          (x1, y1) and the prefix products in global memory (lane-
//          interleaved, coalesced), the added points read from HBM
// and prints additions per second for each and the break-even batch.
// The arithmetic is GF(2^255 - 19) with dev_field.h's field; the affine
// curve formulas are exercised on synthetic coordinates (no exceptional
// cases are handled: a real implementation would need x1 == x2 checks on
// top, so these figures are an upper bound for batch-affine).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "../device/dev_field.h"

#define CHK(x)                                                                           \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);                    \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

static const int TPB = 256;
// the point table read by every kernel: NPTS affine Niels points, reused
// modulo NPTS (large enough to come from HBM / the Infinity Cache, like the
// generator gathers of pass 1)
static const uint32_t NPTS = 1u << 21;

__global__ __launch_bounds__(TPB) void k_madd(const gen *__restrict__ pts, ge *__restrict__ out, int R) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    ge acc;
    ge_identity(acc);
    uint32_t idx = tid * 2654435761u;
    for (int r = 0; r < R; r++) {
        gen q;
        gen_load(q, pts + (idx % NPTS));
        ge_madd(acc, acc, q);
        idx = idx * 1664525u + 1013904223u;
    }
    ge_store(out + tid, acc);
}

__global__ __launch_bounds__(TPB) void k_mul(const fe *__restrict__ in, fe *__restrict__ out, int R, int sq) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    fe x = in[tid % 4096], y = in[(tid + 1) % 4096], u = in[(tid + 2) % 4096];
    for (int r = 0; r < R; r++) {
        if (sq) { fe_sq(x, x); fe_sq(u, u); }
        else { fe_mul(x, x, y); fe_mul(u, u, y); }
    }
    fe_add(x, x, u);
    out[tid] = x;
}

__global__ __launch_bounds__(TPB) void k_inv(const fe *__restrict__ in, fe *__restrict__ out, int R) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    fe x = in[tid % 4096];
    for (int r = 0; r < R; r++) fe_invert(x, x);
    out[tid] = x;
}

// B additions per lane per step into B bucket states held in global memory
// (element k of lane t at [k][t]); R steps.
template <int B>
__global__ __launch_bounds__(TPB) void k_aff(const gen *__restrict__ pts, fe *__restrict__ bx, fe *__restrict__ by,
                                             fe *__restrict__ pre, uint32_t *__restrict__ ids, int R) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, L = gridDim.x * blockDim.x;
    uint32_t idx = tid * 2654435761u;
    fe one;
    fe_one(one);
    for (int r = 0; r < R; r++) {
        // prefix products of the denominators d_k = x2_k - x1_k
        fe acc = one;
        uint32_t id2 = idx;
        for (int k = 0; k < B; k++) {
            gen q;
            gen_load(q, pts + (id2 % NPTS));
            fe x1 = bx[(size_t)k * L + tid], d;
            fe_sub(d, q.YpX, x1);                 // x2 := YpX, y2 := YmX (synthetic coordinates)
            pre[(size_t)k * L + tid] = acc;
            ids[(size_t)k * L + tid] = id2;
            fe_mul(acc, acc, d);
            id2 = id2 * 1664525u + 1013904223u;
        }
        fe inv;
        fe_invert(inv, acc);
        // walk back: 1/d_k = inv * pre_k, inv *= d_k; then the addition
        for (int k = B - 1; k >= 0; k--) {
            const uint32_t idk = ids[(size_t)k * L + tid];   // the same point as above
            gen q;
            gen_load(q, pts + (idk % NPTS));
            fe x1 = bx[(size_t)k * L + tid], y1 = by[(size_t)k * L + tid];
            fe p = pre[(size_t)k * L + tid], di, d, lam, t, x3, y3;
            fe_mul(di, inv, p);
            fe_sub(d, q.YpX, x1);
            fe_mul(inv, inv, d);
            fe_sub(t, q.YmX, y1);
            fe_mul(lam, t, di);                   // lambda
            fe_sq(t, lam);
            fe_sub(t, t, x1);
            fe_sub(x3, t, q.YpX);                 // lambda^2 - x1 - x2 (A omitted: one constant subtraction)
            fe_sub(t, x1, x3);
            fe_mul(y3, lam, t);
            fe_sub(y3, y3, y1);
            bx[(size_t)k * L + tid] = x3;
            by[(size_t)k * L + tid] = y3;
        }
        for (int k = 0; k < B; k++) idx = idx * 1664525u + 1013904223u;
    }
}

// host copy of fe_from_words (8 little-endian words -> 10 limbs of 26/25 bits)
static fe host_fe(const uint32_t w8[8]) {
    fe r{};
    uint32_t w[9];
    for (int i = 0; i < 8; i++) w[i] = w8[i];
    w[8] = 0;
    for (int i = 0; i < 10; i++) {
        const int p = (i >> 1) * 51 + ((i & 1) ? 26 : 0), wi = p >> 5, sh = p & 31;
        const uint64_t x = ((uint64_t)w[wi] | ((uint64_t)w[wi + 1] << 32)) >> sh;
        r.v[i] = (uint32_t)x & ((1u << ((i & 1) ? 25 : 26)) - 1);
    }
    return r;
}

template <class F>
static float time_ms(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();   // warm-up
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int CUS = prop.multiProcessorCount;
    printf("device %s CUs %d clock %d MHz\n", prop.gcnArchName, CUS, prop.clockRate / 1000);
    // random-looking field elements / points (canonical limbs)
    std::vector<gen> hp(NPTS);
    std::vector<fe> hf(4096);
    uint64_t s = 0x9e3779b97f4a7c15ULL;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
    auto rfe = [&](fe &f) {
        uint32_t w[8];
        for (int i = 0; i < 8; i++) w[i] = rnd();
        w[7] &= 0x7fffffffu;
        f = host_fe(w);
    };
    for (auto &p : hp) { rfe(p.YpX); rfe(p.YmX); rfe(p.T2d); p.pad[0] = p.pad[1] = 0; }
    for (auto &f : hf) rfe(f);
    gen *dp;
    fe *df, *dout;
    ge *dge;
    CHK(hipMalloc(&dp, NPTS * sizeof(gen)));
    CHK(hipMalloc(&df, 4096 * sizeof(fe)));
    CHK(hipMemcpy(dp, hp.data(), NPTS * sizeof(gen), hipMemcpyHostToDevice));
    CHK(hipMemcpy(df, hf.data(), 4096 * sizeof(fe), hipMemcpyHostToDevice));
    const int blocks = CUS * 8;   // 2048 threads per CU: full occupancy for every kernel here
    const uint64_t L = (uint64_t)blocks * TPB;
    CHK(hipMalloc(&dout, L * sizeof(fe)));
    CHK(hipMalloc(&dge, L * sizeof(ge)));

    const int RM = 64;
    float ms = time_ms([&] { hipLaunchKernelGGL(k_madd, dim3(blocks), dim3(TPB), 0, 0, dp, dge, RM); });
    const double madd = L * RM / (ms * 1e-3);
    printf("madd (7M, point from HBM)   %8.3f ms  %7.2f G additions/s\n", ms, madd / 1e9);
    const int RMUL = 512;
    ms = time_ms([&] { hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(TPB), 0, 0, df, dout, RMUL, 0); });
    const double mul = 2.0 * L * RMUL / (ms * 1e-3);
    printf("fe_mul                        %8.3f ms  %7.2f G mul/s\n", ms, mul / 1e9);
    ms = time_ms([&] { hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(TPB), 0, 0, df, dout, RMUL, 1); });
    const double sq = 2.0 * L * RMUL / (ms * 1e-3);
    printf("fe_sq                         %8.3f ms  %7.2f G sq/s (%.3f M)\n", ms, sq / 1e9, mul / sq);
    const int RINV = 4;
    ms = time_ms([&] { hipLaunchKernelGGL(k_inv, dim3(blocks), dim3(TPB), 0, 0, df, dout, RINV); });
    const double inv = L * RINV / (ms * 1e-3);
    printf("fe_invert                     %8.3f ms  %7.4f G inv/s (%.1f M)\n", ms, inv / 1e9, mul / inv);
    printf("madd in M: %.2f\n", mul / madd);
    // batch-affine: states and prefixes in global memory, lane-interleaved
    auto run_aff = [&](auto kern, int B, int R) -> int {
        fe *bx, *by, *pre;
        uint32_t *ids;
        CHK(hipMalloc(&ids, (size_t)B * L * sizeof(uint32_t)));
        CHK(hipMalloc(&bx, (size_t)B * L * sizeof(fe)));
        CHK(hipMalloc(&by, (size_t)B * L * sizeof(fe)));
        CHK(hipMalloc(&pre, (size_t)B * L * sizeof(fe)));
        CHK(hipMemset(bx, 1, (size_t)B * L * sizeof(fe)));
        CHK(hipMemset(by, 2, (size_t)B * L * sizeof(fe)));
        float t = time_ms([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(TPB), 0, 0, dp, bx, by, pre, ids, R); });
        const double adds = (double)L * B * R / (t * 1e-3);
        printf("aff<%3d> (state %5zu B/lane) %8.3f ms  %7.2f G additions/s  = %.2f x madd, %.2f M per addition\n", B,
               (size_t)3 * B * sizeof(fe), t, adds / 1e9, adds / madd, mul / adds);
        (void)hipFree(bx);
        (void)hipFree(by);
        (void)hipFree(pre);
        (void)hipFree(ids);
        return 0;
    };
    if (run_aff(k_aff<8>, 8, 8)) return 1;
    if (run_aff(k_aff<32>, 32, 2)) return 1;
    if (run_aff(k_aff<128>, 128, 1)) return 1;
    // break-even batch from the unit costs alone (no memory traffic):
    // 7 = 2 + 3 + S + I / B  ->  B = I / (7 - 5 - S)
    const double Sm = mul / sq, Im = mul / inv;
    printf("model: batch-affine per addition = 5M + %.3fM + %.1fM / B; beats the 7M madd only for B > %.0f\n", Sm, Im,
           Im / (7.0 - 5.0 - Sm));
    return 0;
}
