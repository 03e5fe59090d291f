// fe_variants.hip — throughput and agreement of GF(2^255-19) multiply
// formulations on gfx950:
//   V0  dev_field.h fe_mul (operand scanning, compiler-scheduled carries)
//   V1  product scanning (Comba), v_mad_u64_u32 with its carry-out into a
//       third accumulator word (inline asm, no 64-bit adds)
//   V2  10 limbs of 25.5 bits (2^255 = 19 folding), 100 carry-free
//       v_mad_u64_u32 into 64-bit column sums, then one carry pass
// Each lane runs a dependent chain x <- x*y (2 chains per lane); the final
// values of all variants must agree mod p.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../device/dev_field.h"

// 8 x 32-bit limbs, fold 2^256 == 38 (the layout used before the radix-2^25.5 switch)
struct fe8 { uint32_t v[8]; };
DEVI void fe8_reduce16(fe8 &r, const uint32_t t[16]) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (uint64_t)t[8 + i] * 38u + t[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    c *= 38;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += r.v[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[0] += (uint32_t)c * 38;
}
DEVI void fe8_mul(fe8 &r, const fe8 &a, const fe8 &b) {
    uint32_t t[16];
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) { c += (uint64_t)a.v[0] * b.v[j]; t[j] = (uint32_t)c; c >>= 32; }
    t[8] = (uint32_t)c;
#pragma unroll
    for (int i = 1; i < 8; i++) {
        c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) { c += (uint64_t)a.v[i] * b.v[j] + t[i + j]; t[i + j] = (uint32_t)c; c >>= 32; }
        t[i + 8] = (uint32_t)c;
    }
    fe8_reduce16(r, t);
}
DEVI void fe8_canon(fe8 &r, const fe8 &a) {
    // value < 2^256 -> canonical via the 10-limb path
    fe x = fe_from_words(a.v[0], a.v[1], a.v[2], a.v[3], a.v[4], a.v[5], a.v[6], a.v[7] & 0x7fffffffu);
    x.v[0] += 19 * (a.v[7] >> 31);
    uint32_t w[8]; fe_tow(w, x);
    for (int i = 0; i < 8; i++) r.v[i] = w[i];
}

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

DEVI void mad_cy(uint64_t &acc, uint32_t &hi, uint32_t a, uint32_t b) {
    uint64_t cy;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cy) : "v"(a), "v"(b));
    asm volatile("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(hi), "=s"(cy) : "s"(cy));
}

DEVI void fe_mul_v1(fe8 &r, const fe8 &a, const fe8 &b) {
    uint32_t t[16];
    uint64_t acc = 0;
    uint32_t hi = 0;
#pragma unroll
    for (int k = 0; k < 15; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            int j = k - i;
            if (j < 0 || j > 7) continue;
            mad_cy(acc, hi, a.v[i], b.v[j]);
        }
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
        hi = 0;
    }
    t[15] = (uint32_t)acc;
    fe8_reduce16(r, t);
}

// ---- V2: radix 2^25.5, limbs alternately 26 and 25 bits
struct f10 { uint32_t v[10]; };
DEVI void f10_from(f10 &r, const fe8 &a) {
    fe8 c; fe8_canon(c, a);
    // unpack 255 bits into 26,25,26,25,...
    uint32_t w[8]; for (int i = 0; i < 8; i++) w[i] = c.v[i];
    int pos = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        int bits = (i & 1) ? 25 : 26;
        int wi = pos >> 5, sh = pos & 31;
        uint64_t x = w[wi] >> sh;
        if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
        r.v[i] = (uint32_t)x & ((1u << bits) - 1);
        pos += bits;
    }
}
DEVI void f10_to(fe8 &r, const f10 &a) {
    // value = sum a_i 2^{ceil(25.5 i)}; limbs may exceed their width slightly
    uint32_t w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int pos = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        int bits = (i & 1) ? 25 : 26;
        int wi = pos >> 5, sh = pos & 31;
        uint64_t x = (uint64_t)a.v[i] << sh;
        uint64_t c = 0;
        c = (uint64_t)w[wi] + (uint32_t)x; w[wi] = (uint32_t)c; c >>= 32;
        c += (uint64_t)w[wi + 1] + (uint32_t)(x >> 32); w[wi + 1] = (uint32_t)c; c >>= 32;
        for (int k = wi + 2; k < 9 && c; k++) { c += w[k]; w[k] = (uint32_t)c; c >>= 32; }
        pos += bits;
    }
    // fold w[8] (bits >= 256) and reduce
    uint64_t c = (uint64_t)w[8] * 38;
    for (int i = 0; i < 8; i++) { c += w[i]; r.v[i] = (uint32_t)c; c >>= 32; }
    r.v[0] += (uint32_t)c * 38;
}
DEVI uint64_t m64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }
DEVI void f10_mul(f10 &h, const f10 &f, const f10 &g) {
    uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4], f5 = f.v[5], f6 = f.v[6], f7 = f.v[7],
             f8 = f.v[8], f9 = f.v[9];
    uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4], g5 = g.v[5], g6 = g.v[6], g7 = g.v[7],
             g8 = g.v[8], g9 = g.v[9];
    uint32_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4, g5_19 = 19 * g5, g6_19 = 19 * g6,
             g7_19 = 19 * g7, g8_19 = 19 * g8, g9_19 = 19 * g9;
    uint32_t f1_2 = 2 * f1, f3_2 = 2 * f3, f5_2 = 2 * f5, f7_2 = 2 * f7, f9_2 = 2 * f9;
    uint64_t h0 = m64(f0, g0) + m64(f1_2, g9_19) + m64(f2, g8_19) + m64(f3_2, g7_19) + m64(f4, g6_19) +
                  m64(f5_2, g5_19) + m64(f6, g4_19) + m64(f7_2, g3_19) + m64(f8, g2_19) + m64(f9_2, g1_19);
    uint64_t h1 = m64(f0, g1) + m64(f1, g0) + m64(f2, g9_19) + m64(f3, g8_19) + m64(f4, g7_19) + m64(f5, g6_19) +
                  m64(f6, g5_19) + m64(f7, g4_19) + m64(f8, g3_19) + m64(f9, g2_19);
    uint64_t h2 = m64(f0, g2) + m64(f1_2, g1) + m64(f2, g0) + m64(f3_2, g9_19) + m64(f4, g8_19) +
                  m64(f5_2, g7_19) + m64(f6, g6_19) + m64(f7_2, g5_19) + m64(f8, g4_19) + m64(f9_2, g3_19);
    uint64_t h3 = m64(f0, g3) + m64(f1, g2) + m64(f2, g1) + m64(f3, g0) + m64(f4, g9_19) + m64(f5, g8_19) +
                  m64(f6, g7_19) + m64(f7, g6_19) + m64(f8, g5_19) + m64(f9, g4_19);
    uint64_t h4 = m64(f0, g4) + m64(f1_2, g3) + m64(f2, g2) + m64(f3_2, g1) + m64(f4, g0) + m64(f5_2, g9_19) +
                  m64(f6, g8_19) + m64(f7_2, g7_19) + m64(f8, g6_19) + m64(f9_2, g5_19);
    uint64_t h5 = m64(f0, g5) + m64(f1, g4) + m64(f2, g3) + m64(f3, g2) + m64(f4, g1) + m64(f5, g0) +
                  m64(f6, g9_19) + m64(f7, g8_19) + m64(f8, g7_19) + m64(f9, g6_19);
    uint64_t h6 = m64(f0, g6) + m64(f1_2, g5) + m64(f2, g4) + m64(f3_2, g3) + m64(f4, g2) + m64(f5_2, g1) +
                  m64(f6, g0) + m64(f7_2, g9_19) + m64(f8, g8_19) + m64(f9_2, g7_19);
    uint64_t h7 = m64(f0, g7) + m64(f1, g6) + m64(f2, g5) + m64(f3, g4) + m64(f4, g3) + m64(f5, g2) + m64(f6, g1) +
                  m64(f7, g0) + m64(f8, g9_19) + m64(f9, g8_19);
    uint64_t h8 = m64(f0, g8) + m64(f1_2, g7) + m64(f2, g6) + m64(f3_2, g5) + m64(f4, g4) + m64(f5_2, g3) +
                  m64(f6, g2) + m64(f7_2, g1) + m64(f8, g0) + m64(f9_2, g9_19);
    uint64_t h9 = m64(f0, g9) + m64(f1, g8) + m64(f2, g7) + m64(f3, g6) + m64(f4, g5) + m64(f5, g4) + m64(f6, g3) +
                  m64(f7, g2) + m64(f8, g1) + m64(f9, g0);
    uint64_t c;
    c = h0 >> 26; h1 += c; h0 &= 0x3ffffff;
    c = h4 >> 26; h5 += c; h4 &= 0x3ffffff;
    c = h1 >> 25; h2 += c; h1 &= 0x1ffffff;
    c = h5 >> 25; h6 += c; h5 &= 0x1ffffff;
    c = h2 >> 26; h3 += c; h2 &= 0x3ffffff;
    c = h6 >> 26; h7 += c; h6 &= 0x3ffffff;
    c = h3 >> 25; h4 += c; h3 &= 0x1ffffff;
    c = h7 >> 25; h8 += c; h7 &= 0x1ffffff;
    c = h4 >> 26; h5 += c; h4 &= 0x3ffffff;
    c = h8 >> 26; h9 += c; h8 &= 0x3ffffff;
    c = h9 >> 25; h0 += c * 19; h9 &= 0x1ffffff;
    c = h0 >> 26; h1 += c; h0 &= 0x3ffffff;
    h.v[0] = (uint32_t)h0; h.v[1] = (uint32_t)h1; h.v[2] = (uint32_t)h2; h.v[3] = (uint32_t)h3; h.v[4] = (uint32_t)h4;
    h.v[5] = (uint32_t)h5; h.v[6] = (uint32_t)h6; h.v[7] = (uint32_t)h7; h.v[8] = (uint32_t)h8; h.v[9] = (uint32_t)h9;
}

__device__ void seed_fe(fe8 &x, uint32_t s) {
    for (int i = 0; i < 8; i++) { s = s * 1664525u + 1013904223u; x.v[i] = s; }
    x.v[7] &= 0x7fffffff;
}

template <int V>
__global__ __launch_bounds__(256) void k_chain(uint32_t *out, int iters) {
    uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    fe8 x0, x1, y;
    seed_fe(x0, tid * 3 + 1); seed_fe(x1, tid * 3 + 2); seed_fe(y, 99);
    if (V == 2) {
        f10 a, b, g;
        f10_from(a, x0); f10_from(b, x1); f10_from(g, y);
        for (int i = 0; i < iters; i++) { f10_mul(a, a, g); f10_mul(b, b, g); }
        f10_to(x0, a); f10_to(x1, b);
    } else {
        for (int i = 0; i < iters; i++) {
            if (V == 0) { fe8_mul(x0, x0, y); fe8_mul(x1, x1, y); }
            else { fe_mul_v1(x0, x0, y); fe_mul_v1(x1, x1, y); }
        }
    }
    fe8 c0, c1; fe8_canon(c0, x0); fe8_canon(c1, x1);
    uint32_t h = 0;
    for (int i = 0; i < 8; i++) h = h * 31 + c0.v[i] + 7 * c1.v[i];
    out[tid] = h;
}
// production radix-2^25.5 square (dev_field.h fe_sq)
template <int V>
__global__ __launch_bounds__(256) void k_sqchain(uint32_t *out, int iters) {
    uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    fe8 s0, s1;
    seed_fe(s0, tid * 3 + 1); seed_fe(s1, tid * 3 + 2);
    fe x0 = fe_from_words(s0.v[0], s0.v[1], s0.v[2], s0.v[3], s0.v[4], s0.v[5], s0.v[6], s0.v[7]);
    fe x1 = fe_from_words(s1.v[0], s1.v[1], s1.v[2], s1.v[3], s1.v[4], s1.v[5], s1.v[6], s1.v[7]);
    for (int i = 0; i < iters; i++) { fe_sq(x0, x0); fe_sq(x1, x1); }
    uint32_t w0[8], w1[8]; fe_tow(w0, x0); fe_tow(w1, x1);
    fe8 c0, c1;
    for (int i = 0; i < 8; i++) { c0.v[i] = w0[i]; c1.v[i] = w1[i]; }
    uint32_t h = 0;
    for (int i = 0; i < 8; i++) h = h * 31 + c0.v[i] + 7 * c1.v[i];
    out[tid] = h;
}

int main() {
    hipDeviceProp_t pr;
    CHK(hipGetDeviceProperties(&pr, 0));
    int clk_khz = 0;
    CHK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const int cus = pr.multiProcessorCount, blocks = cus * 8, threads = 256, iters = 2048;
    const size_t nt = (size_t)blocks * threads;
    uint32_t *d;
    CHK(hipMalloc(&d, nt * 4 * 4));
    uint32_t *h = (uint32_t *)malloc(nt * 4 * 4);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    typedef void (*kf)(uint32_t *, int);
    kf ks[4] = {k_chain<0>, k_chain<1>, k_chain<2>, k_sqchain<0>};
    const char *nm[4] = {"V0 8x32 schoolbook", "V1 comba+carry asm", "V2 10x25.5 carry-free", "fe_sq (10x25.5)"};
    for (int v = 0; v < 4; v++) {
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(threads), 0, 0, d + v * nt, iters);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(threads), 0, 0, d + v * nt, iters);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        double muls = 2.0 * nt * iters;
        printf("%-24s %8.3f ms  %7.1f Gmul/s  %6.1f clk/mul/lane-equiv (x64/CU)\n", nm[v], ms, muls / ms / 1e6,
               (ms * 1e-3 * clk_khz * 1e3 * cus * 64) / muls);
    }
    CHK(hipMemcpy(h, d, nt * 4 * 3, hipMemcpyDeviceToHost));
    size_t bad1 = 0, bad2 = 0;
    for (size_t i = 0; i < nt; i++) { bad1 += h[i] != h[nt + i]; bad2 += h[i] != h[2 * nt + i]; }
    printf("agreement: V1 mismatches %zu, V2 mismatches %zu of %zu\n", bad1, bad2, nt);
    return 0;
}
