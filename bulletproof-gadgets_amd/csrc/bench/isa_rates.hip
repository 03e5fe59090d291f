// isa_rates.hip — measured issue rates of the VALU instructions 255-bit
// modular arithmetic can be built from on gfx950 (one wave64 instruction
// stream per SIMD, 8 independent chains per lane so latency is hidden).
// Prints ops/cycle/CU for each instruction; used to pick the limb layout.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define BODY8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ __launch_bounds__(256) void k_mad64(uint64_t *out, uint32_t a, uint32_t b) {
    uint64_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    uint32_t x = a ^ threadIdx.x, y = b;
    for (int it = 0; it < ITERS; it++) {
#define X(k) { uint64_t cy_; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy_) : "v"(x), "v"(y)); }
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mullo(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    uint32_t y = b;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(y));
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mulhi(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    uint32_t y = b;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(y));
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mad24(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    uint32_t x = a ^ threadIdx.x, y = b;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[k]) : "v"(x), "v"(y));
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fma64(uint64_t *out, uint32_t a, uint32_t b) {
    double acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    double x = (double)a * 1e-9, y = (double)b * 1e-9;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[k]) : "v"(x), "v"(y));
        BODY8(X)
#undef X
    }
    double s = 0;
    for (int k = 0; k < 8; k++) s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}
__global__ __launch_bounds__(256) void k_addc(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    uint32_t y = b;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[k]) : "v"(y) : "vcc");
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_add64(uint64_t *out, uint32_t a, uint32_t b) {
    uint64_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    uint64_t y = b;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(y));
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mov(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t acc[8];
    for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + k;
    for (int it = 0; it < ITERS; it++) {
#define X(k) asm volatile("v_mov_b32 %0, %1" : "=v"(acc[k]) : "v"(acc[(k + 1) & 7]));
        BODY8(X)
#undef X
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t *, uint32_t, uint32_t);

int main() {
    int dev = 0;
    hipDeviceProp_t pr;
    CHK(hipGetDeviceProperties(&pr, dev));
    int cus = pr.multiProcessorCount;
    int clk_khz = 0;
    CHK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
    printf("device %s CUs %d clock %.0f MHz\n", pr.gcnArchName, cus, clk_khz / 1e3);
    const int blocks = cus * 8, threads = 256;
    uint64_t *out;
    CHK(hipMalloc(&out, (size_t)blocks * threads * 8));
    struct { const char *name; kfn f; int per; } ks[] = {
        {"v_mad_u64_u32", k_mad64, 1}, {"v_mul_lo_u32", k_mullo, 1}, {"v_mul_hi_u32", k_mulhi, 1},
        {"v_mad_u32_u24", k_mad24, 1}, {"v_fma_f64", k_fma64, 1}, {"v_add_co+v_addc", k_addc, 2},
        {"v_lshl_add_u64", k_add64, 1}, {"v_mov_b32", k_mov, 1}};
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u, 67890u);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 12345u, 67890u);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        double lane_ops = 5.0 * blocks * threads * (double)ITERS * 8 * k.per;
        double per_s = lane_ops / (ms * 1e-3);
        double per_cu_clk = per_s / cus / (clk_khz * 1e3);
        printf("%-18s %8.3f ms  %9.2f Tlane-op/s  %6.2f lane-op/clk/CU (64 = full rate)\n", k.name, ms,
               per_s / 1e12, per_cu_clk);
    }
    return 0;
}
