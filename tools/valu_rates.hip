// Microbenchmark: wave64 issue rates of the integer VALU instructions the
// Montgomery multiply is built from, on every CU of the device.  Pins the
// compute roofline quoted in DESIGN.md (no vendor number exists for
// v_mad_u64_u32 on gfx950).  Build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096

// 8 independent chains per lane, inline asm so nothing is folded
template <int KIND>
__global__ void __launch_bounds__(256) k_rate(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint64_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (uint64_t)(a + i) << 3 | b;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (KIND == 0) {
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
            } else if constexpr (KIND == 1) {
                uint32_t lo = (uint32_t)acc[i], hi = (uint32_t)(acc[i] >> 32);
                asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc"
                             : "+v"(lo), "+v"(hi) : "v"(a) : "vcc");
                acc[i] = ((uint64_t)hi << 32) | lo;
            } else if constexpr (KIND == 2) {
                uint32_t lo = (uint32_t)acc[i];
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
                acc[i] = (acc[i] & 0xffffffff00000000ull) | lo;
            } else if constexpr (KIND == 3) {
                uint32_t lo = (uint32_t)acc[i];
                asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
                acc[i] = (acc[i] & 0xffffffff00000000ull) | lo;
            } else if constexpr (KIND == 4) {
                asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"((uint64_t)b));
            } else if constexpr (KIND == 5) {
                uint32_t lo = (uint32_t)acc[i];
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(b));
                acc[i] = (acc[i] & 0xffffffff00000000ull) | lo;
            } else if constexpr (KIND == 6) {
                double d = (double)acc[i];
                asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d) : "v"((double)b));
                acc[i] = (uint64_t)d;
            }
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= acc[i];
    if (s == 0x1234567) out[0] = (uint32_t)s;
}

template <int KIND>
double run(const char* name, int waves_per_simd) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* d;
    hipMalloc(&d, 4);
    const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_rate<KIND><<<blocks, 256>>>(d, 1);
    hipEventRecord(e0);
    k_rate<KIND><<<blocks, 256>>>(d, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)blocks * 256 * ITERS * 8;  // lane-instructions (asm stmts)
    const double rate = instr / (ms * 1e-3);
    printf("%-28s waves/SIMD=%d  %8.3f ms  %8.3f T lane-op/s  (%.2f cyc/wave-op/SIMD @2.4GHz)\n", name,
           waves_per_simd, ms, rate / 1e12, (cus * 4 * 2.4e9) / (rate / 64));
    hipFree(d);
    return rate;
}

int main() {
    for (int w = 1; w <= 4; w *= 2) {
        run<0>("v_mad_u64_u32", w);
        run<1>("v_add_co+v_addc (pair)", w);
        run<2>("v_mul_lo_u32", w);
        run<3>("v_mul_hi_u32", w);
        run<4>("v_lshl_add_u64", w);
        run<5>("v_add_u32", w);
        run<6>("v_fma_f64", w);
    }
    return 0;
}
