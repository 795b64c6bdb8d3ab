// Sustained-load shader clock: s_memtime (core clock counter) against
// s_memrealtime (100 MHz) around a long v_mad_u64_u32 loop on every SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 clock_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void __launch_bounds__(64) k(uint64_t* out, int iters, uint32_t seed) {
    uint64_t t0, r0, t1, r1;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0));
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint64_t x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3;
    for (int it = 0; it < iters; it++) {
        asm volatile(
            "v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n v_mad_u64_u32 %1, s[42:43], %4, %5, %1\n"
            "v_mad_u64_u32 %2, s[44:45], %4, %5, %2\n v_mad_u64_u32 %3, s[46:47], %4, %5, %3\n"
            "v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n v_mad_u64_u32 %1, s[42:43], %4, %5, %1\n"
            "v_mad_u64_u32 %2, s[44:45], %4, %5, %2\n v_mad_u64_u32 %3, s[46:47], %4, %5, %3\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    }
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1));
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x] = t1 - t0;
        out[3 * blockIdx.x + 1] = r1 - r0;
        out[3 * blockIdx.x + 2] = x0 ^ x1 ^ x2 ^ x3;
    }
}

int main() {
    uint64_t* d;
    const int maxb = 2048;
    (void)hipMalloc(&d, 3 * 8 * maxb);
    uint64_t h[3 * maxb];
    for (int w = 1; w <= 2; w++) {
        for (int iters : {2000, 200000}) {
            const int blocks = 1024 * w;
            k<<<blocks, 64>>>(d, iters, 1);
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            k<<<blocks, 64>>>(d, iters, 2);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            (void)hipMemcpy(h, d, 3 * 8 * blocks, hipMemcpyDeviceToHost);
            double clk = 0, rt = 0;
            for (int b = 0; b < blocks; b++) { clk += h[3 * b]; rt += h[3 * b + 1]; }
            const double mhz = clk / rt * 100.0;
            const double instr = 8.0 * iters;
            printf("waves/SIMD=%d iters=%6d: %8.3f ms, shader clock %.0f MHz, %.2f clk per mad per wave, "
                   "%.2f clk per mad per SIMD\n", w, iters, ms, mhz, (clk / blocks) / instr,
                   (clk / blocks) / instr / w);
        }
    }
    return 0;
}
