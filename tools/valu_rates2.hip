#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
// KIND 0: 8 independent mads per asm block; 1: 8 mads chained through one 64-bit accumulator;
// 2: 4 chains x 2 dependent; 3: 8 x (v_add_co + v_addc) independent pairs; 4: 8 v_lshl_add_u64 indep;
// 5: 8 v_add_u32 indep; 6: 8 v_mul_lo_u32 indep; 7: 8 v_mad_u32_u24; 8: mad with SGPR operand b
template <int KIND>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint64_t x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3, x4 = a + 4, x5 = a + 5, x6 = a + 6, x7 = a + 7;
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == 0) {
            asm volatile(
                "v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n v_mad_u64_u32 %1, s[42:43], %8, %9, %1\n"
                "v_mad_u64_u32 %2, s[44:45], %8, %9, %2\n v_mad_u64_u32 %3, s[46:47], %8, %9, %3\n"
                "v_mad_u64_u32 %4, s[48:49], %8, %9, %4\n v_mad_u64_u32 %5, s[50:51], %8, %9, %5\n"
                "v_mad_u64_u32 %6, s[52:53], %8, %9, %6\n v_mad_u64_u32 %7, s[54:55], %8, %9, %7\n"
                : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                : "v"(a), "v"(b) : "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55");
        } else if constexpr (KIND == 1) {
            asm volatile(
                "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                "v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n"
                : "+v"(x0) : "v"(a), "v"(b) : "s40","s41");
        } else if constexpr (KIND == 2) {
            asm volatile(
                "v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n v_mad_u64_u32 %1, s[42:43], %4, %5, %1\n"
                "v_mad_u64_u32 %2, s[44:45], %4, %5, %2\n v_mad_u64_u32 %3, s[46:47], %4, %5, %3\n"
                "v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n v_mad_u64_u32 %1, s[42:43], %4, %5, %1\n"
                "v_mad_u64_u32 %2, s[44:45], %4, %5, %2\n v_mad_u64_u32 %3, s[46:47], %4, %5, %3\n"
                : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b) : "s40","s41","s42","s43","s44","s45","s46","s47");
        } else if constexpr (KIND == 3) {
            uint32_t l0=(uint32_t)x0,h0=(uint32_t)(x0>>32),l1=(uint32_t)x1,h1=(uint32_t)(x1>>32),l2=(uint32_t)x2,h2=(uint32_t)(x2>>32),l3=(uint32_t)x3,h3=(uint32_t)(x3>>32);
            asm volatile(
                "v_add_co_u32 %0, s[40:41], %0, %8\n v_add_co_u32 %2, s[42:43], %2, %8\n v_add_co_u32 %4, s[44:45], %4, %8\n v_add_co_u32 %6, s[46:47], %6, %8\n"
                "v_addc_co_u32 %1, s[40:41], %1, %8, s[40:41]\n v_addc_co_u32 %3, s[42:43], %3, %8, s[42:43]\n v_addc_co_u32 %5, s[44:45], %5, %8, s[44:45]\n v_addc_co_u32 %7, s[46:47], %7, %8, s[46:47]\n"
                : "+v"(l0),"+v"(h0),"+v"(l1),"+v"(h1),"+v"(l2),"+v"(h2),"+v"(l3),"+v"(h3) : "v"(a) : "s40","s41","s42","s43","s44","s45","s46","s47");
            x0=((uint64_t)h0<<32)|l0; x1=((uint64_t)h1<<32)|l1; x2=((uint64_t)h2<<32)|l2; x3=((uint64_t)h3<<32)|l3;
        } else if constexpr (KIND == 4) {
            uint64_t bb = b;
            asm volatile(
                "v_lshl_add_u64 %0, %0, 0, %8\n v_lshl_add_u64 %1, %1, 0, %8\n v_lshl_add_u64 %2, %2, 0, %8\n v_lshl_add_u64 %3, %3, 0, %8\n"
                "v_lshl_add_u64 %4, %4, 0, %8\n v_lshl_add_u64 %5, %5, 0, %8\n v_lshl_add_u64 %6, %6, 0, %8\n v_lshl_add_u64 %7, %7, 0, %8\n"
                : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(bb));
        } else if constexpr (KIND == 5 || KIND == 6) {
            uint32_t l0=(uint32_t)x0,l1=(uint32_t)x1,l2=(uint32_t)x2,l3=(uint32_t)x3,l4=(uint32_t)x4,l5=(uint32_t)x5,l6=(uint32_t)x6,l7=(uint32_t)x7;
            if constexpr (KIND == 5)
            asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                : "+v"(l0),"+v"(l1),"+v"(l2),"+v"(l3),"+v"(l4),"+v"(l5),"+v"(l6),"+v"(l7) : "v"(b));
            else
            asm volatile("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
                : "+v"(l0),"+v"(l1),"+v"(l2),"+v"(l3),"+v"(l4),"+v"(l5),"+v"(l6),"+v"(l7) : "v"(b));
            x0=l0;x1=l1;x2=l2;x3=l3;x4=l4;x5=l5;x6=l6;x7=l7;
        } else if constexpr (KIND == 7) {
            asm volatile(
                "v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n v_mad_u64_u32 %1, s[42:43], %8, %9, %1\n"
                "v_mad_u64_u32 %2, s[44:45], %8, %9, %2\n v_mad_u64_u32 %3, s[46:47], %8, %9, %3\n"
                "v_mad_u64_u32 %4, s[48:49], %8, %9, %4\n v_mad_u64_u32 %5, s[50:51], %8, %9, %5\n"
                "v_mad_u64_u32 %6, s[52:53], %8, %9, %6\n v_mad_u64_u32 %7, s[54:55], %8, %9, %7\n"
                : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                : "v"(a), "s"(seed * 3u) : "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55");
        }
    }
    uint64_t s = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (s == 0x1234567) out[0] = (uint32_t)s;
}
template <int KIND>
void run(const char* name, int w) {
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* d; hipMalloc(&d, 4);
    int blocks = cus * w;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    k<KIND><<<blocks, 256>>>(d, 1);
    hipEventRecord(e0); k<KIND><<<blocks, 256>>>(d, 2); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double waveops = (double)ITERS * 8;  // per wave
    double cyc = ms * 1e-3 * 2.4e9 / w;  // cycles per wave (w waves share a SIMD)
    printf("%-34s waves/SIMD=%d %8.3f ms  %6.2f cyc per instr per wave-slot (@2.4GHz)\n", name, w, ms, cyc / waveops);
    hipFree(d);
}
int main() {
    for (int w = 1; w <= 2; w++) {
        run<0>("mad x8 independent", w);
        run<7>("mad x8 independent, SGPR b", w);
        run<1>("mad x8 one accumulator chain", w);
        run<2>("mad 4 chains x2", w);
        run<3>("add_co/addc 4 pairs", w);
        run<4>("lshl_add_u64 x8", w);
        run<5>("v_add_u32 x8", w);
        run<6>("v_mul_lo_u32 x8", w);
    }
}
