// Per-instruction issue cost of ONE wave per SIMD (the pairing kernels'
// occupancy at batch 2^16) for the instruction kinds the generated kernels
// emit (tools/pgen/emit.py): how many shader clocks a lone wave spends per
// instruction in a long run of independent ones, and in the mixes a
// Montgomery product leaf is made of.  1024 one-wave blocks (one per SIMD),
// s_memtime around the loop, 16 instructions per iteration.
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/issue_probe.hip -o tools/issue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

// each probe: a name and a 16-instruction asm body over v0..v15-style operands
#define PROBE(NAME, BODY)                                                                                    \
    __global__ void __launch_bounds__(64) NAME(uint64_t* out, int iters) {                                  \
        uint64_t t0, t1;                                                                                    \
        uint32_t a = threadIdx.x * 3 + 1, b = blockIdx.x + 7, c = a ^ 0x55, d = b * 5;                      \
        uint64_t x = a, y = b, z = c, w = d;                                                                \
        asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));                                    \
        for (int it = 0; it < iters; it++) {                                                                \
            asm volatile(BODY : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(x), "+v"(y), "+v"(z), "+v"(w) : : "vcc", "s40", "s41"); \
        }                                                                                                   \
        asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));                                    \
        if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;                                                    \
        if (a == 0x12345 && b == 7 && x == 3 && w == 9) out[blockIdx.x + 4096] = c + d + y + z;              \
    }

// %0..%3 = a b c d (32-bit), %4..%7 = x y z w (64-bit pairs)
PROBE(p_add, R4("v_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %3\n v_add_u32 %1, %1, %0\n v_add_u32 %3, %3, %2\n"))
PROBE(p_add_indep, R4("v_add_u32 %0, %1, %2\n v_add_u32 %3, %1, %2\n v_add_u32 %0, %2, %1\n v_add_u32 %3, %2, %1\n"))
PROBE(p_mul_lo, R4("v_mul_lo_u32 %0, %1, %2\n v_mul_lo_u32 %3, %1, %2\n v_mul_lo_u32 %0, %2, %1\n v_mul_lo_u32 %3, %2, %1\n"))
PROBE(p_mad, R4("v_mad_u64_u32 %4, vcc, %0, %1, %4\n v_mad_u64_u32 %5, vcc, %0, %1, %5\n"
                "v_mad_u64_u32 %6, vcc, %0, %1, %6\n v_mad_u64_u32 %7, vcc, %0, %1, %7\n"))
PROBE(p_mad_add, R4("v_mad_u64_u32 %4, vcc, %0, %1, %4\n v_add_u32 %2, %0, %1\n"
                    "v_mad_u64_u32 %5, vcc, %0, %1, %5\n v_add_u32 %3, %0, %1\n"))
PROBE(p_mad_mullo, R4("v_mad_u64_u32 %4, vcc, %0, %1, %4\n v_mul_lo_u32 %2, %0, %1\n"
                      "v_mad_u64_u32 %5, vcc, %0, %1, %5\n v_mul_lo_u32 %3, %0, %1\n"))
PROBE(p_shr64, R4("v_lshrrev_b64 %4, 28, %4\n v_lshrrev_b64 %5, 28, %5\n v_lshrrev_b64 %6, 28, %6\n v_lshrrev_b64 %7, 28, %7\n"))
PROBE(p_mad_chain, R16("v_mad_u64_u32 %4, vcc, %0, %1, %4\n"))
// one column of a Montgomery product leaf (emit_sop, k < 14): two products into
// the accumulator, the digit m = acc q' mod 2^28, acc += m q0, acc >>= 28 ... x2
PROBE(p_column, R4("v_mad_u64_u32 %4, vcc, %0, %1, %4\n v_mad_u64_u32 %4, vcc, %2, %3, %4\n"
                   "v_mul_lo_u32 %0, %2, %1\n v_and_b32 %0, 0xfffffff, %0\n"))
PROBE(p_accread, R4("v_accvgpr_write_b32 a0, %0\n v_accvgpr_write_b32 a1, %1\n v_accvgpr_read_b32 %2, a2\n v_accvgpr_read_b32 %3, a3\n"))
PROBE(p_cndmask, R4("v_cndmask_b32 %0, %1, %2, vcc\n v_cndmask_b32 %3, %1, %2, vcc\n v_cndmask_b32 %0, %2, %1, vcc\n v_cndmask_b32 %3, %2, %1, vcc\n"))
PROBE(p_cnd_e64s, R4("v_cndmask_b32_e64 %0, %1, %2, s[40:41]\n v_cndmask_b32_e64 %3, %1, %2, s[40:41]\n v_cndmask_b32_e64 %0, %2, %1, s[40:41]\n v_cndmask_b32_e64 %3, %2, %1, s[40:41]\n"))
PROBE(p_cnd_e64vcc, R4("v_cndmask_b32_e64 %0, %1, %2, vcc\n v_cndmask_b32_e64 %3, %1, %2, vcc\n v_cndmask_b32_e64 %0, %2, %1, vcc\n v_cndmask_b32_e64 %3, %2, %1, vcc\n"))
PROBE(p_cnd_add, R4("v_cndmask_b32 %0, %1, %2, vcc\n v_add_u32 %3, %1, %2\n v_cndmask_b32 %0, %2, %1, vcc\n v_add_u32 %3, %2, %1\n"))
PROBE(p_bfi, R4("v_bfi_b32 %0, %1, %2, %3\n v_bfi_b32 %3, %1, %2, %0\n v_bfi_b32 %0, %2, %1, %3\n v_bfi_b32 %3, %2, %1, %0\n"))
PROBE(p_sad, R4("v_sad_u32 %0, %1, %2, %3\n v_sad_u32 %3, %1, %2, %0\n v_sad_u32 %0, %2, %1, %3\n v_sad_u32 %3, %2, %1, %0\n"))

typedef void (*K)(uint64_t*, int);

static void run(const char* name, K k, uint64_t* d, uint64_t* h) {
    const int blocks = 1024, iters = 4000;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, iters);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, iters);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * blocks, hipMemcpyDeviceToHost);
    double clk = 0;
    for (int b = 0; b < blocks; b++) clk += h[b];
    printf("%-12s %6.2f clk per instruction (one wave per SIMD)\n", name, clk / blocks / (16.0 * iters));
}

int main() {
    uint64_t* d;
    if (hipMalloc(&d, 8 * 8192) != hipSuccess) return 1;
    static uint64_t h[8192];
    run("add_dep", p_add, d, h);
    run("add_indep", p_add_indep, d, h);
    run("mul_lo", p_mul_lo, d, h);
    run("mad", p_mad, d, h);
    run("mad+add", p_mad_add, d, h);
    run("mad+mul_lo", p_mad_mullo, d, h);
    run("shr64", p_shr64, d, h);
    run("mad_chain", p_mad_chain, d, h);
    run("column", p_column, d, h);
    run("accvgpr", p_accread, d, h);
    run("cndmask", p_cndmask, d, h);
    run("sad", p_sad, d, h);
    run("cnd_e64_sgpr", p_cnd_e64s, d, h);
    run("cnd_e64_vcc", p_cnd_e64vcc, d, h);
    run("cnd+add", p_cnd_add, d, h);
    run("bfi", p_bfi, d, h);
    (void)hipFree(d);
    return 0;
}
