// v_mad_u64_u32 issue ceiling of the MI355X at 1, 2, 4 and 8 waves per SIMD
// (the roofline peak bench.py divides by).
//
// Every wave runs ITERS x 16 v_mad_u64_u32 in C independent accumulator chains
// (C = 1, 4, 8), the carry-out to VCC as the generated kernels emit it
// (tools/pgen/emit.py) or to four rotating SGPR pairs; the shader clock is read
// with s_memtime against s_memrealtime (100 MHz) around the loop, the kernel
// time with HIP events.  1024 x w one-wave blocks put w waves on each of the
// 1024 SIMDs (256 CUs x 4).  Output: per configuration the clocks per mad per
// SIMD and the chip's limb-MAC rate (T/s) = 1024 SIMDs x 64 lanes x mads / s.
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_peak.hip -o tools/valu_peak
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define MAD_VCC(x) "v_mad_u64_u32 " x ", vcc, %[a], %[b], " x "\n"
#define MAD_S(x, s) "v_mad_u64_u32 " x ", " s ", %[a], %[b], " x "\n"

template <int C, bool VCC>
__global__ void __launch_bounds__(64) k(uint64_t* out, int iters, uint32_t seed) {
    uint64_t t0, r0, t1, r1;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0));
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
    uint64_t x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3, x4 = a + 4, x5 = a + 5, x6 = a + 6, x7 = a + 7;
    for (int it = 0; it < iters; it++) {
        if (C == 1 && VCC) {
            asm volatile(MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]") MAD_VCC("%[x0]")
                         : [x0] "+v"(x0) : [a] "v"(a), [b] "v"(b) : "vcc");
        } else if (C == 4 && VCC) {
            asm volatile(MAD_VCC("%[x0]") MAD_VCC("%[x1]") MAD_VCC("%[x2]") MAD_VCC("%[x3]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x1]") MAD_VCC("%[x2]") MAD_VCC("%[x3]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x1]") MAD_VCC("%[x2]") MAD_VCC("%[x3]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x1]") MAD_VCC("%[x2]") MAD_VCC("%[x3]")
                         : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3)
                         : [a] "v"(a), [b] "v"(b) : "vcc");
        } else if (C == 8 && VCC) {
            asm volatile(MAD_VCC("%[x0]") MAD_VCC("%[x1]") MAD_VCC("%[x2]") MAD_VCC("%[x3]")
                         MAD_VCC("%[x4]") MAD_VCC("%[x5]") MAD_VCC("%[x6]") MAD_VCC("%[x7]")
                         MAD_VCC("%[x0]") MAD_VCC("%[x1]") MAD_VCC("%[x2]") MAD_VCC("%[x3]")
                         MAD_VCC("%[x4]") MAD_VCC("%[x5]") MAD_VCC("%[x6]") MAD_VCC("%[x7]")
                         : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [x4] "+v"(x4),
                           [x5] "+v"(x5), [x6] "+v"(x6), [x7] "+v"(x7)
                         : [a] "v"(a), [b] "v"(b) : "vcc");
        } else {  // C == 8, carry-outs to four SGPR pairs
            asm volatile(MAD_S("%[x0]", "s[40:41]") MAD_S("%[x1]", "s[42:43]") MAD_S("%[x2]", "s[44:45]")
                         MAD_S("%[x3]", "s[46:47]") MAD_S("%[x4]", "s[40:41]") MAD_S("%[x5]", "s[42:43]")
                         MAD_S("%[x6]", "s[44:45]") MAD_S("%[x7]", "s[46:47]") MAD_S("%[x0]", "s[40:41]")
                         MAD_S("%[x1]", "s[42:43]") MAD_S("%[x2]", "s[44:45]") MAD_S("%[x3]", "s[46:47]")
                         MAD_S("%[x4]", "s[40:41]") MAD_S("%[x5]", "s[42:43]") MAD_S("%[x6]", "s[44:45]")
                         MAD_S("%[x7]", "s[46:47]")
                         : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [x4] "+v"(x4),
                           [x5] "+v"(x5), [x6] "+v"(x6), [x7] "+v"(x7)
                         : [a] "v"(a), [b] "v"(b)
                         : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
        }
    }
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1));
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x] = t1 - t0;
        out[3 * blockIdx.x + 1] = r1 - r0;
        out[3 * blockIdx.x + 2] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    }
}

template <int C, bool VCC>
void run(uint64_t* d, uint64_t* h, int w, int iters) {
    const int blocks = 1024 * w;
    k<C, VCC><<<blocks, 64>>>(d, iters, 1);  // warm-up (clock ramp)
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k<C, VCC><<<blocks, 64>>>(d, iters, 2);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(h, d, 3 * 8 * blocks, hipMemcpyDeviceToHost);
    double clk = 0, rt = 0;
    for (int b = 0; b < blocks; b++) {
        clk += h[3 * b];
        rt += h[3 * b + 1];
    }
    const double mhz = clk / rt * 100.0;
    const double mads = 16.0 * iters;                       // per wave
    const double per_wave = (clk / blocks) / mads;          // shader clocks per mad, one wave's view
    const double tmacs = 1024.0 * w * 64.0 * mads / (ms * 1e-3) / 1e12;  // chip-wide, from wall time
    printf("waves/SIMD=%d chains=%d carry=%-5s: %8.3f ms, clock %4.0f MHz, %5.2f clk/mad/wave, %5.2f clk/mad/SIMD, "
           "%6.2f T limb-MAC/s\n",
           w, C, VCC ? "vcc" : "sgpr", ms, mhz, per_wave, per_wave / w, tmacs);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    const int maxb = 1024 * 8;
    uint64_t* d;
    if (hipMalloc(&d, 3 * 8 * maxb) != hipSuccess) return 1;
    static uint64_t h[3 * maxb];
    const int iters = 20000;
    for (int w : {1, 2, 4, 8}) {
        run<1, true>(d, h, w, iters / w);
        run<4, true>(d, h, w, iters / w);
        run<8, true>(d, h, w, iters / w);
        run<8, false>(d, h, w, iters / w);
    }
    (void)hipFree(d);
    return 0;
}
