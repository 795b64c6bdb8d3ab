// Does a VALU instruction cost fewer SIMD cycles when EXEC masks off whole
// 16-lane quarters of the wave?  (If so, an inversion run by half the lanes of
// a lane-pair wave, compacted into lanes 0..31, would cost half.)  A loop of
// 16 independent v_mad_u64_u32 per iteration under EXEC = all lanes, lanes
// 0..31, lanes 0..15, the even lanes, one lane; one or two waves per SIMD;
// s_memtime around the loop.
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/exec_probe.hip -o tools/exec_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R4(x) x x x x

__global__ void __launch_bounds__(64) k_probe(uint64_t* out, int iters, uint64_t mask) {
    uint64_t t0, t1;
    uint32_t a = threadIdx.x * 3 + 1, b = blockIdx.x + 7;
    uint64_t x = a, y = b, z = a ^ 0x55, w = b * 5;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
    for (int it = 0; it < iters; it++) {
        // EXEC is saved in s[44:45], set to the probe mask for the 16
        // instructions and restored before the loop's own (scalar) control
        asm volatile("s_mov_b64 s[44:45], exec\n"
                     "s_mov_b64 exec, %6\n" R4("v_mad_u64_u32 %2, vcc, %0, %1, %2\n v_mad_u64_u32 %3, vcc, %0, %1, %3\n"
                                               "v_mad_u64_u32 %4, vcc, %0, %1, %4\n v_mad_u64_u32 %5, vcc, %0, %1, %5\n")
                     "s_mov_b64 exec, s[44:45]\n"
                     : "+v"(a), "+v"(b), "+v"(x), "+v"(y), "+v"(z), "+v"(w)
                     : "s"(mask)
                     : "vcc", "s44", "s45");
    }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (a == 0x12345 && x == 3 && w == 9) out[blockIdx.x + 8192] = y + z;
}

int main() {
    uint64_t *d, *h = (uint64_t*)malloc(16384 * 8);
    if (hipMalloc(&d, 16384 * 8) != hipSuccess) return 1;
    const int iters = 4000;
    const struct { const char* name; uint64_t mask; } masks[] = {
        {"all 64 lanes", ~0ull}, {"lanes 0..31", 0xffffffffull}, {"lanes 0..15", 0xffffull},
        {"even lanes", 0x5555555555555555ull}, {"lane 0", 1ull}};
    for (int waves = 1; waves <= 2; waves++) {
        const int blocks = 1024 * waves;
        for (const auto& m : masks) {
            for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(64), 0, 0, d, iters, m.mask);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            if (hipMemcpy(h, d, blocks * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
            double s = 0;
            for (int i = 0; i < blocks; i++) s += (double)h[i];
            // s_memtime counts at a fixed reference clock; report per-instruction
            // time relative to the full-mask row of the same occupancy
            printf("%d wave(s)/SIMD  %-14s %8.2f memtime ticks per instruction\n", waves, m.name,
                   s / blocks / (iters * 16.0));
        }
    }
    return 0;
}
