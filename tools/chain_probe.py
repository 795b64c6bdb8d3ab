#!/usr/bin/env python3
"""Emit tools/chain_probe.hip: a lone wave per SIMD runs 16 v_mad_u64_u32
per loop iteration as 1, 2, 4 or 8 interleaved accumulator chains (all in
one asm statement, explicit registers), timed with s_memtime: the dependent
issue latency of the 64-bit multiply-accumulate."""
import os

L = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdint.h>']
for chains in (1, 2, 4, 8):
    body = []
    for i in range(16):
        c = i % chains
        body.append("v_mad_u64_u32 v[%d:%d], vcc, v40, v41, v[%d:%d]" % (2 * c, 2 * c + 1, 2 * c, 2 * c + 1))
    asm = "\\n".join(body)
    clob = ", ".join('"v%d"' % r for r in range(2 * chains)) + ', "v40", "v41", "vcc"'
    L.append("__global__ void __launch_bounds__(64) k%d(uint64_t* out, int iters) {" % chains)
    L.append('  asm volatile("v_mov_b32 v40, 3\\n v_mov_b32 v41, 5" ::: "v40", "v41");')
    L.append("  uint64_t t0, t1;")
    L.append('  asm volatile("s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t0));')
    L.append("  for (int it = 0; it < iters; it++) {")
    L.append('    asm volatile("%s" ::: %s);' % (asm, clob))
    L.append("  }")
    L.append('  asm volatile("s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1));')
    L.append("  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;")
    L.append("}")
L.append("int main() {")
L.append("  uint64_t* d; (void)hipMalloc(&d, 8 * 4096); uint64_t h[4096];")
for chains in (1, 2, 4, 8):
    for waves in (1, 2):
        L.append("  { const int nb = 1024 * %d, it = 20000; k%d<<<nb, 64>>>(d, 100); k%d<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();" % (waves, chains, chains))
        L.append("    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];")
        L.append('    printf("chains=%%d waves/SIMD=%%d: %%.2f clk per mad per wave, %%.2f per SIMD\\n", %d, %d, c / nb / (16.0 * it), c / nb / (16.0 * it) / %d); }' % (chains, waves, waves))
L.append("  return 0; }")
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "chain_probe.hip"), "w").write("\n".join(L) + "\n")
