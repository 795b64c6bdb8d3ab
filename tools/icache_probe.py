#!/usr/bin/env python3
"""Emit tools/icache_probe.hip: loops whose bodies hold K copies of the
28-bit Montgomery product inline (~3.8 KB of code each), to measure how
time per product grows once a loop body exceeds the instruction cache."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_fl import leaf_sop

body, out, clob = leaf_sop(1)
ins = [l for l in body if not l.endswith(":") and not l.startswith(".") and not l.startswith("s_setpc")]
asm = "\\n".join(ins)
clobs = ", ".join('"v%d"' % i for i in range(58)) + ", " + ", ".join('"s%d"' % i for i in range(80, 95)) + ', "vcc"'
K_LIST = [1, 4, 8, 16, 32, 64]
L = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdint.h>',
     '#define BODY asm volatile("%s" ::: %s);' % (asm, clobs)]
for K in K_LIST:
    L.append("__global__ void __launch_bounds__(64) k%d(uint32_t* out, int iters) {" % K)
    L.append("  for (int it = 0; it < iters; it++) {")
    L += ["    BODY"] * K
    L.append("  }")
    L.append("  if (iters < 0) out[threadIdx.x] = 1;")
    L.append("}")
L.append("int main() {")
L.append("  uint32_t* d; (void)hipMalloc(&d, 4096); hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;")
for W in (1, 2):
    for K in K_LIST:
        it = 512 // K
        L.append("  k%d<<<1024 * %d, 64>>>(d, %d); (void)hipEventRecord(e0); k%d<<<1024 * %d, 64>>>(d, %d); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);" % (K, W, it, K, W, it))
        L.append('  (void)hipEventElapsedTime(&ms, e0, e1); printf("waves/SIMD=%d K=%%3d body %%7.1f KB: %%8.3f ms, %%.1f ns per product per SIMD\\n", %d, %d * 3.8, ms, ms * 1e6 / 512 / %d);' % (W, K, K, W))
L.append("  return 0; }")
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "icache_probe.hip"), "w").write("\n".join(L) + "\n")
