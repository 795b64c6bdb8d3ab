#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void __launch_bounds__(64) k1(uint64_t* out, int iters) {
  asm volatile("v_mov_b32 v40, 3\n v_mov_b32 v41, 5" ::: "v40", "v41");
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; it++) {
    asm volatile("v_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]" ::: "v0", "v1", "v40", "v41", "vcc");
  }
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k2(uint64_t* out, int iters) {
  asm volatile("v_mov_b32 v40, 3\n v_mov_b32 v41, 5" ::: "v40", "v41");
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; it++) {
    asm volatile("v_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]" ::: "v0", "v1", "v2", "v3", "v40", "v41", "vcc");
  }
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k4(uint64_t* out, int iters) {
  asm volatile("v_mov_b32 v40, 3\n v_mov_b32 v41, 5" ::: "v40", "v41");
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; it++) {
    asm volatile("v_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[4:5], vcc, v40, v41, v[4:5]\nv_mad_u64_u32 v[6:7], vcc, v40, v41, v[6:7]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[4:5], vcc, v40, v41, v[4:5]\nv_mad_u64_u32 v[6:7], vcc, v40, v41, v[6:7]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[4:5], vcc, v40, v41, v[4:5]\nv_mad_u64_u32 v[6:7], vcc, v40, v41, v[6:7]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[4:5], vcc, v40, v41, v[4:5]\nv_mad_u64_u32 v[6:7], vcc, v40, v41, v[6:7]" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v40", "v41", "vcc");
  }
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k8(uint64_t* out, int iters) {
  asm volatile("v_mov_b32 v40, 3\n v_mov_b32 v41, 5" ::: "v40", "v41");
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int it = 0; it < iters; it++) {
    asm volatile("v_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[4:5], vcc, v40, v41, v[4:5]\nv_mad_u64_u32 v[6:7], vcc, v40, v41, v[6:7]\nv_mad_u64_u32 v[8:9], vcc, v40, v41, v[8:9]\nv_mad_u64_u32 v[10:11], vcc, v40, v41, v[10:11]\nv_mad_u64_u32 v[12:13], vcc, v40, v41, v[12:13]\nv_mad_u64_u32 v[14:15], vcc, v40, v41, v[14:15]\nv_mad_u64_u32 v[0:1], vcc, v40, v41, v[0:1]\nv_mad_u64_u32 v[2:3], vcc, v40, v41, v[2:3]\nv_mad_u64_u32 v[4:5], vcc, v40, v41, v[4:5]\nv_mad_u64_u32 v[6:7], vcc, v40, v41, v[6:7]\nv_mad_u64_u32 v[8:9], vcc, v40, v41, v[8:9]\nv_mad_u64_u32 v[10:11], vcc, v40, v41, v[10:11]\nv_mad_u64_u32 v[12:13], vcc, v40, v41, v[12:13]\nv_mad_u64_u32 v[14:15], vcc, v40, v41, v[14:15]" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v40", "v41", "vcc");
  }
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
int main() {
  uint64_t* d; (void)hipMalloc(&d, 8 * 4096); uint64_t h[4096];
  { const int nb = 1024 * 1, it = 20000; k1<<<nb, 64>>>(d, 100); k1<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 1, 1, c / nb / (16.0 * it), c / nb / (16.0 * it) / 1); }
  { const int nb = 1024 * 2, it = 20000; k1<<<nb, 64>>>(d, 100); k1<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 1, 2, c / nb / (16.0 * it), c / nb / (16.0 * it) / 2); }
  { const int nb = 1024 * 1, it = 20000; k2<<<nb, 64>>>(d, 100); k2<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 2, 1, c / nb / (16.0 * it), c / nb / (16.0 * it) / 1); }
  { const int nb = 1024 * 2, it = 20000; k2<<<nb, 64>>>(d, 100); k2<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 2, 2, c / nb / (16.0 * it), c / nb / (16.0 * it) / 2); }
  { const int nb = 1024 * 1, it = 20000; k4<<<nb, 64>>>(d, 100); k4<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 4, 1, c / nb / (16.0 * it), c / nb / (16.0 * it) / 1); }
  { const int nb = 1024 * 2, it = 20000; k4<<<nb, 64>>>(d, 100); k4<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 4, 2, c / nb / (16.0 * it), c / nb / (16.0 * it) / 2); }
  { const int nb = 1024 * 1, it = 20000; k8<<<nb, 64>>>(d, 100); k8<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 8, 1, c / nb / (16.0 * it), c / nb / (16.0 * it) / 1); }
  { const int nb = 1024 * 2, it = 20000; k8<<<nb, 64>>>(d, 100); k8<<<nb, 64>>>(d, it); (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, d, 8 * nb, hipMemcpyDeviceToHost); double c = 0; for (int b = 0; b < nb; b++) c += h[b];
    printf("chains=%d waves/SIMD=%d: %.2f clk per mad per wave, %.2f per SIMD\n", 8, 2, c / nb / (16.0 * it), c / nb / (16.0 * it) / 2); }
  return 0; }
