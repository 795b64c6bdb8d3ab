// Materialized-G2Prepared pairing kernels, one pairing per lane (the
// fused Miller loop and final exponentiation of the hot path are the
// generated code objects of tools/pgen, gen_launch.hip).
//
//   k_g2_prepare             G2Prepared::from_affine  (mod.rs:168-358)
//   k_miller_loop_prepared   miller_loop([(p, q_prepared)])  (mod.rs:40-102)
//   k_fq12_product           Fq12 tree product (multi-pair miller_loop)
//
// HBM records use the reference's in-memory order (include/pairing_amd.h).
#include "launch.h"
#include "pairing.h"

namespace pa {

constexpr int kAffG1Words = 13;  // {x, y, infinity+pad}
constexpr int kAffG2Words = 25;
constexpr int kPreparedWords = kNumCoeffs * 36 + 1;

__global__ void __launch_bounds__(64) k_g2_prepare(const uint64_t* __restrict__ q_aff,
                                                   uint64_t* __restrict__ prepared, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<Fq2> q;
    load_aff(q, q_aff + kAffG2Words * i);
    uint64_t* dst = prepared + kPreparedWords * i;
    Jac<Fq2> r;
    r.x = q.x;
    r.y = q.y;
    one(r.z);
    EllCoeff c;
    int k = 0;
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        doubling_step(c, r);
        store8(dst + 36 * k, c.c0); store8(dst + 36 * k + 12, c.c1); store8(dst + 36 * k + 24, c.c2);
        k++;
        if (((kBlsX >> 1) >> bit) & 1) {
            addition_step(c, r, q.x, q.y);
            store8(dst + 36 * k, c.c0); store8(dst + 36 * k + 12, c.c1); store8(dst + 36 * k + 24, c.c2);
            k++;
        }
    }
    doubling_step(c, r);
    store8(dst + 36 * k, c.c0); store8(dst + 36 * k + 12, c.c1); store8(dst + 36 * k + 24, c.c2);
    if (q.inf) {
        // reference: coeffs = vec![], infinity = true (mod.rs:169-174)
        for (int w = 0; w < kNumCoeffs * 36; w++) dst[w] = 0;
    }
    dst[kNumCoeffs * 36] = q.inf ? 1ull : 0ull;
}

__global__ void __launch_bounds__(64) k_miller_loop_prepared(const uint64_t* __restrict__ p_aff,
                                                             const uint64_t* __restrict__ prepared,
                                                             uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<Fq> p;
    load_aff(p, p_aff + kAffG1Words * i);
    const uint64_t* src = prepared + kPreparedWords * i;
    const bool qinf = (src[kNumCoeffs * 36] & 0xff) != 0;
    Fq12 f;
    one(f);
    EllCoeff c;
    int k = 0;
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        load8(c.c0, src + 36 * k); load8(c.c1, src + 36 * k + 12); load8(c.c2, src + 36 * k + 24);
        k++;
        ell(f, c, p.x, p.y);
        if (((kBlsX >> 1) >> bit) & 1) {
            load8(c.c0, src + 36 * k); load8(c.c1, src + 36 * k + 12); load8(c.c2, src + 36 * k + 24);
            k++;
            ell(f, c, p.x, p.y);
        }
        sqr(f, f);
    }
    load8(c.c0, src + 36 * k); load8(c.c1, src + 36 * k + 12); load8(c.c2, src + 36 * k + 24);
    ell(f, c, p.x, p.y);
    conjugate(f, f);
    if (p.inf || qinf) one(f);
    store(out + 72 * i, f);
}

// one tree level: work[i] *= work[i + half] for i < cnt - half
__global__ void __launch_bounds__(64) k_fq12_product_level(uint64_t* __restrict__ work, size_t cnt, size_t half) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= half || i + half >= cnt) return;
    Fq12 x, y;
    load(x, work + 72 * i);
    load(y, work + 72 * (i + half));
    mul(x, x, y);
    store(work + 72 * i, x);
}

static inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_g2_prepare(const uint64_t* q_aff, uint64_t* prepared, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_g2_prepare, dim3(blocks_for(n, 64)), dim3(64), 0, stream, q_aff, prepared, n);
    return hipGetLastError();
}
hipError_t launch_miller_loop_prepared(const uint64_t* p_aff, const uint64_t* prepared, uint64_t* out,
                                       size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_miller_loop_prepared, dim3(blocks_for(n, 64)), dim3(64), 0, stream, p_aff, prepared,
                       out, n);
    return hipGetLastError();
}
hipError_t launch_fq12_product(uint64_t* work, size_t n, uint64_t* out, hipStream_t stream) {
    if (n == 0) return hipErrorInvalidValue;
    size_t cnt = n;
    while (cnt > 1) {
        const size_t half = (cnt + 1) / 2;
        hipLaunchKernelGGL(k_fq12_product_level, dim3(blocks_for(half, 64)), dim3(64), 0, stream, work, cnt, half);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        cnt = half;
    }
    if (out == work) return hipSuccess;
    return hipMemcpyAsync(out, work, 72 * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream);
}

}  // namespace pa
