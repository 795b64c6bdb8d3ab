// Materialized-G2Prepared pairing kernels, one pairing per lane on the lazy
// 28-bit core (pairing_fl.h; the fused Miller loop and final exponentiation
// of the hot path are the generated code objects of tools/pgen, gen_launch.hip).
//
//   k_g2_prepare             G2Prepared::from_affine  (mod.rs:168-358)
//   k_miller_loop_prepared   miller_loop([(p, q_prepared)])  (mod.rs:40-102)
//   k_fq12_product           Fq12 tree product (multi-pair miller_loop)
//
// HBM records use the reference's in-memory order (include/pairing_amd.h).
#include "launch.h"
#include "pairing_fl.h"

namespace pa {

constexpr int kAffG1Words = 13;  // {x, y, infinity+pad}
constexpr int kAffG2Words = 25;
constexpr int kPreparedWords = kNumCoeffs * 36 + 1;

// G2Prepared::from_affine on the lazy core: 63 doubling + 5 addition steps,
// each line stored canonical as it is produced.
__global__ void __launch_bounds__(64) k_g2_prepare(const uint64_t* __restrict__ q_aff,
                                                   uint64_t* __restrict__ prepared, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t* src = q_aff + kAffG2Words * i;
    const bool qinf = (src[24] & 0xff) != 0;
    const F2<1> qx = load2(src), qy = load2(src + 12);
    uint64_t* dst = prepared + kPreparedWords * i;
    G2JacFl r{qx, qy, f2_one()};
    int k = 0;
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        store_line(dst + 36 * k++, dbl_step_fl(r));
        if (((kBlsX >> 1) >> bit) & 1) store_line(dst + 36 * k++, add_step_fl(r, qx, qy));
    }
    store_line(dst + 36 * k, dbl_step_fl(r));
    if (qinf) {
        // reference: coeffs = vec![], infinity = true (mod.rs:169-174)
        for (int w = 0; w < kNumCoeffs * 36; w++) dst[w] = 0;
    }
    dst[kNumCoeffs * 36] = qinf ? 1ull : 0ull;
}

// miller_loop over one (G1Affine, G2Prepared) pair per lane on the lazy core
__global__ void __launch_bounds__(64) k_miller_loop_prepared(const uint64_t* __restrict__ p_aff,
                                                             const uint64_t* __restrict__ prepared,
                                                             uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t* pp = p_aff + kAffG1Words * i;
    const bool pinf = (pp[12] & 0xff) != 0;
    const F<1> kx = mul(fl_load(pp), fl_c(FL_TO));
    const F<1> ky = mul(fl_load(pp + 6), fl_c(FL_TO));
    const uint64_t* src = prepared + kPreparedWords * i;
    const bool qinf = (src[kNumCoeffs * 36] & 0xff) != 0;
    F12<1> f = f12_one();
    int k = 0;
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        f = ell_fl(f, src + 36 * k++, kx, ky);
        if (((kBlsX >> 1) >> bit) & 1) f = ell_fl(f, src + 36 * k++, kx, ky);
        f = sqr(f);
    }
    f = ell_fl(f, src + 36 * k, kx, ky);
    f = red(conj(f));
    if (pinf || qinf) f = f12_one();
    store12(out + 72 * i, f);
}

// ---- one G2Prepared shared by a batch of G1 points (lib.rs:88-96: the
// caller passes the same &G2Prepared for every pair -- a verifying key's
// prepared gamma / delta) ----
//
// k_shared_line_table converts the record's 68 lines ONCE per call into the
// line table of the generated kernel pa_gen_miller_loop_shared
// (tools/pgen/kernels.py miller_loop_shared_prog, kcfg.MillerLoopSharedCfg):
// u32 word 0 = the prepared infinity flag, then from byte kSharedTableLines
// per line six 14-limb values
//   c0.c0, c0.c1, c1.c0, c1.c1 as fl_split (raw 28-bit limbs of the ABI
//   integer: the ABI -> lazy conversion rides on the products by P's
//   coordinates, as in ell_fl), c2.c0, c2.c1 as fl_from_abi.
// Every lane of the Miller loop then reads the same table words, so per
// pairing only P (104 B) crosses HBM and no G2 arithmetic runs.
__global__ void __launch_bounds__(64) k_shared_line_table(const uint64_t* __restrict__ prepared,
                                                          uint32_t* __restrict__ table) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) table[0] = (prepared[kNumCoeffs * 36] & 0xff) != 0 ? 1u : 0u;
    if (t >= kNumCoeffs * 6) return;
    const int line = t / 6, j = t % 6;
    Fq w;
    fq_load(w, prepared + 36 * line + 6 * j);
    const F<1> v = j < 4 ? fl_split(w) : fl_from_abi(w);
    uint32_t* dst = table + kSharedTableLines / 4 + kSharedLineWords * line + 14 * j;
#pragma unroll
    for (int l = 0; l < 14; l++) dst[l] = v.w[l];
}

// one tree level: work[i] *= work[i + half] for i < cnt - half
__global__ void __launch_bounds__(64) k_fq12_product_level(uint64_t* __restrict__ work, size_t cnt, size_t half) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= half || i + half >= cnt) return;
    store12(work + 72 * i, mul(load12(work + 72 * i), load12(work + 72 * (i + half))));
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
hipError_t launch_shared_line_table(const uint64_t* prepared, uint32_t* table, hipStream_t stream) {
    hipLaunchKernelGGL(k_shared_line_table, dim3(blocks_for(kNumCoeffs * 6, 64)), dim3(64), 0, stream, prepared,
                       table);
    return hipGetLastError();
}
hipError_t launch_fq12_product(uint64_t* work, size_t n, uint64_t* out, hipStream_t stream) {
    if (n == 0) return hipErrorInvalidValue;
    // up to 2^16 values: levels of 16-value products as mul12 macros on the
    // cooperative VM (~6 us per product, one workgroup per 16 values) beat the
    // one-lane tree (~117 us per level of 2); larger ones use the tree, whose
    // levels are wide enough to fill the GPU
    if (n >= 2 && n <= 65536) return launch_coop_fq12_product(work, n, out, stream);
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
