// Pairing kernels on lane groups (pair_quad.h): one pairing per 32 lanes,
// two per 64-lane block.  The latency form for mid-size batches; values as
// the reference's (the Miller values bit for bit, the final exponentiation's
// result being unique).
#include "launch.h"
#include "pair_quad.h"

namespace pa {
namespace {

// out[i] = miller_loop([(p[i], q[i].prepare())]) (mod.rs:40-102); a pair with
// an infinity side gives one (mod.rs:50-54).  Held to 256 registers (two waves
// per SIMD, 96 B of scratch): 4096 pairings' Miller loops in 2.67 ms instead of
// two rounds of 1.63 (profiles/r06_lane_groups.txt, session 7); the final
// exponentiation comes in both forms below
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_pq_miller_loop(const uint64_t* __restrict__ p_aff,
                                                       const uint64_t* __restrict__ q_aff,
                                                       uint64_t* __restrict__ out, size_t n) {
    const int lane = threadIdx.x;
    const size_t i = (size_t)blockIdx.x * 2 + (lane >> 5);
    if (i >= n) return;   // whole groups leave together
    const dq::Lc l = dq::lctx(lane, pq::NQ);
    const uint64_t* p = p_aff + 13 * i;
    const uint64_t* q = q_aff + 25 * i;
    pq::E12 f;
    if (((p[12] | q[24]) & 0xff) != 0) {
        f = pq::e12_one(l);
    } else {
        const dq::Q<1> px = pq::load_q(p, l), py = pq::load_q(p + 6, l);
        const pq::E2 qx = {pq::load_q(q, l), pq::load_q(q + 6, l)};
        const pq::E2 qy = {pq::load_q(q + 12, l), pq::load_q(q + 18, l)};
        f = pq::miller_loop(px, py, qx, qy, l);
    }
    pq::store12(out + 72 * i, f, false, lane & 31);
}

// out[i] = final_exponentiation(in[i]) (mod.rs:104-160); ok[i] = 0 and a zero
// output iff in[i] == 0 (mod.rs:108); in place allowed (the group reads its
// record before it writes)
__device__ __forceinline__ void pq_final_exp_body(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n) {
    const int lane = threadIdx.x;
    const size_t i = (size_t)blockIdx.x * 2 + (lane >> 5);
    if (i >= n) return;
    const dq::Lc l = dq::lctx(lane, pq::NQ);
    const pq::E12 f = pq::load12(in + 72 * i, l);
    bool good = true;
    const pq::E12 r = pq::final_exp(f, good, l);
    pq::store12(out + 72 * i, r, !good, lane & 31);
    if (ok && (lane & 31) == 0) ok[i] = good ? 1 : 0;
}
// one wave per SIMD (512 registers, 476 B of scratch) -- rounds of 2048 ...
__global__ void __launch_bounds__(64) k_pq_final_exp(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n) {
    pq_final_exp_body(in, out, ok, n);
}
// ... or two (256 registers, 2 KB of scratch): slower per wave (2048 pairs:
// 2.33 vs 2.17 ms) but 4096 at once (3.80 ms instead of two rounds, 4.33)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_pq_final_exp2w(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n) {
    pq_final_exp_body(in, out, ok, n);
}

}  // namespace

hipError_t launch_pq_miller_loop(const uint64_t* p, const uint64_t* q, uint64_t* out, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 0x1fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pq_miller_loop, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, s, p, q, out, n);
    return hipGetLastError();
}
hipError_t launch_pq_final_exp(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 0x1fffffffull) return hipErrorInvalidValue;
    // one round at one wave per SIMD holds 8 records per CU (4 SIMDs x 2 per
    // wave; 2048 on the 256 CUs of an MI355X)
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
        cus = 256;
    if (n > (size_t)8 * (size_t)cus)
        hipLaunchKernelGGL(k_pq_final_exp2w, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, s, in, out, ok, n);
    else
        hipLaunchKernelGGL(k_pq_final_exp, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, s, in, out, ok, n);
    return hipGetLastError();
}

}  // namespace pa
