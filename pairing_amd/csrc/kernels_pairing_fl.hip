// Pairing kernels on the lazy 28-bit-limb core (pairing_fl.h): one pairing
// per lane, no stack -- every value lives in VGPRs/AGPRs and the Montgomery
// products are register-convention leaf calls.
//
//   k_miller_loop_fl   miller_loop([(p, q.prepare())])  (mod.rs:40-102)
//   k_final_exp_fl     final_exponentiation             (mod.rs:104-160)
//
// HBM records use the reference's in-memory order (include/pairing_amd.h):
// G1Affine 13 u64 (x, y, infinity), G2Affine 25 u64, Fq12 72 u64.
#include "launch.h"
#include "pairing_fl.h"

namespace pa {
namespace {

// affine records are 8-byte aligned (104 B / 200 B)
PA_DEV F<1> load_aff_fq(const uint64_t* p) {
    const uint2* v = reinterpret_cast<const uint2*>(p);
    Fq x;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const uint2 t = v[i];
        x.w[2 * i] = t.x;
        x.w[2 * i + 1] = t.y;
    }
    return fl_from_abi(x);
}

__global__ void __launch_bounds__(64) k_miller_loop_fl(const uint64_t* __restrict__ p_aff,
                                                       const uint64_t* __restrict__ q_aff,
                                                       uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t* p = p_aff + 13 * i;
    const uint64_t* q = q_aff + 25 * i;
    __shared__ uint32_t lds[84 * 64];
    const fl::PQ pq{lds + threadIdx.x};
    pq.put(0, load_aff_fq(p));
    pq.put(1, load_aff_fq(p + 6));
    pq.put(2, load_aff_fq(q));
    pq.put(3, load_aff_fq(q + 6));
    pq.put(4, load_aff_fq(q + 12));
    pq.put(5, load_aff_fq(q + 18));
    const bool inf = ((p[12] | q[24]) & 0xff) != 0;
    F12<1> f = fl::miller_loop(pq);
    if (inf) f = f12_one();  // mod.rs:50-54: pairs with an infinity are skipped
    store12(out + 72 * i, f);
}

__global__ void __launch_bounds__(64) k_final_exp_fl(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                     uint8_t* __restrict__ ok, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool good;
    F12<1> r = fl::final_exponentiation(load12(in + 72 * i), good);
    if (!good) r = {f6_zero(), f6_zero()};
    store12(out + 72 * i, r);
    if (ok) ok[i] = good ? 1 : 0;
}

inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

hipError_t launch_miller_loop_fl(const uint64_t* p_aff, const uint64_t* q_aff, uint64_t* out, size_t n,
                                 hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_miller_loop_fl, dim3(blocks_for(n, 64)), dim3(64), 0, stream, p_aff, q_aff, out, n);
    return hipGetLastError();
}
hipError_t launch_final_exp_fl(const uint64_t* in, uint64_t* out, uint8_t* ok, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_final_exp_fl, dim3(blocks_for(n, 64)), dim3(64), 0, stream, in, out, ok, n);
    return hipGetLastError();
}

}  // namespace pa
