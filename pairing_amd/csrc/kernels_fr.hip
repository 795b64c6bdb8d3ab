// Scalar-field (Fr) batch kernels (SURVEY.md §8 f, rank 4: fr.rs:276-646).
//
// One element per lane; operands are the reference's in-memory order (AoS,
// 4 x u64 per Fr), read with two 16-byte loads per lane: a wave reads 64
// contiguous 32-byte records = 2 KiB, every byte used.  The multiply batch is
// HBM-bound (96 B per 64 v_mad_u64_u32 products + 64 reduction products).
#include "fr.h"
#include "launch.h"

namespace pa {

// Field::mul_assign over a batch (fr.rs:438-465), grid-stride; PF = 1
// prefetches the next element's operands before the current multiply (see
// k_fq_mul_batch).
template <int PF>
__global__ void __launch_bounds__(256) k_fr_mul_batch(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                       uint64_t* __restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (PF) {
        if (i >= n) return;
        Fr x, y;
        fr_load(x, a + 4 * i);
        fr_load(y, b + 4 * i);
        for (;;) {
            const size_t j = i + stride;
            Fr xn, yn;
            if (j < n) {
                fr_load(xn, a + 4 * j);
                fr_load(yn, b + 4 * j);
            }
            Fr z;
            fr_mul(z, x, y);
            fr_store(out + 4 * i, z);
            if (j >= n) break;
            x = xn;
            y = yn;
            i = j;
        }
    } else {
        for (; i < n; i += stride) {
            Fr x, y, z;
            fr_load(x, a + 4 * i);
            fr_load(y, b + 4 * i);
            fr_mul(z, x, y);
            fr_store(out + 4 * i, z);
        }
    }
}

template <int OP>
__global__ void __launch_bounds__(64) k_fr_op(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                              uint64_t* __restrict__ out, uint8_t* __restrict__ flag,
                                              const uint64_t* __restrict__ exp, int exp_words, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr x, z;
    fr_load(x, a + 4 * i);
    if constexpr (OP == FR_MUL || OP == FR_ADD || OP == FR_SUB) {
        Fr y;
        fr_load(y, b + 4 * i);
        if constexpr (OP == FR_MUL) fr_mul(z, x, y);
        if constexpr (OP == FR_ADD) fr_add(z, x, y);
        if constexpr (OP == FR_SUB) fr_sub(z, x, y);
    } else if constexpr (OP == FR_SQR) {
        fr_sqr(z, x);
    } else if constexpr (OP == FR_DBL) {
        fr_dbl(z, x);
    } else if constexpr (OP == FR_NEG) {
        fr_neg(z, x);
    } else if constexpr (OP == FR_INV) {
        const bool k = fr_inv(z, x);
        if (!k) fr_zero(z);
        flag[i] = k ? 1 : 0;
    } else if constexpr (OP == FR_FROM_REPR) {
        flag[i] = fr_from_repr(z, x) ? 1 : 0;
    } else if constexpr (OP == FR_INTO_REPR) {
        fr_into_repr(z, x);
    } else if constexpr (OP == FR_POW) {
        fr_pow(z, x, exp, exp_words);
    } else if constexpr (OP == FR_LEGENDRE) {
        flag[i] = (uint8_t)(int8_t)fr_legendre(x);
        return;
    } else if constexpr (OP == FR_SQRT) {
        flag[i] = fr_sqrt(z, x) ? 1 : 0;
    }
    fr_store(out + 4 * i, z);
}

static inline unsigned fr_blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_fr_mul_batch(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    const StreamCfg c = stream_cfg();
    if (blocks > c.max_blocks) blocks = c.max_blocks;
    // 27000 B of (unused) dynamic LDS per 256-thread block caps residency at 5
    // waves per SIMD, as for config 2 (k_fq_mul_batch_fl): 21.2 vs 22.2-22.3 us
    // at 2^20 uncapped; nontemporal loads / stores were 1.5 us slower
    // (profiles/r04_fr_fq_ab.txt); PA_FR_LDS overrides it
    static const unsigned lds = [] {
        const char* e = getenv("PA_FR_LDS");
        return e ? (unsigned)atoi(e) : 27000u;
    }();
    if (c.prefetch)
        hipLaunchKernelGGL(k_fr_mul_batch<1>, dim3((unsigned)blocks), dim3(256), lds, stream, a, b, out, n);
    else
        hipLaunchKernelGGL(k_fr_mul_batch<0>, dim3((unsigned)blocks), dim3(256), lds, stream, a, b, out, n);
    return hipGetLastError();
}

hipError_t launch_fr_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, uint8_t* flag,
                        const uint64_t* exp, int exp_words, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 g(fr_blocks_for(n, 64)), bl(64);
    switch (op) {
#define PA_CASE(OPV) \
    case OPV: hipLaunchKernelGGL(k_fr_op<OPV>, g, bl, 0, stream, a, b, out, flag, exp, exp_words, n); break;
        PA_CASE(FR_MUL)
        PA_CASE(FR_SQR)
        PA_CASE(FR_ADD)
        PA_CASE(FR_SUB)
        PA_CASE(FR_DBL)
        PA_CASE(FR_NEG)
        PA_CASE(FR_INV)
        PA_CASE(FR_FROM_REPR)
        PA_CASE(FR_INTO_REPR)
        PA_CASE(FR_POW)
        PA_CASE(FR_LEGENDRE)
        PA_CASE(FR_SQRT)
#undef PA_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace pa
