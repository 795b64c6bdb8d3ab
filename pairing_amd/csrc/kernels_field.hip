// Field-level kernels: the Fq::mul_assign batch kernel (BASELINE config 2)
// and elementwise tower kernels used by the parity tests and the C ABI.
//
// Layout: every operand is the reference's in-memory order (AoS, 6 x u64
// per Fq), read with 16-byte loads: a wave reads 64 contiguous 48-byte
// records = 3 KiB with three dwordx4 instructions, every byte used.
#include "fl.h"
#include "launch.h"
#include "pairing.h"

namespace pa {

// R^2 mod q (fq.rs:33-40), Montgomery: PrimeField::from_repr's multiplier
__constant__ const uint64_t kFqR2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL,
                                        0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};

// Fq::mul_assign over a batch, fq.rs:909-960.  Grid-stride so one launch
// covers any n with a chip-filling grid; PF = 1 software-pipelines the loop:
// the next element's operands are loaded before the current multiply, so a
// wave's loads overlap its own ~600-instruction multiply instead of every
// wave alternating a memory phase and a compute phase in lockstep.
template <int PF>
__global__ void __launch_bounds__(256) k_fq_mul_batch(const uint64_t* __restrict__ a,
                                                       const uint64_t* __restrict__ b,
                                                       uint64_t* __restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (PF) {
        if (i >= n) return;
        Fq x, y;
        fq_load(x, a + 6 * i);
        fq_load(y, b + 6 * i);
        for (;;) {
            const size_t j = i + stride;
            Fq xn, yn;
            if (j < n) {
                fq_load(xn, a + 6 * j);
                fq_load(yn, b + 6 * j);
            }
            Fq z;
            fq_mul(z, x, y);
            fq_store(out + 6 * i, z);
            if (j >= n) break;
            x = xn;
            y = yn;
            i = j;
        }
    } else {
        for (; i < n; i += stride) {
            Fq x, y, z;
            fq_load(x, a + 6 * i);
            fq_load(y, b + 6 * i);
            fq_mul(z, x, y);
            fq_store(out + 6 * i, z);
        }
    }
}

// Field::pow, lib.rs:306-324: square-and-multiply over the exponent's bits,
// most significant first (BitIterator, lib.rs:582-610); leading zeros square
// one, so starting at the top set bit gives the same value.
template <class F>
PA_DEV void field_pow(F& r, const F& x, const uint64_t* exp, int words) {
    one(r);
    bool started = false;
#pragma unroll 1
    for (int w = words - 1; w >= 0; w--) {
        const uint64_t e = exp[w];
#pragma unroll 1
        for (int bit = 63; bit >= 0; bit--) {
            if (started) sqr(r, r);
            if ((e >> bit) & 1) {
                if (started) mul(r, r, x);
                else r = x;
                started = true;
            }
        }
    }
}

static inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// Config-2 kernel: Fq::mul_assign on the lazy 28-bit core's product leaf.  The
// 14-limb Montgomery product divides by R' = 2^392, the reference's by
// R = 2^384 (fq.rs:909-960), so one operand enters shifted left by 8 bits:
// a 2^8 < 2^389 still splits into 14 limbs below 2^28 (limb bound 1), and
//   (a 2^8) b / 2^392 = a b / 2^384  (mod q),  output < (2^8 q^2 / R' + q) < 2q,
// which one conditional subtraction makes canonical.  392 carry-free
// multiply-accumulates instead of 292 multiply-accumulates + 288 carries.
PA_DEV F<1> fl_split_shl8(const Fq& x) {
    F<1> r;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        const int bit = 28 * i - 8;   // limb i of x 2^8 = bits [bit, bit + 28) of x
        uint64_t v;
        if (bit < 0) {
            v = (uint64_t)x.w[0] << 8;
        } else {
            const int wi = bit >> 5, sh = bit & 31;
            v = (uint64_t)x.w[wi];
            if (wi + 1 < 12) v |= (uint64_t)x.w[wi + 1] << 32;
            v >>= sh;
        }
        r.w[i] = (uint32_t)v & FL_MASK;
    }
    return r;
}
__global__ void __launch_bounds__(256) k_fq_mul_batch_fl(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                          uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq x, y;
    fq_load(x, a + 6 * i);
    fq_load(y, b + 6 * i);
    const F<1> xs = fl_split_shl8(x), ys = fl_split(y);
    F<1> z;
    fl_mul_leaf(z.w, xs.w, ys.w);
    fq_store(out + 6 * i, fl_pack_canon(z));
}

// Config 2 with the device layout SURVEY.md section 8(d) names (SoA): word j of
// element i at a[j n + i], so each of the six 8-byte loads / stores of a wave
// is one contiguous 512-byte run.  Same product and canonicalization as
// k_fq_mul_batch_fl.
__global__ void __launch_bounds__(256) k_fq_mul_batch_soa(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                           uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq x, y;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const uint64_t u = a[j * n + i], v = b[j * n + i];
        x.w[2 * j] = (uint32_t)u;
        x.w[2 * j + 1] = (uint32_t)(u >> 32);
        y.w[2 * j] = (uint32_t)v;
        y.w[2 * j + 1] = (uint32_t)(v >> 32);
    }
    const F<1> xs = fl_split_shl8(x), ys = fl_split(y);
    F<1> z;
    fl_mul_leaf(z.w, xs.w, ys.w);
    const Fq r = fl_pack_canon(z);
#pragma unroll
    for (int j = 0; j < 6; j++) out[j * n + i] = (uint64_t)r.w[2 * j] | ((uint64_t)r.w[2 * j + 1] << 32);
}
hipError_t launch_fq_mul_batch_soa(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    static const unsigned lds = [] {
        const char* e = getenv("PA_FQ_LDS");
        return e ? (unsigned)atoi(e) : 27000u;
    }();
    hipLaunchKernelGGL(k_fq_mul_batch_soa, dim3(blocks_for(n, 256)), dim3(256), lds, stream, a, b, out, n);
    return hipGetLastError();
}

// Probe for config 2 (PA_FQ_VARIANT=9, not the product path): the same record
// traffic with no multiply (z = x ^ y), i.e. the access-pattern bound: 25.0 us at
// 2^20 against 29.0 us with the multiply (profiles/r02_fq_variants_s7.txt; a
// wave-coalesced LDS-staged form of the multiply kernel measured 29.4-29.7 us).
__global__ void __launch_bounds__(256) k_fq_xor_probe(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                       uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq x, y;
    fq_load(x, a + 6 * i);
    fq_load(y, b + 6 * i);
#pragma unroll
    for (int k = 0; k < 12; k++) x.w[k] ^= y.w[k];
    fq_store(out + 6 * i, x);
}
template <int OP>
__global__ void __launch_bounds__(64) k_field_op(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                 uint64_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                 size_t n, int param) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if constexpr (OP == OP_FQ_MUL || OP == OP_FQ_ADD || OP == OP_FQ_SUB) {
        Fq x, y, z;
        fq_load(x, a + 6 * i);
        fq_load(y, b + 6 * i);
        if constexpr (OP == OP_FQ_MUL) fq_mul(z, x, y);
        if constexpr (OP == OP_FQ_ADD) fq_add(z, x, y);
        if constexpr (OP == OP_FQ_SUB) fq_sub(z, x, y);
        fq_store(out + 6 * i, z);
    } else if constexpr (OP == OP_FQ_SQR || OP == OP_FQ_INV) {
        Fq x, z;
        fq_load(x, a + 6 * i);
        if constexpr (OP == OP_FQ_SQR) fq_sqr(z, x);
        if constexpr (OP == OP_FQ_INV) {
            bool k = fq_inv(z, x);
            if (!k) fq_zero(z);
            ok[i] = k ? 1 : 0;
        }
        fq_store(out + 6 * i, z);
    } else if constexpr (OP == OP_FQ_FROM_REPR || OP == OP_FQ_INTO_REPR) {
        Fq x, z;
        fq_load(x, a + 6 * i);
        if constexpr (OP == OP_FQ_FROM_REPR) {
            // PrimeField::from_repr, fq.rs:747-756: a repr < q (is_valid), times R^2
            int c = 0;
#pragma unroll
            for (int k = 11; k >= 0; k--)
                if (c == 0 && x.w[k] != q_word(k)) c = x.w[k] < q_word(k) ? -1 : 1;
            const bool valid = c < 0;
            Fq r2;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                r2.w[2 * k] = (uint32_t)kFqR2[k];
                r2.w[2 * k + 1] = (uint32_t)(kFqR2[k] >> 32);
            }
            if (valid) fq_mul(z, x, r2);
            else fq_zero(z);
            ok[i] = valid ? 1 : 0;
        } else {
            // PrimeField::into_repr, fq.rs:758-775: mont_reduce of the words, a * 1 * R^-1
            Fq one_raw;
            fq_zero(one_raw);
            one_raw.w[0] = 1;
            fq_mul(z, x, one_raw);
        }
        fq_store(out + 6 * i, z);
    } else if constexpr (OP == OP_FQ_POW) {
        Fq x, z;
        fq_load(x, a + 6 * i);
        field_pow(z, x, b, param);
        fq_store(out + 6 * i, z);
    } else if constexpr (OP == OP_FQ2_INV || OP == OP_FQ2_FROB) {
        Fq2 x, z;
        load(x, a + 12 * i);
        if constexpr (OP == OP_FQ2_INV) {
            const bool k = inverse(z, x);
            if (!k) zero(z);
            ok[i] = k ? 1 : 0;
        } else {
            frobenius_map(z, x, param);
        }
        store(out + 12 * i, z);
    } else if constexpr (OP == OP_FQ6_SQR || OP == OP_FQ6_INV || OP == OP_FQ6_FROB) {
        Fq6 x, z;
        load(x, a + 36 * i);
        if constexpr (OP == OP_FQ6_SQR) {
            sqr(z, x);
        } else if constexpr (OP == OP_FQ6_INV) {
            const bool k = inverse(z, x);
            if (!k) zero(z);
            ok[i] = k ? 1 : 0;
        } else {
            frobenius_map(z, x, param);
        }
        store(out + 36 * i, z);
    } else if constexpr (OP == OP_FQ2_MUL || OP == OP_FQ2_SQR) {
        Fq2 x, y, z;
        load(x, a + 12 * i);
        if constexpr (OP == OP_FQ2_MUL) {
            load(y, b + 12 * i);
            mul(z, x, y);
        } else {
            sqr(z, x);
        }
        store(out + 12 * i, z);
    } else if constexpr (OP == OP_FQ6_MUL) {
        Fq6 x, y, z;
        load(x, a + 36 * i);
        load(y, b + 36 * i);
        mul(z, x, y);
        store(out + 36 * i, z);
    } else {
        Fq12 x, z;
        load(x, a + 72 * i);
        if constexpr (OP == OP_FQ12_MUL) {
            Fq12 y;
            load(y, b + 72 * i);
            mul(z, x, y);
        } else if constexpr (OP == OP_FQ12_SQR) {
            sqr(z, x);
        } else if constexpr (OP == OP_FQ12_INV) {
            bool k = inverse(z, x);
            if (!k) { zero(z.c0); zero(z.c1); }
            ok[i] = k ? 1 : 0;
        } else if constexpr (OP == OP_FQ12_FROB) {
            frobenius_map(z, x, param);
        } else if constexpr (OP == OP_FQ12_CYC_SQR) {
            cyclotomic_sqr(z, x);
        } else if constexpr (OP == OP_FQ12_POW) {
            field_pow(z, x, b, param);
        }
        store(out + 72 * i, z);
    }
}

__global__ void __launch_bounds__(64) k_fq12_mul_by_014(const uint64_t* __restrict__ a,
                                                        const uint64_t* __restrict__ c0,
                                                        const uint64_t* __restrict__ c1,
                                                        const uint64_t* __restrict__ c4,
                                                        uint64_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fq12 x, z;
    Fq2 d0, d1, d4;
    load(x, a + 72 * i);
    load(d0, c0 + 12 * i);
    load(d1, c1 + 12 * i);
    load(d4, c4 + 12 * i);
    mul_by_014(z, x, d0, d1, d4);
    store(out + 72 * i, z);
}

hipError_t launch_fq_mul_batch(const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n,
                               hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // Default: the lazy 28-bit core (k_fq_mul_batch_fl, 29.4 us at 2^20
    // against 32.5 us for the 12 x u32 kernel, profiles/r02_fq_variants.txt;
    // wave-coalesced LDS-DMA transfers measured 3 us slower in round 4,
    // profiles/r04_fq_glds_icache.txt; nontemporal loads / stores 10 us slower,
    // a grid-stride prefetching form 3-4 us slower, profiles/r04_fr_fq_ab.txt).
    // PA_FQ_VARIANT=0 selects the 12 x u32 streaming kernel for A/B runs.
    static const int variant = [] {
        const char* e = getenv("PA_FQ_VARIANT");
        return e ? atoi(e) : 4;
    }();
    if (variant == 9) {
        hipLaunchKernelGGL(k_fq_xor_probe, dim3(blocks_for(n, 256)), dim3(256), 0, stream, a, b, out, n);
        return hipGetLastError();
    }
    if (variant != 0) {
        // 27000 B of (unused) dynamic LDS per 256-thread block caps residency at
        // 5 waves per SIMD: fewer waves finish their multiplies together after the
        // last loads land (29.0 vs 30.0-30.3 us at 2^20; 3 waves: 32.2 us;
        // profiles/r02_fq_occupancy.txt).  PA_FQ_LDS overrides it for A/B runs.
        static const unsigned lds = [] {
            const char* e = getenv("PA_FQ_LDS");
            return e ? (unsigned)atoi(e) : 27000u;
        }();
        hipLaunchKernelGGL(k_fq_mul_batch_fl, dim3(blocks_for(n, 256)), dim3(256), lds, stream, a, b, out, n);
        return hipGetLastError();
    }
    size_t blocks = (n + 255) / 256;
    const StreamCfg c = stream_cfg();
    if (blocks > c.max_blocks) blocks = c.max_blocks;
    if (c.prefetch)
        hipLaunchKernelGGL(k_fq_mul_batch<1>, dim3((unsigned)blocks), dim3(256), 0, stream, a, b, out, n);
    else
        hipLaunchKernelGGL(k_fq_mul_batch<0>, dim3((unsigned)blocks), dim3(256), 0, stream, a, b, out, n);
    return hipGetLastError();
}

hipError_t launch_field_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, uint8_t* ok,
                           size_t n, int param, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 g(blocks_for(n, 64)), bl(64);
    switch (op) {
#define PA_CASE(OPV) \
    case OPV: hipLaunchKernelGGL(k_field_op<OPV>, g, bl, 0, stream, a, b, out, ok, n, param); break;
        PA_CASE(OP_FQ_MUL)
        PA_CASE(OP_FQ_SQR)
        PA_CASE(OP_FQ_ADD)
        PA_CASE(OP_FQ_SUB)
        PA_CASE(OP_FQ_INV)
        PA_CASE(OP_FQ_FROM_REPR)
        PA_CASE(OP_FQ_INTO_REPR)
        PA_CASE(OP_FQ2_MUL)
        PA_CASE(OP_FQ2_SQR)
        PA_CASE(OP_FQ6_MUL)
        PA_CASE(OP_FQ12_MUL)
        PA_CASE(OP_FQ12_SQR)
        PA_CASE(OP_FQ12_INV)
        PA_CASE(OP_FQ12_FROB)
        PA_CASE(OP_FQ12_CYC_SQR)
        PA_CASE(OP_FQ2_INV)
        PA_CASE(OP_FQ2_FROB)
        PA_CASE(OP_FQ6_SQR)
        PA_CASE(OP_FQ6_INV)
        PA_CASE(OP_FQ6_FROB)
        PA_CASE(OP_FQ_POW)
        PA_CASE(OP_FQ12_POW)
#undef PA_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_fq12_mul_by_014(const uint64_t* a, const uint64_t* c0, const uint64_t* c1,
                                  const uint64_t* c4, uint64_t* out, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fq12_mul_by_014, dim3(blocks_for(n, 64)), dim3(64), 0, stream, a, c0, c1, c4, out, n);
    return hipGetLastError();
}

}  // namespace pa
