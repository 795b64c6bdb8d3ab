// Device-side scalar field Fr of BLS12-381 for gfx950 (SURVEY.md §8 f, rank 4).
//
// Representation: 8 x u32 little-endian words, Montgomery form with
// R = 2^256 -- the reference's R (src/bls12_381/fr.rs:18-25), so every value
// is the same canonical (< r) bit pattern as the reference's `Fr` and loads /
// stores are the reference's in-memory order (4 x u64 LE, fr.rs:58).
//
// Multiplication is 32-bit-word CIOS on v_mad_u64_u32 (there is no 64x64
// multiply on CDNA4; bignum work gains nothing from MFMA).  Every operation
// returns the canonical value, so results equal the reference's bit for bit
// whatever the algorithm (e.g. Fermat inversion instead of the reference's
// binary Euclid, fr.rs:377-431: the inverse is unique).
//   reference: mul_assign fr.rs:438-465 + mont_reduce fr.rs:520-572,
//              square fr.rs:467-500, add/double/sub/negate fr.rs:341-375,
//              from_repr/into_repr fr.rs:279-303, legendre/sqrt fr.rs:574-646,
//              Field::pow src/lib.rs:306-324
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef PA_DEV
#define PA_DEV __device__ __forceinline__
#endif

namespace pa {

struct Fr {
    uint32_t w[8];
};

// r, little-endian 32-bit words (fr.rs:4-10)
PA_DEV uint32_t fr_r_word(int i) {
    switch (i) {
        case 0: return 0x00000001u; case 1: return 0xffffffffu;
        case 2: return 0xfffe5bfeu; case 3: return 0x53bda402u;
        case 4: return 0x09a1d805u; case 5: return 0x3339d808u;
        case 6: return 0x299d7d48u; default: return 0x73eda753u;
    }
}
constexpr uint32_t kFrInv32 = 0xffffffffu;  // -r^-1 mod 2^32 (r = 1 mod 2^32; fr.rs:37 low half)

// R mod r = Montgomery one (fr.rs:19-25)
PA_DEV void fr_one(Fr& o) {
    o.w[0] = 0xfffffffeu; o.w[1] = 0x00000001u; o.w[2] = 0x00034802u; o.w[3] = 0x5884b7fau;
    o.w[4] = 0xecbc4ff5u; o.w[5] = 0x998c4fefu; o.w[6] = 0xacc5056fu; o.w[7] = 0x1824b159u;
}
// R^2 mod r (fr.rs:28-34)
PA_DEV void fr_r2(Fr& o) {
    o.w[0] = 0xf3f29c6du; o.w[1] = 0xc999e990u; o.w[2] = 0x87925c23u; o.w[3] = 0x2b6cedcbu;
    o.w[4] = 0x7254398fu; o.w[5] = 0x05d31496u; o.w[6] = 0x9f59ff11u; o.w[7] = 0x0748d9d9u;
}
// 2^32-th root of unity, Montgomery form (fr.rs:51-56)
PA_DEV void fr_root_of_unity(Fr& o) {
    o.w[0] = 0x5f0e466au; o.w[1] = 0xb9b58d8cu; o.w[2] = 0x1819d7ecu; o.w[3] = 0x5b1b4c80u;
    o.w[4] = 0x52a31e64u; o.w[5] = 0x0af53ae3u; o.w[6] = 0x19e9b27bu; o.w[7] = 0x5bf3addau;
}

PA_DEV void fr_zero(Fr& r) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = 0;
}
PA_DEV bool fr_is_zero(const Fr& a) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= a.w[i];
    return acc == 0;
}
PA_DEV bool fr_eq(const Fr& a, const Fr& b) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= a.w[i] ^ b.w[i];
    return acc == 0;
}
PA_DEV bool fr_is_one(const Fr& a) {
    Fr o;
    fr_one(o);
    return fr_eq(a, o);
}

// t < 2r (t fits 8 words since 2r < 2^256): r = t >= r ? t - r : t.  Also the
// validity test of from_repr (fr.rs:506-508): returns true iff t < r.
PA_DEV bool fr_reduce_once(Fr& r, const uint32_t t[8]) {
    uint32_t d[8];
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t s = (uint64_t)t[i] - fr_r_word(i) - borrow;
        d[i] = (uint32_t)s;
        borrow = (uint32_t)(s >> 32) & 1u;
    }
    const bool lt = borrow != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = lt ? t[i] : d[i];
    return lt;
}

PA_DEV void fr_add(Fr& r, const Fr& a, const Fr& b) {  // fr.rs:341-348
    uint32_t t[8];
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)a.w[i] + b.w[i];
        t[i] = (uint32_t)c;
        c >>= 32;
    }
    fr_reduce_once(r, t);  // a + b < 2r < 2^256: no carry out
}
PA_DEV void fr_dbl(Fr& r, const Fr& a) { fr_add(r, a, a); }  // fr.rs:350-357
PA_DEV void fr_sub(Fr& r, const Fr& a, const Fr& b) {         // fr.rs:359-367
    uint32_t t[8];
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t s = (uint64_t)a.w[i] - b.w[i] - borrow;
        t[i] = (uint32_t)s;
        borrow = (uint32_t)(s >> 32) & 1u;
    }
    // on borrow add r back (mask instead of a branch)
    const uint32_t mask = 0u - borrow;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)t[i] + (fr_r_word(i) & mask);
        r.w[i] = (uint32_t)c;
        c >>= 32;
    }
}
PA_DEV void fr_neg(Fr& r, const Fr& a) {  // fr.rs:369-375 (0 - a is r - a, and 0 for 0)
    Fr z;
    fr_zero(z);
    fr_sub(r, z, a);
}

// CIOS Montgomery product a*b*2^-256 mod r (fr.rs:438-465 + 520-572)
PA_DEV void fr_mul(Fr& r, const Fr& a, const Fr& b) {
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t p = (uint64_t)a.w[j] * b.w[i] + t[j] + c;
            t[j] = (uint32_t)p;
            c = p >> 32;
        }
        uint64_t s = (uint64_t)t[8] + c;
        t[8] = (uint32_t)s;
        t[9] = (uint32_t)(s >> 32);
        const uint32_t m = t[0] * kFrInv32;
        uint64_t p = (uint64_t)m * fr_r_word(0) + t[0];
        c = p >> 32;
#pragma unroll
        for (int j = 1; j < 8; j++) {
            p = (uint64_t)m * fr_r_word(j) + t[j] + c;
            t[j - 1] = (uint32_t)p;
            c = p >> 32;
        }
        s = (uint64_t)t[8] + c;
        t[7] = (uint32_t)s;
        t[8] = t[9] + (uint32_t)(s >> 32);
    }
    fr_reduce_once(r, t);  // CIOS output < 2r < 2^256
}
PA_DEV void fr_sqr(Fr& r, const Fr& a) { fr_mul(r, a, a); }  // fr.rs:467-500

// Field::pow, src/lib.rs:306-324: square-and-multiply, MSB first, over
// `nwords` little-endian u64 exponent words (uniform across the wave).
PA_DEV void fr_pow(Fr& r, const Fr& a, const uint64_t* exp, int nwords) {
    Fr acc;
    fr_one(acc);
    for (int wi = nwords - 1; wi >= 0; wi--) {
        const uint64_t e = exp[wi];
        for (int bit = 63; bit >= 0; bit--) {
            fr_sqr(acc, acc);
            if ((e >> bit) & 1) fr_mul(acc, acc, a);
        }
    }
    r = acc;
}
template <int N>
PA_DEV void fr_pow_const(Fr& r, const Fr& a, const uint64_t (&exp)[N]) {
    fr_pow(r, a, exp, N);
}

// Field::inverse (fr.rs:377-431) as a^(r-2); false (None) for zero
PA_DEV bool fr_inv(Fr& r, const Fr& a) {
    const uint64_t e[4] = {0xfffffffeffffffffull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                           0x73eda753299d7d48ull};
    fr_pow_const(r, a, e);
    return !fr_is_zero(a);
}

// PrimeField::from_repr (fr.rs:279-288): false if repr >= r
PA_DEV bool fr_from_repr(Fr& r, const Fr& repr) {
    Fr t;
    const bool valid = fr_reduce_once(t, repr.w);
    Fr r2;
    fr_r2(r2);
    fr_mul(r, repr, r2);
    if (!valid) fr_zero(r);
    return valid;
}
// PrimeField::into_repr (fr.rs:290-303): Montgomery reduction of a = a * 1 * R^-1
PA_DEV void fr_into_repr(Fr& r, const Fr& a) {
    Fr one_canon;
    fr_zero(one_canon);
    one_canon.w[0] = 1;
    fr_mul(r, a, one_canon);
}

// SqrtField::legendre (fr.rs:575-590): 0 Zero, 1 QuadraticResidue, -1 QuadraticNonResidue
PA_DEV int fr_legendre(const Fr& a) {
    const uint64_t e[4] = {0x7fffffff80000000ull, 0xa9ded2017fff2dffull, 0x199cec0404d0ec02ull,
                           0x39f6d3a994cebea4ull};
    Fr s;
    fr_pow_const(s, a, e);
    if (fr_is_zero(s)) return 0;
    return fr_is_one(s) ? 1 : -1;
}

// SqrtField::sqrt (fr.rs:592-646): Tonelli-Shanks with the reference's exact
// sequence (the returned root is the reference's choice of +-root).
PA_DEV bool fr_sqrt(Fr& out, const Fr& a) {
    const int l = fr_legendre(a);
    if (l == 0) {
        out = a;
        return true;
    }
    if (l < 0) {
        fr_zero(out);
        return false;
    }
    const uint64_t t_plus_1_over_2[4] = {0x7fff2dff80000000ull, 0x04d0ec02a9ded201ull, 0x94cebea4199cec04ull,
                                         0x0000000039f6d3a9ull};
    const uint64_t t_exp[4] = {0xfffe5bfeffffffffull, 0x09a1d80553bda402ull, 0x299d7d483339d808ull,
                               0x0000000073eda753ull};
    Fr c, r, t;
    fr_root_of_unity(c);
    fr_pow_const(r, a, t_plus_1_over_2);
    fr_pow_const(t, a, t_exp);
    int m = 32;  // S, fr.rs:48
    while (!fr_is_one(t)) {
        int i = 1;
        Fr t2i;
        fr_sqr(t2i, t);
        while (!fr_is_one(t2i) && i < 32) {
            fr_sqr(t2i, t2i);
            i++;
        }
        for (int k = 0; k < m - i - 1; k++) fr_sqr(c, c);
        fr_mul(r, r, c);
        fr_sqr(c, c);
        fr_mul(t, t, c);
        m = i;
    }
    out = r;
    return true;
}

// ---- HBM <-> registers: 4 x u64 LE per element (the reference's layout) ----
PA_DEV void fr_load(Fr& r, const uint64_t* p) {
    const uint4* v = reinterpret_cast<const uint4*>(p);
    const uint4 x0 = v[0], x1 = v[1];
    r.w[0] = x0.x; r.w[1] = x0.y; r.w[2] = x0.z; r.w[3] = x0.w;
    r.w[4] = x1.x; r.w[5] = x1.y; r.w[6] = x1.z; r.w[7] = x1.w;
}
PA_DEV void fr_store(uint64_t* p, const Fr& a) {
    uint4* v = reinterpret_cast<uint4*>(p);
    v[0] = make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]);
    v[1] = make_uint4(a.w[4], a.w[5], a.w[6], a.w[7]);
}

}  // namespace pa
