// Device-side base field Fq of BLS12-381 for gfx950 (CDNA4).
//
// Representation in registers: 12 x u32 little-endian words, Montgomery form
// with R = 2^384 -- the same R as the reference's 6 x u64 limbs
// (src/bls12_381/fq.rs:22-30), so a*b*R^-1 mod q is the same number and every
// value is the same canonical (< q) bit pattern as the reference's `Fq`.
// Memory layout (HBM) is the reference's in-memory order: 6 x u64 LE per element.
//
// Multiplication is 32-bit-word CIOS Montgomery (a*b + m*q interleaved, one
// row per word), built on v_mad_u64_u32 -- there is no 64x64->128 multiply on
// CDNA4 and bignum work gains nothing from MFMA.
//   reference: Fq::mul_assign fq.rs:909-960 + mont_reduce fq.rs:1036-1122
//              add/double/sub/negate fq.rs:812-847, reduce fq.rs:1029-1034
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PA_DEV __device__ __forceinline__

namespace pa {

struct Fq {
    uint32_t w[12];
};

// q, little-endian 32-bit words
#define PA_Q0 0xffffaaabu
#define PA_Q1 0xb9feffffu
#define PA_Q2 0xb153ffffu
#define PA_Q3 0x1eabfffeu
#define PA_Q4 0xf6b0f624u
#define PA_Q5 0x6730d2a0u
#define PA_Q6 0xf38512bfu
#define PA_Q7 0x64774b84u
#define PA_Q8 0x434bacd7u
#define PA_Q9 0x4b1ba7b6u
#define PA_Q10 0x397fe69au
#define PA_Q11 0x1a0111eau
#define PA_INV32 0xfffcfffdu  // -q^-1 mod 2^32

PA_DEV uint32_t q_word(int i) {
    switch (i) {
        case 0: return PA_Q0;  case 1: return PA_Q1;  case 2: return PA_Q2;
        case 3: return PA_Q3;  case 4: return PA_Q4;  case 5: return PA_Q5;
        case 6: return PA_Q6;  case 7: return PA_Q7;  case 8: return PA_Q8;
        case 9: return PA_Q9;  case 10: return PA_Q10; default: return PA_Q11;
    }
}

// R mod q (Montgomery one), little-endian 32-bit words (fq.rs:22-30)
#define PA_R0 0x0002fffdu
#define PA_R1 0x76090000u
#define PA_R2 0xc40c0002u
#define PA_R3 0xebf4000bu
#define PA_R4 0x53c758bau
#define PA_R5 0x5f489857u
#define PA_R6 0x70525745u
#define PA_R7 0x77ce5853u
#define PA_R8 0xa256ec6du
#define PA_R9 0x5c071a97u
#define PA_R10 0xfa80e493u
#define PA_R11 0x15f65ec3u

PA_DEV void fq_zero(Fq& r) {
#pragma unroll
    for (int i = 0; i < 12; i++) r.w[i] = 0;
}
PA_DEV void fq_one(Fq& r) {
    r.w[0] = PA_R0; r.w[1] = PA_R1; r.w[2] = PA_R2; r.w[3] = PA_R3;
    r.w[4] = PA_R4; r.w[5] = PA_R5; r.w[6] = PA_R6; r.w[7] = PA_R7;
    r.w[8] = PA_R8; r.w[9] = PA_R9; r.w[10] = PA_R10; r.w[11] = PA_R11;
}
PA_DEV bool fq_is_zero(const Fq& a) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) acc |= a.w[i];
    return acc == 0;
}
PA_DEV bool fq_eq(const Fq& a, const Fq& b) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) acc |= a.w[i] ^ b.w[i];
    return acc == 0;
}
PA_DEV bool fq_is_one(const Fq& a) {
    Fq o;
    fq_one(o);
    return fq_eq(a, o);
}

// Conditional subtract of q: r = (t >= q) ? t - q : t, for t < 2q.
PA_DEV void fq_reduce_once(Fq& r, const uint32_t t[12]) {
    uint32_t d[12];
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        uint64_t s = (uint64_t)t[i] - q_word(i) - borrow;
        d[i] = (uint32_t)s;
        borrow = (s >> 32) & 1;
    }
    const bool keep = borrow != 0;  // t < q
#pragma unroll
    for (int i = 0; i < 12; i++) r.w[i] = keep ? t[i] : d[i];
}

// fq.rs:812-819 (add then reduce)
PA_DEV void fq_add(Fq& r, const Fq& a, const Fq& b) {
    uint32_t t[12];
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        uint64_t s = (uint64_t)a.w[i] + b.w[i] + c;
        t[i] = (uint32_t)s;
        c = s >> 32;
    }
    fq_reduce_once(r, t);
}
PA_DEV void fq_dbl(Fq& r, const Fq& a) { fq_add(r, a, a); }  // fq.rs:821-828

// fq.rs:830-838: a - b, adding q back on borrow
PA_DEV void fq_sub(Fq& r, const Fq& a, const Fq& b) {
    uint32_t t[12];
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        uint64_t s = (uint64_t)a.w[i] - b.w[i] - borrow;
        t[i] = (uint32_t)s;
        borrow = (s >> 32) & 1;
    }
    const uint32_t mask = borrow ? 0xffffffffu : 0u;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        uint64_t s = (uint64_t)t[i] + (q_word(i) & mask) + c;
        r.w[i] = (uint32_t)s;
        c = s >> 32;
    }
}

// fq.rs:840-847: q - a unless a == 0
PA_DEV void fq_neg(Fq& r, const Fq& a) {
    const uint32_t mask = fq_is_zero(a) ? 0u : 0xffffffffu;
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        uint64_t s = (uint64_t)(q_word(i) & mask) - a.w[i] - borrow;
        r.w[i] = (uint32_t)s;
        borrow = (s >> 32) & 1;
    }
}

// CIOS Montgomery multiply, 32-bit words: r = a*b*2^-384 mod q (canonical).
PA_DEV void fq_mul(Fq& r, const Fq& a, const Fq& b) {
    uint32_t t[13];
    // row 0
    {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 12; j++) {
            uint64_t p = (uint64_t)a.w[0] * b.w[j] + c;
            t[j] = (uint32_t)p;
            c = p >> 32;
        }
        t[12] = (uint32_t)c;
        const uint32_t m = t[0] * PA_INV32;
        uint64_t p = (uint64_t)m * q_word(0) + t[0];
        c = p >> 32;
#pragma unroll
        for (int j = 1; j < 12; j++) {
            p = (uint64_t)m * q_word(j) + t[j] + c;
            t[j - 1] = (uint32_t)p;
            c = p >> 32;
        }
        p = (uint64_t)t[12] + c;
        t[11] = (uint32_t)p;
        t[12] = (uint32_t)(p >> 32);
    }
#pragma unroll
    for (int i = 1; i < 12; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 12; j++) {
            uint64_t p = (uint64_t)a.w[i] * b.w[j] + t[j] + c;
            t[j] = (uint32_t)p;
            c = p >> 32;
        }
        uint64_t s = (uint64_t)t[12] + c;
        t[12] = (uint32_t)s;
        const uint32_t t13 = (uint32_t)(s >> 32);
        const uint32_t m = t[0] * PA_INV32;
        uint64_t p = (uint64_t)m * q_word(0) + t[0];
        c = p >> 32;
#pragma unroll
        for (int j = 1; j < 12; j++) {
            p = (uint64_t)m * q_word(j) + t[j] + c;
            t[j - 1] = (uint32_t)p;
            c = p >> 32;
        }
        p = (uint64_t)t[12] + c;
        t[11] = (uint32_t)p;
        t[12] = t13 + (uint32_t)(p >> 32);
    }
    fq_reduce_once(r, t);
}

PA_DEV void fq_sqr(Fq& r, const Fq& a) { fq_mul(r, a, a); }

// ---- HBM <-> registers: 6 x u64 LE per element (the reference's layout) ----
PA_DEV void fq_load(Fq& r, const uint64_t* p) {
    const uint4* v = reinterpret_cast<const uint4*>(p);
    uint4 x0 = v[0], x1 = v[1], x2 = v[2];
    r.w[0] = x0.x; r.w[1] = x0.y; r.w[2] = x0.z; r.w[3] = x0.w;
    r.w[4] = x1.x; r.w[5] = x1.y; r.w[6] = x1.z; r.w[7] = x1.w;
    r.w[8] = x2.x; r.w[9] = x2.y; r.w[10] = x2.z; r.w[11] = x2.w;
}
PA_DEV void fq_store(uint64_t* p, const Fq& a) {
    uint4* v = reinterpret_cast<uint4*>(p);
    v[0] = make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]);
    v[1] = make_uint4(a.w[4], a.w[5], a.w[6], a.w[7]);
    v[2] = make_uint4(a.w[8], a.w[9], a.w[10], a.w[11]);
}
// constant table entries are u64[6] too
PA_DEV void fq_from_u64(Fq& r, const uint64_t* p) {
#pragma unroll
    for (int i = 0; i < 6; i++) {
        r.w[2 * i] = (uint32_t)p[i];
        r.w[2 * i + 1] = (uint32_t)(p[i] >> 32);
    }
}

}  // namespace pa
