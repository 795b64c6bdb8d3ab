// Device-side extension tower Fq2 / Fq6 / Fq12 of BLS12-381 (gfx950).
//
//   Fq2  = Fq[u]/(u^2+1)        reference src/bls12_381/fq2.rs:39-160
//   Fq6  = Fq2[v]/(v^3-(u+1))   reference src/bls12_381/fq6.rs:30-302
//   Fq12 = Fq6[w]/(w^2-v)       reference src/bls12_381/fq12.rs:29-149
//
// Every tower value is canonical (each Fq coordinate < q), so results are
// bit-identical to the reference whatever multiplication schedule is used
// here; the schedules below are the reference's Karatsuba / CH-SQR2 forms.
//
// Inlining policy: Fq ops are always inlined; Fq2 mul/square are the unit of
// out-of-line code (each ~3 Montgomery multiplies), Fq6/Fq12 routines call
// them.  That keeps the code footprint of the pairing kernels inside the
// instruction cache while each call still does ~2k VALU instructions.
#pragma once
#include "fq_mul_gen.h"
#include "bls_consts.h"
#include "bgcd.h"

#define PA_NOINLINE __device__ __noinline__

namespace pa {

struct Fq2 { Fq c0, c1; };
struct Fq6 { Fq2 c0, c1, c2; };
struct Fq12 { Fq6 c0, c1; };

// ---------------- Fq2 ----------------
PA_DEV void zero(Fq2& r) { fq_zero(r.c0); fq_zero(r.c1); }
PA_DEV void one(Fq2& r) { fq_one(r.c0); fq_zero(r.c1); }
PA_DEV bool is_zero(const Fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
PA_DEV bool eq(const Fq2& a, const Fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }
PA_DEV bool is_one(const Fq2& a) { return fq_is_one(a.c0) && fq_is_zero(a.c1); }
PA_DEV void add(Fq2& r, const Fq2& a, const Fq2& b) { fq_add(r.c0, a.c0, b.c0); fq_add(r.c1, a.c1, b.c1); }
PA_DEV void sub(Fq2& r, const Fq2& a, const Fq2& b) { fq_sub(r.c0, a.c0, b.c0); fq_sub(r.c1, a.c1, b.c1); }
PA_DEV void dbl(Fq2& r, const Fq2& a) { fq_dbl(r.c0, a.c0); fq_dbl(r.c1, a.c1); }
PA_DEV void neg(Fq2& r, const Fq2& a) { fq_neg(r.c0, a.c0); fq_neg(r.c1, a.c1); }
// multiply by xi = u + 1, fq2.rs:41-45
PA_DEV void mul_by_nonresidue(Fq2& r, const Fq2& a) {
    Fq t0, t1;
    fq_sub(t0, a.c0, a.c1);
    fq_add(t1, a.c1, a.c0);
    r.c0 = t0;
    r.c1 = t1;
}
// Karatsuba, fq2.rs:123-136 (3 Fq multiplies)
PA_NOINLINE void mul(Fq2& r, const Fq2& a, const Fq2& b) {
    Fq aa, bb, o, s, x;
    fq_add(o, b.c0, b.c1);
    fq_add(s, a.c1, a.c0);
    fq_mul_x3(aa, a.c0, b.c0, bb, a.c1, b.c1, x, s, o);
    fq_sub(s, x, aa);
    fq_sub(r.c1, s, bb);
    fq_sub(r.c0, aa, bb);
}
// complex squaring, fq2.rs:87-101 (2 Fq multiplies)
PA_NOINLINE void sqr(Fq2& r, const Fq2& a) {
    Fq ab, c0c1, c0m, c0;
    fq_add(c0c1, a.c0, a.c1);
    fq_sub(c0m, a.c0, a.c1);
    fq_mul_x2(ab, a.c0, a.c1, c0, c0m, c0c1);
    fq_dbl(r.c1, ab);
    r.c0 = c0;
}
// Fq2 x Fq (used by ell, mod.rs:61-65)
PA_DEV void mul_by_fq(Fq2& r, const Fq2& a, const Fq& b) {
    fq_mul_x2(r.c0, a.c0, b, r.c1, a.c1, b);
}
PA_DEV void frobenius_map(Fq2& r, const Fq2& a, int power) {  // fq2.rs:157-159
    Fq c;
    fq_from_u64(c, FROB_FQ2_C1[power & 1]);
    r.c0 = a.c0;
    fq_mul(r.c1, a.c1, c);
}
PA_DEV void load_fq2_const(Fq2& r, const uint64_t p[2][6]) {
    fq_from_u64(r.c0, p[0]);
    fq_from_u64(r.c1, p[1]);
}

// ---------------- Fq6 ----------------
PA_DEV void zero(Fq6& r) { zero(r.c0); zero(r.c1); zero(r.c2); }
PA_DEV void one(Fq6& r) { one(r.c0); zero(r.c1); zero(r.c2); }
PA_DEV bool is_zero(const Fq6& a) { return is_zero(a.c0) && is_zero(a.c1) && is_zero(a.c2); }
PA_DEV void add(Fq6& r, const Fq6& a, const Fq6& b) { add(r.c0, a.c0, b.c0); add(r.c1, a.c1, b.c1); add(r.c2, a.c2, b.c2); }
PA_DEV void sub(Fq6& r, const Fq6& a, const Fq6& b) { sub(r.c0, a.c0, b.c0); sub(r.c1, a.c1, b.c1); sub(r.c2, a.c2, b.c2); }
PA_DEV void dbl(Fq6& r, const Fq6& a) { dbl(r.c0, a.c0); dbl(r.c1, a.c1); dbl(r.c2, a.c2); }
PA_DEV void neg(Fq6& r, const Fq6& a) { neg(r.c0, a.c0); neg(r.c1, a.c1); neg(r.c2, a.c2); }
// multiply by v, fq6.rs:32-38
PA_DEV void mul_by_nonresidue(Fq6& r, const Fq6& a) {
    Fq2 t;
    mul_by_nonresidue(t, a.c2);
    r.c2 = a.c1;
    r.c1 = a.c0;
    r.c0 = t;
}
// fq6.rs:199-248 (6 Fq2 multiplies)
PA_NOINLINE void mul(Fq6& r, const Fq6& a, const Fq6& b) {
    Fq2 a_a, b_b, c_c, t1, t2, t3, tmp;
    mul(a_a, a.c0, b.c0);
    mul(b_b, a.c1, b.c1);
    mul(c_c, a.c2, b.c2);

    add(t1, b.c1, b.c2);
    add(tmp, a.c1, a.c2);
    mul(t1, t1, tmp);
    sub(t1, t1, b_b);
    sub(t1, t1, c_c);
    mul_by_nonresidue(t1, t1);
    add(t1, t1, a_a);

    add(t3, b.c0, b.c2);
    add(tmp, a.c0, a.c2);
    mul(t3, t3, tmp);
    sub(t3, t3, a_a);
    add(t3, t3, b_b);
    sub(t3, t3, c_c);

    add(t2, b.c0, b.c1);
    add(tmp, a.c0, a.c1);
    mul(t2, t2, tmp);
    sub(t2, t2, a_a);
    sub(t2, t2, b_b);
    mul_by_nonresidue(c_c, c_c);
    add(t2, t2, c_c);

    r.c0 = t1;
    r.c1 = t2;
    r.c2 = t3;
}
// CH-SQR2, fq6.rs:166-197
PA_NOINLINE void sqr(Fq6& r, const Fq6& a) {
    Fq2 s0, s1, s2, s3, s4, ab, bc;
    sqr(s0, a.c0);
    mul(ab, a.c0, a.c1);
    dbl(s1, ab);
    sub(s2, a.c0, a.c1);
    add(s2, s2, a.c2);
    sqr(s2, s2);
    mul(bc, a.c1, a.c2);
    dbl(s3, bc);
    sqr(s4, a.c2);

    Fq6 o;
    mul_by_nonresidue(o.c0, s3);
    add(o.c0, o.c0, s0);
    mul_by_nonresidue(o.c1, s4);
    add(o.c1, o.c1, s1);
    add(o.c2, s1, s2);
    add(o.c2, o.c2, s3);
    sub(o.c2, o.c2, s0);
    sub(o.c2, o.c2, s4);
    r = o;
}
// fq6.rs:40-66
PA_NOINLINE void mul_by_1(Fq6& r, const Fq6& a, const Fq2& c1) {
    Fq2 b_b, t1, t2, tmp;
    mul(b_b, a.c1, c1);
    add(tmp, a.c1, a.c2);
    mul(t1, c1, tmp);
    sub(t1, t1, b_b);
    mul_by_nonresidue(t1, t1);
    add(tmp, a.c0, a.c1);
    mul(t2, c1, tmp);
    sub(t2, t2, b_b);
    r.c0 = t1;
    r.c1 = t2;
    r.c2 = b_b;
}
// fq6.rs:68-109
PA_NOINLINE void mul_by_01(Fq6& r, const Fq6& a, const Fq2& c0, const Fq2& c1) {
    Fq2 a_a, b_b, t1, t2, t3, tmp;
    mul(a_a, a.c0, c0);
    mul(b_b, a.c1, c1);

    add(tmp, a.c1, a.c2);
    mul(t1, c1, tmp);
    sub(t1, t1, b_b);
    mul_by_nonresidue(t1, t1);
    add(t1, t1, a_a);

    add(tmp, a.c0, a.c2);
    mul(t3, c0, tmp);
    sub(t3, t3, a_a);
    add(t3, t3, b_b);

    add(t2, c0, c1);
    add(tmp, a.c0, a.c1);
    mul(t2, t2, tmp);
    sub(t2, t2, a_a);
    sub(t2, t2, b_b);

    r.c0 = t1;
    r.c1 = t2;
    r.c2 = t3;
}
// fq6.rs:157-164
PA_NOINLINE void frobenius_map(Fq6& r, const Fq6& a, int power) {
    Fq2 k;
    frobenius_map(r.c0, a.c0, power);
    frobenius_map(r.c1, a.c1, power);
    frobenius_map(r.c2, a.c2, power);
    load_fq2_const(k, FROB_FQ6_C1[power % 6]);
    mul(r.c1, r.c1, k);
    load_fq2_const(k, FROB_FQ6_C2[power % 6]);
    mul(r.c2, r.c2, k);
}

// ---------------- Fq12 ----------------
PA_DEV void one(Fq12& r) { one(r.c0); zero(r.c1); }
PA_DEV bool is_zero(const Fq12& a) { return is_zero(a.c0) && is_zero(a.c1); }
PA_DEV void conjugate(Fq12& r, const Fq12& a) { r.c0 = a.c0; neg(r.c1, a.c1); }  // fq12.rs:30-32

// fq12.rs:116-130 (3 Fq6 multiplies)
PA_NOINLINE void mul(Fq12& r, const Fq12& a, const Fq12& b) {
    Fq6 aa, bb, o, s;
    mul(aa, a.c0, b.c0);
    mul(bb, a.c1, b.c1);
    add(o, b.c0, b.c1);
    add(s, a.c1, a.c0);
    mul(s, s, o);
    sub(s, s, aa);
    sub(r.c1, s, bb);
    mul_by_nonresidue(bb, bb);
    add(r.c0, bb, aa);
}
// complex squaring, fq12.rs:99-114 (2 Fq6 multiplies)
PA_NOINLINE void sqr(Fq12& r, const Fq12& a) {
    Fq6 ab, c0c1, c0;
    mul(ab, a.c0, a.c1);
    add(c0c1, a.c0, a.c1);
    mul_by_nonresidue(c0, a.c1);
    add(c0, c0, a.c0);
    mul(c0, c0, c0c1);
    sub(c0, c0, ab);
    dbl(r.c1, ab);
    mul_by_nonresidue(ab, ab);
    sub(r.c0, c0, ab);
}
// sparse multiply by (c0 + c1 v) + (c4 v) w, fq12.rs:34-48
PA_NOINLINE void mul_by_014(Fq12& r, const Fq12& a, const Fq2& c0, const Fq2& c1, const Fq2& c4) {
    Fq6 aa, bb, s;
    Fq2 o;
    mul_by_01(aa, a.c0, c0, c1);
    mul_by_1(bb, a.c1, c4);
    add(o, c1, c4);
    add(s, a.c1, a.c0);
    mul_by_01(s, s, c0, o);
    sub(s, s, aa);
    sub(r.c1, s, bb);
    mul_by_nonresidue(bb, bb);
    add(r.c0, bb, aa);
}
// fq12.rs:90-97
PA_NOINLINE void frobenius_map(Fq12& r, const Fq12& a, int power) {
    Fq2 k;
    frobenius_map(r.c0, a.c0, power);
    frobenius_map(r.c1, a.c1, power);
    load_fq2_const(k, FROB_FQ12_C1[power % 12]);
    mul(r.c1.c0, r.c1.c0, k);
    mul(r.c1.c1, r.c1.c1, k);
    mul(r.c1.c2, r.c1.c2, k);
}

// ---------------- inversion ----------------
// Fq inverse.  The reference uses a variable-time binary extended Euclid
// (fq.rs:849-902); the inverse is unique, so any correct algorithm gives the
// same bits.  bgcd.h's optimized binary GCD (26 x 30 approximate steps) on the
// Montgomery word x = X R gives x^-1; one product by R^3 turns it into the
// Montgomery form R^2 / x = X^-1 R.  ~13x fewer instructions than Fermat
// (a^(q-2), ~570 sequential products), which bounds the latency of every
// normalize / into_affine lane.  Returns false (reference: None) iff a == 0.
PA_NOINLINE bool fq_inv(Fq& r, const Fq& a) {
    constexpr uint32_t kR3[12] = {0xd94ca1e0u, 0xed48ac6bu, 0x03a7adf8u, 0x315f831eu, 0x615e29ddu, 0x9a53352au,
                                  0x921e1761u, 0x34c04e5eu, 0x65724728u, 0x2512d435u, 0x91755d4du, 0x0aa63460u};
    Fq y, r3;
    const bool ok = bgcd::inverse(y.w, a.w);
#pragma unroll
    for (int i = 0; i < 12; i++) r3.w[i] = kR3[i];
    fq_mul(r, y, r3);
    return ok;
}
// Fermat a^(q-2), kept for A/B measurements (same result as fq_inv)
PA_NOINLINE bool fq_inv_fermat(Fq& r, const Fq& a) {
    // exponent q - 2, scanned MSB first; the branch is wave-uniform
    const uint64_t e[6] = {0xb9feffffffffaaa9ULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                           0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
    Fq acc = a;  // bit 380 (the top bit of q - 2) is set
#pragma unroll 1
    for (int bit = 379; bit >= 0; bit--) {
        fq_sqr(acc, acc);
        if ((e[bit >> 6] >> (bit & 63)) & 1) fq_mul(acc, acc, a);
    }
    r = acc;
    return !fq_is_zero(a);
}
// fq2.rs:138-155
PA_NOINLINE bool inverse(Fq2& r, const Fq2& a) {
    Fq t0, t1, t;
    fq_sqr(t1, a.c1);
    fq_sqr(t0, a.c0);
    fq_add(t0, t0, t1);
    bool ok = fq_inv(t, t0);
    fq_mul(r.c0, a.c0, t);
    fq_mul(r.c1, a.c1, t);
    fq_neg(r.c1, r.c1);
    return ok;
}
// fq6.rs:250-301
PA_NOINLINE bool inverse(Fq6& r, const Fq6& a) {
    Fq2 c0, c1, c2, tmp1, tmp2, t;
    mul_by_nonresidue(c0, a.c2);
    mul(c0, c0, a.c1);
    neg(c0, c0);
    sqr(tmp1, a.c0);
    add(c0, c0, tmp1);

    sqr(c1, a.c2);
    mul_by_nonresidue(c1, c1);
    mul(tmp1, a.c0, a.c1);
    sub(c1, c1, tmp1);

    sqr(c2, a.c1);
    mul(tmp1, a.c0, a.c2);
    sub(c2, c2, tmp1);

    mul(tmp1, a.c2, c1);
    mul(tmp2, a.c1, c2);
    add(tmp1, tmp1, tmp2);
    mul_by_nonresidue(tmp1, tmp1);
    mul(tmp2, a.c0, c0);
    add(tmp1, tmp1, tmp2);

    bool ok = inverse(t, tmp1);
    mul(r.c0, t, c0);
    mul(r.c1, t, c1);
    mul(r.c2, t, c2);
    return ok;
}
// fq12.rs:132-148
PA_NOINLINE bool inverse(Fq12& r, const Fq12& a) {
    Fq6 c0s, c1s, t;
    sqr(c0s, a.c0);
    sqr(c1s, a.c1);
    mul_by_nonresidue(c1s, c1s);
    sub(c0s, c0s, c1s);
    bool ok = inverse(t, c0s);
    mul(r.c0, t, a.c0);
    mul(r.c1, t, a.c1);
    neg(r.c1, r.c1);
    return ok;
}

// ---------------- HBM I/O (reference in-memory order) ----------------
PA_DEV void load(Fq2& r, const uint64_t* p) { fq_load(r.c0, p); fq_load(r.c1, p + 6); }
PA_DEV void store(uint64_t* p, const Fq2& a) { fq_store(p, a.c0); fq_store(p + 6, a.c1); }
PA_DEV void load(Fq6& r, const uint64_t* p) { load(r.c0, p); load(r.c1, p + 12); load(r.c2, p + 24); }
PA_DEV void store(uint64_t* p, const Fq6& a) { store(p, a.c0); store(p + 12, a.c1); store(p + 24, a.c2); }
PA_DEV void load(Fq12& r, const uint64_t* p) { load(r.c0, p); load(r.c1, p + 36); }
PA_DEV void store(uint64_t* p, const Fq12& a) { store(p, a.c0); store(p + 36, a.c1); }

}  // namespace pa
