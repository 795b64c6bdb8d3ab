// Extension tower over the lazy base field F<U> (fl.h) for the pairing kernels.
//
//   Fq2  = Fq[u]/(u^2+1)        reference src/bls12_381/fq2.rs:39-160
//   Fq6  = Fq2[v]/(v^3-(u+1))   reference src/bls12_381/fq6.rs:30-302
//   Fq12 = Fq6[w]/(w^2-v)       reference src/bls12_381/fq12.rs:29-149
//
// Every routine computes the same field value as the reference routine it
// cites; the representation is lazy (bound U carried in the type), and each
// Fq coordinate is made canonical only when it leaves the kernel.
//
// Cost model (gfx950, one wave per SIMD): a product leaf costs ~196 mads per
// product term + ~280 instructions per reduction; an Fq2 product is two
// two-term leaves (schoolbook with lazy reduction: c0 = a0 b0 - a1 b1 and
// c1 = a0 b1 + a1 b0 each reduced once).  Fq6/Fq12 products use the
// reference's Karatsuba forms over those, with red() (one pass, ~100 VALU)
// bringing sums back to U = 1 where the next product needs it.
#pragma once
#include "fl.h"

namespace pa {

template <int U> struct F2 { F<U> c0, c1; };
template <int U> struct F6 { F2<U> c0, c1, c2; };
template <int U> struct F12 { F6<U> c0, c1; };

// ======================= Fq2 =======================
template <int U2, int U1>
PA_DEV F2<U2> relax(const F2<U1>& a) { return {relax<U2>(a.c0), relax<U2>(a.c1)}; }
template <int A, int B>
PA_DEV F2<A + B> add(const F2<A>& a, const F2<B>& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
template <int A>
PA_DEV F2<2 * A> dbl(const F2<A>& a) { return add(a, a); }
template <int A, int B>
PA_DEV F2<A + subcu(B)> sub(const F2<A>& a, const F2<B>& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
template <int B>
PA_DEV F2<subcu(B)> neg(const F2<B>& b) { return {neg(b.c0), neg(b.c1)}; }
template <int U>
PA_DEV F2<1> red(const F2<U>& a) { return {red(a.c0), red(a.c1)}; }
// conjugate: Fq2::frobenius_map for odd powers (fq2.rs:157-159, coeff = -1)
template <int U>
PA_DEV F2<cmax(U, subcu(U))> conj(const F2<U>& a) {
    return {relax<cmax(U, subcu(U))>(a.c0), relax<cmax(U, subcu(U))>(neg(a.c1))};
}
// xi * a, xi = u + 1 (fq2.rs:41-45): (a0 - a1, a0 + a1)
template <int U>
PA_DEV F2<U + subcu(U)> mul_xi(const F2<U>& a) {
    return {sub(a.c0, a.c1), relax<U + subcu(U)>(add(a.c0, a.c1))};
}

// Fq2::mul_assign (fq2.rs:123-136): the same value, schoolbook with one
// reduction per coordinate (two two-term leaves)
template <int A, int B>
PA_DEV F2<1> mul(const F2<A>& a, const F2<B>& b) {
    F2<1> r;
    if constexpr (subcu(A) * B <= A * subcu(B)) {
        r.c0 = sop(a.c0, b.c0, neg(a.c1), b.c1);
    } else {
        r.c0 = sop(a.c0, b.c0, a.c1, neg(b.c1));
    }
    r.c1 = sop(a.c0, b.c1, a.c1, b.c0);
    return r;
}
// Fq2::square (fq2.rs:87-101): (a0 + a1)(a0 - a1), 2 a0 a1
template <int A>
PA_DEV F2<1> sqr(const F2<A>& a) {
    F2<1> r;
    if constexpr (2 * A * (A + subcu(A)) <= 17) {
        r.c0 = mul(add(a.c0, a.c1), sub(a.c0, a.c1));
    } else {
        r.c0 = sop(a.c0, a.c0, neg(a.c1), a.c1);
    }
    r.c1 = mul(dbl(a.c0), a.c1);
    return r;
}
template <int A, int B>
PA_DEV F2<1> mul_by_fq(const F2<A>& a, const F<B>& b) { return {mul(a.c0, b), mul(a.c1, b)}; }

PA_DEV F2<1> f2_zero() { return {fl_zero(), fl_zero()}; }
PA_DEV F2<1> f2_one() { return {fl_one(), fl_zero()}; }
PA_DEV F2<1> f2_c(const uint32_t c[2][14]) { return {fl_c(c[0]), fl_c(c[1])}; }

// ======================= Fq6 =======================
template <int U2, int U1>
PA_DEV F6<U2> relax(const F6<U1>& a) { return {relax<U2>(a.c0), relax<U2>(a.c1), relax<U2>(a.c2)}; }
template <int A, int B, int C>
PA_DEV F6<cmax(A, cmax(B, C))> mk6(const F2<A>& c0, const F2<B>& c1, const F2<C>& c2) {
    constexpr int M = cmax(A, cmax(B, C));
    return {relax<M>(c0), relax<M>(c1), relax<M>(c2)};
}
template <int A, int B>
PA_DEV F6<A + B> add(const F6<A>& a, const F6<B>& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
template <int A, int B>
PA_DEV F6<A + subcu(B)> sub(const F6<A>& a, const F6<B>& b) {
    return {sub(a.c0, b.c0), sub(a.c1, b.c1), sub(a.c2, b.c2)};
}
template <int B>
PA_DEV F6<subcu(B)> neg(const F6<B>& b) { return {neg(b.c0), neg(b.c1), neg(b.c2)}; }
template <int U>
PA_DEV F6<1> red(const F6<U>& a) { return {red(a.c0), red(a.c1), red(a.c2)}; }
// v * a (fq6.rs:32-38): (xi a2, a0, a1)
template <int U>
PA_DEV F6<U + subcu(U)> mul_v(const F6<U>& a) { return mk6(mul_xi(a.c2), a.c0, a.c1); }

// operand of an Fq2 product inside Fq6 Karatsuba: keep bound <= 2
template <int U>
PA_DEV auto lim2(const F2<U>& a) {
    if constexpr (U <= 2) return a; else return red(a);
}

// Fq6::mul_assign, fq6.rs:199-248 (Karatsuba, 6 Fq2 products)
template <int A, int B>
PA_DEV F6<1> mul(const F6<A>& a, const F6<B>& b) {
    static_assert(A <= 2 && B <= 2, "reduce Fq6 operands first");
    const F2<1> v0 = mul(a.c0, b.c0);
    const F2<1> v1 = mul(a.c1, b.c1);
    const F2<1> v2 = mul(a.c2, b.c2);
    const F2<1> t0 = mul(lim2(add(a.c1, a.c2)), lim2(add(b.c1, b.c2)));
    const F2<1> t1 = mul(lim2(add(a.c0, a.c1)), lim2(add(b.c0, b.c1)));
    const F2<1> t2 = mul(lim2(add(a.c0, a.c2)), lim2(add(b.c0, b.c2)));
    F6<1> r;
    r.c0 = red(add(mul_xi(sub(t0, add(v1, v2))), v0));
    r.c1 = red(add(sub(t1, add(v0, v1)), mul_xi(v2)));
    r.c2 = red(add(sub(t2, add(v0, v2)), v1));
    return r;
}
// fq6.rs:40-66: a * (c1 v) = (xi a2 c1, a0 c1, a1 c1)
template <int A, int B>
PA_DEV F6<1> mul_by_1(const F6<A>& a, const F2<B>& c1) {
    const auto xc = mul_xi(c1);
    return {mul(a.c2, xc), mul(a.c0, c1), mul(a.c1, c1)};
}
// fq6.rs:68-109: a * (c0 + c1 v), Karatsuba (5 Fq2 products)
template <int A, int B, int C>
PA_DEV F6<1> mul_by_01(const F6<A>& a, const F2<B>& c0, const F2<C>& c1) {
    const F2<1> a_a = mul(a.c0, c0);
    const F2<1> b_b = mul(a.c1, c1);
    const F2<1> t1 = mul(c1, lim2(add(a.c1, a.c2)));
    const F2<1> t3 = mul(c0, lim2(add(a.c0, a.c2)));
    const F2<1> t2 = mul(lim2(add(c0, c1)), lim2(add(a.c0, a.c1)));
    F6<1> r;
    r.c0 = red(add(mul_xi(sub(t1, b_b)), a_a));
    r.c1 = red(sub(t2, add(a_a, b_b)));
    r.c2 = red(add(sub(t3, a_a), b_b));
    return r;
}
// Fq6::frobenius_map, fq6.rs:157-164
PA_DEV F6<1> frobenius(const F6<1>& a, int power) {
    const bool odd = power & 1;
    F2<1> c0 = a.c0, c1 = a.c1, c2 = a.c2;
    if (odd) {  // wave-uniform
        c0 = red(conj(c0));
        c1 = red(conj(c1));
        c2 = red(conj(c2));
    }
    return {c0, mul(c1, f2_c(FL_FROB_FQ6_C1[power % 6])), mul(c2, f2_c(FL_FROB_FQ6_C2[power % 6]))};
}

PA_DEV F6<1> f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
PA_DEV F6<1> f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }

// ======================= Fq12 =======================
template <int U>
PA_DEV F12<1> red(const F12<U>& a) { return {red(a.c0), red(a.c1)}; }
template <int U>
PA_DEV F12<cmax(U, subcu(U))> conj(const F12<U>& a) {  // fq12.rs:30-32
    return {relax<cmax(U, subcu(U))>(a.c0), relax<cmax(U, subcu(U))>(neg(a.c1))};
}
PA_DEV F12<1> f12_one() { return {f6_one(), f6_zero()}; }

// Fq12::mul_assign, fq12.rs:116-130 (3 Fq6 products)
PA_DEV F12<1> mul(const F12<1>& a, const F12<1>& b) {
    const F6<1> aa = mul(a.c0, b.c0);
    const F6<1> bb = mul(a.c1, b.c1);
    const F6<1> cross = mul(add(a.c0, a.c1), add(b.c0, b.c1));
    F12<1> r;
    r.c1 = red(sub(cross, add(aa, bb)));
    r.c0 = red(add(mul_v(bb), aa));
    return r;
}
// Fq12::square, fq12.rs:99-114 (2 Fq6 products)
PA_DEV F12<1> sqr(const F12<1>& a) {
    const F6<1> ab = mul(a.c0, a.c1);
    const F6<1> t = mul(red(add(mul_v(a.c1), a.c0)), add(a.c0, a.c1));
    F12<1> r;
    r.c0 = red(sub(t, add(ab, mul_v(ab))));
    r.c1 = red(add(ab, ab));
    return r;
}
// sparse product by (c0 + c1 v) + (c4 v) w, fq12.rs:34-48
template <int A, int B, int C>
PA_DEV F12<1> mul_by_014(const F12<1>& a, const F2<A>& c0, const F2<B>& c1, const F2<C>& c4) {
    const F6<1> aa = mul_by_01(a.c0, c0, c1);
    const F6<1> bb = mul_by_1(a.c1, c4);
    const F6<1> s = mul_by_01(red(add(a.c1, a.c0)), c0, lim2(add(c1, c4)));
    F12<1> r;
    r.c1 = red(sub(s, add(aa, bb)));
    r.c0 = red(add(mul_v(bb), aa));
    return r;
}
// Fq12::frobenius_map, fq12.rs:90-97
PA_DEV F12<1> frobenius(const F12<1>& a, int power) {
    const F6<1> c0 = frobenius(a.c0, power);
    const F6<1> c1 = frobenius(a.c1, power);
    const F2<1> k = f2_c(FL_FROB_FQ12_C1[power % 12]);
    return {c0, {mul(c1.c0, k), mul(c1.c1, k), mul(c1.c2, k)}};
}

// Granger-Scott squaring for elements of the cyclotomic subgroup (the
// value Fq12::square gives for them).  f = g0 + g1 w, g0 = (a0,a1,a2),
// g1 = (b0,b1,b2); (a0,b1), (b0,a2), (a1,b2) are Fq4 = Fq2[s]/(s^2 - xi).
PA_DEV void fq4_sqr(F2<1>& r0, F2<1>& r1, const F2<1>& a, const F2<1>& b) {
    // (a + b s)^2 = (a^2 + xi b^2) + ((a+b)^2 - a^2 - b^2) s
    const F2<1> t0 = sqr(a);
    const F2<1> t1 = sqr(b);
    const F2<1> t2 = sqr(add(a, b));
    r1 = red(sub(t2, add(t0, t1)));
    r0 = red(add(mul_xi(t1), t0));
}
PA_DEV F12<1> cyclotomic_sqr(const F12<1>& f) {
    F2<1> t0, t1, t2, t3, t4, t5;
    fq4_sqr(t0, t1, f.c0.c0, f.c1.c1);
    fq4_sqr(t2, t3, f.c1.c0, f.c0.c2);
    fq4_sqr(t4, t5, f.c0.c1, f.c1.c2);
    F12<1> r;
    // 3 t - 2 a  and  3 t + 2 b
    r.c0.c0 = red(add(dbl(sub(t0, f.c0.c0)), t0));
    r.c0.c1 = red(add(dbl(sub(t2, f.c0.c1)), t2));
    r.c0.c2 = red(add(dbl(sub(t4, f.c0.c2)), t4));
    const auto t5x = mul_xi(t5);
    r.c1.c0 = red(add(dbl(add(t5x, f.c1.c0)), t5x));
    r.c1.c1 = red(add(dbl(add(t1, f.c1.c1)), t1));
    r.c1.c2 = red(add(dbl(add(t3, f.c1.c2)), t3));
    return r;
}

// ======================= inversion =======================
// Fq inverse by Fermat (a^(q-2)): the inverse is unique, so the value equals
// the reference's binary extended Euclid (fq.rs:849-902).  ok = (a != 0).
PA_DEV F<1> fl_inv(const F<1>& a, bool& ok) {
    const uint64_t e[6] = {0xb9feffffffffaaa9ULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                           0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
    F<1> acc = a;  // bit 380 of q - 2 is its top set bit
#pragma unroll 1
    for (int bit = 379; bit >= 0; bit--) {
        acc = sqr(acc);
        if ((e[bit >> 6] >> (bit & 63)) & 1) acc = mul(acc, a);  // wave-uniform
    }
    ok = !fl_is_zero(a);
    return acc;
}
// fq2.rs:138-155
PA_DEV F2<1> inverse(const F2<1>& a, bool& ok) {
    const F<1> t = fl_inv(sop(a.c0, a.c0, a.c1, a.c1), ok);
    return {mul(a.c0, t), mul(neg(a.c1), t)};
}
// fq6.rs:250-301
PA_DEV F6<1> inverse(const F6<1>& a, bool& ok) {
    const F2<1> c0 = red(sub(sqr(a.c0), mul(mul_xi(a.c2), a.c1)));
    const F2<1> c1 = red(sub(red(mul_xi(sqr(a.c2))), mul(a.c0, a.c1)));
    const F2<1> c2 = red(sub(sqr(a.c1), mul(a.c0, a.c2)));
    const F2<1> s = red(add(mul_xi(add(mul(a.c2, c1), mul(a.c1, c2))), mul(a.c0, c0)));
    const F2<1> t = inverse(s, ok);
    return {mul(t, c0), mul(t, c1), mul(t, c2)};
}
// fq12.rs:132-148
PA_DEV F12<1> inverse(const F12<1>& a, bool& ok) {
    const F6<1> s = red(sub(mul(a.c0, a.c0), mul_v(mul(a.c1, a.c1))));
    const F6<1> t = inverse(s, ok);
    return {mul(a.c0, t), red(neg(mul(a.c1, t)))};
}

// ======================= HBM records =======================
PA_DEV F2<1> load2(const uint64_t* p) { return {fl_load(p), fl_load(p + 6)}; }
template <int U>
PA_DEV void store2(uint64_t* p, const F2<U>& a) { fl_store(p, a.c0); fl_store(p + 6, a.c1); }
PA_DEV F12<1> load12(const uint64_t* p) {
    F12<1> r;
    r.c0 = {load2(p), load2(p + 12), load2(p + 24)};
    r.c1 = {load2(p + 36), load2(p + 48), load2(p + 60)};
    return r;
}
PA_DEV void store12(uint64_t* p, const F12<1>& a) {
    store2(p, a.c0.c0); store2(p + 12, a.c0.c1); store2(p + 24, a.c0.c2);
    store2(p + 36, a.c1.c0); store2(p + 48, a.c1.c1); store2(p + 60, a.c1.c2);
}

}  // namespace pa
