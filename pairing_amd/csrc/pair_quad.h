// Pairings on lane groups (round 6): one pairing per GROUP of 8 lane quads
// (32 lanes, two pairings per wave) -- the latency form between the
// cooperative VM (a four-wave workgroup per pairing, ~1.6 ms, ~270 k
// pairings/s) and the generated lane-pair kernels (32 pairings per wave,
// ~9 ms whatever the batch up to 32768).
//
// The tower and the line functions are tower_fl.h / pairing_fl.h -- the
// same field values as the reference routines they cite -- on values SPREAD
// over a quad (dec_quad.h: lane r of a quad holds limbs 4r..4r+3 of the lazy
// 14 x 28-bit representation; every quad of the group holds every value).
// What changes is the schedule: the products of a step are batched into
// LEVELS of up to four independent Fq2 products, two quads each
// (dq::level2), instead of one after another -- an Fq6 product is two levels,
// an Fq12 product five, a cyclotomic squaring three, a Miller-loop doubling
// with its line three.  The linear combinations run on every quad (each lane
// holds a quarter of a value).  The base-field inversion of the final
// exponentiation is the binary GCD (bgcd.h) on the gathered value, run by
// every lane of the group at once.
//
//   miller_loop     mod.rs:40-102 (reference-form G2 steps: the Miller
//                   values are the reference's, bit for bit once canonical)
//   final_exp       mod.rs:104-160 (cyclotomic squarings inside exp_by_x:
//                   the result is the reference's, the exponent is unique)
#pragma once
#include "bgcd.h"
#include "dec_quad.h"

namespace pa {
namespace pq {
using namespace dq;
constexpr int NQ = 8;   // quads per pairing

template <int U>
struct Q6 {
    Q2<U> c0, c1, c2;
};
template <int U>
struct Q12 {
    Q6<U> c0, c1;
};
using E2 = Q2<1>;
using E6 = Q6<1>;
using E12 = Q12<1>;

// R'^3 mod q (R' = 2^392) in the lazy form: the binary GCD's plain inverse of
// the canonical integer x R' times this constant in one product is x^-1 R'
// (tools: pow(2^392, 3, q), 28-bit limbs)
__constant__ const uint32_t kPqInvFix[14] = {0x1f7b890u, 0x294cc4du, 0x9f3af22u, 0xb5ba56cu, 0xcb5c0ccu,
                                             0xc0d975cu, 0xc89a8c5u, 0x6c968b4u, 0x22672eau, 0x91de8c9u,
                                             0x35652a6u, 0x84977c8u, 0x424bbb9u, 0x00141abu};

// ---------------- Fq2 ----------------
template <int U>
PA_DEV Q2<cmax(U + subcu(U), 2 * U)> xi(const Q2<U>& a, const Lc& l) {   // fq2.rs:41-45
    constexpr int V = cmax(U + subcu(U), 2 * U);
    return {relax<V>(sub(a.c0, a.c1, l)), relax<V>(add(a.c0, a.c1))};
}
template <int U>
PA_DEV Q2<cmax(U, subcu(U))> conj(const Q2<U>& a, const Lc& l) {
    constexpr int V = cmax(U, subcu(U));
    return {relax<V>(a.c0), relax<V>(neg(a.c1, l))};
}
// a product operand: bound <= 2
template <int U>
PA_DEV Q2<2> w2(const Q2<U>& a, const Lc& l) {
    if constexpr (U <= 2) return relax<2>(a);
    else return relax<2>(red(a, l));
}
PA_DEV E2 e2c(const uint32_t (&c)[2][14], const Lc& l) { return {qconst(c[0], l), qconst(c[1], l)}; }
PA_DEV E2 e2_zero() { return {zero_e<Q>(), zero_e<Q>()}; }

// o[k] = x[k] y[k], k < N, in levels of up to four Fq2 products
template <int N, int K = 0>
PA_DEV void prods(E2 (&o)[N], const Q2<2> (&x)[N], const Q2<2> (&y)[N], const Lc& l) {
    if constexpr (K < N) {
        constexpr int M = N - K < NQ / 2 ? N - K : NQ / 2;
        Q2<2> xs[M], ys[M];
        E2 os[M];
#pragma unroll
        for (int m = 0; m < M; m++) {
            xs[m] = x[K + m];
            ys[m] = y[K + m];
        }
        level2<NQ>(os, xs, ys, l);
#pragma unroll
        for (int m = 0; m < M; m++) o[K + m] = os[m];
        prods<N, K + M>(o, x, y, l);
    }
}
// the same with operand k formed by gen(k, x, y) just before its level (k is
// a constant once the level loop unrolls): the operands of one level are live
// at a time, not all N
template <int N, int K = 0, class G>
PA_DEV void prods_g(E2 (&o)[N], const G& gen, const Lc& l) {
    if constexpr (K < N) {
        constexpr int M = N - K < NQ / 2 ? N - K : NQ / 2;
        Q2<2> xs[M], ys[M];
        E2 os[M];
#pragma unroll
        for (int m = 0; m < M; m++) gen(K + m, xs[m], ys[m]);
        level2<NQ>(os, xs, ys, l);
#pragma unroll
        for (int m = 0; m < M; m++) o[K + m] = os[m];
        prods_g<N, K + M>(o, gen, l);
    }
}
template <int UX, int UY>
PA_DEV E2 mul2(const Q2<UX>& x, const Q2<UY>& y, const Lc& l) {
    E2 o[1];
    const Q2<2> xs[1] = {w2(x, l)}, ys[1] = {w2(y, l)};
    prods<1>(o, xs, ys, l);
    return o[0];
}

// ---------------- Fq6 ----------------
template <int U>
PA_DEV Q6<2> w6(const Q6<U>& a, const Lc& l) { return {w2(a.c0, l), w2(a.c1, l), w2(a.c2, l)}; }
template <int U>
PA_DEV E6 red6(const Q6<U>& a, const Lc& l) { return {red(a.c0, l), red(a.c1, l), red(a.c2, l)}; }
template <int A, int B>
PA_DEV Q6<A + B> add6(const Q6<A>& a, const Q6<B>& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
template <int A, int B>
PA_DEV Q6<A + subcu(B)> sub6(const Q6<A>& a, const Q6<B>& b, const Lc& l) {
    return {sub(a.c0, b.c0, l), sub(a.c1, b.c1, l), sub(a.c2, b.c2, l)};
}
// v a = (xi a2, a0, a1), fq6.rs:32-38
template <int U>
PA_DEV Q6<cmax(U + subcu(U), 2 * U)> mul_v(const Q6<U>& a, const Lc& l) {
    constexpr int V = cmax(U + subcu(U), 2 * U);
    return {xi(a.c2, l), relax<V>(a.c0), relax<V>(a.c1)};
}
PA_DEV E6 e6_zero() { return {e2_zero(), e2_zero(), e2_zero()}; }

template <int K>
PA_DEV void mul6s_raw(Q6<10> (&o)[K], const Q6<2> (&a)[K], const Q6<2> (&b)[K], const Lc& l);
// K Fq6 products a[k] b[k] (fq6.rs:199-248, Karatsuba: 6 Fq2 products each),
// all 6 K Fq2 products in one batch
template <int K>
PA_DEV void mul6s(E6 (&o)[K], const Q6<2> (&a)[K], const Q6<2> (&b)[K], const Lc& l) {
    Q6<10> u[K];
    mul6s_raw<K>(u, a, b, l);
#pragma unroll
    for (int k = 0; k < K; k++) o[k] = red6(u[k], l);
}
// the same, the Karatsuba combinations left unreduced (bound 10), for
// callers whose next sums stay within the reduction's bound
template <int K>
PA_DEV void mul6s_raw(Q6<10> (&o)[K], const Q6<2> (&a)[K], const Q6<2> (&b)[K], const Lc& l) {
    E2 p[6 * K];
    prods_g<6 * K>(p, [&](int k, Q2<2>& x, Q2<2>& y) {
        const Q6<2>& u = a[k / 6];
        const Q6<2>& v = b[k / 6];
        switch (k % 6) {
            case 0: x = u.c0; y = v.c0; break;
            case 1: x = u.c1; y = v.c1; break;
            case 2: x = u.c2; y = v.c2; break;
            case 3: x = w2(add(u.c1, u.c2), l); y = w2(add(v.c1, v.c2), l); break;
            case 4: x = w2(add(u.c0, u.c1), l); y = w2(add(v.c0, v.c1), l); break;
            default: x = w2(add(u.c0, u.c2), l); y = w2(add(v.c0, v.c2), l); break;
        }
    }, l);
#pragma unroll
    for (int k = 0; k < K; k++) {
        const E2 v0 = p[6 * k], v1 = p[6 * k + 1], v2 = p[6 * k + 2];
        const E2 t0 = p[6 * k + 3], t1 = p[6 * k + 4], t2 = p[6 * k + 5];
        o[k].c0 = relax<10>(add(xi(sub(t0, add(v1, v2), l), l), v0));
        o[k].c1 = relax<10>(add(sub(t1, add(v0, v1), l), xi(v2, l)));
        o[k].c2 = relax<10>(add(sub(t2, add(v0, v2), l), v1));
    }
}

// the 5 Fq2 products of mul_by_01 (fq6.rs:68-109) into x, y at offset k, and its combination
template <int N, int UA, int UB, int UC>
PA_DEV void by01_ops(Q2<2> (&x)[N], Q2<2> (&y)[N], int k, const Q6<UA>& a, const Q2<UB>& c0, const Q2<UC>& c1,
                     const Lc& l) {
    x[k] = w2(a.c0, l);
    y[k] = w2(c0, l);                                        // a_a
    x[k + 1] = w2(a.c1, l);
    y[k + 1] = w2(c1, l);                                    // b_b
    x[k + 2] = w2(c1, l);
    y[k + 2] = w2(add(a.c1, a.c2), l);                       // t1
    x[k + 3] = w2(c0, l);
    y[k + 3] = w2(add(a.c0, a.c2), l);                       // t3
    x[k + 4] = w2(add(c0, c1), l);
    y[k + 4] = w2(add(a.c0, a.c1), l);                       // t2
}
template <int N>
PA_DEV E6 by01_fin(const E2 (&p)[N], int k, const Lc& l) {
    const E2 a_a = p[k], b_b = p[k + 1], t1 = p[k + 2], t3 = p[k + 3], t2 = p[k + 4];
    E6 r;
    r.c0 = red(add(xi(sub(t1, b_b, l), l), a_a), l);
    r.c1 = red(sub(t2, add(a_a, b_b), l), l);
    r.c2 = red(add(sub(t3, a_a, l), b_b), l);
    return r;
}

// ---------------- Fq12 ----------------
template <int U>
PA_DEV E12 red12(const Q12<U>& a, const Lc& l) { return {red6(a.c0, l), red6(a.c1, l)}; }
PA_DEV E12 conj12(const E12& a, const Lc& l) {   // fq12.rs:30-32
    return {a.c0, {red(neg(a.c1.c0, l), l), red(neg(a.c1.c1, l), l), red(neg(a.c1.c2, l), l)}};
}
PA_DEV E12 e12_one(const Lc& l) { return {{one_e<Q2>(l), e2_zero(), e2_zero()}, e6_zero()}; }

// Fq12::mul_assign, fq12.rs:116-130: 3 Fq6 products = 18 Fq2 products, 5 levels
PA_DEV E12 mul12(const E12& a, const E12& b, const Lc& l) {
    const Q6<2> as[3] = {w6(a.c0, l), w6(a.c1, l), w6(add6(a.c0, a.c1), l)};
    const Q6<2> bs[3] = {w6(b.c0, l), w6(b.c1, l), w6(add6(b.c0, b.c1), l)};
    Q6<10> p[3];
    mul6s_raw<3>(p, as, bs, l);
    const E6 aa = red6(p[0], l), bb = red6(p[1], l);
    E12 r;
    r.c1 = red6(sub6(p[2], add6(aa, bb), l), l);   // cross unreduced: 10 + subcu(2) <= 16
    r.c0 = red6(add6(mul_v(bb, l), aa), l);
    return r;
}
// Fq12::square, fq12.rs:99-114: 2 Fq6 products, 3 levels
PA_DEV E12 sqr12(const E12& a, const Lc& l) {
    const Q6<2> as[2] = {w6(a.c0, l), w6(red6(add6(mul_v(a.c1, l), a.c0), l), l)};
    const Q6<2> bs[2] = {w6(a.c1, l), w6(add6(a.c0, a.c1), l)};
    Q6<10> p[2];
    mul6s_raw<2>(p, as, bs, l);
    const E6 ab = red6(p[0], l);
    E12 r;
    r.c0 = red6(sub6(p[1], add6(ab, mul_v(ab, l)), l), l);   // t unreduced: 10 + subcu(4) <= 16
    r.c1 = red6(add6(ab, ab), l);
    return r;
}
// sparse product by (c0 + c1 v) + (c4 v) w, fq12.rs:34-48: 13 Fq2 products, 4 levels
PA_DEV E12 mul_by_014(const E12& a, const E2& c0, const E2& c1, const E2& c4, const Lc& l) {
    Q2<2> x[13], y[13];
    by01_ops(x, y, 0, a.c0, c0, c1, l);                                 // aa = mul_by_01(a0, c0, c1)
    by01_ops(x, y, 5, red6(add6(a.c1, a.c0), l), c0, w2(add(c1, c4), l), l);   // s
    const auto xc = xi(c4, l);                                         // bb = mul_by_1(a1, c4)
    x[10] = w2(a.c1.c2, l);
    y[10] = w2(xc, l);
    x[11] = w2(a.c1.c0, l);
    y[11] = w2(c4, l);
    x[12] = w2(a.c1.c1, l);
    y[12] = w2(c4, l);
    E2 p[13];
    prods<13>(p, x, y, l);
    // mul_by_01's combinations (by01_fin) left unreduced where the final sums'
    // bounds allow -- aa.c0 (bound 8) is the only one reduced
    auto fin = [&](int k, auto& c0, auto& c1, auto& c2) {
        const E2 a_a = p[k], b_b = p[k + 1], t1 = p[k + 2], t3 = p[k + 3], t2 = p[k + 4];
        c0 = add(xi(sub(t1, b_b, l), l), a_a);
        c1 = relax<4>(sub(t2, add(a_a, b_b), l));
        c2 = relax<4>(add(sub(t3, a_a, l), b_b));
    };
    Q2<8> a0, s0;
    Q2<4> a1, a2, s1, s2;
    fin(0, a0, a1, a2);
    fin(5, s0, s1, s2);
    const E2 aa0 = red(a0, l);
    const E6 bb = {p[10], p[11], p[12]};
    E12 r;
    r.c1 = {red(sub(s0, add(aa0, bb.c0), l), l), red(sub(s1, add(a1, bb.c1), l), l),
            red(sub(s2, add(a2, bb.c2), l), l)};
    r.c0 = {red(add(xi(bb.c2, l), aa0), l), red(add(bb.c0, a1), l), red(add(bb.c1, a2), l)};
    return r;
}
// Fq12::frobenius_map, fq12.rs:90-97 (fq6.rs:157-164 on both halves): 2 levels
PA_DEV E12 frob12(const E12& a, int power, const Lc& l) {
    const bool odd = power & 1;   // wave-uniform
    E6 h0 = a.c0, h1 = a.c1;
    if (odd) {
        h0 = {red(conj(h0.c0, l), l), red(conj(h0.c1, l), l), red(conj(h0.c2, l), l)};
        h1 = {red(conj(h1.c0, l), l), red(conj(h1.c1, l), l), red(conj(h1.c2, l), l)};
    }
    const E2 k1 = e2c(FL_FROB_FQ6_C1[power % 6], l), k2 = e2c(FL_FROB_FQ6_C2[power % 6], l);
    const E2 kw = e2c(FL_FROB_FQ12_C1[power % 12], l);
    const Q2<2> x1[4] = {relax<2>(h0.c1), relax<2>(h0.c2), relax<2>(h1.c1), relax<2>(h1.c2)};
    const Q2<2> y1[4] = {relax<2>(k1), relax<2>(k2), relax<2>(k1), relax<2>(k2)};
    E2 p[4];
    prods<4>(p, x1, y1, l);
    const Q2<2> x2[3] = {relax<2>(h1.c0), relax<2>(p[2]), relax<2>(p[3])};
    const Q2<2> y2[3] = {relax<2>(kw), relax<2>(kw), relax<2>(kw)};
    E2 q[3];
    prods<3>(q, x2, y2, l);
    return {{h0.c0, p[0], p[1]}, {q[0], q[1], q[2]}};
}
// Granger-Scott squaring in the cyclotomic subgroup (tower_fl.h
// cyclotomic_sqr: Fq12::square's value there): 9 Fq2 squares, 3 levels
PA_DEV E12 cyc_sqr(const E12& f, const Lc& l) {
    const E2 pa[3] = {f.c0.c0, f.c1.c0, f.c0.c1}, pb[3] = {f.c1.c1, f.c0.c2, f.c1.c2};
    Q2<2> x[9];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        x[3 * k] = relax<2>(pa[k]);
        x[3 * k + 1] = relax<2>(pb[k]);
        x[3 * k + 2] = w2(add(pa[k], pb[k]), l);
    }
    E2 s[9];
    prods<9>(s, x, x, l);
    // fq4_sqr: r0 = xi b^2 + a^2, r1 = (a + b)^2 - a^2 - b^2, left unreduced
    // (bound 4): 3 t -+ 2 a stays within the reduction's bound 16 (the Fq
    // reductions are half of a level's time, so 12 fewer per squaring count)
    Q2<4> t[6];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        t[2 * k] = add(xi(s[3 * k + 1], l), s[3 * k]);
        t[2 * k + 1] = relax<4>(sub(s[3 * k + 2], add(s[3 * k], s[3 * k + 1]), l));
    }
    E12 r;
    r.c0.c0 = red(add(dbl(sub(t[0], f.c0.c0, l)), t[0]), l);
    r.c0.c1 = red(add(dbl(sub(t[2], f.c0.c1, l)), t[2]), l);
    r.c0.c2 = red(add(dbl(sub(t[4], f.c0.c2, l)), t[4]), l);
    const E2 t5x = red(xi(t[5], l), l);
    r.c1.c0 = red(add(dbl(add(t5x, f.c1.c0)), t5x), l);
    r.c1.c1 = red(add(dbl(add(t[1], f.c1.c1)), t[1]), l);
    r.c1.c2 = red(add(dbl(add(t[3], f.c1.c2)), t[3]), l);
    return r;
}

// ---------------- inversion ----------------
// Fq: the binary GCD on the gathered canonical integer (every lane of the
// group runs it; the inverse is unique, fq.rs:849-902); ok = (a != 0)
PA_DEV Q<1> inv_fq(const Q<1>& a, bool& ok, const Lc& l) {
    const Fq c = fl_pack_canon(whole(a));
    Fq y;
    ok = bgcd::inverse(y.w, c.w);
    const F<1> t = fl_canon(mul(fl_split(y), fl_c(kPqInvFix)));
    return ok ? piece(t, l) : zero_e<Q>();
}
// fq12.rs:132-148 -> fq6.rs:250-301 -> fq2.rs:138-155
PA_DEV E12 inv12(const E12& a, bool& ok, const Lc& l) {
    E6 sq[2];
    {
        const Q6<2> xs[2] = {w6(a.c0, l), w6(a.c1, l)};
        mul6s<2>(sq, xs, xs, l);
    }
    const E6 s = red6(sub6(sq[0], red6(mul_v(sq[1], l), l), l), l);
    // Fq6 inverse of s: c0 = s0^2 - xi s2 s1, c1 = xi s2^2 - s0 s1, c2 = s1^2 - s0 s2
    E2 p[6];
    {
        const Q2<2> x[6] = {relax<2>(s.c0), w2(xi(s.c2, l), l), relax<2>(s.c2), relax<2>(s.c0), relax<2>(s.c1),
                            relax<2>(s.c0)};
        const Q2<2> y[6] = {relax<2>(s.c0), relax<2>(s.c1), relax<2>(s.c2), relax<2>(s.c1), relax<2>(s.c1),
                            relax<2>(s.c2)};
        prods<6>(p, x, y, l);
    }
    const E2 c0 = red(sub(p[0], p[1], l), l);
    const E2 c1 = red(sub(red(xi(p[2], l), l), p[3], l), l);
    const E2 c2 = red(sub(p[4], p[5], l), l);
    E2 u[3];
    {
        const Q2<2> x[3] = {relax<2>(s.c2), relax<2>(s.c1), relax<2>(s.c0)};
        const Q2<2> y[3] = {relax<2>(c1), relax<2>(c2), relax<2>(c0)};
        prods<3>(u, x, y, l);
    }
    const E2 d = red(add(xi(add(u[0], u[1]), l), u[2]), l);
    // Fq2 inverse of d: (d0 t, -d1 t), t = (d0^2 + d1^2)^-1
    const Q<1> nrm = sop(d.c0, d.c0, d.c1, d.c1, l);
    const Q<1> t = inv_fq(nrm, ok, l);
    Q<1> dt[2];
    {
        const Q<1> x[2] = {d.c0, red(neg(d.c1, l), l)}, y[2] = {t, t};
        level<NQ>(dt, x, y, l);
    }
    const E2 di = {dt[0], dt[1]};
    E2 v[3];
    {
        const Q2<2> x[3] = {relax<2>(di), relax<2>(di), relax<2>(di)};
        const Q2<2> y[3] = {relax<2>(c0), relax<2>(c1), relax<2>(c2)};
        prods<3>(v, x, y, l);
    }
    const E6 si = {v[0], v[1], v[2]};
    E6 o[2];
    {
        const Q6<2> x[2] = {w6(a.c0, l), w6(a.c1, l)}, y[2] = {w6(si, l), w6(si, l)};
        mul6s<2>(o, x, y, l);
    }
    return {o[0], {red(neg(o[1].c0, l), l), red(neg(o[1].c1, l), l), red(neg(o[1].c2, l), l)}};
}

// ---------------- final exponentiation, mod.rs:104-160 ----------------
// exp_by_x (mod.rs:116-121): f^|x| by square-and-multiply with cyclotomic
// squarings, then the conjugation (x < 0)
PA_DEV E12 exp_by_x(const E12& f, uint64_t x, const Lc& l) {
    E12 r = f;
    const int top = 63 - __builtin_clzll(x);
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; bit--) {
        r = cyc_sqr(r, l);
        if ((x >> bit) & 1) r = mul12(r, f, l);   // wave-uniform
    }
    return conj12(r, l);
}
PA_DEV E12 final_exp(const E12& f, bool& ok, const Lc& l) {
    constexpr uint64_t kX = 0xd201000000010000ull;
    const E12 f2 = inv12(f, ok, l);
    E12 r = mul12(conj12(f, l), f2, l);
    r = mul12(frob12(r, 2, l), r, l);
    const E12 y0 = cyc_sqr(r, l);
    E12 y1 = exp_by_x(y0, kX, l);
    E12 y2 = exp_by_x(y1, kX >> 1, l);
    y1 = mul12(conj12(mul12(y1, conj12(r, l), l), l), y2, l);
    y2 = exp_by_x(y1, kX, l);
    E12 y3 = exp_by_x(y2, kX, l);
    y1 = conj12(y1, l);
    y3 = mul12(y3, y1, l);
    y1 = mul12(frob12(conj12(y1, l), 3, l), frob12(y2, 2, l), l);
    y2 = mul12(mul12(exp_by_x(y3, kX, l), y0, l), r, l);
    y1 = mul12(y1, y2, l);
    return mul12(y1, frob12(y3, 1, l), l);
}

// ---------------- Miller loop, mod.rs:40-102 ----------------
struct G2J {
    E2 x, y, z;
};
struct Line {
    E2 c0, c1, c2;
};
// doubling_step, mod.rs:176-245 (pairing_fl.h dbl_step_fl): 3 levels
PA_DEV Line dbl_step(G2J& r, const Lc& l) {
    E2 a[4];
    {
        const Q2<2> x[4] = {relax<2>(r.x), relax<2>(r.y), relax<2>(r.z), w2(add(r.z, r.y), l)};
        prods<4>(a, x, x, l);
    }
    const E2 t0 = a[0], t1 = a[1], zz = a[2], zy2 = a[3];
    const E2 t4 = red(add(dbl(t0), t0), l);
    E2 b[4];
    {
        const Q2<2> x[4] = {relax<2>(t1), w2(add(t1, r.x), l), relax<2>(t4), w2(add(r.x, t4), l)};
        prods<4>(b, x, x, l);
    }
    const E2 t2 = b[0], t5 = b[2];
    const E2 t3 = red(dbl(sub(b[1], add(t0, t2), l)), l);
    Line c;
    c.c2 = red(sub(b[3], add(add(t0, t5), dbl(dbl(t1))), l), l);
    const E2 x = red(sub(t5, dbl(t3), l), l);
    const E2 z = red(sub(zy2, add(t1, zz), l), l);
    E2 d[3];
    {
        const Q2<2> xs[3] = {w2(sub(t3, x, l), l), w2(neg(dbl(t4), l), l), w2(dbl(z), l)};
        const Q2<2> ys[3] = {relax<2>(t4), relax<2>(zz), relax<2>(zz)};
        prods<3>(d, xs, ys, l);
    }
    r.y = red(sub(d[0], dbl(dbl(dbl(t2))), l), l);
    r.x = x;
    r.z = z;
    c.c1 = d[1];
    c.c0 = d[2];
    return c;
}
// addition_step (mixed), mod.rs:247-333 (pairing_fl.h add_step_fl): 5 levels
PA_DEV Line add_step(G2J& r, const E2& qx, const E2& qy, const Lc& l) {
    E2 a[3];
    {
        const Q2<2> x[3] = {relax<2>(r.z), relax<2>(qy), w2(add(qy, r.z), l)};
        prods<3>(a, x, x, l);
    }
    const E2 zz = a[0], yy = a[1];
    E2 b[2];
    {
        const Q2<2> x[2] = {relax<2>(zz), w2(sub(a[2], add(yy, zz), l), l)};
        const Q2<2> y[2] = {relax<2>(qx), relax<2>(zz)};
        prods<2>(b, x, y, l);
    }
    const E2 t0 = b[0], t1 = b[1];
    const E2 t2 = red(sub(t0, r.x, l), l);
    const E2 t6 = red(sub(t1, dbl(r.y), l), l);
    E2 c[4];
    {
        const Q2<2> x[4] = {relax<2>(t2), w2(add(r.z, t2), l), relax<2>(t6), relax<2>(t6)};
        const Q2<2> y[4] = {relax<2>(t2), w2(add(r.z, t2), l), relax<2>(qx), relax<2>(t6)};
        prods<4>(c, x, y, l);
    }
    const E2 t3 = c[0], t9 = c[2], t66 = c[3];
    const E2 z = red(sub(c[1], add(zz, t3), l), l);
    const Q2<4> t4 = dbl(dbl(t3));
    E2 d[4];
    {
        const Q2<2> x[4] = {w2(t4, l), w2(t4, l), relax<2>(z), w2(add(qy, z), l)};
        const Q2<2> y[4] = {relax<2>(t2), relax<2>(r.x), relax<2>(z), w2(add(qy, z), l)};
        prods<4>(d, x, y, l);
    }
    const E2 t5 = d[0], t7 = d[1];
    const E2 x = red(sub(t66, red(add(t5, dbl(t7)), l), l), l);
    const E2 t10 = red(sub(d[3], add(yy, d[2]), l), l);
    E2 e[2];
    {
        const Q2<2> xs[2] = {w2(sub(t7, x, l), l), relax<2>(r.y)};
        const Q2<2> ys[2] = {relax<2>(t6), relax<2>(t5)};
        prods<2>(e, xs, ys, l);
    }
    r.y = red(sub(e[0], dbl(e[1]), l), l);
    r.x = x;
    r.z = z;
    Line ln;
    ln.c0 = red(dbl(z), l);
    ln.c1 = red(dbl(neg(t6, l)), l);
    ln.c2 = red(sub(dbl(t9), t10, l), l);
    return ln;
}
// ell, mod.rs:57-69: f.mul_by_014(c2, c1 P.x, c0 P.y)
PA_DEV E12 ell(const E12& f, const Line& c, const Q<1>& px, const Q<1>& py, const Lc& l) {
    Q<1> o[4];
    {
        const Q<1> x[4] = {c.c1.c0, c.c1.c1, c.c0.c0, c.c0.c1}, y[4] = {px, px, py, py};
        level<NQ>(o, x, y, l);
    }
    return mul_by_014(f, c.c2, {o[0], o[1]}, {o[2], o[3]}, l);
}
// the Miller value of one (P, Q) (neither at infinity): the reference's loop
// over the bits of |x| >> 1 below its top, one line per doubling / addition
PA_DEV E12 miller_loop(const Q<1>& px, const Q<1>& py, const E2& qx, const E2& qy, const Lc& l) {
    constexpr uint64_t kMask = (0xD201000000010000ull >> 1) & ((1ull << 62) - 1);
    G2J r = {qx, qy, one_e<Q2>(l)};
    E12 f = e12_one(l);
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        f = ell(f, dbl_step(r, l), px, py, l);
        if ((kMask >> bit) & 1) f = ell(f, add_step(r, qx, qy, l), px, py, l);   // wave-uniform
        f = sqr12(f, l);
    }
    f = ell(f, dbl_step(r, l), px, py, l);
    return conj12(f, l);
}

// ---------------- records ----------------
PA_DEV Q<1> load_q(const uint64_t* p, const Lc& l) {
    Fq x;
    fq_load(x, p);
    return from_abi(x, l);
}
PA_DEV E12 load12(const uint64_t* p, const Lc& l) {
    E2 v[6];
#pragma unroll
    for (int k = 0; k < 6; k++) v[k] = {load_q(p + 12 * k, l), load_q(p + 12 * k + 6, l)};
    return {{v[0], v[1], v[2]}, {v[3], v[4], v[5]}};
}
// the 24 Fq of f, canonical: lane k < 24 of the group stores Fq k (zero: all zero)
PA_DEV void store12(uint64_t* p, const E12& f, bool zero, int lg) {
    const E2 v[6] = {f.c0.c0, f.c0.c1, f.c0.c2, f.c1.c0, f.c1.c1, f.c1.c2};
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const Fq w = to_abi(k & 1 ? v[k >> 1].c1 : v[k >> 1].c0);
        if (lg == k) {
            Fq z = w;
            if (zero) {
#pragma unroll
                for (int i = 0; i < 12; i++) z.w[i] = 0;
            }
            fq_store(p + 6 * k, z);
        }
    }
}

}  // namespace pq
}  // namespace pa
