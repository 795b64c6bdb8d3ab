// Lane-parallel lazy base-field arithmetic for the latency-bound decode path
// (kernels_decode.hip, k_decode_quad): one record per GROUP of NQ quads (G1:
// 4 quads = 16 lanes, G2: 8 quads = 32 lanes).  A value is SPREAD over a
// quad as in the cooperative VM (coop_quad.h): lane r = lane & 3 holds limbs
// 4r .. 4r+3 of the lazy 14 x 28-bit representation (fl.h), so one product is
// ~270 instructions per lane (quad::mont) instead of a ~700-instruction
// one-lane leaf.  The quads of a group run the same instruction stream on
// different operands: a level of independent products (the products of one
// Jacobian doubling level, the two coordinates of an Fq2 product) runs side by
// side, each quad picking its operands by its index j, and the results are
// broadcast back to every quad of the group (ds_swizzle within the group).
//
// Bounds are static as in fl.h: Q<U> has limbs <= U (2^28 - 1) and value
// < U 2q; products need sum U_a U_b <= 17 (the one-lane leaves' contract, so
// quad::mont's 64-bit column accumulators cannot overflow).
#pragma once
#include "coop_quad.h"

namespace pa {
namespace dq {

template <int U>
struct Q {
    static_assert(U >= 1 && U <= 16, "lazy bound out of range");
    uint32_t w[4];
};

// Per-lane context: the quad context (r, q limbs) plus this lane's pieces of
// the subtraction constants FL_SUB_C for subtrahend bounds 1..kSubB.
constexpr int kSubB = 8;
struct Lc {
    quad::Ctx c;
    int j;                       // quad index within the group
    uint32_t sc[kSubB][4];
};
PA_DEV uint32_t limb_of(const uint32_t* full14, int r, int k) {
    // full14[4r + k] without a runtime-indexed register array (pads -> 0)
    const uint32_t v0 = full14[k], v1 = full14[4 + k], v2 = full14[8 + k];
    const uint32_t v3 = k < 2 ? full14[12 + k] : 0u;
    return r == 0 ? v0 : r == 1 ? v1 : r == 2 ? v2 : v3;
}
PA_DEV Lc lctx(int lane, int nq) {
    Lc l;
    l.c = quad::ctx(lane);
    l.j = (lane >> 2) & (nq - 1);
#pragma unroll
    for (int b = 0; b < kSubB; b++) {
        uint32_t full[14];
#pragma unroll
        for (int i = 0; i < 14; i++) full[i] = FL_SUB_C[b][i];
#pragma unroll
        for (int k = 0; k < 4; k++) l.sc[b][k] = limb_of(full, l.c.r, k);
    }
    return l;
}

// ---- conversions between a spread piece and a whole one-lane value ----
template <int U>
PA_DEV Q<U> piece(const F<U>& x, const Lc& l) {
    Q<U> q;
#pragma unroll
    for (int k = 0; k < 4; k++) q.w[k] = limb_of(x.w, l.c.r, k);
    return q;
}
template <int U>
PA_DEV F<U> whole(const Q<U>& a) {
    F<U> f;
    quad::gather(f.w, a.w);
    return f;
}
PA_DEV Q<1> qconst(const uint32_t* c14, const Lc& l) {
    Q<1> q;
#pragma unroll
    for (int k = 0; k < 4; k++) q.w[k] = limb_of(c14, l.c.r, k);
    return q;
}

// ---- additive ops (limb-wise; no carries) ----
template <int A, int B>
PA_DEV Q<A + B> add(const Q<A>& a, const Q<B>& b) {
    Q<A + B> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = a.w[k] + b.w[k];
    return r;
}
template <int A>
PA_DEV Q<2 * A> dbl(const Q<A>& a) { return add(a, a); }
template <int A, int B>
PA_DEV Q<A + subcu(B)> sub(const Q<A>& a, const Q<B>& b, const Lc& l) {
    static_assert(B <= kSubB, "subtrahend bound beyond the loaded constants");
    Q<A + subcu(B)> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = a.w[k] + l.sc[B - 1][k] - b.w[k];
    return r;
}
template <int B>
PA_DEV Q<subcu(B)> neg(const Q<B>& b, const Lc& l) {
    static_assert(B <= kSubB, "subtrahend bound beyond the loaded constants");
    Q<subcu(B)> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = l.sc[B - 1][k] - b.w[k];
    return r;
}
template <int U2, int U1>
PA_DEV Q<U2> relax(const Q<U1>& a) {
    static_assert(U2 >= U1, "relax can only widen a bound");
    Q<U2> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = a.w[k];
    return r;
}
template <int U>
PA_DEV Q<1> red(const Q<U>& a, const Lc& l) {
    Q<1> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = a.w[k];
    if constexpr (U > 1) quad::red(r.w, l.c);
    return r;
}

// ---- products ----
template <int A, int B>
PA_DEV Q<1> mul(const Q<A>& a, const Q<B>& b, const Lc& l) {
    static_assert(A * B <= 17, "product column bound");
    uint32_t fa[14];
    quad::gather(fa, a.w);
    Q<1> r;
    quad::mont<false>(r.w, fa, b.w, nullptr, nullptr, l.c);
    return r;
}
template <int A>
PA_DEV Q<1> sqr(const Q<A>& a, const Lc& l) { return mul(a, a, l); }
// a b + c d, one reduction
template <int A, int B, int C, int D>
PA_DEV Q<1> sop(const Q<A>& a, const Q<B>& b, const Q<C>& c, const Q<D>& d, const Lc& l) {
    static_assert(A * B + C * D <= 17, "sum-of-products column bound");
    uint32_t fa[14], fc[14];
    quad::gather(fa, a.w);
    quad::gather(fc, c.w);
    Q<1> r;
    quad::mont<true>(r.w, fa, b.w, fc, d.w, l.c);
    return r;
}

// ---- per-quad operand choice and group broadcast ----
// v[j] for this lane's quad j (j >= n: the last one), every input widened to U
template <int U, int N>
PA_DEV Q<U> pick(const Q<U> (&v)[N], int j) {
    Q<U> r = v[N - 1];
#pragma unroll
    for (int i = N - 2; i >= 0; i--) {
#pragma unroll
        for (int k = 0; k < 4; k++) r.w[k] = j == i ? v[i].w[k] : r.w[k];
    }
    return r;
}
// quad K's piece of `a`, in every quad of the group (ds_swizzle bit mode on
// 32-lane halves: source lane = (lane & and) | or)
template <int NQ, int K, int U>
PA_DEV Q<U> bq(const Q<U>& a) {
    static_assert(NQ == 4 || NQ == 8, "group of 4 or 8 quads");
    static_assert(K < NQ, "quad index");
    constexpr int and_mask = NQ == 4 ? 0x13 : 0x03;
    constexpr int pattern = and_mask | ((4 * K) << 5);
    Q<U> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = (uint32_t)__builtin_amdgcn_ds_swizzle((int)a.w[k], pattern);
    return r;
}

// ---- tests and exits (one-lane tail over the gathered value) ----
template <int U>
PA_DEV bool is_zero(const Q<U>& a) { return fl_is_zero(whole(a)); }
template <int A, int B>
PA_DEV bool eq(const Q<A>& a, const Q<B>& b, const Lc& l) {
    static_assert(B <= kSubB, "subtrahend bound");
    return is_zero(sub(a, b, l));
}
template <int U>
PA_DEV Fq to_abi(const Q<U>& a) { return fl_to_abi(whole(a)); }
PA_DEV Q<1> from_abi(const Fq& x, const Lc& l) { return piece(fl_from_abi(x), l); }
template <int U>
PA_DEV Q<U> sel(bool c, const Q<U>& a, const Q<U>& b) {
    Q<U> r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.w[k] = c ? a.w[k] : b.w[k];
    return r;
}

// x^e for a wave-uniform exponent e (top = index of e's top set bit): a 4-bit
// sliding window, the odd powers x, x^3, .., x^15 first (same schedule as
// kernels_decode.hip pow_fixed); every quad of the group computes it
PA_DEV Q<1> win_mul(const Q<1>& acc, const Q<1> (&t)[8], int v, const Lc& l) {
    switch (v >> 1) {
        case 0: return mul(acc, t[0], l);
        case 1: return mul(acc, t[1], l);
        case 2: return mul(acc, t[2], l);
        case 3: return mul(acc, t[3], l);
        case 4: return mul(acc, t[4], l);
        case 5: return mul(acc, t[5], l);
        case 6: return mul(acc, t[6], l);
        default: return mul(acc, t[7], l);
    }
}
PA_DEV Q<1> pow_fixed(const Q<1>& x, const uint64_t* e, int top, const Lc& l) {
    auto bit_of = [&](int b) { return (int)((e[b >> 6] >> (b & 63)) & 1); };
    Q<1> t[8];
    t[0] = x;
    const Q<1> x2 = sqr(x, l);
#pragma unroll
    for (int k = 1; k < 8; k++) t[k] = mul(t[k - 1], x2, l);
    Q<1> acc = x;   // the top set bit
    int bit = top - 1;
#pragma unroll 1
    while (bit >= 0) {
        if (!bit_of(bit)) {
            acc = sqr(acc, l);
            bit--;
            continue;
        }
        int lo = bit - 3 < 0 ? 0 : bit - 3;
        while (!bit_of(lo)) lo++;
        int v = 0;
#pragma unroll 1
        for (int b = bit; b >= lo; b--) {
            acc = sqr(acc, l);
            v = 2 * v + bit_of(b);
        }
        acc = win_mul(acc, t, v, l);
        bit = lo - 1;
    }
    return acc;
}

// ---- Fq2 pieces (two spread Fq values) ----
template <int U>
struct Q2 {
    Q<U> c0, c1;
};
template <int A, int B>
PA_DEV Q2<A + B> add(const Q2<A>& a, const Q2<B>& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
template <int A>
PA_DEV Q2<2 * A> dbl(const Q2<A>& a) { return add(a, a); }
template <int A, int B>
PA_DEV Q2<A + subcu(B)> sub(const Q2<A>& a, const Q2<B>& b, const Lc& l) {
    return {sub(a.c0, b.c0, l), sub(a.c1, b.c1, l)};
}
template <int B>
PA_DEV Q2<subcu(B)> neg(const Q2<B>& b, const Lc& l) { return {neg(b.c0, l), neg(b.c1, l)}; }
template <int U2, int U1>
PA_DEV Q2<U2> relax(const Q2<U1>& a) { return {relax<U2>(a.c0), relax<U2>(a.c1)}; }
template <int U>
PA_DEV Q2<1> red(const Q2<U>& a, const Lc& l) { return {red(a.c0, l), red(a.c1, l)}; }
template <int U>
PA_DEV Q2<U> sel(bool c, const Q2<U>& a, const Q2<U>& b) { return {sel(c, a.c0, b.c0), sel(c, a.c1, b.c1)}; }
template <int U>
PA_DEV bool is_zero(const Q2<U>& a) { return is_zero(a.c0) && is_zero(a.c1); }
template <int A, int B>
PA_DEV bool eq(const Q2<A>& a, const Q2<B>& b, const Lc& l) { return is_zero(sub(a, b, l)); }

// ---- one level of independent products over the group's quads ----
namespace detail {
template <int NQ, int U, int M, int K = 0>
PA_DEV void bcast_all(Q<1> (&out)[M], const Q<U>& p) {
    if constexpr (K < M) {
        out[K] = bq<NQ, K>(p);
        bcast_all<NQ, U, M, K + 1>(out, p);
    }
}
template <int NQ, int M, int K = 0>
PA_DEV void bcast_all2(Q2<1> (&out)[M], const Q<1>& p) {
    if constexpr (K < M) {
        out[K].c0 = bq<NQ, 2 * K>(p);
        out[K].c1 = bq<NQ, 2 * K + 1>(p);
        bcast_all2<NQ, M, K + 1>(out, p);
    }
}
}  // namespace detail

// out[m] = x[m] y[m] for m < M <= NQ: quad m computes product m
template <int NQ, int UX, int UY, int M>
PA_DEV void level(Q<1> (&out)[M], const Q<UX> (&x)[M], const Q<UY> (&y)[M], const Lc& l) {
    static_assert(M <= NQ, "one product per quad");
    const Q<1> p = mul(pick(x, l.j), pick(y, l.j), l);
    detail::bcast_all<NQ, 1, M>(out, p);
}
// Fq2 products out[m] = x[m] y[m] (fq2.rs:123-136) for m < M <= NQ / 2: quad
// 2m computes c0 = x0 y0 - x1 y1, quad 2m + 1 computes c1 = x0 y1 + x1 y0, both
// as one two-term product (so every quad runs the same instruction stream)
template <int NQ, int UX, int UY, int M>
PA_DEV void level2(Q2<1> (&out)[M], const Q2<UX> (&x)[M], const Q2<UY> (&y)[M], const Lc& l) {
    static_assert(2 * M <= NQ, "two quads per Fq2 product");
    constexpr int UC = cmax(UX, subcu(UX));
    Q<UX> x0s[M], x1s[M];
    Q<UY> y0s[M], y1s[M];
#pragma unroll
    for (int m = 0; m < M; m++) {
        x0s[m] = x[m].c0;
        x1s[m] = x[m].c1;
        y0s[m] = y[m].c0;
        y1s[m] = y[m].c1;
    }
    const int m = l.j >> 1;
    const bool odd = (l.j & 1) != 0;
    const Q<UX> a = pick(x0s, m), x1 = pick(x1s, m);
    const Q<UY> y0 = pick(y0s, m), y1 = pick(y1s, m);
    const Q<UC> c = sel(odd, relax<UC>(x1), relax<UC>(neg(x1, l)));
    const Q<UY> b = sel(odd, y1, y0), d = sel(odd, y0, y1);
    const Q<1> p = sop(a, b, c, d, l);
    detail::bcast_all2<NQ, M>(out, p);
}

// ---- Jacobian group law over spread values (G1: E = Q, G2: E = Q2) ----
template <template <int> class E>
struct Jq {
    E<1> x, y, z;
};
// the fixed operand T of [|x|] T: T, Z^2, Z^3, 2T
template <template <int> class E>
struct Fixed {
    Jq<E> t, t2;
    E<1> zz, zzz;
};

template <int NQ, int UX, int UY, int M>
PA_DEV void lev(Q<1> (&o)[M], const Q<UX> (&x)[M], const Q<UY> (&y)[M], const Lc& l) {
    level<NQ>(o, x, y, l);
}
template <int NQ, int UX, int UY, int M>
PA_DEV void lev(Q2<1> (&o)[M], const Q2<UX> (&x)[M], const Q2<UY> (&y)[M], const Lc& l) {
    level2<NQ>(o, x, y, l);
}
template <int NQ, template <int> class E, int UX, int UY>
PA_DEV E<1> prod(const E<UX>& x, const E<UY>& y, const Lc& l) {
    E<1> o[1];
    const E<UX> xs[1] = {x};
    const E<UY> ys[1] = {y};
    lev<NQ>(o, xs, ys, l);
    return o[0];
}

// dbl-2009-l (ec.rs:296-354; the field values of kernels_decode.hip
// fl_double_any): product levels {X^2, Y^2, Z Y}, {b^2, (X + b)^2, e^2},
// {e (d - X3)}
template <int NQ, template <int> class E>
PA_DEV void jdbl(Jq<E>& p, const Lc& l) {
    E<1> l1[3];
    {
        const E<1> xs[3] = {p.x, p.y, p.z}, ys[3] = {p.x, p.y, p.y};
        lev<NQ>(l1, xs, ys, l);
    }
    const E<1> a = l1[0], b = l1[1], zy = l1[2];
    const E<1> e = red(add(dbl(a), a), l);
    E<1> l2[3];
    {
        const E<2> xs[3] = {relax<2>(b), add(p.x, b), relax<2>(e)};
        lev<NQ>(l2, xs, xs, l);
    }
    const E<1> c = l2[0], s = l2[1], f = l2[2];
    const E<1> d = red(dbl(sub(s, add(a, c), l)), l);
    p.x = red(sub(f, dbl(d), l), l);
    p.z = red(dbl(zy), l);
    const E<1> y3 = prod<NQ, E>(e, sub(d, p.x, l), l);
    p.y = red(sub(y3, dbl(dbl(dbl(c))), l), l);
}

PA_DEV Q<1> zero_q() {
    Q<1> z;
#pragma unroll
    for (int k = 0; k < 4; k++) z.w[k] = 0;
    return z;
}
template <template <int> class E>
PA_DEV E<1> one_e(const Lc& l);
template <>
PA_DEV Q<1> one_e<Q>(const Lc& l) { return qconst(FL_ONE, l); }
template <>
PA_DEV Q2<1> one_e<Q2>(const Lc& l) { return {qconst(FL_ONE, l), zero_q()}; }
template <template <int> class E>
PA_DEV E<1> zero_e();
template <>
PA_DEV Q<1> zero_e<Q>() { return zero_q(); }
template <>
PA_DEV Q2<1> zero_e<Q2>() { return {zero_q(), zero_q()}; }

// R + T by add-2007-bl (ec.rs:356-444) with T's Z^2, Z^3 and 2T precomputed:
// product levels {Z1^2, X1 Z2^2, Y1 Z2^3, (Z1 + Z2)^2}, {X2 Z1Z1, Z1 Z1Z1},
// {Y2 Z1^3, (2H)^2}, {H I, U1 I, r^2, (..) H}, {r (V - X3), S1 J}; R = 0 gives T,
// R = T gives 2T, R = -T gives 0 (the reference's special cases)
template <int NQ, template <int> class E>
PA_DEV void jadd(Jq<E>& r, const Fixed<E>& f, const Lc& l) {
    const bool rz = is_zero(r.z);
    E<1> l1[4];
    {
        const E<2> zs = add(r.z, f.t.z);
        const E<2> xs[4] = {relax<2>(r.z), relax<2>(r.x), relax<2>(r.y), zs};
        const E<2> ys[4] = {relax<2>(r.z), relax<2>(f.zz), relax<2>(f.zzz), zs};
        lev<NQ>(l1, xs, ys, l);
    }
    const E<1> z1z1 = l1[0], u1 = l1[1], s1 = l1[2], w = l1[3];
    E<1> l2[2];
    {
        const E<1> xs[2] = {f.t.x, r.z}, ys[2] = {z1z1, z1z1};
        lev<NQ>(l2, xs, ys, l);
    }
    const E<1> u2 = l2[0], t1 = l2[1];
    const E<1> h = red(sub(u2, u1, l), l);
    E<1> l3[2];
    {
        const E<2> xs[2] = {relax<2>(f.t.y), dbl(h)}, ys[2] = {relax<2>(t1), dbl(h)};
        lev<NQ>(l3, xs, ys, l);
    }
    const E<1> s2 = l3[0], ii = l3[1];
    const E<1> rr = red(dbl(sub(s2, s1, l)), l);
    const E<1> zp = red(sub(sub(w, z1z1, l), f.zz, l), l);
    E<1> l4[4];
    {
        const E<1> xs[4] = {h, u1, rr, zp}, ys[4] = {ii, ii, rr, h};
        lev<NQ>(l4, xs, ys, l);
    }
    const E<1> j = l4[0], v = l4[1], rsq = l4[2], z3 = l4[3];
    const E<1> x3 = red(sub(sub(rsq, j, l), dbl(v), l), l);
    E<1> l5[2];
    {
        const E<1> xs[2] = {rr, s1};
        const E<3> ys[2] = {sub(v, x3, l), relax<3>(j)};
        lev<NQ>(l5, xs, ys, l);
    }
    const E<1> y3 = red(sub(l5[0], dbl(l5[1]), l), l);
    const bool hz = is_zero(h), rzero = is_zero(rr);
    if (rz) {
        r = f.t;
    } else if (hz && rzero) {
        r = f.t2;
    } else if (hz) {   // R = -T: the zero point
        r.x = one_e<E>(l);
        r.y = one_e<E>(l);
        r.z = zero_e<E>();
    } else {
        r.x = x3;
        r.y = y3;
        r.z = z3;
    }
}

// T with its Z^2, Z^3 and 2T (the fixed operand of repeated additions R + T)
template <int NQ, template <int> class E>
PA_DEV Fixed<E> make_fixed(const Jq<E>& t, const Lc& l) {
    Fixed<E> f;
    f.t = t;
    f.zz = prod<NQ, E>(t.z, t.z, l);
    f.zzz = prod<NQ, E>(f.zz, t.z, l);
    f.t2 = t;
    jdbl<NQ>(f.t2, l);
    return f;
}

// Fq2 square x^2 (fq2.rs:87-101) on two quads with ONE product each: quad 0
// c0 = (x0 + x1)(x0 - x1), quad 1 c1 = (2 x0) x1 (both quads run mul)
template <int NQ>
PA_DEV Q2<1> sqr2(const Q2<1>& x, const Lc& l) {
    const bool odd = (l.j & 1) != 0;
    const Q<2> a = sel(odd, dbl(x.c0), add(x.c0, x.c1));
    const Q<3> b = sel(odd, relax<3>(x.c1), sub(x.c0, x.c1, l));
    const Q<1> p = mul(a, b, l);
    return {bq<NQ, 0>(p), bq<NQ, 1>(p)};
}

}  // namespace dq
}  // namespace pa
