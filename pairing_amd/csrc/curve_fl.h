// G1 Jacobian group law on the lazy 28-bit core (fl.h), for the throughput
// kernels (fixed-base comb, MSM bucket accumulation) and the three-lane
// doubling chains.  Same formulas, same field values as curve.h
// (dbl-2009-l ec.rs:296-354, madd-2007-bl ec.rs:446-526); coordinates are
// F<1> (lazy, value < 2q) and become the reference's canonical bits at
// fl_store.
#pragma once
#include "curve.h"
#include "fl.h"

namespace pa {

// ---- G1 Jacobian arithmetic on the lazy core (same field values as curve.h) ----
struct FlJac {
    F<1> x, y, z;
};
PA_DEV bool fl_eq(const F<1>& a, const F<1>& b) { return fl_is_zero(sub(a, b)); }

// dbl-2009-l, ec.rs:296-354 (caller: z != 0)
PA_DEV void fl_jac_double(FlJac& p) {
    const F<1> a = sqr(p.x);
    const F<1> b = sqr(p.y);
    const F<1> c = sqr(b);
    const F<1> d = red(dbl(sub(sqr(add(p.x, b)), add(a, c))));
    const F<3> e = add(dbl(a), a);
    const F<1> f = sqr(e);
    p.z = red(dbl(mul(p.z, p.y)));
    p.x = red(sub(f, dbl(d)));
    p.y = red(sub(mul(e, sub(d, p.x)), dbl(dbl(dbl(c)))));
}

// madd-2007-bl, ec.rs:446-526: s += (ox, oy), (ox, oy) a nonzero affine point;
// `untouched` marks the initial identity (the reference's zero()), a Jacobian
// zero produced on the way (z == 0) is detected as jac_is_zero does
PA_DEV void fl_jac_add_mixed(FlJac& s, bool& untouched, const F<1>& ox, const F<2>& oy) {
    if (untouched || fl_is_zero(s.z)) {
        s.x = ox;
        s.y = red(oy);
        s.z = fl_one();
        untouched = false;
        return;
    }
    const F<1> z1z1 = sqr(s.z);
    const F<1> u2 = mul(ox, z1z1);
    const F<1> s2 = mul(mul(oy, s.z), z1z1);
    if (fl_eq(s.x, u2) && fl_eq(s.y, s2)) {
        fl_jac_double(s);
        return;
    }
    const F<3> h = sub(u2, s.x);
    const F<1> hh = sqr(h);
    const F<4> i = dbl(dbl(hh));
    const F<1> j = mul(h, i);
    const F<1> r = red(dbl(sub(s2, s.y)));
    const F<1> v = mul(s.x, i);
    const F<1> x3 = red(sub(sub(sub(sqr(r), j), v), v));
    const F<1> y3 = sop(r, sub(v, x3), j, neg(dbl(s.y)));   // r (v - x3) - 2 j y1, one reduction
    const F<1> z3 = red(sub(sub(sqr(add(s.z, red(h))), z1z1), hh));
    s.x = x3;
    s.y = y3;
    s.z = z3;
}

// add-2007-bl, ec.rs:356-444 (doubles when the points are equal); zero is
// z == 0, as jac_is_zero
PA_DEV void fl_jac_add(FlJac& s, const FlJac& o) {
    if (fl_is_zero(s.z)) {
        s = o;
        return;
    }
    if (fl_is_zero(o.z)) return;
    const F<1> z1z1 = sqr(s.z), z2z2 = sqr(o.z);
    const F<1> u1 = mul(s.x, z2z2), u2 = mul(o.x, z1z1);
    const F<1> s1 = mul(mul(s.y, o.z), z2z2), s2 = mul(mul(o.y, s.z), z1z1);
    if (fl_eq(u1, u2) && fl_eq(s1, s2)) {
        fl_jac_double(s);
        return;
    }
    const F<3> h = sub(u2, u1);
    const F<1> i = sqr(red(dbl(h)));
    const F<1> j = mul(h, i);
    const F<1> r = red(dbl(sub(s2, s1)));
    const F<1> v = mul(u1, i);
    const F<1> x3 = red(sub(sub(sub(sqr(r), j), v), v));
    const F<1> y3 = sop(r, sub(v, x3), j, neg(dbl(s1)));    // r (v - x3) - 2 s1 j, one reduction
    const F<1> z3 = mul(red(sub(sub(sqr(add(s.z, o.z)), z1z1), z2z2)), h);
    s.x = x3;
    s.y = y3;
    s.z = z3;
}

PA_DEV FlJac fl_load_jac(const uint64_t* p) {
    FlJac r;
    r.x = fl_load(p);
    r.y = fl_load(p + 6);
    r.z = fl_load(p + 12);
    return r;
}
PA_DEV void fl_store_jac(uint64_t* p, const FlJac& a) {
    fl_store(p, a.x);
    fl_store(p + 6, a.y);
    fl_store(p + 12, a.z);
}

PA_DEV F<1> fl_from_lane(const F<1>& x, int src) {
    F<1> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = (uint32_t)__builtin_amdgcn_readlane((int)x.w[i], src);
    return r;
}

// jac_double_3lane (curve.h) on the lazy core: dbl-2009-l's seven products
// in three dependent levels over lanes 0..2; every lane ends with the point.
// Caller: z != 0.
PA_DEV void fl_jac_double_3lane(FlJac& p, int lane) {
    F<1> m = mul(lane == 0 ? p.x : p.y, lane == 0 ? p.x : (lane == 1 ? p.y : p.z));
    const F<1> a = fl_from_lane(m, 0), b = fl_from_lane(m, 1), t = fl_from_lane(m, 2);
    const F<3> e = add(dbl(a), a);
    const F<3> s = lane == 0 ? relax<3>(b) : (lane == 1 ? relax<3>(add(p.x, b)) : e);
    m = sqr(s);
    const F<1> c = fl_from_lane(m, 0), dd = fl_from_lane(m, 1), f = fl_from_lane(m, 2);
    const F<1> d = red(dbl(sub(dd, add(a, c))));
    p.z = red(dbl(t));
    p.x = red(sub(f, dbl(d)));
    p.y = red(sub(mul(e, sub(d, p.x)), dbl(dbl(dbl(c)))));
}

// ---- four lanes per point (a quad: lanes 4k..4k+3, q = lane & 3) ----
// One coordinate of quad lane `src` in every lane of the quad (DPP
// quad_perm broadcast, no LDS).
template <int SRC>
PA_DEV F<1> fl_from_quad(const F<1>& x) {
    F<1> r;
    constexpr int ctrl = SRC * 0x55;   // quad_perm [SRC, SRC, SRC, SRC]
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.w[i], ctrl, 0xf, 0xf, false);
    return r;
}
template <int U>
PA_DEV F<U> pick4(int q, const F<U>& a, const F<U>& b, const F<U>& c, const F<U>& d) {
    F<U> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = q == 0 ? a.w[i] : (q == 1 ? b.w[i] : (q == 2 ? c.w[i] : d.w[i]));
    return r;
}

// fl_jac_add (add-2007-bl, ec.rs:421-481) with its sixteen products in five
// dependent levels over the four lanes of a quad -- the same products of the
// same operands, so the same field values; every lane of the quad holds both
// points on entry and the sum on exit.
PA_DEV void fl_jac_add_q(FlJac& s, const FlJac& o, int q) {
    if (fl_is_zero(s.z)) {
        s = o;
        return;
    }
    if (fl_is_zero(o.z)) return;
    F<1> m = mul(pick4(q, s.z, o.z, s.y, o.y), pick4(q, s.z, o.z, o.z, s.z));
    const F<1> z1z1 = fl_from_quad<0>(m), z2z2 = fl_from_quad<1>(m), y1z2 = fl_from_quad<2>(m),
               y2z1 = fl_from_quad<3>(m);
    m = mul(pick4(q, s.x, o.x, y1z2, y2z1), pick4(q, z2z2, z1z1, z2z2, z1z1));
    const F<1> u1 = fl_from_quad<0>(m), u2 = fl_from_quad<1>(m), s1 = fl_from_quad<2>(m), s2 = fl_from_quad<3>(m);
    if (fl_eq(u1, u2) && fl_eq(s1, s2)) {
        fl_jac_double(s);
        return;
    }
    const F<3> h = sub(u2, u1);
    const F<1> hh = red(dbl(h));
    const F<1> r = red(dbl(sub(s2, s1)));
    const F<2> zs = add(s.z, o.z);
    m = sqr(pick4(q, relax<2>(hh), relax<2>(r), zs, relax<2>(hh)));
    const F<1> i = fl_from_quad<0>(m), rr = fl_from_quad<1>(m), zz = fl_from_quad<2>(m);
    const F<1> zr = red(sub(sub(zz, z1z1), z2z2));
    m = mul(pick4(q, h, relax<3>(u1), relax<3>(zr), h), pick4(q, relax<3>(i), relax<3>(i), h, relax<3>(i)));
    const F<1> j = fl_from_quad<0>(m), v = fl_from_quad<1>(m), z3 = fl_from_quad<2>(m);
    const F<1> x3 = red(sub(sub(sub(rr, j), v), v));
    m = mul(pick4(q, r, s1, r, s1), pick4(q, relax<3>(sub(v, x3)), relax<3>(j), relax<3>(sub(v, x3)), relax<3>(j)));
    const F<1> t1 = fl_from_quad<0>(m), t2 = fl_from_quad<1>(m);
    s.x = x3;
    s.y = red(sub(t1, dbl(t2)));
    s.z = z3;
}

// fl_jac_double_3lane within a quad (lane 3 repeats lane 0's products)
PA_DEV void fl_jac_double_q(FlJac& p, int q) {
    F<1> m = mul(q == 1 ? p.y : (q == 2 ? p.y : p.x), q == 1 ? p.y : (q == 2 ? p.z : p.x));
    const F<1> a = fl_from_quad<0>(m), b = fl_from_quad<1>(m), t = fl_from_quad<2>(m);
    const F<3> e = add(dbl(a), a);
    const F<3> s = q == 1 ? relax<3>(add(p.x, b)) : (q == 2 ? e : relax<3>(b));
    m = sqr(s);
    const F<1> c = fl_from_quad<0>(m), dd = fl_from_quad<1>(m), f = fl_from_quad<2>(m);
    const F<1> d = red(dbl(sub(dd, add(a, c))));
    p.z = red(dbl(t));
    p.x = red(sub(f, dbl(d)));
    p.y = red(sub(mul(e, sub(d, p.x)), dbl(dbl(dbl(c)))));
}

}  // namespace pa
