// G2 Jacobian group law on the lazy 28-bit core's Fq2 (tower_fl.h), for the
// G2 MSM's bucket phases.  The formulas and field values of curve.h over Fq2
// (dbl-2009-l ec.rs:296-354, add-2007-bl ec.rs:356-444, madd-2007-bl
// ec.rs:446-526); the red() calls sit where an Fq2 product's column bound
// (fl.h, tower_fl.h) would otherwise be exceeded, so they differ from
// curve_fl.h's G1 ones but not in value.  Coordinates leave canonical
// (fl_store), as the 12-word core writes them.
#pragma once
#include "curve_fl.h"
#include "tower_fl.h"

namespace pa {

struct FlJac2 {
    F2<1> x, y, z;
};

template <int U>
PA_DEV bool f2_is_zero(const F2<U>& a) {
    return fl_is_zero(a.c0) && fl_is_zero(a.c1);
}
PA_DEV bool f2_eq(const F2<1>& a, const F2<1>& b) { return f2_is_zero(sub(a, b)); }
PA_DEV FlJac2 fl2_jac_zero() { return {f2_zero(), f2_one(), f2_zero()}; }

// dbl-2009-l, ec.rs:296-354 (caller: z != 0)
PA_DEV void fl2_jac_double(FlJac2& p) {
    const F2<1> a = sqr(p.x);
    const F2<1> b = sqr(p.y);
    const F2<1> c = sqr(b);
    const F2<1> d = red(dbl(sub(sqr(add(p.x, b)), add(a, c))));
    const F2<1> e = red(add(dbl(a), a));
    const F2<1> f = sqr(e);
    p.z = red(dbl(mul(p.z, p.y)));
    p.x = red(sub(f, dbl(d)));
    p.y = red(sub(mul(e, sub(d, p.x)), dbl(dbl(dbl(c)))));
}

// madd-2007-bl, ec.rs:446-526: s += (ox, oy), (ox, oy) a nonzero affine point;
// `untouched` marks the initial identity, a Jacobian zero met on the way
// (z == 0) is detected as jac_is_zero does
PA_DEV void fl2_jac_add_mixed(FlJac2& s, bool& untouched, const F2<1>& ox, const F2<2>& oy) {
    if (untouched || f2_is_zero(s.z)) {
        s.x = ox;
        s.y = red(oy);
        s.z = f2_one();
        untouched = false;
        return;
    }
    const F2<1> z1z1 = sqr(s.z);
    const F2<1> u2 = mul(ox, z1z1);
    const F2<1> s2 = mul(mul(oy, s.z), z1z1);
    if (f2_eq(s.x, u2) && f2_eq(s.y, s2)) {
        fl2_jac_double(s);
        return;
    }
    const F2<1> h = red(sub(u2, s.x));
    const F2<1> hh = sqr(h);
    const F2<4> i = dbl(dbl(hh));
    const F2<1> j = mul(h, i);
    const F2<1> r = red(dbl(sub(s2, s.y)));
    const F2<1> v = mul(s.x, i);
    const F2<1> x3 = red(sub(sub(sub(sqr(r), j), v), v));
    const F2<1> y3 = red(sub(mul(r, sub(v, x3)), dbl(mul(j, s.y))));
    const F2<1> z3 = red(sub(sub(sqr(add(s.z, h)), z1z1), hh));
    s.x = x3;
    s.y = y3;
    s.z = z3;
}

// add-2007-bl, ec.rs:356-444 (doubles when the points are equal); zero is z == 0
PA_DEV void fl2_jac_add(FlJac2& s, const FlJac2& o) {
    if (f2_is_zero(s.z)) {
        s = o;
        return;
    }
    if (f2_is_zero(o.z)) return;
    const F2<1> z1z1 = sqr(s.z), z2z2 = sqr(o.z);
    const F2<1> u1 = mul(s.x, z2z2), u2 = mul(o.x, z1z1);
    const F2<1> s1 = mul(mul(s.y, o.z), z2z2), s2 = mul(mul(o.y, s.z), z1z1);
    if (f2_eq(u1, u2) && f2_eq(s1, s2)) {
        fl2_jac_double(s);
        return;
    }
    const F2<1> h = red(sub(u2, u1));
    const F2<1> i = sqr(red(dbl(h)));
    const F2<1> j = mul(h, i);
    const F2<1> r = red(dbl(sub(s2, s1)));
    const F2<1> v = mul(u1, i);
    const F2<1> x3 = red(sub(sub(sub(sqr(r), j), v), v));
    const F2<1> y3 = red(sub(mul(r, sub(v, x3)), dbl(mul(s1, j))));
    const F2<1> z3 = mul(red(sub(sub(sqr(add(s.z, o.z)), z1z1), z2z2)), h);
    s.x = x3;
    s.y = y3;
    s.z = z3;
}

// pa_g2 records (36 u64: x, y, z as Fq2 = c0, c1)
PA_DEV F2<1> fl2_load(const uint64_t* p) { return {fl_load(p), fl_load(p + 6)}; }
template <int U>
PA_DEV void fl2_store(uint64_t* p, const F2<U>& a) {
    fl_store(p, a.c0);
    fl_store(p + 6, a.c1);
}
PA_DEV FlJac2 fl2_load_jac(const uint64_t* p) { return {fl2_load(p), fl2_load(p + 12), fl2_load(p + 24)}; }
PA_DEV void fl2_store_jac(uint64_t* p, const FlJac2& a) {
    fl2_store(p, a.x);
    fl2_store(p + 12, a.y);
    fl2_store(p + 24, a.z);
}

}  // namespace pa
