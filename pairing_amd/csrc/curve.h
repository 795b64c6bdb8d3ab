// Device-side Jacobian group law for G1 (over Fq) and G2 (over Fq2), gfx950.
//
// One template instantiated twice, as the reference's `curve_impl!` macro is
// (src/bls12_381/ec.rs:1-621).  Jacobian coordinates are NOT canonical, so
// every formula below reproduces the reference's field-value sequence exactly
// (dbl-2009-l ec.rs:296-354, add-2007-bl 356-444, madd-2007-bl 446-526):
// a point computed here has the same (X, Y, Z) bits as the reference's.
#pragma once
#include "tower.h"

namespace pa {

// ---- Fq overloads so the curve template reads the same for G1 and G2 ----
PA_DEV void zero(Fq& r) { fq_zero(r); }
PA_DEV void one(Fq& r) { fq_one(r); }
PA_DEV bool is_zero(const Fq& a) { return fq_is_zero(a); }
PA_DEV bool eq(const Fq& a, const Fq& b) { return fq_eq(a, b); }
PA_DEV bool is_one(const Fq& a) { return fq_is_one(a); }
PA_DEV void add(Fq& r, const Fq& a, const Fq& b) { fq_add(r, a, b); }
PA_DEV void sub(Fq& r, const Fq& a, const Fq& b) { fq_sub(r, a, b); }
PA_DEV void dbl(Fq& r, const Fq& a) { fq_dbl(r, a); }
PA_DEV void neg(Fq& r, const Fq& a) { fq_neg(r, a); }
PA_DEV void mul(Fq& r, const Fq& a, const Fq& b) { fq_mul(r, a, b); }
PA_DEV void sqr(Fq& r, const Fq& a) { fq_sqr(r, a); }
PA_DEV bool inverse(Fq& r, const Fq& a) { return fq_inv(r, a); }
PA_DEV void load(Fq& r, const uint64_t* p) { fq_load(r, p); }
PA_DEV void store(uint64_t* p, const Fq& a) { fq_store(p, a); }

// 8-byte-aligned loads for the affine structs (104 B / 200 B records)
PA_DEV void load8(Fq& r, const uint64_t* p) {
    const uint2* v = reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < 6; i++) {
        uint2 x = v[i];
        r.w[2 * i] = x.x;
        r.w[2 * i + 1] = x.y;
    }
}
PA_DEV void store8(uint64_t* p, const Fq& a) {
    uint2* v = reinterpret_cast<uint2*>(p);
#pragma unroll
    for (int i = 0; i < 6; i++) v[i] = make_uint2(a.w[2 * i], a.w[2 * i + 1]);
}
PA_DEV void load8(Fq2& r, const uint64_t* p) { load8(r.c0, p); load8(r.c1, p + 6); }
PA_DEV void store8(uint64_t* p, const Fq2& a) { store8(p, a.c0); store8(p + 6, a.c1); }

template <class F>
struct Jac {
    F x, y, z;
};
template <class F>
struct Aff {
    F x, y;
    bool inf;
};

// words per field element in the u64 ABI layout
template <class F> struct FieldWords;
template <> struct FieldWords<Fq> { static constexpr int n = 6; };
template <> struct FieldWords<Fq2> { static constexpr int n = 12; };

template <class F>
PA_DEV void jac_zero(Jac<F>& p) {  // ec.rs:224-230
    zero(p.x);
    one(p.y);
    zero(p.z);
}
template <class F>
PA_DEV bool jac_is_zero(const Jac<F>& p) { return is_zero(p.z); }
template <class F>
PA_DEV bool jac_is_normalized(const Jac<F>& p) { return is_zero(p.z) || is_one(p.z); }

template <class F>
PA_DEV void jac_from_affine(Jac<F>& r, const Aff<F>& a) {  // ec.rs:570-582
    if (a.inf) {
        jac_zero(r);
    } else {
        r.x = a.x;
        r.y = a.y;
        one(r.z);
    }
}

// dbl-2009-l, ec.rs:296-354
template <class F>
PA_DEV void jac_double(Jac<F>& p) {
    if (jac_is_zero(p)) return;
    F a, b, c, d, e, f;
    sqr(a, p.x);
    sqr(b, p.y);
    sqr(c, b);
    add(d, p.x, b);
    sqr(d, d);
    sub(d, d, a);
    sub(d, d, c);
    dbl(d, d);
    dbl(e, a);
    add(e, e, a);
    sqr(f, e);
    mul(p.z, p.z, p.y);
    dbl(p.z, p.z);
    sub(p.x, f, d);
    sub(p.x, p.x, d);
    sub(p.y, d, p.x);
    mul(p.y, p.y, e);
    dbl(c, c);
    dbl(c, c);
    dbl(c, c);
    sub(p.y, p.y, c);
}

// add-2007-bl, ec.rs:356-444 (doubles when the points are equal)
template <class F>
PA_DEV void jac_add(Jac<F>& s, const Jac<F>& o) {
    if (jac_is_zero(s)) {
        s = o;
        return;
    }
    if (jac_is_zero(o)) return;
    F z1z1, z2z2, u1, u2, s1, s2;
    sqr(z1z1, s.z);
    sqr(z2z2, o.z);
    mul(u1, s.x, z2z2);
    mul(u2, o.x, z1z1);
    mul(s1, s.y, o.z);
    mul(s1, s1, z2z2);
    mul(s2, o.y, s.z);
    mul(s2, s2, z1z1);
    if (eq(u1, u2) && eq(s1, s2)) {
        jac_double(s);
        return;
    }
    F h, i, j, r, v;
    sub(h, u2, u1);
    dbl(i, h);
    sqr(i, i);
    mul(j, h, i);
    sub(r, s2, s1);
    dbl(r, r);
    mul(v, u1, i);
    sqr(s.x, r);
    sub(s.x, s.x, j);
    sub(s.x, s.x, v);
    sub(s.x, s.x, v);
    sub(s.y, v, s.x);
    mul(s.y, s.y, r);
    mul(s1, s1, j);
    dbl(s1, s1);
    sub(s.y, s.y, s1);
    add(s.z, s.z, o.z);
    sqr(s.z, s.z);
    sub(s.z, s.z, z1z1);
    sub(s.z, s.z, z2z2);
    mul(s.z, s.z, h);
}

// madd-2007-bl, ec.rs:446-526
template <class F>
PA_DEV void jac_add_mixed(Jac<F>& s, const Aff<F>& o) {
    if (o.inf) return;
    if (jac_is_zero(s)) {
        s.x = o.x;
        s.y = o.y;
        one(s.z);
        return;
    }
    F z1z1, u2, s2;
    sqr(z1z1, s.z);
    mul(u2, o.x, z1z1);
    mul(s2, o.y, s.z);
    mul(s2, s2, z1z1);
    if (eq(s.x, u2) && eq(s.y, s2)) {
        jac_double(s);
        return;
    }
    F h, hh, i, j, r, v;
    sub(h, u2, s.x);
    sqr(hh, h);
    dbl(i, hh);
    dbl(i, i);
    mul(j, h, i);
    sub(r, s2, s.y);
    dbl(r, r);
    mul(v, s.x, i);
    sqr(s.x, r);
    sub(s.x, s.x, j);
    sub(s.x, s.x, v);
    sub(s.x, s.x, v);
    mul(j, j, s.y);
    dbl(j, j);
    sub(s.y, v, s.x);
    mul(s.y, s.y, r);
    sub(s.y, s.y, j);
    add(s.z, s.z, h);
    sqr(s.z, s.z);
    sub(s.z, s.z, z1z1);
    sub(s.z, s.z, hh);
}

// ---- cooperative doubling (three lanes of one wave) ----
// Broadcast lane `src`'s value to every lane (v_readlane into SGPRs).
PA_DEV Fq from_lane(const Fq& x, int src) {
    Fq r;
#pragma unroll
    for (int i = 0; i < 12; i++) r.w[i] = (uint32_t)__builtin_amdgcn_readlane((int)x.w[i], src);
    return r;
}
PA_DEV Fq2 from_lane(const Fq2& x, int src) {
    Fq2 r;
    r.c0 = from_lane(x.c0, src);
    r.c1 = from_lane(x.c1, src);
    return r;
}

// dbl-2009-l (ec.rs:296-354) with its seven products spread over three lanes
// of one wave: the products form three dependent levels
//   (A = X^2, B = Y^2, T = Y Z) -> (C = B^2, (X + B)^2, F = (3A)^2) -> E (D - X3)
// so a doubling costs three product latencies instead of seven -- for the
// one-lane serial chains (comb bases, MSM Horner step).  Every lane of the
// wave must call it with the same point; every lane ends with the result,
// the same field values as jac_double.
template <class F>
PA_DEV void jac_double_3lane(Jac<F>& p, int lane) {
    if (is_zero(p.z)) return;  // uniform
    F s1, s2, m;
    s1 = lane == 0 ? p.x : p.y;
    s2 = lane == 0 ? p.x : (lane == 1 ? p.y : p.z);
    mul(m, s1, s2);
    const F a = from_lane(m, 0), b = from_lane(m, 1), t = from_lane(m, 2);
    F e, xb;
    dbl(e, a);
    add(e, e, a);
    add(xb, p.x, b);
    s1 = lane == 0 ? b : (lane == 1 ? xb : e);
    sqr(m, s1);
    const F c = from_lane(m, 0), dd = from_lane(m, 1), f = from_lane(m, 2);
    F d;
    sub(d, dd, a);
    sub(d, d, c);
    dbl(d, d);
    dbl(p.z, t);
    sub(p.x, f, d);
    sub(p.x, p.x, d);
    sub(p.y, d, p.x);
    mul(p.y, p.y, e);
    F c8;
    dbl(c8, c);
    dbl(c8, c8);
    dbl(c8, c8);
    sub(p.y, p.y, c8);
}

// wnaf_form's add_nocarry wrap (wnaf.rs:24-35).  Only the first digit can
// wrap: for an odd repr s with s mod 2^(w+1) > 2^w the recoding adds
// 2^(w+1) - (s mod 2^(w+1)), which overflows 2^256 exactly when bits w..255
// of s are all ones; the digits then spell s - 2^256 = -(2^256 - s).  On such
// an s this replaces s by t = 2^256 - s (< 2^w) and returns true, so the caller
// multiplies by t and negates; window <= 0 keeps s (the exact product).
PA_DEV bool wnaf_wrap(uint64_t s[4], int window) {
    if (window <= 0 || window >= 64 || !(s[0] & 1)) return false;
    const bool wraps = (s[0] | ((1ull << window) - 1)) == ~0ull && (s[1] & s[2] & s[3]) == ~0ull;
    if (wraps) {
        uint64_t c = 1;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t v = ~s[k] + c;
            c = (c && v == 0) ? 1 : 0;
            s[k] = v;
        }
    }
    return wraps;
}

template <class F>
PA_DEV void jac_negate(Jac<F>& p) {  // ec.rs:528-532
    if (!jac_is_zero(p)) neg(p.y, p.y);
}
template <class F>
PA_DEV void jac_sub(Jac<F>& s, const Jac<F>& o) {  // lib.rs:156-160
    Jac<F> t = o;
    jac_negate(t);
    jac_add(s, t);
}

// into_affine, ec.rs:586-619
template <class F>
PA_DEV void jac_to_affine(Aff<F>& a, const Jac<F>& p) {
    if (jac_is_zero(p)) {
        zero(a.x);
        one(a.y);
        a.inf = true;
        return;
    }
    a.inf = false;
    if (is_one(p.z)) {
        a.x = p.x;
        a.y = p.y;
        return;
    }
    F zinv, zp;
    inverse(zinv, p.z);
    sqr(zp, zinv);
    mul(a.x, p.x, zp);
    mul(zp, zp, zinv);
    mul(a.y, p.y, zp);
}

// ---- HBM records (u64 ABI layout) ----
template <class F>
PA_DEV void load_jac(Jac<F>& r, const uint64_t* p) {
    constexpr int W = FieldWords<F>::n;
    load(r.x, p);
    load(r.y, p + W);
    load(r.z, p + 2 * W);
}
template <class F>
PA_DEV void store_jac(uint64_t* p, const Jac<F>& a) {
    constexpr int W = FieldWords<F>::n;
    store(p, a.x);
    store(p + W, a.y);
    store(p + 2 * W, a.z);
}
// affine record: {x, y, u8 infinity, pad[7]} -> 2W+1 u64
template <class F>
PA_DEV void load_aff(Aff<F>& r, const uint64_t* p) {
    constexpr int W = FieldWords<F>::n;
    load8(r.x, p);
    load8(r.y, p + W);
    r.inf = (p[2 * W] & 0xff) != 0;
}
template <class F>
PA_DEV void store_aff(uint64_t* p, const Aff<F>& a) {
    constexpr int W = FieldWords<F>::n;
    store8(p, a.x);
    store8(p + W, a.y);
    p[2 * W] = a.inf ? 1ull : 0ull;
}

}  // namespace pa
