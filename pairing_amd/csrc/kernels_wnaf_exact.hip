// Bit-exact Wnaf (wnaf.rs:1-179) for G1 and G2: the reference's table chain,
// wNAF recoding and exponentiation, so the Jacobian X, Y, Z words equal the
// reference's -- not only the point (the comb of kernels_curve.hip /
// kernels_group.hip is equal as a point, PartialEq ec.rs:45-85).
//
// Fixed scalar (Wnaf::new().scalar(s).base(g), wnaf.rs:111-128, 156-166):
//   k_wx_scalar_digits  wnaf_form of the one scalar (1 lane)
//   k_wx_fixed_scalar   per lane: its base's window table (wnaf_table: the
//                       2^(w-1) entries B, B + 2B, ... by add_assign) and
//                       wnaf_exp over the shared digits
// Fixed base (Wnaf::new().base(g, n).scalar(s_i), wnaf.rs:93-107, 169-178):
//   the table T_k = T_(k-1) + D (D = B.double(), T_0 = B) is a serial chain in
//   the reference.  With add-2007-bl (ec.rs:356-444) on T_(k-1) and D:
//     H = U2 - U1 = Z1^2 Z_D^2 (x_D - x_(k-1)),  Z_k = 2 Z1 Z_D H
//       = c_k Z_(k-1)^3,  c_k = 2 Z_D^3 (x_D - x_(k-1))
//   (x = affine coordinates) and X_k = x_k Z_k^2, Y_k = y_k Z_k^3, since the
//   formula's outputs represent T_k = (2k+1) B and field values are canonical.
//   So the chain is rebuilt in parallel:
//     k_wx_prep     D (the reference's doubling), x_D, 2 Z_D^3         (1 lane)
//     k_wx_affine   affine (2k+1) B per lane (any addition chain)
//     k_wx_coef     C_0 = Z_B, C_k = c_k
//     k_wx_scan     log2(N) steps C_i <- C_i * C_(i-2^s)^(3^(2^s)): after
//                   the last step C_k = Z_k (a Hillis-Steele scan over the
//                   maps z -> c z^(3^e); exponents: wnaf_exact_consts.h)
//     k_wx_finish   T_k = (x_k Z_k^2, y_k Z_k^3, Z_k), T_0 = B's own words
//   The closed form needs the generic branch of every addition (T_(k-1) and
//   D nonzero, x_(k-1) != x_D).  A base for which some step is special (zero,
//   a point of small order: B outside G1) raises a flag in the workspace and
//   k_wx_serial replays the reference's chain on one lane instead; both
//   paths are stream-ordered, no host round trip.
//   k_wx_table_fl        the finished table converted once to the lazy
//                        28-bit core's limbs (fl.h: 14 x u32 per Fq, R = 2^392)
//   k_wx_fixed_base_mul_fl  per scalar: wnaf_form's nonzero digits into a
//                        packed digit-major column, then wnaf_exp on the lazy
//                        core (curve_fl.h / curve_fl2.h: dbl-2009-l and
//                        add-2007-bl with the reference's field-value
//                        sequence), the coordinates canonical at the store --
//                        the same Jacobian words as the 12-word kernel
//                        (k_wx_fixed_base_mul, PA_WX_MUL=word12 for A/B)
#include <cstring>

#include <hipcub/hipcub.hpp>

#include "curve.h"
#include "curve_fl2.h"
#include "dec_quad.h"
#include "launch.h"
#include "wnaf_exact_consts.h"

namespace pa {
namespace {

template <int G> struct Wx;
template <> struct Wx<1> {
    using F = Fq;
    static constexpr int W = 6;
};
template <> struct Wx<2> {
    using F = Fq2;
    static constexpr int W = 12;
};

inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// wnaf_form (wnaf.rs:18-43) of a 4 x u64 FrRepr for window <= kWxMaxWindow:
// digit j to d[j * stride]; returns the count.  sub_noborrow / add_nocarry
// wrap modulo 2^256 as the reference's do (wnaf.rs:30-35).
PA_DEV int wnaf_digits(const uint64_t* s, int window, int32_t* d, size_t stride) {
    uint64_t c0 = s[0], c1 = s[1], c2 = s[2], c3 = s[3];
    const uint64_t mod_mask = (1ull << (window + 1)) - 1;
    const int64_t half = (int64_t)1 << window;
    int len = 0;
    while ((c0 | c1 | c2 | c3) != 0) {
        int64_t u = 0;
        if (c0 & 1) {
            u = (int64_t)(c0 & mod_mask);
            if (u > half) u -= (int64_t)1 << (window + 1);
            if (u > 0) {
                const uint64_t t = (uint64_t)u;
                const uint64_t b0 = c0 < t;
                c0 -= t;
                const uint64_t b1 = c1 < b0;
                c1 -= b0;
                const uint64_t b2 = c2 < b1;
                c2 -= b1;
                c3 -= b2;
            } else {
                const uint64_t t = (uint64_t)(-u);
                c0 += t;
                const uint64_t k0 = c0 < t;
                c1 += k0;
                const uint64_t k1 = k0 && c1 == 0;
                c2 += k1;
                const uint64_t k2 = k1 && c2 == 0;
                c3 += k2;
            }
        }
        d[(size_t)len * stride] = (int32_t)u;
        len++;
        c0 = (c0 >> 1) | (c1 << 63);
        c1 = (c1 >> 1) | (c2 << 63);
        c2 = (c2 >> 1) | (c3 << 63);
        c3 >>= 1;
    }
    return len;
}

// wnaf_form as above, keeping only the nonzero digits, in increasing position
// order, each packed as (digit << 9) | position (positions < kWxMaxDigits <
// 512, |digit| < 2^20): at most wx_max_nonzero(window) entries at d[k stride]
PA_DEV int wnaf_nonzero(const uint64_t* s, int window, int32_t* d, size_t stride) {
    uint64_t c0 = s[0], c1 = s[1], c2 = s[2], c3 = s[3];
    const uint64_t mod_mask = (1ull << (window + 1)) - 1;
    const int64_t half = (int64_t)1 << window;
    int pos = 0, cnt = 0;
    while ((c0 | c1 | c2 | c3) != 0) {
        if (c0 & 1) {
            int64_t u = (int64_t)(c0 & mod_mask);
            if (u > half) u -= (int64_t)1 << (window + 1);
            if (u > 0) {
                const uint64_t t = (uint64_t)u;
                const uint64_t b0 = c0 < t;
                c0 -= t;
                const uint64_t b1 = c1 < b0;
                c1 -= b0;
                const uint64_t b2 = c2 < b1;
                c2 -= b1;
                c3 -= b2;
            } else {
                const uint64_t t = (uint64_t)(-u);
                c0 += t;
                const uint64_t k0 = c0 < t;
                c1 += k0;
                const uint64_t k1 = k0 && c1 == 0;
                c2 += k1;
                const uint64_t k2 = k1 && c2 == 0;
                c3 += k2;
            }
            d[(size_t)cnt * stride] = (int32_t)(((uint32_t)(int32_t)u << 9) | (uint32_t)pos);
            cnt++;
        }
        pos++;
        c0 = (c0 >> 1) | (c1 << 63);
        c1 = (c1 >> 1) | (c2 << 63);
        c2 = (c2 >> 1) | (c3 << 63);
        c3 >>= 1;
    }
    return cnt;
}

// wnaf_exp (wnaf.rs:45-71): entry e of the table at table + 3W estride e (u64),
// digit j at d[j dstride]
template <int G>
PA_DEV void wnaf_exp(Jac<typename Wx<G>::F>& r, const uint64_t* table, size_t estride, const int32_t* d,
                     size_t dstride, int len) {
    using F = typename Wx<G>::F;
    constexpr int JW = 3 * Wx<G>::W;
    jac_zero(r);
    bool found = false;
    for (int j = len - 1; j >= 0; j--) {
        if (found) jac_double(r);
        const int32_t v = d[(size_t)j * dstride];
        if (v != 0) {
            found = true;
            Jac<F> t;
            load_jac(t, table + (size_t)JW * estride * (size_t)((v > 0 ? v : -v) / 2));
            if (v > 0)
                jac_add(r, t);
            else
                jac_sub(r, t);
        }
    }
}

// ---------------- lazy-core helpers (G1: curve_fl.h, G2: curve_fl2.h) ----------------
// table entry layout of k_wx_table_fl: x, y, z as lazy limbs, padded to 16-byte
// pieces (G1: 42 -> 48 u32, G2: 84 -> 96 u32)
template <int G> struct WxL;
template <> struct WxL<1> {
    using J = FlJac;
    static constexpr int EW = 48;
};
template <> struct WxL<2> {
    using J = FlJac2;
    static constexpr int EW = 96;
};

PA_DEV void wl_put(uint32_t* e, const F<1>& a) {
#pragma unroll
    for (int i = 0; i < 14; i++) e[i] = a.w[i];
}
PA_DEV void wl_put(uint32_t* e, const F2<1>& a) {
    wl_put(e, a.c0);
    wl_put(e + 14, a.c1);
}
PA_DEV void wl_get(F<1>& a, const uint32_t* e) {
#pragma unroll
    for (int i = 0; i < 14; i++) a.w[i] = e[i];
}
PA_DEV void wl_get(F2<1>& a, const uint32_t* e) {
    wl_get(a.c0, e);
    wl_get(a.c1, e + 14);
}
PA_DEV void wl_load(F<1>& a, const uint64_t* p) { a = fl_load(p); }
PA_DEV void wl_load(F2<1>& a, const uint64_t* p) { a = fl2_load(p); }
PA_DEV bool wl_zero_test(const F<1>& a) { return fl_is_zero(a); }
PA_DEV bool wl_zero_test(const F2<1>& a) { return f2_is_zero(a); }
PA_DEV void wl_double(FlJac& p) { fl_jac_double(p); }
PA_DEV void wl_double(FlJac2& p) { fl2_jac_double(p); }
PA_DEV void wl_add(FlJac& s, const FlJac& o) { fl_jac_add(s, o); }
PA_DEV void wl_add(FlJac2& s, const FlJac2& o) { fl2_jac_add(s, o); }
PA_DEV void wl_store(uint64_t* p, const FlJac& a) { fl_store_jac(p, a); }
PA_DEV void wl_store(uint64_t* p, const FlJac2& a) { fl2_store_jac(p, a); }
PA_DEV void wl_set_zero(FlJac& r) { r = {fl_zero(), fl_one(), fl_zero()}; }   // ec.rs:224-230
PA_DEV void wl_set_zero(FlJac2& r) { r = fl2_jac_zero(); }

// ---------------- fixed scalar ----------------
__global__ void __launch_bounds__(64) k_wx_scalar_digits(const uint64_t* __restrict__ scalar, int window,
                                                         int32_t* __restrict__ digits, int32_t* __restrict__ len) {
    if (blockIdx.x == 0 && threadIdx.x == 0) len[0] = wnaf_digits(scalar, window, digits, 1);
}

// tables: entry e of lane i at tables[(e n + i) JW] (entry-major, so a wave's
// stores of one entry are adjacent records)
template <int G>
__global__ void __launch_bounds__(64) k_wx_fixed_scalar(const uint64_t* __restrict__ bases, size_t n,
                                                        const int32_t* __restrict__ digits,
                                                        const int32_t* __restrict__ len, int window,
                                                        uint64_t* __restrict__ tables, uint64_t* __restrict__ out) {
    using F = typename Wx<G>::F;
    constexpr int JW = 3 * Wx<G>::W;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // wnaf_table (wnaf.rs:3-15)
    Jac<F> base, dbl;
    load_jac(base, bases + (size_t)JW * i);
    dbl = base;
    jac_double(dbl);
    const size_t entries = (size_t)1 << (window - 1);
    uint64_t* t = tables + (size_t)JW * i;
    for (size_t e = 0; e < entries; e++) {
        store_jac(t + (size_t)JW * n * e, base);
        jac_add(base, dbl);
    }
    // wnaf_exp over this lane's entries (stride n) and the shared digits
    Jac<F> r;
    wnaf_exp<G>(r, t, n, digits, 1, len[0]);
    store_jac(out + (size_t)JW * i, r);
}

// ---------------- fixed base: the table ----------------
// Y^2 == X^3 + b Z^6 (b = 4, ec.rs:885-887; G2: 4 (u + 1), ec.rs:1557-1562)
PA_DEV void times_b(Fq& r, const Fq& a) {
    dbl(r, a);
    dbl(r, r);
}
PA_DEV void times_b(Fq2& r, const Fq2& a) {
    mul_by_nonresidue(r, a);
    dbl(r, r);
    dbl(r, r);
}
template <class F>
PA_DEV bool jac_on_curve(const Jac<F>& p) {
    F y2, x3, z6, t;
    sqr(y2, p.y);
    sqr(x3, p.x);
    mul(x3, x3, p.x);
    sqr(z6, p.z);
    sqr(t, z6);
    mul(z6, t, z6);
    times_b(t, z6);
    add(x3, x3, t);
    return eq(y2, x3);
}

// meta (u64): [0, 3W) D, [3W, 4W) x_D, [4W, 5W) 2 Z_D^3, [5W] special-step flag,
// [5W + 1] B is a nonzero point on the curve: E(Fq) and E'(Fq2) have odd order
// (cofactor times r), so no point of the chain has order 2 and a doubling of a
// nonzero point is nonzero -- the multiply then tests for zero only after adds
template <int G>
__global__ void __launch_bounds__(64) k_wx_prep(const uint64_t* __restrict__ base, uint64_t* __restrict__ meta) {
    using F = typename Wx<G>::F;
    constexpr int W = Wx<G>::W;
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    Jac<F> b, d;
    load_jac(b, base);
    d = b;
    jac_double(d);
    store_jac(meta, d);
    // the closed form recombines (2k + 1) B from another addition chain, which
    // gives the serial chain's values only where the group law holds: a base off
    // the curve takes the serial chain too
    const bool on_curve = !jac_is_zero(b) && jac_on_curve(b);
    uint64_t flag = jac_is_zero(b) || jac_is_zero(d) || !on_curve ? 1 : 0;
    if (!flag) {
        Aff<F> a;
        jac_to_affine(a, d);
        F z3, k2;
        sqr(z3, d.z);
        mul(z3, z3, d.z);
        dbl(k2, z3);
        store(meta + 3 * W, a.x);
        store(meta + 4 * W, k2);
    }
    meta[5 * W] = flag;
    meta[5 * W + 1] = on_curve ? 1 : 0;
}

// affine (2k + 1) B for k < N (a plain double-and-add: affine values do not
// depend on the chain)
template <int G>
__global__ void __launch_bounds__(64) k_wx_affine(const uint64_t* __restrict__ base, size_t N,
                                                  uint64_t* __restrict__ aff, uint64_t* __restrict__ meta) {
    using F = typename Wx<G>::F;
    constexpr int W = Wx<G>::W;
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    Jac<F> b, r;
    load_jac(b, base);
    const uint64_t m = 2 * (uint64_t)k + 1;
    r = b;
    for (int bit = 62 - __builtin_clzll(m); bit >= 0; bit--) {
        jac_double(r);
        if ((m >> bit) & 1) jac_add(r, b);
    }
    Aff<F> a;
    jac_to_affine(a, r);
    if (a.inf) meta[5 * W] = 1;
    store(aff + (size_t)2 * W * k, a.x);
    store(aff + (size_t)2 * W * k + W, a.y);
}

// the same affine multiples on the lazy core (curve_fl.h / curve_fl2.h), the
// inversion of z by the 12-word binary GCD (bgcd.h); the affine values do not
// depend on the chain, so any exact group law gives the same words
PA_DEV bool wl_inverse(F<1>& r, const F<1>& a) {
    Fq t;
    const bool ok = fq_inv(t, fl_to_abi(a));
    r = fl_from_abi(t);
    return ok;
}
PA_DEV bool wl_inverse(F2<1>& r, const F2<1>& a) {   // fq2.rs:138-155
    F<1> t;
    const bool ok = wl_inverse(t, sop(a.c0, a.c0, a.c1, a.c1));
    r = {mul(a.c0, t), mul(red(neg(a.c1)), t)};
    return ok;
}
PA_DEV void wl_store1(uint64_t* p, const F<1>& a) { fl_store(p, a); }
PA_DEV void wl_store1(uint64_t* p, const F2<1>& a) { fl2_store(p, a); }
PA_DEV FlJac wl_load_jac(const uint64_t* p, FlJac*) { return fl_load_jac(p); }
PA_DEV FlJac2 wl_load_jac(const uint64_t* p, FlJac2*) { return fl2_load_jac(p); }

template <int G>
__global__ void __launch_bounds__(64) k_wx_affine_fl(const uint64_t* __restrict__ base, size_t N,
                                                     uint64_t* __restrict__ aff, uint64_t* __restrict__ meta) {
    constexpr int W = Wx<G>::W;
    using J = typename WxL<G>::J;
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N || meta[5 * W]) return;   // a zero B or D: the serial chain runs instead
    const J b = wl_load_jac(base, (J*)nullptr);
    J r = b;
    const uint64_t m = 2 * (uint64_t)k + 1;
    for (int bit = 62 - __builtin_clzll(m); bit >= 0; bit--) {
        if (!wl_zero_test(r.z)) wl_double(r);
        if ((m >> bit) & 1) wl_add(r, b);
    }
    decltype(r.z) zi;
    if (!wl_inverse(zi, r.z)) {   // (2k + 1) B = 0: B has small order
        meta[5 * W] = 1;
        return;
    }
    const auto zi2 = sqr(zi);
    wl_store1(aff + (size_t)2 * W * k, mul(r.x, zi2));
    wl_store1(aff + (size_t)2 * W * k + W, mul(r.y, mul(zi2, zi)));
}

template <int G>
__global__ void __launch_bounds__(64) k_wx_coef(const uint64_t* __restrict__ base, const uint64_t* __restrict__ aff,
                                                size_t N, uint64_t* __restrict__ coef, uint64_t* __restrict__ meta) {
    using F = typename Wx<G>::F;
    constexpr int W = Wx<G>::W;
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N || meta[5 * W]) return;
    F c;
    if (k == 0) {
        load(c, base + 2 * W);   // Z_B
    } else {
        F xp, xd, k2;
        load(xp, aff + (size_t)2 * W * (k - 1));
        load(xd, meta + 3 * W);
        load(k2, meta + 4 * W);
        if (eq(xp, xd)) meta[5 * W] = 1;   // T_(k-1) = +-D: add_assign's special branch
        sub(c, xd, xp);
        mul(c, c, k2);
    }
    store(coef + (size_t)W * k, c);
}

// z^(3^(2^s)) with the reduced exponents of wnaf_exact_consts.h
PA_DEV int top_bit(const uint64_t* e) {
    for (int w = 5; w >= 0; w--)
        if (e[w]) return 64 * w + 63 - __builtin_clzll(e[w]);
    return -1;
}
PA_DEV void pow3(Fq& r, const Fq& z, int s) {
    const uint64_t* e = PA_WX_E1[s];
    one(r);
    for (int b = top_bit(e); b >= 0; b--) {
        sqr(r, r);
        if ((e[b >> 6] >> (b & 63)) & 1) mul(r, r, z);
    }
}
PA_DEV void pow3(Fq2& r, const Fq2& z, int s) {
    // z^(e0 + e1 q) = z^e0 conj(z)^e1 (q = 3 mod 4: z^q = conj(z)), one run of squarings
    const uint64_t* e0 = PA_WX_E2[s][0];
    const uint64_t* e1 = PA_WX_E2[s][1];
    Fq2 zc, zz;
    zc.c0 = z.c0;
    neg(zc.c1, z.c1);
    mul(zz, z, zc);
    one(r);
    const int t0 = top_bit(e0), t1 = top_bit(e1);
    for (int b = t0 > t1 ? t0 : t1; b >= 0; b--) {
        sqr(r, r);
        const bool x0 = (e0[b >> 6] >> (b & 63)) & 1, x1 = (e1[b >> 6] >> (b & 63)) & 1;
        if (x0 && x1)
            mul(r, r, zz);
        else if (x0)
            mul(r, r, z);
        else if (x1)
            mul(r, r, zc);
    }
}

template <int G>
__global__ void __launch_bounds__(64) k_wx_scan(const uint64_t* __restrict__ cin, uint64_t* __restrict__ cout,
                                                size_t N, size_t off, int s, const uint64_t* __restrict__ meta) {
    using F = typename Wx<G>::F;
    constexpr int W = Wx<G>::W;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || meta[5 * W]) return;
    F v;
    load(v, cin + (size_t)W * i);
    if (i >= off) {
        F p, t;
        load(p, cin + (size_t)W * (i - off));
        pow3(t, p, s);
        mul(v, v, t);
    }
    store(cout + (size_t)W * i, v);
}

// The scan step on the lazy core.  G1: one element per lane QUAD, its
// exponentiation spread over the quad (dec_quad.h: a dependent product is ~0.6
// us instead of ~1.6 us on the 12-word core), a 4-bit sliding window over the
// same exponent, so the same field value v * p^(3^(2^s)).
__global__ void __launch_bounds__(256) k_wx_scan_q1(const uint64_t* __restrict__ cin, uint64_t* __restrict__ cout,
                                                    size_t N, size_t off, int s, const uint64_t* __restrict__ meta) {
    const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    if (i >= N || meta[5 * 6]) return;   // whole quads leave together
    const int lane = threadIdx.x & 63;
    Fq v;
    load(v, cin + 6 * i);
    if (i >= off) {
        const dq::Lc l = dq::lctx(lane, 1);
        Fq p;
        load(p, cin + 6 * (i - off));
        const uint64_t* e = PA_WX_E1[s];
        const dq::Q<1> t = dq::pow_fixed(dq::from_abi(p, l), e, top_bit(e), l);
        v = dq::to_abi(dq::mul(dq::from_abi(v, l), t, l));
    }
    if ((lane & 3) == 0) store(cout + 6 * i, v);
}

// Two scan steps s, s + 1 in one launch (radix 4), for the steps whose
// exponents are reduced modulo q - 1 (full size): with a = 2^s,
//   C_i <- C_i C_(i-a)^(E_s) C_(i-2a)^(E_(s+1)) C_(i-3a)^(E_s E_(s+1))
// (a term whose index is negative is absent), the same value the two
// Hillis-Steele steps give; the three powers share one run of squarings
// (Straus, a 4-bit sliding window per exponent): ~630 products against ~930.
PA_DEV int ebit(const uint64_t* e, int b) { return (int)((e[b >> 6] >> (b & 63)) & 1); }
PA_DEV dq::Q<1> pick8(const dq::Q<1> (&t)[8], int k) {
    switch (k) {
        case 0: return t[0];
        case 1: return t[1];
        case 2: return t[2];
        case 3: return t[3];
        case 4: return t[4];
        case 5: return t[5];
        case 6: return t[6];
        default: return t[7];
    }
}
PA_DEV void odd_powers(dq::Q<1> (&t)[8], const dq::Q<1>& x, const dq::Lc& l) {
    t[0] = x;
    const dq::Q<1> x2 = dq::sqr(x, l);
#pragma unroll
    for (int k = 1; k < 8; k++) t[k] = dq::mul(t[k - 1], x2, l);
}
// a 4-bit window of e opens at bit b (e's bit b set): its low end and value
PA_DEV void open_window(const uint64_t* e, int b, int& lo, int& v) {
    int L = b - 3 < 0 ? 0 : b - 3;
    while (!ebit(e, L)) L++;
    int val = 0;
    for (int c = b; c >= L; c--) val = 2 * val + ebit(e, c);
    lo = L;
    v = val;
}
PA_DEV dq::Q<1> pow_multi3(const dq::Q<1>& x0, const dq::Q<1>& x1, const dq::Q<1>& x2, const uint64_t* e0,
                           const uint64_t* e1, const uint64_t* e2, const dq::Lc& l) {
    dq::Q<1> t0[8], t1[8], t2[8];
    odd_powers(t0, x0, l);
    odd_powers(t1, x1, l);
    odd_powers(t2, x2, l);
    int top = top_bit(e0);
    top = top_bit(e1) > top ? top_bit(e1) : top;
    top = top_bit(e2) > top ? top_bit(e2) : top;
    int lo0 = -1, lo1 = -1, lo2 = -1, v0 = 0, v1 = 0, v2 = 0;
    bool started = false;
    dq::Q<1> acc = x0;
    auto close = [&](const dq::Q<1> (&t)[8], int v) {
        const dq::Q<1> f = pick8(t, v >> 1);
        acc = started ? dq::mul(acc, f, l) : f;
        started = true;
    };
#pragma unroll 1
    for (int b = top; b >= 0; b--) {
        if (lo0 < 0 && ebit(e0, b)) open_window(e0, b, lo0, v0);
        if (lo1 < 0 && ebit(e1, b)) open_window(e1, b, lo1, v1);
        if (lo2 < 0 && ebit(e2, b)) open_window(e2, b, lo2, v2);
        if (started) acc = dq::sqr(acc, l);
        if (lo0 == b) {
            close(t0, v0);
            lo0 = -1;
        }
        if (lo1 == b) {
            close(t1, v1);
            lo1 = -1;
        }
        if (lo2 == b) {
            close(t2, v2);
            lo2 = -1;
        }
    }
    return acc;
}

__global__ void __launch_bounds__(256) k_wx_scan4_q1(const uint64_t* __restrict__ cin, uint64_t* __restrict__ cout,
                                                     size_t N, size_t a, int s, const uint64_t* __restrict__ meta) {
    const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    if (i >= N || meta[5 * 6]) return;   // whole quads leave together
    const int lane = threadIdx.x & 63;
    Fq v;
    load(v, cin + 6 * i);
    if (i >= a) {
        const dq::Lc l = dq::lctx(lane, 1);
        const dq::Q<1> one = dq::qconst(FL_ONE, l);
        Fq p;
        load(p, cin + 6 * (i - a));
        const dq::Q<1> x0 = dq::from_abi(p, l);
        dq::Q<1> x1 = one, x2 = one;
        if (i >= 2 * a) {
            load(p, cin + 6 * (i - 2 * a));
            x1 = dq::from_abi(p, l);
        }
        if (i >= 3 * a) {
            load(p, cin + 6 * (i - 3 * a));
            x2 = dq::from_abi(p, l);
        }
        const dq::Q<1> t = pow_multi3(x0, x1, x2, PA_WX_E1[s], PA_WX_E1[s + 1], PA_WX_E1T[s], l);
        v = dq::to_abi(dq::mul(dq::from_abi(v, l), t, l));
    }
    if ((lane & 3) == 0) store(cout + 6 * i, v);
}

// The radix-4 step one element per LANE on the lazy core's one-lane leaves:
// 512 waves for 2^15 entries leave half the SIMDs idle and a lone wave's
// product is ~1.1 us, but a quad product costs 2.5x the issue slots and the
// quad form of these steps is issue-bound at two waves per SIMD
// (PA_WX_SCAN4=quad selects it for A/B)
PA_DEV F<1> pick8(const F<1> (&t)[8], int k) {
    switch (k) {
        case 0: return t[0];
        case 1: return t[1];
        case 2: return t[2];
        case 3: return t[3];
        case 4: return t[4];
        case 5: return t[5];
        case 6: return t[6];
        default: return t[7];
    }
}
PA_DEV void odd_powers(F<1> (&t)[8], const F<1>& x) {
    t[0] = x;
    const F<1> x2 = sqr(x);
#pragma unroll
    for (int k = 1; k < 8; k++) t[k] = mul(t[k - 1], x2);
}
PA_DEV F<1> pow_multi3(const F<1>& x0, const F<1>& x1, const F<1>& x2, const uint64_t* e0, const uint64_t* e1,
                       const uint64_t* e2) {
    F<1> t0[8], t1[8], t2[8];
    odd_powers(t0, x0);
    odd_powers(t1, x1);
    odd_powers(t2, x2);
    int top = top_bit(e0);
    top = top_bit(e1) > top ? top_bit(e1) : top;
    top = top_bit(e2) > top ? top_bit(e2) : top;
    int lo0 = -1, lo1 = -1, lo2 = -1, v0 = 0, v1 = 0, v2 = 0;
    bool started = false;
    F<1> acc = x0;
    auto close = [&](const F<1> (&t)[8], int v) {
        const F<1> f = pick8(t, v >> 1);
        acc = started ? mul(acc, f) : f;
        started = true;
    };
#pragma unroll 1
    for (int b = top; b >= 0; b--) {
        if (lo0 < 0 && ebit(e0, b)) open_window(e0, b, lo0, v0);
        if (lo1 < 0 && ebit(e1, b)) open_window(e1, b, lo1, v1);
        if (lo2 < 0 && ebit(e2, b)) open_window(e2, b, lo2, v2);
        if (started) acc = sqr(acc);
        if (lo0 == b) {
            close(t0, v0);
            lo0 = -1;
        }
        if (lo1 == b) {
            close(t1, v1);
            lo1 = -1;
        }
        if (lo2 == b) {
            close(t2, v2);
            lo2 = -1;
        }
    }
    return acc;
}
__global__ void __launch_bounds__(64) k_wx_scan4_fl1(const uint64_t* __restrict__ cin, uint64_t* __restrict__ cout,
                                                     size_t N, size_t a, int s, const uint64_t* __restrict__ meta) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || meta[5 * 6]) return;
    if (i < a) {
        for (int j = 0; j < 6; j++) cout[6 * i + j] = cin[6 * i + j];
        return;
    }
    const F<1> x0 = fl_load(cin + 6 * (i - a));
    const F<1> x1 = i >= 2 * a ? fl_load(cin + 6 * (i - 2 * a)) : fl_one();
    const F<1> x2 = i >= 3 * a ? fl_load(cin + 6 * (i - 3 * a)) : fl_one();
    const F<1> t = pow_multi3(x0, x1, x2, PA_WX_E1[s], PA_WX_E1[s + 1], PA_WX_E1T[s]);
    fl_store(cout + 6 * i, mul(fl_load(cin + 6 * i), t));
}

// G2: one element per lane on the lazy core's Fq2 (tower_fl.h), z^(e0 + e1 q)
// = z^e0 conj(z)^e1 over one run of squarings, as pow3 above
__global__ void __launch_bounds__(64) k_wx_scan_fl2(const uint64_t* __restrict__ cin, uint64_t* __restrict__ cout,
                                                    size_t N, size_t off, int s, const uint64_t* __restrict__ meta) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N || meta[5 * 12]) return;
    if (i < off) {
        for (int j = 0; j < 12; j++) cout[12 * i + j] = cin[12 * i + j];
        return;
    }
    const F2<1> z = fl2_load(cin + 12 * (i - off));
    const F2<1> zc = red(conj(z));
    const F2<1> zz = mul(z, zc);
    const uint64_t* e0 = PA_WX_E2[s][0];
    const uint64_t* e1 = PA_WX_E2[s][1];
    const int t0 = top_bit(e0), t1 = top_bit(e1);
    F2<1> r = f2_one();
    bool started = false;
    for (int b = t0 > t1 ? t0 : t1; b >= 0; b--) {
        if (started) r = sqr(r);
        const bool x0 = (e0[b >> 6] >> (b & 63)) & 1, x1 = (e1[b >> 6] >> (b & 63)) & 1;
        if (x0 || x1) {
            const F2<1>& f = x0 && x1 ? zz : (x0 ? z : zc);
            r = started ? mul(r, f) : f;
            started = true;
        }
    }
    fl2_store(cout + 12 * i, mul(fl2_load(cin + 12 * i), r));
}

template <int G>
__global__ void __launch_bounds__(64) k_wx_finish(const uint64_t* __restrict__ base, const uint64_t* __restrict__ aff,
                                                  const uint64_t* __restrict__ zs, size_t N,
                                                  uint64_t* __restrict__ table, const uint64_t* __restrict__ meta) {
    using F = typename Wx<G>::F;
    constexpr int W = Wx<G>::W;
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N || meta[5 * W]) return;
    uint64_t* t = table + (size_t)3 * W * k;
    if (k == 0) {
        for (int j = 0; j < 3 * W; j++) t[j] = base[j];   // T_0 = B, its own words
        return;
    }
    F z, x, y, z2;
    load(z, zs + (size_t)W * k);
    load(x, aff + (size_t)2 * W * k);
    load(y, aff + (size_t)2 * W * k + W);
    sqr(z2, z);
    mul(x, x, z2);
    mul(z2, z2, z);
    mul(y, y, z2);
    store(t, x);
    store(t + W, y);
    store(t + 2 * W, z);
}

// the reference's chain itself, for bases whose chain takes a special branch
template <int G>
__global__ void __launch_bounds__(64) k_wx_serial(const uint64_t* __restrict__ base, size_t N,
                                                  uint64_t* __restrict__ table, const uint64_t* __restrict__ meta) {
    using F = typename Wx<G>::F;
    constexpr int W = Wx<G>::W;
    if (blockIdx.x != 0 || threadIdx.x != 0 || !meta[5 * W]) return;
    Jac<F> b, d;
    load_jac(b, base);
    d = b;
    jac_double(d);
    for (size_t k = 0; k < N; k++) {
        store_jac(table + (size_t)3 * W * k, b);
        jac_add(b, d);
    }
}

// ---------------- fixed base: the multiply ----------------
template <int G>
__global__ void __launch_bounds__(64) k_wx_fixed_base_mul(const uint64_t* __restrict__ table,
                                                          const uint64_t* __restrict__ scalars, size_t n, int window,
                                                          int32_t* __restrict__ digits, uint64_t* __restrict__ out) {
    using F = typename Wx<G>::F;
    constexpr int JW = 3 * Wx<G>::W;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int len = wnaf_digits(scalars + 4 * i, window, digits + i, n);
    Jac<F> r;
    wnaf_exp<G>(r, table, 1, digits + i, n, len);
    store_jac(out + (size_t)JW * i, r);
}


// ---------------- fixed base: the multiply on the lazy core ----------------
template <int G>
__global__ void __launch_bounds__(64) k_wx_table_fl(const uint64_t* __restrict__ table, size_t N,
                                                    uint32_t* __restrict__ tfl) {
    constexpr int W = Wx<G>::W, EW = WxL<G>::EW, L = 14 * (W / 6);
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    typename WxL<G>::J t;
    wl_load(t.x, table + (size_t)3 * W * k);
    wl_load(t.y, table + (size_t)3 * W * k + W);
    wl_load(t.z, table + (size_t)3 * W * k + 2 * W);
    uint32_t e[EW];
    wl_put(e, t.x);
    wl_put(e + L, t.y);
    wl_put(e + 2 * L, t.z);
#pragma unroll
    for (int j = 3 * L; j < EW; j++) e[j] = 0;
    uint4* dst = reinterpret_cast<uint4*>(tfl + (size_t)EW * k);
#pragma unroll
    for (int j = 0; j < EW / 4; j++) dst[j] = make_uint4(e[4 * j], e[4 * j + 1], e[4 * j + 2], e[4 * j + 3]);
}

template <int G>
PA_DEV typename WxL<G>::J wl_entry(const uint32_t* __restrict__ tfl, int e) {
    constexpr int EW = WxL<G>::EW, L = 14 * G;
    const uint4* src = reinterpret_cast<const uint4*>(tfl + (size_t)EW * e);
    uint32_t v[EW];
#pragma unroll
    for (int j = 0; j < EW / 4; j++) {
        const uint4 x = src[j];
        v[4 * j] = x.x;
        v[4 * j + 1] = x.y;
        v[4 * j + 2] = x.z;
        v[4 * j + 3] = x.w;
    }
    typename WxL<G>::J t;
    wl_get(t.x, v);
    wl_get(t.y, v + L);
    wl_get(t.z, v + 2 * L);
    return t;
}

// wnaf_exp (wnaf.rs:45-71) over the packed nonzero digits: the reference's
// loop doubles once per digit position below the first nonzero one and adds
// (or subtracts, sub_assign = add of the negation, ec.rs:528-532) the entry of
// each nonzero digit.  double() and negate() leave a zero point's words as they
// are (ec.rs:298-300, 556-560): tested on z, as is_zero does.
// G1: at most 256 registers (VGPR + AGPR), so two waves share a SIMD
template <int G>
__global__ void __launch_bounds__(64, G == 1 ? 2 : 1) k_wx_fixed_base_mul_fl(const uint32_t* __restrict__ tfl,
                                                             const uint64_t* __restrict__ scalars, size_t n,
                                                             int window, int32_t* __restrict__ digits,
                                                             const uint64_t* __restrict__ meta,
                                                             const uint32_t* __restrict__ perm,
                                                             const int32_t* __restrict__ cnts,
                                                             uint64_t* __restrict__ out) {
    constexpr int W = Wx<G>::W, JW = 3 * W;
    using J = typename WxL<G>::J;
    const size_t t_ = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t_ >= n) return;
    const bool on_curve = meta[5 * W + 1] != 0;
    // perm: the scalar this lane takes (k_wx_digit_keys + sort: its digits are
    // in place already); none: the lane's own scalar, digits formed here
    const size_t i = perm ? perm[t_] : t_;
    int32_t* d = digits + i;
    const int cnt = perm ? cnts[i] : wnaf_nonzero(scalars + 4 * i, window, d, n);
    J r;
    wl_set_zero(r);
    bool rz = true;   // r is zero (z == 0)
    auto doublings = [&](int m) {
        if (on_curve) {
            if (!rz)
                for (int j = m; j > 0; j--) wl_double(r);
        } else {
            for (int j = m; j > 0; j--)
                if (!wl_zero_test(r.z)) wl_double(r);
        }
    };
    int prev = -1;
    for (int k = cnt - 1; k >= 0; k--) {
        const int32_t pk = d[(size_t)k * n];
        const int pos = pk & 511, v = pk >> 9;
        if (prev >= 0) doublings(prev - pos);
        J t = wl_entry<G>(tfl, (v > 0 ? v : -v) >> 1);
        if (v < 0 && !wl_zero_test(t.z)) t.y = red(neg(t.y));
        wl_add(r, t);
        rz = wl_zero_test(r.z);
        prev = pos;
    }
    if (prev > 0) doublings(prev);
    wl_store(out + (size_t)JW * i, r);
}

// Lanes of a wave run the wnaf_exp rounds of their scalars in lockstep: each
// round costs the wave its longest gap of doublings, ~30 % more doublings than
// a lane needs for random scalars.  Scalars whose nonzero digits sit at similar
// positions waste less, so the multiply takes them in the order of a key --
// the nonzero-digit count, then the positions of the six highest nonzero
// digits -- sorted by a radix sort (the words of each result are unchanged:
// out[i] is still scalar i's).  Simulated on random scalars: 353 -> 327
// doubling-equivalents per lane.
__global__ void __launch_bounds__(64) k_wx_digit_keys(const uint64_t* __restrict__ scalars, size_t n, int window,
                                                      int32_t* __restrict__ digits, int32_t* __restrict__ cnts,
                                                      uint64_t* __restrict__ keys, uint32_t* __restrict__ idx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t* d = digits + i;
    const int cnt = wnaf_nonzero(scalars + 4 * i, window, d, n);
    uint64_t key = (uint64_t)cnt << 54;
    for (int k = 0; k < 6 && k < cnt; k++) key |= (uint64_t)(d[(size_t)(cnt - 1 - k) * n] & 511) << (45 - 9 * k);
    cnts[i] = cnt;
    keys[i] = key;
    idx[i] = (uint32_t)i;
}

// PA_WX_SORT=0: the scalars in their own order (A/B)
bool wx_sort() {
    static const bool v = !(getenv("PA_WX_SORT") && atoi(getenv("PA_WX_SORT")) == 0);
    return v;
}

// PA_WX_MUL=word12: the round-5 multiply on the 12-word core (A/B); its
// dense digit column needs the larger workspace (wx_layout)
bool wx_mul_word12() {
    static const bool v = getenv("PA_WX_MUL") && strcmp(getenv("PA_WX_MUL"), "word12") == 0;
    return v;
}

bool wx_scan4_quad() {
    static const bool v = getenv("PA_WX_SCAN4") && strcmp(getenv("PA_WX_SCAN4"), "quad") == 0;
    return v;
}
// PA_WX_RADIX4=0: radix-2 steps only (A/B)
bool wx_radix4() {
    static const bool v = !(getenv("PA_WX_RADIX4") && atoi(getenv("PA_WX_RADIX4")) == 0);
    return v;
}

template <int G>
hipError_t wx_fixed_base(const uint64_t* base, const uint64_t* scalars, uint64_t* out, size_t n, int window,
                         void* workspace, hipStream_t stream) {
    constexpr int W = Wx<G>::W;
    const size_t N = (size_t)1 << (window - 1);
    WxLayout L = wx_layout(G, n, window);
    char* ws = static_cast<char*>(workspace);
    uint64_t* meta = reinterpret_cast<uint64_t*>(ws + L.meta);
    uint64_t* table = reinterpret_cast<uint64_t*>(ws + L.table);
    uint64_t* aff = reinterpret_cast<uint64_t*>(ws + L.aff);
    uint64_t* c0 = reinterpret_cast<uint64_t*>(ws + L.c0);
    uint64_t* c1 = reinterpret_cast<uint64_t*>(ws + L.c1);
    int32_t* digits = reinterpret_cast<int32_t*>(ws + L.digits);
    const unsigned gb = blocks_for(N, 64);
    hipLaunchKernelGGL(k_wx_prep<G>, dim3(1), dim3(64), 0, stream, base, meta);
    if (wx_mul_word12())
        hipLaunchKernelGGL(k_wx_affine<G>, dim3(gb), dim3(64), 0, stream, base, N, aff, meta);
    else
        hipLaunchKernelGGL(k_wx_affine_fl<G>, dim3(gb), dim3(64), 0, stream, base, N, aff, meta);
    hipLaunchKernelGGL(k_wx_coef<G>, dim3(gb), dim3(64), 0, stream, base, aff, N, c0, meta);
    int s = 0;
    for (size_t off = 1; off < N; off <<= 1, s++) {
        if constexpr (G == 1) {
            // radix 4 where both steps' exponents are full size (3^(2^s) > q)
            if (!wx_mul_word12() && wx_radix4() && s >= 8 && 2 * off < N) {
                if (wx_scan4_quad())
                    hipLaunchKernelGGL(k_wx_scan4_q1, dim3(blocks_for(4 * N, 256)), dim3(256), 0, stream, c0, c1, N,
                                       off, s, meta);
                else
                    hipLaunchKernelGGL(k_wx_scan4_fl1, dim3(gb), dim3(64), 0, stream, c0, c1, N, off, s, meta);
                uint64_t* t = c0;
                c0 = c1;
                c1 = t;
                off <<= 1;
                s++;
                continue;
            }
        }
        if (wx_mul_word12())
            hipLaunchKernelGGL(k_wx_scan<G>, dim3(gb), dim3(64), 0, stream, c0, c1, N, off, s, meta);
        else if constexpr (G == 1)
            hipLaunchKernelGGL(k_wx_scan_q1, dim3(blocks_for(4 * N, 256)), dim3(256), 0, stream, c0, c1, N, off, s,
                               meta);
        else
            hipLaunchKernelGGL(k_wx_scan_fl2, dim3(gb), dim3(64), 0, stream, c0, c1, N, off, s, meta);
        uint64_t* t = c0;
        c0 = c1;
        c1 = t;
    }
    hipLaunchKernelGGL(k_wx_finish<G>, dim3(gb), dim3(64), 0, stream, base, aff, c0, N, table, meta);
    hipLaunchKernelGGL(k_wx_serial<G>, dim3(1), dim3(64), 0, stream, base, N, table, meta);
    if (n == 0) return hipGetLastError();
    if (wx_mul_word12()) {
        hipLaunchKernelGGL(k_wx_fixed_base_mul<G>, dim3(blocks_for(n, 64)), dim3(64), 0, stream, table, scalars, n,
                           window, digits, out);
    } else {
        uint32_t* tfl = reinterpret_cast<uint32_t*>(ws + L.tfl);
        hipLaunchKernelGGL(k_wx_table_fl<G>, dim3(gb), dim3(64), 0, stream, table, N, tfl);
        const uint32_t* perm = nullptr;
        int32_t* cnts = nullptr;
        if (wx_sort() && n <= 0x7fffffff) {
            uint64_t* keys = reinterpret_cast<uint64_t*>(ws + L.keys);
            uint32_t* idx = reinterpret_cast<uint32_t*>(ws + L.perm);
            cnts = reinterpret_cast<int32_t*>(ws + L.cnts);
            hipLaunchKernelGGL(k_wx_digit_keys, dim3(blocks_for(n, 64)), dim3(64), 0, stream, scalars, n, window,
                               digits, cnts, keys, idx);
            size_t tmp_bytes = L.sort_tmp_bytes;
            hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws + L.sort_tmp, tmp_bytes, keys, keys + n, idx,
                                                              idx + n, (int)n, 0, 64, stream);
            if (e != hipSuccess) return e;
            perm = idx + n;
        }
        hipLaunchKernelGGL(k_wx_fixed_base_mul_fl<G>, dim3(blocks_for(n, 64)), dim3(64), 0, stream, tfl, scalars, n,
                           window, digits, meta, perm, cnts, out);
    }
    (void)W;
    return hipGetLastError();
}

template <int G>
hipError_t wx_fixed_scalar(const uint64_t* bases, size_t n, const uint64_t* scalar, uint64_t* out, int window,
                           void* workspace, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    WxLayout L = wx_scalar_layout(G, n, window);
    char* ws = static_cast<char*>(workspace);
    int32_t* digits = reinterpret_cast<int32_t*>(ws + L.digits);
    int32_t* len = reinterpret_cast<int32_t*>(ws + L.meta);
    uint64_t* tables = reinterpret_cast<uint64_t*>(ws + L.table);
    hipLaunchKernelGGL(k_wx_scalar_digits, dim3(1), dim3(64), 0, stream, scalar, window, digits, len);
    hipLaunchKernelGGL(k_wx_fixed_scalar<G>, dim3(blocks_for(n, 64)), dim3(64), 0, stream, bases, n, digits, len,
                       window, tables, out);
    return hipGetLastError();
}

}  // namespace

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// workspace of the fixed-base path: meta, table, affine multiples, two scan
// buffers, the digit columns of the n scalars
WxLayout wx_layout(int group, size_t n, int window) {
    const size_t W = group == 1 ? 6 : 12, N = (size_t)1 << (window - 1);
    WxLayout L;
    size_t at = 0;
    L.meta = at;
    at = align256(at + 8 * (5 * W + 2));
    L.table = at;
    at = align256(at + 8 * 3 * W * N);
    L.aff = at;
    at = align256(at + 8 * 2 * W * N);
    L.c0 = at;
    at = align256(at + 8 * W * N);
    L.c1 = at;
    at = align256(at + 8 * W * N);
    L.digits = at;
    at = align256(at + 4 * (size_t)(wx_mul_word12() ? kWxMaxDigits : wx_max_nonzero(window)) * n);
    L.tfl = at;
    at = align256(at + (wx_mul_word12() ? 0 : 4 * (size_t)(group == 1 ? WxL<1>::EW : WxL<2>::EW) * N));
    // the scalar order of the multiply: keys and indices in and out of the sort
    L.keys = at;
    at = align256(at + 2 * 8 * n);
    L.perm = at;
    at = align256(at + 2 * 4 * n);
    L.cnts = at;
    at = align256(at + 4 * n);
    L.sort_tmp = at;
    L.sort_tmp_bytes = 0;
    if (n && n <= 0x7fffffff)
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, L.sort_tmp_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                 (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 64);
    at = align256(at + L.sort_tmp_bytes);
    L.bytes = at;
    return L;
}
// fixed scalar: digit count, the digits, a table of 2^(w-1) entries per base
WxLayout wx_scalar_layout(int group, size_t n, int window) {
    const size_t W = group == 1 ? 6 : 12, N = (size_t)1 << (window - 1);
    WxLayout L{};
    size_t at = 0;
    L.meta = at;
    at = align256(at + 8);
    L.digits = at;
    at = align256(at + 4 * (size_t)kWxMaxDigits);
    L.table = at;
    at = align256(at + 8 * 3 * W * N * n);
    L.bytes = at;
    return L;
}

hipError_t launch_wnaf_exact_fixed_base(int group, const uint64_t* base, const uint64_t* scalars, uint64_t* out,
                                        size_t n, int window, void* workspace, hipStream_t stream) {
    return group == 1 ? wx_fixed_base<1>(base, scalars, out, n, window, workspace, stream)
                      : wx_fixed_base<2>(base, scalars, out, n, window, workspace, stream);
}
hipError_t launch_wnaf_exact_fixed_scalar(int group, const uint64_t* bases, size_t n, const uint64_t* scalar,
                                          uint64_t* out, int window, void* workspace, hipStream_t stream) {
    return group == 1 ? wx_fixed_scalar<1>(bases, n, scalar, out, window, workspace, stream)
                      : wx_fixed_scalar<2>(bases, n, scalar, out, window, workspace, stream);
}

}  // namespace pa
