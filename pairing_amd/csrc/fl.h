// Lazy base-field arithmetic for gfx950: F<U>, 14 x 28-bit limbs, R = 2^392.
//
// The ABI and the reference hold canonical Montgomery values with R = 2^384
// (fq.rs:22-30, 6 x u64).  Inside the pairing kernels a value is
// sum w[i] 2^(28 i) with a compile-time bound U:
//
//     every limb <= U (2^28 - 1)   and   value < U * 2q          (U <= 16)
//
//   * products (leaf subroutines of fl_gen.h) return F<1>; they require
//     sum(U_x * U_y) <= 17 over their terms (one 64-bit column accumulator)
//     -- enforced by static_assert, so a formula that would overflow does not
//     compile;
//   * add: limb-wise, no carries, F<A+B>;
//   * sub: a + C_B - b where C_B = k q has limbs >= any limb of a value of
//     bound B (FL_SUB_C), F<A + FL_SUB_CU[B-1]>;
//   * red: one pass that subtracts floor(V/q) (or one less) times q, F<1>.
// fl_from_abi / fl_to_abi convert at the kernel boundary (one product each);
// stores are canonical, so outputs stay bit-identical to the reference's Fq.
#pragma once
#include "fq.h"
#include "fl_gen.h"

namespace pa {

template <int U>
struct F {
    static_assert(U >= 1 && U <= 16, "lazy bound out of range");
    uint32_t w[14];
};

constexpr int subcu(int b) { return FL_SUB_CU[b - 1]; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

// ---- additive ops ----
template <int A, int B>
PA_DEV F<A + B> add(const F<A>& a, const F<B>& b) {
    F<A + B> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = a.w[i] + b.w[i];
    return r;
}
template <int A>
PA_DEV F<2 * A> dbl(const F<A>& a) { return add(a, a); }

template <int A, int B>
PA_DEV F<A + subcu(B)> sub(const F<A>& a, const F<B>& b) {
    static_assert(B <= 14, "subtrahend bound beyond FL_SUB_C");
    F<A + subcu(B)> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = a.w[i] + FL_SUB_C[B - 1][i] - b.w[i];
    return r;
}
template <int B>
PA_DEV F<subcu(B)> neg(const F<B>& b) {
    static_assert(B <= 14, "subtrahend bound beyond FL_SUB_C");
    F<subcu(B)> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = FL_SUB_C[B - 1][i] - b.w[i];
    return r;
}
// widen the static bound (same bits)
template <int U2, int U1>
PA_DEV F<U2> relax(const F<U1>& a) {
    static_assert(U2 >= U1, "relax can only widen a bound");
    F<U2> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = a.w[i];
    return r;
}

// ---- products (leaves) ----
template <int A, int B>
PA_DEV F<1> mul(const F<A>& a, const F<B>& b) {
    static_assert(A * B <= 17, "product column bound");
    F<1> r;
    fl_mul_leaf(r.w, a.w, b.w);
    return r;
}
template <int A>
PA_DEV F<1> sqr(const F<A>& a) {
    static_assert(A <= 3, "square column bound");
    F<1> r;
    fl_sqr_leaf(r.w, a.w);
    return r;
}
// a*b + c*d with one reduction
template <int A, int B, int C, int D>
PA_DEV F<1> sop(const F<A>& a, const F<B>& b, const F<C>& c, const F<D>& d) {
    static_assert(A * B + C * D <= 17, "sum-of-products column bound");
    F<1> r;
    fl_sop2_leaf(r.w, a.w, b.w, c.w, d.w);
    return r;
}

// ---- reduction to F<1> ----
template <int U>
PA_DEV F<1> red(const F<U>& x) {
    // k = floor(T FL_KQ / 2^64), T = x13 2^28 + x12: floor(V/q) or one less
    const uint64_t p1 = (uint64_t)x.w[12] * FL_KQ;
    const uint64_t p2 = (uint64_t)x.w[13] * FL_KQ;
    const uint32_t k = (uint32_t)((p2 + (p1 >> 28)) >> 36);
    F<1> r;
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) {
        acc += (int64_t)x.w[i] - (int64_t)((uint64_t)k * FL_Q[i]);
        r.w[i] = (uint32_t)acc & FL_MASK;
        acc >>= 28;
    }
    acc += (int64_t)x.w[13] - (int64_t)((uint64_t)k * FL_Q[13]);
    r.w[13] = (uint32_t)acc;
    return r;
}
PA_DEV F<1> red(const F<1>& x) { return x; }

// ---- constants ----
PA_DEV F<1> fl_zero() {
    F<1> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = 0;
    return r;
}
PA_DEV F<1> fl_c(const uint32_t* c) {
    F<1> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = c[i];
    return r;
}
PA_DEV F<1> fl_one() { return fl_c(FL_ONE); }

// ---- boundary conversions ----
// 12 x 32-bit words -> 14 x 28-bit limbs (same integer)
PA_DEV F<1> fl_split(const Fq& x) {
    F<1> r;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        const int bit = 28 * i, wi = bit >> 5, sh = bit & 31;
        uint64_t v = x.w[wi];
        if (wi + 1 < 12) v |= (uint64_t)x.w[wi + 1] << 32;
        r.w[i] = (uint32_t)(v >> sh) & FL_MASK;
    }
    return r;
}

// F<1> (limbs < 2^28, value < 2q) -> canonical (< q)
PA_DEV F<1> fl_canon(const F<1>& t) {
    F<1> d;
    int32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        const int32_t s = (int32_t)t.w[i] - (int32_t)FL_Q[i] + borrow;
        d.w[i] = (uint32_t)s & FL_MASK;
        borrow = s >> 28;  // 0 or -1
    }
    const bool keep = borrow != 0;  // t < q
    F<1> r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.w[i] = keep ? t.w[i] : d.w[i];
    return r;
}

// canonical 28-bit limbs -> 12 x 32-bit words
PA_DEV Fq fl_pack(const F<1>& x) {
    Fq r;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        const int bit = 32 * j, li = bit / 28, sh = bit % 28;
        uint64_t v = (uint64_t)x.w[li] >> sh;
        if (li + 1 < 14) v |= (uint64_t)x.w[li + 1] << (28 - sh);
        if (li + 2 < 14 && 56 - sh < 64) v |= (uint64_t)x.w[li + 2] << (56 - sh);
        r.w[j] = (uint32_t)v;
    }
    return r;
}

// canonical 12 x 32-bit words of a bound-1 value (< 2q): pack first, then one
// conditional subtraction of q as a 32-bit borrow chain (v_sub_co / v_subb_co)
// and a select (the config-2 kernel: 209 -> 196 instructions around its product leaf)
PA_DEV Fq fl_pack_canon(const F<1>& x) {
    const Fq t = fl_pack(x);
    Fq d;
    unsigned borrow = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        const uint32_t qj = q_word(j);
        d.w[j] = __builtin_subc(t.w[j], qj, borrow, &borrow);
    }
    Fq r;
#pragma unroll
    for (int j = 0; j < 12; j++) r.w[j] = borrow ? t.w[j] : d.w[j];   // borrow: t < q
    return r;
}

// ABI value (canonical, R = 2^384) -> F<1> with R = 2^392
PA_DEV F<1> fl_from_abi(const Fq& x) { return mul(fl_split(x), fl_c(FL_TO)); }

// any bound -> canonical ABI value (R = 2^384)
template <int U>
PA_DEV Fq fl_to_abi(const F<U>& x) {
    return fl_pack_canon(mul(red(x), fl_c(FL_FROM)));
}

// canonical value is zero
template <int U>
PA_DEV bool fl_is_zero(const F<U>& x) {
    const F<1> c = fl_canon(red(x));
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) acc |= c.w[i];
    return acc == 0;
}

PA_DEV F<1> fl_load(const uint64_t* p) {
    Fq x;
    fq_load(x, p);
    return fl_from_abi(x);
}
template <int U>
PA_DEV void fl_store(uint64_t* p, const F<U>& x) {
    fq_store(p, fl_to_abi(x));
}

}  // namespace pa
