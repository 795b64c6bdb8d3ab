// Point decoding / encoding and square roots (SURVEY.md §8 f, rank 1): the
// step in front of every pairing in a verifier.
//
//   EncodedPoint::into_affine[_unchecked] for G1Uncompressed (ec.rs:662-736),
//   G1Compressed (ec.rs:785-837), G2Uncompressed (ec.rs:1322-1397),
//   G2Compressed (ec.rs:1448-1509); EncodedPoint::from_affine (ec.rs:737-752,
//   839-867, 1398-1415, 1510-1539); SqrtField::sqrt for Fq (fq.rs:1147-1170)
//   and Fq2 (fq2.rs:167-220).
//
// One lane per record.  Every output is canonical (affine coordinates, status
// codes, bytes), so the only freedom used is in how the subgroup membership
// r*P == 0 (ec.rs:142-144) is evaluated: by the equivalent endomorphism
// identities phi(P) == -[x^2]P (G1) and psi(P) == [x]P (G2), see
// in_subgroup below.  Records are
// read as 32-bit words and byte-swapped (the wire format is big-endian).
#include <atomic>
#include <type_traits>

#include "curve.h"
#include "dec_quad.h"
#include "dec_sqrt_sched.h"
#include "tower_fl.h"
#include "launch.h"

namespace pa {
namespace {

// (q - 3) / 4 and (q - 1) / 2: fq.rs:1152-1159, fq2.rs:174-181, 207-214
__constant__ const uint64_t kQm3Div4[6] = {0xee7fbfffffffeaaaULL, 0x07aaffffac54ffffULL, 0xd9cc34a83dac3d89ULL,
                                           0xd91dd2e13ce144afULL, 0x92c6e9ed90d2eb35ULL, 0x0680447a8e5ff9a6ULL};
__constant__ const uint64_t kQm1Div2[6] = {0xdcff7fffffffd555ULL, 0x0f55ffff58a9ffffULL, 0xb39869507b587b12ULL,
                                           0xb23ba5c279c2895fULL, 0x258dd3db21a5d66bULL, 0x0d0088f51cbff34dULL};
// R^2 mod q (fq.rs:33-40) and -1 (fq.rs:501-508), Montgomery
__constant__ const uint64_t kR2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL,
                                      0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
__constant__ const uint64_t kNegOne[6] = {0x43f5fffffffcaaaeULL, 0x32b7fff2ed47fffdULL, 0x07e83a49a2e99d69ULL,
                                          0xeca8f3318332bb7aULL, 0xef148d1ea0f4c069ULL, 0x040ab3263eff0206ULL};
// b = 4 (Montgomery), ec.rs:885-887 / 1557-1562
__constant__ const uint64_t kB[6] = {0xaa270000000cfff3ULL, 0x53cc0032fc34000aULL, 0x478fe97a6b0a807fULL,
                                     0xb1d37ebee6ba24d7ULL, 0x8ec9733bbf78ab2fULL, 0x09d645513d83de7eULL};

enum : uint8_t {
    DEC_OK = 0,
    DEC_NOT_ON_CURVE = 1,
    DEC_NOT_IN_SUBGROUP = 2,
    DEC_X_C0 = 3,
    DEC_X_C1 = 4,
    DEC_Y_C0 = 5,
    DEC_Y_C1 = 6,
    DEC_UNEXPECTED_COMPRESSION_MODE = 7,
    DEC_UNEXPECTED_INFORMATION = 8,
};

PA_DEV void fq_const(Fq& r, const uint64_t* c) { fq_from_u64(r, c); }

// a^e, MSB first; `top` = index of e's top set bit, Field::pow lib.rs:306-324; e is wave-uniform.
// Runs on the lazy 28-bit core (fl.h / tower_fl.h: ~30 % fewer instructions per
// product than the 12-word core); the result is converted back canonical, so
// the bits are unchanged.
PA_DEV F<1> to_fl(const Fq& a) { return fl_from_abi(a); }
PA_DEV F2<1> to_fl(const Fq2& a) { return {fl_from_abi(a.c0), fl_from_abi(a.c1)}; }
PA_DEV void from_fl(Fq& r, const F<1>& a) { r = fl_to_abi(a); }
PA_DEV void from_fl(Fq2& r, const F2<1>& a) {
    r.c0 = fl_to_abi(a.c0);
    r.c1 = fl_to_abi(a.c1);
}
// A 4-bit sliding window over the (wave-uniform) exponent: the odd powers
// x, x^3, .., x^15 first, then one product per window instead of one per set
// bit (the square-root exponents (q-3)/4, (q-1)/2: 605 -> ~466 products).  The
// window value is uniform, so the table pick is a uniform switch, no indexing.
template <class T>
__device__ __forceinline__ T win_mul(const T& acc, const T* t, int v) {
    switch (v >> 1) {
        case 0: return mul(acc, t[0]);
        case 1: return mul(acc, t[1]);
        case 2: return mul(acc, t[2]);
        case 3: return mul(acc, t[3]);
        case 4: return mul(acc, t[4]);
        case 5: return mul(acc, t[5]);
        case 6: return mul(acc, t[6]);
        default: return mul(acc, t[7]);
    }
}
template <class F>
__device__ __forceinline__ void pow_fixed(F& r, const F& a, const uint64_t* e, int top) {
    const auto x = to_fl(a);
    using T = typename std::remove_const<decltype(x)>::type;
    auto bit_of = [&](int b) { return (int)((e[b >> 6] >> (b & 63)) & 1); };
    T t[8];
    t[0] = x;
    const T x2 = sqr(x);
#pragma unroll
    for (int k = 1; k < 8; k++) t[k] = mul(t[k - 1], x2);
    T acc = x;      // the top set bit
    int bit = top - 1;
#pragma unroll 1
    while (bit >= 0) {
        if (!bit_of(bit)) {
            acc = sqr(acc);
            bit--;
            continue;
        }
        int lo = bit - 3 < 0 ? 0 : bit - 3;
        while (!bit_of(lo)) lo++;
        int v = 0;
#pragma unroll 1
        for (int b = bit; b >= lo; b--) {
            acc = sqr(acc);
            v = 2 * v + bit_of(b);
        }
        acc = win_mul(acc, t, v);
        bit = lo - 1;
    }
    from_fl(r, acc);
}

// canonical (into_repr) words of a Montgomery element: a * 1 * R^-1
PA_DEV void fq_canonical(uint32_t c[12], const Fq& a) {
    Fq one_raw, t;
    fq_zero(one_raw);
    one_raw.w[0] = 1;
    fq_mul(t, a, one_raw);
#pragma unroll
    for (int i = 0; i < 12; i++) c[i] = t.w[i];
}
// PartialOrd of Fq (canonical comparison): -1, 0, 1
PA_DEV int fq_cmp(const Fq& a, const Fq& b) {
    uint32_t ca[12], cb[12];
    fq_canonical(ca, a);
    fq_canonical(cb, b);
    int r = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        if (r == 0 && ca[11 - i] != cb[11 - i]) r = ca[11 - i] < cb[11 - i] ? -1 : 1;
    }
    return r;
}
PA_DEV int cmp(const Fq& a, const Fq& b) { return fq_cmp(a, b); }
PA_DEV int cmp(const Fq2& a, const Fq2& b) {  // fq2.rs:21-30: c1 first
    const int c = fq_cmp(a.c1, b.c1);
    return c != 0 ? c : fq_cmp(a.c0, b.c0);
}

// SqrtField::sqrt, fq.rs:1147-1170
PA_DEV bool sqrt(Fq& r, const Fq& a) {
    Fq a1, a0, m1;
    pow_fixed(a1, a, kQm3Div4, 378);
    fq_sqr(a0, a1);
    fq_mul(a0, a0, a);
    fq_const(m1, kNegOne);
    if (fq_eq(a0, m1)) return false;
    fq_mul(r, a1, a);
    return true;
}
// SqrtField::sqrt, fq2.rs:167-220 (Algorithm 9 of eprint 2012/685)
PA_DEV bool sqrt(Fq2& r, const Fq2& a) {
    if (is_zero(a)) {
        zero(r);
        return true;
    }
    Fq2 a1, alpha, a0, m1;
    pow_fixed(a1, a, kQm3Div4, 378);
    sqr(alpha, a1);
    mul(alpha, alpha, a);
    frobenius_map(a0, alpha, 1);
    mul(a0, a0, alpha);
    fq_const(m1.c0, kNegOne);
    fq_zero(m1.c1);
    if (eq(a0, m1)) return false;
    mul(a1, a1, a);
    if (eq(alpha, m1)) {
        Fq2 u;
        fq_zero(u.c0);
        fq_one(u.c1);
        mul(r, a1, u);
    } else {
        Fq2 one2, t;
        one(one2);
        add(alpha, alpha, one2);
        pow_fixed(t, alpha, kQm1Div2, 379);
        mul(r, a1, t);
    }
    return true;
}

// Some square root of a in Fq2 (or false if a is not a square), for decoding:
// point_from_x keeps the root whose sign matches the encoding flag, so any root
// decodes to the same point.  Complex method for q = 3 mod 4: a = a0 + a1 u is
// a square iff its norm n = a0^2 + a1^2 is one in Fq; with s = sqrt(n), one of
// t = (a0 +- s) / 2 is a nonzero square x0^2 (unless a1 = 0), and
// sqrt(a) = x0 + a1 / (2 x0) u.  Two or three Fq exponentiations instead of
// fq2.rs:167-220's two Fq2 ones.  SqrtField::sqrt itself (k_sqrt) keeps the
// reference's algorithm above.
// 1/2 = (q + 1) / 2, Montgomery form (R = 2^384)
__constant__ const uint64_t kHalfMont[6] = {0x1804000000015554ULL, 0x855000053ab00001ULL, 0x633cb57c253c276fULL,
                                            0x6e22d1ec31ebb502ULL, 0xd3916126f2d14ca2ULL, 0x17fbb8571a006596ULL};
PA_DEV bool sqrt_any(Fq2& r, const Fq2& a) {
    if (is_zero(a)) {
        zero(r);
        return true;
    }
    Fq n, s, t, x0, x1;
    {
        Fq b;
        fq_sqr(n, a.c0);
        fq_sqr(b, a.c1);
        fq_add(n, n, b);
    }
    if (!sqrt(s, n)) return false;
    // t = (a0 + s) / 2: halve by a Montgomery product with 2^-1
    Fq half;
    fq_const(half, kHalfMont);
    fq_add(t, a.c0, s);
    fq_mul(t, t, half);
    bool ok = sqrt(x0, t) && !fq_is_zero(x0);
    if (!ok) {
        fq_sub(t, a.c0, s);
        fq_mul(t, t, half);
        ok = sqrt(x0, t) && !fq_is_zero(x0);
    }
    if (!ok) {
        // a1 = 0 and a0 not a square: sqrt(a0) = sqrt(-a0) u
        if (!fq_is_zero(a.c1)) return false;
        Fq m;
        fq_neg(m, a.c0);
        if (!sqrt(x1, m)) return false;
        fq_zero(r.c0);
        r.c1 = x1;
        return true;
    }
    Fq d;
    fq_add(d, x0, x0);
    fq_inv(d, d);
    fq_mul(x1, a.c1, d);
    r.c0 = x0;
    r.c1 = x1;
    return true;
}
PA_DEV bool sqrt_any(Fq& r, const Fq& a) { return sqrt(r, a); }

PA_DEV void coeff_b(Fq& b) { fq_const(b, kB); }
PA_DEV void coeff_b(Fq2& b) {
    fq_const(b.c0, kB);
    fq_const(b.c1, kB);
}

// x^3 + b
template <class F>
PA_DEV void curve_rhs(F& r, const F& x) {
    F b;
    sqr(r, x);
    mul(r, r, x);
    coeff_b(b);
    add(r, r, b);
}

// get_point_from_x, ec.rs:100-121
template <class F>
PA_DEV bool point_from_x(Aff<F>& out, const F& x, bool greatest) {
    F rhs, y, negy;
    curve_rhs(rhs, x);
    if (!sqrt_any(y, rhs)) return false;
    neg(negy, y);
    out.x = x;
    out.y = ((cmp(y, negy) < 0) != greatest) ? y : negy;
    out.inf = false;
    return true;
}

// is_on_curve, ec.rs:125-140 (affine, not infinity)
template <class F>
PA_DEV bool on_curve(const Aff<F>& a) {
    F y2, rhs;
    sqr(y2, a.y);
    curve_rhs(rhs, a.x);
    return eq(y2, rhs);
}

// is_in_correct_subgroup_assuming_on_curve, ec.rs:142-144: r * P == 0.
// The reference multiplies by r (255 doublings + ~128 additions).  For a point
// already on the curve the same yes/no answer comes from an endomorphism
// identity (Scott, "A note on group membership tests for G1, G2 and GT on BLS
// pairing-friendly curves", eprint 2021/1130, sections 4 and 6; the tests the
// zkcrypto bls12_381 crate uses):
//   G1: P in G1  <=>  phi(P) == -[x^2] P,  phi(x, y) = (beta x, y)
//   G2: P in G2  <=>  psi(P) == [x] P = -[|x|] P,
//       psi(x, y) = (conj(x) cx, conj(y) cy), cx = (u+1)^-((q-1)/3), cy = (u+1)^-((q-1)/2)
// with x = -0xd201000000010000 the BLS parameter (mod.rs:23-25): 126 (G1) or
// 63 (G2) doublings instead of 255.  tests/test_decode.py pins the answers to
// the oracle's r * P on the reference's invalid-vector suites plus random
// on-curve points with and without small-order components.
__constant__ const uint64_t kBeta[6] = {0x30f1361b798a64e8ULL, 0xf3b8ddab7ece5a2aULL, 0x16a8ca3ac61577f7ULL,
                                        0xc26a2ff874fd029bULL, 0x3636b76660701c6eULL, 0x051ba4ab241b6160ULL};
__constant__ const uint64_t kPsiX1[6] = {0x890dc9e4867545c3ULL, 0x2af322533285a5d5ULL, 0x50880866309b7e2cULL,
                                         0xa20d1b8c7e881024ULL, 0x14e4f04fe2db9068ULL, 0x14e56d3f1564853aULL};
__constant__ const uint64_t kPsiY0[6] = {0x3e2f585da55c9ad1ULL, 0x4294213d86c18183ULL, 0x382844c88b623732ULL,
                                         0x92ad2afd19103e18ULL, 0x1d794e4fac7cf0b9ULL, 0x0bd592fc7d825ec8ULL};
__constant__ const uint64_t kPsiY1[6] = {0x7bcfa7a25aa30fdaULL, 0xdc17dec12a927e7cULL, 0x2f088dd86b4ebef1ULL,
                                         0xd1ca2087da74d4a7ULL, 0x2da2596696cebc1dULL, 0x0e2b7eedbbfd87d2ULL};
constexpr uint64_t kAbsX = 0xd201000000010000ULL;

// dbl-2009-l (ec.rs:296-354) on the lazy core for G1 (E = F<1>) and G2
// (E = F2<1>): the same field values as jac_double for a nonzero point
template <class E>
struct FlJacE {
    E x, y, z;
};
template <class E>
PA_DEV void fl_double_any(FlJacE<E>& p) {
    const auto a = sqr(p.x);
    const auto b = sqr(p.y);
    const auto c = sqr(b);
    const auto d = red(dbl(sub(sqr(add(p.x, b)), add(a, c))));
    const auto e = red(add(dbl(a), a));
    const auto f = sqr(e);
    p.z = red(dbl(mul(p.z, p.y)));
    p.x = red(sub(f, dbl(d)));
    p.y = red(sub(mul(e, sub(d, p.x)), dbl(dbl(dbl(c)))));
}

// r = [|x|] p: MSB-first double-and-add (63 doublings, 5 additions).  The runs
// of doublings between set bits go through the lazy core; the 5 additions use
// the 12-word jac_add.  A zero point (z = 0) stays zero under either doubling
// and is all the callers look at, so the yes/no result is the 12-word one.
template <class F>
__device__ __forceinline__ void mul_abs_x(Jac<F>& r, const Jac<F>& p) {
    r = p;  // bit 63
    int bit = 62;
#pragma unroll 1
    while (bit >= 0) {
        int stop = bit;  // the run ends at the next set bit (or bit 0)
        while (stop > 0 && !((kAbsX >> stop) & 1)) stop--;
        if (!jac_is_zero(r)) {
            FlJacE<decltype(to_fl(r.x))> t{to_fl(r.x), to_fl(r.y), to_fl(r.z)};
#pragma unroll 1
            for (int k = bit; k >= stop; k--) fl_double_any(t);
            from_fl(r.x, t.x);
            from_fl(r.y, t.y);
            from_fl(r.z, t.z);
        }
        if ((kAbsX >> stop) & 1) jac_add(r, p);
        bit = stop - 1;
    }
}

// affine e == -q (q Jacobian): e.x z^2 == X and e.y z^3 == -Y, q not zero
template <class F>
PA_DEV bool aff_eq_neg_jac(const F& ex, const F& ey, const Jac<F>& q) {
    if (jac_is_zero(q)) return false;
    F zz, t, u;
    sqr(zz, q.z);
    mul(t, ex, zz);
    if (!eq(t, q.x)) return false;
    mul(zz, zz, q.z);
    mul(t, ey, zz);
    add(u, t, q.y);
    return is_zero(u);
}

PA_DEV bool in_subgroup_endo(const Aff<Fq>& a) {
    Jac<Fq> p, t, q;
    jac_from_affine(p, a);
    mul_abs_x(t, p);
    mul_abs_x(q, t);  // [x^2] P
    Fq beta, ex;
    fq_const(beta, kBeta);
    mul(ex, a.x, beta);
    return aff_eq_neg_jac(ex, a.y, q);
}
PA_DEV bool in_subgroup_endo(const Aff<Fq2>& a) {
    Jac<Fq2> p, q;
    jac_from_affine(p, a);
    mul_abs_x(q, p);  // [|x|] P = -[x] P
    Fq2 c, ex, ey, yc;
    yc.c0 = a.y.c0;
    neg(yc.c1, a.y.c1);
    // cx = (0, kPsiX1): conj(x) * cx = (x1 cx1, x0 cx1)
    Fq cx1;
    fq_const(cx1, kPsiX1);
    mul(ex.c0, a.x.c1, cx1);
    mul(ex.c1, a.x.c0, cx1);
    fq_const(c.c0, kPsiY0);
    fq_const(c.c1, kPsiY1);
    mul(ey, yc, c);
    // psi(P) == [x] P == -[|x|] P
    return aff_eq_neg_jac(ex, ey, q);
}

template <class F>
__device__ __forceinline__ bool in_subgroup(const Aff<F>& a) {
    if (a.inf) return true;
    return in_subgroup_endo(a);
}

// 48 big-endian bytes (word-aligned) -> 12 little-endian u32 words
PA_DEV void read_be48(uint32_t w[12], const uint8_t* src) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
#pragma unroll
    for (int j = 0; j < 12; j++) w[11 - j] = __builtin_bswap32(s[j]);
}
PA_DEV void write_be48(uint8_t* dst, const uint32_t w[12]) {
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
    for (int j = 0; j < 12; j++) d[j] = __builtin_bswap32(w[11 - j]);
}

// PrimeField::from_repr, fq.rs:747-756: canonical words < q, then * R^2
PA_DEV bool from_repr(Fq& r, const uint32_t w[12]) {
    int c = 0;
#pragma unroll
    for (int i = 11; i >= 0; i--) {
        if (c == 0 && w[i] != q_word(i)) c = w[i] < q_word(i) ? -1 : 1;
    }
    if (c >= 0) return false;
    Fq x, r2;
#pragma unroll
    for (int i = 0; i < 12; i++) x.w[i] = w[i];
    fq_const(r2, kR2);
    fq_mul(r, x, r2);
    return true;
}

// The flag handling shared by the four into_affine_unchecked bodies.  `b` are
// the record's words in wire order (byte-swapped per word: b[0] holds bytes
// 0..3 with byte 0 in bits 31..24).  Returns -1 to go on decoding.
PA_DEV int check_flags(uint32_t* b, int nwords, bool compressed, bool& greatest) {
    greatest = false;
    const uint32_t top = b[0] >> 24;
    if (((top >> 7) & 1) != (compressed ? 1u : 0u)) return DEC_UNEXPECTED_COMPRESSION_MODE;
    if (top & 0x40) {
        uint32_t any = b[0] & 0x3fffffffu;
        for (int j = 1; j < nwords; j++) any |= b[j];
        return any ? DEC_UNEXPECTED_INFORMATION : DEC_OK;
    }
    if (top & 0x20) {
        if (!compressed) return DEC_UNEXPECTED_INFORMATION;
        greatest = true;
    }
    b[0] &= 0x1fffffffu;
    return -1;
}

// words of coordinate k (48-byte chunk k) of a wire record in little-endian order
PA_DEV void chunk(uint32_t w[12], const uint32_t* b, int k) {
#pragma unroll
    for (int j = 0; j < 12; j++) w[11 - j] = b[12 * k + j];
}

template <class F>
PA_DEV void aff_zero(Aff<F>& a) {
    zero(a.x);
    one(a.y);
    a.inf = true;
}

// G1 / G2 decode of one record; returns the status
template <int G, bool COMPRESSED>
PA_DEV int decode_one(Aff<typename std::conditional<G == 1, Fq, Fq2>::type>& out, const uint8_t* rec, bool checked) {
    using F = typename std::conditional<G == 1, Fq, Fq2>::type;
    constexpr int coords = (G == 1 ? 1 : 2) * (COMPRESSED ? 1 : 2);
    constexpr int nwords = 12 * coords;
    uint32_t b[nwords];
    const uint32_t* s = reinterpret_cast<const uint32_t*>(rec);
#pragma unroll
    for (int j = 0; j < nwords; j++) b[j] = __builtin_bswap32(s[j]);
    bool greatest;
    int st = check_flags(b, nwords, COMPRESSED, greatest);
    aff_zero(out);
    if (st >= 0) return st;
    uint32_t w[12];
    F x, y;
    if constexpr (G == 1) {
        chunk(w, b, 0);
        if (!from_repr(x, w)) return DEC_X_C0;
        if (!COMPRESSED) {
            chunk(w, b, 1);
            if (!from_repr(y, w)) return DEC_Y_C0;
        }
    } else {
        // wire order x.c1, x.c0[, y.c1, y.c0]; the reference decodes c0 first
        chunk(w, b, 1);
        if (!from_repr(x.c0, w)) return DEC_X_C0;
        chunk(w, b, 0);
        if (!from_repr(x.c1, w)) return DEC_X_C1;
        if (!COMPRESSED) {
            chunk(w, b, 3);
            if (!from_repr(y.c0, w)) return DEC_Y_C0;
            chunk(w, b, 2);
            if (!from_repr(y.c1, w)) return DEC_Y_C1;
        }
    }
    Aff<F> a;
    if (COMPRESSED) {
        if (!point_from_x(a, x, greatest)) return DEC_NOT_ON_CURVE;
    } else {
        a.x = x;
        a.y = y;
        a.inf = false;
        if (checked && !on_curve(a)) return DEC_NOT_ON_CURVE;
    }
    if (checked && !in_subgroup(a)) return DEC_NOT_IN_SUBGROUP;
    out = a;
    return DEC_OK;
}

template <int G, bool COMPRESSED>
__global__ void __launch_bounds__(64) k_decode(const uint8_t* __restrict__ enc, size_t n, int checked,
                                               uint64_t* __restrict__ out, uint8_t* __restrict__ status) {
    using F = typename std::conditional<G == 1, Fq, Fq2>::type;
    constexpr int size = (G == 1 ? 48 : 96) * (COMPRESSED ? 1 : 2);
    constexpr int W = FieldWords<F>::n;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<F> a;
    const int st = decode_one<G, COMPRESSED>(a, enc + (size_t)size * i, checked != 0);
    store_aff(out + (size_t)(2 * W + 1) * i, a);
    status[i] = (uint8_t)st;
}

// ---------------- latency form: one record per group of quads ----------------
// The same decode (statuses, canonical outputs) with the field arithmetic
// spread over quads of lanes (dec_quad.h): G1 records on 4 quads (16 lanes),
// G2 records on 8 quads (32 lanes).  The square-root exponentiations run on
// every quad of the group at once (a quad product is ~2.5x shorter than a
// one-lane leaf); the subgroup check's Jacobian doublings and additions run
// their independent products side by side, one per quad (G2: one Fq2
// coordinate per quad), three product levels per doubling instead of ~17
// products in a row.  For a verifier's handful of points this is the path;
// large batches keep one lane per record (k_decode).
namespace qdec {
using dq::Lc;
using dq::Q;
using dq::Q2;

using dq::Fixed;
using dq::Jq;
using dq::jadd;
using dq::jdbl;
using dq::lev;
using dq::make_fixed;
using dq::one_e;
using dq::prod;
using dq::zero_e;

// [|x|] T, |x| = 0xd201000000010000 (mod.rs:23-25): MSB-first double-and-add
template <int NQ, template <int> class E>
PA_DEV Jq<E> mul_abs_x(const Fixed<E>& f, const Lc& l) {
    Jq<E> r = f.t;   // bit 63
#pragma unroll 1
    for (int bit = 62; bit >= 0; bit--) {
        jdbl<NQ>(r, l);
        if ((kAbsX >> bit) & 1) jadd<NQ>(r, f, l);
    }
    return r;
}

PA_DEV Q<1> qconst_abi(const uint64_t* c, const Lc& l) {
    Fq v;
    fq_const(v, c);
    return dq::from_abi(v, l);
}

// some square root of a (decoding keeps the root the flag asks for, so any
// root decodes to the same point); false if a is not a square.  Fq: a^((q+1)/4)
// (fq.rs:1147-1170's value), checked by squaring.
PA_DEV bool qsqrt(Q<1>& y, const Q<1>& a, const Lc& l) {
    const Q<1> w = dq::pow_fixed(a, kQm3Div4, 378, l);
    y = dq::mul(w, a, l);
    return dq::eq(dq::sqr(y, l), a, l);
}
// Fq2, complex method with no inversion and no third exponentiation (q = 3
// mod 4): n = a0^2 + a1^2, s = n^((q+1)/4), t = (a0 + s) / 2 (or (a0 - s) / 2
// if that is 0), w = t^((q-3)/4), x0 = t w.  If x0^2 == t, y = x0 + (a1 w / 2) u
// (1/x0 = w); otherwise x0^2 == -t and y = -(a1 w / 2) + x0 u.  Any failure
// (a not a square) shows in the final check y^2 == a.
template <int NQ>
PA_DEV bool qsqrt(Q2<1>& y, const Q2<1>& a, const Q<1>& half, const Lc& l) {
    using namespace dq;
    const Q<1> n = sop(a.c0, a.c0, a.c1, a.c1, l);
    const Q<1> s = mul(pow_fixed(n, kQm3Div4, 378, l), n, l);
    const Q<1> tp = mul(add(a.c0, s), half, l);
    const Q<1> tm = mul(sub(a.c0, s, l), half, l);
    const Q<1> t = sel(is_zero(tp), tm, tp);
    const Q<1> w = pow_fixed(t, kQm3Div4, 378, l);
    const Q<1> x0 = mul(t, w, l);
    const bool qr = eq(sqr(x0, l), t, l);
    const Q<1> h = mul(mul(a.c1, w, l), half, l);
    y.c0 = sel(qr, x0, red(neg(h, l), l));
    y.c1 = sel(qr, h, x0);
    return eq(prod<NQ, Q2>(y, y, l), a, l);
}

// Fq2 with one exponentiation (tools/gen_sqrt_sched.py): q^2 = 9 mod 16, so
// r = a^((q^2 + 7) / 16) has r^2 = a z, z = a^((q^2 - 1) / 8) a fourth root of
// unity for a square a; y = r c(z) with c(1) = 1, c(-1) = u, c(u) = w^3,
// c(-u) = w (w^2 = u).  The exponent is e0 + e1 q and a^q = conj(a), so one run
// of 380 Fq2 squarings serves both halves (Straus, 4-bit windows over a, a^3,
// .., a^15): ~545 Fq2 products, each one level on two quads (a squaring one
// plain product per quad), against the complex method's 2 x 466 Fq products.  No z matches: a is not a square.
template <int NQ>
PA_DEV bool qsqrt_frob(Q2<1>& y, const Q2<1>& a, const Lc& l) {
    using namespace dq;
    // the odd powers a^(2k+1), k < 8, parked in LDS (16 KB per wave; in
    // registers they would push the kernel into scratch): this lane's pieces
    // at tab[k][coordinate][lane]
    __shared__ uint4 tab[8][2][64];
    const int lane = threadIdx.x & 63;
    auto park = [&](int k, const Q2<1>& v) {
        tab[k][0][lane] = make_uint4(v.c0.w[0], v.c0.w[1], v.c0.w[2], v.c0.w[3]);
        tab[k][1][lane] = make_uint4(v.c1.w[0], v.c1.w[1], v.c1.w[2], v.c1.w[3]);
    };
    {
        const Q2<1> a2 = dq::sqr2<NQ>(a, l);
        Q2<1> t = a;
        park(0, t);
#pragma unroll 1
        for (int k = 1; k < 8; k++) {
            t = prod<NQ, Q2>(t, a2, l);
            park(k, t);
        }
    }
    auto factor = [&](int op) -> Q2<2> {   // op 1..8: a^(2k+1), 9..16: its conjugate
        const int k = (op - 1) & 7;
        const uint4 u0 = tab[k][0][lane], u1 = tab[k][1][lane];
        const Q2<1> f{Q<1>{{u0.x, u0.y, u0.z, u0.w}}, Q<1>{{u1.x, u1.y, u1.z, u1.w}}};
        return op >= 9 ? Q2<2>{relax<2>(f.c0), neg(f.c1, l)} : relax<2>(f);
    };
    Q2<1> r = red(factor(kSqrtSched[0]), l);
#pragma unroll 1
    for (int i = 1; i < kSqrtOps; i++) {
        const int op = kSqrtSched[i];
        r = op == 0 ? dq::sqr2<NQ>(r, l) : prod<NQ, Q2>(r, factor(op), l);
    }
    const Q2<1> r2 = prod<NQ, Q2>(r, r, l);
    const bool z1 = eq(r2, a, l);
    const bool zm1 = is_zero(add(r2, a));
    const bool zu = is_zero(add(r2.c0, a.c1)) && eq(r2.c1, a.c0, l);    // r^2 = a u = (-a1, a0)
    const bool zmu = eq(r2.c0, a.c1, l) && is_zero(add(r2.c1, a.c0));   // r^2 = -a u = (a1, -a0)
    const Q2<1> one{qconst(FL_ONE, l), zero_e<Q>()};
    const Q2<1> uu{zero_e<Q>(), qconst(FL_ONE, l)};
    const Q2<1> w{qconst_abi(kSqrtW[0], l), qconst_abi(kSqrtW[1], l)};
    const Q2<1> w3{qconst_abi(kSqrtW3[0], l), qconst_abi(kSqrtW3[1], l)};
    const Q2<1> c = sel(z1, one, sel(zm1, uu, sel(zu, w3, w)));
    y = prod<NQ, Q2>(r, c, l);
    return z1 || zm1 || zu || zmu;
}

// is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144) by the endomorphism
// identities of in_subgroup_endo above: G1 phi(P) == -[x^2] P
template <int NQ>
PA_DEV bool in_g1(const Q<1>& x, const Q<1>& y, const Lc& l) {
    using namespace dq;
    const Jq<Q> p{x, y, one_e<Q>(l)};
    const Jq<Q> t = mul_abs_x<NQ>(make_fixed<NQ>(p, l), l);
    if (is_zero(t.z)) return false;
    const Jq<Q> q = mul_abs_x<NQ>(make_fixed<NQ>(t, l), l);
    if (is_zero(q.z)) return false;
    const Q<1> bx = mul(qconst_abi(kBeta, l), x, l);
    const Q<1> zz = prod<NQ, Q>(q.z, q.z, l);
    const Q<1> zzz = prod<NQ, Q>(zz, q.z, l);
    if (!eq(prod<NQ, Q>(bx, zz, l), q.x, l)) return false;
    return is_zero(add(prod<NQ, Q>(y, zzz, l), q.y));
}
// G2: psi(P) == [x] P = -[|x|] P, psi(x, y) = (conj(x) cx, conj(y) cy)
template <int NQ>
PA_DEV bool in_g2(const Q2<1>& x, const Q2<1>& y, const Lc& l) {
    using namespace dq;
    const Jq<Q2> p{x, y, one_e<Q2>(l)};
    const Jq<Q2> q = mul_abs_x<NQ>(make_fixed<NQ>(p, l), l);
    if (is_zero(q.z)) return false;
    const Q<1> cx1 = qconst_abi(kPsiX1, l);
    const Q2<1> ex{mul(x.c1, cx1, l), mul(x.c0, cx1, l)};   // conj(x) * (0, cx1)
    const Q2<1> cy{qconst_abi(kPsiY0, l), qconst_abi(kPsiY1, l)};
    const Q2<1> ycj{y.c0, red(neg(y.c1, l), l)};
    const Q2<1> ey = prod<NQ, Q2>(ycj, cy, l);
    const Q2<1> zz = prod<NQ, Q2>(q.z, q.z, l);
    const Q2<1> zzz = prod<NQ, Q2>(zz, q.z, l);
    if (!eq(prod<NQ, Q2>(ex, zz, l), q.x, l)) return false;
    return is_zero(add(prod<NQ, Q2>(ey, zzz, l), q.y));
}

// decode_one's statuses and outputs, computed by the record's group
template <int G, bool COMPRESSED>
PA_DEV int decode_group(Aff<typename std::conditional<G == 1, Fq, Fq2>::type>& out, const uint8_t* rec,
                        bool checked, const Lc& l) {
    using namespace dq;
    using F = typename std::conditional<G == 1, Fq, Fq2>::type;
    constexpr int NQ = G == 1 ? 4 : 8;
    constexpr int coords = (G == 1 ? 1 : 2) * (COMPRESSED ? 1 : 2);
    constexpr int nwords = 12 * coords;
    uint32_t b[nwords];
    const uint32_t* src = reinterpret_cast<const uint32_t*>(rec);
#pragma unroll
    for (int j = 0; j < nwords; j++) b[j] = __builtin_bswap32(src[j]);
    bool greatest;
    const int st = check_flags(b, nwords, COMPRESSED, greatest);
    aff_zero(out);
    if (st >= 0) return st;
    uint32_t w[12];
    F x, y;
    if constexpr (G == 1) {
        chunk(w, b, 0);
        if (!from_repr(x, w)) return DEC_X_C0;
        if (!COMPRESSED) {
            chunk(w, b, 1);
            if (!from_repr(y, w)) return DEC_Y_C0;
        }
        const Q<1> xq = from_abi(x, l);
        const Q<1> rhs = red(add(mul(sqr(xq, l), xq, l), qconst_abi(kB, l)), l);
        Q<1> yq;
        if (COMPRESSED) {
            if (!qsqrt(yq, rhs, l)) return DEC_NOT_ON_CURVE;
            y = to_abi(yq);
            Fq negy;
            fq_neg(negy, y);
            if ((cmp(y, negy) < 0) == greatest) {
                y = negy;
                yq = red(neg(yq, l), l);
            }
        } else {
            yq = from_abi(y, l);
            if (checked && !eq(sqr(yq, l), rhs, l)) return DEC_NOT_ON_CURVE;
        }
        if (checked && !in_g1<NQ>(xq, yq, l)) return DEC_NOT_IN_SUBGROUP;
    } else {
        chunk(w, b, 1);
        if (!from_repr(x.c0, w)) return DEC_X_C0;
        chunk(w, b, 0);
        if (!from_repr(x.c1, w)) return DEC_X_C1;
        if (!COMPRESSED) {
            chunk(w, b, 3);
            if (!from_repr(y.c0, w)) return DEC_Y_C0;
            chunk(w, b, 2);
            if (!from_repr(y.c1, w)) return DEC_Y_C1;
        }
        const Q2<1> xq{from_abi(x.c0, l), from_abi(x.c1, l)};
        const Q<1> b4 = qconst_abi(kB, l);
        const Q2<1> x3 = prod<NQ, Q2>(prod<NQ, Q2>(xq, xq, l), xq, l);
        const Q2<1> rhs{red(add(x3.c0, b4), l), red(add(x3.c1, b4), l)};
        Q2<1> yq;
        if (COMPRESSED) {
            static constexpr bool kComplex = false;   // A/B: the complex method (two Fq exponentiations)
            if (kComplex ? !qsqrt<NQ>(yq, rhs, qconst_abi(kHalfMont, l), l) : !qsqrt_frob<NQ>(yq, rhs, l))
                return DEC_NOT_ON_CURVE;
            y.c0 = to_abi(yq.c0);
            y.c1 = to_abi(yq.c1);
            Fq2 negy;
            neg(negy, y);
            if ((cmp(y, negy) < 0) == greatest) {
                y = negy;
                yq = red(neg(yq, l), l);
            }
        } else {
            yq = Q2<1>{from_abi(y.c0, l), from_abi(y.c1, l)};
            if (checked && !eq(prod<NQ, Q2>(yq, yq, l), rhs, l)) return DEC_NOT_ON_CURVE;
        }
        if (checked && !in_g2<NQ>(xq, yq, l)) return DEC_NOT_IN_SUBGROUP;
    }
    out.x = x;
    out.y = y;
    out.inf = false;
    return DEC_OK;
}

}  // namespace qdec

template <int G, bool COMPRESSED>
__global__ void __launch_bounds__(64) k_decode_quad(const uint8_t* __restrict__ enc, size_t n, int checked,
                                                    uint64_t* __restrict__ out, uint8_t* __restrict__ status) {
    using F = typename std::conditional<G == 1, Fq, Fq2>::type;
    constexpr int NQ = G == 1 ? 4 : 8, L = 4 * NQ, PER = 64 / L;
    constexpr int size = (G == 1 ? 48 : 96) * (COMPRESSED ? 1 : 2);
    constexpr int W = FieldWords<F>::n;
    const int lane = threadIdx.x;
    const size_t i = (size_t)blockIdx.x * PER + lane / L;
    if (i >= n) return;   // whole groups leave together
    const dq::Lc l = dq::lctx(lane, NQ);
    Aff<F> a;
    const int st = qdec::decode_group<G, COMPRESSED>(a, enc + (size_t)size * i, checked != 0, l);
    if (lane % L == 0) {
        store_aff(out + (size_t)(2 * W + 1) * i, a);
        status[i] = (uint8_t)st;
    }
}

// is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144) over affine points
// in HBM, apart from a decode: EncodedPoint::into_affine is
// into_affine_unchecked + this check (ec.rs:676-684, 786-793), so a verifier
// can start its pairing on the unchecked points while the check runs beside it
// (bench.py --workload verify --decode).  The same endomorphism identities as
// the decode's checked path (in_subgroup / qdec::in_g1, in_g2); infinity is in
// the subgroup.  For a point off the curve the answer is unspecified, as the
// reference's name says.  One record per group of quads (latency form) ...
template <int G>
__global__ void __launch_bounds__(64) k_subgroup_quad(const uint64_t* __restrict__ pts, size_t n,
                                                      uint8_t* __restrict__ ok) {
    constexpr int NQ = G == 1 ? 4 : 8, L = 4 * NQ, PER = 64 / L;
    constexpr int RW = G == 1 ? 13 : 25;
    const int lane = threadIdx.x;
    const size_t i = (size_t)blockIdx.x * PER + lane / L;
    if (i >= n) return;   // whole groups leave together
    const dq::Lc l = dq::lctx(lane, NQ);
    const uint64_t* r = pts + (size_t)RW * i;
    bool in = true;
    if ((r[RW - 1] & 0xff) == 0) {   // the infinity byte (pa_g1_affine / pa_g2_affine)
        if constexpr (G == 1) {
            Fq x, y;
            fq_load(x, r);
            fq_load(y, r + 6);
            in = qdec::in_g1<NQ>(dq::from_abi(x, l), dq::from_abi(y, l), l);
        } else {
            Fq v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) fq_load(v[k], r + 6 * k);
            in = qdec::in_g2<NQ>(dq::Q2<1>{dq::from_abi(v[0], l), dq::from_abi(v[1], l)},
                                 dq::Q2<1>{dq::from_abi(v[2], l), dq::from_abi(v[3], l)}, l);
        }
    }
    if (lane % L == 0) ok[i] = in ? 1 : 0;
}
// ... or one lane per record (throughput form, large batches)
template <int G>
__global__ void __launch_bounds__(64) k_subgroup(const uint64_t* __restrict__ pts, size_t n, uint8_t* __restrict__ ok) {
    using F = typename std::conditional<G == 1, Fq, Fq2>::type;
    constexpr int W = FieldWords<F>::n;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<F> a;
    load_aff(a, pts + (size_t)(2 * W + 1) * i);
    ok[i] = in_subgroup(a) ? 1 : 0;
}

// EncodedPoint::from_affine
template <int G, bool COMPRESSED>
__global__ void __launch_bounds__(64) k_encode(const uint64_t* __restrict__ in, size_t n, uint8_t* __restrict__ enc) {
    using F = typename std::conditional<G == 1, Fq, Fq2>::type;
    constexpr int size = (G == 1 ? 48 : 96) * (COMPRESSED ? 1 : 2);
    constexpr int W = FieldWords<F>::n;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<F> a;
    load_aff(a, in + (size_t)(2 * W + 1) * i);
    uint8_t* rec = enc + (size_t)size * i;
    uint32_t* d = reinterpret_cast<uint32_t*>(rec);
    if (a.inf) {
        for (int j = 0; j < size / 4; j++) d[j] = 0;
        d[0] = __builtin_bswap32((COMPRESSED ? 0x80u : 0u) << 24 | 0x40u << 24);
        return;
    }
    uint32_t w[12];
    if constexpr (G == 1) {
        fq_canonical(w, a.x);
        write_be48(rec, w);
        if (!COMPRESSED) {
            fq_canonical(w, a.y);
            write_be48(rec + 48, w);
        }
    } else {
        fq_canonical(w, a.x.c1);
        write_be48(rec, w);
        fq_canonical(w, a.x.c0);
        write_be48(rec + 48, w);
        if (!COMPRESSED) {
            fq_canonical(w, a.y.c1);
            write_be48(rec + 96, w);
            fq_canonical(w, a.y.c0);
            write_be48(rec + 144, w);
        }
    }
    if (COMPRESSED) {
        F negy;
        neg(negy, a.y);
        uint32_t flags = 0x80u;
        if (cmp(a.y, negy) > 0) flags |= 0x20u;  // ec.rs:861-864
        rec[0] |= (uint8_t)flags;
    }
}

template <class F>
__global__ void __launch_bounds__(64) k_sqrt(const uint64_t* __restrict__ in, size_t n, uint64_t* __restrict__ out,
                                             uint8_t* __restrict__ ok) {
    constexpr int W = FieldWords<F>::n;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    F a, r;
    load(a, in + (size_t)W * i);
    const bool s = sqrt(r, a);
    if (!s) zero(r);
    store(out + (size_t)W * i, r);
    ok[i] = s ? 1 : 0;
}

unsigned blocks_for(size_t n) { return (unsigned)((n + 63) / 64); }

}  // namespace

namespace {
std::atomic<int> g_decode_variant{0};   // pa_set_decode_kernel (any host thread): 0 by batch size, 1 one lane per record, 2 quad groups
size_t decode_quad_max() {
    static const size_t v = [] {
        const char* e = getenv("PA_DECODE_QUAD_MAX");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)8192;
    }();
    return v;
}
}  // namespace
void set_decode_variant(int v) { g_decode_variant.store(v, std::memory_order_relaxed); }

hipError_t launch_decode(int group, int compressed, int checked, const uint8_t* enc, size_t n, uint64_t* out,
                         uint8_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // the latency form for small batches with field work (an uncompressed
    // unchecked decode is byte handling only: one lane per record)
    const int dv = g_decode_variant.load(std::memory_order_relaxed);
    const bool quad = (compressed || checked) && (dv == 2 || (dv == 0 && n <= decode_quad_max()));
    if (quad) {
        const unsigned per = group == 1 ? 4 : 2;   // records per 64-lane block
        const unsigned bq = (unsigned)((n + per - 1) / per);
        if (group == 1 && compressed) k_decode_quad<1, true><<<bq, 64, 0, stream>>>(enc, n, checked, out, status);
        else if (group == 1) k_decode_quad<1, false><<<bq, 64, 0, stream>>>(enc, n, checked, out, status);
        else if (compressed) k_decode_quad<2, true><<<bq, 64, 0, stream>>>(enc, n, checked, out, status);
        else k_decode_quad<2, false><<<bq, 64, 0, stream>>>(enc, n, checked, out, status);
        return hipGetLastError();
    }
    const unsigned b = blocks_for(n);
    if (group == 1 && compressed) k_decode<1, true><<<b, 64, 0, stream>>>(enc, n, checked, out, status);
    else if (group == 1) k_decode<1, false><<<b, 64, 0, stream>>>(enc, n, checked, out, status);
    else if (compressed) k_decode<2, true><<<b, 64, 0, stream>>>(enc, n, checked, out, status);
    else k_decode<2, false><<<b, 64, 0, stream>>>(enc, n, checked, out, status);
    return hipGetLastError();
}

hipError_t launch_subgroup_check(int group, const uint64_t* pts, size_t n, uint8_t* ok, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const int dv = g_decode_variant.load(std::memory_order_relaxed);
    if (dv == 2 || (dv == 0 && n <= decode_quad_max())) {
        const unsigned per = group == 1 ? 4 : 2;   // records per 64-lane block
        const unsigned bq = (unsigned)((n + per - 1) / per);
        if (group == 1) k_subgroup_quad<1><<<bq, 64, 0, stream>>>(pts, n, ok);
        else k_subgroup_quad<2><<<bq, 64, 0, stream>>>(pts, n, ok);
        return hipGetLastError();
    }
    const unsigned b = blocks_for(n);
    if (group == 1) k_subgroup<1><<<b, 64, 0, stream>>>(pts, n, ok);
    else k_subgroup<2><<<b, 64, 0, stream>>>(pts, n, ok);
    return hipGetLastError();
}

hipError_t launch_encode(int group, int compressed, const uint64_t* in, size_t n, uint8_t* enc, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned b = blocks_for(n);
    if (group == 1 && compressed) k_encode<1, true><<<b, 64, 0, stream>>>(in, n, enc);
    else if (group == 1) k_encode<1, false><<<b, 64, 0, stream>>>(in, n, enc);
    else if (compressed) k_encode<2, true><<<b, 64, 0, stream>>>(in, n, enc);
    else k_encode<2, false><<<b, 64, 0, stream>>>(in, n, enc);
    return hipGetLastError();
}

hipError_t launch_sqrt(int degree, const uint64_t* in, size_t n, uint64_t* out, uint8_t* ok, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned b = blocks_for(n);
    if (degree == 1) k_sqrt<Fq><<<b, 64, 0, stream>>>(in, n, out, ok);
    else k_sqrt<Fq2><<<b, 64, 0, stream>>>(in, n, out, ok);
    return hipGetLastError();
}

}  // namespace pa
