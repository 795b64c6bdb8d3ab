// BLS12-381 Miller loop and final exponentiation over the lazy tower
// (tower_fl.h), one pairing per lane, every intermediate in registers.
//
//   doubling_step / addition_step   reference src/bls12_381/mod.rs:176-333
//   ell                             mod.rs:57-69
//   Bls12::miller_loop              mod.rs:40-102 (G2 prepare fused)
//   Bls12::final_exponentiation     mod.rs:104-160
//
// The line coefficients and the Jacobian R follow the reference's formulas
// value for value (they are field values, compared canonically); the lazy
// bounds (template arguments) decide where red() runs, nothing else.
#pragma once
#include "tower_fl.h"

namespace pa {
namespace fl {

constexpr uint64_t kX = 0xd201000000010000ULL;  // |x|, x < 0 (mod.rs:23-25)

struct G2J {
    F2<1> x, y, z;
};
struct Line {
    F2<1> c0, c1, c2;
};

// mod.rs:176-245 (Algorithm 26, eprint 2010/354)
PA_DEV Line doubling_step(G2J& r) {
    const F2<1> tmp0 = sqr(r.x);
    const F2<1> tmp1 = sqr(r.y);
    const F2<1> tmp2 = sqr(tmp1);
    const F2<1> tmp3 = red(dbl(sub(sqr(add(tmp1, r.x)), add(tmp0, tmp2))));
    const F2<1> tmp4 = red(add(dbl(tmp0), tmp0));
    const auto tmp6 = add(r.x, tmp4);
    const F2<1> tmp5 = sqr(tmp4);
    const F2<1> zsquared = sqr(r.z);
    const F2<1> x = red(sub(tmp5, dbl(tmp3)));
    const F2<1> z = red(sub(sqr(add(r.z, r.y)), add(tmp1, zsquared)));
    const F2<1> y = red(sub(mul(sub(tmp3, x), tmp4), dbl(dbl(dbl(tmp2)))));
    Line c;
    c.c1 = red(neg(dbl(mul(tmp4, zsquared))));
    c.c2 = red(sub(sub(sqr(tmp6), add(tmp0, tmp5)), dbl(dbl(tmp1))));
    c.c0 = red(dbl(mul(z, zsquared)));
    r.x = x;
    r.y = y;
    r.z = z;
    return c;
}

// mod.rs:247-333 (Algorithm 27, eprint 2010/354)
PA_DEV Line addition_step(G2J& r, const F2<1>& qx, const F2<1>& qy) {
    const F2<1> zsquared = sqr(r.z);
    const F2<1> ysquared = sqr(qy);
    const F2<1> t0 = mul(zsquared, qx);
    const F2<1> t1 = mul(sub(sqr(add(qy, r.z)), add(ysquared, zsquared)), zsquared);
    const F2<1> t2 = red(sub(t0, r.x));
    const F2<1> t3 = sqr(t2);
    const auto t4 = dbl(dbl(t3));
    const F2<1> t5 = mul(t4, t2);
    const F2<1> t6 = red(sub(t1, dbl(r.y)));
    const F2<1> t9 = mul(t6, qx);
    const F2<1> t7 = mul(t4, r.x);
    const F2<1> x = red(sub(sqr(t6), add(t5, dbl(t7))));
    const F2<1> z = red(sub(sqr(add(r.z, t2)), add(zsquared, t3)));
    const F2<1> t8 = mul(sub(t7, x), t6);
    const F2<1> y = red(sub(t8, dbl(mul(r.y, t5))));
    const auto t10 = sub(sqr(add(qy, z)), add(ysquared, sqr(z)));
    Line c;
    c.c2 = red(sub(dbl(t9), t10));
    c.c0 = red(dbl(z));
    c.c1 = red(dbl(neg(t6)));
    r.x = x;
    r.y = y;
    r.z = z;
    return c;
}

// mod.rs:57-69: f.mul_by_014(c2, c1 * P.x, c0 * P.y)
PA_DEV F12<1> ell(const F12<1>& f, const Line& c, const F<1>& px, const F<1>& py) {
    return mul_by_014(f, c.c2, mul_by_fq(c.c1, px), mul_by_fq(c.c0, py));
}

// P and Q are loop-invariant but used only once per step: they live in LDS
// (word-major, one column per lane: conflict-free) and are re-read where
// needed, which keeps ~84 VGPRs free for the Fq12 temporaries.
struct PQ {
    uint32_t* base;  // LDS, [84 words][64 lanes]
    PA_DEV F<1> get(int k) const {
        uint32_t* b = base;
        asm volatile("" : "+v"(b));  // opaque: no hoisting of the reads out of the loop
        F<1> r;
#pragma unroll
        for (int i = 0; i < 14; i++) r.w[i] = b[(14 * k + i) * 64];
        return r;
    }
    PA_DEV void put(int k, const F<1>& x) const {
#pragma unroll
        for (int i = 0; i < 14; i++) base[(14 * k + i) * 64] = x.w[i];
    }
};
// slots: 0 px, 1 py, 2 qx.c0, 3 qx.c1, 4 qy.c0, 5 qy.c1

// One doubling or addition step (wave-uniform choice) with its line folded
// into f.
PA_DEV void line_step(F12<1>& f, G2J& r, bool add_step, const PQ& pq) {
    Line c;
    if (add_step) {
        c = addition_step(r, {pq.get(2), pq.get(3)}, {pq.get(4), pq.get(5)});
    } else {
        c = doubling_step(r);
    }
    f = ell(f, c, pq.get(0), pq.get(1));
}

// Single-pair Miller loop, mod.rs:40-102, with G2 preparation fused in.
// Infinity pairs give one (mod.rs:50-54): those lanes run the same stream
// on their data and are selected out by the caller.
PA_DEV F12<1> miller_loop(const PQ& pq) {
    G2J r{{pq.get(2), pq.get(3)}, {pq.get(4), pq.get(5)}, f2_one()};
    F12<1> f = f12_one();
#pragma unroll 1
    for (int bit = 61; bit >= 0; bit--) {
        const bool set = ((kX >> 1) >> bit) & 1;  // wave-uniform
#pragma unroll 1
        for (int k = 0; k <= (int)set; k++) line_step(f, r, k == 1, pq);
        f = sqr(f);
    }
    line_step(f, r, false, pq);
    return red(conj(f));
}

// exp_by_x (mod.rs:116-121): f^|x| by square-and-multiply (lib.rs:306-324)
// with cyclotomic squarings, then conjugation (x < 0)
__device__ __noinline__ void exp_by_x_into(F12<1>* out, const F12<1>* fp, uint64_t x) {
    const F12<1> f = *fp;
    F12<1> res = f;
    const int top = 63 - __builtin_clzll(x);
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; bit--) {
        res = cyclotomic_sqr(res);
        if ((x >> bit) & 1) res = mul(res, f);  // wave-uniform
    }
    *out = red(conj(res));
}
PA_DEV F12<1> exp_by_x(const F12<1>& f, uint64_t x) {
    F12<1> r;
    exp_by_x_into(&r, &f, x);
    return r;
}

PA_DEV F12<1> cj(const F12<1>& a) { return red(conj(a)); }

// mod.rs:104-160.  ok = false (reference: None) iff f == 0.
PA_DEV F12<1> final_exponentiation(const F12<1>& f, bool& ok) {
    const F12<1> f1 = cj(f);
    F12<1> f2 = inverse(f, ok);
    F12<1> r = mul(f1, f2);
    f2 = r;
    r = frobenius(r, 2);
    r = mul(r, f2);
    uint64_t x = kX;
    const F12<1> y0 = cyclotomic_sqr(r);
    F12<1> y1 = exp_by_x(y0, x);
    x >>= 1;
    F12<1> y2 = exp_by_x(y1, x);
    x <<= 1;
    F12<1> y3 = cj(r);
    y1 = mul(y1, y3);
    y1 = cj(y1);
    y1 = mul(y1, y2);
    y2 = exp_by_x(y1, x);
    y3 = exp_by_x(y2, x);
    y1 = cj(y1);
    y3 = mul(y3, y1);
    y1 = cj(y1);
    y1 = frobenius(y1, 3);
    y2 = frobenius(y2, 2);
    y1 = mul(y1, y2);
    y2 = exp_by_x(y3, x);
    y2 = mul(y2, y0);
    y2 = mul(y2, r);
    y1 = mul(y1, y2);
    y2 = frobenius(y3, 1);
    y1 = mul(y1, y2);
    return y1;
}

}  // namespace fl
}  // namespace pa
