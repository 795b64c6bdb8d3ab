// G2 line precomputation and the prepared Miller loop on the lazy core
// (fl.h / tower_fl.h), one pairing per lane.
//
//   dbl_step_fl   doubling_step   reference src/bls12_381/mod.rs:176-245
//   add_step_fl   addition_step   mod.rs:247-333
//   ell_fl        ell             mod.rs:57-69
//
// Same field values as the reference formulas (pairing.h holds the 12-word
// transcription); the coefficients are stored canonical (fl_store), so a
// G2Prepared record written here is bit-identical to the reference's.  Bounds
// are carried in the types: every red() below is where the next product's
// column bound (fl.h) would otherwise be exceeded.
#pragma once
#include "pairing.h"
#include "tower_fl.h"

namespace pa {

struct G2JacFl {
    F2<1> x, y, z;
};
struct LineFl {
    F2<1> c0, c1, c2;
};

// doubling_step: returns (2 z' z^2, -2 (3x^2) z^2, (x + 3x^2)^2 - x^2 - (3x^2)^2 - 4y^2)
PA_DEV LineFl dbl_step_fl(G2JacFl& r) {
    const F2<1> t0 = sqr(r.x);                                        // x^2
    const F2<1> t1 = sqr(r.y);                                        // y^2
    const F2<1> t2 = sqr(t1);                                         // y^4
    const F2<1> t3 = red(dbl(sub(sqr(add(t1, r.x)), add(t0, t2))));  // 2((x + y^2)^2 - x^2 - y^4)
    const F2<1> t4 = red(add(dbl(t0), t0));                           // 3 x^2
    const F2<1> t5 = sqr(t4);
    const F2<1> zz = sqr(r.z);
    LineFl c;
    c.c2 = red(sub(sqr(add(r.x, t4)), add(add(t0, t5), dbl(dbl(t1)))));
    c.c1 = mul(neg(dbl(t4)), zz);
    const F2<1> x = red(sub(t5, dbl(t3)));
    const F2<1> z = red(sub(sqr(add(r.z, r.y)), add(t1, zz)));
    r.y = red(sub(mul(sub(t3, x), t4), dbl(dbl(dbl(t2)))));
    r.x = x;
    r.z = z;
    c.c0 = mul(dbl(z), zz);
    return c;
}

// addition_step (mixed, q affine)
PA_DEV LineFl add_step_fl(G2JacFl& r, const F2<1>& qx, const F2<1>& qy) {
    const F2<1> zz = sqr(r.z);
    const F2<1> yy = sqr(qy);
    const F2<1> t0 = mul(zz, qx);
    const F2<1> t1 = mul(sub(sqr(add(qy, r.z)), add(yy, zz)), zz);
    const F2<1> t2 = red(sub(t0, r.x));
    const F2<1> t3 = sqr(t2);
    const F2<4> t4 = dbl(dbl(t3));
    const F2<1> t5 = mul(t4, t2);
    const F2<1> t6 = red(sub(t1, dbl(r.y)));
    const F2<1> t9 = mul(t6, qx);
    const F2<1> t7 = mul(t4, r.x);
    const F2<1> x = red(sub(sqr(t6), add(t5, dbl(t7))));
    const F2<1> z = red(sub(sqr(add(r.z, t2)), add(zz, t3)));
    const F2<1> t8 = mul(sub(t7, x), t6);
    r.y = red(sub(t8, dbl(mul(r.y, t5))));
    r.x = x;
    r.z = z;
    const F2<1> t10 = red(sub(sqr(add(qy, z)), add(yy, sqr(z))));
    LineFl c;
    c.c0 = red(dbl(z));
    c.c1 = red(dbl(neg(t6)));
    c.c2 = red(sub(dbl(t9), t10));
    return c;
}

// One line record of a G2Prepared in HBM: (c0, c1, c2), 36 words, canonical
// ABI values (R = 2^384).
PA_DEV void store_line(uint64_t* p, const LineFl& c) {
    store2(p, c.c0);
    store2(p + 12, c.c1);
    store2(p + 24, c.c2);
}

// ell(f, (c0, c1, c2), P) = f.mul_by_014(c2, c1 P.x, c0 P.y) straight from the
// ABI words of a line record.  kx = P.x (R'^2 / R), ky likewise (one product
// each per pairing), so mul(split(c1), kx) = c1 P.x in the lazy domain: the
// ABI -> lazy conversion of c0 and c1 is folded into the products ell needs
// anyway; c2 takes the ordinary conversion.
PA_DEV F12<1> ell_fl(const F12<1>& f, const uint64_t* rec, const F<1>& kx, const F<1>& ky) {
    Fq w[6];
#pragma unroll
    for (int j = 0; j < 6; j++) fq_load(w[j], rec + 6 * j);
    const F2<1> a = {mul(fl_split(w[0]), ky), mul(fl_split(w[1]), ky)};  // c0 * P.y
    const F2<1> b = {mul(fl_split(w[2]), kx), mul(fl_split(w[3]), kx)};  // c1 * P.x
    const F2<1> c = {fl_from_abi(w[4]), fl_from_abi(w[5])};
    return mul_by_014(f, c, b, a);
}

}  // namespace pa
