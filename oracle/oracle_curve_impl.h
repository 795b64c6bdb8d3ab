/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * Jacobian group law restated from the reference's `curve_impl!` macro
 * (src/bls12_381/ec.rs:1-621) plus the wNAF routines (src/wnaf.rs:4-71).
 * Included twice by oracle_curve.c, like the Rust macro is instantiated
 * twice: once with (G1, Fq) and once with (G2, Fq2).
 *
 * Expects: PROJ, AFF, F, CF(name) (curve function name), FF(name) (field
 * function name), COEFF_B(out) (curve b in Montgomery form).
 */

static PROJ CF(zero)(void) {                      /* ec.rs:224-230 */
    PROJ r;
    r.x = FF(zero)();
    r.y = FF(one)();
    r.z = FF(zero)();
    return r;
}
int CF(is_zero)(const PROJ *p) { return FF(is_zero)(&p->z); }          /* ec.rs:238-240 */
int CF(is_normalized)(const PROJ *p) {                                 /* ec.rs:242-244 */
    F one = FF(one)();
    return CF(is_zero)(p) || FF(eq)(&p->z, &one);
}
AFF CF(affine_zero)(void) {                                            /* ec.rs:158-164 */
    AFF a;
    memset(&a, 0, sizeof a);
    a.x = FF(zero)();
    a.y = FF(one)();
    a.infinity = 1;
    return a;
}

/* PartialEq, ec.rs:45-85 (representation-independent). */
int CF(eq)(const PROJ *a, const PROJ *b) {
    if (CF(is_zero)(a)) return CF(is_zero)(b);
    if (CF(is_zero)(b)) return 0;
    F z1 = a->z; FF(square)(&z1);
    F z2 = b->z; FF(square)(&z2);
    F tmp1 = a->x; FF(mul)(&tmp1, &z2);
    F tmp2 = b->x; FF(mul)(&tmp2, &z1);
    if (!FF(eq)(&tmp1, &tmp2)) return 0;
    FF(mul)(&z1, &a->z);
    FF(mul)(&z2, &b->z);
    FF(mul)(&z2, &a->y);
    FF(mul)(&z1, &b->y);
    return FF(eq)(&z1, &z2);
}

/* dbl-2009-l, ec.rs:296-354 */
void CF(double)(PROJ *p) {
    if (CF(is_zero)(p)) return;
    F a = p->x; FF(square)(&a);
    F b = p->y; FF(square)(&b);
    F c = b; FF(square)(&c);
    F d = p->x; FF(add)(&d, &b); FF(square)(&d); FF(sub)(&d, &a); FF(sub)(&d, &c); FF(double)(&d);
    F e = a; FF(double)(&e); FF(add)(&e, &a);
    F f = e; FF(square)(&f);
    FF(mul)(&p->z, &p->y); FF(double)(&p->z);
    p->x = f; FF(sub)(&p->x, &d); FF(sub)(&p->x, &d);
    p->y = d; FF(sub)(&p->y, &p->x); FF(mul)(&p->y, &e);
    FF(double)(&c); FF(double)(&c); FF(double)(&c);
    FF(sub)(&p->y, &c);
}

/* add-2007-bl, ec.rs:356-444 */
void CF(add)(PROJ *s, const PROJ *o) {
    if (CF(is_zero)(s)) { *s = *o; return; }
    if (CF(is_zero)(o)) return;
    F z1z1 = s->z; FF(square)(&z1z1);
    F z2z2 = o->z; FF(square)(&z2z2);
    F u1 = s->x; FF(mul)(&u1, &z2z2);
    F u2 = o->x; FF(mul)(&u2, &z1z1);
    F s1 = s->y; FF(mul)(&s1, &o->z); FF(mul)(&s1, &z2z2);
    F s2 = o->y; FF(mul)(&s2, &s->z); FF(mul)(&s2, &z1z1);
    if (FF(eq)(&u1, &u2) && FF(eq)(&s1, &s2)) {
        CF(double)(s);
        return;
    }
    F h = u2; FF(sub)(&h, &u1);
    F i = h; FF(double)(&i); FF(square)(&i);
    F j = h; FF(mul)(&j, &i);
    F r = s2; FF(sub)(&r, &s1); FF(double)(&r);
    F v = u1; FF(mul)(&v, &i);
    s->x = r; FF(square)(&s->x); FF(sub)(&s->x, &j); FF(sub)(&s->x, &v); FF(sub)(&s->x, &v);
    s->y = v; FF(sub)(&s->y, &s->x); FF(mul)(&s->y, &r);
    FF(mul)(&s1, &j); FF(double)(&s1);
    FF(sub)(&s->y, &s1);
    FF(add)(&s->z, &o->z); FF(square)(&s->z); FF(sub)(&s->z, &z1z1); FF(sub)(&s->z, &z2z2);
    FF(mul)(&s->z, &h);
}

/* madd-2007-bl, ec.rs:446-526 */
void CF(add_mixed)(PROJ *s, const AFF *o) {
    if (o->infinity) return;
    if (CF(is_zero)(s)) {
        s->x = o->x;
        s->y = o->y;
        s->z = FF(one)();
        return;
    }
    F z1z1 = s->z; FF(square)(&z1z1);
    F u2 = o->x; FF(mul)(&u2, &z1z1);
    F s2 = o->y; FF(mul)(&s2, &s->z); FF(mul)(&s2, &z1z1);
    if (FF(eq)(&s->x, &u2) && FF(eq)(&s->y, &s2)) {
        CF(double)(s);
        return;
    }
    F h = u2; FF(sub)(&h, &s->x);
    F hh = h; FF(square)(&hh);
    F i = hh; FF(double)(&i); FF(double)(&i);
    F j = h; FF(mul)(&j, &i);
    F r = s2; FF(sub)(&r, &s->y); FF(double)(&r);
    F v = s->x; FF(mul)(&v, &i);
    s->x = r; FF(square)(&s->x); FF(sub)(&s->x, &j); FF(sub)(&s->x, &v); FF(sub)(&s->x, &v);
    FF(mul)(&j, &s->y); FF(double)(&j);
    s->y = v; FF(sub)(&s->y, &s->x); FF(mul)(&s->y, &r); FF(sub)(&s->y, &j);
    FF(add)(&s->z, &h); FF(square)(&s->z); FF(sub)(&s->z, &z1z1); FF(sub)(&s->z, &hh);
}

void CF(negate)(PROJ *p) {                                            /* ec.rs:528-532 */
    if (!CF(is_zero)(p)) FF(negate)(&p->y);
}
void CF(sub)(PROJ *s, const PROJ *o) {                                /* lib.rs:156-160 */
    PROJ t = *o;
    CF(negate)(&t);
    CF(add)(s, &t);
}

/* mul_assign, ec.rs:534-553: MSB-first double-and-add over the 256-bit FrRepr. */
void CF(mul_assign)(PROJ *p, const uint64_t scalar[4]) {
    PROJ res = CF(zero)();
    int found_one = 0;
    for (int bit = 255; bit >= 0; bit--) {
        int i = (int)((scalar[bit / 64] >> (bit % 64)) & 1);
        if (found_one) CF(double)(&res);
        else found_one = i;
        if (i) CF(add)(&res, p);
    }
    *p = res;
}

PROJ CF(from_affine)(const AFF *a) {                                  /* ec.rs:570-582 */
    if (a->infinity) return CF(zero)();
    PROJ r;
    r.x = a->x;
    r.y = a->y;
    r.z = FF(one)();
    return r;
}

AFF CF(into_affine)(const PROJ *p) {                                  /* ec.rs:586-619 */
    AFF a;
    memset(&a, 0, sizeof a);
    F one = FF(one)();
    if (CF(is_zero)(p)) return CF(affine_zero)();
    if (FF(eq)(&p->z, &one)) {
        a.x = p->x;
        a.y = p->y;
        return a;
    }
    F zinv;
    FF(inverse)(&zinv, &p->z);
    F zp = zinv; FF(square)(&zp);
    a.x = p->x; FF(mul)(&a.x, &zp);
    FF(mul)(&zp, &zinv);
    a.y = p->y; FF(mul)(&a.y, &zp);
    return a;
}

/* mul_bits / CurveAffine::mul, ec.rs:88-95, 174-177 */
PROJ CF(affine_mul)(const AFF *a, const uint64_t scalar[4]) {
    PROJ res = CF(zero)();
    for (int bit = 255; bit >= 0; bit--) {
        CF(double)(&res);
        if ((scalar[bit / 64] >> (bit % 64)) & 1) CF(add_mixed)(&res, a);
    }
    return res;
}

int CF(is_on_curve)(const AFF *a) {                                   /* ec.rs:125-140 */
    if (a->infinity) return 1;
    F y2 = a->y; FF(square)(&y2);
    F x3b = a->x; FF(square)(&x3b); FF(mul)(&x3b, &a->x);
    F b; COEFF_B(&b);
    FF(add)(&x3b, &b);
    return FF(eq)(&y2, &x3b);
}

/* Montgomery's trick, ec.rs:246-294.  Zero and z==1 points are untouched. */
void CF(batch_normalization)(PROJ *v, size_t n) {
    F *prod = (F *)malloc(sizeof(F) * (n ? n : 1));
    size_t *idx = (size_t *)malloc(sizeof(size_t) * (n ? n : 1));
    size_t m = 0;
    F tmp = FF(one)();
    for (size_t k = 0; k < n; k++) {
        if (CF(is_normalized)(&v[k])) continue;
        FF(mul)(&tmp, &v[k].z);
        prod[m] = tmp;
        idx[m++] = k;
    }
    F inv;
    FF(inverse)(&inv, &tmp);
    tmp = inv;
    for (size_t t = m; t-- > 0;) {
        PROJ *g = &v[idx[t]];
        F s = (t == 0) ? FF(one)() : prod[t - 1];
        F newtmp = tmp; FF(mul)(&newtmp, &g->z);
        g->z = tmp; FF(mul)(&g->z, &s);
        tmp = newtmp;
    }
    for (size_t t = 0; t < m; t++) {
        PROJ *g = &v[idx[t]];
        F z = g->z; FF(square)(&z);
        FF(mul)(&g->x, &z);
        FF(mul)(&z, &g->z);
        FF(mul)(&g->y, &z);
        g->z = FF(one)();
    }
    free(prod);
    free(idx);
}

/* wnaf_table, wnaf.rs:4-15: [g, 3g, 5g, ...] of length 2^(w-1). */
void CF(wnaf_table)(PROJ *table, const PROJ *base, int window) {
    PROJ b = *base;
    PROJ dbl = b;
    CF(double)(&dbl);
    for (size_t k = 0; k < ((size_t)1 << (window - 1)); k++) {
        table[k] = b;
        CF(add)(&b, &dbl);
    }
}

/* wnaf_exp, wnaf.rs:49-71 */
PROJ CF(wnaf_exp)(const PROJ *table, const int64_t *wnaf, size_t len) {
    PROJ result = CF(zero)();
    int found_one = 0;
    for (size_t k = len; k-- > 0;) {
        int64_t nd = wnaf[k];
        if (found_one) CF(double)(&result);
        if (nd != 0) {
            found_one = 1;
            if (nd > 0) CF(add)(&result, &table[nd / 2]);
            else CF(sub)(&result, &table[(-nd) / 2]);
        }
    }
    return result;
}
