/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * The pairing engine restated from src/bls12_381/mod.rs:
 *   G2Prepared::from_affine   mod.rs:168-358 (doubling_step 176-245,
 *                                             addition_step 247-333)
 *   Bls12::miller_loop        mod.rs:40-102  (ell 57-69)
 *   final_exponentiation      mod.rs:104-160
 *   Engine::pairing           lib.rs:101-109
 * plus batch entry points (OpenMP over independent items) that serve as the
 * CPU baseline and as the checker for the GPU batch kernels.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"
#include "oracle_consts.h"
#include "oracle_internal.h"

o_g2 o_g2_from_affine(const o_g2_affine *a);
int o_g1_is_zero(const o_g1 *p);

/* doubling_step, mod.rs:176-245 (Algorithm 26 of eprint 2010/354) */
static o_ell_coeff doubling_step(o_g2 *r) {
    o_fq2 tmp0 = r->x; o_fq2_square(&tmp0);
    o_fq2 tmp1 = r->y; o_fq2_square(&tmp1);
    o_fq2 tmp2 = tmp1; o_fq2_square(&tmp2);
    o_fq2 tmp3 = tmp1; o_fq2_add(&tmp3, &r->x); o_fq2_square(&tmp3);
    o_fq2_sub(&tmp3, &tmp0); o_fq2_sub(&tmp3, &tmp2); o_fq2_double(&tmp3);
    o_fq2 tmp4 = tmp0; o_fq2_double(&tmp4); o_fq2_add(&tmp4, &tmp0);
    o_fq2 tmp6 = r->x; o_fq2_add(&tmp6, &tmp4);
    o_fq2 tmp5 = tmp4; o_fq2_square(&tmp5);
    o_fq2 zsquared = r->z; o_fq2_square(&zsquared);

    r->x = tmp5; o_fq2_sub(&r->x, &tmp3); o_fq2_sub(&r->x, &tmp3);
    o_fq2_add(&r->z, &r->y); o_fq2_square(&r->z); o_fq2_sub(&r->z, &tmp1); o_fq2_sub(&r->z, &zsquared);
    r->y = tmp3; o_fq2_sub(&r->y, &r->x); o_fq2_mul(&r->y, &tmp4);
    o_fq2_double(&tmp2); o_fq2_double(&tmp2); o_fq2_double(&tmp2);
    o_fq2_sub(&r->y, &tmp2);

    tmp3 = tmp4; o_fq2_mul(&tmp3, &zsquared); o_fq2_double(&tmp3); o_fq2_negate(&tmp3);
    o_fq2_square(&tmp6); o_fq2_sub(&tmp6, &tmp0); o_fq2_sub(&tmp6, &tmp5);
    o_fq2_double(&tmp1); o_fq2_double(&tmp1);
    o_fq2_sub(&tmp6, &tmp1);
    tmp0 = r->z; o_fq2_mul(&tmp0, &zsquared); o_fq2_double(&tmp0);

    o_ell_coeff c = {{tmp0, tmp3, tmp6}};
    return c;
}

/* addition_step, mod.rs:247-333 (Algorithm 27 of eprint 2010/354) */
static o_ell_coeff addition_step(o_g2 *r, const o_g2_affine *q) {
    o_fq2 zsquared = r->z; o_fq2_square(&zsquared);
    o_fq2 ysquared = q->y; o_fq2_square(&ysquared);
    o_fq2 t0 = zsquared; o_fq2_mul(&t0, &q->x);
    o_fq2 t1 = q->y; o_fq2_add(&t1, &r->z); o_fq2_square(&t1);
    o_fq2_sub(&t1, &ysquared); o_fq2_sub(&t1, &zsquared); o_fq2_mul(&t1, &zsquared);
    o_fq2 t2 = t0; o_fq2_sub(&t2, &r->x);
    o_fq2 t3 = t2; o_fq2_square(&t3);
    o_fq2 t4 = t3; o_fq2_double(&t4); o_fq2_double(&t4);
    o_fq2 t5 = t4; o_fq2_mul(&t5, &t2);
    o_fq2 t6 = t1; o_fq2_sub(&t6, &r->y); o_fq2_sub(&t6, &r->y);
    o_fq2 t9 = t6; o_fq2_mul(&t9, &q->x);
    o_fq2 t7 = t4; o_fq2_mul(&t7, &r->x);

    r->x = t6; o_fq2_square(&r->x); o_fq2_sub(&r->x, &t5); o_fq2_sub(&r->x, &t7); o_fq2_sub(&r->x, &t7);
    o_fq2_add(&r->z, &t2); o_fq2_square(&r->z); o_fq2_sub(&r->z, &zsquared); o_fq2_sub(&r->z, &t3);
    o_fq2 t10 = q->y; o_fq2_add(&t10, &r->z);
    o_fq2 t8 = t7; o_fq2_sub(&t8, &r->x); o_fq2_mul(&t8, &t6);
    t0 = r->y; o_fq2_mul(&t0, &t5); o_fq2_double(&t0);
    r->y = t8; o_fq2_sub(&r->y, &t0);

    o_fq2_square(&t10); o_fq2_sub(&t10, &ysquared);
    o_fq2 ztsquared = r->z; o_fq2_square(&ztsquared);
    o_fq2_sub(&t10, &ztsquared);
    o_fq2_double(&t9); o_fq2_sub(&t9, &t10);
    t10 = r->z; o_fq2_double(&t10);
    o_fq2_negate(&t6);
    t1 = t6; o_fq2_double(&t1);

    o_ell_coeff c = {{t10, t1, t9}};
    return c;
}

/* G2Prepared::from_affine, mod.rs:168-358 */
void o_g2_prepare(o_g2_prepared *out, const o_g2_affine *q) {
    memset(out, 0, sizeof *out);
    if (q->infinity) {
        out->infinity = 1;
        return;
    }
    o_g2 r = o_g2_from_affine(q);
    size_t n = 0;
    int found_one = 0;
    for (int bit = 63; bit >= 0; bit--) {                 /* BitIterator::new([BLS_X >> 1]) */
        int i = (int)(((O_BLS_X >> 1) >> bit) & 1);
        if (!found_one) {
            found_one = i;
            continue;
        }
        out->coeffs[n++] = doubling_step(&r);
        if (i) out->coeffs[n++] = addition_step(&r, q);
    }
    out->coeffs[n++] = doubling_step(&r);
    /* n == O_G2_PREPARED_COEFFS by construction of BLS_X (62 + 5 + 1) */
}

/* ell, mod.rs:57-69 */
static void ell(o_fq12 *f, const o_ell_coeff *coeffs, const o_g1_affine *p) {
    o_fq2 c0 = coeffs->c[0];
    o_fq2 c1 = coeffs->c[1];
    o_fq_mul(&c0.c0, &p->y);
    o_fq_mul(&c0.c1, &p->y);
    o_fq_mul(&c1.c0, &p->x);
    o_fq_mul(&c1.c1, &p->x);
    o_fq12_mul_by_014(f, &coeffs->c[2], &c1, &c0);
}

/* Bls12::miller_loop over n pairs (the product semantics), mod.rs:40-102.
 * Pairs with an infinity side are skipped (mod.rs:50-54). */
void o_miller_loop(o_fq12 *out, const o_g1_affine *ps, const o_g2_prepared *qs, size_t n) {
    size_t *live = (size_t *)malloc(sizeof(size_t) * (n ? n : 1));
    size_t m = 0;
    for (size_t k = 0; k < n; k++)
        if (!ps[k].infinity && !qs[k].infinity) live[m++] = k;
    size_t ci = 0;
    o_fq12 f = o_fq12_one();
    int found_one = 0;
    for (int bit = 63; bit >= 0; bit--) {
        int i = (int)(((O_BLS_X >> 1) >> bit) & 1);
        if (!found_one) {
            found_one = i;
            continue;
        }
        for (size_t t = 0; t < m; t++) ell(&f, &qs[live[t]].coeffs[ci], &ps[live[t]]);
        ci++;
        if (i) {
            for (size_t t = 0; t < m; t++) ell(&f, &qs[live[t]].coeffs[ci], &ps[live[t]]);
            ci++;
        }
        o_fq12_square(&f);
    }
    for (size_t t = 0; t < m; t++) ell(&f, &qs[live[t]].coeffs[ci], &ps[live[t]]);
    o_fq12_conjugate(&f);                                  /* BLS_X_IS_NEGATIVE */
    free(live);
    *out = f;
}

static void exp_by_x(o_fq12 *f, uint64_t x) {                               /* mod.rs:116-121 */
    o_fq12 t;
    o_fq12_pow(&t, f, &x, 1);
    *f = t;
    o_fq12_conjugate(f);
}

/* final_exponentiation, mod.rs:104-160.  Returns 0 (None) iff r == 0. */
int o_final_exponentiation(o_fq12 *out, const o_fq12 *r_in) {
    o_fq12 f1 = *r_in;
    o_fq12_conjugate(&f1);
    o_fq12 f2;
    if (!o_fq12_inverse(&f2, r_in)) return 0;
    o_fq12 r = f1;
    o_fq12_mul(&r, &f2);
    f2 = r;
    o_fq12_frobenius_map(&r, 2);
    o_fq12_mul(&r, &f2);

    uint64_t x = O_BLS_X;
    o_fq12 y0 = r; o_fq12_square(&y0);
    o_fq12 y1 = y0; exp_by_x(&y1, x);
    x >>= 1;
    o_fq12 y2 = y1; exp_by_x(&y2, x);
    x <<= 1;
    o_fq12 y3 = r; o_fq12_conjugate(&y3);
    o_fq12_mul(&y1, &y3);
    o_fq12_conjugate(&y1);
    o_fq12_mul(&y1, &y2);
    y2 = y1; exp_by_x(&y2, x);
    y3 = y2; exp_by_x(&y3, x);
    o_fq12_conjugate(&y1);
    o_fq12_mul(&y3, &y1);
    o_fq12_conjugate(&y1);
    o_fq12_frobenius_map(&y1, 3);
    o_fq12_frobenius_map(&y2, 2);
    o_fq12_mul(&y1, &y2);
    y2 = y3; exp_by_x(&y2, x);
    o_fq12_mul(&y2, &y0);
    o_fq12_mul(&y2, &r);
    o_fq12_mul(&y1, &y2);
    y2 = y3; o_fq12_frobenius_map(&y2, 1);
    o_fq12_mul(&y1, &y2);
    *out = y1;
    return 1;
}

/* Engine::pairing, lib.rs:101-109 */
void o_pairing(o_fq12 *out, const o_g1_affine *p, const o_g2_affine *q) {
    o_g2_prepared *prep = (o_g2_prepared *)malloc(sizeof(o_g2_prepared));
    o_g2_prepare(prep, q);
    o_fq12 f;
    o_miller_loop(&f, p, prep, 1);
    o_final_exponentiation(out, &f);
    free(prep);
}

/* ---- batch entry points: n independent items, OpenMP over items ---- */
#define NT(nthreads) num_threads((nthreads) > 0 ? (nthreads) : 1)

void o_pairing_batch(const o_g1_affine *p, const o_g2_affine *q, size_t n, o_fq12 *out, int nthreads) {
#pragma omp parallel for schedule(dynamic, 1) NT(nthreads)
    for (size_t k = 0; k < n; k++) o_pairing(&out[k], &p[k], &q[k]);
}
void o_g2_prepare_batch(const o_g2_affine *q, size_t n, o_g2_prepared *out, int nthreads) {
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) o_g2_prepare(&out[k], &q[k]);
}
/* independent single-pair Miller loops: out[k] = miller_loop([(p[k], q[k])]) */
void o_miller_loop_batch(const o_g1_affine *p, const o_g2_prepared *q, size_t n, o_fq12 *out, int nthreads) {
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) o_miller_loop(&out[k], &p[k], &q[k], 1);
}
void o_final_exponentiation_batch(const o_fq12 *in, size_t n, o_fq12 *out, uint8_t *ok, int nthreads) {
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) {
        int r = o_final_exponentiation(&out[k], &in[k]);
        if (!r) memset(&out[k], 0, sizeof(o_fq12));
        ok[k] = (uint8_t)r;
    }
}

/* ---- field batch helpers for the GPU parity tests ---- */
void o_fq_mul_batch(const o_fq *a, const o_fq *b, o_fq *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq t = a[k]; o_fq_mul(&t, &b[k]); out[k] = t; }
}
void o_fq_square_batch(const o_fq *a, o_fq *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq t = a[k]; o_fq_square(&t); out[k] = t; }
}
void o_fq_add_batch(const o_fq *a, const o_fq *b, o_fq *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq t = a[k]; o_fq_add(&t, &b[k]); out[k] = t; }
}
void o_fq_sub_batch(const o_fq *a, const o_fq *b, o_fq *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq t = a[k]; o_fq_sub(&t, &b[k]); out[k] = t; }
}
void o_fq_inverse_batch(const o_fq *a, o_fq *out, uint8_t *ok, size_t n) {
    for (size_t k = 0; k < n; k++) {
        ok[k] = (uint8_t)o_fq_inverse(&out[k], &a[k]);
        if (!ok[k]) memset(&out[k], 0, sizeof(o_fq));
    }
}
void o_fq2_mul_batch(const o_fq2 *a, const o_fq2 *b, o_fq2 *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq2 t = a[k]; o_fq2_mul(&t, &b[k]); out[k] = t; }
}
void o_fq2_square_batch(const o_fq2 *a, o_fq2 *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq2 t = a[k]; o_fq2_square(&t); out[k] = t; }
}
void o_fq6_mul_batch(const o_fq6 *a, const o_fq6 *b, o_fq6 *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq6 t = a[k]; o_fq6_mul(&t, &b[k]); out[k] = t; }
}
void o_fq12_mul_batch(const o_fq12 *a, const o_fq12 *b, o_fq12 *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq12 t = a[k]; o_fq12_mul(&t, &b[k]); out[k] = t; }
}
void o_fq12_square_batch(const o_fq12 *a, o_fq12 *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fq12 t = a[k]; o_fq12_square(&t); out[k] = t; }
}
void o_fq12_inverse_batch(const o_fq12 *a, o_fq12 *out, uint8_t *ok, size_t n) {
    for (size_t k = 0; k < n; k++) {
        ok[k] = (uint8_t)o_fq12_inverse(&out[k], &a[k]);
        if (!ok[k]) memset(&out[k], 0, sizeof(o_fq12));
    }
}
void o_fq12_frobenius_batch(const o_fq12 *a, o_fq12 *out, size_t n, size_t power) {
    for (size_t k = 0; k < n; k++) { o_fq12 t = a[k]; o_fq12_frobenius_map(&t, power); out[k] = t; }
}
void o_fq12_mul_by_014_batch(const o_fq12 *a, const o_fq2 *c0, const o_fq2 *c1, const o_fq2 *c4,
                             o_fq12 *out, size_t n) {
    for (size_t k = 0; k < n; k++) {
        o_fq12 t = a[k];
        o_fq12_mul_by_014(&t, &c0[k], &c1[k], &c4[k]);
        out[k] = t;
    }
}
void o_fq12_pow_batch(const o_fq12 *a, const uint64_t *exp, size_t exp_limbs, o_fq12 *out, size_t n) {
    for (size_t k = 0; k < n; k++) o_fq12_pow(&out[k], &a[k], exp, exp_limbs);
}
