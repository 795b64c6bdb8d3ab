/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * Batch wrappers over the curve restatement, exported for the Python test
 * harness (ctypes).  Each loops the single-item reference routine.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"
#include "oracle_consts.h"
#include "oracle_internal.h"

o_g1 o_g1_from_affine(const o_g1_affine *a);
o_g1_affine o_g1_into_affine(const o_g1 *p);
void o_g1_mul_assign(o_g1 *p, const uint64_t scalar[4]);
void o_g1_double(o_g1 *p);
void o_g1_add(o_g1 *s, const o_g1 *o);
void o_g1_add_mixed(o_g1 *s, const o_g1_affine *o);
void o_g1_batch_normalization(o_g1 *v, size_t n);
int o_g1_eq(const o_g1 *a, const o_g1 *b);
o_g1_affine o_g1_generator(void);
o_g2 o_g2_from_affine(const o_g2_affine *a);
o_g2_affine o_g2_into_affine(const o_g2 *p);
void o_g2_mul_assign(o_g2 *p, const uint64_t scalar[4]);
void o_g2_double(o_g2 *p);
void o_g2_add(o_g2 *s, const o_g2 *o);
void o_g2_add_mixed(o_g2 *s, const o_g2_affine *o);
void o_g2_batch_normalization(o_g2 *v, size_t n);
int o_g2_eq(const o_g2 *a, const o_g2 *b);
o_g2_affine o_g2_generator(void);

#define NT(nthreads) num_threads((nthreads) > 0 ? (nthreads) : 1)

/* k*G as affine points (G::one().mul_assign(k).into_affine()). */
void o_g1_mul_generator_batch(const uint64_t *scalars, size_t n, o_g1_affine *out, int nthreads) {
    o_g1_affine g = o_g1_generator();
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) {
        o_g1 p = o_g1_from_affine(&g);
        o_g1_mul_assign(&p, &scalars[4 * k]);
        out[k] = o_g1_into_affine(&p);
    }
}
void o_g2_mul_generator_batch(const uint64_t *scalars, size_t n, o_g2_affine *out, int nthreads) {
    o_g2_affine g = o_g2_generator();
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) {
        o_g2 p = o_g2_from_affine(&g);
        o_g2_mul_assign(&p, &scalars[4 * k]);
        out[k] = o_g2_into_affine(&p);
    }
}
/* Jacobian k*G (not normalized), for batch_normalization / wNAF inputs. */
void o_g1_mul_generator_jacobian_batch(const uint64_t *scalars, size_t n, o_g1 *out, int nthreads) {
    o_g1_affine g = o_g1_generator();
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) {
        o_g1 p = o_g1_from_affine(&g);
        o_g1_mul_assign(&p, &scalars[4 * k]);
        out[k] = p;
    }
}
void o_g1_mul_batch(const o_g1 *p, const uint64_t *scalars, size_t n, o_g1 *out) {
    for (size_t k = 0; k < n; k++) { o_g1 t = p[k]; o_g1_mul_assign(&t, &scalars[4 * k]); out[k] = t; }
}
void o_g2_mul_batch(const o_g2 *p, const uint64_t *scalars, size_t n, o_g2 *out) {
    for (size_t k = 0; k < n; k++) { o_g2 t = p[k]; o_g2_mul_assign(&t, &scalars[4 * k]); out[k] = t; }
}
void o_g1_double_batch(const o_g1 *p, size_t n, o_g1 *out) {
    for (size_t k = 0; k < n; k++) { o_g1 t = p[k]; o_g1_double(&t); out[k] = t; }
}
void o_g2_double_batch(const o_g2 *p, size_t n, o_g2 *out) {
    for (size_t k = 0; k < n; k++) { o_g2 t = p[k]; o_g2_double(&t); out[k] = t; }
}
void o_g1_add_batch(const o_g1 *a, const o_g1 *b, size_t n, o_g1 *out) {
    for (size_t k = 0; k < n; k++) { o_g1 t = a[k]; o_g1_add(&t, &b[k]); out[k] = t; }
}
void o_g2_add_batch(const o_g2 *a, const o_g2 *b, size_t n, o_g2 *out) {
    for (size_t k = 0; k < n; k++) { o_g2 t = a[k]; o_g2_add(&t, &b[k]); out[k] = t; }
}
void o_g1_add_mixed_batch(const o_g1 *a, const o_g1_affine *b, size_t n, o_g1 *out) {
    for (size_t k = 0; k < n; k++) { o_g1 t = a[k]; o_g1_add_mixed(&t, &b[k]); out[k] = t; }
}
void o_g2_add_mixed_batch(const o_g2 *a, const o_g2_affine *b, size_t n, o_g2 *out) {
    for (size_t k = 0; k < n; k++) { o_g2 t = a[k]; o_g2_add_mixed(&t, &b[k]); out[k] = t; }
}
void o_g1_into_affine_batch(const o_g1 *p, size_t n, o_g1_affine *out) {
    for (size_t k = 0; k < n; k++) out[k] = o_g1_into_affine(&p[k]);
}
void o_g2_into_affine_batch(const o_g2 *p, size_t n, o_g2_affine *out) {
    for (size_t k = 0; k < n; k++) out[k] = o_g2_into_affine(&p[k]);
}
void o_g1_from_affine_batch(const o_g1_affine *a, size_t n, o_g1 *out) {
    for (size_t k = 0; k < n; k++) out[k] = o_g1_from_affine(&a[k]);
}
void o_g2_from_affine_batch(const o_g2_affine *a, size_t n, o_g2 *out) {
    for (size_t k = 0; k < n; k++) out[k] = o_g2_from_affine(&a[k]);
}
void o_g1_eq_batch(const o_g1 *a, const o_g1 *b, size_t n, uint8_t *out) {
    for (size_t k = 0; k < n; k++) out[k] = (uint8_t)o_g1_eq(&a[k], &b[k]);
}
void o_g2_eq_batch(const o_g2 *a, const o_g2 *b, size_t n, uint8_t *out) {
    for (size_t k = 0; k < n; k++) out[k] = (uint8_t)o_g2_eq(&a[k], &b[k]);
}
void o_fq_from_repr_batch(const uint64_t *repr, size_t n, o_fq *out, uint8_t *ok) {
    for (size_t k = 0; k < n; k++) {
        ok[k] = (uint8_t)o_fq_from_repr(&out[k], &repr[6 * k]);
        if (!ok[k]) memset(&out[k], 0, sizeof(o_fq));
    }
}
void o_fq_into_repr_batch(const o_fq *a, size_t n, uint64_t *out) {
    for (size_t k = 0; k < n; k++) o_fq_into_repr(&out[6 * k], &a[k]);
}
size_t o_sizeof(int which) {
    switch (which) {
        case 0: return sizeof(o_fq);
        case 1: return sizeof(o_fq2);
        case 2: return sizeof(o_fq6);
        case 3: return sizeof(o_fq12);
        case 4: return sizeof(o_g1_affine);
        case 5: return sizeof(o_g1);
        case 6: return sizeof(o_g2_affine);
        case 7: return sizeof(o_g2);
        case 8: return sizeof(o_g2_prepared);
        default: return 0;
    }
}

/* CurveAffine::mul (ec.rs:174-177 -> mul_bits ec.rs:88-95), Jacobian out. */
void o_g1_affine_mul_batch(const o_g1_affine *p, const uint64_t *scalars, size_t n, o_g1 *out, int nthreads) {
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) out[k] = o_g1_affine_mul(&p[k], &scalars[4 * k]);
}
void o_g2_affine_mul_batch(const o_g2_affine *p, const uint64_t *scalars, size_t n, o_g2 *out, int nthreads) {
#pragma omp parallel for schedule(dynamic, 4) NT(nthreads)
    for (size_t k = 0; k < n; k++) out[k] = o_g2_affine_mul(&p[k], &scalars[4 * k]);
}
/* sum_i s_i * P_i the way a caller of the reference writes it: CurveAffine::mul
 * per term, then add_assign (ec.rs:356-444) in index order.  The terms are
 * computed in parallel; the sum is serial, so the result does not depend on
 * the thread count. */
void o_g1_multiexp(const o_g1_affine *p, const uint64_t *scalars, size_t n, o_g1 *out, int nthreads) {
    o_g1 *t = (o_g1 *)malloc(sizeof(o_g1) * (n ? n : 1));
    o_g1_affine_mul_batch(p, scalars, n, t, nthreads);
    o_g1 acc = t[0];
    if (n == 0) { o_g1_affine z = o_g1_affine_zero(); acc = o_g1_from_affine(&z); }
    for (size_t k = 1; k < n; k++) o_g1_add(&acc, &t[k]);
    *out = acc;
    free(t);
}
void o_g2_multiexp(const o_g2_affine *p, const uint64_t *scalars, size_t n, o_g2 *out, int nthreads) {
    o_g2 *t = (o_g2 *)malloc(sizeof(o_g2) * (n ? n : 1));
    o_g2_affine_mul_batch(p, scalars, n, t, nthreads);
    o_g2 acc = t[0];
    if (n == 0) { o_g2_affine z = o_g2_affine_zero(); acc = o_g2_from_affine(&z); }
    for (size_t k = 1; k < n; k++) o_g2_add(&acc, &t[k]);
    *out = acc;
    free(t);
}
