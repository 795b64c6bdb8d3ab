/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * G1 / G2 instantiations of the Jacobian group law (ec.rs:623-643 and
 * 1270-1290 instantiate `curve_impl!`), the wNAF recoding (wnaf.rs:18-43),
 * the window heuristics (ec.rs:894-921, 1585-1613) and the point encodings
 * used by the reference's `.dat` vectors (ec.rs:737-752, 839-867,
 * 1398-1415, 1510-1539; wire format src/bls12_381/README.md "Serialization").
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"
#include "oracle_consts.h"
#include "oracle_internal.h"

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)

/* ---- G1 over Fq ---- */
static void g1_coeff_b(o_fq *b) { memcpy(b->l, O_FQ_B_COEFF, 48); }     /* ec.rs:885-887 */
#define PROJ o_g1
#define AFF o_g1_affine
#define F o_fq
#define CF(name) CAT(o_g1_, name)
#define FF(name) CAT(o_fq_, name)
#define COEFF_B g1_coeff_b
#include "oracle_curve_impl.h"
#undef PROJ
#undef AFF
#undef F
#undef CF
#undef FF
#undef COEFF_B

/* ---- G2 over Fq2 ---- */
static void g2_coeff_b(o_fq2 *b) {                                       /* ec.rs:1557-1562 */
    memcpy(b->c0.l, O_FQ_B_COEFF, 48);
    memcpy(b->c1.l, O_FQ_B_COEFF, 48);
}
#define PROJ o_g2
#define AFF o_g2_affine
#define F o_fq2
#define CF(name) CAT(o_g2_, name)
#define FF(name) CAT(o_fq2_, name)
#define COEFF_B g2_coeff_b
#include "oracle_curve_impl.h"
#undef PROJ
#undef AFF
#undef F
#undef CF
#undef FF
#undef COEFF_B

o_g1_affine o_g1_generator(void) {                                       /* ec.rs:877-883 */
    o_g1_affine a;
    memset(&a, 0, sizeof a);
    memcpy(a.x.l, O_FQ_G1_X, 48);
    memcpy(a.y.l, O_FQ_G1_Y, 48);
    return a;
}
o_g2_affine o_g2_generator(void) {                                       /* ec.rs:1543-1555 */
    o_g2_affine a;
    memset(&a, 0, sizeof a);
    memcpy(a.x.c0.l, O_FQ_G2_X_C0, 48);
    memcpy(a.x.c1.l, O_FQ_G2_X_C1, 48);
    memcpy(a.y.c0.l, O_FQ_G2_Y_C0, 48);
    memcpy(a.y.c1.l, O_FQ_G2_Y_C1, 48);
    return a;
}

/* wnaf_form, wnaf.rs:18-43, on a 4-limb FrRepr.  Returns the digit count. */
size_t o_wnaf_form(int64_t *wnaf, const uint64_t scalar[4], int window) {
    uint64_t c[4];
    memcpy(c, scalar, 32);
    size_t len = 0;
    while (!o_repr_is_zero(c, 4)) {
        int64_t u;
        if (c[0] & 1) {
            u = (int64_t)(c[0] % ((uint64_t)1 << (window + 1)));
            if (u > ((int64_t)1 << window)) u -= (int64_t)1 << (window + 1);
            uint64_t t[4] = {0, 0, 0, 0};
            if (u > 0) {
                t[0] = (uint64_t)u;
                o_repr_sub_noborrow(c, t, 4);
            } else {
                t[0] = (uint64_t)(-u);
                o_repr_add_nocarry(c, t, 4);
            }
        } else {
            u = 0;
        }
        wnaf[len++] = u;
        o_repr_div2(c, 4);
    }
    return len;
}

static int num_bits4(const uint64_t s[4]) {                              /* fr.rs num_bits */
    int ret = 256;
    for (int i = 3; i >= 0; i--) {
        int lead = s[i] ? __builtin_clzll(s[i]) : 64;
        ret -= lead;
        if (lead != 64) break;
    }
    return ret;
}
int o_g1_recommended_wnaf_for_scalar(const uint64_t s[4]) {              /* ec.rs:895-905 */
    int nb = num_bits4(s);
    return nb >= 130 ? 4 : (nb >= 34 ? 3 : 2);
}
int o_g2_recommended_wnaf_for_scalar(const uint64_t s[4]) {              /* ec.rs:1586-1596 */
    int nb = num_bits4(s);
    return nb >= 103 ? 4 : (nb >= 37 ? 3 : 2);
}
static int recommend_num(size_t n, const size_t *rec, int cnt) {
    int ret = 4;
    for (int i = 0; i < cnt; i++) {
        if (n > rec[i]) ret++;
        else break;
    }
    return ret;
}
int o_g1_recommended_wnaf_for_num_scalars(size_t n) {                    /* ec.rs:907-921 */
    static const size_t rec[12] = {1, 3, 7, 20, 43, 120, 273, 563, 1630, 3128, 7933, 62569};
    return recommend_num(n, rec, 12);
}
int o_g2_recommended_wnaf_for_num_scalars(size_t n) {                    /* ec.rs:1598-1612 */
    static const size_t rec[11] = {1, 3, 8, 20, 47, 126, 260, 826, 1501, 4555, 84071};
    return recommend_num(n, rec, 11);
}

void o_g1_wnaf_fixed_base_w(const o_g1 *base, const uint64_t *scalars, size_t n, int w, o_g1 *out, int nthreads);
void o_g2_wnaf_fixed_base_w(const o_g2 *base, const uint64_t *scalars, size_t n, int w, o_g2 *out, int nthreads);

/* Wnaf::new().base(g, num_scalars) then .scalar(s) per scalar (wnaf.rs:93-107,
 * 169-178): one shared table, one wNAF per scalar.  OpenMP over scalars is
 * what `Wnaf::shared()` (wnaf.rs:131-141) exists for. */
void o_g1_wnaf_fixed_base(const o_g1 *base, const uint64_t *scalars, size_t n, o_g1 *out, int nthreads) {
    o_g1_wnaf_fixed_base_w(base, scalars, n, o_g1_recommended_wnaf_for_num_scalars(n), out, nthreads);
}
void o_g2_wnaf_fixed_base(const o_g2 *base, const uint64_t *scalars, size_t n, o_g2 *out, int nthreads) {
    o_g2_wnaf_fixed_base_w(base, scalars, n, o_g2_recommended_wnaf_for_num_scalars(n), out, nthreads);
}
/* the same with the window given: Wnaf::new().base(g, num_scalars) fixes the
 * window from num_scalars, and its shared() copies multiply any count */
void o_g1_wnaf_fixed_base_w(const o_g1 *base, const uint64_t *scalars, size_t n, int w, o_g1 *out, int nthreads) {
    o_g1 *table = (o_g1 *)malloc(sizeof(o_g1) * ((size_t)1 << (w - 1)));
    o_g1_wnaf_table(table, base, w);
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
    for (size_t k = 0; k < n; k++) {
        int64_t digits[300];
        size_t len = o_wnaf_form(digits, &scalars[4 * k], w);
        out[k] = o_g1_wnaf_exp(table, digits, len);
    }
    free(table);
}
void o_g2_wnaf_fixed_base_w(const o_g2 *base, const uint64_t *scalars, size_t n, int w, o_g2 *out, int nthreads) {
    o_g2 *table = (o_g2 *)malloc(sizeof(o_g2) * ((size_t)1 << (w - 1)));
    o_g2_wnaf_table(table, base, w);
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
    for (size_t k = 0; k < n; k++) {
        int64_t digits[300];
        size_t len = o_wnaf_form(digits, &scalars[4 * k], w);
        out[k] = o_g2_wnaf_exp(table, digits, len);
    }
    free(table);
}

/* Wnaf::new().scalar(s) then .base(g) per base (wnaf.rs:111-128, 156-165):
 * the window is recommended_wnaf_for_scalar(s), one wNAF form, a table per base */
void o_g1_wnaf_fixed_scalar(const o_g1 *bases, const uint64_t scalar[4], size_t n, o_g1 *out, int nthreads) {
    int w = o_g1_recommended_wnaf_for_scalar(scalar);
    int64_t digits[300];
    size_t len = o_wnaf_form(digits, scalar, w);
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads > 0 ? nthreads : 1)
    for (size_t k = 0; k < n; k++) {
        o_g1 table[8];
        o_g1_wnaf_table(table, &bases[k], w);
        out[k] = o_g1_wnaf_exp(table, digits, len);
    }
}
void o_g2_wnaf_fixed_scalar(const o_g2 *bases, const uint64_t scalar[4], size_t n, o_g2 *out, int nthreads) {
    int w = o_g2_recommended_wnaf_for_scalar(scalar);
    int64_t digits[300];
    size_t len = o_wnaf_form(digits, scalar, w);
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads > 0 ? nthreads : 1)
    for (size_t k = 0; k < n; k++) {
        o_g2 table[8];
        o_g2_wnaf_table(table, &bases[k], w);
        out[k] = o_g2_wnaf_exp(table, digits, len);
    }
}

/* ---- encodings (README.md "Serialization") ---- */
static void write_be_fq(uint8_t *dst, const o_fq *a) {                   /* into_repr().write_be */
    uint64_t r[6];
    o_fq_into_repr(r, a);
    for (int i = 0; i < 6; i++) {
        uint64_t w = r[5 - i];
        for (int b = 0; b < 8; b++) dst[8 * i + b] = (uint8_t)(w >> (56 - 8 * b));
    }
}
void o_g1_encode_uncompressed(uint8_t out[96], const o_g1_affine *a) {   /* ec.rs:737-752 */
    memset(out, 0, 96);
    if (a->infinity) { out[0] |= 1 << 6; return; }
    write_be_fq(out, &a->x);
    write_be_fq(out + 48, &a->y);
}
void o_g1_encode_compressed(uint8_t out[48], const o_g1_affine *a) {     /* ec.rs:839-867 */
    memset(out, 0, 48);
    if (a->infinity) {
        out[0] |= 1 << 6;
    } else {
        write_be_fq(out, &a->x);
        o_fq negy = a->y;
        o_fq_negate(&negy);
        if (o_fq_cmp(&a->y, &negy) > 0) out[0] |= 1 << 5;
    }
    out[0] |= 1 << 7;
}
void o_g2_encode_uncompressed(uint8_t out[192], const o_g2_affine *a) {  /* ec.rs:1398-1415 */
    memset(out, 0, 192);
    if (a->infinity) { out[0] |= 1 << 6; return; }
    write_be_fq(out, &a->x.c1);
    write_be_fq(out + 48, &a->x.c0);
    write_be_fq(out + 96, &a->y.c1);
    write_be_fq(out + 144, &a->y.c0);
}
void o_g2_encode_compressed(uint8_t out[96], const o_g2_affine *a) {     /* ec.rs:1510-1539 */
    memset(out, 0, 96);
    if (a->infinity) {
        out[0] |= 1 << 6;
    } else {
        write_be_fq(out, &a->x.c1);
        write_be_fq(out + 48, &a->x.c0);
        o_fq2 negy = a->y;
        o_fq2_negate(&negy);
        if (o_fq2_cmp(&a->y, &negy) > 0) out[0] |= 1 << 5;
    }
    out[0] |= 1 << 7;
}

/* The `.dat` vector generator of bls12_381/tests/mod.rs:55-77: record k is the
 * encoding of k*G built by repeated add_assign(G::one()) and into_affine. */
void o_g1_kg_vectors(uint8_t *out, size_t count, int compressed) {
    o_g1_affine g = o_g1_generator();
    o_g1 one = o_g1_from_affine(&g);
    o_g1 e = o_g1_zero();
    size_t sz = compressed ? 48 : 96;
    for (size_t k = 0; k < count; k++) {
        o_g1_affine a = o_g1_into_affine(&e);
        if (compressed) o_g1_encode_compressed(out + k * sz, &a);
        else o_g1_encode_uncompressed(out + k * sz, &a);
        o_g1_add(&e, &one);
    }
}
void o_g2_kg_vectors(uint8_t *out, size_t count, int compressed) {
    o_g2_affine g = o_g2_generator();
    o_g2 one = o_g2_from_affine(&g);
    o_g2 e = o_g2_zero();
    size_t sz = compressed ? 96 : 192;
    for (size_t k = 0; k < count; k++) {
        o_g2_affine a = o_g2_into_affine(&e);
        if (compressed) o_g2_encode_compressed(out + k * sz, &a);
        else o_g2_encode_uncompressed(out + k * sz, &a);
        o_g2_add(&e, &one);
    }
}
