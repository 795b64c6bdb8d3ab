/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * Fq / Fq2 / Fq6 / Fq12 restated from the reference crate:
 *   limb arithmetic      src/lib.rs:645-679 (u128-support variant)
 *   FqRepr               src/bls12_381/fq.rs:554-697
 *   Fq                   src/bls12_381/fq.rs:744-1122
 *   Fq2                  src/bls12_381/fq2.rs:39-160
 *   Fq6                  src/bls12_381/fq6.rs:30-302
 *   Fq12                 src/bls12_381/fq12.rs:29-149
 *   Field::pow           src/lib.rs:306-324
 */
#include <string.h>
#include "oracle.h"
#include "oracle_consts.h"
#include "oracle_internal.h"

typedef unsigned __int128 u128;

/* ---- L0 limb arithmetic: lib.rs:650-678 ---- */
static inline uint64_t sbb(uint64_t a, uint64_t b, uint64_t *borrow) {
    u128 tmp = ((u128)1 << 64) + (u128)a - (u128)b - (u128)(*borrow);
    *borrow = (tmp >> 64) == 0 ? 1 : 0;
    return (uint64_t)tmp;
}
static inline uint64_t adc(uint64_t a, uint64_t b, uint64_t *carry) {
    u128 tmp = (u128)a + (u128)b + (u128)(*carry);
    *carry = (uint64_t)(tmp >> 64);
    return (uint64_t)tmp;
}
static inline uint64_t mac_with_carry(uint64_t a, uint64_t b, uint64_t c, uint64_t *carry) {
    u128 tmp = (u128)a + (u128)b * (u128)c + (u128)(*carry);
    *carry = (uint64_t)(tmp >> 64);
    return (uint64_t)tmp;
}

/* ---- FqRepr: fq.rs:554-697 (generic over limb count n) ---- */
int o_repr_cmp(const uint64_t *a, const uint64_t *b, int n) {   /* fq.rs:554-567 */
    for (int i = n - 1; i >= 0; i--) {
        if (a[i] < b[i]) return -1;
        if (a[i] > b[i]) return 1;
    }
    return 0;
}
int o_repr_is_zero(const uint64_t *a, int n) {                  /* fq.rs:587-590 */
    for (int i = 0; i < n; i++) if (a[i]) return 0;
    return 1;
}
void o_repr_div2(uint64_t *a, int n) {                          /* fq.rs:619-627 */
    uint64_t t = 0;
    for (int i = n - 1; i >= 0; i--) {
        uint64_t t2 = a[i] << 63;
        a[i] >>= 1;
        a[i] |= t;
        t = t2;
    }
}
static void repr_mul2(uint64_t *a, int n) {                     /* fq.rs:630-638 */
    uint64_t last = 0;
    for (int i = 0; i < n; i++) {
        uint64_t tmp = a[i] >> 63;
        a[i] <<= 1;
        a[i] |= last;
        last = tmp;
    }
}
void o_repr_add_nocarry(uint64_t *a, const uint64_t *b, int n) { /* fq.rs:681-687 */
    uint64_t carry = 0;
    for (int i = 0; i < n; i++) a[i] = adc(a[i], b[i], &carry);
}
void o_repr_sub_noborrow(uint64_t *a, const uint64_t *b, int n) { /* fq.rs:690-696 */
    uint64_t borrow = 0;
    for (int i = 0; i < n; i++) a[i] = sbb(a[i], b[i], &borrow);
}

/* ---- Fq: fq.rs:796-1122 ---- */
static const o_fq FQ_ZERO = {{0, 0, 0, 0, 0, 0}};

o_fq o_fq_zero(void) { return FQ_ZERO; }
o_fq o_fq_one(void) { o_fq r; memcpy(r.l, O_FQ_R, 48); return r; }          /* fq.rs:803-805 */
int o_fq_is_zero(const o_fq *a) { return o_repr_is_zero(a->l, 6); }
int o_fq_eq(const o_fq *a, const o_fq *b) { return memcmp(a->l, b->l, 48) == 0; }

static inline int fq_is_valid(const o_fq *a) { return o_repr_cmp(a->l, O_FQ_MODULUS, 6) < 0; } /* fq.rs:1023-1025 */
static inline void fq_reduce(o_fq *a) {                                       /* fq.rs:1029-1034 */
    if (!fq_is_valid(a)) o_repr_sub_noborrow(a->l, O_FQ_MODULUS, 6);
}
void o_fq_add(o_fq *a, const o_fq *b) {                                       /* fq.rs:812-819 */
    o_repr_add_nocarry(a->l, b->l, 6);
    fq_reduce(a);
}
void o_fq_double(o_fq *a) {                                                   /* fq.rs:821-828 */
    repr_mul2(a->l, 6);
    fq_reduce(a);
}
void o_fq_sub(o_fq *a, const o_fq *b) {                                       /* fq.rs:830-838 */
    if (o_repr_cmp(b->l, a->l, 6) > 0) o_repr_add_nocarry(a->l, O_FQ_MODULUS, 6);
    o_repr_sub_noborrow(a->l, b->l, 6);
}
void o_fq_negate(o_fq *a) {                                                   /* fq.rs:840-847 */
    if (!o_fq_is_zero(a)) {
        uint64_t tmp[6];
        memcpy(tmp, O_FQ_MODULUS, 48);
        o_repr_sub_noborrow(tmp, a->l, 6);
        memcpy(a->l, tmp, 48);
    }
}

/* mont_reduce: fq.rs:1036-1122 (HAC 14.32), written as the loop it unrolls. */
static void fq_mont_reduce(o_fq *out, uint64_t r[12]) {
    uint64_t carry2 = 0;
    for (int i = 0; i < 6; i++) {
        uint64_t k = r[i] * O_FQ_INV64;
        uint64_t carry = 0;
        mac_with_carry(r[i], k, O_FQ_MODULUS[0], &carry);
        for (int j = 1; j < 6; j++) r[i + j] = mac_with_carry(r[i + j], k, O_FQ_MODULUS[j], &carry);
        r[i + 6] = adc(r[i + 6], carry2, &carry);
        carry2 = carry;
    }
    memcpy(out->l, &r[6], 48);
    fq_reduce(out);
}

void o_fq_mul(o_fq *a, const o_fq *b) {                                       /* fq.rs:909-960 */
    uint64_t r[12];
    memset(r, 0, sizeof r);
    for (int i = 0; i < 6; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 6; j++) r[i + j] = mac_with_carry(r[i + j], a->l[i], b->l[j], &carry);
        r[i + 6] = carry;
    }
    fq_mont_reduce(a, r);
}

void o_fq_square(o_fq *a) {                                                   /* fq.rs:962-1016 */
    uint64_t r[12];
    memset(r, 0, sizeof r);
    /* off-diagonal products */
    for (int i = 0; i < 5; i++) {
        uint64_t carry = 0;
        for (int j = i + 1; j < 6; j++) r[i + j] = mac_with_carry(r[i + j], a->l[i], a->l[j], &carry);
        r[i + 6] = carry;
    }
    /* double them (fq.rs:990-1000) */
    r[11] = r[10] >> 63;
    for (int k = 10; k >= 2; k--) r[k] = (r[k] << 1) | (r[k - 1] >> 63);
    r[1] = r[1] << 1;
    /* add the diagonal (fq.rs:1002-1014) */
    uint64_t carry = 0;
    r[0] = mac_with_carry(0, a->l[0], a->l[0], &carry);
    r[1] = adc(r[1], 0, &carry);
    for (int i = 1; i < 6; i++) {
        r[2 * i] = mac_with_carry(r[2 * i], a->l[i], a->l[i], &carry);
        r[2 * i + 1] = adc(r[2 * i + 1], 0, &carry);
    }
    fq_mont_reduce(a, r);
}

/* Binary extended Euclid, fq.rs:849-902.  Returns 0 (None) for zero. */
int o_fq_inverse(o_fq *out, const o_fq *a) {
    if (o_fq_is_zero(a)) return 0;
    uint64_t one[6] = {1, 0, 0, 0, 0, 0};
    uint64_t u[6], v[6];
    o_fq b, c;
    memcpy(u, a->l, 48);
    memcpy(v, O_FQ_MODULUS, 48);
    memcpy(b.l, O_FQ_R2, 48);
    c = FQ_ZERO;
    while (memcmp(u, one, 48) != 0 && memcmp(v, one, 48) != 0) {
        while ((u[0] & 1) == 0) {
            o_repr_div2(u, 6);
            if ((b.l[0] & 1) == 0) {
                o_repr_div2(b.l, 6);
            } else {
                o_repr_add_nocarry(b.l, O_FQ_MODULUS, 6);
                o_repr_div2(b.l, 6);
            }
        }
        while ((v[0] & 1) == 0) {
            o_repr_div2(v, 6);
            if ((c.l[0] & 1) == 0) {
                o_repr_div2(c.l, 6);
            } else {
                o_repr_add_nocarry(c.l, O_FQ_MODULUS, 6);
                o_repr_div2(c.l, 6);
            }
        }
        if (o_repr_cmp(v, u, 6) < 0) {
            o_repr_sub_noborrow(u, v, 6);
            o_fq_sub(&b, &c);
        } else {
            o_repr_sub_noborrow(v, u, 6);
            o_fq_sub(&c, &b);
        }
    }
    *out = (memcmp(u, one, 48) == 0) ? b : c;
    return 1;
}

/* from_repr / into_repr: fq.rs:747-775 */
int o_fq_from_repr(o_fq *out, const uint64_t repr[6]) {
    o_fq r;
    memcpy(r.l, repr, 48);
    if (!fq_is_valid(&r)) return 0;
    o_fq r2;
    memcpy(r2.l, O_FQ_R2, 48);
    o_fq_mul(&r, &r2);
    *out = r;
    return 1;
}
void o_fq_into_repr(uint64_t out[6], const o_fq *a) {
    uint64_t r[12];
    memcpy(r, a->l, 48);
    memset(&r[6], 0, 48);
    o_fq t;
    fq_mont_reduce(&t, r);
    memcpy(out, t.l, 48);
}
/* Fq ordering (fq.rs:703-708): lexicographic on the canonical repr. */
int o_fq_cmp(const o_fq *a, const o_fq *b) {
    uint64_t ra[6], rb[6];
    o_fq_into_repr(ra, a);
    o_fq_into_repr(rb, b);
    return o_repr_cmp(ra, rb, 6);
}

/* ---- Fq2: fq2.rs:39-160 ---- */
o_fq2 o_fq2_zero(void) { o_fq2 r = {FQ_ZERO, FQ_ZERO}; return r; }
o_fq2 o_fq2_one(void) { o_fq2 r = {o_fq_one(), FQ_ZERO}; return r; }
int o_fq2_is_zero(const o_fq2 *a) { return o_fq_is_zero(&a->c0) && o_fq_is_zero(&a->c1); }
int o_fq2_eq(const o_fq2 *a, const o_fq2 *b) { return o_fq_eq(&a->c0, &b->c0) && o_fq_eq(&a->c1, &b->c1); }
int o_fq2_cmp(const o_fq2 *a, const o_fq2 *b) {                               /* fq2.rs:21-30 */
    int c = o_fq_cmp(&a->c1, &b->c1);
    return c != 0 ? c : o_fq_cmp(&a->c0, &b->c0);
}

void o_fq2_mul_by_nonresidue(o_fq2 *a) {                                      /* fq2.rs:41-45 */
    o_fq t0 = a->c0;
    o_fq_sub(&a->c0, &a->c1);
    o_fq_add(&a->c1, &t0);
}
void o_fq2_square(o_fq2 *a) {                                                 /* fq2.rs:87-101 */
    o_fq ab = a->c0;
    o_fq_mul(&ab, &a->c1);
    o_fq c0c1 = a->c0;
    o_fq_add(&c0c1, &a->c1);
    o_fq c0 = a->c1;
    o_fq_negate(&c0);
    o_fq_add(&c0, &a->c0);
    o_fq_mul(&c0, &c0c1);
    o_fq_sub(&c0, &ab);
    a->c1 = ab;
    o_fq_add(&a->c1, &ab);
    o_fq_add(&c0, &ab);
    a->c0 = c0;
}
void o_fq2_double(o_fq2 *a) { o_fq_double(&a->c0); o_fq_double(&a->c1); }
void o_fq2_negate(o_fq2 *a) { o_fq_negate(&a->c0); o_fq_negate(&a->c1); }
void o_fq2_add(o_fq2 *a, const o_fq2 *b) { o_fq_add(&a->c0, &b->c0); o_fq_add(&a->c1, &b->c1); }
void o_fq2_sub(o_fq2 *a, const o_fq2 *b) { o_fq_sub(&a->c0, &b->c0); o_fq_sub(&a->c1, &b->c1); }
void o_fq2_mul(o_fq2 *a, const o_fq2 *b) {                                    /* fq2.rs:123-136 */
    o_fq aa = a->c0;
    o_fq_mul(&aa, &b->c0);
    o_fq bb = a->c1;
    o_fq_mul(&bb, &b->c1);
    o_fq o = b->c0;
    o_fq_add(&o, &b->c1);
    o_fq_add(&a->c1, &a->c0);
    o_fq_mul(&a->c1, &o);
    o_fq_sub(&a->c1, &aa);
    o_fq_sub(&a->c1, &bb);
    a->c0 = aa;
    o_fq_sub(&a->c0, &bb);
}
int o_fq2_inverse(o_fq2 *out, const o_fq2 *a) {                               /* fq2.rs:138-155 */
    o_fq t1 = a->c1;
    o_fq_square(&t1);
    o_fq t0 = a->c0;
    o_fq_square(&t0);
    o_fq_add(&t0, &t1);
    o_fq t;
    if (!o_fq_inverse(&t, &t0)) return 0;
    o_fq2 tmp = *a;
    o_fq_mul(&tmp.c0, &t);
    o_fq_mul(&tmp.c1, &t);
    o_fq_negate(&tmp.c1);
    *out = tmp;
    return 1;
}
void o_fq2_frobenius_map(o_fq2 *a, size_t power) {                            /* fq2.rs:157-159 */
    o_fq c;
    memcpy(c.l, O_FROB_FQ2_C1[power % 2], 48);
    o_fq_mul(&a->c1, &c);
}

/* ---- Fq6: fq6.rs:30-302 ---- */
o_fq6 o_fq6_zero(void) { o_fq6 r = {o_fq2_zero(), o_fq2_zero(), o_fq2_zero()}; return r; }
o_fq6 o_fq6_one(void) { o_fq6 r = {o_fq2_one(), o_fq2_zero(), o_fq2_zero()}; return r; }
int o_fq6_is_zero(const o_fq6 *a) {
    return o_fq2_is_zero(&a->c0) && o_fq2_is_zero(&a->c1) && o_fq2_is_zero(&a->c2);
}

void o_fq6_mul_by_nonresidue(o_fq6 *a) {                                      /* fq6.rs:32-38 */
    o_fq2 t = a->c2;
    a->c2 = a->c1;
    a->c1 = a->c0;
    a->c0 = t;
    o_fq2_mul_by_nonresidue(&a->c0);
}
void o_fq6_mul_by_1(o_fq6 *a, const o_fq2 *c1) {                              /* fq6.rs:40-66 */
    o_fq2 b_b = a->c1;
    o_fq2_mul(&b_b, c1);
    o_fq2 t1 = *c1;
    {
        o_fq2 tmp = a->c1;
        o_fq2_add(&tmp, &a->c2);
        o_fq2_mul(&t1, &tmp);
        o_fq2_sub(&t1, &b_b);
        o_fq2_mul_by_nonresidue(&t1);
    }
    o_fq2 t2 = *c1;
    {
        o_fq2 tmp = a->c0;
        o_fq2_add(&tmp, &a->c1);
        o_fq2_mul(&t2, &tmp);
        o_fq2_sub(&t2, &b_b);
    }
    a->c0 = t1;
    a->c1 = t2;
    a->c2 = b_b;
}
void o_fq6_mul_by_01(o_fq6 *a, const o_fq2 *c0, const o_fq2 *c1) {          /* fq6.rs:68-109 */
    o_fq2 a_a = a->c0;
    o_fq2 b_b = a->c1;
    o_fq2_mul(&a_a, c0);
    o_fq2_mul(&b_b, c1);
    o_fq2 t1 = *c1;
    {
        o_fq2 tmp = a->c1;
        o_fq2_add(&tmp, &a->c2);
        o_fq2_mul(&t1, &tmp);
        o_fq2_sub(&t1, &b_b);
        o_fq2_mul_by_nonresidue(&t1);
        o_fq2_add(&t1, &a_a);
    }
    o_fq2 t3 = *c0;
    {
        o_fq2 tmp = a->c0;
        o_fq2_add(&tmp, &a->c2);
        o_fq2_mul(&t3, &tmp);
        o_fq2_sub(&t3, &a_a);
        o_fq2_add(&t3, &b_b);
    }
    o_fq2 t2 = *c0;
    o_fq2_add(&t2, c1);
    {
        o_fq2 tmp = a->c0;
        o_fq2_add(&tmp, &a->c1);
        o_fq2_mul(&t2, &tmp);
        o_fq2_sub(&t2, &a_a);
        o_fq2_sub(&t2, &b_b);
    }
    a->c0 = t1;
    a->c1 = t2;
    a->c2 = t3;
}
void o_fq6_double(o_fq6 *a) { o_fq2_double(&a->c0); o_fq2_double(&a->c1); o_fq2_double(&a->c2); }
void o_fq6_negate(o_fq6 *a) { o_fq2_negate(&a->c0); o_fq2_negate(&a->c1); o_fq2_negate(&a->c2); }
void o_fq6_add(o_fq6 *a, const o_fq6 *b) {
    o_fq2_add(&a->c0, &b->c0); o_fq2_add(&a->c1, &b->c1); o_fq2_add(&a->c2, &b->c2);
}
void o_fq6_sub(o_fq6 *a, const o_fq6 *b) {
    o_fq2_sub(&a->c0, &b->c0); o_fq2_sub(&a->c1, &b->c1); o_fq2_sub(&a->c2, &b->c2);
}
void o_fq6_frobenius_map(o_fq6 *a, size_t power) {                            /* fq6.rs:157-164 */
    o_fq2_frobenius_map(&a->c0, power);
    o_fq2_frobenius_map(&a->c1, power);
    o_fq2_frobenius_map(&a->c2, power);
    o_fq2 k1, k2;
    memcpy(&k1, O_FROB_FQ6_C1[power % 6], 96);
    memcpy(&k2, O_FROB_FQ6_C2[power % 6], 96);
    o_fq2_mul(&a->c1, &k1);
    o_fq2_mul(&a->c2, &k2);
}
void o_fq6_square(o_fq6 *a) {                                                 /* fq6.rs:166-197 */
    o_fq2 s0 = a->c0;
    o_fq2_square(&s0);
    o_fq2 ab = a->c0;
    o_fq2_mul(&ab, &a->c1);
    o_fq2 s1 = ab;
    o_fq2_double(&s1);
    o_fq2 s2 = a->c0;
    o_fq2_sub(&s2, &a->c1);
    o_fq2_add(&s2, &a->c2);
    o_fq2_square(&s2);
    o_fq2 bc = a->c1;
    o_fq2_mul(&bc, &a->c2);
    o_fq2 s3 = bc;
    o_fq2_double(&s3);
    o_fq2 s4 = a->c2;
    o_fq2_square(&s4);

    a->c0 = s3;
    o_fq2_mul_by_nonresidue(&a->c0);
    o_fq2_add(&a->c0, &s0);

    a->c1 = s4;
    o_fq2_mul_by_nonresidue(&a->c1);
    o_fq2_add(&a->c1, &s1);

    a->c2 = s1;
    o_fq2_add(&a->c2, &s2);
    o_fq2_add(&a->c2, &s3);
    o_fq2_sub(&a->c2, &s0);
    o_fq2_sub(&a->c2, &s4);
}
void o_fq6_mul(o_fq6 *a, const o_fq6 *b) {                                    /* fq6.rs:199-248 */
    o_fq2 a_a = a->c0, b_b = a->c1, c_c = a->c2;
    o_fq2_mul(&a_a, &b->c0);
    o_fq2_mul(&b_b, &b->c1);
    o_fq2_mul(&c_c, &b->c2);

    o_fq2 t1 = b->c1;
    o_fq2_add(&t1, &b->c2);
    {
        o_fq2 tmp = a->c1;
        o_fq2_add(&tmp, &a->c2);
        o_fq2_mul(&t1, &tmp);
        o_fq2_sub(&t1, &b_b);
        o_fq2_sub(&t1, &c_c);
        o_fq2_mul_by_nonresidue(&t1);
        o_fq2_add(&t1, &a_a);
    }
    o_fq2 t3 = b->c0;
    o_fq2_add(&t3, &b->c2);
    {
        o_fq2 tmp = a->c0;
        o_fq2_add(&tmp, &a->c2);
        o_fq2_mul(&t3, &tmp);
        o_fq2_sub(&t3, &a_a);
        o_fq2_add(&t3, &b_b);
        o_fq2_sub(&t3, &c_c);
    }
    o_fq2 t2 = b->c0;
    o_fq2_add(&t2, &b->c1);
    {
        o_fq2 tmp = a->c0;
        o_fq2_add(&tmp, &a->c1);
        o_fq2_mul(&t2, &tmp);
        o_fq2_sub(&t2, &a_a);
        o_fq2_sub(&t2, &b_b);
        o_fq2_mul_by_nonresidue(&c_c);
        o_fq2_add(&t2, &c_c);
    }
    a->c0 = t1;
    a->c1 = t2;
    a->c2 = t3;
}
int o_fq6_inverse(o_fq6 *out, const o_fq6 *a) {                               /* fq6.rs:250-301 */
    o_fq2 c0 = a->c2;
    o_fq2_mul_by_nonresidue(&c0);
    o_fq2_mul(&c0, &a->c1);
    o_fq2_negate(&c0);
    {
        o_fq2 c0s = a->c0;
        o_fq2_square(&c0s);
        o_fq2_add(&c0, &c0s);
    }
    o_fq2 c1 = a->c2;
    o_fq2_square(&c1);
    o_fq2_mul_by_nonresidue(&c1);
    {
        o_fq2 c01 = a->c0;
        o_fq2_mul(&c01, &a->c1);
        o_fq2_sub(&c1, &c01);
    }
    o_fq2 c2 = a->c1;
    o_fq2_square(&c2);
    {
        o_fq2 c02 = a->c0;
        o_fq2_mul(&c02, &a->c2);
        o_fq2_sub(&c2, &c02);
    }
    o_fq2 tmp1 = a->c2;
    o_fq2_mul(&tmp1, &c1);
    o_fq2 tmp2 = a->c1;
    o_fq2_mul(&tmp2, &c2);
    o_fq2_add(&tmp1, &tmp2);
    o_fq2_mul_by_nonresidue(&tmp1);
    tmp2 = a->c0;
    o_fq2_mul(&tmp2, &c0);
    o_fq2_add(&tmp1, &tmp2);

    o_fq2 t;
    if (!o_fq2_inverse(&t, &tmp1)) return 0;
    o_fq6 r = {t, t, t};
    o_fq2_mul(&r.c0, &c0);
    o_fq2_mul(&r.c1, &c1);
    o_fq2_mul(&r.c2, &c2);
    *out = r;
    return 1;
}

/* ---- Fq12: fq12.rs:29-149 ---- */
o_fq12 o_fq12_one(void) { o_fq12 r = {o_fq6_one(), o_fq6_zero()}; return r; }
o_fq12 o_fq12_zero(void) { o_fq12 r = {o_fq6_zero(), o_fq6_zero()}; return r; }
int o_fq12_is_zero(const o_fq12 *a) { return o_fq6_is_zero(&a->c0) && o_fq6_is_zero(&a->c1); }
int o_fq12_eq(const o_fq12 *a, const o_fq12 *b) { return memcmp(a, b, sizeof(o_fq12)) == 0; }

void o_fq12_conjugate(o_fq12 *a) { o_fq6_negate(&a->c1); }                   /* fq12.rs:30-32 */
void o_fq12_mul_by_014(o_fq12 *a, const o_fq2 *c0, const o_fq2 *c1, const o_fq2 *c4) { /* fq12.rs:34-48 */
    o_fq6 aa = a->c0;
    o_fq6_mul_by_01(&aa, c0, c1);
    o_fq6 bb = a->c1;
    o_fq6_mul_by_1(&bb, c4);
    o_fq2 o = *c1;
    o_fq2_add(&o, c4);
    o_fq6_add(&a->c1, &a->c0);
    o_fq6_mul_by_01(&a->c1, c0, &o);
    o_fq6_sub(&a->c1, &aa);
    o_fq6_sub(&a->c1, &bb);
    a->c0 = bb;
    o_fq6_mul_by_nonresidue(&a->c0);
    o_fq6_add(&a->c0, &aa);
}
void o_fq12_add(o_fq12 *a, const o_fq12 *b) { o_fq6_add(&a->c0, &b->c0); o_fq6_add(&a->c1, &b->c1); }
void o_fq12_sub(o_fq12 *a, const o_fq12 *b) { o_fq6_sub(&a->c0, &b->c0); o_fq6_sub(&a->c1, &b->c1); }
void o_fq12_frobenius_map(o_fq12 *a, size_t power) {                          /* fq12.rs:90-97 */
    o_fq6_frobenius_map(&a->c0, power);
    o_fq6_frobenius_map(&a->c1, power);
    o_fq2 k;
    memcpy(&k, O_FROB_FQ12_C1[power % 12], 96);
    o_fq2_mul(&a->c1.c0, &k);
    o_fq2_mul(&a->c1.c1, &k);
    o_fq2_mul(&a->c1.c2, &k);
}
void o_fq12_square(o_fq12 *a) {                                               /* fq12.rs:99-114 */
    o_fq6 ab = a->c0;
    o_fq6_mul(&ab, &a->c1);
    o_fq6 c0c1 = a->c0;
    o_fq6_add(&c0c1, &a->c1);
    o_fq6 c0 = a->c1;
    o_fq6_mul_by_nonresidue(&c0);
    o_fq6_add(&c0, &a->c0);
    o_fq6_mul(&c0, &c0c1);
    o_fq6_sub(&c0, &ab);
    a->c1 = ab;
    o_fq6_add(&a->c1, &ab);
    o_fq6_mul_by_nonresidue(&ab);
    o_fq6_sub(&c0, &ab);
    a->c0 = c0;
}
void o_fq12_mul(o_fq12 *a, const o_fq12 *b) {                                 /* fq12.rs:116-130 */
    o_fq6 aa = a->c0;
    o_fq6_mul(&aa, &b->c0);
    o_fq6 bb = a->c1;
    o_fq6_mul(&bb, &b->c1);
    o_fq6 o = b->c0;
    o_fq6_add(&o, &b->c1);
    o_fq6_add(&a->c1, &a->c0);
    o_fq6_mul(&a->c1, &o);
    o_fq6_sub(&a->c1, &aa);
    o_fq6_sub(&a->c1, &bb);
    a->c0 = bb;
    o_fq6_mul_by_nonresidue(&a->c0);
    o_fq6_add(&a->c0, &aa);
}
int o_fq12_inverse(o_fq12 *out, const o_fq12 *a) {                            /* fq12.rs:132-148 */
    o_fq6 c0s = a->c0;
    o_fq6_square(&c0s);
    o_fq6 c1s = a->c1;
    o_fq6_square(&c1s);
    o_fq6_mul_by_nonresidue(&c1s);
    o_fq6_sub(&c0s, &c1s);
    o_fq6 t;
    if (!o_fq6_inverse(&t, &c0s)) return 0;
    o_fq12 tmp = {t, t};
    o_fq6_mul(&tmp.c0, &a->c0);
    o_fq6_mul(&tmp.c1, &a->c1);
    o_fq6_negate(&tmp.c1);
    *out = tmp;
    return 1;
}

/* Field::pow, lib.rs:306-324, with BitIterator (lib.rs:582-610): MSB first
 * over all 64*n bits; the first set bit multiplies `one` by self. */
#define DEFINE_POW(T, ONE, SQ, MUL)                                                  \
    void o_##T##_pow(o_##T *out, const o_##T *a, const uint64_t *exp, size_t n) {     \
        o_##T res = ONE();                                                            \
        int found_one = 0;                                                            \
        for (size_t bit = 64 * n; bit-- > 0;) {                                       \
            int i = (int)((exp[bit / 64] >> (bit % 64)) & 1);                         \
            if (found_one) SQ(&res);                                                  \
            else found_one = i;                                                       \
            if (i) MUL(&res, a);                                                      \
        }                                                                             \
        *out = res;                                                                   \
    }
DEFINE_POW(fq, o_fq_one, o_fq_square, o_fq_mul)
DEFINE_POW(fq2, o_fq2_one, o_fq2_square, o_fq2_mul)
DEFINE_POW(fq6, o_fq6_one, o_fq6_square, o_fq6_mul)
DEFINE_POW(fq12, o_fq12_one, o_fq12_square, o_fq12_mul)
