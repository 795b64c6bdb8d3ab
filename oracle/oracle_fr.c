/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * The scalar field Fr of BLS12-381, restated from the reference crate
 * (src/bls12_381/fr.rs):
 *   constants            fr.rs:4-56 (MODULUS, R, R2, INV, GENERATOR, S, ROOT_OF_UNITY)
 *   from_repr/into_repr  fr.rs:279-303
 *   add/double/sub/neg   fr.rs:341-375
 *   inverse (BEA)        fr.rs:377-431
 *   mul_assign / square  fr.rs:438-500 (schoolbook product + mont_reduce fr.rs:520-572)
 *   is_valid / reduce    fr.rs:506-518
 *   legendre / sqrt      fr.rs:574-646 (Tonelli-Shanks, 2^32 | r-1)
 *   Field::pow           src/lib.rs:306-324
 * Fr = u64[4] little-endian limbs, Montgomery form with R = 2^256, < r.
 */
#include <string.h>
#include "oracle.h"
#include "oracle_internal.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t l[4]; } o_fr;

static const uint64_t FR_MODULUS[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                       0x73eda753299d7d48ull};                            /* fr.rs:4-10 */
static const uint64_t FR_R[4] = {0x1fffffffeull, 0x5884b7fa00034802ull, 0x998c4fefecbc4ff5ull,
                                 0x1824b159acc5056full};                                  /* fr.rs:19-25 */
static const uint64_t FR_R2[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full,
                                  0x0748d9d99f59ff11ull};                                 /* fr.rs:28-34 */
static const uint64_t FR_INV = 0xfffffffeffffffffull;                                     /* fr.rs:37 */
static const uint32_t FR_S = 32;                                                          /* fr.rs:48 */
static const uint64_t FR_ROOT_OF_UNITY[4] = {0xb9b58d8c5f0e466aull, 0x5b1b4c801819d7ecull,
                                             0x0af53ae352a31e64ull, 0x5bf3adda19e9b27bull}; /* fr.rs:51-56 */
static const uint64_t FR_LEGENDRE_EXP[4] = {0x7fffffff80000000ull, 0xa9ded2017fff2dffull,
                                            0x199cec0404d0ec02ull, 0x39f6d3a994cebea4ull}; /* fr.rs:577-582 */
static const uint64_t FR_T_PLUS_1_OVER_2[4] = {0x7fff2dff80000000ull, 0x04d0ec02a9ded201ull,
                                               0x94cebea4199cec04ull, 0x0000000039f6d3a9ull}; /* fr.rs:603-608 */
static const uint64_t FR_T[4] = {0xfffe5bfeffffffffull, 0x09a1d80553bda402ull, 0x299d7d483339d808ull,
                                 0x0000000073eda753ull};                                  /* fr.rs:610-615 */

static inline uint64_t adc(uint64_t a, uint64_t b, uint64_t *carry) {   /* lib.rs:659-666 */
    u128 t = (u128)a + b + *carry;
    *carry = (uint64_t)(t >> 64);
    return (uint64_t)t;
}
static inline uint64_t mac(uint64_t a, uint64_t b, uint64_t c, uint64_t *carry) {   /* lib.rs:670-678 */
    u128 t = (u128)a + (u128)b * c + *carry;
    *carry = (uint64_t)(t >> 64);
    return (uint64_t)t;
}

static o_fr fr_zero(void) { o_fr z; memset(&z, 0, sizeof z); return z; }
static o_fr fr_one(void) { o_fr o; memcpy(o.l, FR_R, 32); return o; }
static int fr_is_zero(const o_fr *a) { return o_repr_is_zero(a->l, 4); }
static int fr_eq(const o_fr *a, const o_fr *b) { return memcmp(a->l, b->l, 32) == 0; }
static int fr_is_valid(const o_fr *a) { return o_repr_cmp(a->l, FR_MODULUS, 4) < 0; }   /* fr.rs:506-508 */
static void fr_reduce(o_fr *a) {                                                        /* fr.rs:513-518 */
    if (!fr_is_valid(a)) o_repr_sub_noborrow(a->l, FR_MODULUS, 4);
}

static void fr_add(o_fr *a, const o_fr *b) {                                            /* fr.rs:341-348 */
    o_repr_add_nocarry(a->l, b->l, 4);
    fr_reduce(a);
}
static void fr_double(o_fr *a) {                                                        /* fr.rs:350-357 */
    uint64_t last = 0;
    for (int i = 0; i < 4; i++) {                                                       /* FrRepr::mul2 fr.rs:177-186 */
        uint64_t t = a->l[i] >> 63;
        a->l[i] = (a->l[i] << 1) | last;
        last = t;
    }
    fr_reduce(a);
}
static void fr_sub(o_fr *a, const o_fr *b) {                                            /* fr.rs:359-367 */
    if (o_repr_cmp(b->l, a->l, 4) > 0) o_repr_add_nocarry(a->l, FR_MODULUS, 4);
    o_repr_sub_noborrow(a->l, b->l, 4);
}
static void fr_negate(o_fr *a) {                                                        /* fr.rs:369-375 */
    if (!fr_is_zero(a)) {
        uint64_t t[4];
        memcpy(t, FR_MODULUS, 32);
        o_repr_sub_noborrow(t, a->l, 4);
        memcpy(a->l, t, 32);
    }
}

/* mont_reduce, fr.rs:520-572 (HAC 14.32), r[0..8) little-endian */
static void fr_mont_reduce(o_fr *a, uint64_t r[8]) {
    uint64_t carry2 = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t k = r[i] * FR_INV, carry = 0;
        mac(r[i], k, FR_MODULUS[0], &carry);
        for (int j = 1; j < 4; j++) r[i + j] = mac(r[i + j], k, FR_MODULUS[j], &carry);
        r[i + 4] = adc(r[i + 4], carry2, &carry);
        carry2 = carry;
    }
    memcpy(a->l, r + 4, 32);
    fr_reduce(a);
}
static void fr_mul(o_fr *a, const o_fr *b) {                                            /* fr.rs:438-465 */
    uint64_t r[8] = {0};
    for (int i = 0; i < 4; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 4; j++) r[i + j] = mac(r[i + j], a->l[i], b->l[j], &carry);
        r[i + 4] = carry;
    }
    fr_mont_reduce(a, r);
}
static void fr_square(o_fr *a) {                                                        /* fr.rs:467-500 */
    uint64_t r[8] = {0}, carry;
    for (int i = 0; i < 3; i++) {           /* off-diagonal products */
        carry = 0;
        for (int j = i + 1; j < 4; j++) r[i + j] = mac(r[i + j], a->l[i], a->l[j], &carry);
        r[i + 4] = carry;
    }
    r[7] = r[6] >> 63;                      /* double */
    for (int k = 6; k >= 2; k--) r[k] = (r[k] << 1) | (r[k - 1] >> 63);
    r[1] <<= 1;
    carry = 0;                              /* diagonal */
    for (int i = 0; i < 4; i++) {
        r[2 * i] = mac(r[2 * i], a->l[i], a->l[i], &carry);
        r[2 * i + 1] = adc(r[2 * i + 1], 0, &carry);
    }
    fr_mont_reduce(a, r);
}

static int fr_inverse(o_fr *out, const o_fr *a) {                                      /* fr.rs:377-431 */
    if (fr_is_zero(a)) return 0;
    const uint64_t one[4] = {1, 0, 0, 0};
    uint64_t u[4], v[4];
    memcpy(u, a->l, 32);
    memcpy(v, FR_MODULUS, 32);
    o_fr b, c = fr_zero();
    memcpy(b.l, FR_R2, 32);
    while (o_repr_cmp(u, one, 4) != 0 && o_repr_cmp(v, one, 4) != 0) {
        while ((u[0] & 1) == 0) {
            o_repr_div2(u, 4);
            if ((b.l[0] & 1) == 0) o_repr_div2(b.l, 4);
            else { o_repr_add_nocarry(b.l, FR_MODULUS, 4); o_repr_div2(b.l, 4); }
        }
        while ((v[0] & 1) == 0) {
            o_repr_div2(v, 4);
            if ((c.l[0] & 1) == 0) o_repr_div2(c.l, 4);
            else { o_repr_add_nocarry(c.l, FR_MODULUS, 4); o_repr_div2(c.l, 4); }
        }
        if (o_repr_cmp(v, u, 4) < 0) {
            o_repr_sub_noborrow(u, v, 4);
            fr_sub(&b, &c);
        } else {
            o_repr_sub_noborrow(v, u, 4);
            fr_sub(&c, &b);
        }
    }
    *out = o_repr_cmp(u, one, 4) == 0 ? b : c;
    return 1;
}

static int fr_from_repr(o_fr *out, const uint64_t repr[4]) {                            /* fr.rs:279-288 */
    o_fr r;
    memcpy(r.l, repr, 32);
    if (!fr_is_valid(&r)) return 0;
    o_fr r2;
    memcpy(r2.l, FR_R2, 32);
    fr_mul(&r, &r2);
    *out = r;
    return 1;
}
static void fr_into_repr(uint64_t out[4], const o_fr *a) {                              /* fr.rs:290-303 */
    uint64_t r[8] = {a->l[0], a->l[1], a->l[2], a->l[3], 0, 0, 0, 0};
    o_fr t;
    fr_mont_reduce(&t, r);
    memcpy(out, t.l, 32);
}

static void fr_pow(o_fr *out, const o_fr *a, const uint64_t *exp, size_t n) {           /* lib.rs:306-324 */
    o_fr res = fr_one();
    int found_one = 0;
    for (size_t bit = 64 * n; bit-- > 0;) {     /* BitIterator, MSB first (lib.rs:582-610) */
        int i = (int)((exp[bit / 64] >> (bit % 64)) & 1);
        if (found_one) fr_square(&res);
        else found_one = i;
        if (i) fr_mul(&res, a);
    }
    *out = res;
}

/* LegendreSymbol: 0 = Zero, 1 = QuadraticResidue, -1 = QuadraticNonResidue (lib.rs:423-428) */
static int fr_legendre(const o_fr *a) {                                                 /* fr.rs:575-590 */
    o_fr s;
    fr_pow(&s, a, FR_LEGENDRE_EXP, 4);
    o_fr z = fr_zero(), o = fr_one();
    if (fr_eq(&s, &z)) return 0;
    if (fr_eq(&s, &o)) return 1;
    return -1;
}
static int fr_sqrt(o_fr *out, const o_fr *a) {                                          /* fr.rs:592-646 */
    int l = fr_legendre(a);
    if (l == 0) { *out = *a; return 1; }
    if (l < 0) return 0;
    o_fr c, r, t, one = fr_one();
    memcpy(c.l, FR_ROOT_OF_UNITY, 32);
    fr_pow(&r, a, FR_T_PLUS_1_OVER_2, 4);
    fr_pow(&t, a, FR_T, 4);
    uint32_t m = FR_S;
    while (!fr_eq(&t, &one)) {
        uint32_t i = 1;
        o_fr t2i = t;
        fr_square(&t2i);
        while (!fr_eq(&t2i, &one)) {
            fr_square(&t2i);
            i++;
        }
        for (uint32_t k = 0; k + i + 1 < m; k++) fr_square(&c);
        fr_mul(&r, &c);
        fr_square(&c);
        fr_mul(&t, &c);
        m = i;
    }
    *out = r;
    return 1;
}

/* ---- batch exports (ctypes) ---- */
#define FR(p) ((o_fr *)(p))
#define CFR(p) ((const o_fr *)(p))
void o_fr_mul_batch(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fr t = CFR(a)[k]; fr_mul(&t, &CFR(b)[k]); FR(out)[k] = t; }
}
void o_fr_square_batch(const uint64_t *a, uint64_t *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fr t = CFR(a)[k]; fr_square(&t); FR(out)[k] = t; }
}
void o_fr_add_batch(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fr t = CFR(a)[k]; fr_add(&t, &CFR(b)[k]); FR(out)[k] = t; }
}
void o_fr_sub_batch(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fr t = CFR(a)[k]; fr_sub(&t, &CFR(b)[k]); FR(out)[k] = t; }
}
void o_fr_double_batch(const uint64_t *a, uint64_t *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fr t = CFR(a)[k]; fr_double(&t); FR(out)[k] = t; }
}
void o_fr_negate_batch(const uint64_t *a, uint64_t *out, size_t n) {
    for (size_t k = 0; k < n; k++) { o_fr t = CFR(a)[k]; fr_negate(&t); FR(out)[k] = t; }
}
void o_fr_inverse_batch(const uint64_t *a, uint64_t *out, uint8_t *ok, size_t n) {
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < n; k++) {
        o_fr t = fr_zero();
        ok[k] = (uint8_t)fr_inverse(&t, &CFR(a)[k]);
        FR(out)[k] = t;
    }
}
void o_fr_from_repr_batch(const uint64_t *repr, size_t n, uint64_t *out, uint8_t *ok) {
    for (size_t k = 0; k < n; k++) {
        o_fr t = fr_zero();
        ok[k] = (uint8_t)fr_from_repr(&t, &repr[4 * k]);
        FR(out)[k] = t;
    }
}
void o_fr_into_repr_batch(const uint64_t *a, size_t n, uint64_t *out) {
    for (size_t k = 0; k < n; k++) fr_into_repr(&out[4 * k], &CFR(a)[k]);
}
void o_fr_pow_batch(const uint64_t *a, const uint64_t *exp, size_t nwords, uint64_t *out, size_t n) {
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < n; k++) fr_pow(&FR(out)[k], &CFR(a)[k], exp, nwords);
}
void o_fr_legendre_batch(const uint64_t *a, int8_t *out, size_t n) {
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < n; k++) out[k] = (int8_t)fr_legendre(&CFR(a)[k]);
}
void o_fr_sqrt_batch(const uint64_t *a, size_t n, uint64_t *out, uint8_t *ok) {
#pragma omp parallel for schedule(dynamic, 16)
    for (size_t k = 0; k < n; k++) {
        o_fr t = fr_zero();
        ok[k] = (uint8_t)fr_sqrt(&t, &CFR(a)[k]);
        FR(out)[k] = t;
    }
}
void o_fr_constants(uint64_t *modulus, uint64_t *r, uint64_t *root_of_unity) {
    memcpy(modulus, FR_MODULUS, 32);
    memcpy(r, FR_R, 32);
    memcpy(root_of_unity, FR_ROOT_OF_UNITY, 32);
}
