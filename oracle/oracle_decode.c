/* TEST INFRASTRUCTURE ONLY -- see oracle/oracle.h.
 *
 * Point decoding (SURVEY.md §8 f, rank 1): EncodedPoint::into_affine for the
 * four wire formats (src/bls12_381/README.md "Serialization"):
 *   G1Uncompressed ec.rs:662-736, G1Compressed ec.rs:785-837,
 *   G2Uncompressed ec.rs:1322-1397, G2Compressed ec.rs:1448-1509,
 * with get_point_from_x (ec.rs:100-121), is_on_curve (ec.rs:125-140),
 * is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144: affine.mul(r) is
 * zero, mul_bits ec.rs:88-95) and the square roots of SqrtField for Fq
 * (fq.rs:1147-1170) and Fq2 (fq2.rs:167-220).
 *
 * Results are a status byte per record, the GroupDecodingError variant
 * (lib.rs:469-481) in the order the reference checks them.
 */
#include <string.h>
#include "oracle.h"
#include "oracle_consts.h"
#include "oracle_internal.h"

/* (q - 3) / 4 and (q - 1) / 2, fq.rs:1152-1159, fq2.rs:174-181, 207-214 */
static const uint64_t QM3_DIV4[6] = {0xee7fbfffffffeaaaULL, 0x07aaffffac54ffffULL, 0xd9cc34a83dac3d89ULL,
                                     0xd91dd2e13ce144afULL, 0x92c6e9ed90d2eb35ULL, 0x0680447a8e5ff9a6ULL};
static const uint64_t QM1_DIV2[6] = {0xdcff7fffffffd555ULL, 0x0f55ffff58a9ffffULL, 0xb39869507b587b12ULL,
                                     0xb23ba5c279c2895fULL, 0x258dd3db21a5d66bULL, 0x0d0088f51cbff34dULL};
/* Fr::char() = r, fr.rs:5-10 */
static const uint64_t FR_MODULUS[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                       0x73eda753299d7d48ULL};

int o_fq_sqrt(o_fq *out, const o_fq *a) {                                   /* fq.rs:1147-1170 */
    o_fq a1, a0;
    o_fq_pow(&a1, a, QM3_DIV4, 6);
    a0 = a1;
    o_fq_square(&a0);
    o_fq_mul(&a0, a);
    o_fq neg1;
    memcpy(neg1.l, O_FQ_NEGATIVE_ONE, 48);
    if (o_fq_eq(&a0, &neg1)) return 0;
    o_fq_mul(&a1, a);
    *out = a1;
    return 1;
}

int o_fq2_sqrt(o_fq2 *out, const o_fq2 *a) {                                /* fq2.rs:167-220 */
    if (o_fq2_is_zero(a)) {
        *out = o_fq2_zero();
        return 1;
    }
    o_fq2 a1, alpha, a0;
    o_fq2_pow(&a1, a, QM3_DIV4, 6);
    alpha = a1;
    o_fq2_square(&alpha);
    o_fq2_mul(&alpha, a);
    a0 = alpha;
    o_fq2_frobenius_map(&a0, 1);
    o_fq2_mul(&a0, &alpha);
    o_fq2 neg1 = o_fq2_zero();
    memcpy(neg1.c0.l, O_FQ_NEGATIVE_ONE, 48);
    if (o_fq2_eq(&a0, &neg1)) return 0;
    o_fq2_mul(&a1, a);
    if (o_fq2_eq(&alpha, &neg1)) {
        o_fq2 u = o_fq2_zero();
        u.c1 = o_fq_one();
        o_fq2_mul(&a1, &u);
    } else {
        o_fq2 one = o_fq2_one();
        o_fq2_add(&alpha, &one);
        o_fq2 t;
        o_fq2_pow(&t, &alpha, QM1_DIV2, 6);
        o_fq2_mul(&a1, &t);
    }
    *out = a1;
    return 1;
}

/* FqRepr::read_be of 48 bytes (big-endian limbs, most significant first) */
static void read_be(uint64_t r[6], const uint8_t *src) {
    for (int i = 0; i < 6; i++) {
        uint64_t w = 0;
        for (int b = 0; b < 8; b++) w = (w << 8) | src[8 * i + b];
        r[5 - i] = w;
    }
}

/* the flag checks shared by all four into_affine_unchecked bodies; returns
 * -1 to go on decoding, otherwise a status (and *inf for the point at infinity) */
static int check_flags(uint8_t *copy, size_t len, int compressed, int *inf, int *greatest) {
    *inf = 0;
    *greatest = 0;
    if (((copy[0] >> 7) & 1) != compressed) return O_DEC_UNEXPECTED_COMPRESSION_MODE;
    if (copy[0] & (1 << 6)) {
        copy[0] &= 0x3f;
        for (size_t i = 0; i < len; i++)
            if (copy[i]) return O_DEC_UNEXPECTED_INFORMATION;
        *inf = 1;
        return O_DEC_OK;
    }
    if (copy[0] & (1 << 5)) {
        if (!compressed) return O_DEC_UNEXPECTED_INFORMATION;
        *greatest = 1;
    }
    copy[0] &= 0x1f;
    return -1;
}

static int fq_from_be(o_fq *out, const uint8_t *src) {
    uint64_t r[6];
    read_be(r, src);
    return o_fq_from_repr(out, r);
}

/* ---- G1 ---- */
static int g1_subgroup(const o_g1_affine *a) {                              /* ec.rs:142-144 */
    o_g1 t = o_g1_affine_mul(a, FR_MODULUS);
    return o_g1_is_zero(&t);
}

static int g1_point_from_x(o_g1_affine *out, const o_fq *x, int greatest) {    /* ec.rs:100-121 */
    o_fq x3b = *x;
    o_fq_square(&x3b);
    o_fq_mul(&x3b, x);
    o_fq b;
    memcpy(b.l, O_FQ_B_COEFF, 48);
    o_fq_add(&x3b, &b);
    o_fq y;
    if (!o_fq_sqrt(&y, &x3b)) return 0;
    o_fq negy = y;
    o_fq_negate(&negy);
    memset(out, 0, sizeof *out);
    out->x = *x;
    out->y = ((o_fq_cmp(&y, &negy) < 0) ^ greatest) ? y : negy;
    return 1;
}

int o_g1_decode(o_g1_affine *out, const uint8_t *enc, int compressed, int checked) {
    uint8_t copy[96];
    const size_t len = compressed ? 48 : 96;
    memcpy(copy, enc, len);
    int inf, greatest;
    int st = check_flags(copy, len, compressed, &inf, &greatest);
    if (st >= 0) {
        if (st == O_DEC_OK) *out = o_g1_affine_zero();
        return st;
    }
    if (compressed) {                                                        /* ec.rs:792-837 */
        o_fq x;
        if (!fq_from_be(&x, copy)) return O_DEC_X_C0;
        if (!g1_point_from_x(out, &x, greatest)) return O_DEC_NOT_ON_CURVE;
        if (checked && !g1_subgroup(out)) return O_DEC_NOT_IN_SUBGROUP;
        return O_DEC_OK;
    }
    memset(out, 0, sizeof *out);                                             /* ec.rs:669-736 */
    if (!fq_from_be(&out->x, copy)) return O_DEC_X_C0;
    if (!fq_from_be(&out->y, copy + 48)) return O_DEC_Y_C0;
    if (!checked) return O_DEC_OK;
    if (!o_g1_is_on_curve(out)) return O_DEC_NOT_ON_CURVE;
    if (!g1_subgroup(out)) return O_DEC_NOT_IN_SUBGROUP;
    return O_DEC_OK;
}

/* ---- G2 ---- */
static int g2_subgroup(const o_g2_affine *a) {
    o_g2 t = o_g2_affine_mul(a, FR_MODULUS);
    return o_g2_is_zero(&t);
}

static int g2_point_from_x(o_g2_affine *out, const o_fq2 *x, int greatest) {
    o_fq2 x3b = *x;
    o_fq2_square(&x3b);
    o_fq2_mul(&x3b, x);
    o_fq2 b;
    memcpy(b.c0.l, O_FQ_B_COEFF, 48);                                        /* ec.rs:1557-1562 */
    memcpy(b.c1.l, O_FQ_B_COEFF, 48);
    o_fq2_add(&x3b, &b);
    o_fq2 y;
    if (!o_fq2_sqrt(&y, &x3b)) return 0;
    o_fq2 negy = y;
    o_fq2_negate(&negy);
    memset(out, 0, sizeof *out);
    out->x = *x;
    out->y = ((o_fq2_cmp(&y, &negy) < 0) ^ greatest) ? y : negy;
    return 1;
}

int o_g2_decode(o_g2_affine *out, const uint8_t *enc, int compressed, int checked) {
    uint8_t copy[192];
    const size_t len = compressed ? 96 : 192;
    memcpy(copy, enc, len);
    int inf, greatest;
    int st = check_flags(copy, len, compressed, &inf, &greatest);
    if (st >= 0) {
        if (st == O_DEC_OK) *out = o_g2_affine_zero();
        return st;
    }
    o_fq2 x;
    /* wire order x.c1, x.c0[, y.c1, y.c0]; errors reported c0 first */
    if (!fq_from_be(&x.c0, copy + 48)) return O_DEC_X_C0;
    if (!fq_from_be(&x.c1, copy)) return O_DEC_X_C1;
    if (compressed) {                                                        /* ec.rs:1455-1509 */
        if (!g2_point_from_x(out, &x, greatest)) return O_DEC_NOT_ON_CURVE;
        if (checked && !g2_subgroup(out)) return O_DEC_NOT_IN_SUBGROUP;
        return O_DEC_OK;
    }
    memset(out, 0, sizeof *out);                                             /* ec.rs:1333-1397 */
    out->x = x;
    if (!fq_from_be(&out->y.c0, copy + 144)) return O_DEC_Y_C0;
    if (!fq_from_be(&out->y.c1, copy + 96)) return O_DEC_Y_C1;
    if (!checked) return O_DEC_OK;
    if (!o_g2_is_on_curve(out)) return O_DEC_NOT_ON_CURVE;
    if (!g2_subgroup(out)) return O_DEC_NOT_IN_SUBGROUP;
    return O_DEC_OK;
}

void o_g1_decode_batch(const uint8_t *enc, size_t n, int compressed, int checked, o_g1_affine *out,
                       uint8_t *status, int nthreads) {
    const size_t sz = compressed ? 48 : 96;
#pragma omp parallel for schedule(dynamic, 8) num_threads(nthreads > 0 ? nthreads : 1)
    for (size_t k = 0; k < n; k++) {
        status[k] = (uint8_t)o_g1_decode(&out[k], enc + k * sz, compressed, checked);
        if (status[k] != O_DEC_OK) out[k] = o_g1_affine_zero();   /* the product's convention */
    }
}

void o_g2_decode_batch(const uint8_t *enc, size_t n, int compressed, int checked, o_g2_affine *out,
                       uint8_t *status, int nthreads) {
    const size_t sz = compressed ? 96 : 192;
#pragma omp parallel for schedule(dynamic, 8) num_threads(nthreads > 0 ? nthreads : 1)
    for (size_t k = 0; k < n; k++) {
        status[k] = (uint8_t)o_g2_decode(&out[k], enc + k * sz, compressed, checked);
        if (status[k] != O_DEC_OK) out[k] = o_g2_affine_zero();
    }
}

void o_fq_sqrt_batch(const o_fq *a, size_t n, o_fq *out, uint8_t *ok) {
    for (size_t k = 0; k < n; k++) ok[k] = (uint8_t)o_fq_sqrt(&out[k], &a[k]);
}
void o_fq2_sqrt_batch(const o_fq2 *a, size_t n, o_fq2 *out, uint8_t *ok) {
    for (size_t k = 0; k < n; k++) ok[k] = (uint8_t)o_fq2_sqrt(&out[k], &a[k]);
}
