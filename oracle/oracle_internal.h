/* TEST INFRASTRUCTURE ONLY -- internal prototypes of the C oracle (oracle/). */
#ifndef PAIRING_ORACLE_INTERNAL_H
#define PAIRING_ORACLE_INTERNAL_H
#include "oracle.h"

int o_repr_cmp(const uint64_t *a, const uint64_t *b, int n);
int o_repr_is_zero(const uint64_t *a, int n);
void o_repr_div2(uint64_t *a, int n);
void o_repr_add_nocarry(uint64_t *a, const uint64_t *b, int n);
void o_repr_sub_noborrow(uint64_t *a, const uint64_t *b, int n);

o_fq o_fq_zero(void);
o_fq o_fq_one(void);
int o_fq_is_zero(const o_fq *a);
int o_fq_eq(const o_fq *a, const o_fq *b);
void o_fq_add(o_fq *a, const o_fq *b);
void o_fq_double(o_fq *a);
void o_fq_sub(o_fq *a, const o_fq *b);
void o_fq_negate(o_fq *a);
void o_fq_mul(o_fq *a, const o_fq *b);
void o_fq_square(o_fq *a);
int o_fq_inverse(o_fq *out, const o_fq *a);
int o_fq_from_repr(o_fq *out, const uint64_t repr[6]);
void o_fq_into_repr(uint64_t out[6], const o_fq *a);
int o_fq_cmp(const o_fq *a, const o_fq *b);
void o_fq_pow(o_fq *out, const o_fq *a, const uint64_t *exp, size_t n);

o_fq2 o_fq2_zero(void);
o_fq2 o_fq2_one(void);
int o_fq2_is_zero(const o_fq2 *a);
int o_fq2_eq(const o_fq2 *a, const o_fq2 *b);
int o_fq2_cmp(const o_fq2 *a, const o_fq2 *b);
void o_fq2_mul_by_nonresidue(o_fq2 *a);
void o_fq2_square(o_fq2 *a);
void o_fq2_double(o_fq2 *a);
void o_fq2_negate(o_fq2 *a);
void o_fq2_add(o_fq2 *a, const o_fq2 *b);
void o_fq2_sub(o_fq2 *a, const o_fq2 *b);
void o_fq2_mul(o_fq2 *a, const o_fq2 *b);
int o_fq2_inverse(o_fq2 *out, const o_fq2 *a);
void o_fq2_frobenius_map(o_fq2 *a, size_t power);
void o_fq2_pow(o_fq2 *out, const o_fq2 *a, const uint64_t *exp, size_t n);

o_fq6 o_fq6_zero(void);
o_fq6 o_fq6_one(void);
int o_fq6_is_zero(const o_fq6 *a);
void o_fq6_mul_by_nonresidue(o_fq6 *a);
void o_fq6_mul_by_1(o_fq6 *a, const o_fq2 *c1);
void o_fq6_mul_by_01(o_fq6 *a, const o_fq2 *c0, const o_fq2 *c1);
void o_fq6_double(o_fq6 *a);
void o_fq6_negate(o_fq6 *a);
void o_fq6_add(o_fq6 *a, const o_fq6 *b);
void o_fq6_sub(o_fq6 *a, const o_fq6 *b);
void o_fq6_frobenius_map(o_fq6 *a, size_t power);
void o_fq6_square(o_fq6 *a);
void o_fq6_mul(o_fq6 *a, const o_fq6 *b);
int o_fq6_inverse(o_fq6 *out, const o_fq6 *a);
void o_fq6_pow(o_fq6 *out, const o_fq6 *a, const uint64_t *exp, size_t n);

o_fq12 o_fq12_one(void);
o_fq12 o_fq12_zero(void);
int o_fq12_is_zero(const o_fq12 *a);
int o_fq12_eq(const o_fq12 *a, const o_fq12 *b);
void o_fq12_conjugate(o_fq12 *a);
void o_fq12_mul_by_014(o_fq12 *a, const o_fq2 *c0, const o_fq2 *c1, const o_fq2 *c4);
void o_fq12_add(o_fq12 *a, const o_fq12 *b);
void o_fq12_sub(o_fq12 *a, const o_fq12 *b);
void o_fq12_frobenius_map(o_fq12 *a, size_t power);
void o_fq12_square(o_fq12 *a);
void o_fq12_mul(o_fq12 *a, const o_fq12 *b);
int o_fq12_inverse(o_fq12 *out, const o_fq12 *a);
void o_fq12_pow(o_fq12 *out, const o_fq12 *a, const uint64_t *exp, size_t n);

/* curve_impl instantiations used by the decoders (oracle_curve_impl.h) */
int o_g1_is_zero(const o_g1 *p);
int o_g2_is_zero(const o_g2 *p);
o_g1_affine o_g1_affine_zero(void);
o_g2_affine o_g2_affine_zero(void);
o_g1 o_g1_affine_mul(const o_g1_affine *a, const uint64_t scalar[4]);
o_g2 o_g2_affine_mul(const o_g2_affine *a, const uint64_t scalar[4]);
int o_g1_is_on_curve(const o_g1_affine *a);
int o_g2_is_on_curve(const o_g2_affine *a);

/* decoding status = GroupDecodingError (lib.rs:469-481); same codes as
 * PA_DECODE_* in include/pairing_amd.h.  CoordinateDecodingError carries the
 * coordinate name: G1 "x coordinate" / "y coordinate" map to X_C0 / Y_C0. */
enum {
    O_DEC_OK = 0,
    O_DEC_NOT_ON_CURVE = 1,
    O_DEC_NOT_IN_SUBGROUP = 2,
    O_DEC_X_C0 = 3,
    O_DEC_X_C1 = 4,
    O_DEC_Y_C0 = 5,
    O_DEC_Y_C1 = 6,
    O_DEC_UNEXPECTED_COMPRESSION_MODE = 7,
    O_DEC_UNEXPECTED_INFORMATION = 8,
};
int o_fq_sqrt(o_fq *out, const o_fq *a);
int o_fq2_sqrt(o_fq2 *out, const o_fq2 *a);
int o_g1_decode(o_g1_affine *out, const uint8_t *enc, int compressed, int checked);
int o_g2_decode(o_g2_affine *out, const uint8_t *enc, int compressed, int checked);

#endif
