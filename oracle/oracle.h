/* TEST INFRASTRUCTURE ONLY -- the parity oracle for pairing_amd.
 *
 * A plain-C restatement of the reference crate `pairing` v0.14.2
 * (dignifiedquire/pairing, Rust) BLS12-381 hot path.  Every function cites
 * the reference file:line it follows.  It is pinned against the reference's
 * own known answers (RELIC pairing KAT, the four k*G `.dat` vector files,
 * the raw-limb Fq/Fq2/G1/G2 KATs) by tests/test_oracle.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the CPU baseline.  The
 * product path (pairing_amd/) never links or calls it.
 *
 * Memory layout is the one the C ABI of the product uses
 * (include/pairing_amd.h), i.e. the Rust in-memory order:
 *   Fq  = u64[6] little-endian limbs, Montgomery form (R = 2^384), < q
 *   Fq2 = {c0, c1}; Fq6 = {c0, c1, c2}; Fq12 = {c0, c1}
 *   G1 affine = {x, y, u8 infinity, pad[7]}   (104 B)
 *   G2 affine = {x, y, u8 infinity, pad[7]}   (200 B)
 *   Jacobian  = {x, y, z}, zero iff z == 0
 *   G2Prepared = 68 x (Fq2, Fq2, Fq2) + infinity flag
 */
#ifndef PAIRING_ORACLE_H
#define PAIRING_ORACLE_H
#include <stddef.h>
#include <stdint.h>

typedef struct { uint64_t l[6]; } o_fq;
typedef struct { o_fq c0, c1; } o_fq2;
typedef struct { o_fq2 c0, c1, c2; } o_fq6;
typedef struct { o_fq6 c0, c1; } o_fq12;
typedef struct { uint64_t l[4]; } o_fr_repr;

typedef struct { o_fq x, y; uint8_t infinity; uint8_t pad[7]; } o_g1_affine;
typedef struct { o_fq x, y, z; } o_g1;
typedef struct { o_fq2 x, y; uint8_t infinity; uint8_t pad[7]; } o_g2_affine;
typedef struct { o_fq2 x, y, z; } o_g2;

#define O_G2_PREPARED_COEFFS 68
typedef struct { o_fq2 c[3]; } o_ell_coeff;
typedef struct {
    o_ell_coeff coeffs[O_G2_PREPARED_COEFFS];
    uint8_t infinity;
    uint8_t pad[7];
} o_g2_prepared;

#endif
