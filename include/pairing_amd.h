/*
 * pairing_amd -- MI355X-native batched BLS12-381 engine, C ABI.
 *
 * This is the drop-in boundary for the hot path of the Rust crate `pairing`
 * v0.14.2 (dignifiedquire/pairing).  The reference has no FFI of its own: its
 * interface is the Rust trait surface in src/lib.rs.  Each entry point below
 * names the trait method (reference file:line) it replaces, batched over n
 * independent items.  INTEGRATION.md shows the Rust `extern "C"` block a
 * maintainer would add to bind it.
 *
 * Data layout (host and device) is the Rust in-memory order of the reference
 * types, so a `&[G1Affine]` can be passed by pointer:
 *   Fq        = 6 x u64, little-endian limbs, Montgomery form (R = 2^384), < q
 *               (src/bls12_381/fq.rs:699-700)
 *   Fq2       = {c0, c1}            Fq6 = {c0, c1, c2}       Fq12 = {c0, c1}
 *   G1Affine  = {Fq x, Fq y, u8 infinity, 7 pad}   (104 B)   ec.rs:13-18
 *   G2Affine  = {Fq2 x, Fq2 y, u8 infinity, 7 pad} (200 B)
 *   G1 / G2   = Jacobian {x, y, z}, zero iff z == 0 (144 B / 288 B) ec.rs:31-36
 *   FrRepr    = 4 x u64 little-endian, canonical (not Montgomery) fr.rs:58
 *   G2Prepared= 68 x (Fq2, Fq2, Fq2) line coefficients + u8 infinity + 7 pad
 *               (ec.rs:1615-1619, built by mod.rs:168-358) = 19 592 B
 *
 * Conventions
 *   - Every function returns 0 (PA_OK) or a negative PA_ERR_* code; nothing
 *     aborts across the ABI.  pa_last_error() describes the last failure on
 *     the calling thread.
 *   - Per-item Option results (reference returns None) are reported through a
 *     caller-provided u8 `ok` array: 1 = Some, 0 = None.
 *   - Host-pointer functions (no suffix) are synchronous: they copy inputs to
 *     the current device, run, and copy outputs back.  The caller owns all
 *     buffers; nothing is retained after return.  `out` may alias an input of
 *     the same type (giving the reference's *_assign in-place semantics).
 *   - `_device` functions take device pointers and a hipStream_t (as void*,
 *     NULL = default stream) and return after enqueueing; inputs must stay
 *     valid until the stream reaches the work.
 *   - Thread safety: all entry points are reentrant (the reference traits are
 *     Send + Sync, lib.rs:114-121, 185-186).  The device used is the calling
 *     thread's current HIP device (pa_set_device).
 */
#ifndef PAIRING_AMD_H
#define PAIRING_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PA_OK 0
#define PA_ERR_INVALID_ARGUMENT (-1)
#define PA_ERR_HIP (-2)
#define PA_ERR_OUT_OF_MEMORY (-3)
#define PA_ERR_NO_DEVICE (-4)

#define PA_G2_PREPARED_COEFFS 68

typedef struct { uint64_t l[6]; } pa_fq;
typedef struct { pa_fq c0, c1; } pa_fq2;
typedef struct { pa_fq2 c0, c1, c2; } pa_fq6;
typedef struct { pa_fq6 c0, c1; } pa_fq12;
typedef struct { uint64_t l[4]; } pa_fr_repr;   /* canonical scalar, fr.rs:58 */
typedef struct { uint64_t l[6]; } pa_fq_repr;   /* canonical base-field words, FqRepr fq.rs:699-700 */
typedef struct { uint64_t l[4]; } pa_fr;        /* Montgomery form (R = 2^256), < r, fr.rs:247 */
typedef struct { pa_fq x, y; uint8_t infinity; uint8_t _pad[7]; } pa_g1_affine;
typedef struct { pa_fq2 x, y; uint8_t infinity; uint8_t _pad[7]; } pa_g2_affine;
typedef struct { pa_fq x, y, z; } pa_g1;
typedef struct { pa_fq2 x, y, z; } pa_g2;
typedef struct {
    pa_fq2 coeffs[PA_G2_PREPARED_COEFFS][3];
    uint8_t infinity;
    uint8_t _pad[7];
} pa_g2_prepared;

/* ---- runtime ---- */
const char *pa_version(void);
const char *pa_last_error(void);
int pa_device_count(int *count);
int pa_set_device(int device);
int pa_synchronize(void);
/* Tuning knob: which kernels run the Miller loop / final exponentiation
 * (identical results):
 *   0 = default, by batch size n: n <= PA_PQ_MIN (768) on the
 *       cooperative kernels (a four-wave quad-VM workgroup per pairing,
 *       kernels_coop.hip: the verifier shape, ~1.6 ms), n <= PA_PQ_MAX
 *       (4096) on the lane-group kernels (round 6, kernels_pair_quad.hip:
 *       one pairing per 32 lanes, rounds of up to 2048 pairings at ~3.8 ms;
 *       with PA_PQ_MAX = 0 the cooperative kernels run up to PA_COOP_MAX
 *       = 2304), n <= PA_PAIR_MAX
 *       (32768) on the generated kernels with a lane pair per pairing
 *       (~8.6-9.3 ms), n <= PA_PAIR_MAX + PA_TAIL_MAX (34816; round 6)
 *       as the first 32768 on lane pairs and the tail on a stream forked
 *       from the caller's -- on the cooperative kernels up to 832 tail
 *       pairings, the lane-group kernels above (32769 pairs in ~10.8 ms,
 *       34816 in ~13.0; not under stream capture, where the
 *       one-pairing-per-lane kernels run up to 34048, ~15.7 ms), larger
 *       batches on lane
 *       pairs again, two waves per SIMD (2^16 in ~15.7 ms; tools/pgen: own
 *       register allocation, code objects lib/pa_gen_*.hsaco, each loaded
 *       at its first use).  e(P, Q) entries (pa_pairing_batch, multi_pairing)
 *       run the pairing-only Miller loops (lane pairs and, round 6, one lane
 *       per pairing); the Miller-loop entries keep the reference's values and
 *       switch from one lane to lane pairs above 38912 (PA_ML_ONE_MAX)
 *   1 = generated kernels with a lane pair per pairing, every size (A/B)
 *   2 = cooperative kernels for every size (A/B, tests)
 *   3 = generated one-pairing-per-lane kernels for every size (A/B, tests)
 *   4 = cooperative kernels for every size on the round-2 one-wave VM
 *       (A/B, tests; added in round 3 -- 0 and 2 now run batches of up to
 *       PA_COOP_QUAD_MAX items on the four-wave quad VM, same results)
 *   5 = lane-group kernels for every size (round 6: one pairing per 32
 *       lanes, the tower's products batched into levels over 8 lane quads,
 *       kernels_pair_quad.hip; the Miller values are the reference's)
 * Process-wide; not part of the reference interface.
 * Behavior change in round 2: the numbering was 0 = hipcc lazy core,
 * 1 / 2 = hipcc 32-bit word kernels (one lane / two lanes), 3 = generated,
 * 4 / 5 = generated lane pairs / lazy reduction.  Those kernels are gone; the
 * values above now mean what is listed and anything outside 0..4 returns
 * PA_ERR_INVALID_ARGUMENT (4 was "lazy reduction" before round 2 and is the
 * one-wave cooperative VM since round 3). */
int pa_set_pairing_kernel(int variant);
/* Point-decoding kernel selection (A/B, tests): 0 = by batch size (default:
 * up to PA_DECODE_QUAD_MAX records, 8192 unless the environment says
 * otherwise, one record per group of lane quads -- the verifier's latency
 * form; larger batches one lane per record), 1 = one lane per record, 2 =
 * quad groups for every size.  Same statuses and outputs.  Process-wide; not
 * part of the reference interface. */
int pa_set_decode_kernel(int variant);

/* ---- Fq (src/bls12_381/fq.rs, Field trait src/lib.rs:267-325) ---- */
/* Field::mul_assign, fq.rs:909-960 + mont_reduce fq.rs:1036-1122 */
int pa_fq_mul_batch(const pa_fq *a, const pa_fq *b, pa_fq *out, size_t n);
/* Field::square, fq.rs:962-1016 */
int pa_fq_square_batch(const pa_fq *a, pa_fq *out, size_t n);
/* Field::add_assign / sub_assign, fq.rs:812-838 */
int pa_fq_add_batch(const pa_fq *a, const pa_fq *b, pa_fq *out, size_t n);
int pa_fq_sub_batch(const pa_fq *a, const pa_fq *b, pa_fq *out, size_t n);
/* Field::inverse, fq.rs:849-902 (ok[i] = 0 for a zero input) */
int pa_fq_inverse_batch(const pa_fq *a, pa_fq *out, uint8_t *ok, size_t n);
/* PrimeField::from_repr, fq.rs:747-756: ok[i] = 0 = Err(NotInField) when repr >= q (out[i] = 0);
 * otherwise out[i] = repr * R^2 (Montgomery form) */
int pa_fq_from_repr_batch(const pa_fq_repr *repr, pa_fq *out, uint8_t *ok, size_t n);
/* PrimeField::into_repr, fq.rs:758-775: the canonical words (mont_reduce of a) */
int pa_fq_into_repr_batch(const pa_fq *a, pa_fq_repr *out, size_t n);

/* ---- tower (fq2.rs, fq6.rs, fq12.rs) ---- */
int pa_fq2_mul_batch(const pa_fq2 *a, const pa_fq2 *b, pa_fq2 *out, size_t n);     /* fq2.rs:123-136 */
int pa_fq2_square_batch(const pa_fq2 *a, pa_fq2 *out, size_t n);                   /* fq2.rs:87-101 */
int pa_fq6_mul_batch(const pa_fq6 *a, const pa_fq6 *b, pa_fq6 *out, size_t n);     /* fq6.rs:199-248 */
int pa_fq12_mul_batch(const pa_fq12 *a, const pa_fq12 *b, pa_fq12 *out, size_t n); /* fq12.rs:116-130 */
int pa_fq12_square_batch(const pa_fq12 *a, pa_fq12 *out, size_t n);                /* fq12.rs:99-114 */
int pa_fq12_inverse_batch(const pa_fq12 *a, pa_fq12 *out, uint8_t *ok, size_t n);  /* fq12.rs:132-148 */
int pa_fq12_frobenius_map_batch(const pa_fq12 *a, pa_fq12 *out, size_t n, size_t power); /* fq12.rs:90-97 */
int pa_fq2_inverse_batch(const pa_fq2 *a, pa_fq2 *out, uint8_t *ok, size_t n);    /* fq2.rs:138-155 */
int pa_fq2_frobenius_map_batch(const pa_fq2 *a, pa_fq2 *out, size_t n, size_t power); /* fq2.rs:157-159 */
int pa_fq6_square_batch(const pa_fq6 *a, pa_fq6 *out, size_t n);                   /* fq6.rs:166-197 */
int pa_fq6_inverse_batch(const pa_fq6 *a, pa_fq6 *out, uint8_t *ok, size_t n);    /* fq6.rs:250-301 */
int pa_fq6_frobenius_map_batch(const pa_fq6 *a, pa_fq6 *out, size_t n, size_t power); /* fq6.rs:157-164 */
/* Field::pow, lib.rs:306-324, one exponent (exp_words u64, little-endian) for every element */
int pa_fq_pow_batch(const pa_fq *a, const uint64_t *exp, size_t exp_words, pa_fq *out, size_t n);
int pa_fq12_pow_batch(const pa_fq12 *a, const uint64_t *exp, size_t exp_words, pa_fq12 *out, size_t n);
/* Fq12::mul_by_014, fq12.rs:34-48 */
int pa_fq12_mul_by_014_batch(const pa_fq12 *a, const pa_fq2 *c0, const pa_fq2 *c1, const pa_fq2 *c4,
                             pa_fq12 *out, size_t n);

/* ---- G2 line precomputation: G2Prepared::from_affine, mod.rs:168-358 ---- */
int pa_g2_prepare_batch(const pa_g2_affine *q, pa_g2_prepared *out, size_t n);

/* ---- Engine (src/lib.rs:34-110, src/bls12_381/mod.rs:30-161) ---- */
/* n independent single-pair loops: out[i] = Bls12::miller_loop([(p[i], q[i])]) (mod.rs:40-102) */
int pa_miller_loop_batch(const pa_g1_affine *p, const pa_g2_prepared *q, pa_fq12 *out, size_t n);
/* One G2Prepared shared by every pair -- Engine::miller_loop takes &G2Prepared
 * references (lib.rs:88-96, Prepared: Clone lib.rs:192), so a caller may pass the
 * same prepared Q for each P (a verifying key's prepared gamma / delta):
 * out[i] = Bls12::miller_loop([(p[i], q)]) (mod.rs:40-102) for i < n, where `q`
 * is ONE record.  Its lines are staged once per call; no G2 arithmetic per pair.
 * Same bits as pa_miller_loop_batch with q repeated n times. */
int pa_miller_loop_shared_prepared(const pa_g1_affine *p, size_t n, const pa_g2_prepared *q, pa_fq12 *out);
/* Engine::miller_loop over n pairs: the product semantics of mod.rs:40-102 */
int pa_multi_miller_loop(const pa_g1_affine *p, const pa_g2_prepared *q, size_t n, pa_fq12 *out);
/* Engine::final_exponentiation, mod.rs:104-160; ok[i] = 0 iff in[i] == 0 */
int pa_final_exponentiation_batch(const pa_fq12 *in, pa_fq12 *out, uint8_t *ok, size_t n);
/* Engine::pairing, lib.rs:101-109: out[i] = e(p[i], q[i]) (prepare fused on device) */
int pa_pairing_batch(const pa_g1_affine *p, const pa_g2_affine *q, pa_fq12 *out, size_t n);

/* ---- G1 (config 3: parameter generation) ---- */
/* CurveProjective::batch_normalization, ec.rs:246-294, in place.  Zero and
 * already-normalized points are left untouched; others get z = 1. */
int pa_g1_batch_normalization(pa_g1 *v, size_t n);
/* Wnaf::new().base(*base, n).scalar(scalars[i]) for every i (wnaf.rs:93-107,
 * 169-178): out[i] = the reference's wNAF product of scalars[i] and base as a
 * Jacobian point (equal as a point to the reference's; representation-
 * independent PartialEq, ec.rs:45-85).  That is scalars[i] * base for every
 * 256-bit FrRepr except where the reference's wnaf_form wraps in add_nocarry
 * (wnaf.rs:30-35: s odd with bits w..255 all ones, w the window
 * recommended_wnaf_for_num_scalars(n)); there it is (s - 2^256) * base, which
 * these entries reproduce. */
int pa_g1_wnaf_fixed_base(const pa_g1 *base, const pa_fr_repr *scalars, size_t n, pa_g1 *out);
/* the same with the window given: Wnaf::new().base(*base, num_scalars) picks
 * window = recommended_wnaf_for_num_scalars(num_scalars) and .shared() copies
 * may then multiply any number n of scalars (wnaf.rs:93-107, 131-154);
 * window in 1..62 */
int pa_g1_wnaf_fixed_base_window(const pa_g1 *base, const pa_fr_repr *scalars, size_t n, int window, pa_g1 *out);

/* ---- CurveProjective / CurveAffine per-op batches, G1 and G2 ----
 * The `curve_impl!` group law (ec.rs:1-621) for both groups, one item per
 * lane, replaying the reference's formula sequence: Jacobian outputs equal
 * the reference's X, Y, Z words bit for bit (zero = z == 0; a zero produced
 * by P + (-P) keeps the x, y words the formulas leave, ec.rs:398, 477). */
/* CurveProjective::double, dbl-2009-l, ec.rs:296-354 */
int pa_g1_double_batch(const pa_g1 *a, pa_g1 *out, size_t n);
int pa_g2_double_batch(const pa_g2 *a, pa_g2 *out, size_t n);
/* CurveProjective::add_assign, add-2007-bl, ec.rs:356-444: out[i] = a[i] + b[i] */
int pa_g1_add_batch(const pa_g1 *a, const pa_g1 *b, pa_g1 *out, size_t n);
int pa_g2_add_batch(const pa_g2 *a, const pa_g2 *b, pa_g2 *out, size_t n);
/* CurveProjective::add_assign_mixed, madd-2007-bl, ec.rs:446-526 */
int pa_g1_add_mixed_batch(const pa_g1 *a, const pa_g1_affine *b, pa_g1 *out, size_t n);
int pa_g2_add_mixed_batch(const pa_g2 *a, const pa_g2_affine *b, pa_g2 *out, size_t n);
/* CurveProjective::negate, ec.rs:528-532 */
int pa_g1_negate_batch(const pa_g1 *a, pa_g1 *out, size_t n);
int pa_g2_negate_batch(const pa_g2 *a, pa_g2 *out, size_t n);
/* CurveProjective::sub_assign = negate + add_assign, lib.rs:156-160 */
int pa_g1_sub_batch(const pa_g1 *a, const pa_g1 *b, pa_g1 *out, size_t n);
int pa_g2_sub_batch(const pa_g2 *a, const pa_g2 *b, pa_g2 *out, size_t n);
/* CurveProjective::into_affine, ec.rs:586-619 (zero -> the point at infinity) */
int pa_g1_into_affine_batch(const pa_g1 *a, pa_g1_affine *out, size_t n);
int pa_g2_into_affine_batch(const pa_g2 *a, pa_g2_affine *out, size_t n);
/* CurveAffine::into_projective, ec.rs:570-582 */
int pa_g1_into_projective_batch(const pa_g1_affine *a, pa_g1 *out, size_t n);
int pa_g2_into_projective_batch(const pa_g2_affine *a, pa_g2 *out, size_t n);
/* PartialEq for the projective types, ec.rs:45-85 (representation independent:
 * X1 Z2^2 == X2 Z1^2 and Y1 Z2^3 == Y2 Z1^3; zero equals only zero):
 * eq[i] = 1 if a[i] == b[i], else 0 */
int pa_g1_eq_batch(const pa_g1 *a, const pa_g1 *b, uint8_t *eq, size_t n);
int pa_g2_eq_batch(const pa_g2 *a, const pa_g2 *b, uint8_t *eq, size_t n);
/* G2 CurveProjective::batch_normalization, ec.rs:246-294, in place */
int pa_g2_batch_normalization(pa_g2 *v, size_t n);
/* G2 Wnaf::new().base(*base, n).scalar(scalars[i]) (wnaf.rs:93-107, 169-178):
 * out[i] = the reference's wNAF product, equal as a point to the reference's
 * (PartialEq, ec.rs:45-85), including its add_nocarry wrap (wnaf.rs:30-35; see
 * pa_g1_wnaf_fixed_base); _window: the window given, 1..62 */
int pa_g2_wnaf_fixed_base(const pa_g2 *base, const pa_fr_repr *scalars, size_t n, pa_g2 *out);
int pa_g2_wnaf_fixed_base_window(const pa_g2 *base, const pa_fr_repr *scalars, size_t n, int window, pa_g2 *out);
/* Bit-exact Wnaf (wnaf.rs:1-179): the reference's window table chain
 * (wnaf_table, wnaf.rs:3-15), wnaf_form (:18-43) and wnaf_exp (:45-71), so the
 * Jacobian X, Y, Z words equal the reference's -- not only the point, as the
 * comb behind pa_g{1,2}_wnaf_fixed_base gives.  Slower than the comb (the
 * table is 2^(w-1) Jacobian entries, the multiply 256 doublings per scalar).
 * Fixed base: Wnaf::new().base(*base, num).scalar(scalars[i]) for every i
 * (wnaf.rs:93-107, 169-178); window 1..20, or 0 for
 * recommended_wnaf_for_num_scalars(n).  The table is rebuilt in parallel from
 * the chain's closed form (kernels_wnaf_exact.hip); a base whose chain takes a
 * special branch (outside G1) gets the serial chain. */
int pa_g1_wnaf_fixed_base_exact(const pa_g1 *base, const pa_fr_repr *scalars, size_t n, int window, pa_g1 *out);
int pa_g2_wnaf_fixed_base_exact(const pa_g2 *base, const pa_fr_repr *scalars, size_t n, int window, pa_g2 *out);
/* Fixed scalar: Wnaf::new().scalar(*scalar).base(bases[i]) for every i
 * (wnaf.rs:111-128, 156-166); window 1..12, or 0 for
 * recommended_wnaf_for_scalar(*scalar) */
int pa_g1_wnaf_fixed_scalar_exact(const pa_g1 *bases, size_t n, const pa_fr_repr *scalar, int window, pa_g1 *out);
int pa_g2_wnaf_fixed_scalar_exact(const pa_g2 *bases, size_t n, const pa_fr_repr *scalar, int window, pa_g2 *out);
/* device forms: `workspace` holds pa_wnaf_exact_workspace_bytes(group, n,
 * window, fixed_scalar) bytes (window as resolved: 1..20 / 1..12; the fixed-
 * scalar device form takes its window explicitly, its scalar being device memory) */
size_t pa_wnaf_exact_workspace_bytes(int group, size_t n, int window, int fixed_scalar);
int pa_g1_wnaf_fixed_base_exact_device(const pa_g1 *base, const pa_fr_repr *scalars, pa_g1 *out, size_t n,
                                       int window, void *workspace, size_t workspace_bytes, void *stream);
int pa_g2_wnaf_fixed_base_exact_device(const pa_g2 *base, const pa_fr_repr *scalars, pa_g2 *out, size_t n,
                                       int window, void *workspace, size_t workspace_bytes, void *stream);
int pa_g1_wnaf_fixed_scalar_exact_device(const pa_g1 *bases, size_t n, const pa_fr_repr *scalar, pa_g1 *out,
                                         int window, void *workspace, size_t workspace_bytes, void *stream);
int pa_g2_wnaf_fixed_scalar_exact_device(const pa_g2 *bases, size_t n, const pa_fr_repr *scalar, pa_g2 *out,
                                         int window, void *workspace, size_t workspace_bytes, void *stream);
/* CurveProjective::recommended_wnaf_for_scalar / _for_num_scalars
 * (lib.rs:166-174; G1 ec.rs:895-921, G2 ec.rs:1586-1612): the window the
 * reference's Wnaf would pick (returned as a positive int).  The GPU
 * fixed-base path does not depend on it (signed base-256 comb). */
int pa_g1_recommended_wnaf_for_scalar(const pa_fr_repr *scalar);
int pa_g2_recommended_wnaf_for_scalar(const pa_fr_repr *scalar);
int pa_g1_recommended_wnaf_for_num_scalars(size_t num_scalars);
int pa_g2_recommended_wnaf_for_num_scalars(size_t num_scalars);

/* ---- point encodings and square roots (SURVEY.md §8 f, rank 1) ----
 * Wire format of src/bls12_381/README.md "Serialization": big-endian
 * coordinates (G2: x.c1, x.c0, y.c1, y.c0), flag bits in byte 0 (bit 7
 * compressed, bit 6 infinity, bit 5 lexicographically largest y).  Record
 * sizes: G1 uncompressed 96 B, compressed 48 B; G2 192 B / 96 B.
 * status[i] is the GroupDecodingError (lib.rs:469-481) of record i: */
#define PA_DECODE_OK 0
#define PA_DECODE_NOT_ON_CURVE 1
#define PA_DECODE_NOT_IN_SUBGROUP 2
#define PA_DECODE_COORDINATE_X_C0 3   /* G1: "x coordinate"; G2: "x coordinate (c0)" */
#define PA_DECODE_COORDINATE_X_C1 4   /* G2: "x coordinate (c1)" */
#define PA_DECODE_COORDINATE_Y_C0 5   /* G1: "y coordinate"; G2: "y coordinate (c0)" */
#define PA_DECODE_COORDINATE_Y_C1 6   /* G2: "y coordinate (c1)" */
#define PA_DECODE_UNEXPECTED_COMPRESSION_MODE 7
#define PA_DECODE_UNEXPECTED_INFORMATION 8
/* EncodedPoint::into_affine (checked = 1: on-curve + subgroup checks,
 * ec.rs:662-668, 785-792, 1322-1332, 1448-1455) or into_affine_unchecked
 * (checked = 0).  Records that fail get status != 0 and out[i] = the point at
 * infinity. */
int pa_g1_decode_batch(const uint8_t *enc, size_t n, int compressed, int checked, pa_g1_affine *out,
                       uint8_t *status);
int pa_g2_decode_batch(const uint8_t *enc, size_t n, int compressed, int checked, pa_g2_affine *out,
                       uint8_t *status);
/* is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144, r * P == 0) for
 * affine points: ok[i] = 1 in the subgroup (infinity included), 0 not.
 * into_affine = into_affine_unchecked + is_on_curve + this check (ec.rs:676-684,
 * 786-793, 1323-1331, 1449-1457); for compressed encodings the unchecked
 * decode already rejects points off the curve, so decode(checked) ==
 * decode(unchecked) followed by this check (a failing point: status
 * PA_DECODE_NOT_IN_SUBGROUP, output the point at infinity).  Apart, a verifier
 * can start its pairing on the unchecked points while the check runs beside it
 * (bench.py --workload verify --decode).  Points off the curve: unspecified
 * (the reference's "assuming on curve"). */
int pa_g1_subgroup_check_batch(const pa_g1_affine *p, size_t n, uint8_t *ok);
int pa_g2_subgroup_check_batch(const pa_g2_affine *p, size_t n, uint8_t *ok);
/* EncodedPoint::from_affine (ec.rs:737-752, 839-867, 1398-1415, 1510-1539) */
int pa_g1_encode_batch(const pa_g1_affine *in, size_t n, int compressed, uint8_t *enc);
int pa_g2_encode_batch(const pa_g2_affine *in, size_t n, int compressed, uint8_t *enc);
/* SqrtField::sqrt, fq.rs:1147-1170 / fq2.rs:167-220; ok[i] = 0 for a non-residue */
int pa_fq_sqrt_batch(const pa_fq *a, pa_fq *out, uint8_t *ok, size_t n);
int pa_fq2_sqrt_batch(const pa_fq2 *a, pa_fq2 *out, uint8_t *ok, size_t n);

/* ---- multi-pairing and multi-device (SURVEY.md §8 b, e, f rank 2) ---- */
/* Engine::miller_loop over n (G1Affine, G2Affine) pairs -- prepare fused on
 * device -- = the product of the per-pair loops (mod.rs:40-102); then, for
 * pa_multi_pairing, Engine::final_exponentiation (mod.rs:104-160): the
 * batch-verification shape e(P_1,Q_1)...e(P_n,Q_n).  ok = 0 iff the product
 * Miller value is zero (None). */
int pa_multi_miller_loop_affine(const pa_g1_affine *p, const pa_g2_affine *q, size_t n, pa_fq12 *out);
int pa_multi_pairing(const pa_g1_affine *p, const pa_g2_affine *q, size_t n, pa_fq12 *out, uint8_t *ok);
/* pa_pairing_batch split over devices 0..ndev-1 of this process (contiguous
 * shards, one host thread per device); ndev <= pa_device_count.  The
 * environment variable PA_DEVICE_MAP (a comma list of device ordinals) maps
 * shard d to its d-th entry instead, e.g. "4,5,6,7"; then ndev <= its length. */
int pa_pairing_batch_multi_gpu(const pa_g1_affine *p, const pa_g2_affine *q, pa_fq12 *out, size_t n, int ndev);

/* ---- variable-base scalar multiplication and MSM (SURVEY.md §8 f, rank 3) ----
 * Scalars are FrRepr (canonical 4 x u64 LE; any 256-bit value, as the
 * reference's BitIterator takes).  Per-item outputs are Jacobian and equal
 * the reference's X, Y, Z words bit for bit. */
/* CurveAffine::mul, ec.rs:174-177 (mul_bits ec.rs:88-95): out[i] = s[i] * p[i] */
int pa_g1_affine_mul_batch(const pa_g1_affine *p, const pa_fr_repr *s, pa_g1 *out, size_t n);
int pa_g2_affine_mul_batch(const pa_g2_affine *p, const pa_fr_repr *s, pa_g2 *out, size_t n);
/* CurveProjective::mul_assign, ec.rs:534-553: out[i] = s[i] * p[i] (p Jacobian) */
int pa_g1_mul_assign_batch(const pa_g1 *p, const pa_fr_repr *s, pa_g1 *out, size_t n);
int pa_g2_mul_assign_batch(const pa_g2 *p, const pa_fr_repr *s, pa_g2 *out, size_t n);
/* Multi-scalar multiplication: *out = sum_i s[i] * bases[i] (Pippenger buckets
 * on the device), the prover's multiexp over CurveAffine::mul + add_assign.
 * The Jacobian result is equal as a point (PartialEq, ec.rs:45-85) to the
 * reference's sum; n = 0 gives the zero point.  n < 2^31. */
int pa_g1_multiexp(const pa_g1_affine *bases, const pa_fr_repr *s, size_t n, pa_g1 *out);
int pa_g2_multiexp(const pa_g2_affine *bases, const pa_fr_repr *s, size_t n, pa_g2 *out);
/* device workspace bytes for pa_g{1,2}_multiexp_device (group 1 or 2) */
size_t pa_multiexp_workspace_bytes(int group, size_t n);

/* ---- scalar field Fr (src/bls12_381/fr.rs; SURVEY.md §8 f, rank 4) ----
 * pa_fr = 4 x u64 LE limbs, Montgomery form with R = 2^256, < r: the
 * reference's `Fr` in memory.  Every result is canonical, so it equals the
 * reference's bit for bit. */
int pa_fr_mul_batch(const pa_fr *a, const pa_fr *b, pa_fr *out, size_t n);  /* mul_assign fr.rs:438-465 */
int pa_fr_square_batch(const pa_fr *a, pa_fr *out, size_t n);              /* square fr.rs:467-500 */
int pa_fr_add_batch(const pa_fr *a, const pa_fr *b, pa_fr *out, size_t n);  /* add_assign fr.rs:341-348 */
int pa_fr_sub_batch(const pa_fr *a, const pa_fr *b, pa_fr *out, size_t n);  /* sub_assign fr.rs:359-367 */
int pa_fr_double_batch(const pa_fr *a, pa_fr *out, size_t n);              /* double fr.rs:350-357 */
int pa_fr_negate_batch(const pa_fr *a, pa_fr *out, size_t n);              /* negate fr.rs:369-375 */
/* inverse fr.rs:377-431; ok[i] = 0 (None) for zero */
int pa_fr_inverse_batch(const pa_fr *a, pa_fr *out, uint8_t *ok, size_t n);
/* PrimeField::from_repr fr.rs:279-288; ok[i] = 0 = Err(NotInField) when repr >= r (out[i] = 0) */
int pa_fr_from_repr_batch(const pa_fr_repr *repr, pa_fr *out, uint8_t *ok, size_t n);
/* PrimeField::into_repr fr.rs:290-303 */
int pa_fr_into_repr_batch(const pa_fr *a, pa_fr_repr *out, size_t n);
/* Field::pow lib.rs:306-324 with one exponent (exp_words u64, LE) for every element */
int pa_fr_pow_batch(const pa_fr *a, const uint64_t *exp, size_t exp_words, pa_fr *out, size_t n);
/* SqrtField::legendre fr.rs:575-590: out[i] = 0 Zero, 1 QuadraticResidue, -1 QuadraticNonResidue */
int pa_fr_legendre_batch(const pa_fr *a, int8_t *out, size_t n);
/* SqrtField::sqrt fr.rs:592-646 (the reference's Tonelli-Shanks root); ok[i] = 0 (None) for a non-residue */
int pa_fr_sqrt_batch(const pa_fr *a, pa_fr *out, uint8_t *ok, size_t n);

/* ---- device-resident variants (pointers are device memory) ---- */
int pa_g1_decode_batch_device(const uint8_t *enc, size_t n, int compressed, int checked, pa_g1_affine *out,
                              uint8_t *status, void *stream);
int pa_g2_decode_batch_device(const uint8_t *enc, size_t n, int compressed, int checked, pa_g2_affine *out,
                              uint8_t *status, void *stream);
int pa_g1_subgroup_check_batch_device(const pa_g1_affine *p, size_t n, uint8_t *ok, void *stream);
int pa_g2_subgroup_check_batch_device(const pa_g2_affine *p, size_t n, uint8_t *ok, void *stream);
int pa_g1_batch_normalization_device(pa_g1 *v, size_t n, void *stream);
/* u64 words of the fixed-base table and of the scratch used to build it.  The
 * multiply stages below give the reference's wNAF point for the window
 * recommended_wnaf_for_num_scalars(n) (its add_nocarry wrap included, see
 * pa_g1_wnaf_fixed_base). */
size_t pa_g1_fixed_base_table_words(void);
size_t pa_g1_fixed_base_workspace_words(void);
int pa_g1_fixed_base_table_device(const pa_g1 *base, uint64_t *table, uint64_t *workspace, void *stream);
int pa_g1_fixed_base_mul_device(const uint64_t *table, const pa_fr_repr *scalars, pa_g1 *out, size_t n,
                                void *stream);
/* The same product in its GLV form as two stream-ordered stages (s = q x^2 + rem, s P = rem P - q phi(P) when
 * phi(P) == -[x^2] P; the table's 17 base rows plus their phi images and a membership flag in `workspace`); the
 * multiply stage falls back to a double-and-add from `base` when the flag says the base failed the check.  Equal as points to pa_g1_fixed_base_table_device + pa_g1_fixed_base_mul_device. */
int pa_g1_fixed_base_glv_table_device(const pa_g1 *base, uint64_t *table, uint64_t *workspace, void *stream);
int pa_g1_fixed_base_glv_mul_device(const pa_g1 *base, const uint64_t *table, const uint64_t *workspace,
                                    const pa_fr_repr *scalars, pa_g1 *out, size_t n, void *stream);
/* Wnaf::new().base(base, n).scalar(s_i) for every i (wnaf.rs:93-107, 169-178) in one call: the GLV table build
 * and multiply with the table's serial base chain overlapped (per-device side streams, ordered after `stream` by
 * events); equal as points to pa_g1_fixed_base_table_device + pa_g1_fixed_base_mul_device. */
int pa_g1_wnaf_fixed_base_device(const pa_g1 *base, const pa_fr_repr *scalars, pa_g1 *out, size_t n,
                                 uint64_t *table, uint64_t *workspace, void *stream);
int pa_g1_wnaf_fixed_base_window_device(const pa_g1 *base, const pa_fr_repr *scalars, pa_g1 *out, size_t n,
                                        int window, uint64_t *table, uint64_t *workspace, void *stream);
int pa_fq_mul_batch_device(const pa_fq *a, const pa_fq *b, pa_fq *out, size_t n, void *stream);
/* Fq::mul_assign (fq.rs:909-960) on the SoA device layout of SURVEY.md 8(d) config 2: u64 word j
 * (0..5, little-endian, Montgomery, < q) of element i at a[j * n + i]; same bits as the AoS form */
int pa_fq_mul_batch_soa_device(const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n, void *stream);
int pa_fr_mul_batch_device(const pa_fr *a, const pa_fr *b, pa_fr *out, size_t n, void *stream);
int pa_g1_multiexp_device(const pa_g1_affine *bases, const pa_fr_repr *s, size_t n, pa_g1 *out, void *workspace,
                          size_t workspace_bytes, void *stream);
int pa_g2_multiexp_device(const pa_g2_affine *bases, const pa_fr_repr *s, size_t n, pa_g2 *out, void *workspace,
                          size_t workspace_bytes, void *stream);
/* G2 batch_normalization and fixed-base multiply on device memory; the G2
 * table / workspace hold pa_g2_fixed_base_table_words() /
 * pa_g2_fixed_base_workspace_words() u64 */
int pa_g2_batch_normalization_device(pa_g2 *v, size_t n, void *stream);
size_t pa_g2_fixed_base_table_words(void);
size_t pa_g2_fixed_base_workspace_words(void);
int pa_g2_wnaf_fixed_base_device(const pa_g2 *base, const pa_fr_repr *scalars, pa_g2 *out, size_t n,
                                 uint64_t *table, uint64_t *workspace, void *stream);
int pa_g2_wnaf_fixed_base_window_device(const pa_g2 *base, const pa_fr_repr *scalars, pa_g2 *out, size_t n,
                                        int window, uint64_t *table, uint64_t *workspace, void *stream);
/* group law on device memory (see the host batches above) */
int pa_g1_double_batch_device(const pa_g1 *a, pa_g1 *out, size_t n, void *stream);
int pa_g2_double_batch_device(const pa_g2 *a, pa_g2 *out, size_t n, void *stream);
int pa_g1_add_batch_device(const pa_g1 *a, const pa_g1 *b, pa_g1 *out, size_t n, void *stream);
int pa_g2_add_batch_device(const pa_g2 *a, const pa_g2 *b, pa_g2 *out, size_t n, void *stream);
int pa_g1_add_mixed_batch_device(const pa_g1 *a, const pa_g1_affine *b, pa_g1 *out, size_t n, void *stream);
int pa_g2_add_mixed_batch_device(const pa_g2 *a, const pa_g2_affine *b, pa_g2 *out, size_t n, void *stream);
int pa_g1_into_affine_batch_device(const pa_g1 *a, pa_g1_affine *out, size_t n, void *stream);
int pa_g2_into_affine_batch_device(const pa_g2 *a, pa_g2_affine *out, size_t n, void *stream);
int pa_g1_eq_batch_device(const pa_g1 *a, const pa_g1 *b, uint8_t *eq, size_t n, void *stream);
int pa_g2_eq_batch_device(const pa_g2 *a, const pa_g2 *b, uint8_t *eq, size_t n, void *stream);
int pa_miller_loop_fused_batch_device(const pa_g1_affine *p, const pa_g2_affine *q, pa_fq12 *out, size_t n,
                                      void *stream);
/* The first stage of pa_pairing_batch_device, on its own (so a caller can time
 * or overlap the two stages): Miller values from which
 * pa_final_exponentiation_batch_device gives exactly e(p[i], q[i]).  They equal
 * the reference's miller_loop values only up to an Fq2 factor per pair (the
 * lane-pair kernel's G2 steps use homogeneous coordinates and their own line
 * scaling; the final exponentiation removes any Fq2 factor, since
 * (q^12 - 1) / r is a multiple of q^2 - 1), so do not use them as Miller
 * values -- pa_miller_loop_fused_batch_device gives those. */
int pa_pairing_miller_loop_batch_device(const pa_g1_affine *p, const pa_g2_affine *q, pa_fq12 *out, size_t n,
                                        void *stream);
/* final_exponentiation (mod.rs:104-160) on device records: one kernel launch
 * on `stream` (the cooperative kernel up to PA_COOP_MAX records, the generated
 * one above); `out` may equal `in` (in place) or lie apart from it, in which
 * case `in` is left unchanged.  ok[i] = 0 iff in[i] == 0 (None). */
int pa_final_exponentiation_batch_device(const pa_fq12 *in, pa_fq12 *out, uint8_t *ok, size_t n, void *stream);
/* pa_multi_pairing on device memory (the verifier's check without host copies); `work` holds n
 * pa_fq12 (the per-pair Miller values, reduced in place to their product) */
int pa_multi_pairing_device(const pa_g1_affine *p, const pa_g2_affine *q, size_t n, pa_fq12 *out, uint8_t *ok,
                            pa_fq12 *work, void *stream);
/* G2Prepared::from_affine (mod.rs:168-358) and miller_loop over (G1Affine,
 * G2Prepared) pairs (mod.rs:40-102) on device records: the north-star form
 * whose line coefficients are materialized in HBM (19 592 B per point).
 * Same records and bits as pa_g2_prepare_batch / pa_miller_loop_batch. */
int pa_g2_prepare_batch_device(const pa_g2_affine *q, pa_g2_prepared *out, size_t n, void *stream);
int pa_miller_loop_batch_device(const pa_g1_affine *p, const pa_g2_prepared *q, pa_fq12 *out, size_t n,
                                void *stream);
/* pa_miller_loop_shared_prepared on device records (p: n records, q: one) */
int pa_miller_loop_shared_prepared_device(const pa_g1_affine *p, size_t n, const pa_g2_prepared *q,
                                          pa_fq12 *out, void *stream);
/* e(p[i], q[i]); `scratch` must hold n pa_fq12 (the Miller-loop values) */
int pa_pairing_batch_device(const pa_g1_affine *p, const pa_g2_affine *q, pa_fq12 *out, pa_fq12 *scratch,
                            size_t n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PAIRING_AMD_H */
