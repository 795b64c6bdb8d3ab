"""pairing_amd -- MI355X-native batched BLS12-381 engine.

The batched counterpart of the Rust crate `pairing` v0.14.2 hot path
(dignifiedquire/pairing): Fq Montgomery multiply, the Fq2/Fq6/Fq12 tower,
G2 line precomputation (`G2Prepared`), `miller_loop` and
`final_exponentiation`, all as hand-written HIP kernels for gfx950 behind
the C ABI of include/pairing_amd.h.

Two layers:
  * batch functions over numpy arrays in the ABI layout (this module), e.g.
    `pairing(p, q)` for n independent pairs;
  * include/pairing_amd.hpp: the C++ mirror of the reference's trait surface
    (`Bls12::pairing`, `Bls12::miller_loop`, `G1Affine::prepare`,
    `G1Compressed::into_affine`, `Wnaf`, ...) over the same C ABI.
Device-resident entry points for torch tensors live in `pairing_amd.device`.
"""
import numpy as np

from ._native import (W_FQ, W_FQ2, W_FQ6, W_FQ12, W_FR, W_G1A, W_G1, W_G2A, W_G2, W_G2P, PairingError, _lib,
                      as_rows, call, device_count, ptr, set_decode_kernel, set_device, set_pairing_kernel, version)

__all__ = [
    "PairingError", "version", "device_count", "set_device", "set_pairing_kernel", "set_decode_kernel",
    "fq_mul", "fq_square", "fq_add", "fq_sub", "fq_inverse", "fq_from_repr", "fq_into_repr",
    "fq2_mul", "fq2_square", "fq6_mul", "fq12_mul", "fq12_square", "fq12_inverse",
    "fq12_frobenius_map", "fq12_cyclotomic_square", "fq12_mul_by_014",
    "fq2_inverse", "fq2_frobenius_map", "fq6_square", "fq6_inverse", "fq6_frobenius_map", "fq_pow", "fq12_pow",
    "g1_batch_normalization", "g1_wnaf_fixed_base",
    "g2_prepare", "miller_loop_batch", "miller_loop_shared_prepared", "multi_miller_loop", "final_exponentiation", "pairing",
    "multi_miller_loop_affine", "multi_pairing", "pairing_multi_gpu",
    "fq_sqrt", "fq2_sqrt", "g1_decode", "g2_decode", "g1_encode", "g2_encode", "DECODE_STATUS",
    "g1_subgroup_check", "g2_subgroup_check",
    "fr_mul", "fr_square", "fr_add", "fr_sub", "fr_double", "fr_negate", "fr_inverse",
    "fr_from_repr", "fr_into_repr", "fr_pow", "fr_legendre", "fr_sqrt",
    "g1_affine_mul", "g2_affine_mul", "g1_mul_assign", "g2_mul_assign", "g1_multiexp", "g2_multiexp",
    "g1_eq", "g2_eq", "g1_double", "g2_double", "g1_add", "g2_add", "g1_add_mixed", "g2_add_mixed", "g1_negate", "g2_negate",
    "g1_sub", "g2_sub", "g1_into_affine", "g2_into_affine", "g1_into_projective", "g2_into_projective",
    "g2_batch_normalization", "g2_wnaf_fixed_base",
    "g1_wnaf_fixed_base_exact", "g2_wnaf_fixed_base_exact", "g1_wnaf_fixed_scalar_exact", "g2_wnaf_fixed_scalar_exact",
    "g1_recommended_wnaf_for_scalar", "g2_recommended_wnaf_for_scalar",
    "g1_recommended_wnaf_for_num_scalars", "g2_recommended_wnaf_for_num_scalars",
]


def _binary(name, a, b, width):
    a = as_rows(a, width, "a")
    b = as_rows(b, width, "b")
    if a.shape != b.shape:
        raise ValueError("operand shapes differ: %s vs %s" % (a.shape, b.shape))
    out = np.empty_like(a)
    call(name, ptr(a), ptr(b), ptr(out), a.shape[0])
    return out


def _unary(name, a, width):
    a = as_rows(a, width, "a")
    out = np.empty_like(a)
    call(name, ptr(a), ptr(out), a.shape[0])
    return out


def _inverse(name, a, width):
    a = as_rows(a, width, "a")
    out = np.empty_like(a)
    ok = np.zeros(a.shape[0], np.uint8)
    call(name, ptr(a), ptr(out), ptr(ok), a.shape[0])
    return out, ok.astype(bool)


# ---- Fq: src/bls12_381/fq.rs ----
def fq_mul(a, b):
    """Fq::mul_assign (fq.rs:909-960) elementwise."""
    return _binary("pa_fq_mul_batch", a, b, W_FQ)


def fq_square(a):
    """Fq::square (fq.rs:962-1016)."""
    return _unary("pa_fq_square_batch", a, W_FQ)


def fq_add(a, b):
    return _binary("pa_fq_add_batch", a, b, W_FQ)


def fq_sub(a, b):
    return _binary("pa_fq_sub_batch", a, b, W_FQ)


def fq_inverse(a):
    """Fq::inverse (fq.rs:849-902): (values, ok) with ok False where the reference returns None."""
    return _inverse("pa_fq_inverse_batch", a, W_FQ)


def fq_from_repr(repr_rows):
    """PrimeField::from_repr (fq.rs:747-756): (values, ok), ok False = Err(NotInField) (repr >= q)."""
    r = as_rows(repr_rows, W_FQ, "repr")
    out = np.empty_like(r)
    ok = np.zeros(r.shape[0], np.uint8)
    call("pa_fq_from_repr_batch", ptr(r), ptr(out), ptr(ok), r.shape[0])
    return out, ok.astype(bool)


def fq_into_repr(a):
    """PrimeField::into_repr (fq.rs:758-775): canonical FqRepr rows."""
    return _unary("pa_fq_into_repr_batch", a, W_FQ)


# ---- tower ----
def fq2_mul(a, b):
    return _binary("pa_fq2_mul_batch", a, b, W_FQ2)


def fq2_square(a):
    return _unary("pa_fq2_square_batch", a, W_FQ2)


def fq6_mul(a, b):
    return _binary("pa_fq6_mul_batch", a, b, W_FQ6)


def fq12_mul(a, b):
    return _binary("pa_fq12_mul_batch", a, b, W_FQ12)


def fq12_square(a):
    return _unary("pa_fq12_square_batch", a, W_FQ12)


def fq12_cyclotomic_square(a):
    """Granger-Scott squaring; equals fq12_square for elements of the cyclotomic subgroup."""
    return _unary("pa_fq12_cyclotomic_square_batch", a, W_FQ12)


def fq12_inverse(a):
    return _inverse("pa_fq12_inverse_batch", a, W_FQ12)


def fq2_inverse(a):
    """Fq2::inverse (fq2.rs:138-155): (values, ok)."""
    return _inverse("pa_fq2_inverse_batch", a, W_FQ2)


def fq2_frobenius_map(a, power):
    """Fq2::frobenius_map (fq2.rs:157-159)."""
    return _frob("pa_fq2_frobenius_map_batch", a, W_FQ2, power)


def fq6_square(a):
    """Fq6::square (fq6.rs:166-197)."""
    return _unary("pa_fq6_square_batch", a, W_FQ6)


def fq6_inverse(a):
    """Fq6::inverse (fq6.rs:250-301): (values, ok)."""
    return _inverse("pa_fq6_inverse_batch", a, W_FQ6)


def fq6_frobenius_map(a, power):
    """Fq6::frobenius_map (fq6.rs:157-164)."""
    return _frob("pa_fq6_frobenius_map_batch", a, W_FQ6, power)


def _frob(name, a, width, power):
    a = as_rows(a, width, "a")
    out = np.empty_like(a)
    call(name, ptr(a), ptr(out), a.shape[0], int(power))
    return out


def _pow(name, a, width, exp_limbs):
    a = as_rows(a, width, "a")
    e = np.ascontiguousarray(np.asarray(exp_limbs, dtype=np.uint64).reshape(-1))
    out = np.empty_like(a)
    call(name, ptr(a), ptr(e), e.size, ptr(out), a.shape[0])
    return out


def fq_pow(a, exp_limbs):
    """Field::pow (lib.rs:306-324) for Fq, one exponent (u64 LE limbs) for every element."""
    return _pow("pa_fq_pow_batch", a, W_FQ, exp_limbs)


def fq12_pow(a, exp_limbs):
    """Field::pow (lib.rs:306-324) for Fq12."""
    return _pow("pa_fq12_pow_batch", a, W_FQ12, exp_limbs)


def fq12_frobenius_map(a, power):
    a = as_rows(a, W_FQ12, "a")
    out = np.empty_like(a)
    call("pa_fq12_frobenius_map_batch", ptr(a), ptr(out), a.shape[0], int(power))
    return out


def fq12_mul_by_014(a, c0, c1, c4):
    """Fq12::mul_by_014 (fq12.rs:34-48)."""
    a = as_rows(a, W_FQ12, "a")
    c0, c1, c4 = (as_rows(c, W_FQ2, "c") for c in (c0, c1, c4))
    out = np.empty_like(a)
    call("pa_fq12_mul_by_014_batch", ptr(a), ptr(c0), ptr(c1), ptr(c4), ptr(out), a.shape[0])
    return out


# ---- engine: src/bls12_381/mod.rs ----
def g2_prepare(q):
    """G2Prepared::from_affine (mod.rs:168-358) for each G2 affine point."""
    q = as_rows(q, W_G2A, "q")
    out = np.empty((q.shape[0], W_G2P), np.uint64)
    call("pa_g2_prepare_batch", ptr(q), ptr(out), q.shape[0])
    return out


def miller_loop_batch(p, q_prepared):
    """out[i] = Bls12::miller_loop([(p[i], q[i])]) -- n independent loops."""
    p = as_rows(p, W_G1A, "p")
    q = as_rows(q_prepared, W_G2P, "q_prepared")
    if p.shape[0] != q.shape[0]:
        raise ValueError("p and q_prepared lengths differ")
    out = np.empty((p.shape[0], W_FQ12), np.uint64)
    call("pa_miller_loop_batch", ptr(p), ptr(q), ptr(out), p.shape[0])
    return out


def miller_loop_shared_prepared(p, q_prepared):
    """out[i] = Bls12::miller_loop([(p[i], q)]) for ONE prepared q shared by every
    p[i] (lib.rs:88-96 called with the same &G2Prepared; mod.rs:40-102): the
    verifier's fixed-key shape.  q_prepared: one record, shape (W_G2P,) or (1, W_G2P)."""
    p = as_rows(p, W_G1A, "p")
    q = as_rows(q_prepared, W_G2P, "q_prepared")
    if q.shape[0] != 1:
        raise ValueError("q_prepared must be ONE G2Prepared record")
    out = np.empty((p.shape[0], W_FQ12), np.uint64)
    call("pa_miller_loop_shared_prepared", ptr(p), p.shape[0], ptr(q), ptr(out))
    return out


def multi_miller_loop(p, q_prepared):
    """Engine::miller_loop over all pairs: the product (mod.rs:40-102)."""
    p = as_rows(p, W_G1A, "p") if len(p) else np.zeros((0, W_G1A), np.uint64)
    q = as_rows(q_prepared, W_G2P, "q_prepared") if len(q_prepared) else np.zeros((0, W_G2P), np.uint64)
    if p.shape[0] != q.shape[0]:
        raise ValueError("p and q_prepared lengths differ")
    out = np.empty((1, W_FQ12), np.uint64)
    call("pa_multi_miller_loop", ptr(p), ptr(q), p.shape[0], ptr(out))
    return out[0]


def final_exponentiation(f):
    """Engine::final_exponentiation (mod.rs:104-160): (values, ok); ok False iff f == 0."""
    f = as_rows(f, W_FQ12, "f")
    out = np.empty_like(f)
    ok = np.zeros(f.shape[0], np.uint8)
    call("pa_final_exponentiation_batch", ptr(f), ptr(out), ptr(ok), f.shape[0])
    return out, ok.astype(bool)


def pairing(p, q, out=None):
    """Engine::pairing (lib.rs:101-109) for n independent (G1Affine, G2Affine) pairs.
    `out`: an optional (n, 72) uint64 C-contiguous array to write into -- a caller
    that reuses it saves the first-touch page faults of a fresh 37.7 MB result
    per 2^16 pairs (tools/pcie_rate.py measures both)."""
    p = as_rows(p, W_G1A, "p")
    q = as_rows(q, W_G2A, "q")
    if p.shape[0] != q.shape[0]:
        raise ValueError("p and q lengths differ")
    if out is None:
        out = np.empty((p.shape[0], W_FQ12), np.uint64)
    elif (not isinstance(out, np.ndarray) or out.dtype != np.uint64 or out.shape != (p.shape[0], W_FQ12)
          or not out.flags.c_contiguous or not out.flags.writeable):
        raise ValueError("out must be a writeable C-contiguous (%d, %d) uint64 array" % (p.shape[0], W_FQ12))
    call("pa_pairing_batch", ptr(p), ptr(q), ptr(out), p.shape[0])
    return out


# ---- G1 parameter-generation path (config 3) ----
def g1_batch_normalization(v):
    """CurveProjective::batch_normalization (ec.rs:246-294); returns the normalized copy."""
    v = as_rows(v, W_G1, "v").copy()
    call("pa_g1_batch_normalization", ptr(v), v.shape[0])
    return v


def g1_wnaf_fixed_base(base, scalars, window=None):
    """Wnaf::new().base(base, n).scalar(s) for each FrRepr scalar (wnaf.rs:93-107,
    169-178): Jacobian points equal to the reference's wNAF products -- s_i *
    base, or (s_i - 2^256) * base where its wnaf_form wraps (wnaf.rs:30-35).
    `window`: the table's window (default recommended_wnaf_for_num_scalars(n))."""
    b = as_rows(base, W_G1, "base")
    s = as_rows(scalars, 4, "scalars")
    out = np.empty((s.shape[0], W_G1), np.uint64)
    if window is None:
        call("pa_g1_wnaf_fixed_base", ptr(b), ptr(s), s.shape[0], ptr(out))
    else:
        call("pa_g1_wnaf_fixed_base_window", ptr(b), ptr(s), s.shape[0], int(window), ptr(out))
    return out


def _wnaf_exact(group, fixed_scalar, bases, scalars, window):
    wj = W_G1 if group == 1 else W_G2
    b = as_rows(bases, wj, "base" if not fixed_scalar else "bases")
    s = as_rows(scalars, 4, "scalar" if fixed_scalar else "scalars")
    # the fixed operand is ONE record (Wnaf::base(g, ..) / Wnaf::scalar(s)); a
    # second row would be ignored silently, so refuse it
    if fixed_scalar and s.shape[0] != 1:
        raise ValueError("scalar: expected exactly one record, got %d" % s.shape[0])
    if not fixed_scalar and b.shape[0] != 1:
        raise ValueError("base: expected exactly one record, got %d" % b.shape[0])
    n = b.shape[0] if fixed_scalar else s.shape[0]
    out = np.empty((n, wj), np.uint64)
    w = 0 if window is None else int(window)
    if fixed_scalar:
        call("pa_g%d_wnaf_fixed_scalar_exact" % group, ptr(b), n, ptr(s), w, ptr(out))
    else:
        call("pa_g%d_wnaf_fixed_base_exact" % group, ptr(b), ptr(s), n, w, ptr(out))
    return out


def g1_wnaf_fixed_base_exact(base, scalars, window=None):
    """Wnaf::new().base(base, n).scalar(s_i) with the reference's exact table chain,
    wnaf_form and wnaf_exp (wnaf.rs:1-179): Jacobian words bit-identical to the
    reference's.  `window`: 1..20 (default recommended_wnaf_for_num_scalars(n))."""
    return _wnaf_exact(1, False, base, scalars, window)


def g2_wnaf_fixed_base_exact(base, scalars, window=None):
    """G2 form of g1_wnaf_fixed_base_exact."""
    return _wnaf_exact(2, False, base, scalars, window)


def g1_wnaf_fixed_scalar_exact(bases, scalar, window=None):
    """Wnaf::new().scalar(s).base(g_i) (wnaf.rs:111-128, 156-166) for every Jacobian
    base, bit-identical Jacobian words.  `window`: 1..12 (default
    recommended_wnaf_for_scalar(s))."""
    return _wnaf_exact(1, True, bases, scalar, window)


def g2_wnaf_fixed_scalar_exact(bases, scalar, window=None):
    """G2 form of g1_wnaf_fixed_scalar_exact."""
    return _wnaf_exact(2, True, bases, scalar, window)


# ---- multi-pairing (SURVEY.md §8 f rank 2) and in-process multi-device ----
def _pairs(p, q):
    p = as_rows(p, W_G1A, "p") if len(p) else np.zeros((0, W_G1A), np.uint64)
    q = as_rows(q, W_G2A, "q") if len(q) else np.zeros((0, W_G2A), np.uint64)
    if p.shape[0] != q.shape[0]:
        raise ValueError("p and q lengths differ")
    return p, q


def multi_miller_loop_affine(p, q):
    """Engine::miller_loop over (G1Affine, G2Affine) pairs, prepare fused on device:
    the product of the per-pair loops (mod.rs:40-102)."""
    p, q = _pairs(p, q)
    out = np.empty((1, W_FQ12), np.uint64)
    call("pa_multi_miller_loop_affine", ptr(p), ptr(q), p.shape[0], ptr(out))
    return out[0]


def multi_pairing(p, q):
    """final_exponentiation(miller_loop(pairs)) -- the batch-verification product
    e(P_1,Q_1)...e(P_n,Q_n); returns (Fq12, ok)."""
    p, q = _pairs(p, q)
    out = np.empty((1, W_FQ12), np.uint64)
    ok = np.zeros(1, np.uint8)
    call("pa_multi_pairing", ptr(p), ptr(q), p.shape[0], ptr(out), ptr(ok))
    return out[0], bool(ok[0])


def pairing_multi_gpu(p, q, ndev):
    """pairing(p, q) split over devices 0..ndev-1 of this process."""
    p, q = _pairs(p, q)
    out = np.empty((p.shape[0], W_FQ12), np.uint64)
    call("pa_pairing_batch_multi_gpu", ptr(p), ptr(q), ptr(out), p.shape[0], int(ndev))
    return out


# ---- square roots and point encodings (SURVEY.md §8 f rank 1) ----
# status byte -> GroupDecodingError (lib.rs:469-481)
DECODE_STATUS = {
    0: "Ok", 1: "NotOnCurve", 2: "NotInSubgroup",
    3: "CoordinateDecodingError(x / x.c0)", 4: "CoordinateDecodingError(x.c1)",
    5: "CoordinateDecodingError(y / y.c0)", 6: "CoordinateDecodingError(y.c1)",
    7: "UnexpectedCompressionMode", 8: "UnexpectedInformation",
}
ENCODED_SIZE = {(1, False): 96, (1, True): 48, (2, False): 192, (2, True): 96}


def fq_sqrt(a):
    """SqrtField::sqrt for Fq (fq.rs:1147-1170): (roots, ok); ok False for non-residues."""
    return _inverse("pa_fq_sqrt_batch", a, W_FQ)


def fq2_sqrt(a):
    """SqrtField::sqrt for Fq2 (fq2.rs:167-220): (roots, ok)."""
    return _inverse("pa_fq2_sqrt_batch", a, W_FQ2)


def _decode(group, enc, compressed, checked):
    size = ENCODED_SIZE[(group, bool(compressed))]
    enc = np.ascontiguousarray(np.asarray(enc, dtype=np.uint8))
    if enc.ndim == 1:
        enc = enc.reshape(-1, size)
    if enc.ndim != 2 or enc.shape[1] != size:
        raise ValueError("encodings must have shape (n, %d), got %s" % (size, enc.shape))
    n = enc.shape[0]
    out = np.empty((n, W_G1A if group == 1 else W_G2A), np.uint64)
    status = np.zeros(n, np.uint8)
    call("pa_g%d_decode_batch" % group, ptr(enc), n, int(bool(compressed)), int(bool(checked)), ptr(out),
         ptr(status))
    return out, status


def g1_decode(enc, compressed, checked=True):
    """G1Uncompressed / G1Compressed ::into_affine (checked) or ::into_affine_unchecked
    (ec.rs:662-837) for (n, 96|48) uint8 records: (affine points, status bytes)."""
    return _decode(1, enc, compressed, checked)


def g2_decode(enc, compressed, checked=True):
    """G2Uncompressed / G2Compressed ::into_affine[_unchecked] (ec.rs:1322-1509)."""
    return _decode(2, enc, compressed, checked)


def _subgroup(group, pts):
    pts = as_rows(pts, W_G1A if group == 1 else W_G2A, "points")
    ok = np.zeros(pts.shape[0], np.uint8)
    call("pa_g%d_subgroup_check_batch" % group, ptr(pts), pts.shape[0], ptr(ok))
    return ok.astype(bool)


def g1_subgroup_check(pts):
    """is_in_correct_subgroup_assuming_on_curve (ec.rs:142-144) for (n, 13) affine
    rows: True where r * P == 0 (infinity included); unspecified off the curve."""
    return _subgroup(1, pts)


def g2_subgroup_check(pts):
    """is_in_correct_subgroup_assuming_on_curve for (n, 25) G2 affine rows."""
    return _subgroup(2, pts)


def _encode(group, pts, compressed):
    pts = as_rows(pts, W_G1A if group == 1 else W_G2A, "points")
    size = ENCODED_SIZE[(group, bool(compressed))]
    enc = np.zeros((pts.shape[0], size), np.uint8)
    call("pa_g%d_encode_batch" % group, ptr(pts), pts.shape[0], int(bool(compressed)), ptr(enc))
    return enc


def g1_encode(pts, compressed):
    """EncodedPoint::from_affine for G1 (ec.rs:737-752, 839-867)."""
    return _encode(1, pts, compressed)


def g2_encode(pts, compressed):
    """EncodedPoint::from_affine for G2 (ec.rs:1398-1415, 1510-1539)."""
    return _encode(2, pts, compressed)


# ---- Fr: src/bls12_381/fr.rs (rows (n,4): Montgomery Fr or canonical FrRepr) ----
def fr_mul(a, b):
    """Fr::mul_assign (fr.rs:438-465) elementwise."""
    return _binary("pa_fr_mul_batch", a, b, W_FR)


def fr_square(a):
    """Fr::square (fr.rs:467-500)."""
    return _unary("pa_fr_square_batch", a, W_FR)


def fr_add(a, b):
    """Fr::add_assign (fr.rs:341-348)."""
    return _binary("pa_fr_add_batch", a, b, W_FR)


def fr_sub(a, b):
    """Fr::sub_assign (fr.rs:359-367)."""
    return _binary("pa_fr_sub_batch", a, b, W_FR)


def fr_double(a):
    """Fr::double (fr.rs:350-357)."""
    return _unary("pa_fr_double_batch", a, W_FR)


def fr_negate(a):
    """Fr::negate (fr.rs:369-375)."""
    return _unary("pa_fr_negate_batch", a, W_FR)


def fr_inverse(a):
    """Fr::inverse (fr.rs:377-431): (values, ok), ok False where the reference returns None."""
    return _inverse("pa_fr_inverse_batch", a, W_FR)


def fr_from_repr(repr_rows):
    """PrimeField::from_repr (fr.rs:279-288): (values, ok), ok False = Err(NotInField)."""
    r = as_rows(repr_rows, W_FR, "repr")
    out = np.empty_like(r)
    ok = np.zeros(r.shape[0], np.uint8)
    call("pa_fr_from_repr_batch", ptr(r), ptr(out), ptr(ok), r.shape[0])
    return out, ok.astype(bool)


def fr_into_repr(a):
    """PrimeField::into_repr (fr.rs:290-303): canonical FrRepr rows."""
    return _unary("pa_fr_into_repr_batch", a, W_FR)


def fr_pow(a, exp_limbs):
    """Field::pow (lib.rs:306-324) of every element by one exponent (u64 LE limbs)."""
    a = as_rows(a, W_FR, "a")
    e = np.ascontiguousarray(np.asarray(exp_limbs, dtype=np.uint64).reshape(-1))
    out = np.empty_like(a)
    call("pa_fr_pow_batch", ptr(a), ptr(e), e.size, ptr(out), a.shape[0])
    return out


def fr_legendre(a):
    """SqrtField::legendre (fr.rs:575-590): int8 0 Zero, 1 QuadraticResidue, -1 QuadraticNonResidue."""
    a = as_rows(a, W_FR, "a")
    out = np.zeros(a.shape[0], np.int8)
    call("pa_fr_legendre_batch", ptr(a), ptr(out), a.shape[0])
    return out


def fr_sqrt(a):
    """SqrtField::sqrt (fr.rs:592-646): (roots, ok), ok False where the reference returns None."""
    return _inverse("pa_fr_sqrt_batch", a, W_FR)


# ---- variable-base scalar multiplication and MSM (ec.rs:88-95, 174-177, 534-553) ----
def _scalar_mul(name, p, scalars, in_width, out_width):
    p = as_rows(p, in_width, "points")
    s = as_rows(scalars, 4, "scalars")
    if p.shape[0] != s.shape[0]:
        raise ValueError("points and scalars differ in length: %d vs %d" % (p.shape[0], s.shape[0]))
    out = np.zeros((p.shape[0], out_width), np.uint64)
    call(name, ptr(p), ptr(s), ptr(out), p.shape[0])
    return out


def g1_affine_mul(p, scalars):
    """CurveAffine::mul (ec.rs:174-177): Jacobian s_i * P_i, bit-exact with the reference."""
    return _scalar_mul("pa_g1_affine_mul_batch", p, scalars, W_G1A, W_G1)


def g2_affine_mul(p, scalars):
    return _scalar_mul("pa_g2_affine_mul_batch", p, scalars, W_G2A, W_G2)


def g1_mul_assign(p, scalars):
    """CurveProjective::mul_assign (ec.rs:534-553) on Jacobian points, bit-exact."""
    return _scalar_mul("pa_g1_mul_assign_batch", p, scalars, W_G1, W_G1)


def g2_mul_assign(p, scalars):
    return _scalar_mul("pa_g2_mul_assign_batch", p, scalars, W_G2, W_G2)


def _multiexp(name, bases, scalars, in_width, out_width):
    b = as_rows(bases, in_width, "bases") if len(bases) else np.zeros((0, in_width), np.uint64)
    s = as_rows(scalars, 4, "scalars") if len(scalars) else np.zeros((0, 4), np.uint64)
    if b.shape[0] != s.shape[0]:
        raise ValueError("bases and scalars differ in length: %d vs %d" % (b.shape[0], s.shape[0]))
    out = np.zeros((1, out_width), np.uint64)
    call(name, ptr(b), ptr(s), b.shape[0], ptr(out))
    return out


def g1_multiexp(bases, scalars):
    """sum_i s_i * P_i over G1 affine bases (Pippenger on the device): one Jacobian row,
    equal as a point to the reference's sum of CurveAffine::mul results."""
    return _multiexp("pa_g1_multiexp", bases, scalars, W_G1A, W_G1)


def g2_multiexp(bases, scalars):
    return _multiexp("pa_g2_multiexp", bases, scalars, W_G2A, W_G2)


# ---- CurveProjective / CurveAffine surface for G1 and G2 (ec.rs:1-621) ----
_JW = {1: W_G1, 2: W_G2}
_AW = {1: W_G1A, 2: W_G2A}


def _group_unary(group, op, a, in_width, out_width):
    a = as_rows(a, in_width, "points")
    out = np.zeros((a.shape[0], out_width), np.uint64)
    call("pa_g%d_%s_batch" % (group, op), ptr(a), ptr(out), a.shape[0])
    return out


def _group_binary(group, op, a, b, b_width):
    a = as_rows(a, _JW[group], "a")
    b = as_rows(b, b_width, "b")
    if a.shape[0] != b.shape[0]:
        raise ValueError("operand lengths differ: %d vs %d" % (a.shape[0], b.shape[0]))
    out = np.zeros_like(a)
    call("pa_g%d_%s_batch" % (group, op), ptr(a), ptr(b), ptr(out), a.shape[0])
    return out


def _group_eq(group, a, b):
    a = as_rows(a, _JW[group], "a")
    b = as_rows(b, _JW[group], "b")
    if a.shape[0] != b.shape[0]:
        raise ValueError("operand lengths differ: %d vs %d" % (a.shape[0], b.shape[0]))
    out = np.zeros(a.shape[0], np.uint8)
    call("pa_g%d_eq_batch" % group, ptr(a), ptr(b), ptr(out), a.shape[0])
    return out.astype(bool)


def g1_eq(a, b):
    """PartialEq for G1 (ec.rs:45-85): a[i] == b[i] as points, per item."""
    return _group_eq(1, a, b)


def g2_eq(a, b):
    """PartialEq for G2 (ec.rs:45-85): a[i] == b[i] as points, per item."""
    return _group_eq(2, a, b)


def g1_double(a):
    """CurveProjective::double (dbl-2009-l, ec.rs:296-354), Jacobian words bit-exact."""
    return _group_unary(1, "double", a, W_G1, W_G1)


def g2_double(a):
    return _group_unary(2, "double", a, W_G2, W_G2)


def g1_add(a, b):
    """CurveProjective::add_assign (add-2007-bl, ec.rs:356-444)."""
    return _group_binary(1, "add", a, b, W_G1)


def g2_add(a, b):
    return _group_binary(2, "add", a, b, W_G2)


def g1_add_mixed(a, b):
    """CurveProjective::add_assign_mixed (madd-2007-bl, ec.rs:446-526), b affine."""
    return _group_binary(1, "add_mixed", a, b, W_G1A)


def g2_add_mixed(a, b):
    return _group_binary(2, "add_mixed", a, b, W_G2A)


def g1_negate(a):
    """CurveProjective::negate (ec.rs:528-532)."""
    return _group_unary(1, "negate", a, W_G1, W_G1)


def g2_negate(a):
    return _group_unary(2, "negate", a, W_G2, W_G2)


def g1_sub(a, b):
    """CurveProjective::sub_assign = negate + add_assign (lib.rs:156-160)."""
    return _group_binary(1, "sub", a, b, W_G1)


def g2_sub(a, b):
    return _group_binary(2, "sub", a, b, W_G2)


def g1_into_affine(a):
    """CurveProjective::into_affine (ec.rs:586-619)."""
    return _group_unary(1, "into_affine", a, W_G1, W_G1A)


def g2_into_affine(a):
    return _group_unary(2, "into_affine", a, W_G2, W_G2A)


def g1_into_projective(a):
    """CurveAffine::into_projective (ec.rs:570-582)."""
    return _group_unary(1, "into_projective", a, W_G1A, W_G1)


def g2_into_projective(a):
    return _group_unary(2, "into_projective", a, W_G2A, W_G2)


def g2_batch_normalization(v):
    """G2 CurveProjective::batch_normalization (ec.rs:246-294); returns the normalized copy."""
    v = as_rows(v, W_G2, "v").copy()
    call("pa_g2_batch_normalization", ptr(v), v.shape[0])
    return v


def g2_wnaf_fixed_base(base, scalars, window=None):
    """G2 Wnaf::new().base(base, n).scalar(s) (wnaf.rs:93-107, 169-178): points
    equal to the reference's wNAF products (see g1_wnaf_fixed_base)."""
    b = as_rows(base, W_G2, "base")
    s = as_rows(scalars, 4, "scalars")
    out = np.empty((s.shape[0], W_G2), np.uint64)
    if window is None:
        call("pa_g2_wnaf_fixed_base", ptr(b), ptr(s), s.shape[0], ptr(out))
    else:
        call("pa_g2_wnaf_fixed_base_window", ptr(b), ptr(s), s.shape[0], int(window), ptr(out))
    return out


def _window(name, arg):
    w = getattr(_lib, name)(arg)
    if w <= 0:
        raise PairingError("%s failed (%d)" % (name, w))
    return w


def g1_recommended_wnaf_for_scalar(scalar):
    """CurveProjective::recommended_wnaf_for_scalar for G1 (ec.rs:895-905), scalar a FrRepr row."""
    s = as_rows(scalar, 4, "scalar")
    return _window("pa_g1_recommended_wnaf_for_scalar", ptr(s))


def g2_recommended_wnaf_for_scalar(scalar):
    s = as_rows(scalar, 4, "scalar")
    return _window("pa_g2_recommended_wnaf_for_scalar", ptr(s))


def g1_recommended_wnaf_for_num_scalars(n):
    """CurveProjective::recommended_wnaf_for_num_scalars for G1 (ec.rs:907-921)."""
    return _window("pa_g1_recommended_wnaf_for_num_scalars", int(n))


def g2_recommended_wnaf_for_num_scalars(n):
    return _window("pa_g2_recommended_wnaf_for_num_scalars", int(n))
