"""pairing_amd -- MI355X-native batched BLS12-381 engine.

The batched counterpart of the Rust crate `pairing` v0.14.2 hot path
(dignifiedquire/pairing): Fq Montgomery multiply, the Fq2/Fq6/Fq12 tower,
G2 line precomputation (`G2Prepared`), `miller_loop` and
`final_exponentiation`, all as hand-written HIP kernels for gfx950 behind
the C ABI of include/pairing_amd.h.

Two layers:
  * batch functions over numpy arrays in the ABI layout (this module), e.g.
    `pairing(p, q)` for n independent pairs;
  * `pairing_amd.engine`: a mirror of the reference's trait surface
    (`Bls12.pairing`, `Bls12.miller_loop`, `Bls12.final_exponentiation`,
    `G1Affine.prepare`, ...) so code written against the crate reads the same.
Device-resident entry points for torch tensors live in `pairing_amd.device`.
"""
import numpy as np

from ._native import (W_FQ, W_FQ2, W_FQ6, W_FQ12, W_G1A, W_G1, W_G2A, W_G2, W_G2P, PairingError,
                      as_rows, call, device_count, ptr, set_device, set_pairing_kernel, version)

__all__ = [
    "PairingError", "version", "device_count", "set_device", "set_pairing_kernel",
    "fq_mul", "fq_square", "fq_add", "fq_sub", "fq_inverse",
    "fq2_mul", "fq2_square", "fq6_mul", "fq12_mul", "fq12_square", "fq12_inverse",
    "fq12_frobenius_map", "fq12_cyclotomic_square", "fq12_mul_by_014",
    "g1_batch_normalization", "g1_wnaf_fixed_base",
    "g2_prepare", "miller_loop_batch", "multi_miller_loop", "final_exponentiation", "pairing",
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


def pairing(p, q):
    """Engine::pairing (lib.rs:101-109) for n independent (G1Affine, G2Affine) pairs."""
    p = as_rows(p, W_G1A, "p")
    q = as_rows(q, W_G2A, "q")
    if p.shape[0] != q.shape[0]:
        raise ValueError("p and q lengths differ")
    out = np.empty((p.shape[0], W_FQ12), np.uint64)
    call("pa_pairing_batch", ptr(p), ptr(q), ptr(out), p.shape[0])
    return out


# ---- G1 parameter-generation path (config 3) ----
def g1_batch_normalization(v):
    """CurveProjective::batch_normalization (ec.rs:246-294); returns the normalized copy."""
    v = as_rows(v, W_G1, "v").copy()
    call("pa_g1_batch_normalization", ptr(v), v.shape[0])
    return v


def g1_wnaf_fixed_base(base, scalars):
    """Wnaf::new().base(base, n).scalar(s) for each FrRepr scalar (wnaf.rs:93-107,
    169-178): Jacobian points equal to scalars[i] * base."""
    b = as_rows(base, W_G1, "base")
    s = as_rows(scalars, 4, "scalars")
    out = np.empty((s.shape[0], W_G1), np.uint64)
    call("pa_g1_wnaf_fixed_base", ptr(b), ptr(s), s.shape[0], ptr(out))
    return out
