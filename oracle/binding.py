"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the C parity oracle.

Loads oracle/liboracle.so (the C restatement of the reference crate's
BLS12-381 hot path, see oracle/oracle.h).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the
product package pairing_amd/.

Arrays are numpy uint64 in the ABI layout (include/pairing_amd.h):
  Fq (n,6)  Fq2 (n,12)  Fq6 (n,36)  Fq12 (n,72)
  G1Affine (n,13)  G1 (n,18)  G2Affine (n,25)  G2 (n,36)  G2Prepared (n,2449)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PA_ORACLE_LIB selects another build of the same sources (the sanitizer
# build `make -C oracle asan` -> liboracle_asan.so, tests/test_sanitizer.py)
LIB_PATH = os.environ.get("PA_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

W_FQ, W_FQ2, W_FQ6, W_FQ12 = 6, 12, 36, 72
W_G1A, W_G1, W_G2A, W_G2 = 13, 18, 25, 36
W_G2P = 68 * 3 * 12 + 1

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


_P = ctypes.c_void_p
_N = ctypes.c_size_t
_I = ctypes.c_int


def _declare(L):
    sig = {
        "o_fq_mul_batch": [_P, _P, _P, _N],
        "o_fq_square_batch": [_P, _P, _N],
        "o_fq_add_batch": [_P, _P, _P, _N],
        "o_fq_sub_batch": [_P, _P, _P, _N],
        "o_fq_inverse_batch": [_P, _P, _P, _N],
        "o_fq2_mul_batch": [_P, _P, _P, _N],
        "o_fq2_square_batch": [_P, _P, _N],
        "o_fq6_mul_batch": [_P, _P, _P, _N],
        "o_fq12_mul_batch": [_P, _P, _P, _N],
        "o_fq12_square_batch": [_P, _P, _N],
        "o_fq12_inverse_batch": [_P, _P, _P, _N],
        "o_fq12_frobenius_batch": [_P, _P, _N, _N],
        "o_fq12_mul_by_014_batch": [_P, _P, _P, _P, _P, _N],
        "o_fq12_pow_batch": [_P, _P, _N, _P, _N],
        "o_fq_from_repr_batch": [_P, _N, _P, _P],
        "o_fq_into_repr_batch": [_P, _N, _P],
        "o_g1_mul_generator_batch": [_P, _N, _P, _I],
        "o_g2_mul_generator_batch": [_P, _N, _P, _I],
        "o_g1_mul_generator_jacobian_batch": [_P, _N, _P, _I],
        "o_g1_mul_batch": [_P, _P, _N, _P],
        "o_g2_mul_batch": [_P, _P, _N, _P],
        "o_g1_double_batch": [_P, _N, _P],
        "o_g2_double_batch": [_P, _N, _P],
        "o_g1_add_batch": [_P, _P, _N, _P],
        "o_g2_add_batch": [_P, _P, _N, _P],
        "o_g1_add_mixed_batch": [_P, _P, _N, _P],
        "o_g2_add_mixed_batch": [_P, _P, _N, _P],
        "o_g1_into_affine_batch": [_P, _N, _P],
        "o_g2_into_affine_batch": [_P, _N, _P],
        "o_g1_from_affine_batch": [_P, _N, _P],
        "o_g2_from_affine_batch": [_P, _N, _P],
        "o_g1_eq_batch": [_P, _P, _N, _P],
        "o_g2_eq_batch": [_P, _P, _N, _P],
        "o_g1_batch_normalization": [_P, _N],
        "o_g2_batch_normalization": [_P, _N],
        "o_g1_wnaf_fixed_base": [_P, _P, _N, _P, _I],
        "o_g2_wnaf_fixed_base": [_P, _P, _N, _P, _I],
        "o_g1_wnaf_fixed_base_w": [_P, _P, _N, _I, _P, _I],
        "o_g2_wnaf_fixed_base_w": [_P, _P, _N, _I, _P, _I],
        "o_g1_wnaf_fixed_scalar": [_P, _P, _N, _P, _I],
        "o_g2_wnaf_fixed_scalar": [_P, _P, _N, _P, _I],
        "o_g1_kg_vectors": [_P, _N, _I],
        "o_g2_kg_vectors": [_P, _N, _I],
        "o_g2_prepare_batch": [_P, _N, _P, _I],
        "o_miller_loop": [_P, _P, _P, _N],
        "o_miller_loop_batch": [_P, _P, _N, _P, _I],
        "o_final_exponentiation_batch": [_P, _N, _P, _P, _I],
        "o_pairing_batch": [_P, _P, _N, _P, _I],
        "o_wnaf_form": [_P, _P, _I],
        "o_g1_recommended_wnaf_for_num_scalars": [_N],
        "o_g2_recommended_wnaf_for_num_scalars": [_N],
        "o_g1_recommended_wnaf_for_scalar": [_P],
        "o_g2_recommended_wnaf_for_scalar": [_P],
        "o_sizeof": [_I],
        "o_g1_decode_batch": [_P, _N, _I, _I, _P, _P, _I],
        "o_g2_decode_batch": [_P, _N, _I, _I, _P, _P, _I],
        "o_fq_sqrt_batch": [_P, _N, _P, _P],
        "o_fr_mul_batch": [_P, _P, _P, _N],
        "o_fr_square_batch": [_P, _P, _N],
        "o_fr_add_batch": [_P, _P, _P, _N],
        "o_fr_sub_batch": [_P, _P, _P, _N],
        "o_fr_double_batch": [_P, _P, _N],
        "o_fr_negate_batch": [_P, _P, _N],
        "o_fr_inverse_batch": [_P, _P, _P, _N],
        "o_fr_from_repr_batch": [_P, _N, _P, _P],
        "o_fr_into_repr_batch": [_P, _N, _P],
        "o_fr_pow_batch": [_P, _P, _N, _P, _N],
        "o_fr_legendre_batch": [_P, _P, _N],
        "o_fr_sqrt_batch": [_P, _N, _P, _P],
        "o_fr_constants": [_P, _P, _P],
        "o_g1_affine_mul_batch": [_P, _P, _N, _P, _I],
        "o_g2_affine_mul_batch": [_P, _P, _N, _P, _I],
        "o_g1_multiexp": [_P, _P, _N, _P, _I],
        "o_g2_multiexp": [_P, _P, _N, _P, _I],
        "o_fq2_sqrt_batch": [_P, _N, _P, _P],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = None
    L.o_wnaf_form.restype = _N
    L.o_sizeof.restype = _N
    for name in ("o_g1_recommended_wnaf_for_num_scalars", "o_g2_recommended_wnaf_for_num_scalars",
                 "o_g1_recommended_wnaf_for_scalar", "o_g2_recommended_wnaf_for_scalar"):
        getattr(L, name).restype = _I


def _p(a):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def _out(n, w, dtype=np.uint64):
    return np.zeros((n, w), dtype=dtype)


def _n(a):
    return a.shape[0]


# ---- field ops ----
def fq_mul(a, b):
    o = _out(_n(a), W_FQ); lib().o_fq_mul_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fq_square(a):
    o = _out(_n(a), W_FQ); lib().o_fq_square_batch(_p(a), _p(o), _n(a)); return o


def fq_add(a, b):
    o = _out(_n(a), W_FQ); lib().o_fq_add_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fq_sub(a, b):
    o = _out(_n(a), W_FQ); lib().o_fq_sub_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fq_inverse(a):
    o = _out(_n(a), W_FQ); ok = np.zeros(_n(a), np.uint8)
    lib().o_fq_inverse_batch(_p(a), _p(o), _p(ok), _n(a)); return o, ok


def fq2_mul(a, b):
    o = _out(_n(a), W_FQ2); lib().o_fq2_mul_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fq2_square(a):
    o = _out(_n(a), W_FQ2); lib().o_fq2_square_batch(_p(a), _p(o), _n(a)); return o


def fq6_mul(a, b):
    o = _out(_n(a), W_FQ6); lib().o_fq6_mul_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fq12_mul(a, b):
    o = _out(_n(a), W_FQ12); lib().o_fq12_mul_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fq12_square(a):
    o = _out(_n(a), W_FQ12); lib().o_fq12_square_batch(_p(a), _p(o), _n(a)); return o


def fq12_inverse(a):
    o = _out(_n(a), W_FQ12); ok = np.zeros(_n(a), np.uint8)
    lib().o_fq12_inverse_batch(_p(a), _p(o), _p(ok), _n(a)); return o, ok


def fq12_frobenius(a, power):
    o = _out(_n(a), W_FQ12); lib().o_fq12_frobenius_batch(_p(a), _p(o), _n(a), power); return o


def fq12_mul_by_014(a, c0, c1, c4):
    o = _out(_n(a), W_FQ12)
    lib().o_fq12_mul_by_014_batch(_p(a), _p(c0), _p(c1), _p(c4), _p(o), _n(a)); return o


def fq12_pow(a, exp_limbs):
    e = np.ascontiguousarray(np.asarray(exp_limbs, dtype=np.uint64))
    o = _out(_n(a), W_FQ12); lib().o_fq12_pow_batch(_p(a), _p(e), e.size, _p(o), _n(a)); return o


def fq_from_repr(r):
    o = _out(_n(r), W_FQ); ok = np.zeros(_n(r), np.uint8)
    lib().o_fq_from_repr_batch(_p(r), _n(r), _p(o), _p(ok)); return o, ok


def fq_into_repr(a):
    o = _out(_n(a), W_FQ); lib().o_fq_into_repr_batch(_p(a), _n(a), _p(o)); return o


# ---- Fr (scalar field, fr.rs): (n,4) u64 Montgomery R = 2^256 ----
W_FR = 4


def fr_mul(a, b):
    o = _out(_n(a), W_FR); lib().o_fr_mul_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fr_square(a):
    o = _out(_n(a), W_FR); lib().o_fr_square_batch(_p(a), _p(o), _n(a)); return o


def fr_add(a, b):
    o = _out(_n(a), W_FR); lib().o_fr_add_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fr_sub(a, b):
    o = _out(_n(a), W_FR); lib().o_fr_sub_batch(_p(a), _p(b), _p(o), _n(a)); return o


def fr_double(a):
    o = _out(_n(a), W_FR); lib().o_fr_double_batch(_p(a), _p(o), _n(a)); return o


def fr_negate(a):
    o = _out(_n(a), W_FR); lib().o_fr_negate_batch(_p(a), _p(o), _n(a)); return o


def fr_inverse(a):
    o = _out(_n(a), W_FR); ok = np.zeros(_n(a), np.uint8)
    lib().o_fr_inverse_batch(_p(a), _p(o), _p(ok), _n(a)); return o, ok.astype(bool)


def fr_from_repr(r):
    o = _out(_n(r), W_FR); ok = np.zeros(_n(r), np.uint8)
    lib().o_fr_from_repr_batch(_p(r), _n(r), _p(o), _p(ok)); return o, ok.astype(bool)


def fr_into_repr(a):
    o = _out(_n(a), W_FR); lib().o_fr_into_repr_batch(_p(a), _n(a), _p(o)); return o


def fr_pow(a, exp_limbs):
    e = np.ascontiguousarray(np.asarray(exp_limbs, dtype=np.uint64))
    o = _out(_n(a), W_FR); lib().o_fr_pow_batch(_p(a), _p(e), e.size, _p(o), _n(a)); return o


def fr_legendre(a):
    o = np.zeros(_n(a), np.int8); lib().o_fr_legendre_batch(_p(a), _p(o), _n(a)); return o


def fr_sqrt(a):
    o = _out(_n(a), W_FR); ok = np.zeros(_n(a), np.uint8)
    lib().o_fr_sqrt_batch(_p(a), _n(a), _p(o), _p(ok)); return o, ok.astype(bool)


def fr_constants():
    """(modulus, R, root_of_unity) as (4,) u64 arrays (fr.rs:4-56)."""
    m, r, w = (np.zeros(4, np.uint64) for _ in range(3))
    lib().o_fr_constants(_p(m), _p(r), _p(w)); return m, r, w


# ---- curve ops ----
def g1_mul_generator(scalars, nthreads=1):
    o = _out(_n(scalars), W_G1A); lib().o_g1_mul_generator_batch(_p(scalars), _n(scalars), _p(o), nthreads); return o


def g2_mul_generator(scalars, nthreads=1):
    o = _out(_n(scalars), W_G2A); lib().o_g2_mul_generator_batch(_p(scalars), _n(scalars), _p(o), nthreads); return o


def g1_mul_generator_jacobian(scalars, nthreads=1):
    o = _out(_n(scalars), W_G1)
    lib().o_g1_mul_generator_jacobian_batch(_p(scalars), _n(scalars), _p(o), nthreads); return o


def g1_mul(p, scalars):
    o = _out(_n(p), W_G1); lib().o_g1_mul_batch(_p(p), _p(scalars), _n(p), _p(o)); return o


def g2_mul(p, scalars):
    o = _out(_n(p), W_G2); lib().o_g2_mul_batch(_p(p), _p(scalars), _n(p), _p(o)); return o


def g1_affine_mul(p, scalars, nthreads=1):
    """CurveAffine::mul (ec.rs:174-177): Jacobian rows."""
    o = _out(_n(p), W_G1); lib().o_g1_affine_mul_batch(_p(p), _p(scalars), _n(p), _p(o), nthreads); return o


def g2_affine_mul(p, scalars, nthreads=1):
    o = _out(_n(p), W_G2); lib().o_g2_affine_mul_batch(_p(p), _p(scalars), _n(p), _p(o), nthreads); return o


def g1_multiexp(p, scalars, nthreads=1):
    """sum_i s_i * P_i: CurveAffine::mul per term + add_assign in index order; (1, 18)."""
    o = _out(1, W_G1); lib().o_g1_multiexp(_p(p), _p(scalars), _n(p), _p(o), nthreads); return o


def g2_multiexp(p, scalars, nthreads=1):
    o = _out(1, W_G2); lib().o_g2_multiexp(_p(p), _p(scalars), _n(p), _p(o), nthreads); return o


def g1_double(p):
    o = _out(_n(p), W_G1); lib().o_g1_double_batch(_p(p), _n(p), _p(o)); return o


def g2_double(p):
    o = _out(_n(p), W_G2); lib().o_g2_double_batch(_p(p), _n(p), _p(o)); return o


def g1_add(a, b):
    o = _out(_n(a), W_G1); lib().o_g1_add_batch(_p(a), _p(b), _n(a), _p(o)); return o


def g2_add(a, b):
    o = _out(_n(a), W_G2); lib().o_g2_add_batch(_p(a), _p(b), _n(a), _p(o)); return o


def g1_add_mixed(a, b):
    o = _out(_n(a), W_G1); lib().o_g1_add_mixed_batch(_p(a), _p(b), _n(a), _p(o)); return o


def g2_add_mixed(a, b):
    o = _out(_n(a), W_G2); lib().o_g2_add_mixed_batch(_p(a), _p(b), _n(a), _p(o)); return o


def g1_into_affine(p):
    o = _out(_n(p), W_G1A); lib().o_g1_into_affine_batch(_p(p), _n(p), _p(o)); return o


def g2_into_affine(p):
    o = _out(_n(p), W_G2A); lib().o_g2_into_affine_batch(_p(p), _n(p), _p(o)); return o


def g1_from_affine(a):
    o = _out(_n(a), W_G1); lib().o_g1_from_affine_batch(_p(a), _n(a), _p(o)); return o


def g2_from_affine(a):
    o = _out(_n(a), W_G2); lib().o_g2_from_affine_batch(_p(a), _n(a), _p(o)); return o


def g1_eq(a, b):
    o = np.zeros(_n(a), np.uint8); lib().o_g1_eq_batch(_p(a), _p(b), _n(a), _p(o)); return o.astype(bool)


def g2_eq(a, b):
    o = np.zeros(_n(a), np.uint8); lib().o_g2_eq_batch(_p(a), _p(b), _n(a), _p(o)); return o.astype(bool)


def g1_batch_normalization(v):
    v = np.ascontiguousarray(v.copy()); lib().o_g1_batch_normalization(_p(v), _n(v)); return v


def g2_batch_normalization(v):
    v = np.ascontiguousarray(v.copy()); lib().o_g2_batch_normalization(_p(v), _n(v)); return v


def g1_wnaf_fixed_base(base, scalars, nthreads=1, window=None):
    """Wnaf::new().base(base, n).scalar(s_i) (wnaf.rs:93-107, 169-178); window
    default recommended_wnaf_for_num_scalars(n)"""
    b = np.ascontiguousarray(base.reshape(1, W_G1))
    o = _out(_n(scalars), W_G1)
    if window is None:
        lib().o_g1_wnaf_fixed_base(_p(b), _p(scalars), _n(scalars), _p(o), nthreads)
    else:
        lib().o_g1_wnaf_fixed_base_w(_p(b), _p(scalars), _n(scalars), int(window), _p(o), nthreads)
    return o


def g2_wnaf_fixed_base(base, scalars, nthreads=1, window=None):
    b = np.ascontiguousarray(base.reshape(1, W_G2))
    o = _out(_n(scalars), W_G2)
    if window is None:
        lib().o_g2_wnaf_fixed_base(_p(b), _p(scalars), _n(scalars), _p(o), nthreads)
    else:
        lib().o_g2_wnaf_fixed_base_w(_p(b), _p(scalars), _n(scalars), int(window), _p(o), nthreads)
    return o


def g1_wnaf_fixed_scalar(bases, scalar, nthreads=1):
    """Wnaf::new().scalar(s).base(g_i) (wnaf.rs:111-128, 156-165)"""
    b = np.ascontiguousarray(bases.reshape(-1, W_G1))
    s = np.ascontiguousarray(np.asarray(scalar, np.uint64).reshape(4))
    o = _out(b.shape[0], W_G1)
    lib().o_g1_wnaf_fixed_scalar(_p(b), _p(s), b.shape[0], _p(o), nthreads); return o


def g2_wnaf_fixed_scalar(bases, scalar, nthreads=1):
    b = np.ascontiguousarray(bases.reshape(-1, W_G2))
    s = np.ascontiguousarray(np.asarray(scalar, np.uint64).reshape(4))
    o = _out(b.shape[0], W_G2)
    lib().o_g2_wnaf_fixed_scalar(_p(b), _p(s), b.shape[0], _p(o), nthreads); return o


def wnaf_form(scalar, window):
    s = np.ascontiguousarray(np.asarray(scalar, dtype=np.uint64))
    d = np.zeros(300, np.int64)
    n = lib().o_wnaf_form(_p(d), _p(s), window)
    return d[:n]


def kg_vectors(group, count, compressed):
    size = {(1, False): 96, (1, True): 48, (2, False): 192, (2, True): 96}[(group, bool(compressed))]
    o = np.zeros(count * size, np.uint8)
    fn = lib().o_g1_kg_vectors if group == 1 else lib().o_g2_kg_vectors
    fn(_p(o), count, int(bool(compressed)))
    return o.tobytes()


# ---- point decoding (EncodedPoint::into_affine[_unchecked]) ----
ENC_SIZE = {(1, False): 96, (1, True): 48, (2, False): 192, (2, True): 96}


def decode(group, enc, compressed, checked=True, nthreads=1):
    """enc: (n, size) uint8 records -> (affine points, status bytes)"""
    enc = np.ascontiguousarray(enc, dtype=np.uint8)
    n = enc.shape[0]
    assert enc.shape[1] == ENC_SIZE[(group, bool(compressed))]
    o = _out(n, W_G1A if group == 1 else W_G2A)
    st = np.zeros(n, np.uint8)
    fn = lib().o_g1_decode_batch if group == 1 else lib().o_g2_decode_batch
    fn(_p(enc), n, int(bool(compressed)), int(bool(checked)), _p(o), _p(st), nthreads)
    return o, st


def fq_sqrt(a):
    o = _out(_n(a), W_FQ); ok = np.zeros(_n(a), np.uint8)
    lib().o_fq_sqrt_batch(_p(a), _n(a), _p(o), _p(ok)); return o, ok


def fq2_sqrt(a):
    o = _out(_n(a), W_FQ2); ok = np.zeros(_n(a), np.uint8)
    lib().o_fq2_sqrt_batch(_p(a), _n(a), _p(o), _p(ok)); return o, ok


# ---- pairing ----
def g2_prepare(q, nthreads=1):
    o = _out(_n(q), W_G2P); lib().o_g2_prepare_batch(_p(q), _n(q), _p(o), nthreads); return o


def miller_loop(ps, qs_prepared):
    """Engine::miller_loop over all pairs (product semantics, mod.rs:40-102)."""
    o = _out(1, W_FQ12); lib().o_miller_loop(_p(o), _p(ps), _p(qs_prepared), _n(ps)); return o[0]


def miller_loop_batch(ps, qs_prepared, nthreads=1):
    o = _out(_n(ps), W_FQ12); lib().o_miller_loop_batch(_p(ps), _p(qs_prepared), _n(ps), _p(o), nthreads); return o


def final_exponentiation(f, nthreads=1):
    o = _out(_n(f), W_FQ12); ok = np.zeros(_n(f), np.uint8)
    lib().o_final_exponentiation_batch(_p(f), _n(f), _p(o), _p(ok), nthreads); return o, ok


def pairing(p, q, nthreads=1):
    o = _out(_n(p), W_FQ12); lib().o_pairing_batch(_p(p), _p(q), _n(p), _p(o), nthreads); return o
