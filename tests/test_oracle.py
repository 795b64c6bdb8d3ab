"""Pin the C oracle (oracle/, the restatement of the reference) to the
reference's own known answers, and cross-check it against an independent
pure-Python model.  CPU only."""
import hashlib

import numpy as np
import pytest

import pymodel as pm
from helpers import (Q, R_ORDER, RMONT, fq12_one, from_limbs, hexlimbs, limbs, load_json, mont, random_fq,
                     random_scalars, relic_fq12, rng, set_infinity, small_scalars, unmont)

KAT = load_json("kat_limbs.json")


def fqrow(vals):
    return np.array([limbs(v) for v in vals], dtype=np.uint64)


def mrow(vals):
    """canonical ints -> Montgomery rows"""
    return np.array([mont(v) for v in vals], dtype=np.uint64)


def from_repr_rows(arrs):
    """Fq::from_repr of reference FqRepr hex arrays -> Montgomery rows."""
    return np.array([mont(from_limbs(hexlimbs(a))) for a in arrs], dtype=np.uint64)


# ---------------- known answers of the reference ----------------

def test_relic_pairing_kat(oracle):
    # bls12_381/tests/mod.rs:4-53
    one = small_scalars([1])
    got = oracle.pairing(oracle.g1_mul_generator(one), oracle.g2_mul_generator(one))
    np.testing.assert_array_equal(got, relic_fq12())


@pytest.mark.parametrize("fname,group,compressed", [
    ("g1_uncompressed_valid_test_vectors.dat", 1, False),
    ("g1_compressed_valid_test_vectors.dat", 1, True),
    ("g2_uncompressed_valid_test_vectors.dat", 2, False),
    ("g2_compressed_valid_test_vectors.dat", 2, True),
])
def test_kg_vector_files(oracle, fname, group, compressed):
    # bls12_381/tests/mod.rs:55-97: record k = encoding of k*G, k = 0..999
    ref = load_json("dat_vectors.json")[fname]
    got = oracle.kg_vectors(group, ref["records"], compressed)
    assert hashlib.sha256(got).hexdigest() == ref["sha256"]
    size = ref["record_size"]
    for k, rec in enumerate(ref["first_records_hex"]):
        assert got[k * size:(k + 1) * size].hex() == rec


def test_fq_mul_assign_kat(oracle):
    # fq.rs:2558-2584, raw Montgomery limbs
    a, b, c = (np.array([hexlimbs(v)], np.uint64) for v in KAT["test_fq_mul_assign"])
    np.testing.assert_array_equal(oracle.fq_mul(a, b), c)


def test_fq_squaring_kat(oracle):
    # fq.rs:2630-2651: raw input, expected given through from_repr
    raw, exp = KAT["test_fq_squaring"]
    a = np.array([hexlimbs(raw)], np.uint64)
    np.testing.assert_array_equal(oracle.fq_square(a), from_repr_rows([exp]))


def test_fq2_kats(oracle):
    one, zero = mont(1), [0] * 6
    # fq2.rs:272-345
    a = np.array([one + one, zero + one], np.uint64)          # u + 1, u
    got = oracle.fq2_square(a)
    np.testing.assert_array_equal(got[0], np.array(zero + mont(2), np.uint64))   # 2u
    np.testing.assert_array_equal(got[1], np.array(mont(Q - 1) + zero, np.uint64))  # -1
    s = from_repr_rows(KAT["test_fq2_squaring"])
    np.testing.assert_array_equal(oracle.fq2_square(s[0:2].reshape(1, 12)), s[2:4].reshape(1, 12))
    # fq2.rs:346-409
    m = from_repr_rows(KAT["test_fq2_mul"])
    np.testing.assert_array_equal(oracle.fq2_mul(m[0:2].reshape(1, 12), m[2:4].reshape(1, 12)),
                                  m[4:6].reshape(1, 12))
    # fq2.rs:411-458 through the Fq12 inverse of an element whose only nonzero coordinate is c0.c0
    inv = from_repr_rows(KAT["test_fq2_inverse"])
    f = np.zeros((1, 72), np.uint64)
    f[0, :12] = inv[0:2].reshape(12)
    got, ok = oracle.fq12_inverse(f)
    assert ok[0]
    np.testing.assert_array_equal(got[0, :12], inv[2:4].reshape(12))
    assert not got[0, 12:].any()


def _aff(rows, w):
    out = np.zeros((1, 2 * w + 1), np.uint64)
    out[0, :2 * w] = rows.reshape(-1)
    return out


def test_g1_add_double_kats(oracle):
    # ec.rs:1059-1125 (addition), 1127-1175 (doubling); Jacobian inputs with z = 1
    v = from_repr_rows(KAT["test_g1_addition_correctness"])
    p = oracle.g1_from_affine(_aff(v[0:2], 6))
    q = oracle.g1_from_affine(_aff(v[2:4], 6))
    got = oracle.g1_into_affine(oracle.g1_add(p, q))
    np.testing.assert_array_equal(got[0, :12], v[4:6].reshape(12))
    v = from_repr_rows(KAT["test_g1_doubling_correctness"])
    got = oracle.g1_into_affine(oracle.g1_double(oracle.g1_from_affine(_aff(v[0:2], 6))))
    np.testing.assert_array_equal(got[0, :12], v[2:4].reshape(12))


def test_g2_add_double_kats(oracle):
    # ec.rs:1801-1927 (addition), 1929-2017 (doubling)
    v = from_repr_rows(KAT["test_g2_addition_correctness"])
    p = oracle.g2_from_affine(_aff(v[0:4], 12))
    q = oracle.g2_from_affine(_aff(v[4:8], 12))
    got = oracle.g2_into_affine(oracle.g2_add(p, q))
    np.testing.assert_array_equal(got[0, :24], v[8:12].reshape(24))
    v = from_repr_rows(KAT["test_g2_doubling_correctness"])
    got = oracle.g2_into_affine(oracle.g2_double(oracle.g2_from_affine(_aff(v[0:4], 12))))
    np.testing.assert_array_equal(got[0, :24], v[4:8].reshape(24))


# ---------------- independent pure-Python cross-checks ----------------

def test_fq_ops_vs_python_ints(oracle):
    g = rng(101)
    a, b = random_fq(g, 300), random_fq(g, 300)
    a[0] = 0
    b[1] = 0
    ia = [unmont(r) for r in a]
    ib = [unmont(r) for r in b]
    exp_mul = mrow([x * y for x, y in zip(ia, ib)])
    np.testing.assert_array_equal(oracle.fq_mul(a, b), exp_mul)
    np.testing.assert_array_equal(oracle.fq_square(a), mrow([x * x for x in ia]))
    np.testing.assert_array_equal(oracle.fq_add(a, b), mrow([x + y for x, y in zip(ia, ib)]))
    np.testing.assert_array_equal(oracle.fq_sub(a, b), mrow([x - y for x, y in zip(ia, ib)]))
    inv, ok = oracle.fq_inverse(a)
    assert not ok[0] and ok[1:].all()
    np.testing.assert_array_equal(inv[1:], mrow([pow(x, Q - 2, Q) for x in ia[1:]]))
    # repr round trip (fq.rs:747-775)
    np.testing.assert_array_equal(oracle.fq_into_repr(a), fqrow(ia))
    back, okr = oracle.fq_from_repr(fqrow(ia))
    assert okr.all()
    np.testing.assert_array_equal(back, a)
    _, bad = oracle.fq_from_repr(fqrow([Q]))
    assert not bad[0]  # q itself is not a valid repr


def _rand12(seed, n):
    return random_fq(rng(seed), n * 12).reshape(n, 72)


def test_fq12_mul_square_inverse_vs_pymodel(oracle):
    a, b = _rand12(102, 6), _rand12(103, 6)
    for k in range(6):
        x, y = pm.fq12_from_limbs(a[k]), pm.fq12_from_limbs(b[k])
        assert pm.fq12_from_limbs(oracle.fq12_mul(a[k:k + 1], b[k:k + 1])[0]) == pm.f12mul(x, y)
        assert pm.fq12_from_limbs(oracle.fq12_square(a[k:k + 1])[0]) == pm.f12sqr(x)
        inv, ok = oracle.fq12_inverse(a[k:k + 1])
        assert ok[0] and pm.fq12_from_limbs(inv[0]) == pm.f12inv(x)


def test_fq12_frobenius_is_q_power(oracle):
    # random_frobenius_tests, field.rs:4-20: frobenius_map(i) == pow(q^i)
    a = _rand12(104, 2)
    for i in range(0, 13, 3):
        e = np.array(limbs(Q ** i, 6 * max(i, 1)), np.uint64)
        np.testing.assert_array_equal(oracle.fq12_frobenius(a, i), oracle.fq12_pow(a, e))


def test_mul_by_014_is_sparse_mul(oracle):
    # fq12.rs:154-181
    a = _rand12(105, 16)
    g = rng(106)
    c0, c1, c5 = (random_fq(g, 32).reshape(16, 12) for _ in range(3))
    dense = np.zeros((16, 72), np.uint64)
    dense[:, 0:12], dense[:, 12:24], dense[:, 48:60] = c0, c1, c5
    np.testing.assert_array_equal(oracle.fq12_mul_by_014(a, c0, c1, c5), oracle.fq12_mul(a, dense))


def test_final_exponentiation_is_the_fixed_power(oracle):
    # The hard part (mod.rs:116-156) evaluates f^(3 (q^12-1)/r): check with an
    # independent square-and-multiply in the pure-Python model.
    f = _rand12(107, 1)
    exp, ok = oracle.final_exponentiation(f)
    assert ok[0]
    x = pm.fq12_from_limbs(f[0])
    want = pm.f12pow(x, 3 * (Q ** 12 - 1) // R_ORDER)
    assert pm.fq12_from_limbs(exp[0]) == want


# ---------------- engine property tests (src/tests/engine.rs) ----------------

@pytest.fixture(scope="module")
def points(oracle):
    g = rng(110)
    s1, s2 = random_scalars(g, 8), random_scalars(g, 8)
    return s1, s2, oracle.g1_mul_generator(s1, 8), oracle.g2_mul_generator(s2, 8)


def test_infinity_gives_one(oracle, points):
    # engine.rs:16-33
    _, _, p, q = points
    pz, qz = set_infinity(p[:2].copy(), [0, 1]), set_infinity(q[:2].copy(), [0, 1])
    one = fq12_one()
    np.testing.assert_array_equal(oracle.pairing(pz, q[:2]), np.repeat(one, 2, 0))
    np.testing.assert_array_equal(oracle.pairing(p[:2], qz), np.repeat(one, 2, 0))


def test_multi_miller_loop_is_product_of_pairings(oracle, points):
    # engine.rs:68-90
    _, _, p, q = points
    prep = oracle.g2_prepare(q[:2])
    f = oracle.miller_loop(p[:2], prep)
    both, ok = oracle.final_exponentiation(f.reshape(1, 72))
    e = oracle.pairing(p[:2], q[:2])
    np.testing.assert_array_equal(both, oracle.fq12_mul(e[0:1], e[1:2]))


def test_bilinearity(oracle, points):
    # engine.rs:93-126: e(aP, bQ) == e(P, Q)^(ab)
    s1, s2, p, q = points
    one = small_scalars([1])
    e11 = oracle.pairing(oracle.g1_mul_generator(one), oracle.g2_mul_generator(one))
    e = oracle.pairing(p[:3], q[:3])
    for k in range(3):
        ab = from_limbs(s1[k]) * from_limbs(s2[k]) % R_ORDER
        np.testing.assert_array_equal(e[k], oracle.fq12_pow(e11, np.array(limbs(ab, 4), np.uint64))[0])


# ---------------- curve property tests (src/tests/curve.rs) ----------------

def test_wnaf_matches_double_and_add(oracle):
    # curve.rs:68-92 for G1 and G2: wnaf_exp(wnaf_table(g, w), wnaf_form(s, w)) == g * s
    g = rng(120)
    base1 = oracle.g1_from_affine(oracle.g1_mul_generator(random_scalars(g, 1)))
    base2 = oracle.g2_from_affine(oracle.g2_mul_generator(random_scalars(g, 1)))
    s = random_scalars(g, 6)
    s[0] = 0
    s[1] = limbs(1, 4)
    s[2] = limbs(R_ORDER - 1, 4)
    exp1 = oracle.g1_mul(np.repeat(base1, len(s), 0), s)
    exp2 = oracle.g2_mul(np.repeat(base2, len(s), 0), s)
    for n_scalars in (1, 4, 100, 10000):  # windows 4, 6, 10, 14 (ec.rs:907-921)
        got1 = oracle.g1_wnaf_fixed_base(base1, s) if n_scalars == 1 else None
        if got1 is not None:
            assert oracle.g1_eq(got1, exp1).all()
    got1 = oracle.g1_wnaf_fixed_base(base1, s)
    got2 = oracle.g2_wnaf_fixed_base(base2, s)
    assert oracle.g1_eq(got1, exp1).all()
    assert oracle.g2_eq(got2, exp2).all()
    # digit shape of wnaf_form (wnaf.rs:18-43): odd digits in (-2^w, 2^w], zeros between
    for w in range(2, 14):
        for row in s[2:]:
            d = oracle.wnaf_form(row, w)
            v = sum(int(x) << k for k, x in enumerate(d))
            assert v == from_limbs(row)
            nz = d[d != 0]
            assert (nz % 2 != 0).all() and (np.abs(nz) <= (1 << w)).all()


def test_window_heuristics(oracle):
    L = oracle.lib()
    # ec.rs:907-921 / 1598-1612
    assert L.o_g1_recommended_wnaf_for_num_scalars(1 << 18) == 16
    assert L.o_g1_recommended_wnaf_for_num_scalars(1) == 4
    assert L.o_g1_recommended_wnaf_for_num_scalars(2) == 5
    assert L.o_g2_recommended_wnaf_for_num_scalars(1 << 18) == 15
    s = np.array(limbs(1 << 200, 4), np.uint64)
    assert L.o_g1_recommended_wnaf_for_scalar(s.ctypes.data) == 4


def test_batch_normalization_semantics(oracle):
    # curve.rs:357-387: 1000 random points with zeros and normalized points
    # sprinkled in; result == into_affine of each; zeros/normalized untouched
    g = rng(130)
    v = oracle.g1_mul_generator_jacobian(random_scalars(g, 200), 8)
    v[[3, 50, 199], 17 - 5:18] = 0  # z = 0: zero (keeps garbage x, y)
    norm_idx = [7, 80]
    v[norm_idx] = oracle.g1_from_affine(oracle.g1_into_affine(v[norm_idx]))
    out = oracle.g1_batch_normalization(v)
    exp_aff = oracle.g1_into_affine(v)
    for k in range(len(v)):
        if k in (3, 50, 199) or k in norm_idx:
            np.testing.assert_array_equal(out[k], v[k])
        else:
            np.testing.assert_array_equal(out[k, :12], exp_aff[k, :12])
            np.testing.assert_array_equal(out[k, 12:], np.array(limbs(RMONT), np.uint64))
