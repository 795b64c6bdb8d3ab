"""Scalar field Fr (src/bls12_381/fr.rs; SURVEY.md §8 f, rank 4).

CPU: the C oracle's Fr (oracle/oracle_fr.c) pinned to the reference's own
known answers (fr.rs:911-1505, extracted into tests/golden/kat_limbs.json) and
to an independent Python big-integer model, plus the reference's property
suites (associativity, (a-b)+(b-a)=0, pow, sqrt, root of unity).
GPU (-m gpu): every Fr kernel behind the C ABI against the oracle on the same
seeded inputs, bit-exact (canonical outputs)."""
import numpy as np
import pytest

from helpers import R_ORDER, from_limbs, hexlimbs, limbs, load_json, rng

KAT = load_json("kat_limbs.json")
FR_R = pow(2, 256, R_ORDER)
FR_RINV = pow(FR_R, -1, R_ORDER)


def fr_mont(v):
    """canonical int -> Montgomery limbs (Fr::from_repr, fr.rs:279-288)"""
    return limbs(v % R_ORDER * FR_R % R_ORDER, 4)


def fr_val(ws):
    """Montgomery limbs -> canonical int (Fr::into_repr, fr.rs:290-303)"""
    return from_limbs(ws) * FR_RINV % R_ORDER


def rows(vals):
    return np.array([limbs(v, 4) for v in vals], dtype=np.uint64)


def random_fr(gen, n):
    """n uniform Fr in Montgomery form (Fr::rand, fr.rs:255-267: 4 random u64,
    top bit shaved, rejection at r) -- Montgomery limbs are themselves uniform below r."""
    out = np.zeros((n, 4), np.uint64)
    k = 0
    while k < n:
        c = gen.integers(0, 1 << 64, size=(n, 4), dtype=np.uint64)
        c[:, 3] &= np.uint64((1 << 63) - 1)
        for row in c:
            if from_limbs(row) < R_ORDER:
                out[k] = row
                k += 1
                if k == n:
                    break
    return out


def edge_fr():
    vals = [0, 1, 2, R_ORDER - 1, R_ORDER - 2, (R_ORDER - 1) // 2, FR_R, (1 << 254) + 12345]
    return rows([v % R_ORDER for v in vals])


def kat(name):
    return [hexlimbs(a) for a in KAT[name]]


def one_row(ws):
    return np.array([ws], dtype=np.uint64)


# ---------------- oracle vs the reference's known answers ----------------

def test_fr_add_assign_kat(oracle):
    k = kat("test_fr_add_assign")   # fr.rs:1041-1122
    a, a1, x, s, rm1, y, z, s2 = (one_row(k[i]) for i in (0, 2, 3, 4, 5, 6, 7, 8))
    zero = np.zeros((1, 4), np.uint64)
    np.testing.assert_array_equal(oracle.fr_add(a, zero), a)
    np.testing.assert_array_equal(oracle.fr_add(a, rows([1])), a1)
    np.testing.assert_array_equal(oracle.fr_add(a1, x), s)
    assert not oracle.fr_add(rm1, rows([1])).any()
    np.testing.assert_array_equal(oracle.fr_add(y, z), s2)


def test_fr_sub_assign_kat(oracle):
    k = kat("test_fr_sub_assign")   # fr.rs:1150-1238
    np.testing.assert_array_equal(oracle.fr_sub(one_row(k[0]), one_row(k[1])), one_row(k[2]))
    np.testing.assert_array_equal(oracle.fr_sub(one_row(k[3]), one_row(k[4])), one_row(k[5]))
    zero = np.zeros((1, 4), np.uint64)
    assert not oracle.fr_sub(zero, zero).any()
    np.testing.assert_array_equal(oracle.fr_sub(one_row(k[6]), zero), one_row(k[7]))


def test_fr_mul_assign_kat(oracle):
    k = kat("test_fr_mul_assign")   # fr.rs:1240-1304
    np.testing.assert_array_equal(oracle.fr_mul(one_row(k[0]), one_row(k[1])), one_row(k[2]))


def test_fr_squaring_kat(oracle):
    k = kat("test_fr_squaring")     # fr.rs:1306-1340: expected is from_repr(...)
    exp, ok = oracle.fr_from_repr(one_row(k[1]))
    assert ok.all()
    np.testing.assert_array_equal(oracle.fr_square(one_row(k[0])), exp)


def test_fr_from_into_repr_kat(oracle):
    k = kat("test_fr_from_into_repr")   # fr.rs:1450-1504
    m, _, _ = oracle.fr_constants()
    _, ok = oracle.fr_from_repr(np.stack([np.array(k[0], np.uint64), m]))
    assert not ok.any()                 # r + 1 and r are not in the field
    a, oka = oracle.fr_from_repr(one_row(k[1]))
    b, okb = oracle.fr_from_repr(one_row(k[2]))
    assert oka.all() and okb.all()
    np.testing.assert_array_equal(oracle.fr_into_repr(oracle.fr_mul(a, b)), one_row(k[3]))
    z, okz = oracle.fr_from_repr(np.zeros((1, 4), np.uint64))
    assert okz.all() and not z.any()


def test_fr_legendre_kat(oracle):
    k = kat("test_fr_legendre")     # fr.rs:911-930
    one = rows([FR_R])
    qr, _ = oracle.fr_from_repr(one_row(k[0]))
    qnr, _ = oracle.fr_from_repr(one_row(k[1]))
    got = oracle.fr_legendre(np.concatenate([one, np.zeros((1, 4), np.uint64), qr, qnr]))
    assert got.tolist() == [1, 0, 1, -1]


def test_fr_root_of_unity(oracle):
    # fr.rs:1584-1600: generator 7, generator^t = root of unity, root^(2^32) = 1, 7 is a non-residue
    m, r, w = oracle.fr_constants()
    assert fr_val(r) == 1
    g, _ = oracle.fr_from_repr(rows([7]))
    t = [0xfffe5bfeffffffff, 0x9a1d80553bda402, 0x299d7d483339d808, 0x73eda753]
    np.testing.assert_array_equal(oracle.fr_pow(g, t)[0], w)
    np.testing.assert_array_equal(oracle.fr_pow(w.reshape(1, 4), [1 << 32])[0], r)
    _, ok = oracle.fr_sqrt(g)
    assert not ok.any()
    assert from_limbs(m) == R_ORDER


# ---------------- oracle vs an independent big-integer model ----------------

def test_fr_oracle_matches_python_model(oracle):
    g = rng(11)
    a = np.concatenate([edge_fr(), random_fr(g, 200)])
    b = np.concatenate([edge_fr()[::-1], random_fr(g, 200)])
    A = [from_limbs(x) for x in a]
    B = [from_limbs(x) for x in b]
    assert [from_limbs(x) for x in oracle.fr_mul(a, b)] == [x * y * FR_RINV % R_ORDER for x, y in zip(A, B)]
    assert [from_limbs(x) for x in oracle.fr_square(a)] == [x * x * FR_RINV % R_ORDER for x in A]
    assert [from_limbs(x) for x in oracle.fr_add(a, b)] == [(x + y) % R_ORDER for x, y in zip(A, B)]
    assert [from_limbs(x) for x in oracle.fr_sub(a, b)] == [(x - y) % R_ORDER for x, y in zip(A, B)]
    assert [from_limbs(x) for x in oracle.fr_double(a)] == [2 * x % R_ORDER for x in A]
    assert [from_limbs(x) for x in oracle.fr_negate(a)] == [(-x) % R_ORDER for x in A]
    inv, ok = oracle.fr_inverse(a)
    for x, y, k in zip(A, inv, ok):
        assert k == (x != 0)
        if x:
            assert fr_val(y) * (x * FR_RINV) % R_ORDER == 1
    assert [from_limbs(x) for x in oracle.fr_into_repr(a)] == [x * FR_RINV % R_ORDER for x in A]


def test_fr_reference_properties(oracle):
    g = rng(12)
    a, b, c = random_fr(g, 300), random_fr(g, 300), random_fr(g, 300)
    # associativity (fr.rs:1124-1147), (a-b)+(b-a)=0 (fr.rs:1226-1238)
    np.testing.assert_array_equal(oracle.fr_add(oracle.fr_add(a, b), c), oracle.fr_add(oracle.fr_add(b, c), a))
    assert not oracle.fr_add(oracle.fr_sub(a, b), oracle.fr_sub(b, a)).any()
    # pow by i == repeated multiplication; pow by r is the identity (fr.rs:1395-1417)
    for i in (0, 1, 2, 7, 64):
        acc = np.tile(rows([FR_R]), (4, 1))
        for _ in range(i):
            acc = oracle.fr_mul(acc, a[:4])
        np.testing.assert_array_equal(oracle.fr_pow(a[:4], [i]), acc)
    np.testing.assert_array_equal(oracle.fr_pow(a[:16], limbs(R_ORDER, 4)), a[:16])
    # sqrt(a^2) = +-a; sqrt(a)^2 = a when it exists (fr.rs:1419-1448)
    sq = oracle.fr_square(a)
    root, ok = oracle.fr_sqrt(sq)
    assert ok.all()
    neg = oracle.fr_negate(a)
    assert all((r == x).all() or (r == y).all() for r, x, y in zip(root, a, neg))
    root, ok = oracle.fr_sqrt(b)
    np.testing.assert_array_equal(oracle.fr_square(root[ok]), b[ok])
    assert 0.3 < ok.mean() < 0.7
    z, okz = oracle.fr_sqrt(np.zeros((1, 4), np.uint64))
    assert okz.all() and not z.any()


# ---------------- GPU parity ----------------

@pytest.mark.gpu
def test_fr_kats_on_gpu(gpu):
    k = kat("test_fr_mul_assign")
    np.testing.assert_array_equal(gpu.fr_mul(one_row(k[0]), one_row(k[1])), one_row(k[2]))
    k = kat("test_fr_from_into_repr")
    a, oka = gpu.fr_from_repr(one_row(k[1]))
    b, okb = gpu.fr_from_repr(one_row(k[2]))
    assert oka.all() and okb.all()
    np.testing.assert_array_equal(gpu.fr_into_repr(gpu.fr_mul(a, b)), one_row(k[3]))
    _, bad = gpu.fr_from_repr(np.stack([np.array(k[0], np.uint64), np.array(limbs(R_ORDER, 4), np.uint64)]))
    assert not bad.any()


@pytest.mark.gpu
def test_fr_elementwise_match_oracle(gpu, oracle):
    g = rng(21)
    a = np.concatenate([edge_fr(), random_fr(g, 4096)])
    b = np.concatenate([edge_fr()[::-1], random_fr(g, 4096)])
    np.testing.assert_array_equal(gpu.fr_mul(a, b), oracle.fr_mul(a, b))
    np.testing.assert_array_equal(gpu.fr_square(a), oracle.fr_square(a))
    np.testing.assert_array_equal(gpu.fr_add(a, b), oracle.fr_add(a, b))
    np.testing.assert_array_equal(gpu.fr_sub(a, b), oracle.fr_sub(a, b))
    np.testing.assert_array_equal(gpu.fr_double(a), oracle.fr_double(a))
    np.testing.assert_array_equal(gpu.fr_negate(a), oracle.fr_negate(a))
    np.testing.assert_array_equal(gpu.fr_into_repr(a), oracle.fr_into_repr(a))
    reprs = np.concatenate([a, rows([R_ORDER, R_ORDER + 1, (1 << 256) - 1])])
    got, ok = gpu.fr_from_repr(reprs)
    exp, eok = oracle.fr_from_repr(reprs)
    np.testing.assert_array_equal(ok, eok)
    np.testing.assert_array_equal(got[eok], exp[eok])


@pytest.mark.gpu
def test_fr_inverse_pow_legendre_sqrt_match_oracle(gpu, oracle):
    g = rng(22)
    a = np.concatenate([edge_fr(), random_fr(g, 512)])
    got, ok = gpu.fr_inverse(a)
    exp, eok = oracle.fr_inverse(a)
    np.testing.assert_array_equal(ok, eok)
    np.testing.assert_array_equal(got[eok], exp[eok])
    for e in ([0], [5], limbs(R_ORDER, 4), [0xdeadbeefcafebabe, 0x1234, 0, 0, 7]):
        np.testing.assert_array_equal(gpu.fr_pow(a, e), oracle.fr_pow(a, e))
    np.testing.assert_array_equal(gpu.fr_legendre(a), oracle.fr_legendre(a))
    b = np.concatenate([a, oracle.fr_square(a)])
    got, ok = gpu.fr_sqrt(b)
    exp, eok = oracle.fr_sqrt(b)
    np.testing.assert_array_equal(ok, eok)
    np.testing.assert_array_equal(got, exp)     # the reference's choice of root, bit for bit
