"""Field trait methods of the Fq2 / Fq6 / Fq12 mirror types on the GPU
(lib.rs:267-325): Fq2::inverse / frobenius_map (fq2.rs:138-159), Fq6::square
/ inverse / frobenius_map (fq6.rs:157-301), Field::pow for Fq and Fq12
(lib.rs:306-324).  The oracle is the Fq12 restatement applied to the
subfield element embedded in Fq12 (c0.c0 = a for Fq2, c0 = a for Fq6): the
tower embeds each subfield, so inverse / square / Frobenius / pow of the
embedded element is the embedding of the result.  All outputs are canonical,
so the comparison is bit-exact."""
import numpy as np
import pytest

from helpers import random_fq, rng

pytestmark = pytest.mark.gpu


def _tower(seed, n, width):
    return random_fq(rng(seed), n * width // 6).reshape(n, width)


def _embed(a):
    e = np.zeros((a.shape[0], 72), np.uint64)
    e[:, :a.shape[1]] = a
    return e


def test_fq2_inverse_frobenius(gpu, oracle):
    a = _tower(1, 256, 12)
    a[5] = 0
    got, ok = gpu.fq2_inverse(a)
    exp, eok = oracle.fq12_inverse(_embed(a))
    np.testing.assert_array_equal(ok, eok.astype(bool))
    assert not ok[5] and ok.sum() == 255
    np.testing.assert_array_equal(got[ok], exp[ok][:, :12])
    for power in range(4):
        np.testing.assert_array_equal(gpu.fq2_frobenius_map(a, power), oracle.fq12_frobenius(_embed(a), power)[:, :12])


def test_fq6_square_inverse_frobenius(gpu, oracle):
    a = _tower(2, 256, 36)
    a[9] = 0
    np.testing.assert_array_equal(gpu.fq6_square(a), oracle.fq12_square(_embed(a))[:, :36])
    got, ok = gpu.fq6_inverse(a)
    exp, eok = oracle.fq12_inverse(_embed(a))
    np.testing.assert_array_equal(ok, eok.astype(bool))
    assert not ok[9]
    np.testing.assert_array_equal(got[ok], exp[ok][:, :36])
    for power in range(7):
        np.testing.assert_array_equal(gpu.fq6_frobenius_map(a, power), oracle.fq12_frobenius(_embed(a), power)[:, :36])


@pytest.mark.parametrize("exp", [[0], [1], [2], [0xD201000000010000], [3, 5, 7, 1 << 63], [0, 0, 0, 0, 0, 1]])
def test_fq_and_fq12_pow(gpu, oracle, exp):
    e = np.array(exp, np.uint64)
    a = _tower(3, 64, 6)
    np.testing.assert_array_equal(gpu.fq_pow(a, e), oracle.fq12_pow(_embed(a), e)[:, :6])
    f = _tower(4, 32, 72)
    np.testing.assert_array_equal(gpu.fq12_pow(f, e), oracle.fq12_pow(f, e))
