"""PrimeField::from_repr / into_repr for Fq over a batch (fq.rs:747-775):
pa_fq_from_repr_batch / pa_fq_into_repr_batch against the oracle (itself
pinned to a Python big-integer model in tests/test_oracle.py), with the
validity edges of FqRepr::is_valid (fq.rs:777-780): q - 1 valid, q, q + 1,
2^381 and 2^384 - 1 not (Err(NotInField), out = 0)."""
import numpy as np
import pytest

from helpers import Q, limbs, mont, random_fq, rng


def repr_rows(vals):
    return np.array([limbs(v % (1 << 384)) for v in vals], np.uint64)


EDGE = [0, 1, 2, Q - 1, Q - 2, (1 << 380) - 1, 1 << 380, Q, Q + 1, 1 << 381, (1 << 384) - 1, 2 * Q]


def test_fq_repr_oracle_matches_python_model(oracle):
    g = rng(61)
    vals = EDGE + [int.from_bytes(g.bytes(48), "little") % Q for _ in range(200)]
    out, ok = oracle.fq_from_repr(repr_rows(vals))
    for v, o, k in zip(vals, out, ok):
        assert bool(k) == (v < Q)
        if v < Q:
            assert [int(w) for w in o] == mont(v)
    a = random_fq(g, 300)
    back = oracle.fq_into_repr(a)
    again, okb = oracle.fq_from_repr(back)
    assert okb.all()
    np.testing.assert_array_equal(again, a)


@pytest.mark.gpu
def test_fq_from_into_repr_match_oracle(gpu, oracle):
    g = rng(62)
    vals = EDGE + [int.from_bytes(g.bytes(48), "little") % Q for _ in range(4096)] + \
        [int.from_bytes(g.bytes(48), "little") for _ in range(1024)]      # ~all >= q: Err
    r = repr_rows(vals)
    out, ok = gpu.fq_from_repr(r)
    exp, exp_ok = oracle.fq_from_repr(r)
    np.testing.assert_array_equal(ok, exp_ok.astype(bool))
    np.testing.assert_array_equal(out[ok], exp[ok])
    assert not out[~ok].any()
    assert ok.sum() == sum(v < Q for v in vals)
    a = np.concatenate([exp[exp_ok.astype(bool)], random_fq(g, 4096)])
    np.testing.assert_array_equal(gpu.fq_into_repr(a), oracle.fq_into_repr(a))
    # round trip: from_repr(into_repr(a)) == a
    back, okb = gpu.fq_from_repr(gpu.fq_into_repr(a))
    assert okb.all()
    np.testing.assert_array_equal(back, a)
    # empty batch
    e, eok = gpu.fq_from_repr(np.zeros((0, 6), np.uint64))
    assert e.shape == (0, 6) and eok.shape == (0,)
