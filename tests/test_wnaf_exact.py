"""Bit-exact Wnaf (wnaf.rs:1-179) on the GPU: the Jacobian X, Y, Z words of
Wnaf::new().base(g, n).scalar(s_i) and Wnaf::new().scalar(s).base(g_i) equal
the oracle's restatement of the reference's table chain, wnaf_form and
wnaf_exp (oracle/oracle_curve.c o_g{1,2}_wnaf_fixed_base_w / _fixed_scalar).

The fixed-base table is rebuilt from the chain's closed form (a prefix scan
over z -> c z^3, kernels_wnaf_exact.hip); bases whose chain takes a special
branch (zero, small-order points outside G1) take the serial chain.  Both are
covered here, as are the wnaf_form edges: zero, one, r - 1, values above r,
and the add_nocarry wrap (wnaf.rs:30-35) at every window tested."""
import numpy as np
import pytest

from helpers import RMONT, R_ORDER, limbs, random_fq, random_scalars, rng

NT = 8


def _edge_scalars(g, n):
    s = random_scalars(g, n)
    edges = [0, 1, 2, 3, R_ORDER - 1, R_ORDER, (1 << 255) - 1, (1 << 256) - 1, (1 << 256) - 3,
             (1 << 256) - 5, (1 << 256) - 0x1001, 128 + 256 * 128, 0x81 << 128, (1 << 64) - 1, 1 << 200]
    for k, v in enumerate(edges):
        s[k] = limbs(v, 4)
    return s


def _g1_base(oracle, seed):
    """a non-normalized Jacobian base in G1"""
    return oracle.g1_double(oracle.g1_mul_generator_jacobian(random_scalars(rng(seed), 1)))


def _g2_base(oracle, seed):
    return oracle.g2_double(oracle.g2_from_affine(oracle.g2_mul_generator(random_scalars(rng(seed), 1))))


def _torsion_bases(oracle, group):
    """Jacobian bases outside the subgroup: a pure small-order point (its chain
    hits the zero point: serial path) and subgroup + torsion (generic branches)"""
    from decode_cases import subgroup_records
    recs, truth = subgroup_records(group, 7, n=3)
    aff, st = oracle.decode(group, recs, False, checked=False)
    assert (st == 0).all()
    jac = oracle.g1_from_affine(aff) if group == 1 else oracle.g2_from_affine(aff)
    return jac[~truth]


def _check_fixed_base(gpu, oracle, group, base, s, window):
    if group == 1:
        got = gpu.g1_wnaf_fixed_base_exact(base, s, window)
        exp = oracle.g1_wnaf_fixed_base(base, s, NT, window=window)
    else:
        got = gpu.g2_wnaf_fixed_base_exact(base, s, window)
        exp = oracle.g2_wnaf_fixed_base(base, s, NT, window=window)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("window", [1, 2, 3, 5, 9, 12, 16])
def test_g1_fixed_base_exact_words(gpu, oracle, window):
    g = rng(300 + window)
    _check_fixed_base(gpu, oracle, 1, _g1_base(oracle, window), _edge_scalars(g, 257), window)


@pytest.mark.gpu
@pytest.mark.parametrize("window", [1, 4, 7, 15])
def test_g2_fixed_base_exact_words(gpu, oracle, window):
    g = rng(320 + window)
    _check_fixed_base(gpu, oracle, 2, _g2_base(oracle, window), _edge_scalars(g, 129), window)


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_fixed_base_exact_default_window(gpu, oracle, group):
    """window None = recommended_wnaf_for_num_scalars(n), as Wnaf::base picks"""
    g = rng(340 + group)
    s = _edge_scalars(g, 700)
    base = _g1_base(oracle, 41) if group == 1 else _g2_base(oracle, 42)
    got = (gpu.g1_wnaf_fixed_base_exact if group == 1 else gpu.g2_wnaf_fixed_base_exact)(base, s)
    exp = (oracle.g1_wnaf_fixed_base if group == 1 else oracle.g2_wnaf_fixed_base)(base, s, NT)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_fixed_base_exact_special_bases(gpu, oracle, group):
    """zero bases (reference zero and z = 0 with other words), a normalized base,
    and bases outside the subgroup: the serial chain or the closed form, words equal"""
    g = rng(350 + group)
    s = _edge_scalars(g, 40)
    jw = 18 if group == 1 else 36
    fw = jw // 3
    base = _g1_base(oracle, 43) if group == 1 else _g2_base(oracle, 44)
    zero_ref = np.zeros((1, jw), np.uint64)
    zero_ref[0, fw:fw + 6] = limbs(RMONT)        # G::zero() = (0, 1, 0), ec.rs:224-230
    zero_odd = base.copy()
    zero_odd[0, 2 * fw:] = 0
    norm = oracle.g1_batch_normalization(base) if group == 1 else oracle.g2_batch_normalization(base)
    cases = [zero_ref, zero_odd, norm] + [t.reshape(1, jw) for t in _torsion_bases(oracle, group)[:4]]
    for b in cases:
        for w in (2, 5):
            _check_fixed_base(gpu, oracle, group, np.ascontiguousarray(b), s, w)


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_fixed_base_exact_off_curve_bases(gpu, oracle, group):
    """Jacobian words that are not a curve point (the reference computes its
    chain on them all the same): the serial chain, and the multiply with a zero
    test before every doubling"""
    g = rng(355 + group)
    s = _edge_scalars(g, 40)
    jw = 18 if group == 1 else 36
    base = random_fq(g, jw // 6).reshape(1, jw)
    for w in (1, 3, 6):
        _check_fixed_base(gpu, oracle, group, np.ascontiguousarray(base), s, w)


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_fixed_scalar_exact_words(gpu, oracle, group):
    """Wnaf::new().scalar(s).base(g_i): a table per base (zeros, normalized and
    Jacobian bases mixed), the recommended window and explicit ones"""
    from test_group import _jacobian
    bases, _ = _jacobian(oracle, group, 360 + group, 150)
    g = rng(370 + group)
    fn = gpu.g1_wnaf_fixed_scalar_exact if group == 1 else gpu.g2_wnaf_fixed_scalar_exact
    ofs = oracle.g1_wnaf_fixed_scalar if group == 1 else oracle.g2_wnaf_fixed_scalar
    ofb = oracle.g1_wnaf_fixed_base if group == 1 else oracle.g2_wnaf_fixed_base
    for s in list(_edge_scalars(g, 20)[:15]) + list(random_scalars(g, 2)) + [limbs(5, 4), limbs(1 << 40, 4)]:
        s = np.ascontiguousarray(np.asarray(s, np.uint64).reshape(1, 4))
        np.testing.assert_array_equal(fn(bases, s), ofs(bases, s[0], NT))
    # explicit windows: the same table chain and digits as a one-scalar fixed base
    s = np.ascontiguousarray(random_scalars(g, 1))
    for w in (1, 6):
        got = fn(bases[:12], s, w)
        exp = np.concatenate([ofb(np.ascontiguousarray(bases[k:k + 1]), s, 1, window=w) for k in range(12)])
        np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
def test_g1_fixed_base_exact_config3_size(gpu, oracle):
    """2^18 scalars at the recommended window (16): sampled rows bit-exact"""
    n = 1 << 18
    g = rng(380)
    base = _g1_base(oracle, 45)
    s = np.ascontiguousarray(random_scalars(g, 4096)[np.arange(n) % 4096])
    s[:, 0] ^= np.arange(n, dtype=np.uint64)
    got = gpu.g1_wnaf_fixed_base_exact(base, s)
    idx = rng(381).choice(n, 192, replace=False)
    exp = oracle.g1_wnaf_fixed_base(base, np.ascontiguousarray(s[idx]), NT, window=16)
    np.testing.assert_array_equal(got[idx], exp)


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_wnaf_exact_device_entries(gpu, oracle, group):
    """the _device forms on torch-owned HBM, stream-ordered"""
    import torch
    from pairing_amd import device as pdev
    g = rng(390 + group)
    jw = 18 if group == 1 else 36
    base = _g1_base(oracle, 46) if group == 1 else _g2_base(oracle, 47)
    s = _edge_scalars(g, 100)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")  # noqa: E731
    out = pdev.empty_records(100, jw, "cuda:0")
    ws = pdev.wnaf_exact_workspace(group, 100, 6, False, "cuda:0")
    pdev.wnaf_fixed_base_exact(group, to(base), to(s), out, 6, ws)
    torch.cuda.synchronize()
    ofb = oracle.g1_wnaf_fixed_base if group == 1 else oracle.g2_wnaf_fixed_base
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), ofb(base, s, NT, window=6))
    bases = np.concatenate([base] * 5)
    out2 = pdev.empty_records(5, jw, "cuda:0")
    ws2 = pdev.wnaf_exact_workspace(group, 5, 4, True, "cuda:0")
    pdev.wnaf_fixed_scalar_exact(group, to(bases), to(s[7:8]), out2, 4, ws2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out2.cpu().numpy().view(np.uint64), np.concatenate([ofb(base, s[7:8], 1, window=4)] * 5))


def test_wnaf_exact_workspace_sizes():
    """host-side layout: grows with n and window, 0 outside the accepted windows"""
    from pairing_amd._native import _lib
    for group in (1, 2):
        assert _lib.pa_wnaf_exact_workspace_bytes(group, 1000, 0, 0) == 0
        assert _lib.pa_wnaf_exact_workspace_bytes(group, 1000, 21, 0) == 0
        assert _lib.pa_wnaf_exact_workspace_bytes(group, 1000, 13, 1) == 0
        a = _lib.pa_wnaf_exact_workspace_bytes(group, 1000, 4, 0)
        b = _lib.pa_wnaf_exact_workspace_bytes(group, 1000, 16, 0)
        c = _lib.pa_wnaf_exact_workspace_bytes(group, 2000, 16, 0)
        assert 0 < a < b < c
        # the table alone: 2^15 entries of 3 field elements
        assert b >= (1 << 15) * 3 * (48 if group == 1 else 96)
    assert _lib.pa_wnaf_exact_workspace_bytes(3, 10, 4, 0) == 0


def test_wnaf_exact_window_rejected():
    """windows outside the exact entries' range fail loudly before any GPU work"""
    import pairing_amd as pa
    from pairing_amd._native import PairingError
    base = np.zeros((1, 18), np.uint64)
    s = np.zeros((3, 4), np.uint64)
    with pytest.raises(PairingError):
        pa.g1_wnaf_fixed_base_exact(base, s, 21)
    with pytest.raises(PairingError):
        pa.g1_wnaf_fixed_scalar_exact(np.zeros((3, 18), np.uint64), s[:1], 13)
