"""The CurveProjective / CurveAffine surface for G1 and G2 (ec.rs:1-621,
lib.rs:114-234): per-op batches, G2 batch_normalization, G2 fixed-base
wNAF and the window heuristics, against the oracle.

Jacobian outputs of the group law must be bit-identical to the reference's
(same formula sequence); fixed-base outputs equal as points (PartialEq,
ec.rs:45-85) and bit-identical after batch_normalization."""
import numpy as np
import pytest

from helpers import Q, R_ORDER, RMONT, limbs, random_scalars, rng, set_infinity, small_scalars

NT = 8


def _neg_rows(rows, y0, fw):
    """negate the Fq/Fq2 y coordinate words [y0, y0 + fw) of nonzero entries (Montgomery q - y)"""
    out = rows.copy()
    for k in range(out.shape[0]):
        for c in range(fw // 6):
            s = y0 + 6 * c
            v = sum(int(w) << (64 * i) for i, w in enumerate(out[k, s:s + 6]))
            out[k, s:s + 6] = limbs((Q - v) % Q)
    return out


def _jacobian(oracle, group, seed, n):
    """non-normalized Jacobian points with zeros (garbage x, y, z = 0),
    normalized points and a doubled point mixed in"""
    g = rng(seed)
    s = random_scalars(g, n)
    if group == 1:
        v = oracle.g1_mul_generator_jacobian(s, NT)
        aff = oracle.g1_into_affine(v)
        v = oracle.g1_double(v)
        fw = 6
    else:
        aff = oracle.g2_mul_generator(s, NT)
        v = oracle.g2_double(oracle.g2_from_affine(aff))
        fw = 12
    v[[1, n // 3], 2 * fw:3 * fw] = 0                                  # zeros
    norm = [2, n // 2]
    v[norm] = (oracle.g1_from_affine if group == 1 else oracle.g2_from_affine)(
        (oracle.g1_into_affine if group == 1 else oracle.g2_into_affine)(v[norm]))
    return v, aff


# ---------------- window heuristics (host only, CPU) ----------------
def test_recommended_wnaf_matches_reference(oracle):
    import pairing_amd as pa
    L = oracle.lib()
    for n in list(range(0, 130)) + [562, 563, 564, 1630, 1631, 3128, 3129, 7933, 7934, 62569, 62570, 84071,
                                    84072, 1 << 18, 1 << 20, 10 ** 9]:
        assert pa.g1_recommended_wnaf_for_num_scalars(n) == L.o_g1_recommended_wnaf_for_num_scalars(n)
        assert pa.g2_recommended_wnaf_for_num_scalars(n) == L.o_g2_recommended_wnaf_for_num_scalars(n)
    vals = [0, 1, 2, 3] + [(1 << b) - 1 for b in (33, 34, 35, 36, 37, 38, 102, 103, 104, 129, 130, 131, 255, 256)] \
        + [1 << b for b in (33, 36, 102, 129, 200)] + [R_ORDER - 1]
    for v in vals:
        s = np.array([limbs(v, 4)], np.uint64)
        assert pa.g1_recommended_wnaf_for_scalar(s) == L.o_g1_recommended_wnaf_for_scalar(s.ctypes.data), v
        assert pa.g2_recommended_wnaf_for_scalar(s) == L.o_g2_recommended_wnaf_for_scalar(s.ctypes.data), v


# ---------------- group law on the GPU ----------------
@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_group_law_bit_exact(gpu, oracle, group):
    n = 130
    a, aff_a = _jacobian(oracle, group, 60 + group, n)
    b, aff_b = _jacobian(oracle, group, 70 + group, n)
    fw = 6 if group == 1 else 12
    o = (oracle.g1_double, oracle.g1_add, oracle.g1_add_mixed, oracle.g1_into_affine, oracle.g1_from_affine,
         oracle.g1_eq) if group == 1 else \
        (oracle.g2_double, oracle.g2_add, oracle.g2_add_mixed, oracle.g2_into_affine, oracle.g2_from_affine,
         oracle.g2_eq)
    dbl, add, madd, to_aff, from_aff, eq = o
    G = lambda name: getattr(gpu, "g%d_%s" % (group, name))
    # the doubling fallback of add (u1 == u2, s1 == s2, ec.rs:394-396) and P + (-P) (ec.rs:398)
    b[5] = a[5]
    b[6] = _neg_rows(a[6:7], fw, fw)[0]
    aff_b = aff_b.copy()
    aff_b[7] = to_aff(a[7:8])[0]
    aff_b[8] = to_aff(_neg_rows(a[8:9], fw, fw))[0]
    set_infinity(aff_b, [9])
    np.testing.assert_array_equal(G("double")(a), dbl(a))
    np.testing.assert_array_equal(G("add")(a, b), add(a, b))
    np.testing.assert_array_equal(G("add_mixed")(a, aff_b), madd(a, aff_b))
    neg = G("negate")(a)
    nz = a[:, 2 * fw:3 * fw].any(axis=1)
    np.testing.assert_array_equal(neg[~nz], a[~nz])                      # zero stays untouched
    np.testing.assert_array_equal(neg[nz], _neg_rows(a[nz], fw, fw))
    np.testing.assert_array_equal(G("sub")(a, b), add(a, _neg_rows_nonzero(b, fw)))
    np.testing.assert_array_equal(G("into_affine")(a), to_aff(a))
    np.testing.assert_array_equal(G("into_projective")(aff_a), from_aff(aff_a))
    inf = aff_a.copy()
    set_infinity(inf, [0, 3])
    np.testing.assert_array_equal(G("into_projective")(inf), from_aff(inf))
    # a + b == b + a as points
    assert eq(G("add")(a, b), G("add")(b, a)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_partial_eq_matches_reference(gpu, oracle, group):
    """PartialEq (ec.rs:45-85) per item: the same point in two Jacobian
    representations, a point and its negation (same X Z^-2, other Y), zero vs
    zero (garbage x, y), zero vs nonzero, unrelated points"""
    n = 130
    a, _ = _jacobian(oracle, group, 90 + group, n)
    fw = 6 if group == 1 else 12
    to_aff, from_aff, add, eq = (oracle.g1_into_affine, oracle.g1_from_affine, oracle.g1_add, oracle.g1_eq) \
        if group == 1 else (oracle.g2_into_affine, oracle.g2_from_affine, oracle.g2_add, oracle.g2_eq)
    b = from_aff(to_aff(a))                          # same points, Z = 1 (zero stays zero)
    b[10:20] = _neg_rows_nonzero(a[10:20], fw)       # negations
    b[20:30] = add(a[20:30], a[30:40])               # other points
    a[40] = a[1]                                     # zero vs zero: two garbage encodings
    b[40] = a[1]
    b[40, :2 * fw] = np.uint64(5)
    b[41] = a[1]                                     # zero vs nonzero
    got = getattr(gpu, "g%d_eq" % group)(a, b)
    want = eq(a, b)
    np.testing.assert_array_equal(got, want)
    assert want[:10].all() and not want[10:30].any() and want[40] and not want[41]
    assert want[1] and want[n // 3]                  # a zero against its own copy


def _neg_rows_nonzero(rows, fw):
    out = rows.copy()
    nz = rows[:, 2 * fw:3 * fw].any(axis=1)
    out[nz] = _neg_rows(rows[nz], fw, fw)
    return out


@pytest.mark.gpu
def test_group_add_device_entry(gpu, oracle):
    import torch
    import pairing_amd.device as pdev
    a, _ = _jacobian(oracle, 2, 80, 300)
    b, _ = _jacobian(oracle, 2, 81, 300)
    da = torch.from_numpy(a.view(np.int64)).to("cuda:0")
    db = torch.from_numpy(b.view(np.int64)).to("cuda:0")
    out = pdev.empty_records(300, 36, "cuda:0")
    pdev.group_add(2, da, db, out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), oracle.g2_add(a, b))


# ---------------- G2 batch_normalization ----------------
@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3, 4, 5, 1000, 4099])
def test_g2_batch_normalization_bit_exact(gpu, oracle, n):
    v, _ = _jacobian(oracle, 2, 90 + n, max(n, 8))
    v = v[:n].copy()
    np.testing.assert_array_equal(gpu.g2_batch_normalization(v), oracle.g2_batch_normalization(v))


# ---------------- G2 fixed-base wNAF ----------------
@pytest.mark.gpu
@pytest.mark.parametrize("zero_base", [False, True])
def test_g2_fixed_base_equals_reference_wnaf(gpu, oracle, zero_base):
    g = rng(95)
    base = oracle.g2_double(oracle.g2_from_affine(oracle.g2_mul_generator(random_scalars(g, 1))))
    if zero_base:
        base[0, 24:36] = 0
    s = random_scalars(g, 700)
    s[0] = 0
    s[1] = limbs(1, 4)
    s[2] = limbs(R_ORDER - 1, 4)
    s[3] = limbs((1 << 255) - 1, 4)
    s[4] = limbs(128 + 256 * 128, 4)    # digit edges of the signed recoding
    s[5] = limbs(0x81 << 128, 4)
    got = gpu.g2_wnaf_fixed_base(base, s)
    exp = oracle.g2_wnaf_fixed_base(base, s, NT)
    assert oracle.g2_eq(got, exp).all()
    if not zero_base:
        np.testing.assert_array_equal(gpu.g2_batch_normalization(got), oracle.g2_batch_normalization(exp))


@pytest.mark.gpu
def test_g2_fixed_base_linearity(gpu, oracle):
    """(s_i + s_j) g == s_i g + s_j g over a 2^14 batch"""
    g = rng(96)
    base = oracle.g2_from_affine(oracle.g2_mul_generator(small_scalars([7])))
    n = 1 << 14
    s = np.ascontiguousarray(random_scalars(g, 2048)[np.arange(n) % 2048])
    s[:, 0] ^= np.arange(n, dtype=np.uint64)
    s[:, 3] &= np.uint64(0x0fffffffffffffff)
    got = gpu.g2_wnaf_fixed_base(base, s)
    i, j = np.arange(0, 64), np.arange(n - 64, n)
    ssum = np.array([limbs((sum(int(x) << (64 * k) for k, x in enumerate(s[a])) +
                            sum(int(x) << (64 * k) for k, x in enumerate(s[b]))) % R_ORDER, 4)
                     for a, b in zip(i, j)], np.uint64)
    lhs = gpu.g2_add(np.ascontiguousarray(got[i]), np.ascontiguousarray(got[j]))
    assert oracle.g2_eq(lhs, oracle.g2_wnaf_fixed_base(base, ssum, NT)).all()
