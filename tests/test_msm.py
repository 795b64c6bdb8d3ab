"""Variable-base scalar multiplication and multi-scalar multiplication
(SURVEY.md §8 f, rank 3).

Per-item products (CurveAffine::mul ec.rs:174-177 / mul_bits 88-95,
CurveProjective::mul_assign ec.rs:534-553) are bit-exact Jacobian words.
The MSM sum is compared as a point (PartialEq, ec.rs:45-85) with the oracle's
sum of CurveAffine::mul terms, and -- at sizes where the oracle's sum would be
slow -- with the size-independent identity
    sum_i s_i * (a_i G) = ((sum_i s_i a_i) mod r) * G
whose right side is the k*G path the reference's .dat vectors pin."""
import numpy as np
import pytest

from helpers import R_ORDER, from_limbs, limbs, random_scalars, rng, set_infinity, small_scalars

NT = 8


def edge_scalars():
    return small_scalars([0, 1, 2, 3, R_ORDER - 1, R_ORDER, R_ORDER + 1, (1 << 256) - 1, 1 << 255, 0xffff])


def combined_scalar(a, s):
    tot = sum(from_limbs(x) * from_limbs(y) for x, y in zip(a, s)) % R_ORDER
    return small_scalars([tot])


# ---------------- oracle ----------------

def test_oracle_affine_mul_matches_projective_mul(oracle):
    g = rng(31)
    s = np.concatenate([edge_scalars(), random_scalars(g, 22)])
    for gen, mul_aff, from_aff, mul_proj, eq in (
            (oracle.g1_mul_generator, oracle.g1_affine_mul, oracle.g1_from_affine, oracle.g1_mul, oracle.g1_eq),
            (oracle.g2_mul_generator, oracle.g2_affine_mul, oracle.g2_from_affine, oracle.g2_mul, oracle.g2_eq)):
        p = gen(random_scalars(g, len(s)), NT)
        set_infinity(p, [3])
        a = mul_aff(p, s, NT)
        b = mul_proj(from_aff(p), s)
        assert eq(a, b).all()


def test_oracle_affine_mul_of_generator_is_kg(oracle):
    # into_affine(G.mul(k)) equals the k*G path pinned by the reference's .dat vectors
    g = rng(32)
    k = np.concatenate([edge_scalars(), random_scalars(g, 6)])
    one = small_scalars([1])
    for gen, mul_aff, into in ((oracle.g1_mul_generator, oracle.g1_affine_mul, oracle.g1_into_affine),
                               (oracle.g2_mul_generator, oracle.g2_affine_mul, oracle.g2_into_affine)):
        base = np.repeat(gen(one), len(k), axis=0)
        np.testing.assert_array_equal(into(mul_aff(base, k)), gen(k))


def test_oracle_multiexp_identity(oracle):
    g = rng(33)
    n = 40
    a = random_scalars(g, n)
    s = np.concatenate([edge_scalars(), random_scalars(g, n - 10)])
    for gen, msm, eq, into in ((oracle.g1_mul_generator, oracle.g1_multiexp, oracle.g1_eq, oracle.g1_into_affine),
                               (oracle.g2_mul_generator, oracle.g2_multiexp, oracle.g2_eq, oracle.g2_into_affine)):
        got = msm(gen(a, NT), s, NT)
        np.testing.assert_array_equal(into(got), gen(combined_scalar(a, s)))
        zero = msm(gen(a[:0]), s[:0])
        assert into(zero)[0, -1] == 1   # empty sum = zero point


def test_python_layer_rejects_mismatched_lengths():
    import pairing_amd as pa
    with pytest.raises(ValueError):
        pa.g1_multiexp(np.zeros((3, 13), np.uint64), np.zeros((2, 4), np.uint64))
    with pytest.raises(ValueError):
        pa.g2_affine_mul(np.zeros((3, 25), np.uint64), np.zeros((4, 4), np.uint64))
    with pytest.raises(ValueError):
        pa.g1_mul_assign(np.zeros((3, 13), np.uint64), np.zeros((3, 4), np.uint64))


# ---------------- GPU parity ----------------

@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_scalar_mul_bit_exact(gpu, oracle, group):
    g = rng(40 + group)
    s = np.concatenate([edge_scalars(), random_scalars(g, 118)])
    gen = oracle.g1_mul_generator if group == 1 else oracle.g2_mul_generator
    p = gen(random_scalars(g, len(s)), NT)
    set_infinity(p, [5, 77])
    if group == 1:
        np.testing.assert_array_equal(gpu.g1_affine_mul(p, s), oracle.g1_affine_mul(p, s, NT))
        pj = oracle.g1_mul(oracle.g1_from_affine(p), small_scalars([7] * len(s)))  # non-normalized z
        np.testing.assert_array_equal(gpu.g1_mul_assign(pj, s), oracle.g1_mul(pj, s))
    else:
        np.testing.assert_array_equal(gpu.g2_affine_mul(p, s), oracle.g2_affine_mul(p, s, NT))
        pj = oracle.g2_mul(oracle.g2_from_affine(p), small_scalars([7] * len(s)))
        np.testing.assert_array_equal(gpu.g2_mul_assign(pj, s), oracle.g2_mul(pj, s))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 2, 3, 17, 300, 4099, 9000])
def test_g1_multiexp_matches_oracle(gpu, oracle, n):
    g = rng(50 + n)
    p = oracle.g1_mul_generator(random_scalars(g, n), NT)
    s = random_scalars(g, n)
    if n >= 17:
        s[:10] = edge_scalars()
        set_infinity(p, [11])
        p[12] = p[13]            # equal bases and digits: doubling inside a bucket
        s[12] = s[13]
        p[14] = p[15]            # P and -P
        p[14, 6:12] = oracle.fq_sub(np.zeros((1, 6), np.uint64), p[15:16, 6:12])[0]
        s[14] = s[15]
    got = gpu.g1_multiexp(p, s)
    exp = oracle.g1_multiexp(p, s, NT)
    assert oracle.g1_eq(got, exp).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 5, 200])
def test_g2_multiexp_matches_oracle(gpu, oracle, n):
    g = rng(60 + n)
    p = oracle.g2_mul_generator(random_scalars(g, n), NT)
    s = random_scalars(g, n)
    if n >= 5:
        s[:4] = small_scalars([0, 1, R_ORDER - 1, (1 << 256) - 1])
        set_infinity(p, [4])
    got = gpu.g2_multiexp(p, s)
    exp = oracle.g2_multiexp(p, s, NT)
    assert oracle.g2_eq(got, exp).all()


@pytest.mark.gpu
def test_g1_multiexp_large_identity(gpu, oracle):
    # 2^16 terms, window c = 13: sum s_i (a_i G) == (sum s_i a_i mod r) G
    g = rng(70)
    n = 1 << 16
    a = random_scalars(g, n)
    s = random_scalars(g, n)
    p = oracle.g1_mul_generator(a, NT)
    got = oracle.g1_into_affine(gpu.g1_multiexp(p, s))
    np.testing.assert_array_equal(got, oracle.g1_mul_generator(combined_scalar(a, s)))


@pytest.mark.gpu
def test_g1_multiexp_deterministic(gpu, oracle):
    # the bucketing sort is stable (term order inside a bucket), so two runs
    # give the same Jacobian words, not just the same point; 2^14 terms,
    # c = 11: two counting-sort passes, the second over 2 bits
    g = rng(80)
    n = 1 << 14
    p = oracle.g1_mul_generator(random_scalars(g, n), NT)
    s = random_scalars(g, n)
    s[100:300] = s[7]            # crowded buckets: runs far longer than a tile's share
    a = gpu.g1_multiexp(p, s)
    b = gpu.g1_multiexp(p, s)
    np.testing.assert_array_equal(a, b)
    assert oracle.g1_eq(a, oracle.g1_multiexp(p, s, NT)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("group,n", [(1, 9000), (2, 2000)])
def test_multiexp_crowded_buckets(gpu, oracle, group, n):
    """Every scalar equal: one bucket per window holds all n terms, spanning
    n/64 chunks, so its continuation pieces go through k_msm_long_fix (a block
    per bucket) instead of one lane; a few infinity bases and a second scalar
    value keep the rest of the machinery busy"""
    g = rng(95 + group)
    gen, msm, eq = ((oracle.g1_mul_generator, gpu.g1_multiexp, oracle.g1_eq) if group == 1 else
                    (oracle.g2_mul_generator, gpu.g2_multiexp, oracle.g2_eq))
    p = gen(random_scalars(g, n), NT)
    s = np.repeat(random_scalars(g, 1), n, axis=0)
    s[n // 3:n // 3 + 50] = random_scalars(g, 1)
    set_infinity(p, [5, n // 2])
    ref = oracle.g1_multiexp if group == 1 else oracle.g2_multiexp
    assert eq(msm(p, s), ref(p, s, NT)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("parts,chunk,wlo", [("1", "32", None), ("3", "8", None), ("8", "16", None), ("2", "512", None),
                                             ("3", "64", "12,5"), ("2", "64", "3,40"), ("3", "64", "5,10"),
                                             ("2", "64", "40"), ("2", "64", "0")])
def test_multiexp_window_parts(gpu, oracle, parts, chunk, wlo):
    """The MSM's launch structure (kernels_msm.hip msm_run): the windows in
    PA_MSM_PARTS parts on side streams, PA_MSM_CHUNK sorted items per lane
    (read once per process, hence a subprocess): small chunks put most buckets
    across several chunks (the continuation pieces), many parts cut chunks at
    window boundaries; the sum stays the same point (ec.rs:45-85).  PA_MSM_WLO
    (unequal parts, A/B) is taken whole or not at all: a malformed list (wrong
    length, not descending, a bound of 0 or >= W) falls back to the even split"""
    import os
    import subprocess
    import sys
    import tempfile
    g = rng(90)
    n1, n2 = 4099, 200
    p1 = oracle.g1_mul_generator(random_scalars(g, n1), NT)
    s1 = random_scalars(g, n1)
    s1[:10] = edge_scalars()
    set_infinity(p1, [11])
    s1[100:300] = s1[7]          # crowded buckets
    p2 = oracle.g2_mul_generator(random_scalars(g, n2), NT)
    s2 = random_scalars(g, n2)
    s2[:4] = small_scalars([0, 1, R_ORDER - 1, (1 << 256) - 1])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import pairing_amd as pa; d = sys.argv[1]; "
            "np.save(d + '/o1.npy', pa.g1_multiexp(np.load(d + '/p1.npy'), np.load(d + '/s1.npy'))); "
            "np.save(d + '/o2.npy', pa.g2_multiexp(np.load(d + '/p2.npy'), np.load(d + '/s2.npy')))" % root)
    with tempfile.TemporaryDirectory() as d:
        for name, a in (("p1", p1), ("s1", s1), ("p2", p2), ("s2", s2)):
            np.save(os.path.join(d, name + ".npy"), a)
        env = dict(os.environ, PA_MSM_PARTS=parts, PA_MSM_CHUNK=chunk)
        if wlo is not None:
            env["PA_MSM_WLO"] = wlo
        r = subprocess.run([sys.executable, "-c", code, d], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        o1, o2 = np.load(os.path.join(d, "o1.npy")), np.load(os.path.join(d, "o2.npy"))
    assert oracle.g1_eq(o1, oracle.g1_multiexp(p1, s1, NT)).all()
    assert oracle.g2_eq(o2, oracle.g2_multiexp(p2, s2, NT)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("group,n", [(1, 1 << 20), (2, 1 << 18)])
def test_multiexp_bench_size_identity(gpu, oracle, group, n):
    """bench.py --workload msm's size (2^20 G1 terms: c = 16, two window parts
    on side streams, 64-item chunks) and 2^18 G2 terms (c = 15, whose
    carry-only top window crowds ~45 % of the terms into one bucket, folded by
    k_msm_long_fix): bases a_i g made on the device (fixed-base comb + batch
    normalization, both checked elsewhere), the size-independent identity
    sum s_i (a_i g) = (sum s_i a_i mod r) g; a run of equal scalars and a few
    zeros ride along"""
    import torch
    import pairing_amd.device as pdev
    from helpers import from_limbs
    g = rng(120 + group)
    a = random_scalars(g, n)
    s = random_scalars(g, n)
    s[1000:3000] = s[5]
    s[7:12] = 0
    w, aw = (18, 13) if group == 1 else (36, 25)
    gen_aff = (oracle.g1_mul_generator if group == 1 else oracle.g2_mul_generator)(small_scalars([1]))
    base = torch.from_numpy((oracle.g1_from_affine if group == 1 else oracle.g2_from_affine)(gen_aff)
                            .view(np.int64)).cuda()
    ka = torch.from_numpy(a.view(np.int64)).cuda()
    jac = pdev.empty_records(n, w, "cuda")
    if group == 1:
        table, _ = pdev.g1_fixed_base_table(base)
        pdev.g1_fixed_base_mul(table, ka, jac)
        pdev.g1_batch_normalization(jac)
    else:
        table, ws = pdev.g2_fixed_base_buffers("cuda")
        pdev.g2_wnaf_fixed_base(base, ka, jac, table, ws)
        pdev.g2_batch_normalization(jac)
    bases = torch.zeros((n, aw), dtype=torch.int64, device="cuda")
    bases[:, :aw - 1] = jac[:, :aw - 1]
    del jac, table
    out = pdev.empty_records(1, w, "cuda")
    pdev.multiexp(group, bases, torch.from_numpy(s.view(np.int64)).cuda(), out, pdev.multiexp_workspace(group, n, "cuda"))
    torch.cuda.synchronize()
    tot = sum(from_limbs(x) * from_limbs(y) for x, y in zip(a, s)) % R_ORDER
    into = oracle.g1_into_affine if group == 1 else oracle.g2_into_affine
    gen = oracle.g1_mul_generator if group == 1 else oracle.g2_mul_generator
    np.testing.assert_array_equal(into(out.cpu().numpy().view(np.uint64)), gen(small_scalars([tot])))
