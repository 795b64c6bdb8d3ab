"""Point decoding / encoding and square roots (SURVEY.md §8 f, rank 1).

CPU (oracle): the reference's invalid-vector suites
(src/bls12_381/tests/mod.rs:98-560, re-expressed in decode_cases.py) give the
expected GroupDecodingError for every record; the k*G vectors (pinned to the
reference's .dat files by test_oracle.py) decode to k*G and re-encode to the
same bytes; Fq sqrt equals a^((q+1)/4) computed with Python integers.

GPU (-m gpu): the HIP kernels behind pa_g{1,2}_{decode,encode}_batch and
pa_fq{,2}_sqrt_batch equal the oracle bit for bit (points, status bytes,
encodings, roots) on the same records, checked and unchecked.  Every decode
test runs on both decode kernels (pa_set_decode_kernel): one lane per record
(k_decode, large batches) and one record per group of lane quads
(k_decode_quad, the latency form small batches take by default).
"""
import numpy as np
import pytest

import decode_cases as D
from helpers import Q, limbs, mont, random_fq, rng, small_scalars, unmont

SIZES = {(1, False): 96, (1, True): 48, (2, False): 192, (2, True): 96}
FORMATS = [(1, False), (1, True), (2, False), (2, True)]


def _cases(group, compressed):
    c = D.g1_cases(compressed) if group == 1 else D.g2_cases(compressed)
    return D.as_array(c, SIZES[(group, compressed)])


def _kg(oracle, group, compressed, count):
    raw = oracle.kg_vectors(group, count, compressed)
    return np.frombuffer(raw, np.uint8).reshape(count, SIZES[(group, compressed)]).copy()


def _kg_points(oracle, group, count):
    s = small_scalars(list(range(count)))
    return oracle.g1_mul_generator(s) if group == 1 else oracle.g2_mul_generator(s)


def _mixed_records(oracle, group, compressed, seed):
    """reference suites + k*G + garbage: the parity input of the GPU tests"""
    enc_c, _ = _cases(group, compressed)
    kg = _kg(oracle, group, compressed, 200)
    junk = D.garbage(rng(seed), 200, SIZES[(group, compressed)], compressed)
    return np.concatenate([enc_c, kg, junk])


# ---------------- CPU: the oracle against the reference's own suites ----------------
@pytest.mark.parametrize("group,compressed", FORMATS)
def test_oracle_invalid_vector_suites(oracle, group, compressed):
    enc, want = _cases(group, compressed)
    _, st = oracle.decode(group, enc, compressed)
    assert st.tolist() == want.tolist()


@pytest.mark.parametrize("group,compressed", FORMATS)
def test_oracle_decodes_kg_vectors(oracle, group, compressed):
    """tests/mod.rs:55-97 reads the .dat records back the same way"""
    n = 100
    enc = _kg(oracle, group, compressed, n)
    pts, st = oracle.decode(group, enc, compressed)
    assert not st.any()
    assert np.array_equal(pts, _kg_points(oracle, group, n))


@pytest.mark.parametrize("group,compressed", FORMATS)
def test_oracle_unchecked_skips_curve_and_subgroup(oracle, group, compressed):
    enc, want = _cases(group, compressed)
    _, st = oracle.decode(group, enc, compressed, checked=False)
    exp = want.copy()
    exp[exp == D.NOT_IN_SUBGROUP] = D.OK
    if not compressed:   # decompression still needs a square root
        exp[exp == D.NOT_ON_CURVE] = D.OK
    assert st.tolist() == exp.tolist()


def test_oracle_fq_sqrt_matches_integer_model(oracle):
    a = random_fq(rng(3), 64)
    a[0] = 0
    root, ok = oracle.fq_sqrt(a)
    for k in range(a.shape[0]):
        v = unmont(a[k])
        assert bool(ok[k]) == D.is_square_fq(v)
        if ok[k]:
            assert unmont(root[k]) == pow(v, (Q + 1) // 4, Q)


def test_oracle_fq2_sqrt_matches_integer_model(oracle):
    a = random_fq(rng(4), 32).reshape(16, 12)
    root, ok = oracle.fq2_sqrt(a)
    for k in range(a.shape[0]):
        v = (unmont(a[k, :6]), unmont(a[k, 6:]))
        assert bool(ok[k]) == D.is_square_fq2(v)
        if ok[k]:
            assert (unmont(root[k, :6]), unmont(root[k, 6:])) == D.sqrt_fq2(v)


# ---------------- GPU parity ----------------
@pytest.fixture(params=[1, 2], ids=["one_lane", "quad"])
def decode_kernel(request, gpu):
    gpu.set_decode_kernel(request.param)
    yield request.param
    gpu.set_decode_kernel(0)


@pytest.mark.gpu
@pytest.mark.parametrize("group,compressed", FORMATS)
@pytest.mark.parametrize("checked", [True, False])
def test_gpu_decode_matches_oracle(gpu, oracle, decode_kernel, group, compressed, checked):
    enc = _mixed_records(oracle, group, compressed, seed=10 * group + compressed)
    want_pts, want_st = oracle.decode(group, enc, compressed, checked=checked, nthreads=16)
    dec = gpu.g1_decode if group == 1 else gpu.g2_decode
    pts, st = dec(enc, compressed, checked)
    assert st.tolist() == want_st.tolist()
    assert np.array_equal(pts, want_pts)


@pytest.mark.gpu
@pytest.mark.parametrize("group,compressed", FORMATS)
def test_gpu_decode_reference_suites(gpu, decode_kernel, group, compressed):
    enc, want = _cases(group, compressed)
    dec = gpu.g1_decode if group == 1 else gpu.g2_decode
    _, st = dec(enc, compressed)
    assert st.tolist() == want.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("group,compressed", FORMATS)
def test_gpu_encode_reproduces_kg_vectors(gpu, oracle, group, compressed):
    n = 500
    pts = _kg_points(oracle, group, n)
    enc = (gpu.g1_encode if group == 1 else gpu.g2_encode)(pts, compressed)
    assert np.array_equal(enc, _kg(oracle, group, compressed, n))


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_gpu_encode_decode_round_trip_random_points(gpu, oracle, decode_kernel, group):
    from helpers import random_scalars
    s = random_scalars(rng(20 + group), 300)
    pts = oracle.g1_mul_generator(s, 16) if group == 1 else oracle.g2_mul_generator(s, 16)
    enc_f = gpu.g1_encode if group == 1 else gpu.g2_encode
    dec_f = gpu.g1_decode if group == 1 else gpu.g2_decode
    for compressed in (False, True):
        enc = enc_f(pts, compressed)
        back, st = dec_f(enc, compressed)
        assert not st.any()
        assert np.array_equal(back, pts)


@pytest.mark.gpu
def test_gpu_fq_sqrt_matches_oracle(gpu, oracle):
    a = random_fq(rng(30), 4096)
    a[0] = 0
    a[1] = mont(Q - 1)   # -1 is a non-residue (q = 3 mod 4)
    a[2] = mont(4)
    want, want_ok = oracle.fq_sqrt(a)
    got, ok = gpu.fq_sqrt(a)
    assert ok.tolist() == want_ok.astype(bool).tolist()
    assert np.array_equal(got[ok], want[ok])
    assert 1500 < int(ok.sum()) < 2600


@pytest.mark.gpu
def test_gpu_fq2_sqrt_matches_oracle(gpu, oracle):
    a = random_fq(rng(31), 2048).reshape(1024, 12)
    a[0] = 0
    a[1, :6] = mont(Q - 1)   # -1 (alpha == -1 branch candidates)
    a[1, 6:] = 0
    a[2, :6] = 0
    a[2, 6:] = limbs(0)
    sq = oracle.fq2_square(a[3:400].copy())   # squares: always Some
    a[3:400] = sq
    want, want_ok = oracle.fq2_sqrt(a)
    got, ok = gpu.fq2_sqrt(a)
    assert ok.tolist() == want_ok.astype(bool).tolist()
    assert np.array_equal(got[ok], want[ok])
    assert ok[3:400].all()


# ---------------- subgroup membership: r * P == 0 vs the GPU's endomorphism test ----------------
@pytest.fixture(scope="module", params=[1, 2])
def subgroup_case(request):
    enc, truth = D.subgroup_records(request.param, seed=40 + request.param, n=3)
    return request.param, enc, truth


def test_oracle_subgroup_check_matches_integer_model(oracle, subgroup_case):
    group, enc, truth = subgroup_case
    _, st = oracle.decode(group, enc, False, checked=True, nthreads=4)
    assert st.tolist() == [D.OK if t else D.NOT_IN_SUBGROUP for t in truth]
    assert truth.any() and not truth.all()


@pytest.mark.gpu
def test_gpu_subgroup_check_matches_oracle(gpu, oracle, decode_kernel, subgroup_case):
    group, enc, truth = subgroup_case
    want_pts, want_st = oracle.decode(group, enc, False, checked=True, nthreads=4)
    pts, st = (gpu.g1_decode if group == 1 else gpu.g2_decode)(enc, False, True)
    assert st.tolist() == want_st.tolist()
    assert np.array_equal(pts, want_pts)


@pytest.mark.gpu
def test_gpu_subgroup_check_entry(gpu, oracle, decode_kernel, subgroup_case):
    """pa_g{1,2}_subgroup_check_batch (is_in_correct_subgroup_assuming_on_curve,
    ec.rs:142-144) on the unchecked decode's points == r * P == 0, infinity in;
    and decode(checked) == decode(unchecked) + this check (into_affine,
    ec.rs:1322-1332: the uncompressed points here are all on the curve)"""
    group, enc, truth = subgroup_case
    dec = gpu.g1_decode if group == 1 else gpu.g2_decode
    chk = gpu.g1_subgroup_check if group == 1 else gpu.g2_subgroup_check
    pts, st = dec(enc, False, False)
    assert (st == D.OK).all()
    ok = chk(pts)
    assert ok.tolist() == list(truth)
    want_pts, want_st = oracle.decode(group, enc, False, checked=True, nthreads=4)
    assert want_st.tolist() == [D.OK if t else D.NOT_IN_SUBGROUP for t in ok]
    assert np.array_equal(pts[ok], want_pts[ok])
    # infinity rows (from zero encodings) are in the subgroup
    zero = np.zeros_like(pts[:2])
    zero[:, -1] = 1
    assert chk(np.concatenate([zero, pts[:2]])).tolist() == [True, True] + list(truth[:2])


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_gpu_subgroup_check_device_large_batch(gpu, group):
    """the device entry over more points than the latency form takes (one lane
    per record): the generator's multiples in, each one's image under a point
    of small order (off the subgroup) out, in a seeded interleaving"""
    import torch
    import pairing_amd.device as pdev
    pts, truth = D.subgroup_points(group, seed=90 + group, n=2)
    base = np.array([D.aff_record(group, P) for P in pts], np.uint64)
    idx = np.random.default_rng(3).integers(0, len(pts), size=9001)
    rows = np.ascontiguousarray(base[idx])
    ok = torch.empty(len(rows), dtype=torch.uint8, device="cuda:0")
    pdev.subgroup_check(group, torch.from_numpy(rows.view(np.int64)).cuda(), ok)
    torch.cuda.synchronize()
    assert ok.cpu().numpy().astype(bool).tolist() == [bool(truth[k]) for k in idx]


@pytest.mark.gpu
@pytest.mark.parametrize("group", [1, 2])
def test_gpu_subgroup_check_compressed(gpu, oracle, decode_kernel, group):
    """the same points (in and outside the subgroup, small-order components
    included) compressed: square root, flag-selected root, then the subgroup
    check; each x with both sign flags"""
    pts, truth = D.subgroup_points(group, seed=50 + group, n=3)
    enc_f = D.enc_g1 if group == 1 else D.enc_g2
    recs = [enc_f(x, y, True, greatest) for greatest in (False, True) for x, y in pts]
    enc = np.frombuffer(b"".join(recs), np.uint8).reshape(-1, 48 if group == 1 else 96).copy()
    want_pts, want_st = oracle.decode(group, enc, True, checked=True, nthreads=4)
    assert want_st.tolist() == [D.OK if t else D.NOT_IN_SUBGROUP for t in list(truth) * 2]
    pts_g, st = (gpu.g1_decode if group == 1 else gpu.g2_decode)(enc, True, True)
    assert st.tolist() == want_st.tolist()
    assert np.array_equal(pts_g, want_pts)
