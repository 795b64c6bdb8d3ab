"""GPU parity: every HIP kernel behind the C ABI against the C oracle
(oracle/, the restatement of the reference) on identical seeded inputs.
The bar is bit-exact: all of this is integer arithmetic with canonical
(fully reduced) outputs."""
import numpy as np
import pytest

from helpers import (Q, R_ORDER, RMONT, fq12_one, hexlimbs, limbs, load_json, mont, random_fq, random_scalars,
                     relic_fq12, rng, set_infinity, small_scalars)

pytestmark = pytest.mark.gpu

NT = 8  # oracle threads for the larger reference computations


def _edge_fq():
    vals = [0, 1, 2, Q - 1, Q - 2, (Q - 1) // 2, RMONT, (1 << 380) - 1]
    return np.array([limbs(v % Q) for v in vals], dtype=np.uint64)


def _fq_inputs(seed, n):
    g = rng(seed)
    a = np.concatenate([_edge_fq(), random_fq(g, n)])
    b = np.concatenate([_edge_fq()[::-1], random_fq(g, n)])
    return a, b


def test_fq_mul_matches_oracle(gpu, oracle):
    a, b = _fq_inputs(1, 4096)
    np.testing.assert_array_equal(gpu.fq_mul(a, b), oracle.fq_mul(a, b))


def test_fq_mul_reference_kat(gpu):
    # test_fq_mul_assign, fq.rs:2558-2584 (raw Montgomery limbs)
    kat = [hexlimbs(v) for v in load_json("kat_limbs.json")["test_fq_mul_assign"]]
    a = np.array([kat[0]], np.uint64)
    b = np.array([kat[1]], np.uint64)
    np.testing.assert_array_equal(gpu.fq_mul(a, b)[0], np.array(kat[2], np.uint64))


def test_fq_square_add_sub_match_oracle(gpu, oracle):
    a, b = _fq_inputs(2, 2048)
    np.testing.assert_array_equal(gpu.fq_square(a), oracle.fq_square(a))
    np.testing.assert_array_equal(gpu.fq_add(a, b), oracle.fq_add(a, b))
    np.testing.assert_array_equal(gpu.fq_sub(a, b), oracle.fq_sub(a, b))


def test_fq_inverse_matches_oracle(gpu, oracle):
    a, _ = _fq_inputs(3, 256)
    got, ok = gpu.fq_inverse(a)
    exp, eok = oracle.fq_inverse(a)
    np.testing.assert_array_equal(ok, eok.astype(bool))
    assert not ok[0]  # inverse of zero is None (fq.rs:850-851)
    np.testing.assert_array_equal(got[ok], exp[ok])


def _rand_tower(seed, n, width):
    g = rng(seed)
    return random_fq(g, n * width // 6).reshape(n, width)


def test_fq2_ops_match_oracle(gpu, oracle):
    a = _rand_tower(4, 1024, 12)
    b = _rand_tower(5, 1024, 12)
    np.testing.assert_array_equal(gpu.fq2_mul(a, b), oracle.fq2_mul(a, b))
    np.testing.assert_array_equal(gpu.fq2_square(a), oracle.fq2_square(a))


def test_fq6_fq12_mul_square_match_oracle(gpu, oracle):
    a6, b6 = _rand_tower(6, 256, 36), _rand_tower(7, 256, 36)
    np.testing.assert_array_equal(gpu.fq6_mul(a6, b6), oracle.fq6_mul(a6, b6))
    a, b = _rand_tower(8, 256, 72), _rand_tower(9, 256, 72)
    np.testing.assert_array_equal(gpu.fq12_mul(a, b), oracle.fq12_mul(a, b))
    np.testing.assert_array_equal(gpu.fq12_square(a), oracle.fq12_square(a))


def test_fq12_inverse_frobenius_match_oracle(gpu, oracle):
    a = _rand_tower(10, 64, 72)
    a[3] = 0  # zero has no inverse
    got, ok = gpu.fq12_inverse(a)
    exp, eok = oracle.fq12_inverse(a)
    np.testing.assert_array_equal(ok, eok.astype(bool))
    assert not ok[3]
    np.testing.assert_array_equal(got[ok], exp[ok])
    for power in range(12):
        np.testing.assert_array_equal(gpu.fq12_frobenius_map(a, power), oracle.fq12_frobenius(a, power))


def test_fq12_mul_by_014_matches_oracle(gpu, oracle):
    a = _rand_tower(11, 256, 72)
    c0, c1, c4 = (_rand_tower(s, 256, 12) for s in (12, 13, 14))
    np.testing.assert_array_equal(gpu.fq12_mul_by_014(a, c0, c1, c4), oracle.fq12_mul_by_014(a, c0, c1, c4))


def _cyclotomic(oracle, f):
    """f^((q^6-1)(q^2+1)): the easy part of mod.rs:105-114."""
    inv, ok = oracle.fq12_inverse(f)
    conj = f.copy()
    conj[:, 36:] = oracle.fq_sub(np.zeros((f.shape[0] * 6, 6), np.uint64),
                                 f[:, 36:].reshape(-1, 6)).reshape(-1, 36)
    r = oracle.fq12_mul(conj, inv)
    return oracle.fq12_mul(oracle.fq12_frobenius(r, 2), r)


def test_cyclotomic_square_equals_square_in_subgroup(gpu, oracle):
    f = _cyclotomic(oracle, _rand_tower(15, 128, 72))
    np.testing.assert_array_equal(gpu.fq12_cyclotomic_square(f), oracle.fq12_square(f))


def _points(seed, n, inf_every=0):
    g = rng(seed)
    s1 = random_scalars(g, n)
    s2 = random_scalars(g, n)
    return s1, s2


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["default", "gen2", "coop", "gen", "coop1"])
def lanes(request, gpu):
    gpu.set_pairing_kernel(request.param)
    yield request.param
    gpu.set_pairing_kernel(0)


@pytest.fixture(scope="module")
def pairs(oracle):
    s1, s2 = _points(21, 96)
    p = oracle.g1_mul_generator(s1, NT)
    q = oracle.g2_mul_generator(s2, NT)
    # sprinkle infinity on either side (mod.rs:50-54)
    set_infinity(p, [5, 40])
    set_infinity(q, [17, 40, 77])
    return p, q


def test_g2_prepare_matches_oracle_bit_exact(gpu, oracle, pairs):
    _, q = pairs
    np.testing.assert_array_equal(gpu.g2_prepare(q), oracle.g2_prepare(q, NT))


def test_miller_loop_batch_matches_oracle(gpu, oracle, pairs):
    p, q = pairs
    prep = oracle.g2_prepare(q, NT)
    np.testing.assert_array_equal(gpu.miller_loop_batch(p, prep), oracle.miller_loop_batch(p, prep, NT))


def test_multi_miller_loop_is_product(gpu, oracle, pairs):
    p, q = pairs
    prep = oracle.g2_prepare(q[:9], NT)
    exp = oracle.miller_loop(p[:9], prep)
    np.testing.assert_array_equal(gpu.multi_miller_loop(p[:9], prep), exp)
    # empty product is one
    np.testing.assert_array_equal(gpu.multi_miller_loop(p[:0], prep[:0]), fq12_one()[0])


def test_multi_miller_loop_affine_is_product(gpu, oracle, pairs, lanes):
    """prepare fused on device, then the product tree (mod.rs:40-102)"""
    p, q = pairs
    exp = oracle.miller_loop(p[:41], oracle.g2_prepare(q[:41], NT))   # includes infinity pairs 5, 17, 40
    np.testing.assert_array_equal(gpu.multi_miller_loop_affine(p[:41], q[:41]), exp)
    np.testing.assert_array_equal(gpu.multi_miller_loop_affine(p[:0], q[:0]), fq12_one()[0])


def _neg_g1(aff):
    out = aff.copy()
    for k in range(out.shape[0]):
        y = sum(int(w) << (64 * i) for i, w in enumerate(out[k, 6:12])) * pow(RMONT, -1, Q) % Q
        out[k, 6:12] = limbs((Q - y) % Q * RMONT % Q)
    return out


def test_multi_pairing_batch_verification(gpu, oracle):
    """e(aP, Q) * e(-P, aQ) == 1 (the verifier shape, engine.rs:50-92 product
    semantics) and multi_pairing == final_exponentiation(product)"""
    g = rng(35)
    a = random_scalars(g, 4)
    s = random_scalars(g, 4)
    t = random_scalars(g, 4)
    for k in range(4):
        sp = oracle.g1_mul_generator(s[k:k + 1])
        tq = oracle.g2_mul_generator(t[k:k + 1])
        sa = limbs(sum(int(w) << (64 * i) for i, w in enumerate(s[k])) *
                   sum(int(w) << (64 * i) for i, w in enumerate(a[k])) % R_ORDER, 4)
        ta = limbs(sum(int(w) << (64 * i) for i, w in enumerate(t[k])) *
                   sum(int(w) << (64 * i) for i, w in enumerate(a[k])) % R_ORDER, 4)
        p = np.concatenate([oracle.g1_mul_generator(np.array([sa], np.uint64)), _neg_g1(sp)])
        q = np.concatenate([tq, oracle.g2_mul_generator(np.array([ta], np.uint64))])
        out, ok = gpu.multi_pairing(p, q)
        assert ok
        np.testing.assert_array_equal(out, fq12_one()[0])
    p = oracle.g1_mul_generator(s)
    q = oracle.g2_mul_generator(t)
    exp, eok = oracle.final_exponentiation(oracle.miller_loop(p, oracle.g2_prepare(q))[None, :].copy())
    out, ok = gpu.multi_pairing(p, q)
    assert ok and eok[0]
    np.testing.assert_array_equal(out, exp[0])


def test_pairing_multi_gpu_entry(gpu, oracle, pairs):
    p, q = pairs
    np.testing.assert_array_equal(gpu.pairing_multi_gpu(p, q, 1), gpu.pairing(p, q))
    with pytest.raises(gpu.PairingError):
        gpu.pairing_multi_gpu(p, q, gpu.device_count() + 1)


@pytest.mark.gpu
def test_pairing_multi_gpu_workers_over_a_device_map(gpu, oracle, pairs, monkeypatch):
    """ndev = 2 and 3 worker threads (ragged contiguous shards) mapped onto
    device 0 by PA_DEVICE_MAP: the multi-device sharding and join logic on a
    one-GPU box, bit-exact vs the single call"""
    p, q = pairs
    want = gpu.pairing(p, q)
    for m, ndev in (("0,0", 2), ("0,0,0", 3)):
        monkeypatch.setenv("PA_DEVICE_MAP", m)
        np.testing.assert_array_equal(gpu.pairing_multi_gpu(p[:-1], q[:-1], ndev), want[:-1])
    monkeypatch.setenv("PA_DEVICE_MAP", "0,0")
    with pytest.raises(gpu.PairingError):
        gpu.pairing_multi_gpu(p, q, 3)
    monkeypatch.setenv("PA_DEVICE_MAP", "0,x")
    with pytest.raises(gpu.PairingError):
        gpu.pairing_multi_gpu(p, q, 1)


def test_final_exponentiation_matches_oracle(gpu, oracle, pairs, lanes):
    p, q = pairs
    f = oracle.miller_loop_batch(p[:32], oracle.g2_prepare(q[:32], NT), NT)
    f[7] = 0  # final_exponentiation(0) is None (mod.rs:108, 157-158)
    got, ok = gpu.final_exponentiation(f)
    exp, eok = oracle.final_exponentiation(f, NT)
    np.testing.assert_array_equal(ok, eok.astype(bool))
    assert not ok[7] and ok.sum() == 31
    np.testing.assert_array_equal(got[ok], exp[ok])


def test_pairing_matches_oracle(gpu, oracle, pairs, lanes):
    p, q = pairs
    np.testing.assert_array_equal(gpu.pairing(p, q), oracle.pairing(p, q, NT))


def test_pairing_relic_kat(gpu, oracle, lanes):
    one = small_scalars([1])
    p = oracle.g1_mul_generator(one)
    q = oracle.g2_mul_generator(one)
    np.testing.assert_array_equal(gpu.pairing(p, q), relic_fq12())


def test_pairing_bilinearity(gpu, oracle, lanes):
    # e(aP, bQ) == e(abP, Q) == e(P, abQ) (engine.rs:93-126), all on the GPU
    g = rng(33)
    a = random_scalars(g, 16)
    b = random_scalars(g, 16)
    ab = np.array([limbs(
        (int(sum(int(x) << (64 * i) for i, x in enumerate(a[k])))
         * int(sum(int(x) << (64 * i) for i, x in enumerate(b[k])))) % R_ORDER, 4) for k in range(16)],
        np.uint64)
    one = np.tile(small_scalars([1]), (16, 1))
    e1 = gpu.pairing(oracle.g1_mul_generator(a, NT), oracle.g2_mul_generator(b, NT))
    e2 = gpu.pairing(oracle.g1_mul_generator(ab, NT), oracle.g2_mul_generator(one, NT))
    e3 = gpu.pairing(oracle.g1_mul_generator(one, NT), oracle.g2_mul_generator(ab, NT))
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_array_equal(e1, e3)


# ---------------- config 3: G1 batch_normalization + fixed-base (wNAF path) ----------------

def _jacobian_points(oracle, seed, n):
    g = rng(seed)
    v = oracle.g1_mul_generator_jacobian(random_scalars(g, n), NT)
    # zeros keep garbage x, y with z = 0 (ec.rs:398, 477); normalized points have z = 1
    zero_idx = [1, n // 3, n - 1]
    v[zero_idx, 12:18] = 0
    norm_idx = [2, n // 2]
    v[norm_idx] = oracle.g1_from_affine(oracle.g1_into_affine(v[norm_idx]))
    return v


@pytest.mark.parametrize("n", [1, 7, 8, 1000, 4099])
def test_g1_batch_normalization_bit_exact(gpu, oracle, n):
    v = _jacobian_points(oracle, 40 + n, max(n, 8))[:n]
    np.testing.assert_array_equal(gpu.g1_batch_normalization(v), oracle.g1_batch_normalization(v))


def test_g1_fixed_base_equals_reference_wnaf(gpu, oracle):
    g = rng(50)
    base = oracle.g1_mul_generator_jacobian(random_scalars(g, 1))  # non-normalized base
    s = random_scalars(g, 512)
    s[0] = 0
    s[1] = limbs(1, 4)
    s[2] = limbs(R_ORDER - 1, 4)
    s[3] = limbs((1 << 255) - 1, 4)   # > r: any 256-bit FrRepr is accepted
    s[4] = limbs(128 + 256 * 128, 4)  # digit edge cases of the signed recoding
    got = gpu.g1_wnaf_fixed_base(base, s)
    exp = oracle.g1_wnaf_fixed_base(base, s, NT)
    assert oracle.g1_eq(got, exp).all()  # PartialEq (ec.rs:45-85)
    np.testing.assert_array_equal(gpu.g1_batch_normalization(got), oracle.g1_batch_normalization(exp))


def test_g1_config3_full_size_properties(gpu, oracle):
    """2^18 scalars (BASELINE config 3): sampled equality with the oracle and
    linearity out[i] + out[j] == (s_i + s_j) * g on sampled pairs."""
    n = 1 << 18
    g = rng(51)
    base = oracle.g1_mul_generator_jacobian(random_scalars(g, 1))
    s = np.ascontiguousarray(random_scalars(g, 4096)[np.arange(n) % 4096])
    s[:, 0] ^= np.arange(n, dtype=np.uint64)  # distinct scalars, still < 2^256
    got = gpu.g1_batch_normalization(gpu.g1_wnaf_fixed_base(base, s))
    idx = rng(52).choice(n, 256, replace=False)
    exp = oracle.g1_batch_normalization(oracle.g1_wnaf_fixed_base(base, np.ascontiguousarray(s[idx]), NT))
    np.testing.assert_array_equal(got[idx], exp)
    i, j = idx[:64], idx[64:128]
    ssum = np.array([limbs((sum(int(x) << (64 * k) for k, x in enumerate(s[a])) +
                            sum(int(x) << (64 * k) for k, x in enumerate(s[b]))) % R_ORDER, 4)
                     for a, b in zip(i, j)], np.uint64)
    lhs = oracle.g1_add(np.ascontiguousarray(got[i]), np.ascontiguousarray(got[j]))
    rhs = oracle.g1_wnaf_fixed_base(base, ssum, NT)
    assert oracle.g1_eq(lhs, rhs).all()


@pytest.mark.parametrize("zero_base", [False, True])
def test_g1_fixed_base_overlapped_halves(gpu, oracle, zero_base):
    """pa_g1_wnaf_fixed_base runs the table build overlapped with the multiply
    (side stream, window halves [0, 17) and [17, 33)): equal as points to the
    reference's wNAF for scalars whose nonzero digits sit in one half only,
    digit/carry edges at the split, and the zero base (ec.rs:299-301)."""
    g = rng(53)
    base = oracle.g1_mul_generator_jacobian(random_scalars(g, 1))
    if zero_base:
        base[0, 12:18] = 0
    s = random_scalars(g, 3000)
    s[0] = 0
    s[1] = limbs(1, 4)
    s[2] = limbs(R_ORDER - 1, 4)
    s[3] = limbs((1 << 255) - 1, 4)
    s[8] = limbs((1 << 256) - 1, 4)    # wnaf_form's add_nocarry wraps (wnaf.rs:30-35): -base
    s[4] = limbs(1 << 200, 4)          # only the high half
    s[5] = limbs((1 << 130) - 1, 4)    # low half + carry into window 17
    s[6] = limbs(0x80 << 128, 4)       # digit 128 at window 16, no carry
    s[7] = limbs(0x81 << 128, 4)       # digit -127 at window 16, carry into window 17
    got = gpu.g1_wnaf_fixed_base(base, s)
    k = 256
    exp = oracle.g1_wnaf_fixed_base(base, np.ascontiguousarray(s[:k]), NT)
    assert oracle.g1_eq(got[:k], exp).all()
    if not zero_base:  # a zero base gives zeros whose (x, y) bits are whatever the add chain copied (ec.rs:398)
        np.testing.assert_array_equal(gpu.g1_batch_normalization(got[:k]), oracle.g1_batch_normalization(exp))


_X2 = 0xd201000000010000 ** 2  # x^2, the GLV split's divisor (kernels_curve.hip glv_split)


def _glv_edge_scalars():
    vals = [0, 1, _X2 - 1, _X2, _X2 + 1, 2 * _X2 - 1, 2 * _X2, (1 << 128) - 1, 1 << 128,
            (_X2 << 1) + (1 << 127), R_ORDER - 1, R_ORDER, (1 << 255) - 1, (1 << 256) - (1 << 200),
            (1 << 128) * _X2, ((1 << 256) - (1 << 200)) // _X2 * _X2, 0x80 * _X2 + 0x80, 0x81 * _X2 + 0x81, (0x80 << 120) * _X2 + (0x81 << 120)]
    return np.array([limbs(v, 4) for v in vals], np.uint64)


@pytest.mark.parametrize("which", ["subgroup", "outside"])
def test_g1_fixed_base_glv_and_fallback(gpu, oracle, which):
    """pa_g1_wnaf_fixed_base takes the GLV split s = q x^2 + rem when the base
    passes phi(P) == -[x^2] P and the plain 33-window comb otherwise (the
    kernels of both are launched; the flag picks one).  Bases: on-curve points
    in and outside G1 (cofactor components of order 3 and others, tests/
    decode_cases.py), non-normalized (random z); scalars at the split's and the
    signed digits' edges plus random ones.  Equal as points to the oracle's wNAF."""
    import decode_cases as D
    pts, truth = D.subgroup_points(1, seed=60, n=2)
    sel = [P for P, t in zip(pts, truth) if t == (which == "subgroup")]
    assert sel
    g = rng(61)
    s = np.concatenate([_glv_edge_scalars(), random_scalars(g, 200, bits=256)])
    for k, (x, y) in enumerate(sel[:3]):
        z = (k + 2) * 0x1234567 % Q
        base = np.array([mont(x * z * z) + mont(y * z * z * z) + mont(z)], np.uint64)
        got = gpu.g1_wnaf_fixed_base(base, s)
        exp = oracle.g1_wnaf_fixed_base(base, s, NT)
        assert oracle.g1_eq(got, exp).all(), (which, k)
