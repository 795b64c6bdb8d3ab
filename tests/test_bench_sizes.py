"""Parity of the exact kernels bench.py times, at the sizes it times them.

bench.py measures the `_device` entry points (HBM-resident tensors through
pairing_amd.device): config 2 is `pa_fq_mul_batch_device` at 2^20 elements
(k_fq_mul_batch: grid-stride loop with register prefetch and a 4096-block
grid cap), the Fr leg `pa_fr_mul_batch_device` at 2^20, config 4
`pa_pairing_batch_device` at 2^16 pairs on bench.make_pairs' inputs.  Each is
compared here bit for bit with the oracle (fq.rs:909-960, fr.rs:438-465,
mod.rs:40-160), at the benched size and at a ragged size that leaves a
partial tail for the grid-stride loop.  A last test runs two pairing batches
on two streams at the same time (each launch must get its own spill
workspace, gen_launch.hip)."""
import os

import numpy as np
import pytest

from helpers import Q, R_ORDER, limbs, random_scalars, rng

pytestmark = pytest.mark.gpu

FQ_TOP = Q >> 320            # top limb of q
FR_TOP = R_ORDER >> 192


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16")), 16))


def _field_rows(seed, n, words, top, edges):
    """n values < modulus (top limb drawn below the modulus' top limb), the
    edge values first."""
    g = rng(seed)
    a = g.integers(0, 1 << 64, size=(n, words), dtype=np.uint64)
    a[:, words - 1] = g.integers(0, top, size=n, dtype=np.uint64)
    e = np.array([limbs(v, words) for v in edges], np.uint64)
    a[:len(e)] = e
    return a


def _fq_rows(seed, n):
    return _field_rows(seed, n, 6, FQ_TOP, [0, 1, 2, Q - 1, Q - 2, (Q - 1) // 2, (1 << 380) - 1])


def _fr_rows(seed, n):
    return _field_rows(seed, n, 4, FR_TOP, [0, 1, 2, R_ORDER - 1, R_ORDER - 2, (R_ORDER - 1) // 2])


def _dev(a):
    import torch
    return torch.from_numpy(a.view(np.int64)).to("cuda:0")


def _host(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("n", [1 << 20, (1 << 20) + 37, 4096 * 256 * 2 + 5])
def test_fq_mul_device_bit_exact_at_bench_size(gpu, oracle, n):
    """config 2: the benched kernel, every element against Fq::mul_assign"""
    import torch
    import pairing_amd.device as pdev
    a, b = _fq_rows(100 + n % 97, n), _fq_rows(200 + n % 89, n)[::-1].copy()
    out = pdev.empty_records(n, 6, "cuda:0")
    pdev.fq_mul(_dev(a), _dev(b), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.fq_mul(a, b))


@pytest.mark.parametrize("n", [1 << 20, (1 << 20) + 37])
def test_fr_mul_device_bit_exact_at_bench_size(gpu, oracle, n):
    import torch
    import pairing_amd.device as pdev
    a, b = _fr_rows(300 + n % 97, n), _fr_rows(400 + n % 89, n)[::-1].copy()
    out = pdev.empty_records(n, 4, "cuda:0")
    pdev.fr_mul(_dev(a), _dev(b), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.fr_mul(a, b))


@pytest.mark.parametrize("variant", [0, 3], ids=["default_lane_pairs", "one_lane"])
def test_pairing_device_bit_exact_at_bench_size(gpu, oracle, variant):
    """config 4: 2^16 pairings on the bench's own inputs, every pairing against
    the oracle -- on the default selection (round 5: lane pairs, 2048 waves,
    two per SIMD) and on the one-lane kernels (1024 waves), every wave with its
    own spill workspace"""
    import torch
    import bench
    import pairing_amd.device as pdev
    n = 1 << 16
    p_np, q_np = bench.make_pairs(n, 0)
    out = pdev.empty_records(n, 72, "cuda:0")
    scratch = pdev.empty_records(n, 72, "cuda:0")
    gpu.set_pairing_kernel(variant)
    try:
        pdev.pairing(_dev(p_np), _dev(q_np), out, scratch)
        torch.cuda.synchronize()
    finally:
        gpu.set_pairing_kernel(0)
    got = _host(out)
    exp = oracle.pairing(p_np, q_np, _threads())
    np.testing.assert_array_equal(got, exp)
    # infinity pairs (1/128 of P) give one
    inf = np.nonzero(p_np[:, 12] != 0)[0]
    assert len(inf) == n // 128
    one = np.zeros(72, np.uint64)
    one[:6] = limbs(pow(2, 384, Q))
    assert (got[inf] == one).all()


@pytest.mark.parametrize("n", [2305, 32768, 32769, 33600, 33601, 34816, 34817])
def test_pairing_default_mid_size_batches(gpu, oracle, n):
    """The default selection's regime boundaries (PA_PQ_MAX < n <= PA_PAIR_MAX:
    lane pairs at one wave per SIMD; PA_PAIR_MAX < n <= PA_PAIR_MAX + PA_TAIL_MAX
    (34816): the first PA_PAIR_MAX on lane pairs and the tail on a forked stream,
    on the cooperative kernels up to 832 tail pairs (33600) and the lane groups
    above; above: lane pairs at two waves per SIMD) on both sides, every pairing
    against the oracle"""
    import torch
    import bench
    import pairing_amd.device as pdev
    p_np, q_np = bench.make_pairs(n, 0, seed=29)
    out = pdev.empty_records(n, 72, "cuda:0")
    scratch = pdev.empty_records(n, 72, "cuda:0")
    pdev.pairing(_dev(p_np), _dev(q_np), out, scratch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.pairing(p_np, q_np, _threads()))


@pytest.mark.parametrize("tail", [300, 1500], ids=["coop_tail", "lane_group_tail"])
def test_split_batch_stages_with_zeros_and_infinity(gpu, oracle, tail):
    """A batch just above PA_PAIR_MAX through the two stages apart: the Miller
    loop stage (lane pairs for the head; on the forked stream the cooperative
    kernel for a tail of up to 1024, the lane groups above) then the final exponentiation (split the same way) ==
    the oracle's pairing, with infinity Q on both sides of the split; and the
    final exponentiation alone over such a batch with zero Miller values in the
    head and in the tail: ok = 0 / zero output exactly there, in place too"""
    import torch
    import bench
    import pairing_amd.device as pdev
    n = 32768 + tail
    p_np, q_np = bench.make_pairs(n, 0, seed=31)
    for k in (7, 32768 + 3, n - 1):
        q_np[k, :24] = 0
        q_np[k, 12:18] = limbs(pow(2, 384, Q))
        q_np[k, 24] = 1
    f = pdev.empty_records(n, 72, "cuda:0")
    out = pdev.empty_records(n, 72, "cuda:0")
    pdev.pairing_miller_loop(_dev(p_np), _dev(q_np), f)
    pdev.final_exponentiation(f, out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.pairing(p_np, q_np, _threads()))
    fv = _host(f)
    zeros = [11, 32768, 32768 + tail - 1]
    fv[zeros] = 0
    exp, ok_exp = oracle.final_exponentiation(fv, _threads())
    d = _dev(fv)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    pdev.final_exponentiation(d, d, ok)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d), exp)
    okh = ok.cpu().numpy()
    np.testing.assert_array_equal(okh, np.asarray(ok_exp, np.uint8))
    assert (okh[zeros] == 0).all() and okh.sum() == n - len(zeros)


def test_pairing_two_streams_concurrently(gpu, oracle):
    """Two pairing batches enqueued on two streams before either finishes:
    both bit-exact (each launch draws its own spill workspace)"""
    import torch
    import bench
    import pairing_amd.device as pdev
    n = 4096
    p0, q0 = bench.make_pairs(n, 0, seed=11)
    p1, q1 = bench.make_pairs(n, 1, seed=57)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for (p, q), s in (((p0, q0), s0), ((p1, q1), s1)):
        with torch.cuda.stream(s):
            dp, dq = _dev(p), _dev(q)
            out = pdev.empty_records(n, 72, "cuda:0")
            scratch = pdev.empty_records(n, 72, "cuda:0")
        s.synchronize()
        outs.append((dp, dq, out, scratch, s))
    for dp, dq, out, scratch, s in outs:       # both enqueued back to back
        pdev.pairing(dp, dq, out, scratch, s)
    torch.cuda.synchronize()
    t = _threads()
    np.testing.assert_array_equal(_host(outs[0][2]), oracle.pairing(p0, q0, t))
    np.testing.assert_array_equal(_host(outs[1][2]), oracle.pairing(p1, q1, t))


def test_pairing_host_pipeline_chunks_and_threads(gpu, oracle, monkeypatch):
    """pa_pairing_batch on host buffers: a multi-chunk pipelined call
    (PA_PIPELINE_CHUNK shrinks the chunk so the pipeline's double buffers
    turn over, ragged last chunk) and two host threads calling at once (each
    on its own per-thread stream and scratch), all bit-exact"""
    import threading
    import bench
    p, q = bench.make_pairs(3000, 0, seed=3)
    monkeypatch.setenv("PA_PIPELINE_CHUNK", "700")
    got = gpu.pairing(p, q)
    monkeypatch.delenv("PA_PIPELINE_CHUNK")
    t = _threads()
    exp = oracle.pairing(p, q, t)
    np.testing.assert_array_equal(got, exp)
    res = [None, None]

    def run(k):
        for _ in range(3):
            res[k] = gpu.pairing(p[k * 1500:(k + 1) * 1500], q[k * 1500:(k + 1) * 1500])

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    np.testing.assert_array_equal(np.concatenate(res), exp)


def test_pairing_host_pipeline_pieces_with_empty_last_piece(oracle):
    """the pipelined host path cut into pieces (PA_PIPELINE_PIECES=4, read once
    per process, hence a child process) with chunks of 5 pairs: the last piece
    of every chunk is empty (per = 2: 2 + 2 + 1 + 0), so the kernels' wait for
    the D2H of chunk ci-2 must not hang on that piece's event (ADVICE r02,
    capi.hip: one 'chunk copied out' event after the piece loop)"""
    import subprocess
    import sys
    code = ("import numpy as np, sys; sys.path[:0] = [%r, %r]; import bench, pairing_amd; "
            "p, q = bench.make_pairs(23, 0, seed=9); np.save(sys.argv[1], pairing_amd.pairing(p, q))"
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
               os.path.dirname(os.path.abspath(__file__))))
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.npy")
        env = dict(os.environ, PA_PIPELINE_CHUNK="5", PA_PIPELINE_PIECES="4")
        r = subprocess.run([sys.executable, "-c", code, path], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        got = np.load(path)
    import bench
    p, q = bench.make_pairs(23, 0, seed=9)
    np.testing.assert_array_equal(got, oracle.pairing(p, q, _threads()))


@pytest.mark.parametrize("n", [1 << 16, 333])
def test_prepared_path_device_bit_exact_at_bench_size(gpu, oracle, n):
    """bench.py --workload prepared: pa_g2_prepare_batch_device writes the
    reference's G2Prepared records (68 line coefficients, mod.rs:168-358) and
    pa_miller_loop_batch_device + the final exponentiation over them give
    e(P, Q) (mod.rs:40-160), bit for bit; some Q at infinity (empty coeffs +
    flag, mod.rs:169-174) besides bench.make_pairs' infinite P"""
    import torch
    import bench
    import pairing_amd.device as pdev
    from pairing_amd._native import W_G2P
    p_np, q_np = bench.make_pairs(n, 0, seed=11)
    qinf = np.arange(n)[np.arange(n) % 97 == 3]
    q_np[qinf, :24] = 0
    q_np[qinf, 12:18] = limbs(pow(2, 384, Q))
    q_np[qinf, 24] = 1
    dq = _dev(q_np)
    prep = pdev.empty_records(n, W_G2P, "cuda:0")
    pdev.g2_prepare(dq, prep)
    f = pdev.empty_records(n, 72, "cuda:0")
    out = pdev.empty_records(n, 72, "cuda:0")
    pdev.miller_loop_prepared(_dev(p_np), prep, f)
    pdev.final_exponentiation(f, out)
    torch.cuda.synchronize()
    exp_prep = oracle.g2_prepare(q_np, _threads())
    np.testing.assert_array_equal(_host(prep), exp_prep)
    np.testing.assert_array_equal(_host(f), oracle.miller_loop_batch(p_np, exp_prep, _threads()))
    np.testing.assert_array_equal(_host(out), oracle.pairing(p_np, q_np, _threads()))


@pytest.mark.parametrize("n", [0, 1, 2, 5, 16, 17, 300, 3001])
def test_multi_pairing_device_matches_oracle(gpu, oracle, n):
    """bench.py --workload verify: pa_multi_pairing_device (cooperative Miller
    loops; up to 16 pairs the Miller values' product inside the cooperative
    final exponentiation, more first in levels of 16-value cooperative
    products) == the oracle's
    final_exponentiation(miller_loop(pairs)); the empty product is one"""
    import torch
    import bench
    import pairing_amd.device as pdev
    from helpers import fq12_one
    p_np, q_np = bench.make_pairs(max(n, 1), 0, seed=3)
    p_np, q_np = p_np[:n], q_np[:n]
    out = pdev.empty_records(1, 72, "cuda:0")
    ok = torch.zeros(1, dtype=torch.uint8, device="cuda:0")
    work = pdev.empty_records(max(n, 1), 72, "cuda:0")
    dp = _dev(np.ascontiguousarray(p_np)) if n else torch.zeros((0, 13), dtype=torch.int64, device="cuda:0")
    dq = _dev(np.ascontiguousarray(q_np)) if n else torch.zeros((0, 25), dtype=torch.int64, device="cuda:0")
    pdev.multi_pairing(dp, dq, out, ok, work)
    torch.cuda.synchronize()
    if n == 0:
        exp = fq12_one()[0]
    else:
        f = oracle.miller_loop(np.ascontiguousarray(p_np), oracle.g2_prepare(np.ascontiguousarray(q_np)))
        exp, eok = oracle.final_exponentiation(f[None, :].copy())
        exp = exp[0]
    assert int(ok.item()) == 1
    np.testing.assert_array_equal(_host(out)[0], exp)


@pytest.mark.parametrize("n", [4099, 1 << 16])
def test_pairing_miller_loop_stage_then_final_exp(gpu, oracle, n):
    """bench.py's timed pairing step: pa_pairing_miller_loop_batch_device (the
    pairing-only lane-pair Miller loop: homogeneous G2 steps, its own line
    scaling) then pa_final_exponentiation_batch_device == the oracle's pairing,
    bit for bit, with infinity P and Q mixed in; its Miller values differ from
    the reference's (by Fq2 factors) where neither point is at infinity"""
    import torch
    import bench
    import pairing_amd.device as pdev
    p_np, q_np = bench.make_pairs(n, 0, seed=29)
    q_np[5::301, :24] = 0
    q_np[5::301, 12:18] = limbs(pow(2, 384, Q))
    q_np[5::301, 24] = 1
    dp, dq = _dev(p_np), _dev(q_np)
    f = pdev.empty_records(n, 72, "cuda:0")
    out = pdev.empty_records(n, 72, "cuda:0")
    pdev.pairing_miller_loop(dp, dq, f)
    pdev.final_exponentiation(f, out)
    torch.cuda.synchronize()
    want = np.concatenate([oracle.pairing(p_np[k:k + 8192], q_np[k:k + 8192], _threads())
                           for k in range(0, n, 8192)])
    np.testing.assert_array_equal(_host(out), want)
    ref = pdev.empty_records(64, 72, "cuda:0")
    pdev.miller_loop(dp[:64], dq[:64], ref)
    torch.cuda.synchronize()
    fin = (p_np[:64, 12] & 0xff) | (q_np[:64, 24] & 0xff)
    differ = (_host(f)[:64] != _host(ref)).any(axis=1)
    assert differ[fin == 0].all() and not differ[fin != 0].any()


@pytest.mark.parametrize("which", ["subgroup", "outside"])
def test_g1_glv_stages_device_match_oracle(gpu, oracle, which):
    """config 3's GLV stages as bench.py times them for the roofline
    (pa_g1_fixed_base_glv_table_device, then pa_g1_fixed_base_glv_mul_device
    with its plain-comb fallback) and the fused pa_g1_wnaf_fixed_base_device,
    for a base in G1 and one outside it: equal as points to the reference's
    wNAF (wnaf.rs:93-178), then bit-exact after batch_normalization."""
    import torch
    import decode_cases as D
    import pairing_amd.device as pdev
    from helpers import mont
    pts, truth = D.subgroup_points(1, seed=70, n=1)
    x, y = next(P for P, t in zip(pts, truth) if t == (which == "subgroup"))
    z = 0x5eed % Q
    base_np = np.array([mont(x * z * z) + mont(y * z * z * z) + mont(z)], np.uint64)
    n = 4096 + 17
    g = rng(71)
    s = np.zeros((n, 4), np.uint64)
    for k in range(n):
        s[k] = limbs(int(g.integers(0, 1 << 62)) << 190 | int(g.integers(0, 1 << 62)) << 128
                     | int(g.integers(0, 1 << 62)) << 64 | int(g.integers(0, 1 << 62)), 4)
    base, scal = _dev(base_np), _dev(s)
    table, ws = pdev.fixed_base_buffers("cuda:0")
    out1 = pdev.empty_records(n, 18, "cuda:0")
    out2 = pdev.empty_records(n, 18, "cuda:0")
    pdev.g1_fixed_base_glv_table(base, table, ws)
    pdev.g1_fixed_base_glv_mul(base, table, ws, scal, out1)
    pdev.g1_wnaf_fixed_base(base, scal, out2, table, ws)
    torch.cuda.synchronize()
    got1, got2 = _host(out1), _host(out2)
    idx = np.concatenate([np.arange(64), np.arange(n - 64, n)])
    exp = oracle.g1_wnaf_fixed_base(base_np, np.ascontiguousarray(s[idx]), 8)
    assert oracle.g1_eq(np.ascontiguousarray(got1[idx]), exp).all()
    assert oracle.g1_eq(np.ascontiguousarray(got2[idx]), exp).all()
    np.testing.assert_array_equal(oracle.g1_batch_normalization(got1), oracle.g1_batch_normalization(got2))


def test_final_exp_apart_and_in_place_agree(gpu, oracle):
    """pa_final_exponentiation_batch_device with out apart from in and with
    out == in (both run the one generated kernel, pa_gen_final_exp, at this
    size on variant 3): both equal the oracle, including f == 0 (reference
    None: zero, ok = 0), and `in` is left unchanged when apart."""
    import torch
    import pairing_amd.device as pdev
    n = 2300
    gpu.set_pairing_kernel(3)   # the one-lane generated kernels
    try:
        f = _field_rows(41, n * 12, 6, FQ_TOP, [1]).reshape(n, 72)
        f[7] = 0
        exp, ok_exp = oracle.final_exponentiation(f, _threads())
        d_in = _dev(f)
        out = pdev.empty_records(n, 72, "cuda:0")
        ok = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        pdev.final_exponentiation(d_in, out, ok)
        d_same = _dev(f)
        ok2 = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        pdev.final_exponentiation(d_same, d_same, ok2)
        torch.cuda.synchronize()
    finally:
        gpu.set_pairing_kernel(0)
    np.testing.assert_array_equal(_host(out), exp)
    np.testing.assert_array_equal(_host(d_in), f)
    np.testing.assert_array_equal(_host(d_same), exp)
    np.testing.assert_array_equal(ok.cpu().numpy(), np.asarray(ok_exp, np.uint8))
    np.testing.assert_array_equal(ok2.cpu().numpy(), np.asarray(ok_exp, np.uint8))
    assert ok.cpu().numpy()[7] == 0


@pytest.mark.parametrize("n", [1 << 20, (1 << 20) + 37])
def test_fq_mul_soa_device_bit_exact(gpu, oracle, n):
    """config 2 on the SoA device layout: every element
    against the oracle, words transposed on the host"""
    import torch
    import pairing_amd.device as pdev
    a = _fq_rows(7, n)
    b = _fq_rows(8, n)[::-1].copy()
    da = torch.from_numpy(np.ascontiguousarray(a.T).view(np.int64)).to("cuda:0")
    db = torch.from_numpy(np.ascontiguousarray(b.T).view(np.int64)).to("cuda:0")
    out = torch.empty((6, n), dtype=torch.int64, device="cuda:0")
    pdev.fq_mul_soa(da, db, out)
    torch.cuda.synchronize()
    got = np.ascontiguousarray(out.cpu().numpy().view(np.uint64).T)
    np.testing.assert_array_equal(got, oracle.fq_mul(a, b))


def _config3_inputs(n):
    """bench.py --workload wnaf's inputs (config 3): the G1 base of
    tests/golden/bench_points.npz with z = 1 and the tiled scalars"""
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bench_points.npz"))
    base = np.zeros((1, 18), np.uint64)
    base[0, :12] = d["g1"][0, :12]
    base[0, 12:18] = np.array([0x760900000002fffd, 0xebf4000bc40c0002, 0x5f48985753c758ba,
                               0x77ce585370525745, 0x5c071a97a256ec6d, 0x15f65ec3fa80e493], np.uint64)
    s = np.ascontiguousarray(d["s1"][np.arange(n) % 256])
    s[:, 0] ^= np.arange(n, dtype=np.uint64) << np.uint64(8)
    return base, s


def test_config3_full_size_bit_exact(gpu, oracle):
    """config 3 exactly as bench.py times it -- pa_g1_wnaf_fixed_base_device then
    pa_g1_batch_normalization_device on the bench's 2^18 scalars -- against
    the oracle's Wnaf::base(g, 2^18).scalar(s_i) (wnaf.rs:93-107, 169-178)
    followed by G1::batch_normalization (ec.rs:246-294): every output, bit
    for bit (the normalized records are canonical)."""
    import torch
    import pairing_amd.device as pdev
    n = 1 << 18
    base_np, s_np = _config3_inputs(n)
    base, scal = _dev(base_np), _dev(s_np)
    out = pdev.empty_records(n, 18, "cuda:0")
    table, ws = pdev.fixed_base_buffers("cuda:0")
    pdev.g1_wnaf_fixed_base(base, scal, out, table, ws)
    pdev.g1_batch_normalization(out)
    torch.cuda.synchronize()
    exp = oracle.g1_batch_normalization(oracle.g1_wnaf_fixed_base(base_np, s_np, _threads()))
    np.testing.assert_array_equal(_host(out), exp)


def _wrap_scalars(w, g):
    """reprs at the edge of wnaf_form's add_nocarry wrap for window w
    (wnaf.rs:24-35: an odd s with bits w..255 all ones wraps to s - 2^256),
    both sides of it, and random reprs"""
    top = 1 << 256
    vals = [top - 1, top - 2, top - (1 << w) - 1, top - (1 << (w + 1)) + 1, top - (1 << w) + 1,
            top - (1 << w) + 3, top - 3, top - (1 << w), R_ORDER - 1, 0, 1]
    s = np.array([limbs(v, 4) for v in vals], np.uint64)
    return np.concatenate([s, random_scalars(g, 21, bits=256)])


def _wraps(v, w):
    return v & 1 and (v >> w) == (1 << (256 - w)) - 1


@pytest.mark.parametrize("w", [4, 9, 16])
def test_fixed_base_wrapping_reprs_equal_reference(gpu, oracle, w):
    """pa_g1_wnaf_fixed_base_window_device reproduces the reference's wnaf_form
    wrap (wnaf.rs:24-35, 93-107, 169-178): where the first negative digit's
    add_nocarry overflows 2^256 the reference multiplies by s - 2^256 (e.g. -g
    for s = 2^256 - 1).  Equal as points to the oracle's Wnaf::base(g, .)
    .scalar(s) with the same window -- w = 16 is the window of the benched
    2^18 batch -- for a base in G1 (GLV comb) and one outside (the
    double-and-add fallback); the default-window entry at its own n, the
    two-stage GLV and plain-comb entries too."""
    import torch
    import pairing_amd.device as pdev
    import decode_cases as D
    from helpers import mont, Q
    g = rng(70 + w)
    s = _wrap_scalars(w, g)
    vals = [sum(int(x) << (64 * k) for k, x in enumerate(r)) for r in s]
    assert sum(_wraps(v, w) for v in vals) == 4
    base_in, _ = _config3_inputs(1)
    pts, truth = D.subgroup_points(1, seed=61, n=2)
    x, y = next(P for P, t in zip(pts, truth) if not t)
    z = 0x1234567
    base_out = np.array([mont(x * z * z % Q) + mont(y * z * z * z % Q) + mont(z)], np.uint64)
    table, ws = pdev.fixed_base_buffers("cuda:0")
    for base_np in (base_in, base_out):
        out = pdev.empty_records(len(s), 18, "cuda:0")
        pdev.g1_wnaf_fixed_base(_dev(base_np), _dev(s), out, table, ws, window=w)
        torch.cuda.synchronize()
        exp = oracle.g1_wnaf_fixed_base(base_np, s, window=w)
        assert oracle.g1_eq(_host(out), exp).all()
    neg_g = oracle.g1_mul(base_in, np.array([limbs(R_ORDER - 1, 4)], np.uint64))
    assert oracle.g1_eq(oracle.g1_wnaf_fixed_base(base_in, s[:1], window=w), neg_g).all()   # s = 2^256 - 1: -g
    # default window (recommended_wnaf_for_num_scalars(n)) through every G1 fixed-base entry
    n = len(s)
    wd = oracle.lib().o_g1_recommended_wnaf_for_num_scalars(n)
    sd = _wrap_scalars(wd, g)
    exp = oracle.g1_wnaf_fixed_base(base_in, sd)
    b, sc = _dev(base_in), _dev(sd)
    outs = [pdev.empty_records(n, 18, "cuda:0") for _ in range(3)]
    pdev.g1_wnaf_fixed_base(b, sc, outs[0], table, ws)
    pdev.g1_fixed_base_glv_table(b, table, ws)
    pdev.g1_fixed_base_glv_mul(b, table, ws, sc, outs[1])
    table2, _ = pdev.g1_fixed_base_table(b)
    pdev.g1_fixed_base_mul(table2, sc, outs[2])
    torch.cuda.synchronize()
    for o in outs:
        assert oracle.g1_eq(_host(o), exp).all()


@pytest.mark.parametrize("w", [4, 15])
def test_g2_fixed_base_wrapping_reprs_equal_reference(gpu, oracle, w):
    """G2: the same wrap through pa_g2_wnaf_fixed_base_window_device (w = 15 is
    the G2 window at 2^18) and the default-window pa_g2_wnaf_fixed_base_device"""
    import torch
    import pairing_amd.device as pdev
    g = rng(80 + w)
    base = oracle.g2_from_affine(oracle.g2_mul_generator(np.array([limbs(5, 4)], np.uint64)))
    s = _wrap_scalars(w, g)
    table, ws = pdev.g2_fixed_base_buffers("cuda:0")
    out = pdev.empty_records(len(s), 36, "cuda:0")
    pdev.g2_wnaf_fixed_base(_dev(base), _dev(s), out, table, ws, window=w)
    torch.cuda.synchronize()
    assert oracle.g2_eq(_host(out), oracle.g2_wnaf_fixed_base(base, s, window=w)).all()
    wd = oracle.lib().o_g2_recommended_wnaf_for_num_scalars(len(s))
    sd = _wrap_scalars(wd, g)
    out2 = pdev.empty_records(len(sd), 36, "cuda:0")
    pdev.g2_wnaf_fixed_base(_dev(base), _dev(sd), out2, table, ws)
    torch.cuda.synchronize()
    assert oracle.g2_eq(_host(out2), oracle.g2_wnaf_fixed_base(base, sd)).all()
