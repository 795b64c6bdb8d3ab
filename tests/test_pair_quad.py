"""The lane-group pairing kernels (kernels_pair_quad.hip, pair_quad.h: one
pairing per 32 lanes, the tower's products batched into levels over 8 lane
quads), selected by pa_set_pairing_kernel(5): Miller values bit-exact against
the oracle's miller_loop (mod.rs:40-102, reference-form G2 steps), the final
exponentiation and the pairing bit-exact against the oracle (mod.rs:104-160,
lib.rs:101-109), with infinity pairs, zero Miller values (None) and odd batch
sizes (a half-empty last wave)."""
import numpy as np
import pytest

from helpers import Q, limbs
from test_bench_sizes import _dev, _host, _threads

pytestmark = pytest.mark.gpu


@pytest.fixture
def lane_groups(gpu):
    gpu.set_pairing_kernel(5)
    yield gpu
    gpu.set_pairing_kernel(0)


def _pairs(n, seed):
    import bench
    p, q = bench.make_pairs(n, 0, seed=seed)
    if n > 3:   # an infinity Q besides the infinity P make_pairs mixes in
        q[3, :24] = 0
        q[3, 12:18] = limbs(pow(2, 384, Q))
        q[3, 24] = 1
    return p, q


@pytest.mark.parametrize("n", [1, 2, 37, 130])
def test_lane_group_miller_loop_bit_exact(lane_groups, oracle, n):
    import torch
    import pairing_amd.device as pdev
    p, q = _pairs(n, 41 + n)
    f = pdev.empty_records(n, 72, "cuda:0")
    pdev.miller_loop(_dev(p), _dev(q), f)
    torch.cuda.synchronize()
    want = oracle.miller_loop_batch(p, oracle.g2_prepare(q, _threads()), _threads())
    np.testing.assert_array_equal(_host(f), want)


@pytest.mark.parametrize("n", [1, 37, 130])
def test_lane_group_pairing_bit_exact(lane_groups, oracle, n):
    import torch
    import pairing_amd.device as pdev
    p, q = _pairs(n, 7 + n)
    out = pdev.empty_records(n, 72, "cuda:0")
    scratch = pdev.empty_records(n, 72, "cuda:0")
    pdev.pairing(_dev(p), _dev(q), out, scratch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.pairing(p, q, _threads()))


def test_lane_group_final_exp_zero_and_in_place(lane_groups, oracle):
    """f == 0 gives ok = 0 and a zero output (mod.rs:108); in place == apart"""
    import torch
    import pairing_amd.device as pdev
    from test_bench_sizes import _field_rows, FQ_TOP
    n = 21
    f = _field_rows(43, n * 12, 6, FQ_TOP, [1]).reshape(n, 72)
    f[4] = 0
    exp, ok_exp = oracle.final_exponentiation(f, _threads())
    d = _dev(f)
    out = pdev.empty_records(n, 72, "cuda:0")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    pdev.final_exponentiation(d, out, ok)
    ok2 = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    pdev.final_exponentiation(d, d, ok2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), exp)
    np.testing.assert_array_equal(_host(d), exp)
    np.testing.assert_array_equal(ok.cpu().numpy(), np.asarray(ok_exp, np.uint8))
    np.testing.assert_array_equal(ok2.cpu().numpy(), np.asarray(ok_exp, np.uint8))
    assert ok.cpu().numpy()[4] == 0


def test_lane_group_multi_pairing(lane_groups, oracle):
    import pairing_amd
    p, q = _pairs(9, 77)
    got, ok = pairing_amd.multi_pairing(p, q)
    assert ok
    f = oracle.miller_loop(p, oracle.g2_prepare(q))
    exp, _ = oracle.final_exponentiation(f[None, :].copy())
    np.testing.assert_array_equal(np.asarray(got).reshape(-1), exp.reshape(-1))


@pytest.mark.parametrize("n", [768, 769, 4096, 4097])
def test_default_selection_lane_group_window_edges(gpu, oracle, n):
    """the default selection runs (PA_PQ_MIN, PA_PQ_MAX] = (768, 4096] on the
    lane-group kernels and the cooperative ones on both sides: bit-exact
    pairings either side of both edges"""
    import torch
    import pairing_amd.device as pdev
    p, q = _pairs(n, 90 + n % 7)
    out = pdev.empty_records(n, 72, "cuda:0")
    scratch = pdev.empty_records(n, 72, "cuda:0")
    pdev.pairing(_dev(p), _dev(q), out, scratch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.pairing(p, q, _threads()))



def test_lane_group_miller_loop_points_outside_the_subgroups(lane_groups, oracle):
    """the Miller loop is defined for any curve points (mod.rs:40-102 does no
    subgroup check): G1 and G2 points with small-order components give the
    oracle's Miller values bit for bit"""
    import torch
    import decode_cases as D
    import pairing_amd.device as pdev
    p1, _ = D.subgroup_points(1, seed=93, n=2)
    p2, _ = D.subgroup_points(2, seed=94, n=2)
    m = min(len(p1), len(p2))
    p = np.array([D.aff_record(1, P) for P in p1[:m]], np.uint64)
    q = np.array([D.aff_record(2, P) for P in p2[:m]], np.uint64)
    f = pdev.empty_records(m, 72, "cuda:0")
    pdev.miller_loop(_dev(p), _dev(q), f)
    torch.cuda.synchronize()
    want = oracle.miller_loop_batch(p, oracle.g2_prepare(q))
    np.testing.assert_array_equal(_host(f), want)
