"""One G2Prepared shared by a batch of G1 points (VERDICT r04 "missing" 1).

Engine::miller_loop takes &G2Prepared references (reference src/lib.rs:88-96)
and Prepared is Clone (lib.rs:192), so a caller may pair many P with the same
prepared Q -- a verifying key's prepared gamma / delta.  The product path
pa_miller_loop_shared_prepared[_device] stages the 68 lines once per call
(k_shared_line_table) and runs the generated kernel pa_gen_miller_loop_shared
(tools/pgen/kernels.py miller_loop_shared_prog) with no G2 arithmetic.  It
must give, bit for bit, what the reference's miller_loop([(P_i, Q)])
(mod.rs:40-102) gives -- checked here against the oracle's miller_loop_batch
with the one prepared record repeated, at the bench size 2^16 and ragged
sizes, with infinity P (bench.make_pairs: 1/128 of them) and infinity Q
(empty coeffs + flag, mod.rs:169-174).

The CPU tests check the DSL program and the emitted code (simulator) against
the oracle's line coefficients; the GPU tests call through the C ABI."""
import os
import sys

import numpy as np
import pytest

from helpers import Q, limbs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNK = 4096


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16")), 16))


def _expected(oracle, p_np, prep1):
    """the reference's miller_loop([(p[i], q)]) for every i, q = prep1[0]"""
    out = []
    for k in range(0, p_np.shape[0], CHUNK):
        pc = p_np[k:k + CHUNK]
        out.append(oracle.miller_loop_batch(pc, np.repeat(prep1, pc.shape[0], axis=0), _threads()))
    return np.concatenate(out) if out else np.zeros((0, 72), np.uint64)


def _infinity_q():
    q = np.zeros((1, 25), np.uint64)
    q[0, 12:18] = limbs(pow(2, 384, Q))
    q[0, 24] = 1
    return q


def _coeff_ints(prep1):
    """68 lines x six ABI integers of one G2Prepared record"""
    rec = prep1.reshape(-1)
    out = []
    for line in range(68):
        vals = []
        for j in range(6):
            w = rec[36 * line + 6 * j: 36 * line + 6 * j + 6]
            vals.append(sum(int(x) << (64 * i) for i, x in enumerate(w)))
        out.append(vals)
    return out


# ---------------- CPU: the generated program and its emitted code ----------------
def _pgen():
    sys.path[:0] = [os.path.join(ROOT, "tools", "pgen"), os.path.join(ROOT, "tools")]
    import build_gen  # noqa: F401
    import dsl
    import kernels
    return dsl, kernels


def test_dsl_shared_miller_loop_matches_oracle(oracle):
    """the DSL program over the line table of a real G2Prepared equals the
    oracle's miller_loop with that record (raw / lazy table values as
    k_shared_line_table writes them)"""
    import bench
    dsl, kernels = _pgen()
    p_np, q_np = bench.make_pairs(4, 0, seed=21)
    prep1 = oracle.g2_prepare(q_np[1:2], 1)
    lines = kernels.shared_table_lines(_coeff_ints(prep1))
    prog = kernels.miller_loop_shared_prog()
    want = _expected(oracle, p_np, prep1)
    for i in range(4):
        if p_np[i, 12] & 0xff:
            continue   # infinity P is the kernel's lane select, outside the DSL
        px = sum(int(x) << (64 * k) for k, x in enumerate(p_np[i, 0:6]))
        py = sum(int(x) << (64 * k) for k, x in enumerate(p_np[i, 6:12]))
        got = dsl.evaluate(prog, {0: px, 1: py, "lines": lines})
        row = np.array([limbs(got[k]) for k in range(12)], np.uint64).reshape(-1)
        np.testing.assert_array_equal(row, want[i])


def test_sim_shared_miller_loop_kernel():
    """the emitted instruction stream of pa_gen_miller_loop_shared under the
    gfx950 subset simulator equals the DSL trace value by value"""
    _pgen()
    import sim_check
    assert sim_check.check("mls", debug=True)


# ---------------- GPU: through the C ABI ----------------
def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")


def _host(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1 << 16, 333, 1])
def test_shared_prepared_device_bit_exact(gpu, oracle, n):
    import torch
    import bench
    import pairing_amd.device as pdev
    p_np, q_np = bench.make_pairs(n, 0, seed=13)
    prep1 = oracle.g2_prepare(q_np[n // 2: n // 2 + 1], 1)
    out = pdev.empty_records(n, 72, "cuda:0")
    pdev.miller_loop_shared_prepared(_dev(p_np), _dev(prep1), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), _expected(oracle, p_np, prep1))


@pytest.mark.gpu
def test_shared_prepared_infinity_q_and_p(gpu, oracle):
    """a prepared infinity Q contributes one for every P; infinity P gives one"""
    import torch
    import bench
    import pairing_amd.device as pdev
    n = 777
    p_np, _ = bench.make_pairs(n, 0, seed=17)
    p_np[::5, :12] = 0
    p_np[::5, 12] = 1
    prep_inf = oracle.g2_prepare(_infinity_q(), 1)
    assert prep_inf[0, -1] == 1
    out = pdev.empty_records(n, 72, "cuda:0")
    pdev.miller_loop_shared_prepared(_dev(p_np), _dev(prep_inf), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), _expected(oracle, p_np, prep_inf))


@pytest.mark.gpu
def test_shared_prepared_host_api_and_pairing(gpu, oracle):
    """the host-buffer entry, and final_exponentiation over its output = e(P_i, Q)"""
    import bench
    import pairing_amd
    n = 300
    p_np, q_np = bench.make_pairs(n, 0, seed=19)
    q1 = q_np[7:8]
    prep1 = pairing_amd.g2_prepare(q1)
    np.testing.assert_array_equal(prep1, oracle.g2_prepare(q1, 1))
    f = pairing_amd.miller_loop_shared_prepared(p_np, prep1)
    np.testing.assert_array_equal(f, _expected(oracle, p_np, prep1))
    e = pairing_amd.final_exponentiation(f)
    e = e[0] if isinstance(e, tuple) else e
    np.testing.assert_array_equal(e, oracle.pairing(p_np, np.repeat(q1, n, axis=0), _threads()))
    with pytest.raises(ValueError):
        pairing_amd.miller_loop_shared_prepared(p_np, np.repeat(prep1, 2, axis=0))
