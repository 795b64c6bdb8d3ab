"""The generated Miller loop over (P_i, G2Prepared_i) pairs -- the
reference's Engine::miller_loop call shape (src/lib.rs:88-96; bls12_381/
mod.rs:40-102 with each pair's own G2Prepared, prepared by mod.rs:153-213).

pa_miller_loop_batch[_device] and pa_multi_miller_loop run
pa_gen_miller_loop_prepared (tools/pgen/kernels.py miller_loop_prepared_prog,
kcfg.MillerLoopPreparedCfg): each lane reads the lines of its own record, in
the ABI form (c2 converted in the kernel by one product).  The CPU tests check
the DSL program against the oracle and the emitted code against the DSL
(simulator); the GPU tests compare the C ABI's output with the oracle's
miller_loop_batch bit for bit, at the bench size 2^16 and ragged sizes, with
infinity P and infinity Q records mixed in."""
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


def _expected(oracle, p_np, prep):
    out = []
    for k in range(0, p_np.shape[0], CHUNK):
        out.append(oracle.miller_loop_batch(p_np[k:k + CHUNK], prep[k:k + CHUNK], _threads()))
    return np.concatenate(out) if out else np.zeros((0, 72), np.uint64)


def _coeff_ints(rec):
    rec = rec.reshape(-1)
    return [[sum(int(x) << (64 * i) for i, x in enumerate(rec[36 * line + 6 * j: 36 * line + 6 * j + 6]))
             for j in range(6)] for line in range(68)]


def _pgen():
    sys.path[:0] = [os.path.join(ROOT, "tools", "pgen"), os.path.join(ROOT, "tools")]
    import build_gen  # noqa: F401
    import dsl
    import kernels
    return dsl, kernels


# ---------------- CPU ----------------
def test_dsl_prepared_miller_loop_matches_oracle(oracle):
    """the DSL program over real G2Prepared records (raw ABI values) equals the
    oracle's miller_loop of each pair"""
    import bench
    dsl, kernels = _pgen()
    p_np, q_np = bench.make_pairs(3, 0, seed=31)
    prep = oracle.g2_prepare(q_np, 1)
    want = _expected(oracle, p_np, prep)
    prog = kernels.miller_loop_prepared_prog()
    for i in range(3):
        if p_np[i, 12] & 0xff:
            continue   # infinity P: the kernel's lane select, outside the DSL
        px = sum(int(x) << (64 * k) for k, x in enumerate(p_np[i, 0:6]))
        py = sum(int(x) << (64 * k) for k, x in enumerate(p_np[i, 6:12]))
        got = dsl.evaluate(prog, {0: px, 1: py, "lines": kernels.prepared_table_lines(_coeff_ints(prep[i]))})
        row = np.array([limbs(got[k]) for k in range(12)], np.uint64).reshape(-1)
        np.testing.assert_array_equal(row, want[i])


def test_sim_prepared_miller_loop_kernel():
    """pa_gen_miller_loop_prepared's instruction stream under the gfx950 subset
    simulator equals the DSL trace value by value (per-lane loads, deferred
    in-place limb split)"""
    _pgen()
    import sim_check
    assert sim_check.check("mlp", debug=True)


# ---------------- GPU: through the C ABI ----------------
def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda:0")


def _host(t):
    return t.cpu().numpy().view(np.uint64)


def _infinity_q(n):
    q = np.zeros((n, 25), np.uint64)
    q[:, 12:18] = limbs(pow(2, 384, Q))
    q[:, 24] = 1
    return q


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1 << 16, 4097, 65, 1])
def test_prepared_device_bit_exact(gpu, oracle, n):
    """the bench's call shape: G2Prepared records on the device (prepared by
    pa_g2_prepare_batch_device, itself checked bit-exact in test_gpu_parity),
    infinity P (1/128 of bench.make_pairs) and a few infinity Q"""
    import torch
    import bench
    import pairing_amd.device as pdev
    p_np, q_np = bench.make_pairs(n, 0, seed=41)
    q_np[3::97] = _infinity_q(len(q_np[3::97]))
    dq = _dev(q_np)
    prep = pdev.empty_records(n, 2449, "cuda:0")
    pdev.g2_prepare(dq, prep)
    out = pdev.empty_records(n, 72, "cuda:0")
    pdev.miller_loop_prepared(_dev(p_np), prep, out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), _expected(oracle, p_np, _host(prep)))


@pytest.mark.gpu
def test_prepared_host_api_and_multi_miller_loop(gpu, oracle):
    """the host entries: miller_loop_batch, and multi_miller_loop (the product
    over the pairs, mod.rs:40-102) on the same kernel"""
    import bench
    import pairing_amd
    n = 130
    p_np, q_np = bench.make_pairs(n, 0, seed=43)
    prep = oracle.g2_prepare(q_np, _threads())
    f = pairing_amd.miller_loop_batch(p_np, prep)
    np.testing.assert_array_equal(f, _expected(oracle, p_np, prep))
    m = pairing_amd.multi_miller_loop(p_np[:17], prep[:17])
    np.testing.assert_array_equal(m, oracle.miller_loop(p_np[:17], prep[:17]))
