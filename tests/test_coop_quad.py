"""GPU unit test of the quad-cooperative field operations (coop_quad.h, the
verifier VM Vm4 of kernels_coop.hip): four lanes per value, DPP limb / carry
exchange.  Each must return exactly the limbs of the one-lane code it stands
in for (the fl_gen.h product leaves and fl.h red), which the cooperative
schedules' replay (tools/pgen/coop.py, tests/test_pgen.py) models; the values
are also checked against Python big integers.  Operands are lazy values at
the bounds the VM's contract allows (sum of U normalized values, limbs up to
U (2^28 - 1)), including maximal limbs and zeros.  Test-only code object:
tests/hip/coop_quad_unit.hip -> pairing_amd/lib/test/coop_quad_unit.hsaco."""
import ctypes
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CO = os.path.join(ROOT, "pairing_amd", "lib", "test", "coop_quad_unit.hsaco")
Q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
M = (1 << 28) - 1
RINV = pow(1 << 392, -1, Q)


def digits(v):
    return [(v >> (28 * i)) & M for i in range(13)] + [v >> (28 * 13)]


def lazy(g, u, edge=None):
    """limb-wise sum of u normalized values < 2q (bound U = u)"""
    limbs = [0] * 14
    for _ in range(u):
        v = {"max": 2 * Q - 1, "zero": 0}.get(edge, None)
        if v is None:
            v = g.randrange(2 * Q)
        for i, d in enumerate(digits(v)):
            limbs[i] += d
    return limbs


def value(limbs):
    return sum(int(x) << (28 * i) for i, x in enumerate(limbs))


def run(op, cases, kernel="coop_quad_unit", per_block=64):
    import torch
    import hipmod
    n = len(cases)
    buf = np.zeros((n, 4, 16), dtype=np.uint32)
    for i, ops in enumerate(cases):
        for k, limbs in enumerate(ops):
            buf[i, k, :14] = limbs
    src = torch.from_numpy(buf.view(np.int32)).cuda()
    out = torch.zeros((n, 2, 16), dtype=torch.int32, device="cuda")
    hipmod.launch_kernel(CO, kernel,
                         [(ctypes.c_uint64, src.data_ptr()), (ctypes.c_uint64, out.data_ptr()),
                          (ctypes.c_uint32, n), (ctypes.c_uint32, op)], (n + per_block - 1) // per_block, 256)
    return out.cpu().numpy().view(np.uint32)


BOUNDS = {0: [(1, 1), (4, 4), (16, 1), (1, 16), (2, 8)],
          1: [((1, 1), (1, 1)), ((4, 2), (3, 3)), ((8, 2), (1, 1)), ((1, 1), (16, 1))],
          2: [(1,), (2,), (3,)],
          3: [(1,), (4,), (16,)],
          4: [(1, 1), (4, 4), (2, 8)]}


@pytest.mark.parametrize("op", [0, 1, 2, 3, 4], ids=["mul", "sop2", "sqr", "red", "gather_mul"])
def test_quad_ops_bit_identical_to_one_lane(op):
    g = random.Random(100 + op)
    cases = []
    for bnd in BOUNDS[op]:
        for t in range(160):
            edge = "max" if t % 40 == 0 else "zero" if t % 40 == 1 else None
            if op == 1:
                (ua, ub), (uc, ud) = bnd
                cases.append([lazy(g, ua, edge), lazy(g, ub, edge), lazy(g, uc), lazy(g, ud, edge)])
            elif op in (2, 3):
                cases.append([lazy(g, bnd[0], edge), [0] * 14, [0] * 14, [0] * 14])
            else:
                ua, ub = bnd
                cases.append([lazy(g, ua, edge), lazy(g, ub), [0] * 14, [0] * 14])
    got = run(op, cases)
    assert (got[:, 0, :] == got[:, 1, :]).all(), \
        "quad != one-lane at cases %s" % np.nonzero((got[:, 0, :] != got[:, 1, :]).any(axis=1))[0][:10]
    for i, (a, b, c, d) in enumerate(cases):
        va, vb, vc, vd = value(a), value(b), value(c), value(d)
        r = value(got[i, 0, :14])
        if op in (0, 4):
            want = va * vb * RINV
        elif op == 1:
            want = (va * vb + vc * vd) * RINV
        elif op == 2:
            want = va * va * RINV
        else:
            want = va
        assert r % Q == want % Q and r < 2 * Q, (op, i)
        assert all(int(x) <= M for x in got[i, 0, :13]) and got[i, 0, 14] == 0 and got[i, 0, 15] == 0


@pytest.mark.parametrize("op", [0, 1, 2, 4], ids=["mul", "sop2", "sqr", "gather_mul"])
def test_hex_ops_bit_identical_to_one_lane(op):
    """coop_hex.h (experiment): one value per 16-lane DPP row, the digit
    broadcast by row_newbcast and the accumulator shift by row_shl -- the same
    limbs as the one-lane leaves at the bounds the quad test uses"""
    g = random.Random(200 + op)
    cases = []
    for bnd in BOUNDS[op]:
        for t in range(160):
            edge = "max" if t % 40 == 0 else "zero" if t % 40 == 1 else None
            if op == 1:
                (ua, ub), (uc, ud) = bnd
                cases.append([lazy(g, ua, edge), lazy(g, ub, edge), lazy(g, uc), lazy(g, ud, edge)])
            elif op == 2:
                cases.append([lazy(g, bnd[0], edge), [0] * 14, [0] * 14, [0] * 14])
            else:
                ua, ub = bnd
                cases.append([lazy(g, ua, edge), lazy(g, ub), [0] * 14, [0] * 14])
    got = run(op, cases, kernel="coop_hex_unit", per_block=16)
    assert (got[:, 0, :] == got[:, 1, :]).all(), \
        "hex != one-lane at cases %s" % np.nonzero((got[:, 0, :] != got[:, 1, :]).any(axis=1))[0][:10]
