"""GPU tests of single pieces of the generated kernels' code, on test-only
code objects (tools/pgen/unit_progs.py -> pairing_amd/lib/test/): the
in-kernel binary-GCD inversion, the zero-test select, and Karabina
decompression including its b0 = 0 branch (tests/golden/karabina_b0zero.json),
each against the DSL model that the simulator and the final exponentiation's
oracle parity already pin (tests/test_pgen.py)."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tools", "pgen"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import dsl  # noqa: E402
import unit_progs  # noqa: E402

pytestmark = pytest.mark.gpu


def _run(name, prog, rows, lanes=1, ws_slots=1):
    """rows: lists of 12 canonical ABI integers; returns (gpu rows, model rows)"""
    import torch
    import hipmod
    n = len(rows)
    words = np.zeros((n, 72), dtype=np.uint64)
    for i, r in enumerate(rows):
        for k, x in enumerate(r):
            for j in range(6):
                words[i, 6 * k + j] = (x >> (64 * j)) & ((1 << 64) - 1)
    src = torch.from_numpy(words.view(np.int64)).cuda()
    out = torch.zeros_like(src)
    hipmod.launch(name, src, out, None, n, ws_slots=ws_slots, lanes=lanes)
    got = out.cpu().numpy().view(np.uint64)
    gpu = [[sum(int(got[i, 6 * k + j]) << (64 * j) for j in range(6)) for k in range(12)] for i in range(n)]
    model = []
    for r in rows:
        o = dsl.evaluate(prog, {k: r[k] for k in range(12)})
        model.append([o[k] for k in range(12)])
    return gpu, model


def test_binv_and_selz_on_gpu():
    """1 000 lanes: random operands, and lanes whose products / sums are 0 or
    q (inverse 0) and whose select tests are zero"""
    g = random.Random(11)
    Q = dsl.Q
    rows = []
    for i in range(1000):
        r = [g.randrange(Q) for _ in range(12)]
        if i % 7 == 1:
            r[4] = r[5] = r[6] = 0
        if i % 11 == 2:
            r[0] = 0
        if i % 13 == 3:
            r[2] = (Q - r[3]) % Q
        rows.append(r)
    gpu, model = _run("tunit", unit_progs.unit_prog(), rows)
    assert gpu == model
    one = (1 << 384) % Q
    assert all(gr[4] == (one if r[0] and r[1] else 0) for gr, r in zip(gpu, rows))


def test_karabina_decompression_on_gpu():
    """decompression rebuilds cyclotomic elements exactly: random ones, the
    constructed b0 = 0 element (the select's rare branch) and the identity"""
    import test_pgen as tp
    import pymodel as pm
    elems = [tp._cyclotomic(s) for s in range(20)] + [tp._b0_zero_element(), pm.F12ONE]
    rows = [tp._abi_words(f) for f in elems] * 3
    gpu, model = _run("tdec", unit_progs.dec_prog(), rows)
    assert gpu == model == rows


def test_karabina_decompression_lane_pairs_on_gpu():
    """the same on the lane-pair tower (round 5: the lane-pair final
    exponentiation squares compressed too): the b0 == 0 select reads both
    lanes' coordinates, the norm's binary GCD runs on both lanes"""
    import test_pgen as tp
    import pymodel as pm
    elems = [tp._cyclotomic(s) for s in range(20)] + [tp._b0_zero_element(), pm.F12ONE]
    rows = [tp._abi_words(f) for f in elems] * 3
    gpu, model = _run("tdec2", unit_progs.dec_prog(lanes=2), rows, lanes=2, ws_slots=64)
    assert gpu == model == rows
