#!/usr/bin/env python3
"""DSL golden model vs the C oracle: evaluate the generated kernels' programs
on random pairs (exact limb semantics, every bound asserted) and compare the
Miller-loop and final-exponentiation outputs bit for bit."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "tests"), ROOT]
import numpy as np  # noqa: E402

import dsl  # noqa: E402
import kernels  # noqa: E402
from helpers import random_scalars, rng  # noqa: E402
from oracle import binding as O  # noqa: E402


def words_to_int(ws):
    return sum(int(w) << (64 * i) for i, w in enumerate(ws))


def run(n=2, seed=3, lanes=1):
    g = rng(seed)
    p = O.g1_mul_generator(random_scalars(g, n))
    q = O.g2_mul_generator(random_scalars(g, n))
    ml_ref = O.miller_loop_batch(p, O.g2_prepare(q))
    fe_ref, _ = O.final_exponentiation(ml_ref)
    ml, fe = kernels.miller_loop_prog(lanes=lanes), kernels.final_exp_prog(lanes=lanes)
    for i in range(n):
        ins = {k: words_to_int(p[i, 6 * k:6 * k + 6]) for k in range(2)}
        ins.update({2 + k: words_to_int(q[i, 6 * k:6 * k + 6]) for k in range(4)})
        t = time.time()
        st = dsl.Stats()
        out = dsl.evaluate(ml, ins, st)
        got = [out[k] for k in range(12)]
        want = [words_to_int(ml_ref[i, 6 * k:6 * k + 6]) for k in range(12)]
        assert got == want, "miller loop mismatch at pair %d" % i
        print("pair %d: miller loop OK (%.1fs) %s" % (i, time.time() - t, st.counts))
        t = time.time()
        st = dsl.Stats()
        out = dsl.evaluate(fe, {k: want[k] for k in range(12)}, st)
        got = [out[k] for k in range(12)]
        want2 = [words_to_int(fe_ref[i, 6 * k:6 * k + 6]) for k in range(12)]
        assert got == want2, "final exp mismatch at pair %d" % i
        print("pair %d: final exp OK (%.1fs) %s" % (i, time.time() - t, st.counts))


if __name__ == "__main__":
    for lanes in (int(a) for a in (sys.argv[1:] or ["1", "2"])):
        print("lanes =", lanes)
        run(lanes=lanes)
