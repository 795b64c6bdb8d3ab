#!/usr/bin/env python3
"""Run a generated code object on the GPU through the HIP module API (ctypes
on libamdhip64) and compare with the DSL golden model (dsl.evaluate).

  python tools/pgen/gpu_check.py small|ml|fe HSACO [n]
"""
import ctypes
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
import numpy as np  # noqa: E402

import dsl  # noqa: E402

hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
LANES = 1
P = ctypes.c_void_p


def ck(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: %d" % (what, rc))


def dev(nbytes):
    p = P()
    ck(hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 8))), "hipMalloc")
    return p


def h2d(p, arr):
    ck(hip.hipMemcpy(p, arr.ctypes.data_as(P), ctypes.c_size_t(arr.nbytes), 1), "h2d")


def d2h(arr, p):
    ck(hip.hipMemcpy(arr.ctypes.data_as(P), p, ctypes.c_size_t(arr.nbytes), 2), "d2h")


def launch(hsaco, kname, args, n, ws_bytes_per_wave, lds_unused=0, reps=3):
    mod, fn = P(), P()
    ck(hip.hipModuleLoad(ctypes.byref(mod), hsaco.encode()), "hipModuleLoad")
    ck(hip.hipModuleGetFunction(ctypes.byref(fn), mod, kname.encode()), "hipModuleGetFunction")
    nblk = (n * LANES + 63) // 64
    ws = dev(ws_bytes_per_wave * nblk)
    buf = (ctypes.c_uint64 * 5)(*(list(args[:3]) + [n, ws.value or 0]))
    size = ctypes.c_size_t(ctypes.sizeof(buf))
    extra = (P * 5)(P(1), ctypes.cast(buf, P), P(2), ctypes.cast(ctypes.byref(size), P), P(3))
    ck(hip.hipDeviceSynchronize(), "sync0")
    t = time.time()
    for _ in range(reps):
        ck(hip.hipModuleLaunchKernel(fn, nblk, 1, 1, 64, 1, 1, 0, None, None, extra), "launch")
    ck(hip.hipDeviceSynchronize(), "sync")
    return (time.time() - t) / reps


def rand_fq(rng):
    return rng.randrange(dsl.Q)


def to_words(xs):
    out = []
    for x in xs:
        out += [(x >> (64 * i)) & (2**64 - 1) for i in range(6)]
    return out


def main():
    which, hsaco = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    import importlib
    meta = importlib.import_module("build_gen").PROGRAMS[which]
    prog, cfg, kname, nmem = meta()
    global LANES
    LANES = prog.lanes
    rng = random.Random(5)
    if which in ("small", "fe", "fe2", "cyc"):
        ins = [[rand_fq(rng) for _ in range(12)] for _ in range(n)]
        ins[1] = [0] * 12  # f == 0 lane
        rec_in = np.array([to_words(r) for r in ins], dtype=np.uint64)
        d_in, d_out, d_ok = dev(rec_in.nbytes), dev(rec_in.nbytes), dev(n)
        h2d(d_in, rec_in)
        dt = launch(hsaco, kname, [d_in.value, d_out.value, d_ok.value], n, nmem * 3584)
        out = np.zeros_like(rec_in)
        d2h(out, d_out)
        ok = np.zeros(n, np.uint8)
        d2h(ok, d_ok)
        bad = 0
        for lane in range(min(n, 8)):
            if lane == 1:
                good = ok[1] == 0 and not out[1].any()
            else:
                want = dsl.evaluate(prog, {k: ins[lane][k] for k in range(12)})
                got = [sum(int(out[lane, 6 * k + i]) << (64 * i) for i in range(6)) for k in range(12)]
                good = got == [want[k] for k in range(12)] and ok[lane] == 1
            bad += not good
            print("lane %d: %s" % (lane, "OK" if good else "MISMATCH"))
        print("time %.3f ms for n=%d" % (dt * 1e3, n))
        sys.exit(1 if bad else 0)
    if which in ("ml", "ml2"):
        ins = [[rand_fq(rng) for _ in range(6)] for _ in range(n)]
        prec = np.array([to_words(r[:2]) + [0] for r in ins], dtype=np.uint64)
        qrec = np.array([to_words(r[2:]) + [0] for r in ins], dtype=np.uint64)
        prec[2, 12] = 1   # P at infinity
        qrec[4, 24] = 1   # Q at infinity
        d_p, d_q, d_out = dev(prec.nbytes), dev(qrec.nbytes), dev(n * 576)
        h2d(d_p, prec)
        h2d(d_q, qrec)
        dt = launch(hsaco, kname, [d_p.value, d_q.value, d_out.value], n, nmem * 3584)
        out = np.zeros((n, 72), np.uint64)
        d2h(out, d_out)
        one = [(1 << 384) % dsl.Q] + [0] * 11
        bad = 0
        for lane in range(min(n, 8)):
            got = [sum(int(out[lane, 6 * k + i]) << (64 * i) for i in range(6)) for k in range(12)]
            if lane in (2, 4):
                good = got == one
            else:
                want = dsl.evaluate(prog, {k: ins[lane][k] for k in range(6)})
                good = got == [want[k] for k in range(12)]
            bad += not good
            print("lane %d: %s" % (lane, "OK" if good else "MISMATCH"))
        print("time %.3f ms for n=%d" % (dt * 1e3, n))
        sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
