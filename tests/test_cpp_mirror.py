"""The C++ mirror of the reference trait surface (include/pairing_amd.hpp):
CPU -- it compiles with g++ against the C ABI and links libpairing_amd.so;
GPU -- tests/cpp/test_engine.cpp (the reference's engine / encoding / curve /
field / wNAF tests written against the mirror) passes on the device, with
reference-computed inputs supplied by the C oracle."""
import os
import subprocess

import numpy as np
import pytest

from helpers import R_ORDER, limbs, random_scalars, relic_fq12, rng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "pairing_amd", "lib")
SRC = os.path.join(ROOT, "tests", "cpp", "test_engine.cpp")


def _compile(out):
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"), SRC,
           "-o", out, "-L" + LIBDIR, "-lpairing_amd", "-Wl,-rpath," + LIBDIR, "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)


def test_cpp_mirror_compiles_and_links(tmp_path):
    out = str(tmp_path / "test_engine")
    _compile(out)
    assert os.path.getsize(out) > 0


def _to_int(row):
    return sum(int(w) << (64 * i) for i, w in enumerate(row))


def _write_data(oracle, path, n=8):
    g = rng(77)
    a = random_scalars(g, n)
    b = random_scalars(g, n)
    ab = np.array([limbs(_to_int(a[k]) * _to_int(b[k]) % R_ORDER, 4) for k in range(n)], np.uint64)
    a_p = oracle.g1_mul_generator(a, 8)
    b_q = oracle.g2_mul_generator(b, 8)
    ab_p = oracle.g1_mul_generator(ab, 8)
    e_ab = oracle.pairing(a_p, b_q, 8)
    with open(path, "wb") as f:
        f.write(np.uint64(n).tobytes())
        f.write(relic_fq12().tobytes())
        for arr in (a_p, b_q, ab_p, e_ab, a):
            f.write(np.ascontiguousarray(arr, np.uint64).tobytes())


@pytest.mark.gpu
def test_cpp_engine_suite_on_gpu(oracle, tmp_path):
    exe = str(tmp_path / "test_engine")
    _compile(exe)
    data = str(tmp_path / "data.bin")
    _write_data(oracle, data)
    r = subprocess.run([exe, data], capture_output=True, text=True, timeout=600)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok  ") == 10   # tests/cpp/test_engine.cpp main(): ten suites
