"""CPU check of the device Fq inversion algorithm (pairing_amd/csrc/bgcd.h,
optimized binary GCD) against Python's modular inverse.

The same header is compiled for gfx950 inside fq_inv (tower.h); here it is
built with g++ so the algorithm is checked without a GPU.  The reference's
Fq::inverse is fq.rs:849-902 (None iff the input is zero)."""
import ctypes
import os
import random
import shutil
import subprocess

import pytest

from pymodel import Q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bg(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    d = tmp_path_factory.mktemp("bgcd")
    src = d / "bg.cpp"
    src.write_text('#include "bgcd.h"\n'
                   'extern "C" int bg_inverse(uint32_t* out, const uint32_t* y) '
                   '{ return pa::bgcd::inverse(out, y) ? 1 : 0; }\n')
    so = d / "libbg.so"
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I", os.path.join(ROOT, "pairing_amd", "csrc"),
                    str(src), "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))

    def inv(y):
        a = (ctypes.c_uint32 * 12)(*[(y >> (32 * i)) & 0xffffffff for i in range(12)])
        o = (ctypes.c_uint32 * 12)()
        ok = lib.bg_inverse(o, a)
        return bool(ok), sum(o[i] << (32 * i) for i in range(12))
    return inv


def test_bgcd_edges(bg):
    assert bg(0) == (False, 0)  # fq.rs:850-851: None for zero
    for y in [1, 2, 3, Q - 1, Q - 2, (Q - 1) // 2, 1 << 380, (1 << 381) % Q, (1 << 64) - 1, (1 << 62), 3 ** 200 % Q]:
        ok, r = bg(y)
        assert ok and r == pow(y, -1, Q), hex(y)


def test_bgcd_random(bg):
    g = random.Random(20201016)
    ys = [g.randrange(1, Q) for _ in range(20000)]
    ys += [g.randrange(1, 1 << g.randrange(1, 382)) % Q or 1 for _ in range(5000)]
    for y in ys:
        ok, r = bg(y)
        assert ok and r == pow(y, -1, Q), hex(y)
