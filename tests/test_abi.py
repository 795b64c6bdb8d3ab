"""The C ABI library loads and exports every entry point include/pairing_amd.h
declares; the struct layouts match the reference's in-memory order; the
Python layer validates shapes before touching the device.  CPU only: no
compute call is made (there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pairing_amd.h")
LIB = os.path.join(ROOT, "pairing_amd", "lib", "libpairing_amd.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(pa_\w+)\s*\(", src, flags=re.M)


def test_header_declares_the_hot_path():
    names = set(declared_functions())
    for must in ("pa_fq_mul_batch", "pa_g2_prepare_batch", "pa_miller_loop_batch", "pa_multi_miller_loop",
                 "pa_final_exponentiation_batch", "pa_pairing_batch", "pa_pairing_batch_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (pa_\w+)", out))
    assert set(declared_functions()) <= exported


def test_struct_layout_matches_reference_order(tmp_path):
    """sizeof/offsetof of the ABI structs, compiled from the header itself."""
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "pairing_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n",
    sizeof(pa_fq), sizeof(pa_fq2), sizeof(pa_fq6), sizeof(pa_fq12), sizeof(pa_g1_affine),
    offsetof(pa_g1_affine, infinity), sizeof(pa_g2_affine), offsetof(pa_g2_affine, infinity),
    sizeof(pa_g1), sizeof(pa_g2), sizeof(pa_g2_prepared));
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals == [48, 96, 288, 576, 104, 96, 200, 192, 144, 288, 68 * 3 * 96 + 8]


def test_python_layer_checks_shapes_without_device():
    import pairing_amd
    with pytest.raises(ValueError):
        pairing_amd.fq_mul(np.zeros((4, 6), np.uint64), np.zeros((3, 6), np.uint64))
    with pytest.raises(ValueError):
        pairing_amd.pairing(np.zeros((2, 12), np.uint64), np.zeros((2, 25), np.uint64))
    with pytest.raises(ValueError):
        pairing_amd.fq12_mul(np.zeros((2, 71), np.uint64), np.zeros((2, 71), np.uint64))


def test_empty_batches_are_noops():
    import pairing_amd
    assert pairing_amd.fq_mul(np.zeros((0, 6), np.uint64), np.zeros((0, 6), np.uint64)).shape == (0, 6)


def test_no_cpu_fallback_in_product():
    """The product package never loads the oracle (the checker) or any CPU path."""
    pkg = os.path.join(ROOT, "pairing_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                for bad in ("import oracle", "from oracle", "liboracle", "binding.pairing"):
                    assert bad not in text, (f, bad)


def test_errors_are_reported_not_aborted():
    """Invalid arguments return a negative code and a message (no abort across the ABI)."""
    lib = ctypes.CDLL(LIB)
    lib.pa_fq_mul_batch.restype = ctypes.c_int
    lib.pa_fq_mul_batch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t]
    lib.pa_last_error.restype = ctypes.c_char_p
    rc = lib.pa_fq_mul_batch(None, None, None, 5)
    assert rc == -1
    assert b"null" in lib.pa_last_error()


def test_device_layer_rejects_undersized_buffers():
    """pairing_amd.device validates what the kernels would write past (ADVICE
    r02): row counts of q / out / work against p, the ok flags' dtype and
    size, and the fixed-base table / workspace sizes -- before any device call,
    so these checks run without a GPU on CPU tensors shaped like the real ones"""
    import pytest
    import torch
    import pairing_amd.device as pdev

    class FakeCuda:
        """shape/dtype/contiguity of a tensor, reporting is_cuda"""
        def __init__(self, t):
            self.t = t
            self.is_cuda = True
            self.shape, self.dtype = t.shape, t.dtype

        def is_contiguous(self):
            return True

        def dim(self):
            return self.t.dim()

        def numel(self):
            return self.t.numel()

        def data_ptr(self):
            return 0

    f = lambda *s, dt=torch.int64: FakeCuda(torch.zeros(*s, dtype=dt))  # noqa: E731
    with pytest.raises(ValueError, match="work"):
        pdev.multi_pairing(f(4, 13), f(4, 25), f(1, 72), f(1, dt=torch.uint8), f(3, 72))
    with pytest.raises(ValueError, match="q"):
        pdev.multi_pairing(f(4, 13), f(3, 25), f(1, 72), f(1, dt=torch.uint8), f(4, 72))
    with pytest.raises(ValueError, match="ok"):
        pdev.multi_pairing(f(4, 13), f(4, 25), f(1, 72), f(1, dt=torch.int64), f(4, 72))
    with pytest.raises(ValueError, match="ok"):
        pdev.final_exponentiation(f(5, 72), f(5, 72), f(4, dt=torch.uint8))
    with pytest.raises(ValueError, match="out"):
        pdev.miller_loop(f(5, 13), f(5, 25), f(4, 72))
    with pytest.raises(ValueError, match="table"):
        pdev.g1_wnaf_fixed_base(f(1, 18), f(8, 4), f(8, 18), f(3), f(10 ** 6))
