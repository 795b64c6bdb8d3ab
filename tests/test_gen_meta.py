"""Every generated code object states the HBM spill slots per wave it uses
(`<kernel>_mem_slots`, tools/pgen/render.py); gen_launch.hip refuses one
that needs more workspace than the library allocates (a stale or swapped
file, PA_GEN_DIR) instead of letting its waves write past their slices."""
import os
import re
import shutil
import subprocess
import sys

import pytest

from elfsym import read_u32, symbol_offset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pairing_amd", "lib")
# every code object the library loads (gen_launch.hip kFile)
KERNELS = ["pa_gen_miller_loop", "pa_gen_final_exp", "pa_gen_miller_loop2", "pa_gen_final_exp2",
           "pa_gen_miller_loop_shared", "pa_gen_miller_loop_prepared", "pa_gen_miller_loop2p",
           "pa_gen_miller_loop1p"]


def test_kernel_list_matches_the_loader():
    with open(os.path.join(ROOT, "pairing_amd", "csrc", "gen_launch.hip")) as f:
        src = f.read()
    files = re.search(r"kFile\[kKernels\] = \{(.*?)\};", src, re.S).group(1)
    assert re.findall(r'"(pa_gen_\w+)\.hsaco"', files) == KERNELS


def meta_slots():
    with open(os.path.join(ROOT, "pairing_amd", "csrc", "pa_gen_meta.h")) as f:
        return {m.group(1).lower(): int(m.group(2))
                for m in re.finditer(r"#define PA_GEN_(\w+)_MEM_SLOTS (\d+)", f.read())}


def test_code_objects_state_their_workspace_slots():
    meta = meta_slots()
    for k in KERNELS:
        path = os.path.join(LIB, k + ".hsaco")
        assert read_u32(path, k + "_mem_slots") == meta[k[len("pa_gen_"):]], k


@pytest.mark.gpu
def test_oversized_code_object_is_refused(tmp_path):
    """a copy of the code objects whose final exponentiation claims more
    workspace slots than the library allocates: the pairing call fails with
    the loader's message, no kernel runs"""
    for k in KERNELS:
        shutil.copy(os.path.join(LIB, k + ".hsaco"), tmp_path / (k + ".hsaco"))
    path = str(tmp_path / "pa_gen_final_exp.hsaco")
    off, _ = symbol_offset(path, "pa_gen_final_exp_mem_slots")
    with open(path, "r+b") as f:
        f.seek(off)
        f.write((100000).to_bytes(4, "little"))
    code = ("import numpy as np, pairing_amd, sys\n"
            "sys.path.insert(0, 'tests')\n"
            "import bench\n"
            "pairing_amd.set_pairing_kernel(3)\n"   # the generated one-lane kernels at any size
            "p, q = bench.make_pairs(64, 0)\n"
            "try:\n"
            "    pairing_amd.pairing(p, q)\n"
            "except pairing_amd.PairingError as e:\n"
            "    print('REFUSED', e)\n"
            "    sys.exit(0)\n"
            "print('NOT REFUSED')\n"
            "sys.exit(1)\n")
    env = dict(os.environ, PA_GEN_DIR=str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "workspace slots" in r.stdout, r.stdout
