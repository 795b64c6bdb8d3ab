"""the C restatement (oracle/) under AddressSanitizer +
UndefinedBehaviorSanitizer.

`make -C oracle asan` builds the same sources into oracle/liboracle_asan.so
with -fsanitize=address,undefined and every report fatal; the CPU oracle
suites then run in a child Python with libasan preloaded and
PA_ORACLE_LIB pointing the binding at that build.  The variable-time binary
extended GCD (`Fq::inverse`, fq.rs:849-902), the window heuristics and the
decoding paths (ec.rs:662-837) are the code most worth sanitizing; the suites
below reach all of them.  CPU only (no GPU involved).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_oracle.py", "tests/test_fr.py", "tests/test_decode.py", "tests/test_group.py",
          "tests/test_msm.py"]


def _libasan():
    out = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    path = out.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def _env(lib):
    env = dict(os.environ)
    env.update(LD_PRELOAD=_libasan(), PA_ORACLE_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return env


@pytest.fixture(scope="module")
def asan_lib():
    if _libasan() is None:
        pytest.skip("gcc has no libasan in this image")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    lib = os.path.join(ROOT, "oracle", "liboracle_asan.so")
    assert os.path.exists(lib)
    return lib


def test_sanitized_oracle_is_the_one_loaded(asan_lib):
    code = ("import sys; sys.path.insert(0, %r); from oracle import binding; binding.lib();"
            "maps = open('/proc/self/maps').read();"
            "assert 'liboracle_asan.so' in maps and 'liboracle.so' not in maps, maps;"
            "assert 'libasan' in maps; print('ok')") % ROOT
    r = subprocess.run([sys.executable, "-c", code], env=_env(asan_lib), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-3000:]


def test_oracle_suites_clean_under_asan_ubsan(asan_lib):
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"]
                       + SUITES, cwd=ROOT, env=_env(asan_lib), capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error:" not in tail, tail
    assert " passed" in tail
