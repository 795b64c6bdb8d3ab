#!/bin/bash
# G2 comb base chain on quad groups: G2 fixed-base tests, probe vs the previous build, kernel split
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "g2 or G2 or wnaf or fixed" > gpurun_out/g2_tests.txt 2>&1
timeout -k 10 300 python tools/g2_comb_probe.py 16384 65536 262144 > gpurun_out/g2_comb.txt 2>&1
PA_LIB_PATH=$PWD/gpuvar/head/libpairing_amd.so timeout -k 10 300 python tools/g2_comb_probe.py 16384 65536 262144 >> gpurun_out/g2_comb.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g2c -o run -- python tools/g2_comb_probe.py 65536 > gpurun_out/g2c_prof.txt 2>&1
