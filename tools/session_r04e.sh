#!/bin/bash
# G2 comb on the lazy core: parity tests touching G2 fixed base, probe vs the previous build; NT stream A/B
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "g2 or G2 or wnaf or fixed" > gpurun_out/g2_tests.txt 2>&1
timeout -k 10 300 python tools/g2_comb_probe.py 16384 65536 262144 > gpurun_out/g2_comb.txt 2>&1
PA_LIB_PATH=$PWD/gpuvar/head/libpairing_amd.so timeout -k 10 300 python tools/g2_comb_probe.py 16384 65536 262144 >> gpurun_out/g2_comb.txt 2>&1
CONFIGS="PA_FR_NT=0|PA_FR_NT=1|PA_FR_NT=0|PA_FR_NT=1" bash tools/fr_ab.sh
WL=fq_mul CONFIGS="PA_FQ_VARIANT=4|PA_FQ_VARIANT=7|PA_FQ_VARIANT=4|PA_FQ_VARIANT=7|PA_FQ_VARIANT=7 PA_FQ_LDS=0" bash tools/fr_ab.sh
