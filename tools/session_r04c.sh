#!/bin/bash
# MSM tests (long-bucket fix, G2 lazy), the G2 probe lazy vs 12-word, G1 bench
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_msm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/msm_tests.txt 2>&1
PA_MSM_G2_LAZY=1 timeout -k 10 300 python tools/msm_g2_probe.py 65536 262144 > gpurun_out/g2_probe.txt 2>&1
PA_MSM_G2_LAZY=0 timeout -k 10 300 python tools/msm_g2_probe.py 65536 262144 >> gpurun_out/g2_probe.txt 2>&1
NOTEST=1 CONFIGS="PA_MSM_PARTS=2|PA_MSM_PARTS=1" bash tools/msm_ab.sh
