#!/bin/bash
# MSM: adaptive chunk; G2 probe over segment lengths; MSM tests; G1 bench
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/msm_tests.txt 2>&1
for seg in 8 4 2; do
    PA_MSM_SEG=$seg timeout -k 10 300 python tools/msm_g2_probe.py 65536 262144 | sed "s/^/seg $seg: /" >> gpurun_out/g2_probe.txt 2>&1
done
NOTEST=1 CONFIGS="PA_MSM_PARTS=2|PA_MSM_PARTS=2 PA_MSM_SEG=4" bash tools/msm_ab.sh
