#!/bin/bash
# Round-4 GPU session: MSM tests (G2 on the lazy core), the G2 MSM probe
# (lazy vs 12-word), Fr and Fq batch-multiply A/B, PMC traffic + kernel stats.
# Every step under its own limit; the first failure ends the session.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/msm_tests.txt 2>&1
PA_MSM_G2_LAZY=1 timeout -k 10 300 python tools/msm_g2_probe.py 65536 262144 > gpurun_out/g2_probe.txt 2>&1
PA_MSM_G2_LAZY=0 timeout -k 10 300 python tools/msm_g2_probe.py 65536 262144 >> gpurun_out/g2_probe.txt 2>&1
CONFIGS="PA_FR_LDS=0|PA_FR_LDS=12000|PA_FR_LDS=16000|PA_FR_LDS=20000|PA_FR_LDS=27000|PA_FR_LDS=40000|PA_FR_LDS=0" bash tools/fr_ab.sh
WL=fq_mul CONFIGS="PA_FQ_VARIANT=4|PA_FQ_VARIANT=6 PA_STREAM_BLOCKS=2048|PA_FQ_VARIANT=6 PA_STREAM_BLOCKS=1024|PA_FQ_VARIANT=6 PA_STREAM_BLOCKS=512|PA_FQ_VARIANT=6 PA_STREAM_BLOCKS=1024 PA_FQ_LDS=16000|PA_FQ_VARIANT=6 PA_STREAM_BLOCKS=2048 PA_FQ_LDS=27000|PA_FQ_VARIANT=4" bash tools/fr_ab.sh
bash tools/gpu_session.sh pmccsv prof
