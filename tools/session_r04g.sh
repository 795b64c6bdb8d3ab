#!/bin/bash
# G2 MSM segment default: MSM tests, G2 probe, headline bench twice
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/msm_tests.txt 2>&1
timeout -k 10 300 python tools/msm_g2_probe.py 65536 262144 > gpurun_out/g2_probe.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_a.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_b.txt 2>&1
