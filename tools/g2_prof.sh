#!/bin/bash
# G2 MSM kernel split at 2^16 and 2^18 (rocprofv3 kernel trace of tools/msm_g2_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g2 -o run -- python tools/msm_g2_probe.py ${N:-262144} > gpurun_out/g2_prof.txt 2>&1
