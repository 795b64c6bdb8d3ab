#!/bin/bash
# MSM A/B over environment configurations (CONFIGS, '|'-separated), one GPU
# session: tests/test_msm.py first (default config), then bench.py --workload msm
# per configuration; PROF=<config index> adds a rocprofv3 kernel trace of that one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
    timeout -k 10 400 python -u -m pytest tests/test_msm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/msm_tests.txt 2>&1 || exit $?
fi
IFS='|' read -ra CFG <<< "${CONFIGS:-PA_MSM_PARTS=1|PA_MSM_PARTS=2}"
i=0
for c in "${CFG[@]}"; do
    env $c timeout -k 10 300 python bench.py --workload msm --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/msm_ab_$i.txt 2>&1 || exit $?
    echo "[$c] $(tail -1 gpurun_out/msm_ab_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M terms/s", round(d["ms_per_step"],3), "ms")')" >> gpurun_out/msm_ab.txt
    i=$((i+1))
done
if [ -n "$PROF" ]; then
    env ${CFG[$PROF]} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_msm_ab -o run -- python bench.py --workload msm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/msm_prof.txt 2>&1
fi
