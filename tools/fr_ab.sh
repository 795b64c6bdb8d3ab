#!/bin/bash
# Fr batch multiply A/B over environment configurations (CONFIGS, '|'-separated)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
IFS='|' read -ra CFG <<< "${CONFIGS:-PA_FR_LDS=0}"
i=0
for c in "${CFG[@]}"; do
    env $c timeout -k 10 300 python bench.py --workload ${WL:-fr_mul} --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${WL:-fr_mul}_ab_$i.txt 2>&1 || exit $?
    echo "[$c] $(tail -1 gpurun_out/${WL:-fr_mul}_ab_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(r["avg_launch_ms"]*1e3,2), "us", round(r["achieved"]), "GB/s frac", round(r["frac"],3))')" >> gpurun_out/${WL:-fr_mul}_ab.txt
    i=$((i+1))
done
