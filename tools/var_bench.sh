#!/bin/bash
# A/B timing of generated kernel variants: tools/var_bench.sh NAME... (gpuvar/NAME)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
    echo "=== $v"
    PA_GEN_DIR=$PWD/gpuvar/$v PA_GEN_WS_SLOTS=160 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 \
        > gpurun_out/var_$v.txt 2>&1 || exit $?
    grep -o '"kernel_ms": {[^}]*}' gpurun_out/var_$v.txt
done
