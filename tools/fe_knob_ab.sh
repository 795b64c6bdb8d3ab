#!/bin/bash
# FE emitter-knob A/B: bench.py with PA_GEN_DIR=gpuvar/<variant> (code objects
# built by tools/pgen/build_gen.py --outdir under PGEN_* settings), default first and last
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in default ${VARIANTS}; do
    if [ "$v" = default ]; then unset PA_GEN_DIR; else export PA_GEN_DIR=$PWD/gpuvar/$v; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fe_ab_$v.txt 2>&1
    echo "$v $(grep '^{' gpurun_out/fe_ab_$v.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["config"]["kernel_ms"])')" >> gpurun_out/fe_ab.txt
done
unset PA_GEN_DIR
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fe_ab_default2.txt 2>&1
echo "default2 $(grep '^{' gpurun_out/fe_ab_default2.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["config"]["kernel_ms"])')" >> gpurun_out/fe_ab.txt
