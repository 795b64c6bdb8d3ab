#!/bin/bash
# A/B of the streaming batch-multiply launch shapes (PA_STREAM_BLOCKS / PA_STREAM_PREFETCH):
#   tools/stream_ab.sh  -> gpurun_out/stream_ab.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/stream_ab.txt
: > $out
for wl in fq_mul fr_mul; do
  for cfg in "0 2048" "1 1024" "1 2048" "1 4096" "0 4096"; do
    set -- $cfg
    echo "=== $wl prefetch=$1 blocks=$2" >> $out
    PA_STREAM_PREFETCH=$1 PA_STREAM_BLOCKS=$2 timeout -k 10 120 python bench.py --workload $wl --steps 200 --warmup 10 --no-cpu-baseline >> $out 2>&1 || exit $?
  done
done
grep -o '"value": [0-9.e+]*\|===.*\|"avg_launch_ms": [0-9.]*' $out
