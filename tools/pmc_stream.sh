#!/bin/bash
# HBM traffic of the streaming batch multiplies (config 2 and Fr): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes (a pass cannot hold both on gfx950).
#   tools/pmc_stream.sh -> gpurun_out/pmc_{fq,fr}_{fetch,write}/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in fq_mul fr_mul; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_${wl}_${c}
    echo "=== $wl $c"
    timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o run -- python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > $d.log 2>&1 || exit $?
  done
done
echo done
