#!/bin/bash
# A/B of the config-2 kernel (PA_FQ_VARIANT=0: 12 x u32 streaming kernel;
# default: lazy 28-bit core, kernels_field.hip) plus parity at 2^20
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
run() {
  echo "== $*"
  env "$@" timeout -k 10 120 python bench.py --workload fq_mul --steps 50 --warmup 5 --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('avg %.2f us  %.0f GB/s  frac %.3f  copy %.0f GB/s' % (r['avg_launch_ms']*1e3, r['achieved'], r['frac'], r['copy_GBs']))"
}
run PA_FQ_VARIANT=0 && run PA_FQ_VARIANT=4 && run PA_FQ_VARIANT=0 && run PA_FQ_VARIANT=4 || exit 1
timeout -k 10 200 python -m pytest -q tests/test_bench_sizes.py -k fq_mul --timeout 150 2>&1 | tail -1
