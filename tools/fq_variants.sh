#!/bin/bash
# A/B of the config-2 kernel variants (PA_FQ_VARIANT, kernels_field.hip:
# 0 12 x u32 streaming kernel; 4 lazy 28-bit core (default);
# 9 the record traffic alone, no multiply)
# plus parity of each product variant at 2^20
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
run() {
  echo "== $*"
  env "$@" timeout -k 10 120 python bench.py --workload fq_mul --steps 50 --warmup 5 --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('avg %.2f us  %.0f GB/s  frac %.3f  copy %.0f GB/s' % (r['avg_launch_ms']*1e3, r['achieved'], r['frac'], r['copy_GBs']))"
}
for v in ${FQ_VARIANTS:-4 9 4 9}; do run PA_FQ_VARIANT=$v || exit 1; done
for v in ${FQ_PARITY:-4}; do
  PA_FQ_VARIANT=$v timeout -k 10 200 python -m pytest -q tests/test_bench_sizes.py -k fq_mul --timeout 150 2>&1 | tail -1
done
