cd "${GRAFT_REPO_ROOT}"
run() { echo "== $*"; env "$@" timeout -k 10 120 python bench.py --workload fq_mul --steps 50 --warmup 5 --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('avg %.2f us  frac %.3f' % (r['avg_launch_ms']*1e3, r['frac']))"; }
for l in 0 27000 32000 40000 54000 80000 0; do run PA_FQ_VARIANT=4 PA_FQ_LDS=$l || exit 1; done
