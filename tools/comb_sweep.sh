#!/bin/bash
# config-3 (wnaf workload) sweep over the GLV comb's window parts:
# PA_COMB_PARTS / PA_COMB_FIRST pairs given as "parts:first" arguments
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for pf in "$@"; do
    p=${pf%%:*}; f=${pf##*:}
    echo "== parts $p first $f"
    PA_COMB_PARTS=$p PA_COMB_FIRST=$f timeout -k 10 200 python bench.py --workload wnaf --steps 5 --warmup 1 \
        --no-cpu-baseline | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' || exit 1
done
