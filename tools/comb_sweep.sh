#!/bin/bash
# config-3 (wnaf workload) sweep over the GLV comb's window parts:
# each argument is a PA_COMB_SPLIT value (first window of every part after
# the first, e.g. 5 or 2,7)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for sp in "$@"; do
    echo "== split $sp"
    PA_COMB_SPLIT=$sp timeout -k 10 200 python bench.py --workload wnaf --steps 5 --warmup 1 \
        --no-cpu-baseline | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' || exit 1
done
