#!/bin/bash
# A/B of config-3 builds (gpuvar/curve_TAG/libpairing_amd.so, made from the
# same sources with -D switches of kernels_curve.hip): bench line + GLV parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for t in "$@"; do
    echo "== $t"
    lib=$PWD/gpuvar/curve_$t/libpairing_amd.so
    PA_LIB_PATH=$lib timeout -k 10 200 python bench.py --workload wnaf --steps 10 --warmup 2 --no-cpu-baseline \
        | grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}' || exit 1
    PA_LIB_PATH=$lib timeout -k 10 200 python -m pytest -q tests/test_gpu_parity.py -m gpu -k glv --timeout 150 2>&1 | tail -1
done
