# r06: the lane-group pairing kernels (pa_set_pairing_kernel(5)): parity, then
# batch-size latency against the default selection
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/pq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pair_quad.py -m gpu > $O/tests.log 2>&1 || exit 1
COOP_LAT_VARIANTS=5,0 timeout -k 10 600 python tools/coop_latency.py ${PQ_SIZES:-1 64 512 2048 4096 8192 16384} > $O/regimes.txt 2>&1 || exit 1
