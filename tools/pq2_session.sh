# r06: lane groups in the default selection: their tests, the window edges,
# the cooperative / mid-size regressions
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/pq2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pair_quad.py tests/test_gpu_parity.py tests/test_bench_sizes.py -m gpu -k "lane_group or window or coop or multi_pairing or mid_size or split_batch" > $O/tests.log 2>&1 || exit 1
COOP_LAT_VARIANTS=0 timeout -k 10 300 python tools/coop_latency.py 1024 1152 1153 1536 2048 2049 2304 > $O/regimes.txt 2>&1 || exit 1
