# r06: the split batch's tail on the lane-group kernels (PA_TAIL_KIND=pq)
# against the cooperative tail, tails up to 4096
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/tail2
mkdir -p $O
export TMPDIR=/tmp
PA_TAIL_KIND=pq PA_TAIL_MAX=4096 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_sizes.py -m gpu -k "split_batch" > $O/tests.log 2>&1 || exit 1
S="32769 33792 34048 34816 35840 36864"
PA_TAIL_KIND=pq PA_TAIL_MAX=4096 COOP_LAT_VARIANTS=0 timeout -k 10 400 python tools/coop_latency.py $S > $O/regimes_pq.txt 2>&1 || exit 1
PA_TAIL_MAX=4096 COOP_LAT_VARIANTS=0 timeout -k 10 400 python tools/coop_latency.py $S > $O/regimes_coop.txt 2>&1 || exit 1
