# r05: the lane-pair final exponentiation with Karabina squarings: parity, then
# lane pairs vs one lane across batch sizes (tools/coop_latency.py), the bench
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gen_units.py tests/test_gpu_parity.py tests/test_bench_sizes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lp_tests.txt 2>&1 || { tail -30 gpurun_out/lp_tests.txt; exit 1; }
tail -3 gpurun_out/lp_tests.txt
COOP_LAT_VARIANTS=1,3 timeout -k 10 300 python tools/coop_latency.py 4096 8192 16384 32768 32769 40960 49152 65536 > gpurun_out/lp_sizes.txt 2>&1 || exit 1
grep "pairing batch" gpurun_out/lp_sizes.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lp_bench.txt 2>&1 || exit 1
tail -1 gpurun_out/lp_bench.txt | cut -c1-400
