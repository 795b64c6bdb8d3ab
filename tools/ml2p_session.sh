# r05: the pairing-only lane-pair Miller loop: parity, then bench / kernel time
# against PA_PAIRING_ML=ref (the reference-scaled pa_gen_miller_loop2)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/ml2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_sizes.py tests/test_gpu_parity.py -m gpu -k "pairing" > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_new_$r.json 2> $O/err_new_$r.txt || exit 1
  PA_PAIRING_ML=ref timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_ref_$r.json 2> $O/err_ref_$r.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
