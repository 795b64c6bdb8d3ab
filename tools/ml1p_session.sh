# r06: the one-lane pairing-only Miller loop (pa_gen_miller_loop1p) in the
# one-lane window: pairing parity (default selection and variant 3), then
# lane pairs (1) vs one lane (3) around the window
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/ml1p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_sizes.py tests/test_gpu_parity.py -m gpu -k "pairing" > $O/tests.log 2>&1 || exit 1
COOP_LAT_VARIANTS=1,3 timeout -k 10 500 python tools/coop_latency.py ${RG_SIZES:-32769 34048 34816 35840 36864 37888 38912} > $O/regimes.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/err.txt || exit 1
