# r06: mul2's operand pair by a DPP broadcast + fused negate/DPP select
# (PGEN_PAIR_DPP): pairing parity, then the headline bench against the
# round-5 pair formation (gpuvar/nodpp, PA_GEN_DIR), alternating
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/pairdpp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_sizes.py tests/test_gpu_parity.py tests/test_gen_units.py -m gpu -k "pairing or final_exp or miller or karabina or unit" > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_new_$r.json 2> $O/err_new_$r.txt || exit 1
  PA_GEN_DIR=$PWD/gpuvar/nodpp timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_old_$r.json 2> $O/err_old_$r.txt || exit 1
done
