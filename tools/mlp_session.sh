# r05: the generated per-pair prepared Miller loop: parity, bench (against the
# hipcc kernel), kernel time and the SQ wait counters
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/mlp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_prepared_gen.py tests/test_gpu_parity.py -m gpu -k "prepared or miller" > $O/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --workload prepared > $O/bench_gen.json 2> $O/bench_gen.err && \
PA_ML_PREPARED=hipcc timeout -k 10 200 python bench.py --workload prepared > $O/bench_hipcc.json 2> $O/bench_hipcc.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload prepared --steps 10 --warmup 2 > $O/prof.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 bench.py --workload prepared --steps 3 --warmup 1 --no-cpu-baseline > $O/sq.log 2>&1
