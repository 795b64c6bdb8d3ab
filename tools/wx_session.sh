# r06: the bit-exact Wnaf multiply on the lazy core: parity, then the exact
# path's time (bench --workload wnaf "separately: bit-exact wnaf") against the
# round-5 12-word multiply (PA_WX_MUL=word12), and its per-kernel split
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/wx
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_wnaf_exact.py tests/test_fq_repr.py -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload wnaf --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_fl.json 2> $O/err_fl.txt || exit 1
PA_WX_SORT=0 timeout -k 10 300 python bench.py --workload wnaf --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_r2.json 2> $O/err_r2.txt || exit 1
PA_WX_MUL=word12 timeout -k 10 300 python bench.py --workload wnaf --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_w12.json 2> $O/err_w12.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload wnaf --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
