# r06: the verifier from compressed points with the subgroup checks beside the
# pairing (pa_g{1,2}_subgroup_check_batch_device): parity, then the verify
# bench with the split and without it (checked decodes, then the pairing)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/vsplit
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_decode.py tests/test_cpp_mirror.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --workload verify --decode --steps 20 --warmup 3 --no-cpu-baseline > $O/split_$r.json 2> $O/err_split_$r.txt || exit 1
  PA_VERIFY_SPLIT=0 timeout -k 10 200 python bench.py --workload verify --decode --steps 20 --warmup 3 --no-cpu-baseline > $O/serial_$r.json 2> $O/err_serial_$r.txt || exit 1
done
timeout -k 10 200 python bench.py --workload verify --steps 20 --warmup 3 --no-cpu-baseline > $O/verify_only.json 2> $O/err_vo.txt || exit 1
