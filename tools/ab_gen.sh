cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_def.txt 2>&1 &&
PA_GEN_DIR=$PWD/gpuvar/ko1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_ko1.txt 2>&1 &&
PA_GEN_DIR=$PWD/gpuvar/ko1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pairing" > gpurun_out/ab_ko1_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_def2.txt 2>&1
echo rc=$?
