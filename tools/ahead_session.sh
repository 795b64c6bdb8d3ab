# r06: workspace reload distance (PGEN_AHEAD_M) of the lane-pair kernels, A/B
# against the built kernels, alternating, one box
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/ahead
mkdir -p $O
for r in 1 2; do
  for v in lib ahead250 ahead1000 ahead2000; do
    if [ $v = lib ]; then D=$PWD/pairing_amd/lib; else D=$PWD/gpuvar/$v; fi
    PA_GEN_DIR=$D timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/err_${v}_$r.txt || exit 1
  done
done
