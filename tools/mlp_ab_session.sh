# A/B of the prepared Miller loop code object: PA_GEN_DIR=gpuvar/<v> for each
# variant named, against the in-tree build (kernel time from rocprofv3 --stats;
# timing only)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/mlpab
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o run -- python3 bench.py --workload prepared --steps 6 --warmup 2 --no-cpu-baseline > $O/base.log 2>&1 || exit 1
for v in "$@"; do
  PA_GEN_DIR=gpuvar/$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --workload prepared --steps 6 --warmup 2 --no-cpu-baseline > $O/$v.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base2 -o run -- python3 bench.py --workload prepared --steps 6 --warmup 2 --no-cpu-baseline > $O/base2.log 2>&1 || exit 1
grep -H miller_loop_prepared $O/*/run_kernel_stats.csv
