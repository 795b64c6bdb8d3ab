cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
set -o pipefail
for n in 65536 32768 40000; do
  timeout -k 10 120 python tools/pair_pmc.py $n 1 3 > gpurun_out/prio_default_$n.txt 2>&1 || exit $?
  PA_GEN_DIR=gpuvar/prio2 timeout -k 10 120 python tools/pair_pmc.py $n 1 3 > gpurun_out/prio_toggle_$n.txt 2>&1 || exit $?
done
PA_GEN_DIR=gpuvar/prio2 timeout -k 10 120 rocprofv3 --pmc MeanOccupancyPerCU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmcprio -o run -- python tools/pair_pmc.py 65536 1 1 > gpurun_out/pmcprio.txt 2>&1 || exit $?
grep -h variant gpurun_out/prio_*.txt
