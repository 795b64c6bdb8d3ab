# r05: config 2 attribution: TA / TCP / SQ counters of
# k_fq_mul_batch_fl (default) and the no-multiply access probe (PA_FQ_VARIANT=9)
# at 2^20, one counter block per pass (rocprofv3 limits: 2 TA, 4 TCP, 8 SQ)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/fqpmc
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --workload fq_mul --steps 3 --warmup 1 --no-cpu-baseline"
for v in 4 9; do
  PA_FQ_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum --output-format csv -d $O/ta_$v -o run -- python3 $B > $O/ta_$v.log 2>&1 || exit 1
  PA_FQ_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d $O/tcp_$v -o run -- python3 $B > $O/tcp_$v.log 2>&1 || exit 1
  PA_FQ_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq_$v -o run -- python3 $B > $O/sq_$v.log 2>&1 || exit 1
  PA_FQ_VARIANT=$v timeout -k 10 90 python3 bench.py --workload fq_mul --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
done
echo done
