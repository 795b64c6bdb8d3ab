# r05: the per-pair prepared Miller loop (pa_gen_miller_loop_prepared) against
# the shared one (pa_gen_miller_loop_shared): SQ instruction mix, waits and the
# instruction cache, one counter set per pass
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/mlppmc
mkdir -p $O
export TMPDIR=/tmp
for w in prepared prepared_shared; do
B="bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES --output-format csv -d $O/$w/sq -o run -- python3 $B > $O/$w.sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM --output-format csv -d $O/$w/ic -o run -- python3 $B > $O/$w.ic.log 2>&1 || exit 1
done
echo done
