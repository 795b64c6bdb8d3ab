# r05: what a cooperative-VM step spends its cycles on (2-pair multi_pairing, verifier shape):
# SQ instruction mix, waits and the SQC instruction cache, one counter set per pass
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/vpmc
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --workload verify --steps 5 --warmup 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS --output-format csv -d $O/ic -o run -- python3 $B > $O/ic.log 2>&1 || exit 1
echo done
