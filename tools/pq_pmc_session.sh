# r06: counters of the lane-group kernels (one round, 2048 pairings)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/pqpmc
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/p1 -o run -- python tools/pair_pmc.py 2048 5 2 > $O/p1.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/p2 -o run -- python tools/pair_pmc.py 2048 5 2 > $O/p2.txt 2>&1 || exit 1
