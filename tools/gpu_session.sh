#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; a fault,
# abort, segfault or timeout ends the session (no further GPU work), a plain
# test failure (exit 1) does not.  Usage: tools/gpu_session.sh STEP...
#   steps: valu | tests | smoke | bench | prof | pmc | fqbench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
    local name=$1 limit=$2
    shift 2
    echo "=== $name: $*" | tee -a gpurun_out/session.log
    local t0=$(date +%s)
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a gpurun_out/session.log
    tail -5 "gpurun_out/$name.txt"
    case $rc in
        0|1) return 0 ;;
        *) echo "=== stopping after $name (rc=$rc)" | tee -a gpurun_out/session.log; exit $rc ;;
    esac
}
for step in "$@"; do
    case $step in
        valu) run valu 120 ./tools/valu_rates ;;
        valupeak) run valu_peak 120 ./tools/valu_peak ;;
        issue) run issue_probe 120 ./tools/issue_probe ;;
        hostrate) run host_rate1 300 python tools/pcie_rate.py &&
                  run host_rate2 300 env PA_PIPELINE_PIECES=2 python tools/pcie_rate.py &&
                  run host_rate4 300 env PA_PIPELINE_PIECES=4 python tools/pcie_rate.py &&
                  run host_trace 300 env PA_PIPELINE_TRACE=1 python tools/pcie_rate.py ;;
        tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
        alltests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
        unittests) run pytest_units 300 python -u -m pytest tests/test_gen_units.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        sizetests) run pytest_sizes 600 python -u -m pytest tests/test_bench_sizes.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ;;
        benchnc) run bench_nc 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        verifybench) run bench_verify 300 python bench.py --workload verify --steps 10 --warmup 2 --no-cpu-baseline ;;
        fqsoa) run bench_fq_soa 300 python bench.py --workload fq_mul --layout soa --steps 20 --warmup 3 --no-cpu-baseline ;;
        proffqsoa) run prof_fq_soa 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fq_soa -o run -- python bench.py --workload fq_mul --layout soa --steps 10 --warmup 2 --no-cpu-baseline ;;
        soatests) run pytest_soa 300 python -u -m pytest tests/test_bench_sizes.py -m gpu -k "soa or fq_mul" -v --timeout 120 --timeout-method thread ;;
        rcclbench) run bench_rccl1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline ;;
        benchgen2) run bench_gen2 600 env PA_PAIRING_KERNEL=1 python bench.py --no-cpu-baseline ;;
        wnafbench) run bench_wnaf 300 python bench.py --workload wnaf --steps 5 --warmup 1 ;;
        decbench) run bench_decode 300 python bench.py --workload decode --steps 5 --warmup 1 ;;
        newtests) run pytest_new 600 python -u -m pytest tests/test_fr.py tests/test_msm.py -m gpu -v --timeout 300 --timeout-method thread ;;
        frbench) run bench_fr 300 python bench.py --workload fr_mul --steps 20 --warmup 3 ;;
        msmtests) run pytest_msm 600 python -u -m pytest tests/test_msm.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        msmbench) run bench_msm 400 python bench.py --workload msm --steps 5 --warmup 1 ;;
        profmsm) run prof_msm 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_msm -o run -- python bench.py --workload msm --steps 3 --warmup 1 --no-cpu-baseline ;;
        profwnaf) run prof_wnaf 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wnaf -o run -- python bench.py --workload wnaf --steps 3 --warmup 1 --no-cpu-baseline ;;
        profdec) run prof_dec 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec -o run -- python bench.py --workload decode --steps 3 --warmup 1 --no-cpu-baseline ;;
        fqbench) run bench_fq 300 python bench.py --workload fq_mul --steps 20 --warmup 3 --no-cpu-baseline ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        frbench_nc) run bench_fr 300 python bench.py --workload fr_mul --steps 20 --warmup 3 --no-cpu-baseline ;;
        proffq) run prof_fq 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fq -o run -- python bench.py --workload fq_mul --steps 10 --warmup 2 --no-cpu-baseline ;;
        pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline &&
             run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
        pmccsv) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline &&
                run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
        pmcsq) run pmc_sq1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES -d gpurun_out/pmc_sq1 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline &&
               run pmc_sq2 600 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR -d gpurun_out/pmc_sq2 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
        pmcsq4) run pmc4_sq1 300 env PA_PAIRING_KERNEL=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES -d gpurun_out/pmc4_sq1 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline &&
                run pmc4_sq2 300 env PA_PAIRING_KERNEL=1 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR -d gpurun_out/pmc4_sq2 -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
        pmcdec) run pmc_dec 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_dec -o run -- python bench.py --workload decode --steps 2 --warmup 1 --no-cpu-baseline ;;
        pmcmsm) run pmc_msm 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_msm -o run -- python bench.py --workload msm --steps 2 --warmup 1 --no-cpu-baseline &&
                run pmc_msm_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_msm_fetch -o run -- python bench.py --workload msm --steps 2 --warmup 1 --no-cpu-baseline &&
                run pmc_msm_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_msm_write -o run -- python bench.py --workload msm --steps 2 --warmup 1 --no-cpu-baseline ;;
        cooptests) run pytest_coop 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_sizes.py -m gpu -k "coop or multi_pairing" -x -v --timeout 200 --timeout-method thread ;;
        coopprof) run coop_prof 120 ./tools/coop_prof ;;
        quadtests) run pytest_quad 300 python -u -m pytest tests/test_coop_quad.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        hextests) run pytest_hex 300 python -u -m pytest tests/test_coop_quad.py -m gpu -v --timeout 120 --timeout-method thread ;;
        hexlat) run hex_latency 120 python tools/hex_latency.py 2000 ;;
        cooplat_small) run coop_latency 300 python tools/coop_latency.py 1 2 16 64 256 1024 2048 ;;
        cooplat) run coop_latency 300 python tools/coop_latency.py ;;
        distwl) for w in fq_mul fr_mul wnaf decode msm; do
                    run dist1_$w 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline || exit 1
                done
                run dist1_msm_global 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29514 bench.py --workload msm --global-batch 1000003 --steps 3 --warmup 1 --no-cpu-baseline ;;
        profverify) run prof_verify 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_verify -o run -- python bench.py --workload verify --steps 10 --warmup 2 --no-cpu-baseline ;;
        profprep) run prof_prep 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_prep -o run -- python bench.py --workload prepared --steps 3 --warmup 1 --no-cpu-baseline ;;
        prepbench) run bench_prepared 400 python bench.py --workload prepared --steps 5 --warmup 1 ;;
        preptests) run pytest_prep 600 python -u -m pytest tests/test_bench_sizes.py tests/test_gpu_parity.py -m gpu -k "prepare or miller_loop" -x -v --timeout 300 --timeout-method thread ;;
        verifycpu) run bench_verify_cpu 300 python bench.py --workload verify --steps 10 --warmup 2 ;;
        allbench) run bench 600 python bench.py &&
                  run bench_prepared 300 python bench.py --workload prepared --steps 20 --warmup 5 &&
                  run bench_prepared_shared 300 python bench.py --workload prepared_shared --steps 20 --warmup 5 &&
                  run bench_verify_cpu 300 python bench.py --workload verify --steps 10 --warmup 2 &&
                  run bench_verify_decode 300 python bench.py --workload verify --decode --steps 10 --warmup 2 &&
                  run bench_decode 300 python bench.py --workload decode --steps 5 --warmup 1 &&
                  run bench_msm 400 python bench.py --workload msm --steps 5 --warmup 1 &&
                  run bench_wnaf 300 python bench.py --workload wnaf --steps 5 --warmup 1 &&
                  run bench_fq 300 python bench.py --workload fq_mul --steps 20 --warmup 3 &&
                  run bench_fr 300 python bench.py --workload fr_mul --steps 20 --warmup 3 ;;
        sharedtests) run pytest_shared 600 python -u -m pytest tests/test_shared_prepared.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        sharedbench) run bench_shared 300 python bench.py --workload prepared_shared --steps 10 --warmup 2 --no-cpu-baseline ;;
        sharedbenchcpu) run bench_shared_cpu 400 python bench.py --workload prepared_shared --steps 10 --warmup 2 ;;
        profshared) run prof_shared 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_shared -o run -- python bench.py --workload prepared_shared --steps 5 --warmup 1 --no-cpu-baseline ;;
        pmcpair)  # r05: counters of lane-pair vs one-lane kernels and the leaf probe
            P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
            P2="SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
            P3="MeanOccupancyPerCU SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32"
            P4="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE InstrFetchLatency"
            for cfg in "1 65536" "1 32768" "3 65536" "3 32768"; do
                set -- $cfg
                run pair_time_v$1_n$2 120 python tools/pair_pmc.py $2 $1 2 || exit 1
                for k in 1 2 3 4; do
                    eval "ctrs=\$P$k"
                    run pmcpair_v$1_n$2_p$k 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmcpair/v$1_n$2_p$k -o run -- python tools/pair_pmc.py $2 $1 1 || exit 1
                done
            done
            for k in 1 2 3 4; do
                eval "ctrs=\$P$k"
                run pmcprobe_p$k 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmcpair/probe_p$k -o run -- ./tools/icache_probe || exit 1
            done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
