# r06 (round-5 verdict item 2): does workspace traffic cost clock under the
# power cap?  The lane-pair final exponentiation as built (lib/) against a
# variant whose Karabina state lives in the workspace instead of AGPRs
# (gpuvar/fe2kc: PGEN_KC_HOME=M, every compressed squaring reads and writes
# it): time, HBM bytes (FETCH_SIZE / WRITE_SIZE passes) and the shader clock
# (GRBM_GUI_ACTIVE per dispatch) for each
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/tab
mkdir -p $O
export TMPDIR=/tmp
for v in lib fe2kc; do
  if [ $v = lib ]; then D=$PWD/pairing_amd/lib; else D=$PWD/gpuvar/$v; fi
  for r in 1 2; do
    PA_GEN_DIR=$D timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/err_${v}_$r.txt || exit 1
  done
  PA_GEN_DIR=$D timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${v}_fetch -o run -- python tools/pair_pmc.py 65536 1 2 > $O/${v}_fetch.txt 2>&1 || exit 1
  PA_GEN_DIR=$D timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${v}_write -o run -- python tools/pair_pmc.py 65536 1 2 > $O/${v}_write.txt 2>&1 || exit 1
  PA_GEN_DIR=$D timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/${v}_clk -o run -- python tools/pair_pmc.py 65536 1 2 > $O/${v}_clk.txt 2>&1 || exit 1
  PA_GEN_DIR=$D timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_kt -o run -- python tools/pair_pmc.py 65536 1 2 > $O/${v}_kt.txt 2>&1 || exit 1
done
