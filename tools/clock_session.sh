# r05: shader clock during the pairing kernels at one and two waves per SIMD
# (GRBM_GUI_ACTIVE / GRBM_COUNT per dispatch against its duration)
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/clk
for cfg in "1 32768" "1 65536" "3 65536" "3 32768"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/clk/v$1_n$2 -o run -- python tools/pair_pmc.py $2 $1 2 > gpurun_out/clk/v$1_n$2.txt 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/clk/probe -o run -- ./tools/icache_probe > gpurun_out/clk/probe.txt 2>&1 || exit $?
echo done
