# r05: lane-pair Miller-loop homes A/B (f in LDS vs AGPR-first homes that fall to the workspace)
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/ml2h
for r in 1 2; do
  timeout -k 10 120 python tools/pair_pmc.py 65536 1 3 > gpurun_out/ml2h/new_$r.txt 2>&1 || exit 1
  PA_GEN_DIR=gpuvar/ml2old timeout -k 10 120 python tools/pair_pmc.py 65536 1 3 > gpurun_out/ml2h/old_$r.txt 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ml2h/fetch -o run -- python tools/pair_pmc.py 65536 1 1 > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ml2h/write -o run -- python tools/pair_pmc.py 65536 1 1 > /dev/null 2>&1 || exit 1
grep -H run gpurun_out/ml2h/*.txt
