# r05: batch-size regimes after the lane-pair FE change (variant 0 thresholds)
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
COOP_LAT_VARIANTS=2,1 timeout -k 10 300 python tools/coop_latency.py 1024 1536 2048 2560 3072 4096 > gpurun_out/rg_small.txt 2>&1 || exit 1
grep "pairing batch" gpurun_out/rg_small.txt
COOP_LAT_VARIANTS=1,3 timeout -k 10 400 python tools/coop_latency.py 36864 40960 43008 45056 47104 98304 131072 > gpurun_out/rg_large.txt 2>&1 || exit 1
grep "pairing batch" gpurun_out/rg_large.txt
