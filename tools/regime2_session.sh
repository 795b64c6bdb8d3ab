# r05 (after the pairing-only lane-pair Miller loop): lane pairs (1) vs one lane (3)
# in and around the one-lane regime (32768, 38912]
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
COOP_LAT_VARIANTS=1,3 timeout -k 10 400 python tools/coop_latency.py ${RG_SIZES:-30000 32769 34816 36864 38912 40960} > gpurun_out/rg2.txt 2>&1 || exit 1
grep "pairing batch" gpurun_out/rg2.txt
