# r06: batches just above PA_PAIR_MAX split into a lane-pair head and a
# cooperative tail on a forked stream: parity at the regime edges, then the
# default selection's curve (forked tail, serial tail, no split)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/tail
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_sizes.py -m gpu -k "mid_size or split_batch or two_streams" > $O/tests.log 2>&1 || exit 1
S="${RG_SIZES:-32768 32769 33024 33792 34048 34816 35072}"
COOP_LAT_VARIANTS=0 timeout -k 10 400 python tools/coop_latency.py $S > $O/regimes_fork.txt 2>&1 || exit 1
PA_TAIL_SERIAL=1 COOP_LAT_VARIANTS=0 timeout -k 10 400 python tools/coop_latency.py $S > $O/regimes_serial.txt 2>&1 || exit 1
PA_TAIL_MAX=0 COOP_LAT_VARIANTS=0 timeout -k 10 400 python tools/coop_latency.py $S > $O/regimes_nosplit.txt 2>&1 || exit 1
