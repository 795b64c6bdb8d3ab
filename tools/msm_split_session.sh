# r05: MSM window-part splits (PA_MSM_WLO: descending lower window bounds of the parts)
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/msmsplit
mkdir -p $O
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --workload msm --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -o '"value": [0-9.e+]*' $O/$n.log)"
}
for r in 1 2; do
  run p2_even_$r PA_MSM_PARTS=2
  run p2_w6_$r PA_MSM_PARTS=2 PA_MSM_WLO=6
  run p2_w4_$r PA_MSM_PARTS=2 PA_MSM_WLO=4
  run p2_w10_$r PA_MSM_PARTS=2 PA_MSM_WLO=10
  run p3_w8_3_$r PA_MSM_PARTS=3 PA_MSM_WLO=9,3
  run p3_w11_4_$r PA_MSM_PARTS=3 PA_MSM_WLO=11,4
done
