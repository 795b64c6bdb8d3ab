cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for cfg in "X=1" "ROC_ENABLE_LARGE_BAR=0" "GPU_FORCE_BLIT_COPY_SIZE=0" ; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python tools/pcie_rate.py 2>&1 | grep -v amdgpu.ids || exit 1
done
export ROC_ENABLE_LARGE_BAR=0
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pcie_prof3 -o run -- python tools/pcie_rate.py > /dev/null 2>&1
python tools/timeline_gaps.py $(find gpurun_out/pcie_prof3 -name "*.db" | head -1) --last 16
