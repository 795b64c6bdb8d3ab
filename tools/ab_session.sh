# A/B of generated code objects in one session (same box, alternating runs):
# PA_GEN_DIR=gpuvar/$1 against the in-tree build, pairing batch 2^16 on lane pairs
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  timeout -k 10 120 python tools/pair_pmc.py 65536 1 4 > gpurun_out/ab/new_$r.txt 2>&1 || exit 1
  PA_GEN_DIR=gpuvar/$1 timeout -k 10 120 python tools/pair_pmc.py 65536 1 4 > gpurun_out/ab/$1_$r.txt 2>&1 || exit 1
done
grep -H " run " gpurun_out/ab/*.txt
