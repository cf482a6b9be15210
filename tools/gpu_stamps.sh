# GPU box: per-phase cycles (workgroup 0) of the diagnostic builds named in $LIBS (tools/kbench.py prints kernel
# times and the phase stamps). bash tools/gpu_stamps.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03g}
for lib in ${LIBS:-build_exp/libstamps.so}; do
  echo "== $lib"
  BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/kbench.py --iters 20
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_stamps.txt
