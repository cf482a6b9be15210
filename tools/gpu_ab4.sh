# GPU box: FC_small kernel A/B of the libraries in $AB_LIBS against the working tree, then a kernel trace of the
# sampling workload (where its step time goes beyond k_inverse_mfma). bash tools/gpu_ab4.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03i}
for i in 1 2; do
  timeout -k 10 120 python tools/abk.py
  for lib in $AB_LIBS; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/abk.py; done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab_kernels.txt
if [ -n "$TRACE_SAMPLE" ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_sample_trace -o sample -- python3 $R/bench.py --workload sample --steps 5 --warmup 2 > $R/gpurun_out/${T}_sample_bench.json 2> $R/gpurun_out/${T}_sample_bench.err
  find $R/gpurun_out/${T}_sample_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/${T}_sample_kernel_stats.csv
  head -30 $R/gpurun_out/${T}_sample_kernel_stats.csv
fi
