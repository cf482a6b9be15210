# GPU box: training tests of the working tree, then the FC_small kernel A/B against the libraries in
# $AB_LIBS (default build_exp/libhead.so = the last commit). Each GPU step has its own limit; the chain stops at the
# first failure.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03e}
TESTS=${TESTS:-tests/test_gpu_train.py}
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
AB_LIBS=${AB_LIBS:-build_exp/libhead.so}
for i in 1 2; do
  timeout -k 10 120 python tools/abk.py
  for lib in $AB_LIBS; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/abk.py; done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab_kernels.txt
