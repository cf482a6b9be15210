# GPU box: FC_small training / fold / parity GPU tests, then same-box A/B of the headline step (working tree vs
# build_exp/libhead.so): bench.py without sub-lines, twice each
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fold.py tests/test_gpu_parity.py tests/test_gpu_dp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_step_tests.log 2>&1 || { tail -40 gpurun_out/${T}_step_tests.log; exit 1; }
tail -1 gpurun_out/${T}_step_tests.log
for r in 1 2; do
  for lib in default ${AB_LIBS:-build_exp/libhead.so}; do
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/ab_s.json 2>/dev/null
    else
      BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline > gpurun_out/ab_s.json 2>/dev/null
    fi
    python -c "import json; d=json.loads(open('gpurun_out/ab_s.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']/1e6, 2), 'M samples/s', d['kernels_us'])"
  done
done 2>&1 | tee gpurun_out/${T}_ab_step.txt
