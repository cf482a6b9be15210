set -e
mkdir -p gpurun_out
for v in old new old new; do BCNF_AMD_LIB=build_exp/lib$v.so timeout -k 10 200 python bench.py --workload sample --no-cpu-baseline > gpurun_out/s_$v.json 2>&1; echo $v $(tail -1 gpurun_out/s_$v.json | cut -c100-200); done
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_sampling.py tests/test_calibration.py tests/test_gpu_fold.py > gpurun_out/t6.log 2>&1 || { tail -40 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
