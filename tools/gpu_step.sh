set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py -k "t176x176w11 or gemm_layouts or auto" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 300 python bench.py --workload fc_large --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fcl.json 2>&1
tail -1 gpurun_out/fcl.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['kernels_us'])"
