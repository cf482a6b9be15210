# GPU box: the full GPU suite, then the default bench line (each step under its own limit, chained).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03}
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'], {k: (v.get('value'), v.get('roofline', {}).get('frac')) for k, v in d['secondary'].items()})"
