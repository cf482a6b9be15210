# GPU box: re-simulation tests + the resimulate bench line + its kernel trace
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r03}
timeout -k 10 180 python -u -m pytest tests/test_resim.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_resim_tests.log 2>&1 || { tail -40 gpurun_out/${T}_resim_tests.log; exit 1; }
tail -1 gpurun_out/${T}_resim_tests.log
timeout -k 10 300 python bench.py --workload resimulate --steps 5 --warmup 2 > gpurun_out/${T}_resim_bench.json
python -c "import json; d=json.load(open('gpurun_out/${T}_resim_bench.json')); print(d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_resim_prof -o resim -- python bench.py --workload resimulate --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_resim_prof.log 2>&1
find gpurun_out/${T}_resim_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_resim_kernel_stats.csv \;
head -4 gpurun_out/${T}_resim_kernel_stats.csv | cut -c1-200
# FC_large kernel trace for the inter-kernel gap analysis (tools/gaps.py)
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_fcl_prof -o fcl -- python bench.py --workload fc_large --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_fcl_prof.log 2>&1
python tools/gaps.py $(find gpurun_out/${T}_fcl_prof -name "*results.db" | head -1) 30 > gpurun_out/${T}_fcl_gaps.txt
head -25 gpurun_out/${T}_fcl_gaps.txt
