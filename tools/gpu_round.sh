# GPU box, one call: issue probes, the full GPU suite, A/B of the working tree vs build_exp/libhead.so (the last
# commit) on the FC_small kernels and on sampling, then the default bench line. Each GPU step has its own limit and
# the chain stops at the first failure.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r03}
PROBES=${PROBES:-}
if [ -n "$PROBES" ]; then timeout -k 10 120 python tools/probe_issue.py $PROBES > gpurun_out/${T}_probe.txt 2>&1; cat gpurun_out/${T}_probe.txt; fi
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
AB_LIBS=${AB_LIBS:-build_exp/libhead.so}
for i in 1 2; do
  timeout -k 10 120 python tools/abk.py
  for lib in $AB_LIBS; do BCNF_AMD_LIB=$lib timeout -k 10 120 python tools/abk.py; done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_ab_kernels.txt
if [ -n "$AB_SAMPLE" ]; then bash tools/ab_sample.sh $AB_SAMPLE 2>&1 | tee gpurun_out/${T}_ab_sample.txt; fi
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['kernels_us'], {k: (v.get('value'), v.get('roofline', {}).get('frac')) for k, v in d['secondary'].items()})"
