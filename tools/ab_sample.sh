# A/B of the sampling workload (GPU box): bash tools/ab_sample.sh build_exp/libA.so ...  (default library first)
set -e
for r in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --workload sample --no-cpu-baseline > gpurun_out/ab_s.json 2>/dev/null
    else
      BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --workload sample --no-cpu-baseline > gpurun_out/ab_s.json 2>/dev/null
    fi
    python -c "import json; d=json.loads(open('gpurun_out/ab_s.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']/1e6, 1), 'M draws/s')"
  done
done
