# A/B of the wide workloads (GPU box): bash tools/ab_wide.sh fc_large build_exp/libA.so ...  (default library first)
set -e
w=${1:-fc_large}
shift || true
for r in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_w.json 2>/dev/null
    else
      BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_w.json 2>/dev/null
    fi
    python -c "import json; d=json.loads(open('gpurun_out/ab_w.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']/1e3, 1), 'k samples/s', d['roofline']['frac'], d.get('kernels_us'))"
  done
done
