# A/B of the re-simulation workload (GPU box): bash tools/ab_resim.sh build_exp/libA.so ...  (default library first)
set -e
for r in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then
      timeout -k 10 120 python bench.py --workload resimulate --no-cpu-baseline > gpurun_out/ab_r.json
    else
      BCNF_AMD_LIB=$lib timeout -k 10 120 python bench.py --workload resimulate --no-cpu-baseline > gpurun_out/ab_r.json
    fi
    python -c "import json; d=json.load(open('gpurun_out/ab_r.json')); print('$lib', d['ms_per_step'], round(d['value']/1e9, 3), 'G traj/s', d['roofline']['avg_us'])"
  done
done
