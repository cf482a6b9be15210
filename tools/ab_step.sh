# A/B of the FC_small training step (GPU box): bash tools/ab_step.sh build_exp/libA.so ...  (default library first)
set -e
for r in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab_st.json 2>/dev/null
    else
      BCNF_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab_st.json 2>/dev/null
    fi
    python -c "import json; d=json.loads(open('gpurun_out/ab_st.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], round(d['value']/1e6, 2), 'M samples/s', d.get('kernels_us'))"
  done
done
