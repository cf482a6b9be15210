# FC_large / LSTM_large step, HIP-graph replay vs eager launches (the overlap mode's step shape), 1 GPU, alternating:
#   bash tools/eager_vs_graph.sh   (GPU box)
cd $GRAFT_REPO_ROOT
for i in 1 2; do for wl in fc_large lstm_large; do for g in graph eager; do
  if [ $g = eager ]; then fl=--no-graph; else fl=; fi
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 3 $fl > gpurun_out/evg.json 2>/dev/null
  python -c "import json; d=json.loads(open('gpurun_out/evg.json').read().strip().splitlines()[-1]); print('$wl', '$g', d['ms_per_step'], round(d['value']), d['config'].get('hip_graph'))"
done; done; done
