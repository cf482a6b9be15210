# A/B of the bench's batch feed (GPU box): per-step index copy vs the device-resident epoch cursor
for mode in "--indexed" ""; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --kernel-iters 2 $mode > gpurun_out/ab.log 2>&1 || exit 1
  echo "feed=${mode:-epoch} $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
