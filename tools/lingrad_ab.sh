#!/bin/bash
# FC_large bench with the hidden-layer LINGRAD GEMM forced to each tiling (BCNF_LINGRAD_TILING; -1 = dispatcher).
set -e
mkdir -p gpurun_out
for t in -1 3 4 2 0; do
  BCNF_LINGRAD_TILING=$t timeout -k 10 120 python bench.py --workload fc_large --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/lingrad_$t.json 2>&1
  echo "tiling $t: $(grep -o '"kernels_us[^}]*}' gpurun_out/lingrad_$t.json)"
done
