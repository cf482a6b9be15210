# SQ stall / issue counters of the sampling kernel and the wide chain GEMM (GPU box): bash tools/pmc_probe.sh TAG
# Each pass its own rocprofv3 run (counters never combined with traces), each under its own time limit.
set -e
TAG=${1:-r03}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/s$i -o s$i -- \
    python bench.py --workload sample --steps 2 --warmup 1 --no-cpu-baseline > $OUT/s$i.log 2>&1
  echo sample_pass$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/w$i -o w$i -- \
    python bench.py --workload fc_large --steps 2 --warmup 1 --no-cpu-baseline > $OUT/w$i.log 2>&1
  echo wide_pass$i
done
