# Wide workloads' matrix-pipe utilisation (GPU box): per-kernel SQ counters and a kernel trace of short FC_large /
# LSTM_large bench runs, each pass alone.   bash tools/pmc_wide.sh TAG   (then python tools/pmc_wide.py TAG)
set -e
TAG=${1:-r04}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmcw_$TAG
mkdir -p $OUT
for wl in fc_large lstm_large; do
  B="python bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --kernel-iters 2"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$wl -o t -- $B > $OUT/trace_$wl.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA \
    --output-format csv -d $OUT/pmc_$wl -o p -- $B > $OUT/pmc_$wl.log 2>&1
  echo ${wl}_ok
done
