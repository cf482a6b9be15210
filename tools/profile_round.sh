# Usage (on the GPU box): bash tools/profile_round.sh r02
# 1) rocprofv3 --kernel-trace --stats of the bench command  2) FETCH_SIZE pass  3) WRITE_SIZE pass
# 4) instruction / utilisation counters (8 SQ counters, one pass). Counters in their own passes, never combined
# with runtime / sys traces; each pass profiles a short bench run (the real training step's kernels).
set -e
TAG=${1:-r02}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --kernel-iters 5"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary > $OUT/bench_under_trace.log 2>&1
echo trace_ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $BENCH > $OUT/fetch.log 2>&1
echo fetch_ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $BENCH > $OUT/write.log 2>&1
echo write_ok
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/insts -o insts -- $BENCH > $OUT/insts.log 2>&1
echo insts_ok
