# Usage (on the GPU box): bash tools/profile_round.sh r01
# 1) rocprofv3 --kernel-trace --stats of the bench command  2) FETCH_SIZE pass  3) WRITE_SIZE pass
# (counters in their own passes, never combined with runtime / sys traces)
set -e
TAG=${1:-r01}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench_under_trace.log 2>&1
echo trace_ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
  python tools/kbench.py --iters 10 > $OUT/fetch.log 2>&1
echo fetch_ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
  python tools/kbench.py --iters 10 > $OUT/write.log 2>&1
echo write_ok
