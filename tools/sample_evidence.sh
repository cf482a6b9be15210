# Sampling evidence on the GPU box: bash tools/sample_evidence.sh TAG
# bench line (with CPU baseline), rocprofv3 kernel stats of the same workload, SQ counters of k_inverse_mfma.
set -e
TAG=${1:-r02z}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}_sample
mkdir -p $OUT
timeout -k 10 300 python bench.py --workload sample > gpurun_out/${TAG}_sample_bench.json 2> $OUT/bench.err
echo sample_bench_ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python bench.py --workload sample --no-cpu-baseline > $OUT/bench_under_trace.log 2>&1
echo sample_trace_ok
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/insts -o insts -- \
  python bench.py --workload sample --steps 3 --warmup 1 --no-cpu-baseline > $OUT/insts.log 2>&1
echo sample_insts_ok
