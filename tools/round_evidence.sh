# Round-end evidence on the GPU box: bash tools/round_evidence.sh TAG
# FC_small trace + PMC passes (tools/profile_round.sh), the other workloads' bench lines, and SQ counters of the
# sampling kernel (k_inverse). Every GPU step has its own time limit; the chain stops at the first failure.
set -e
TAG=${1:-r02y}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_round.sh $TAG
for w in fc_large lstm_large sample; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/${TAG}_${w}_bench.json 2> gpurun_out/${TAG}_${w}_bench.err
  echo ${w}_ok
done
OUT=gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/inv -o inv -- \
  python bench.py --workload sample --steps 3 --warmup 1 --no-cpu-baseline > $OUT/inv.log 2>&1
echo inv_ok
