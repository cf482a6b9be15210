# Round-end evidence on the GPU box: bash tools/round_evidence.sh TAG
# FC_small trace + PMC passes (tools/profile_round.sh), the other workloads' bench lines, and SQ counters of the
# sampling kernel (k_inverse). Every GPU step has its own time limit; the chain stops at the first failure.
set -e
TAG=${1:-r02y}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_FC_SMALL" ] || bash tools/profile_round.sh $TAG   # SKIP_FC_SMALL=1: its passes ran already
mkdir -p gpurun_out/prof_$TAG
for w in fc_large lstm_large sample resimulate; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/${TAG}_${w}_bench.json 2> gpurun_out/${TAG}_${w}_bench.err
  echo ${w}_ok
done
OUT=gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/inv -o inv -- \
  python bench.py --workload sample --steps 3 --warmup 1 --no-cpu-baseline > $OUT/inv.log 2>&1
echo inv_ok
# re-simulation: kernel trace + FETCH / WRITE passes of k_resim (summarize_profile.py merges them into pmc_traffic.json)
RES="python bench.py --workload resimulate --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_resim -o resim -- $RES > $OUT/resim_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch/resim -o fetch -- $RES > $OUT/resim_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write/resim -o write -- $RES > $OUT/resim_write.log 2>&1
echo resim_prof_ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_sample -o sample -- python bench.py --workload sample --steps 5 --warmup 2 --no-cpu-baseline > $OUT/sample_trace.log 2>&1
echo sample_trace_ok
