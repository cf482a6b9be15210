# PMC passes over the wide-family micro-benchmark, restricted to kernels matching $2 (default k_wlink).
# Each --pmc pass alone (no trace domains). Usage (GPU box): bash tools/pmc_wide.sh TAG [regex]
set -e
TAG=${1:-wide}
RX=${2:-k_wlink}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmcw_$TAG
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o p$i -- \
    python tools/kbench_wide.py --iters 2 > $OUT/p$i.log 2>&1
  echo pass$i ok
done
