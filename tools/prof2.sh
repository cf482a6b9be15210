set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc2 -o pass1 -- python tools/kbench.py --iters 3 > gpurun_out/pmc2a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc2 -o pass2 -- python tools/kbench.py --iters 3 > gpurun_out/pmc2b.log 2>&1
echo done
